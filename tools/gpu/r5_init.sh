#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/init_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
BREAKDOWN=1 timeout -k 10 120 python -u tools/predictor_init_prof.py > $O/init.log 2>&1 || { tail -20 $O/init.log; exit 1; }
cat $O/init.log
