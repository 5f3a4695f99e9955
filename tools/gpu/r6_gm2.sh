#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_gm2
mkdir -p $O
for i in 1 2; do for cfg in "4 4" "4 2" "3 4" "4 8"; do
  set -- $cfg
  CAAMD_GEMM_GROUP_M=$1 CAAMD_TN_GROUP_M=$2 timeout -k 10 300 python -u bench.py > $O/bench_${1}_${2}_$i.log 2>&1 || { tail -5 $O/bench_${1}_${2}_$i.log; exit 1; }
  echo "k64_group=$1 tn_group=$2 $(grep -o '"value": [0-9.]*' $O/bench_${1}_${2}_$i.log)"
done; done
