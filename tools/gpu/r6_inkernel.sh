#!/bin/bash
# Round 6: TN weight-gradient split-K combine in-kernel (algo 26) vs the reduce launch -- step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_inkernel
mkdir -p $O
for i in 1 2; do
  for f in 1 0; do
    CAAMD_WGRAD_TN_INKERNEL=$f timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${f}_$i.log 2>&1 || { tail -5 $O/bench_${f}_$i.log; exit 1; }
    echo "tn_inkernel=$f $(grep -o '"value": [0-9.]*' $O/bench_${f}_$i.log)"
  done
done
