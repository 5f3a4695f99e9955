#!/bin/bash
# Round 6: k64 GEMM tile-order group (m-tiles per group) -- step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_groupm
mkdir -p $O
for i in 1 2; do for g in ${GM_LIST:-16 8 4}; do
  CAAMD_GEMM_GROUP_M=$g timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${g}_$i.log 2>&1 || { tail -5 $O/bench_${g}_$i.log; exit 1; }
  echo "group_m=$g $(grep -o '"value": [0-9.]*' $O/bench_${g}_$i.log)"
done; done
