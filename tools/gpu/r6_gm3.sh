#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_gm3
mkdir -p $O
for i in 1 2; do for g in 3 4 5 2; do
  CAAMD_GEMM_GROUP_M=$g timeout -k 10 300 python -u bench.py > $O/bench_${g}_$i.log 2>&1 || { tail -5 $O/bench_${g}_$i.log; exit 1; }
  echo "k64_group=$g $(grep -o '"value": [0-9.]*' $O/bench_${g}_$i.log)"
done; done
bash tools/gpu/r6_tail.sh
