#!/bin/bash
# Round 6: k64 split-K tail (max slices of the partial last round, K >= 4096 shapes) -- step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_tail
mkdir -p $O
for i in 1 2; do for t in 4 2 8 1; do
  CAAMD_GEMM_TAIL_SPLIT=$t timeout -k 10 300 python -u bench.py > $O/bench_${t}_$i.log 2>&1 || { tail -5 $O/bench_${t}_$i.log; exit 1; }
  echo "tail_split=$t $(grep -o '"value": [0-9.]*' $O/bench_${t}_$i.log)"
done; done
