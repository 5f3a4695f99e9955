#!/bin/bash
# Round 4: k64 GEMM numerics + step A/B (CAAMD_GEMM_K64=1 vs 0), alternating on one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/k64_ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  for k in 1 0; do
    CAAMD_GEMM_K64=$k timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > $O/bench_k${k}_$i.log 2>&1 || { echo "bench k=$k failed"; tail -20 $O/bench_k${k}_$i.log; exit 1; }
    echo "k64=$k run $i: $(grep '"metric"' $O/bench_k${k}_$i.log)"
  done
done
