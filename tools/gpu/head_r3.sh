#!/bin/bash
# Chunked fused LM head: numerics, isolated head timing, then step A/B
# (CAAMD_FUSED_HEAD=1 vs 0, alternating, SPMD, same box).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/head_r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_head_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python -u tools/bench_head.py > $O/bench_head.log 2>&1 || { echo "bench_head failed"; tail -20 $O/bench_head.log; exit 1; }
cat $O/bench_head.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run fused$r CAAMD_FUSED_HEAD=1
  run base$r CAAMD_FUSED_HEAD=0
done
