#!/bin/bash
# algo 8 (persistent async-epilogue GEMM): numerics, isolated timings, step A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/pst_r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_pst.py > $O/bench_pst.log 2>&1 || { echo "bench_pst failed"; tail -20 $O/bench_pst.log; exit 1; }
cat $O/bench_pst.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run pst$r CAAMD_GEMM_PST=1
  run base$r CAAMD_GEMM_PST=0
done
