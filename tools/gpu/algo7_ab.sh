#!/bin/bash
# GEMM algo 7 (DMA pieces between the MFMA groups, distance 3) vs algo 2, same box:
# numerics under both, then alternating 10-step SPMD bench arms.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/algo7_ab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_a2.log 2>&1 || { echo "pytest algo2 failed"; tail -20 $O/pytest_a2.log; exit 1; }
CAAMD_GEMM_ALGO=7 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_a7.log 2>&1 || { echo "pytest algo7 failed"; tail -20 $O/pytest_a7.log; exit 1; }
echo "pytest ok: $(tail -1 $O/pytest_a2.log) | $(tail -1 $O/pytest_a7.log)"
run() {
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run a2_$r CAAMD_GEMM_ALGO=2
  run a7_$r CAAMD_GEMM_ALGO=7
done
