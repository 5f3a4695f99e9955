#!/bin/bash
# LayerNorm backward column-split (variant 3) vs one-row-per-wave (variant 0) in the
# training step, same box, alternating arms; kernel tests first.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ln_ab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
echo "pytest: $(tail -1 $O/pytest.log)"
run() {
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run v0_$r CAAMD_LN_BWD_VARIANT=0
  run v3_$r CAAMD_LN_BWD_VARIANT=3
done
