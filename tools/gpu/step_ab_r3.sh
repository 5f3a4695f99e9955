#!/bin/bash
# Round-3 step A/B: GEMM split tail and the weight-gradient kernel, alternating
# arms in one call (same box), SPMD mode, 10 timed steps each.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ab_r3
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run base$r CAAMD_GEMM_TAIL=0 CAAMD_WGRAD_SK=0
  run tail$r CAAMD_GEMM_TAIL=1 CAAMD_WGRAD_SK=0
  run both$r CAAMD_GEMM_TAIL=1 CAAMD_WGRAD_SK=1
done
