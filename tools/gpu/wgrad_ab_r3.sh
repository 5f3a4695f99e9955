#!/bin/bash
# Step A/B: fc2 / qkv weight gradients on gemm.hip (CAAMD_WGRAD_EXTRA) vs hipBLASLt.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/wgrad_ab
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run base$r
  run fc2s3_$r CAAMD_WGRAD_EXTRA=1600x6400:420
  run fc2sk_$r CAAMD_WGRAD_EXTRA=1600x6400:280
  run qkv2_$r CAAMD_WGRAD_EXTRA=4800x1600:190
done
