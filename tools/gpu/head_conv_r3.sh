#!/bin/bash
# Round 3: chunked fused LM head + own implicit-GEMM conv. Numerics first, then
# isolated timings, then step / ResNet A/B (alternating arms, same box).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/hc_r3
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_head_gpu.py tests/test_conv_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python -u tools/bench_head.py > $O/bench_head.log 2>&1 || { echo "bench_head failed"; tail -20 $O/bench_head.log; exit 1; }
cat $O/bench_head.log
for r in 1 2; do
  for own in 1 0; do
    CAAMD_OWN_CONV=$own timeout -k 10 240 python -u tools/bench_resnet.py > $O/resnet_own${own}_$r.log 2>&1 || { echo "resnet $own failed"; tail -20 $O/resnet_own${own}_$r.log; exit 1; }
    echo "resnet own=$own: $(tail -1 $O/resnet_own${own}_$r.log)"
  done
done
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run fused$r CAAMD_FUSED_HEAD=1
  run base$r CAAMD_FUSED_HEAD=0
done
