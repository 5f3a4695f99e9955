#!/bin/bash
# conv numerics + per-shape timings + ResNet-50 graph throughput
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/conv_r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_conv.py --tiles ${TILES:-0,1,2} > $O/bench_conv.log 2>&1 || { echo "bench_conv failed"; tail -20 $O/bench_conv.log; exit 1; }
tail -1 $O/bench_conv.log
for r in 1 2; do
timeout -k 10 240 python -u tools/bench_resnet.py > $O/resnet_$r.log 2>&1 || { echo "resnet failed"; tail -20 $O/resnet_$r.log; exit 1; }
tail -1 $O/resnet_$r.log
done
