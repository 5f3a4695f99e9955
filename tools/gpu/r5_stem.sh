#!/bin/bash
# pixel-pair stem: tests, then ResNet graph throughput with / without it, then the Data bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py tests/test_vision.py > gpurun_out/stem_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
for r in 1 2; do
for ps in 1 0; do
CAAMD_RESNET_PAIR_STEM=$ps timeout -k 10 120 python -u tools/bench_resnet.py --batch-size 512 --iters 30 > gpurun_out/stem_bench.log 2>&1 || { tail -10 gpurun_out/stem_bench.log; exit 1; }
echo "PAIR=$ps $(grep '{' gpurun_out/stem_bench.log | tail -1)"
done
done
