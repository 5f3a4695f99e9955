#!/bin/bash
# Data TTFB after lazy graph capture: vision GPU tests, actor start-up phases, e2e bench
set -o pipefail
mkdir -p gpurun_out/data
timeout -k 10 300 python -u -m pytest tests/test_vision.py -x -v --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/data/pytest_vision.log 2>&1 &&
timeout -k 10 240 python -u tools/data_ttfb.py > gpurun_out/data/ttfb_phases.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > gpurun_out/data/bench_data.log 2>&1
rc=$?
tail -3 gpurun_out/data/pytest_vision.log; cat gpurun_out/data/ttfb_phases.log | grep '{'; head -c 900 gpurun_out/data/bench_data.log
exit $rc
