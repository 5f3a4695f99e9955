#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k bias_grad_rowsum > gpurun_out/bg_tests.log 2>&1 || { tail -30 gpurun_out/bg_tests.log; exit 1; }
tail -1 gpurun_out/bg_tests.log
for r in 1 2; do
BG_SO=ab_so/_C_base.so timeout -k 10 60 python -u tools/bench_bias_grad.py 2>&1 | grep '"so"'
timeout -k 10 60 python -u tools/bench_bias_grad.py 2>&1 | grep '"so"'
done
