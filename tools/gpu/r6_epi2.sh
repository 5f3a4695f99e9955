#!/bin/bash
# production dGELU early-Z epilogue: GEMM + parity tests, then the default bench
set -o pipefail
mkdir -p gpurun_out/epi2
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gemm_gpu.py tests/test_gpt2_parity_gpu.py tests/test_fused_head_gpu.py > gpurun_out/epi2/tests.log 2>&1; rc=$?
tail -3 gpurun_out/epi2/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/epi2/bench.log 2>&1 || { tail -5 gpurun_out/epi2/bench.log; exit 1; }
grep '"metric"' gpurun_out/epi2/bench.log
timeout -k 10 300 python -u bench.py > gpurun_out/epi2/bench2.log 2>&1 || { tail -5 gpurun_out/epi2/bench2.log; exit 1; }
grep '"metric"' gpurun_out/epi2/bench2.log
