#!/bin/bash
# dGELU epilogue early-Z variant A/B + the qkv-bias drain change's GPU tests
set -o pipefail
mkdir -p gpurun_out/epi
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpt2_parity_gpu.py tests/test_fused_head_gpu.py tests/test_zero_gpu.py tests/test_kernels_gpu.py -k "flash or attn or gpt2 or parity or zero or head" > gpurun_out/epi/tests.log 2>&1; rc=$?
tail -3 gpurun_out/epi/tests.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 300 python -u tools/gemm_epi_ab.py > gpurun_out/epi/ab.jsonl 2> gpurun_out/epi/ab.err || { tail -5 gpurun_out/epi/ab.err; exit 1; }
cat gpurun_out/epi/ab.jsonl
