#!/bin/bash
# dK/dV: K rows by LDS-DMA in the prologue (OPT 104) vs per-lane global loads (OPT 40)
set -o pipefail
cd $GRAFT_REPO_ROOT
CAAMD_FA64_DKDV_OPT=104 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpt2_parity_gpu.py -m gpu -k "flash or attention or parity" > gpurun_out/kdma_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/kdma_tests.log; exit 1; }
tail -1 gpurun_out/kdma_tests.log
for r in 1 2 3; do
for o in 40 104; do
CAAMD_FA64_DKDV_OPT=$o timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/kdma_$o.log 2>&1 || { echo "opt $o failed"; tail -5 gpurun_out/kdma_$o.log; exit 1; }
echo "OPT=$o $(grep -o '"bwd_us": [0-9.]*' gpurun_out/kdma_$o.log)"
done
done
