#!/bin/bash
# head-dim-128 forward: pre-scaled Q + -max accumulator init vs FMA per score
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_llm_gpu.py -m gpu -k "flash or prefill or llama or gqa" > gpurun_out/fa128_pre_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fa128_pre_tests.log; exit 1; }
tail -1 gpurun_out/fa128_pre_tests.log
for r in 1 2 3; do
for p in 0 1; do
CAAMD_FA64_FWD_PRE=$p ATTN_SHAPE=16,512,32,128 timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/fa128_pre_$p.log 2>&1 || { echo "pre $p failed"; tail -5 gpurun_out/fa128_pre_$p.log; exit 1; }
echo "PRE=$p $(grep -o '"fwd_us": [0-9.]*' gpurun_out/fa128_pre_$p.log)"
done
done
