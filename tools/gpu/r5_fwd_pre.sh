#!/bin/bash
# forward: Q pre-scaled + -max accumulator init (PRE) vs FMA per score
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpt2_parity_gpu.py tests/test_llm_gpu.py -m gpu -k "flash or attention or parity or gqa" > gpurun_out/fwd_pre_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fwd_pre_tests.log; exit 1; }
tail -1 gpurun_out/fwd_pre_tests.log
for r in 1 2 3; do
for p in 0 1; do
CAAMD_FA64_FWD_PRE=$p timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/fwd_pre_$p.log 2>&1 || { echo "pre $p failed"; tail -5 gpurun_out/fwd_pre_$p.log; exit 1; }
echo "PRE=$p $(grep fwd_us gpurun_out/fwd_pre_$p.log)"
done
done
