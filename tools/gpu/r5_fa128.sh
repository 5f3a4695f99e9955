#!/bin/bash
# head-dim-128 second-generation forward: tests, then timing vs the first generation
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_llm_gpu.py -m gpu -k "flash or prefill or llama" > gpurun_out/fa128_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fa128_tests.log; exit 1; }
tail -1 gpurun_out/fa128_tests.log
for r in 1 2; do
for v in 0 1; do
CAAMD_FA_V1=$v ATTN_SHAPE=16,512,32,128 timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/fa128_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/fa128_$v.log; exit 1; }
echo "V1=$v $(grep fwd_us gpurun_out/fa128_$v.log)"
done
done
