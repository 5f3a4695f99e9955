#!/bin/bash
# one-step-ahead greedy decode: engine tests, then bench_llm A/B (CAAMD_LLM_ASYNC)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/llm_async
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py tests/test_data_llm_gpu.py tests/test_llm.py -m gpu > gpurun_out/llm_async/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/llm_async/tests.log; exit 1; }
tail -1 gpurun_out/llm_async/tests.log
for r in 1 2; do
for a in 1; do
CAAMD_LLM_ASYNC=$a timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > gpurun_out/llm_async/b_$a.log 2>&1 || { echo "bench $a failed"; tail -20 gpurun_out/llm_async/b_$a.log; exit 1; }
echo "ASYNC=$a $(grep metric gpurun_out/llm_async/b_$a.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_p50_s"], d["tpot_p50_ms"], d["steady_tpot_p50_ms"])')"
done
done
