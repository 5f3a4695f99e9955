#!/bin/bash
# engine tests + serving bench after the pinned-buffer fix
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/llm_fix
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py -m gpu -k "engine or argmax" > gpurun_out/llm_fix/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/llm_fix/tests.log; exit 1; }
tail -1 gpurun_out/llm_fix/tests.log
for r in 1 2; do
timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > gpurun_out/llm_fix/b$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/llm_fix/b$r.log; exit 1; }
echo "run$r $(grep metric gpurun_out/llm_fix/b$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_p50_s"], d["steady_tpot_p50_ms"])')"
done
