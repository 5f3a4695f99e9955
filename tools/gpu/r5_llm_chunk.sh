#!/bin/bash
# Serving: prefill chunk size (max_num_batched_tokens) vs TTFT / throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/llm_r5
for t in 16384 8192 4096; do
timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 --max-batched-tokens $t > gpurun_out/llm_r5/chunk_$t.log 2>&1 || { echo "bench $t failed"; tail -20 gpurun_out/llm_r5/chunk_$t.log; exit 1; }
grep '"metric"' gpurun_out/llm_r5/chunk_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($t, {k: d.get(k) for k in ('value','ttft_p50_s','tpot_p50_ms','steady_tpot_p50_ms','elapsed_s')})"
done
