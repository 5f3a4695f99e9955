#!/bin/bash
# Round 5 final profiles: GPT-2-XL step and Llama-3-8B serving kernel summaries (no Cijk_*).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final_prof_r5
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fp5/step -o run -- python3 $R/bench.py --mode spmd --steps 6 --warmup 2 > $O/step_bench.log 2>&1 || { echo "step prof failed"; tail -20 $O/step_bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/step_bench.log
python3 $R/tools/prof_summary.py /tmp/fp5/step $O/step_summary.md && sed -n '/Top kernels/,$p' $O/step_summary.md | head -16
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fp5/llm -o run -- python3 $R/tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/llm.log 2>&1 || { echo "llm prof failed"; tail -20 $O/llm.log; exit 1; }
grep metric $O/llm.log | tail -1 | grep -o '"value": [0-9.]*\|"ttft_p50_s": [0-9.]*\|"steady_tpot_p50_ms": [0-9.]*'
python3 $R/tools/prof_summary.py /tmp/fp5/llm $O/llm_summary.md && sed -n '/Top kernels/,$p' $O/llm_summary.md | head -16
echo "Cijk kernels in serving: $(grep -c Cijk $O/llm_summary.md || true)"
