#!/bin/bash
# Round-3 kernel profiles: GPT-2-XL step (fused head) and Llama-3-8B decode.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r3
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 $R/bench.py --mode spmd --steps 6 --warmup 2 > $O/step_bench.log 2>&1 || { echo "step prof failed"; tail -20 $O/step_bench.log; exit 1; }
tail -1 $O/step_bench.log
python3 $R/tools/prof_summary.py $O/step $O/step_summary.md && head -45 $O/step_summary.md
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/llm -o run -- python3 $R/tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/llm_bench.log 2>&1 || { echo "llm prof failed"; tail -20 $O/llm_bench.log; exit 1; }
grep metric $O/llm_bench.log | tail -1
python3 $R/tools/prof_summary.py $O/llm $O/llm_summary.md && sed -n '/Top kernels/,$p' $O/llm_summary.md | head -30
