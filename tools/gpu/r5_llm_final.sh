#!/bin/bash
# serving bench (256 x 512 x 128, 128 seqs), two runs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/llm_final
for r in 1 2; do
timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > gpurun_out/llm_final/b$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/llm_final/b$r.log; exit 1; }
grep metric gpurun_out/llm_final/b$r.log
done
