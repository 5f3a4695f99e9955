#!/bin/bash
# end-of-round serving bench on the final tree (Llama-3-8B shape, random init), twice
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/llm_final
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 500 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  grep -E '^\{' $O/bench_$i.log | tail -1
done
