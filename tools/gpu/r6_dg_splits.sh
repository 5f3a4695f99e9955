#!/bin/bash
# Round 6: decode split-K counts A/B (o / down / qkv), serving bench, alternating arms
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_dgs
mkdir -p $O
ARMS=("" "4096x4096:4,4096x14336:4" "4096x4096:6,4096x14336:6" "6144x4096:4,4096x4096:4" "4096x14336:12")
for i in 1 2; do
  for a in 0 1 2 3 4; do
    CAAMD_DG_SPLITS="${ARMS[$a]}" timeout -k 10 240 python3 -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/b_${a}_$i.log 2>&1 || { echo "arm $a failed"; tail -20 $O/b_${a}_$i.log; exit 1; }
    echo "arm $a [${ARMS[$a]}] $(grep -o '"value": [0-9.]*\|"steady_tpot_p50_ms": [0-9.]*\|"ttft_p50_s": [0-9.]*' $O/b_${a}_$i.log | tr '\n' ' ')"
  done
done
