#!/bin/bash
# Round 6: LayerNorm backward grid caps (step form with dxsum), then step A/B of the best cap
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_ln2
mkdir -p $O
LN_BWD_CAPS=0,256,512,768,1024,1536 timeout -k 10 300 python -u tools/bench_ln_bwd.py > $O/ln.jsonl 2>&1 || { tail -5 $O/ln.jsonl; exit 1; }
grep dxsum $O/ln.jsonl | cut -c1-110
for i in 1 2; do
  for nb in 1024 0; do
    CAAMD_LN_BWD_BLOCKS=$nb timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${nb}_$i.log 2>&1 || { tail -5 $O/bench_${nb}_$i.log; exit 1; }
    echo "ln_bwd_blocks=$nb $(grep -o '"value": [0-9.]*' $O/bench_${nb}_$i.log)"
  done
done
