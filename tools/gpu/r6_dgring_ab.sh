#!/bin/bash
# serving bench A/B: decode GEMM ring depths (6, 3) default vs (4, 4) (CAAMD_DG_RING=2), alternating
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dgring
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for g in 0 2; do
    CAAMD_DG_RING=$g timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/b_${g}_$r.log 2>&1 || { tail -20 $O/b_${g}_$r.log; exit 1; }
    echo "ring=$g round $r: $(grep -E '^\{' $O/b_${g}_$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_p50_s"], d["steady_tpot_p50_ms"])')"
  done
done
