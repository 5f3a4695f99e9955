#!/bin/bash
# serving bench: decode GEMM ring depths (W, X images) -- 2 (4,4), 3 (5,5), 4 (6,4), 5 (4,6), 0 (6,3)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dgring2
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py -k "decode_gemm" > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for g in 2 3 4 5 0; do
    CAAMD_DG_RING=$g timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/b_${g}_$r.log 2>&1 || { tail -20 $O/b_${g}_$r.log; exit 1; }
    echo "ring=$g round $r: $(grep -E '^\{' $O/b_${g}_$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_p50_s"], d["steady_tpot_p50_ms"])')"
  done
done
