#!/bin/bash
# (historical: the A/B environment knob this script sets was removed after the measurement;
#  the script records how the committed profile was produced)
# Llama decode with qkv / o on the decode GEMM + split-K reduce launch vs before.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dgllm
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
A="--num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len ${OUTLEN:-128}"
for v in ${ORDER:-new old new old}; do
  case $v in
    old) E="CAAMD_DG_EXT=0 CAAMD_DECODE_ATTN_GEMM=0" ;;
    mid) E="CAAMD_DECODE_NORM_FUSED=0" ;;
    ring1) E="CAAMD_DG_RING=1" ;;
    merge) E="CAAMD_PAGED_MERGE=1" ;;
    ring2) E="CAAMD_DG_RING=2" ;;
    *) E="" ;;
  esac
  env $E timeout -k 10 300 python -u tools/bench_llm.py $A > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_$v.log; exit 1; }
  echo $v $(grep -o '"steady_tpot_p50_ms": [0-9.]*\|"value": [0-9.]*' $O/bench_$v.log | tr '\n' ' ')
  grep metric $O/bench_$v.log | tail -1 >> $O/bench.jsonl
done
