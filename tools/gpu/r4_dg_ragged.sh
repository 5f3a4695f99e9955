#!/bin/bash
# (historical: the A/B environment knob this script sets was removed after the measurement;
#  the script records how the committed profile was produced)
# Round 4: ragged split-K in the decode GEMM (Llama-3-8B qkv: 5 splits on 240 CUs vs 4 on 192) --
# decode GEMM tests, then the LLM serving bench alternating ragged / equal splits.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dg_ragged
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
A="--num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128"
for v in ragged even ragged even; do
  case $v in
    even) E="CAAMD_DG_EVEN_SPLITS=1" ;;
    *) E="CAAMD_DG_EVEN_SPLITS=0" ;;
  esac
  env $E timeout -k 10 300 python -u tools/bench_llm.py $A > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_$v.log; exit 1; }
  echo $v $(grep -o '"ttft_p50_s": [0-9.]*\|"steady_tpot_p50_ms": [0-9.]*\|"value": [0-9.]*' $O/bench_$v.log | tr '\n' ' ')
  grep metric $O/bench_$v.log | tail -1 >> $O/bench.jsonl
done
