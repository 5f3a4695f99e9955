#!/bin/bash
# Round 4: after the spill fix -- wgrad tests + K sweep (algo 15 vs in-kernel), step A/B
# (CAAMD_WGRAD_EXT 1 vs 0), LLM bench with the packed prefill on algo 9.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/batch4_r4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 240 python -u tools/wgrad_bench.py --ksweep > $O/ksweep.jsonl 2> $O/ksweep.err || { echo "ksweep failed"; tail -5 $O/ksweep.err; exit 1; }
cat $O/ksweep.jsonl
for i in 1 2; do
  for e in 1 0; do
    CAAMD_WGRAD_EXT=$e timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > $O/bench_ext${e}_$i.log 2>&1 || { echo "bench ext=$e failed"; tail -20 $O/bench_ext${e}_$i.log; exit 1; }
    echo "ext=$e run $i: $(grep -o '"value": [0-9.]*' $O/bench_ext${e}_$i.log)"
  done
done
A="--num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128"
timeout -k 10 300 python -u tools/bench_llm.py $A > $O/llm.log 2>&1 || { echo "llm bench failed"; tail -5 $O/llm.log; exit 1; }
grep -o '"ttft_p50_s": [0-9.]*\|"steady_tpot_p50_ms": [0-9.]*\|"value": [0-9.]*' $O/llm.log | tr '\n' ' '
