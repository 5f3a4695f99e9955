#!/bin/bash
# serving bench: per-shape prefill algos (default) vs algo 9 everywhere (CAAMD_PREFILL_ALGO=9), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pa_ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py -m gpu -k "prefill or engine or llama" > gpurun_out/pa_ab/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pa_ab/tests.log; exit 1; }
tail -1 gpurun_out/pa_ab/tests.log
for r in 1 2 3; do
for v in old new; do
if [ $v = old ]; then export CAAMD_PREFILL_ALGO=9; else unset CAAMD_PREFILL_ALGO; fi
timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > gpurun_out/pa_ab/b_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/pa_ab/b_$v.log; exit 1; }
echo "$v $(grep metric gpurun_out/pa_ab/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_p50_s"], d["tpot_p50_ms"], d["steady_tpot_p50_ms"])')"
done
done
