#!/bin/bash
# fused decode reduce + residual + RMSNorm: tests, then bench_llm A/B (256 x 512 x 128, 128 seqs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rn
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py -m gpu > gpurun_out/rn/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rn/tests.log; exit 1; }
tail -1 gpurun_out/rn/tests.log
for r in 1 2 3; do
for f in 1 0; do
CAAMD_DECODE_REDUCE_NORM=$f timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > gpurun_out/rn/b_$f.log 2>&1 || { echo "bench $f failed"; tail -20 gpurun_out/rn/b_$f.log; exit 1; }
echo "RN=$f $(grep metric gpurun_out/rn/b_$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_p50_s"], d["steady_tpot_p50_ms"])')"
done
done
