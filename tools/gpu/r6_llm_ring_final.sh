#!/bin/bash
# decode (4, 4) ring default: decode GEMM + Llama GPU tests (incl. the HF parity test), then the serving bench twice
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/llm_ring_final
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_llm_gpu.py tests/test_llama_hf_parity_gpu.py > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 400 python -u tools/bench_llm.py --num-prompts 256 --max-num-seqs 128 --input-len 512 --output-len 128 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  grep -E '^\{' $O/bench_$i.log | tail -1
done
