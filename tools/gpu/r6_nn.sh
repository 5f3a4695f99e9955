#!/bin/bash
# Round 6: NN GEMM kernel (algo 27) -- tests, standalone A/B, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_nn
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gpt2_parity_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/gemm_nn_ab.py > $O/nn_ab.jsonl 2>&1 || { tail -5 $O/nn_ab.jsonl; exit 1; }
grep shape $O/nn_ab.jsonl
for i in 1 2; do
  for f in 1 0; do
    CAAMD_GEMM_NN=$f timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${f}_$i.log 2>&1 || { tail -5 $O/bench_${f}_$i.log; exit 1; }
    echo "nn=$f $(grep -o '"value": [0-9.]*' $O/bench_${f}_$i.log)"
  done
done
