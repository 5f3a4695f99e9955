#!/bin/bash
# Round 6: full-line kernel on the 1600 x 1600 projection -- tests, then step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_k64min
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gpt2_parity_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  for m in 1536 4096; do
    CAAMD_GEMM_K64_MIN=$m timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${m}_$i.log 2>&1 || { tail -5 $O/bench_${m}_$i.log; exit 1; }
    echo "k64_min=$m $(grep -o '"value": [0-9.]*' $O/bench_${m}_$i.log)"
  done
done
