#!/bin/bash
# Round 6: paired dK/dV kernel -- numerics, kernel timing A/B, step A/B.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_attn
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  for p in 1 0; do
    CAAMD_FA64_PAIR=$p timeout -k 10 120 python -u tools/bench_attn.py > $O/attn_${p}_$i.log 2>&1 || { tail -5 $O/attn_${p}_$i.log; exit 1; }
    echo "pair=$p: $(tail -2 $O/attn_${p}_$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for p in 1 0; do
    CAAMD_FA64_PAIR=$p timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${p}_$i.log 2>&1 || { tail -5 $O/bench_${p}_$i.log; exit 1; }
    echo "step pair=$p $(grep -o '"value": [0-9.]*' $O/bench_${p}_$i.log)"
  done
done
