#!/bin/bash
# Round 6: TN weight-gradient kernel tile-order group -- tests (with group 4 forced), step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_tngm
mkdir -p $O
CAAMD_TN_GROUP_M=4 timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gpt2_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
for i in 1 2; do for g in 4 8 16; do
  CAAMD_TN_GROUP_M=$g timeout -k 10 300 python -u bench.py > $O/bench_${g}_$i.log 2>&1 || { tail -5 $O/bench_${g}_$i.log; exit 1; }
  echo "tn_group_m=$g $(grep -o '"value": [0-9.]*' $O/bench_${g}_$i.log)"
done; done
