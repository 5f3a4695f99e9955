#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_xent
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_head_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
for i in 1 2; do for t in 512 1024; do
  CAAMD_XENT_TPB=$t timeout -k 10 120 python -u tools/bench_xent.py 2>&1 | grep tpb || exit 1
done; done
for i in 1 2; do for t in 512 1024; do
  CAAMD_XENT_TPB=$t timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${t}_$i.log 2>&1 || { tail -5 $O/bench_${t}_$i.log; exit 1; }
  echo "xent_tpb=$t $(grep -o '"value": [0-9.]*' $O/bench_${t}_$i.log)"
done; done
