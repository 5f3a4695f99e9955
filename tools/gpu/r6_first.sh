#!/bin/bash
# Round 6, first call: side-stream prefetch race tests + default bench (box baseline).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_first
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_device_transfer_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log
