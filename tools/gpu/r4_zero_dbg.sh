#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/zero_dbg
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_zero_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "AssertionError|assert|Error|passed|failed" $O/pytest.log | head -30
exit $rc
