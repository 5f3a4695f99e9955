#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_lntest
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpt2_parity_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench.log
