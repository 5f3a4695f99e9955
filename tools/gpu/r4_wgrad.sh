#!/bin/bash
# Round 4: lockstep (slice-major) vs stream-K weight-gradient order; numerics first.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/wgrad_r4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad or k64" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/wgrad_bench.py > $O/wgrad.jsonl 2> $O/wgrad.err || { echo "bench failed"; tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
