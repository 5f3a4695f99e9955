#!/bin/bash
# Round 5: TN full-line weight-gradient kernel: numerics, then timings vs stream-K / hipBLASLt.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/tn_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "tn64" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/wgrad_bench.py --tn > $O/tn.jsonl 2> $O/tn.err || { echo "bench failed"; tail -20 $O/tn.err; exit 1; }
cat $O/tn.jsonl
