#!/bin/bash
# Round 4: algo 15 (external lockstep combine) numerics + timing, prefill GEMM per-shape comparison.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/batch2_r4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_zero_gpu.py -x -q --timeout 200 --timeout-method thread -k "wgrad or zero" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 240 python -u tools/wgrad_bench.py --ksweep > $O/ksweep.jsonl 2> $O/ksweep.err || { echo "ksweep failed"; tail -5 $O/ksweep.err; exit 1; }
cat $O/ksweep.jsonl
timeout -k 10 300 python -u tools/bench_prefill_gemm.py > $O/prefill.jsonl 2> $O/prefill.err || { echo "prefill bench failed"; tail -5 $O/prefill.err; exit 1; }
cat $O/prefill.jsonl
