#!/bin/bash
# Round 4: ZeRO world-1 check after the readiness fix, wgrad K sweep (algo 15 vs in-kernel combine),
# prefill GEMM per-shape comparison, attention PMC pass 1.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/batch3_r4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_zero_gpu.py -x -q --timeout 200 --timeout-method thread > $O/zero.log 2>&1; zrc=$?
echo "zero rc=$zrc"; grep -E "^E |passed|failed" $O/zero.log | head -8
[ $zrc -eq 0 ] || [ $zrc -eq 1 ] || exit $zrc
timeout -k 10 240 python -u tools/wgrad_bench.py --ksweep > $O/ksweep.jsonl 2> $O/ksweep.err || { echo "ksweep failed"; tail -5 $O/ksweep.err; exit 1; }
cat $O/ksweep.jsonl
timeout -k 10 300 python -u tools/bench_prefill_gemm.py > $O/prefill.jsonl 2> $O/prefill.err || { echo "prefill bench failed"; tail -5 $O/prefill.err; exit 1; }
cat $O/prefill.jsonl
