#!/bin/bash
# dK/dV schedule variants A/B (bench_attn: fwd + full backward, B32 T1024 H25 D64)
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for o in 0 4 6 2; do
CAAMD_FA64_DKDV_OPT=$o timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/dkdv_opt_$o.log 2>&1 || { echo "opt $o failed"; tail -5 gpurun_out/dkdv_opt_$o.log; exit 1; }
echo "OPT=$o $(grep bwd_us gpurun_out/dkdv_opt_$o.log)"
done
done
CAAMD_FA64_DKDV_OPT=4 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "flash or attention" > gpurun_out/dkdv_opt_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/dkdv_opt_tests.log; exit 1; }
tail -2 gpurun_out/dkdv_opt_tests.log
