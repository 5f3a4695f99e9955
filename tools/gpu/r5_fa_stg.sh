#!/bin/bash
# LDS-staged whole-row output stores in the D=64 attention kernels: tests + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "flash or attention or gqa or prefill or paged" > gpurun_out/fa_stg_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fa_stg_tests.log; exit 1; }
tail -1 gpurun_out/fa_stg_tests.log
for r in 1 2 3; do
for g in 0 1; do
CAAMD_FA64_STG=$g timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/fa_stg_$g.log 2>&1 || { echo "stg $g failed"; tail -5 gpurun_out/fa_stg_$g.log; exit 1; }
echo "STG=$g $(grep bwd_us gpurun_out/fa_stg_$g.log)"
done
done
