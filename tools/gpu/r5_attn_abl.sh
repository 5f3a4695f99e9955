#!/bin/bash
# dK/dV ablations (whole backward timed by tools/bench_attn.py; dQ unchanged)
set -o pipefail
cd $GRAFT_REPO_ROOT
for a in 0 7 15 23 31 0; do
CAAMD_FA64_BWD_ABL=$a timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/abl_$a.log 2>&1 || { echo "abl $a failed"; tail -5 gpurun_out/abl_$a.log; exit 1; }
echo "ABL=$a $(grep bwd_us gpurun_out/abl_$a.log)"
done
