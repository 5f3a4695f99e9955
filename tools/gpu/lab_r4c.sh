#!/bin/bash
# Round 4: k64 GEMM with L2 prefetch of K-tile t+2 (v5/v6/v7) vs 2-phase (v4) and the pp kernel.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/lab_r4c
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/gemm_lab/gemm_lab "" 10 5 2,4009,6009,5009,7009 > $O/lab.log 2>&1 || { echo "lab failed rc=$?"; tail -20 $O/lab.log; exit 1; }
grep shape $O/lab.log
timeout -k 10 200 tools/gemm_lab/gemm_lab fc_fwd_plain 10 5 4009,4069,6009,6069,6039,6089 > $O/abl.log 2>&1 || { echo "abl failed"; tail -20 $O/abl.log; exit 1; }
grep shape $O/abl.log
