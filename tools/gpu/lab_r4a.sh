#!/bin/bash
# Round 4: full-line (BK = 64) GEMM kernel vs the 32-deep ping-pong kernel, lab harness.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/lab_r4a
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/gemm_lab/gemm_lab "" 10 5 2,9,1009,3009 > $O/lab.log 2>&1 || { echo "lab failed rc=$?"; tail -20 $O/lab.log; exit 1; }
grep shape $O/lab.log
timeout -k 10 200 tools/gemm_lab/gemm_lab fc_fwd_plain 10 5 2,9,19,29,39,49,69,89 > $O/abl.log 2>&1 || { echo "abl failed"; tail -20 $O/abl.log; exit 1; }
grep shape $O/abl.log
