#!/bin/bash
# Round 4: four-wave 256 x 256 kernel (algo 20) vs the full-line kernel on the prefill and fc shapes.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/lab_w4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/gemm_lab/gemm_lab pf_ 10 5 9,1009,20 > $O/pf.log 2>&1 || { echo "lab pf failed rc=$?"; tail -20 $O/pf.log; exit 1; }
grep -E "shape|check" $O/pf.log
timeout -k 10 300 tools/gemm_lab/gemm_lab fc 10 5 4009,20 > $O/fc.log 2>&1 || { echo "lab fc failed rc=$?"; tail -20 $O/fc.log; exit 1; }
grep -E "shape|check" $O/fc.log
