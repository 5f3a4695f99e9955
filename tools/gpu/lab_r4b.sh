#!/bin/bash
# Round 4: k64 GEMM -- 2-phase variant (v4) and DMA diagnostics (no-wait / L2-hot).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/lab_r4b
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/gemm_lab/gemm_lab "" 10 5 2,3009,4009 > $O/lab.log 2>&1 || { echo "lab failed rc=$?"; tail -20 $O/lab.log; exit 1; }
grep shape $O/lab.log
# ablations, 4-phase (2009+) and 2-phase (4009+): 1 noDMA 2 noRead 3 MFMA+bar 4 noMFMA 6 DMA+bar 8 noEpi 22 DMA+bar,nowait 38 DMA+bar,hot 54 DMA+bar,hot,nowait
timeout -k 10 200 tools/gemm_lab/gemm_lab fc_fwd_plain 10 5 2009,2019,2029,2039,2049,2069,2089,2229,2389,2549,4009,4019,4029,4039,4049,4069,4089,4229,4389,4549 > $O/abl.log 2>&1 || { echo "abl failed"; tail -20 $O/abl.log; exit 1; }
grep shape $O/abl.log
