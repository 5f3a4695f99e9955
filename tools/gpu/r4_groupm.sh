#!/bin/bash
# Round 4: tile-order group size (m-tiles per group) sweep of the full-line GEMM kernel.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/groupm_r4
mkdir -p $O
cd $GRAFT_REPO_ROOT
for g in 8 4 16 2 32 8; do
  timeout -k 10 240 tools/gemm_lab/gemm_lab "" 10 5 4009 $g > $O/g$g.log 2>&1 || { echo "lab g=$g failed"; tail -5 $O/g$g.log; exit 1; }
  echo "== g=$g"; grep shape $O/g$g.log
done
