#!/bin/bash
# Round 6: MFMA shape (16x16x32 vs 32x32x16, LDS-fed, random data) and full-line tile
# (256x320 vs 256x256) measurements for the GEMM review items.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_lab
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/lab/mfma_shape_bench 4000 > $O/mfma_shape.jsonl 2>&1 || { cat $O/mfma_shape.jsonl; exit 1; }
cat $O/mfma_shape.jsonl
timeout -k 10 300 python -u tools/gemm_tile_ab.py > $O/tile_ab.jsonl 2>&1 || { tail -5 $O/tile_ab.jsonl; exit 1; }
cat $O/tile_ab.jsonl
