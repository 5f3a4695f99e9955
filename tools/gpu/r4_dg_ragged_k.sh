#!/bin/bash
# (historical: the A/B environment knob this script sets was removed after the measurement;
#  the script records how the committed profile was produced)
# Round 4: decode GEMM per-shape times, ragged vs equal split-K (bench_decode_gemm3.py, cache-cold weights).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dg_ragged_k
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  CAAMD_DG_EVEN_SPLITS=$v timeout -k 10 300 python -u tools/bench_decode_gemm3.py > $O/even$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/even$v.log; exit 1; }
  echo "even=$v"; grep -E '"gemm": "qkv"|layer_total' $O/even$v.log
done
