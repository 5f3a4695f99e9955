#!/bin/bash
# Round 6: qkv bias gradient from the attention backward (CAAMD_FUSED_QKV_BGRAD) -- step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_qkvb
mkdir -p $O
for i in 1 2; do
  for f in 1 0; do
    CAAMD_FUSED_QKV_BGRAD=$f timeout -k 10 300 python -u bench.py --mode spmd > $O/bench_${f}_$i.log 2>&1 || { tail -5 $O/bench_${f}_$i.log; exit 1; }
    echo "fused_qkv_bgrad=$f $(grep -o '"value": [0-9.]*' $O/bench_${f}_$i.log)"
  done
done
