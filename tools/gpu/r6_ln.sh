#!/bin/bash
# Round 6: LayerNorm backward (step form with dxsum) row-batch / grid variants, then step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_ln
mkdir -p $O
timeout -k 10 300 python -u tools/bench_ln_bwd.py > $O/ln.jsonl 2>&1 || { tail -5 $O/ln.jsonl; exit 1; }
grep dxsum $O/ln.jsonl
