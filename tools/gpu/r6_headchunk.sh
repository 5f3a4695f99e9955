#!/bin/bash
# LM-head chunk rows A/B on the default bench (alternating on one box)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/headchunk
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for c in 16384 32768 8192; do
    CAAMD_HEAD_CHUNK=$c timeout -k 10 300 python -u bench.py > $O/b_${c}_$r.log 2>&1 || { tail -20 $O/b_${c}_$r.log; exit 1; }
    echo "chunk $c round $r: $(grep '"metric"' $O/b_${c}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
  done
done
