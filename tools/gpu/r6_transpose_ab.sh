#!/bin/bash
# step A/B: dword-LDS transpose (default) vs the previous kernel (CAAMD_TRANSPOSE_V1=1)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/transpose_ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in 0 1; do
    CAAMD_TRANSPOSE_V1=$v timeout -k 10 300 python -u bench.py > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
    echo "v1=$v round $r: $(grep '"metric"' $O/b_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
