#!/bin/bash
# Data bench: actors per GPU 3 (default) vs 4 vs 2, alternating on one box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_apg
mkdir -p $O
cd $GRAFT_REPO_ROOT
summ() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', {k: d[k] for k in ('value','seconds','time_to_first_batch_s','steady_state_rows_per_s')})"; }
for i in 1 2; do
  for a in 3 4 2; do
    timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 --actors-per-gpu $a > $O/b_${a}_$i.log 2>&1 || { tail -20 $O/b_${a}_$i.log; exit 1; }
    grep '"metric"' $O/b_${a}_$i.log | summ apg=$a
  done
done
