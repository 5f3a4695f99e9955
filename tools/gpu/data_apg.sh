#!/bin/bash
# Data e2e bench: actors per GPU sweep (same box)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_apg
mkdir -p $O
for i in 1 2; do for a in 3 4; do
  timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 --actors-per-gpu $a > $O/apg${a}_$i.log 2>&1 || { tail -20 $O/apg${a}_$i.log; exit 1; }
  echo "apg=$a run=$i $(grep -o '"value": [0-9.]*\|"time_to_first_batch_s": [0-9.]*\|"steady_state_rows_per_s": [0-9.]*' $O/apg${a}_$i.log | tr '\n' ' ')"
done; done
