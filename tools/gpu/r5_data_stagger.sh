#!/bin/bash
# Data bench: staggered actor-pool start (CAAMD_DATA_ACTOR_STAGGER_S), alternating
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 51200 > $O/stag_warm.log 2>&1 || { echo "warm failed"; tail -20 $O/stag_warm.log; exit 1; }
for i in 1 2; do
for s in 0 0.15 0.3; do
CAAMD_DATA_ACTOR_STAGGER_S=$s timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/stag_${s}_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/stag_${s}_$i.log; exit 1; }
echo "STAGGER=$s $(grep '"metric"' $O/stag_${s}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','time_to_first_batch_s','steady_state_rows_per_s')})")"
done
done
