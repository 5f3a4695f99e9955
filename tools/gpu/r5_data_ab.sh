#!/bin/bash
# Data bench A/B: pixel-pair stem on / off, alternating
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
for ps in 1 0; do
CAAMD_RESNET_PAIR_STEM=$ps timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/ab_${ps}_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/ab_${ps}_$i.log; exit 1; }
echo "PAIR=$ps $(grep '"metric"' $O/ab_${ps}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','time_to_first_batch_s','steady_state_rows_per_s')})")"
done
done
