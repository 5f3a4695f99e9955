#!/bin/bash
# Round 6: Data bench (ResNet-50 map_batches, 1 GPU, 204800 rows), two runs
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_r6
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/bench_final_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_final_$i.log; exit 1; }
grep '"metric"' $O/bench_final_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','seconds','time_to_first_batch_s','steady_state_rows_per_s')})"
done
