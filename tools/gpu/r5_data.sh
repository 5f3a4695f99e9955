#!/bin/bash
# Round 5: Data bench (ResNet-50 map_batches, 1 GPU) with the actor start-up timeline.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vision.py tests/test_conv_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u tools/predictor_init_prof.py > $O/init.log 2>&1 || { tail -20 $O/init.log; exit 1; }
cat $O/init.log
for i in 1 2; do
CAAMD_BENCH_DATA_TRACE=1 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_$i.log; exit 1; }
grep '"metric"' $O/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','seconds','time_to_first_batch_s','steady_state_rows_per_s')})"
done
