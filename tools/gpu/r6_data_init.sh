#!/bin/bash
# Data start-up A/B: fused weights drawn directly + worker HIP prewarm (default) vs the
# module init route without prewarm; alternating, then one traced run of the default
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_init
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_vision.py tests/test_conv_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', {k: d[k] for k in ('value','seconds','time_to_first_batch_s','steady_state_rows_per_s')})"; }
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/new_$i.log 2>&1 || { tail -20 $O/new_$i.log; exit 1; }
  grep '"metric"' $O/new_$i.log | summ new
  CAAMD_PREDICTOR_MODULE_INIT=1 CAAMD_WORKER_HIP_PREWARM=0 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/old_$i.log 2>&1 || { tail -20 $O/old_$i.log; exit 1; }
  grep '"metric"' $O/old_$i.log | summ old
done
CAAMD_BENCH_DATA_TRACE=1 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -E "ACTOR_TIMES|T0|FIRST|metric" $O/trace.log
