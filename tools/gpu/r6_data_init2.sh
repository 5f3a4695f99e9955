#!/bin/bash
# Data start-up: worker HIP prewarm through ctypes (GIL released) on top of the directly
# drawn fused weights, vs no prewarm; alternating, then one traced run of the default
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_init2
mkdir -p $O
cd $GRAFT_REPO_ROOT
summ() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', {k: d[k] for k in ('value','seconds','time_to_first_batch_s','steady_state_rows_per_s')})"; }
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/new_$i.log 2>&1 || { tail -20 $O/new_$i.log; exit 1; }
  grep '"metric"' $O/new_$i.log | summ prewarm
  CAAMD_WORKER_HIP_PREWARM=0 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/old_$i.log 2>&1 || { tail -20 $O/old_$i.log; exit 1; }
  grep '"metric"' $O/old_$i.log | summ no_prewarm
done
CAAMD_BENCH_DATA_TRACE=1 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -E "ACTOR_TIMES|T0|FIRST|metric" $O/trace.log
