#!/bin/bash
# Data start-up: the predictor's weights from one seg_fill_ launch vs torch randn /
# foreach / cast (CAAMD_PREDICTOR_SEG_FILL=0), both with the worker HIP prewarm
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_init3
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_vision.py tests/test_conv_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
timeout -k 10 120 python -u tools/probe_fused_random.py > $O/fr.jsonl 2>&1 || { tail -5 $O/fr.jsonl; exit 1; }
cat $O/fr.jsonl
summ() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', {k: d[k] for k in ('value','seconds','time_to_first_batch_s','steady_state_rows_per_s')})"; }
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/new_$i.log 2>&1 || { tail -20 $O/new_$i.log; exit 1; }
  grep '"metric"' $O/new_$i.log | summ seg_fill
  CAAMD_PREDICTOR_SEG_FILL=0 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/old_$i.log 2>&1 || { tail -20 $O/old_$i.log; exit 1; }
  grep '"metric"' $O/old_$i.log | summ torch_init
done
CAAMD_BENCH_DATA_TRACE=1 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -E "ACTOR_TIMES|T0|FIRST|metric" $O/trace.log
