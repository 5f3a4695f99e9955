#!/bin/bash
# same-box A/B of ResNetPredictor start-up variants in the Data e2e bench:
# L = lazy graph capture (CAAMD_PREDICTOR_LAZY_CAPTURE), P = arena pinning started in __init__ (CAAMD_PREDICTOR_EARLY_PIN)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_ab
mkdir -p $O
for i in 1 2; do
  for v in "1 1" "1 0" "0 0"; do
    set -- $v
    CAAMD_PREDICTOR_LAZY_CAPTURE=$1 CAAMD_PREDICTOR_EARLY_PIN=$2 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/L$1P$2_$i.log 2>&1 || { tail -20 $O/L$1P$2_$i.log; exit 1; }
    echo "L$1 P$2 run=$i $(grep -o '"value": [0-9.]*\|"time_to_first_batch_s": [0-9.]*\|"steady_state_rows_per_s": [0-9.]*' $O/L$1P$2_$i.log | tr '\n' ' ')"
  done
done
