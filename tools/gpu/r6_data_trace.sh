#!/bin/bash
# Round 6: Data bench start-up timeline (actor init profile, first call) on 1 GPU
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/data_trace_r6
mkdir -p $O
cd $GRAFT_REPO_ROOT
CAAMD_BENCH_DATA_TRACE=1 timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/trace.log 2>&1 || { echo "bench failed"; tail -20 $O/trace.log; exit 1; }
grep -E "^T0|^FIRST|ACTOR_TIMES|ACTOR_FIRST_CALL|READ" $O/trace.log | head -40
grep '"metric"' $O/trace.log | cut -c1-600
