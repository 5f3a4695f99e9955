#!/bin/bash
# Round 3 Data path with the own implicit-GEMM conv: ResNet-50 kernel profile, then
# the end-to-end Data bench (actors per GPU 2/3, one timeline run for the host side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/data_r3
mkdir -p $O
timeout -k 10 300 python -u tools/bench_conv.py > $O/bench_conv.log 2>&1 || { echo "bench_conv failed"; tail -20 $O/bench_conv.log; exit 1; }
cat $O/bench_conv.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o resnet -- python3 tools/bench_resnet.py --iters 10 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $O/prof $O/resnet_prof.md > /dev/null 2>&1 || true
head -40 $O/resnet_prof.md
for a in 2 3; do
  timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 --actors-per-gpu $a > $O/apg$a.log 2>&1 || { echo "data apg=$a failed"; tail -20 $O/apg$a.log; exit 1; }
  echo "apg=$a $(grep -o '"value": [0-9.]*\|"time_to_first_batch_s": [0-9.]*\|"steady_state_rows_per_s": [0-9.]*' $O/apg$a.log | tr '\n' ' ')"
done
timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 204800 --actors-per-gpu 3 --timeline $O/timeline.json > $O/apg3_tl.log 2>&1 || { echo "timeline run failed"; tail -20 $O/apg3_tl.log; exit 1; }
grep -v "^{" $O/apg3_tl.log | tail -20
echo "apg=3 tl $(grep -o '"value": [0-9.]*\|"steady_state_rows_per_s": [0-9.]*' $O/apg3_tl.log | tr '\n' ' ')"
rm -f $O/timeline.json
