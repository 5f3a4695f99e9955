#!/bin/bash
# Round 5: default bench (actor mode) + kernel-trace profile of 6 SPMD steps.
# usage: r5_step.sh <tag> [extra bench commands run first]
set -o pipefail
TAG=${1:-step}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -n "$PRE" ]; then timeout -k 10 300 bash -c "$PRE" > $O/pre.log 2>&1 || { echo "pre failed"; tail -20 $O/pre.log; exit 1; }; cat $O/pre.log | grep -v amdgpu.ids; fi
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 $R/bench.py --mode spmd --steps 6 --warmup 2 > $O/step_bench.log 2>&1 || { echo "step prof failed"; tail -20 $O/step_bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/step_bench.log
python3 $R/tools/prof_summary.py $O/step $O/summary.md && sed -n '/Top kernels/,$p' $O/summary.md | head -24
