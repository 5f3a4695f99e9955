#!/bin/bash
# GPT-2-XL step kernel profile (current defaults) -> gpurun_out/prof_step/summary.md
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_step${TAG}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 $R/bench.py --mode spmd --steps 6 --warmup 2 > $O/step_bench.log 2>&1 || { echo "step prof failed"; tail -20 $O/step_bench.log; exit 1; }
tail -1 $O/step_bench.log | grep -o '"value": [0-9.]*'
python3 $R/tools/prof_summary.py $O/step $O/summary.md && sed -n '/Top kernels/,$p' $O/summary.md | head -24
