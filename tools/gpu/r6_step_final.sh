#!/bin/bash
# Round 6, final tree: step kernel profile (rocprofv3 kernel trace + stats), SPMD mode
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/step_final
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 $R/bench.py --mode spmd --steps 6 --warmup 2 > $O/step_bench.log 2>&1 || { echo "step prof failed"; tail -20 $O/step_bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/step_bench.log
python3 $R/tools/prof_summary.py $O/step $O/summary.md && sed -n '/Top kernels/,$p' $O/summary.md | head -30
