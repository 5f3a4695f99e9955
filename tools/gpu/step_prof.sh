set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/step_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/step_prof/kt -o run -- python3 $R/bench.py --mode spmd --steps 5 --warmup 1 > $R/gpurun_out/step_prof/bench.log 2>&1
echo prof=$?; tail -1 $R/gpurun_out/step_prof/bench.log
python3 $R/tools/prof_summary.py $R/gpurun_out/step_prof/kt $R/gpurun_out/step_prof/summary.md && head -30 $R/gpurun_out/step_prof/summary.md
