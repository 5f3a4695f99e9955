cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest gpu rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_tuned.log 2>&1 || { tail -20 gpurun_out/bench_tuned.log; exit 3; }
tail -1 gpurun_out/bench_tuned.log
CAAMD_TUNED_GEMMS=0 timeout -k 10 600 python bench.py > gpurun_out/bench_untuned.log 2>&1 || { tail -20 gpurun_out/bench_untuned.log; exit 4; }
tail -1 gpurun_out/bench_untuned.log
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof4.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof4.log; exit 5; }
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/prof4 gpurun_out/prof4_summary.md && head -40 gpurun_out/prof4_summary.md
