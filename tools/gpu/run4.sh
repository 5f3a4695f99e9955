cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_mbs8.log 2>&1 || exit 3
tail -1 gpurun_out/bench_mbs8.log
CAAMD_MBS=16 timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_mbs16.log 2>&1 || exit 4
tail -1 gpurun_out/bench_mbs16.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1 || exit 5
echo prof ok
