cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -4 gpurun_out/pytest_gpu.log
for mbs in 8 16 32; do
CAAMD_MBS=$mbs timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_mbs$mbs.log 2>&1 || exit 3
tail -1 gpurun_out/bench_mbs$mbs.log | cut -c1-200
done
cd /tmp && CAAMD_MBS=16 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1 || exit 5
echo prof ok
