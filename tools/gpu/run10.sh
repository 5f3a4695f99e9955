cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vision.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_vision.log 2>&1; rc=$?; echo "pytest vision rc=$rc"; tail -12 gpurun_out/pytest_vision.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/bench_data.py --gpus 1 --rows 30000 --batch-size 512 > gpurun_out/bench_data.log 2>&1 || { tail -30 gpurun_out/bench_data.log; exit 2; }
tail -1 gpurun_out/bench_data.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_data -o run -- python $GRAFT_REPO_ROOT/tools/bench_data.py --gpus 1 --rows 8192 --batch-size 512 > $GRAFT_REPO_ROOT/gpurun_out/prof_data.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_data.log; exit 3; }
ls -R $GRAFT_REPO_ROOT/gpurun_out/prof_data | head -20
