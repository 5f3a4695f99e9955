cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "layernorm or gpt2" > gpurun_out/pytest_ln.log 2>&1; rc=$?; echo "pytest ln rc=$rc"; tail -5 gpurun_out/pytest_ln.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_resnet.py --batch-size 512 > gpurun_out/bench_resnet.log 2>&1 || { tail -30 gpurun_out/bench_resnet.log; exit 2; }
tail -1 gpurun_out/bench_resnet.log
timeout -k 10 600 python bench.py > gpurun_out/bench_ln2.log 2>&1 || { tail -20 gpurun_out/bench_ln2.log; exit 3; }
tail -1 gpurun_out/bench_ln2.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_resnet -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --batch-size 512 --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_resnet.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_resnet.log; exit 4; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_resnet gpurun_out/prof_resnet_summary.md > /dev/null && head -45 gpurun_out/prof_resnet_summary.md
