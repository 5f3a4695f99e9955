cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_vision.py -m gpu -x -v --timeout 200 --timeout-method thread -k "layernorm or gpt2 or vision or bias_act or resnet or predictor or normalize" > gpurun_out/pytest_12.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_12.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_resnet.py --batch-size 512 > gpurun_out/bench_resnet2.log 2>&1 || { tail -30 gpurun_out/bench_resnet2.log; exit 2; }
tail -1 gpurun_out/bench_resnet2.log
timeout -k 10 600 python bench.py > gpurun_out/bench_ln3.log 2>&1 || { tail -20 gpurun_out/bench_ln3.log; exit 3; }
tail -1 gpurun_out/bench_ln3.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_resnet2 -o run -- python $GRAFT_REPO_ROOT/tools/bench_resnet.py --batch-size 512 --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_resnet2.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_resnet2.log; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ln3 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_ln3.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_ln3.log; exit 5; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_resnet2 gpurun_out/prof_resnet2_summary.md > /dev/null && head -30 gpurun_out/prof_resnet2_summary.md && python tools/prof_summary.py gpurun_out/prof_ln3 gpurun_out/prof_ln3_summary.md > /dev/null && head -24 gpurun_out/prof_ln3_summary.md
