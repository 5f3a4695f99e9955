cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k flash > gpurun_out/pytest_flash.log 2>&1; FRC=$?
echo "flash rc=$FRC"; tail -5 gpurun_out/pytest_flash.log
if [ $FRC -eq 134 ] || [ $FRC -eq 139 ] || [ $FRC -eq 124 ] || [ $FRC -eq 137 ]; then exit 5; fi
timeout -k 10 600 python -m pytest tests -m gpu -q -k "not flash" > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
if [ $FRC -ne 0 ]; then export CAAMD_ATTN=sdpa; fi
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels.log 2>&1; echo "kb rc=$?"; tail -2 gpurun_out/bench_kernels.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench2.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench2.log
