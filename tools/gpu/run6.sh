cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_llm_gpu.py -q --timeout 300 -x > gpurun_out/pytest_llm_gpu.log 2>&1; rc=$?; echo "pytest llm rc=$rc"; tail -15 gpurun_out/pytest_llm_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/bench_llm.py --num-prompts 128 --input-len 512 --output-len 128 > gpurun_out/bench_llm.log 2>&1 || { tail -20 gpurun_out/bench_llm.log; exit 2; }
tail -1 gpurun_out/bench_llm.log
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest all rc=$?"; tail -4 gpurun_out/pytest_gpu.log
