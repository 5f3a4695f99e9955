#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/k64_tests.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/k64_tests.log; exit 1; }
tail -1 gpurun_out/k64_tests.log
for r in 1 2; do
K64_KS=1600,3200 K64_ALGOS=4009 K64_SO=ab_so/_C_base.so timeout -k 10 200 python -u tools/k64_overhead.py > gpurun_out/k64_base.log 2>&1 || { tail -20 gpurun_out/k64_base.log; exit 1; }
grep '"so"' gpurun_out/k64_base.log
K64_KS=1600,3200 K64_ALGOS=4009 timeout -k 10 200 python -u tools/k64_overhead.py > gpurun_out/k64_new.log 2>&1 || { tail -20 gpurun_out/k64_new.log; exit 1; }
grep '"so"' gpurun_out/k64_new.log
done
