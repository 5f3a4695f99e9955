#!/bin/bash
# De-phased full-line GEMM launches: tests, standalone A/B, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
CAAMD_GEMM_DEPHASE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_gpt2_parity_gpu.py > gpurun_out/dephase_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/dephase_tests.log; exit 1; }
tail -1 gpurun_out/dephase_tests.log
for r in 1 2; do
for d in 0 1; do
CAAMD_GEMM_DEPHASE=$d K64_KS=1600,3200 K64_ALGOS=4009 timeout -k 10 200 python -u tools/k64_overhead.py > gpurun_out/dephase_$d.log 2>&1 || { tail -20 gpurun_out/dephase_$d.log; exit 1; }
echo "DEPHASE=$d"; grep '"so"' gpurun_out/dephase_$d.log
done
done
bash tools/gpu/r5_ab.sh "CAAMD_GEMM_DEPHASE=1" "CAAMD_GEMM_DEPHASE=0" 2
