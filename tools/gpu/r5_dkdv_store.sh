#!/bin/bash
# dK/dV kernel time with / without its dK / dV stores (ABL bit 5) and with the
# LDS-staged whole-row stores (OPT bit 3), production and stripped
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CAAMD_FA64_DKDV_OPT=8 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "flash or attention" > gpurun_out/dkdv_st_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/dkdv_st_tests.log; exit 1; }
tail -1 gpurun_out/dkdv_st_tests.log
for v in 0:0 32:0 0:8 0:12 31:0 63:0 95:0; do
a=${v%:*}; o=${v#*:}
CAAMD_FA64_BWD_ABL=$a CAAMD_FA64_DKDV_OPT=$o timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/st${a}_$o -o run -- python3 -u tools/bench_attn.py > gpurun_out/st${a}_$o.log 2>&1 || { echo "abl $a failed"; tail -20 gpurun_out/st${a}_$o.log; exit 1; }
echo "ABL=$a OPT=$o $(grep bwd_us gpurun_out/st${a}_$o.log)"
done
