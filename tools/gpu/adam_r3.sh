#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/adam_r3
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k adamw > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/bench_adamw.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
