#!/bin/bash
# Round 4: LayerNorm backward with the merged column-sum launch -- numerics + GPT-2 step tests + bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ln_r4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -10 $O/bench_$i.log; exit 1; }
  echo "step: $(grep -o '"value": [0-9.]*' $O/bench_$i.log)"
done
