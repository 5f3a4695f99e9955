#!/bin/bash
# Round 4: LayerNorm weight / bias gradients accumulated into their main-grads inside the
# backward's column-sum launch -- GPU suite, bench, kernel profile of the step.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ln_main
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_$i.log; exit 1; }
  echo "step: $(grep -o '"value": [0-9.]*' $O/bench_$i.log)"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 $R/bench.py --mode spmd --steps 6 --warmup 2 > $O/step_bench.log 2>&1 || { echo "step prof failed"; tail -20 $O/step_bench.log; exit 1; }
python3 $R/tools/prof_summary.py $O/step $O/summary.md && sed -n '/Top kernels/,$p' $O/summary.md | head -40
