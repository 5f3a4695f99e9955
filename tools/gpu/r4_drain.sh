#!/bin/bash
# Round 4: fc bias gradient drained from a persistent fp32 accumulator into its main-grad
# (one launch instead of fill + convert + add) -- GPU suite, bench x2.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/drain
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_$i.log; exit 1; }
  echo "step: $(grep -o '"value": [0-9.]*' $O/bench_$i.log)"
done
