#!/bin/bash
# End-of-work check on the current tree: full GPU suite + smoke, default bench
# (actor mode, the driver's invocation), Data e2e with the own conv.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/final_r3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
grep '"metric"' $O/bench_default.log
timeout -k 10 300 python -u tools/bench_data.py --gpus 1 --rows 409600 --actors-per-gpu 3 > $O/data.log 2>&1 || { echo "data failed"; tail -20 $O/data.log; exit 1; }
grep -o '"value": [0-9.]*\|"time_to_first_batch_s": [0-9.]*\|"steady_state_rows_per_s": [0-9.]*' $O/data.log | tr '\n' ' '; echo
