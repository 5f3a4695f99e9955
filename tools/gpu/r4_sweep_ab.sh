#!/bin/bash
# Round 4: same-box check that the /dev/shm sweep at init does not move the bench (sweep on / off).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/sweep_ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/on_$i.log 2>&1 || { tail -5 $O/on_$i.log; exit 1; }
  echo "sweep on: $(grep -o '"value": [0-9.]*' $O/on_$i.log)"
  timeout -k 10 300 python -u -c "
import runpy, sys
import cluster_anywhere_amd.core.api as a
a._sweep_stale_stores = lambda: 0
sys.argv = ['bench.py']
runpy.run_path('bench.py', run_name='__main__')" > $O/off_$i.log 2>&1 || { tail -5 $O/off_$i.log; exit 1; }
  echo "sweep off: $(grep -o '"value": [0-9.]*' $O/off_$i.log)"
done
