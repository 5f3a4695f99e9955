#!/bin/bash
# bench.py actor vs spmd mode on one box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mode_ab
for r in 1 2; do
for m in actor spmd; do
timeout -k 10 300 python -u bench.py --mode $m > gpurun_out/mode_ab/$m$r.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/mode_ab/$m$r.log; exit 1; }
echo "$m $(grep '"metric"' gpurun_out/mode_ab/$m$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
