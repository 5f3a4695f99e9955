#!/bin/bash
# three default bench.py runs on one box (variance record)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bench_runs
for r in 1 2 3; do
timeout -k 10 300 python -u bench.py > gpurun_out/bench_runs/b$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_runs/b$r.log; exit 1; }
echo "run$r $(grep '"metric"' gpurun_out/bench_runs/b$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
