#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/fc2nn
mkdir -p $O
timeout -k 10 120 python tools/bench_fc2_nn.py > $O/bench.jsonl 2>&1 || { tail $O/bench.jsonl; exit 1; }
cat $O/bench.jsonl
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --mode spmd --steps 10 --warmup 3 > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
}
for r in 1 2; do
  run nn$r CAAMD_FC2_NN=1
  run nt$r
done
bash tools/gpu/prof_step_r3.sh
