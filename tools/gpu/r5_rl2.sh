#!/bin/bash
# Round 5: RLlib PPO FakeAtari (native batched env): CPU runners vs a few GPU runners.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/rl2_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 200 python -u tools/bench_rllib.py --seconds 25 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }; grep '"metric"' $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['sample_s'], d['learn_s'], d['config']['runner_device'], d['config']['weights_transport'])"; }
run cpu12x8 --runners 12 --envs-per-runner 8
run gpu4x64 --runners 4 --envs-per-runner 64 --runner-gpus 0.1
run gpu6x48 --runners 6 --envs-per-runner 48 --runner-gpus 0.1
run gpu4x96 --runners 4 --envs-per-runner 96 --runner-gpus 0.1
