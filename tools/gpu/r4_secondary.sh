#!/bin/bash
# Round 4 secondary benches: Data map_batches ResNet-50 (1 GPU) and RLlib PPO FakeAtari.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/secondary_r4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/bench_data.py --gpus 1 --rows 204800 > $O/data.log 2>&1 || { echo "data bench failed"; tail -10 $O/data.log; exit 1; }
grep '"metric"' $O/data.log
timeout -k 10 300 python -u tools/bench_rllib.py --runners 14 --envs-per-runner 8 --seconds 60 > $O/rllib.log 2>&1 || { echo "rllib bench failed"; tail -10 $O/rllib.log; exit 1; }
grep '"metric"' $O/rllib.log
