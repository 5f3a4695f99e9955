#!/bin/bash
# Round 5: GPU tests of the new pieces, then RLlib PPO FakeAtari with CPU vs GPU runners.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/rl_r5
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_reporter_gpu.py tests/test_rllib_gpu_runners.py tests/test_gpt2_parity_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|reporter gpus|worst grad|lowest update" $O/tests.log | cut -c1-600
timeout -k 10 200 python -u tools/bench_rllib.py --runners 12 --envs-per-runner 8 --seconds 30 > $O/rl_cpu.log 2>&1 || { echo "rl cpu failed"; tail -20 $O/rl_cpu.log; exit 1; }
tail -1 $O/rl_cpu.log
timeout -k 10 200 python -u tools/bench_rllib.py --runners 12 --envs-per-runner 8 --seconds 30 --runner-gpus 0.05 > $O/rl_gpu.log 2>&1 || { echo "rl gpu failed"; tail -20 $O/rl_gpu.log; exit 1; }
tail -1 $O/rl_gpu.log
