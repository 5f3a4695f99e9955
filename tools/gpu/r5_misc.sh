#!/bin/bash
# Round 5: new GPU tests (learner IPC hand-off, vision) then the step PMC table.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/misc_r5
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rllib_learner_ipc_gpu.py tests/test_vision.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/gpu/r5_step_pmc.sh
