#!/bin/bash
# greedy argmax kernel: tests + timing at [128, 128256]
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py -m gpu -k "argmax or engine" > gpurun_out/argmax_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/argmax_tests.log; exit 1; }
tail -1 gpurun_out/argmax_tests.log
timeout -k 10 120 python -u - <<'PY'
import torch
from cluster_anywhere_amd.ops._lib import kernels
x = torch.randn(128, 128256, device="cuda").bfloat16()
C = kernels()
for _ in range(5): C.argmax_rows(x)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(50): C.argmax_rows(x)
e.record(); e.synchronize()
print("argmax_rows us", round(s.elapsed_time(e) / 50 * 1e3, 2))
PY
