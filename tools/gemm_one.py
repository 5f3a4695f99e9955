"""Run one GEMM shape/algorithm a few times (for rocprofv3 counter passes)."""
import sys

import torch

sys.path.insert(0, ".")
from tools.gemm_dev import mk, run  # noqa: E402

layout, M, N, K, bm, bn, algo = (int(x) for x in sys.argv[1:8])
a, b = mk(layout, M, N, K)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    run(layout, a, b, bm, bn, out=c, algo=algo)
torch.cuda.synchronize()
