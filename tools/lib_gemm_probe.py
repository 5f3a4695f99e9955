"""Run the plain NT GEMMs of the GPT-2-XL step through torch with the shipped TunableOp
selections (ops/gemm_tuning.py), a few times each: under rocprofv3 --kernel-trace the
library kernel names (Tensile macro tile, depth, ...) and per-call times show up."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from cluster_anywhere_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
M = 32768
for N, K in ((4800, 1600), (1600, 1600), (6400, 1600), (1600, 6400), (1600, 4800)):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        F.linear(x, w)
    torch.cuda.synchronize()
    print(N, K, "done", flush=True)
