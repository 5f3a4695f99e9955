"""gemm.hip transpose_bf16_kernel on the GPT-2-XL weight shapes (W -> W^T for the
dgrad GEMMs): device time per call and bytes moved, checked against torch.

    python tools/bench_transpose.py   -> one JSON line per shape
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import gemm as G  # noqa: E402
from tools.gemm_algo_ab import timeit  # noqa: E402

for name, r, c in (("fc", 6400, 1600), ("fc2", 1600, 6400), ("qkv", 4800, 1600), ("proj", 1600, 1600)):
    w = torch.randn(r, c, device="cuda", dtype=torch.bfloat16)
    ok = torch.equal(G.transpose(w), w.t().contiguous())
    mn, med = timeit(lambda: G.transpose(w), iters=200)
    print(json.dumps({"shape": name, "R": r, "C": c, "us_min": round(mn, 2), "us_med": round(med, 2),
                      "TBps": round(2 * r * c * 2 / med / 1e6, 2), "equal": ok}), flush=True)
