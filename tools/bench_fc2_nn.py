"""fc2 forward from transposed storage: transpose + NT GEMM vs the NN layout
(32768 x 1600 x 6400, bias epilogue), with numerics vs fp32."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import gemm as G  # noqa: E402


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(n):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / n * 1e3


u = torch.randn(32768, 6400, device="cuda").bfloat16()
wt = (torch.randn(6400, 1600, device="cuda") * 0.02).bfloat16()
b = torch.randn(1600, device="cuda").bfloat16()
ref = u.float() @ wt.float() + b.float()
y_nt = G.linear_nt(u, G.transpose(wt), b)
y_nn = G.linear_nn(u, wt, b)
rel = lambda a: ((a.float() - ref).norm() / ref.norm()).item()  # noqa: E731
print(json.dumps({"transpose_us": round(t(lambda: G.transpose(wt)), 1),
                  "nt_us": round(t(lambda: G.linear_nt(u, G.transpose(wt), b)), 1),
                  "nn_us": round(t(lambda: G.linear_nn(u, wt, b)), 1),
                  "rel_nt": round(rel(y_nt), 5), "rel_nn": round(rel(y_nn), 5)}), flush=True)
