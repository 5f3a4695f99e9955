"""LM-head logits GEMM (16384 x 50432 x 1600, 256 x 256 tiles): ping-pong (algo 2)
vs full-line (algo 4009), interleaved rounds; numerics vs fp32 first."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import gemm as G  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    xs = []
    for _ in range(it):
        s.record()
        fn()
        e.record()
        e.synchronize()
        xs.append(s.elapsed_time(e) * 1e3)
    return sorted(xs)[len(xs) // 2]


M, N, K = 16384, 50432, 1600
a = torch.randn(M, K, device="cuda").bfloat16()
b = torch.randn(N, K, device="cuda").bfloat16()
ref = (a[:512].float() @ b.float().t())
for algo in (2, 4009):
    c = G.gemm(a, b, 0, algo=algo, tile=(256, 256))
    err = ((c[:512].float() - ref).norm() / ref.norm()).item()
    print(json.dumps({"algo": algo, "rel_err": err}), flush=True)
    assert err < 5e-3
for rnd in range(2):
    for algo in (2, 4009):
        us = t(lambda: G.gemm(a, b, 0, algo=algo, tile=(256, 256)))
        print(json.dumps({"algo": algo, "us": round(us, 1), "pfs": round(2 * M * N * K / us / 1e9, 3)}), flush=True)
