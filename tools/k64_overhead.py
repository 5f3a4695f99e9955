#!/usr/bin/env python
"""Per-tile fixed cost of the full-line k64 GEMM (prologue DMA + epilogue +
workgroup turnover): time 32768 x 6400 x K for several K (the slope is the main
loop, the intercept the per-tile overhead) and the no-epilogue-store ablation."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import gemm as G  # noqa: E402

if os.environ.get("K64_SO"):  # another build of the extension (same-box A/B of kernel versions)
    import importlib.machinery
    import importlib.util

    _ld = importlib.machinery.ExtensionFileLoader("caamd_ab._C", os.environ["K64_SO"])
    _spec = importlib.util.spec_from_loader("caamd_ab._C", _ld)
    _C = importlib.util.module_from_spec(_spec)
    _ld.exec_module(_C)
    G.kernels = lambda: _C
KS = [int(k) for k in os.environ.get("K64_KS", "128,256,512,1024,1600,3200").split(",")]
ALGOS = [int(a) for a in os.environ.get("K64_ALGOS", "4009,4089,4019").split(",")]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


M, N = 32768, 6400
for K in KS:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for algo in ALGOS:
        us = bench(lambda: G.gemm(a, b, 0, algo=algo, tile=(256, 320)))
        print(json.dumps({"so": os.environ.get("K64_SO", "tree"), "M": M, "N": N, "K": K, "algo": algo, "us": round(us, 1),
                          "pfs": round(2 * M * N * K / us / 1e9, 3)}), flush=True)
