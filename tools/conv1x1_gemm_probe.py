#!/usr/bin/env python
"""Would the full-line GEMM (algo 4009) beat conv.hip on the ResNet-50 1x1 stride-1
convs (plain NT GEMMs: NHWC input [pixels, Cin] x weight [Cout, Cin])? Times the
GEMM (bias epilogue) at each shape next to conv2d_nhwc (bias + ReLU)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import gemm as G  # noqa: E402
from cluster_anywhere_amd.ops.vision import conv2d_nhwc  # noqa: E402


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


# (N img, H, Cin, Cout)
SHAPES = [(512, 56, 64, 256), (512, 28, 128, 512), (512, 28, 512, 256), (512, 14, 256, 1024),
          (512, 14, 1024, 256), (512, 14, 1024, 512), (512, 7, 512, 2048), (512, 7, 2048, 512)]
for n, h, cin, cout in SHAPES:
    M = n * h * h
    x = torch.randn(n, h, h, cin, device="cuda").to(torch.bfloat16)
    w2d = (torch.randn(cout, cin, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.randn(cout, device="cuda").to(torch.bfloat16)
    conv_us = bench(lambda: conv2d_nhwc(x, w2d, b, 1, 1, 0, True, None))
    a2 = x.view(M, cin)
    row = {"shape": [n, h, cin, cout], "M": M, "conv_us": round(conv_us, 1)}
    for bn in (256, 320):
        if cout % bn == 0 and cin % 64 == 0:
            row[f"k64_{bn}_us"] = round(bench(lambda: G.gemm(a2, w2d, 0, algo=4009, tile=(256, bn))), 1)
    row["pp_us"] = round(bench(lambda: G.gemm(a2, w2d, 0, algo=2, tile=(256, 256))), 1) if cout % 256 == 0 else None
    print(json.dumps(row), flush=True)
