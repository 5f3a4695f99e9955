"""Decode GEMMs of Llama-3-8B (batch 128): hipBLASLt F.linear vs the weight-streaming
MFMA kernel (skinny_gemm.hip). Prints per-shape us and weight-stream TB/s."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402
from cluster_anywhere_amd.ops.llm import skinny_linear as decode_linear, skinny_splits  # noqa: E402

use_tuned_gemms()
M = int(os.environ.get("DECODE_M", "128"))
COLD = os.environ.get("DECODE_COLD", "1") == "1"


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters * 1e3


tot = {"hipblaslt": 0.0, "ours": 0.0}
for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
                   ("lm_head", 128256, 4096)):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    if COLD:
        # rotate over enough weight copies (>= 1 GB) that every call streams from HBM,
        # as in a decode step (one layer's weights are evicted by the other 31 layers'
        # before they are read again); the 256 MB MALL would otherwise serve small W
        nw = max(2, -(-(1 << 30) // (N * K * 2)))
        ws = [w] + [w.clone() for _ in range(nw - 1)]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % nw
            return ws[it[0]]

        a = timeit(lambda: F.linear(x, nxt()))
        b = timeit(lambda: decode_linear(x, nxt()))
    else:
        a = timeit(lambda: F.linear(x, w))
        b = timeit(lambda: decode_linear(x, w))
    err = ((decode_linear(x, w).float() - F.linear(x, w).float()).norm() / F.linear(x, w).float().norm()).item()
    gb = N * K * 2 / 1e9
    if name != "lm_head":
        tot["hipblaslt"] += a
        tot["ours"] += b
    print(json.dumps({"gemm": name, "M": M, "cold": COLD, "N": N, "K": K, "splits": skinny_splits(N, K),
                      "hipblaslt_us": round(a, 1), "ours_us": round(b, 1),
                      "hipblaslt_TBps": round(gb / a * 1e3, 2), "ours_TBps": round(gb / b * 1e3, 2),
                      "rel_err": round(err, 5)}), flush=True)
print(json.dumps({"per_layer_us": {k: round(v, 1) for k, v in tot.items()}}))
