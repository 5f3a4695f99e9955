"""Weight-gradient GEMM study at the GPT-2-XL shapes (dW[out, in] += dY^T X, K = 32768
tokens): hipBLASLt addmm_ vs the hand-written MFMA kernel in layout 2 (both operands
read K-rows, transposed in LDS by ds_read_b64_tr_b16) with split-K partial slabs.

    python tools/bench_wgrad.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops._lib import kernels  # noqa: E402

C = kernels()
TOK = 32768


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters * 1e3


for name, out_f, in_f in (("fc", 6400, 1600), ("fc2", 1600, 6400), ("qkv", 4800, 1600), ("proj", 1600, 1600)):
    dy = torch.randn(TOK, out_f, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(TOK, in_f, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(out_f, in_f, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * TOK * out_f * in_f
    row = {"gemm": name, "M": out_f, "N": in_f}
    row["hipblaslt_us"] = round(timeit(lambda: g.addmm_(dy.t(), x)), 1)
    ref = (dy.float().t() @ x.float())
    # ours: C[M=out, N=in] with A = dy [K, M], B = x [K, N]
    for (bm, bn) in ((256, 320), (256, 256), (128, 320)):
        if out_f % bm or in_f % bn:
            continue
        for sk in (1, 2, 3, 4, 6):
            ws = torch.empty(sk * out_f * in_f, device="cuda", dtype=torch.float32)
            for algo in (0, 2):
                c = torch.zeros(out_f, in_f, device="cuda", dtype=torch.bfloat16)
                fn = lambda: C.gemm_bf16(dy, x, c, 2, 0, bm, bn, None, None, None, None, sk,
                                          ws if sk > 1 else None, False, algo)
                try:
                    us = timeit(fn)
                except Exception as e:  # noqa: BLE001
                    row[f"{bm}x{bn}_s{sk}_a{algo}"] = str(e)[:60]
                    continue
                err = ((c.float() - ref).norm() / ref.norm()).item()
                row[f"{bm}x{bn}_s{sk}_a{algo}"] = [round(us, 1), round(fl / us / 1e9, 3), round(err, 4)]
            del ws
    print(json.dumps(row), flush=True)
