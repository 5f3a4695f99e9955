"""Time the causal flash-attention kernels at the GPT-2-XL shape (B32 T1024 H25 D64).

    python tools/bench_attn.py            # current kernels
    CAAMD_FA_V1=1 python tools/bench_attn.py   # first-generation D=64 kernels

TF/s use the causal (useful) flop count: fwd 4*B*H*T*T/2*D, bwd 2.5x fwd.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops._lib import kernels  # noqa: E402

B, T, H, D = (int(v) for v in os.environ.get("ATTN_SHAPE", "32,1024,25,64").split(","))
if os.environ.get("ATTN_SO"):  # another build of the extension (same-box A/B of kernel versions)
    import importlib.machinery
    import importlib.util

    _ld = importlib.machinery.ExtensionFileLoader("caamd_ab._C", os.environ["ATTN_SO"])
    _spec = importlib.util.spec_from_loader("caamd_ab._C", _ld)
    C = importlib.util.module_from_spec(_spec)
    _ld.exec_module(C)
else:
    C = kernels()
qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16)
out, lse = C.flash_attn_fwd(qkv, H, True)
dout = torch.randn_like(out)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters * 1e3  # us


fwd_us = timeit(lambda: C.flash_attn_fwd(qkv, H, True))
bwd_us = timeit(lambda: C.flash_attn_bwd(qkv, out, dout, lse, H, True))
fl = 4.0 * B * H * T * T / 2 * D
print(json.dumps({"shape": [B, T, H, D], "v1": os.environ.get("CAAMD_FA_V1", "0") == "1",
                  "fwd_us": round(fwd_us, 1), "bwd_us": round(bwd_us, 1),
                  "fwd_tflops": round(fl / fwd_us / 1e6, 1), "bwd_tflops": round(2.5 * fl / bwd_us / 1e6, 1),
                  "per_layer_ms": round((fwd_us + bwd_us) / 1e3, 3)}), flush=True)
