"""Micro-benchmarks of the HIP kernels vs the torch/library equivalents on the
GPT-2-XL training shapes (B=8, T=1024, H=25, D=64, d_model=1600)."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    from cluster_anywhere_amd.ops.flash import flash_attention_qkv

    B, T, H, D = 8, 1024, 25, 64
    res = {}
    qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    flops_fwd = 4 * B * H * T * T * D / 2

    def ours_fwd():
        return flash_attention_qkv(qkv, H, True)

    def sdpa_fwd():
        q, k, v = qkv.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
        return F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, H * D)

    for name, f in [("flash_ours", ours_fwd), ("sdpa_torch", sdpa_fwd)]:
        with torch.no_grad():
            ms = timeit(f)
        res[f"{name}_fwd_ms"] = round(ms, 3)
        res[f"{name}_fwd_TFs"] = round(flops_fwd / ms / 1e9, 1)
        o = f()
        do = torch.randn_like(o)

        def fb():
            qkv.grad = None
            f().backward(do)

        ms2 = timeit(fb)
        res[f"{name}_fwdbwd_ms"] = round(ms2, 3)
        res[f"{name}_fwdbwd_TFs"] = round(3.5 * flops_fwd / ms2 / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
