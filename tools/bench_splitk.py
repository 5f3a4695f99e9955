#!/usr/bin/env python
"""Weight-gradient GEMM study: dW[N,K] += dY[M,N]^T X[M,K] with M = 32768 tokens.
These GEMMs have few output tiles (1600x4800 -> 133 tiles of 256x256 on a
256-CU chip), so a single GEMM under-fills the GPU. Compares the library GEMM
(with the shipped tuned table) against split-K over M as one batched GEMM
(s partial products, fp32 or bf16 partials) + reduction into the bf16 grad."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    use_tuned_gemms()
    M = 32768
    dev = "cuda"
    res = []
    for (N, K) in [(4800, 1600), (1600, 1600), (6400, 1600), (1600, 6400)]:
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        mg = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
        flop = 2 * M * N * K
        r = {"N": N, "K": K}
        r["addmm_ms"] = timeit(lambda: mg.addmm_(dy.t(), x))
        ref = (dy.float().t() @ x.float())
        for s in (2, 3, 4, 6, 8):
            if M % s:
                continue
            dys = dy.view(s, M // s, N).transpose(1, 2)
            xs = x.view(s, M // s, K)

            def f32():
                p = torch.bmm(dys, xs, out_dtype=torch.float32)
                mg.add_(p.sum(0))

            def bf16():
                p = torch.bmm(dys, xs)
                mg.add_(p.sum(0, dtype=torch.float32))
            try:
                r[f"bmm{s}_f32_ms"] = timeit(f32)
            except Exception as e:  # noqa: BLE001
                r[f"bmm{s}_f32_ms"] = str(e)[:80]
            r[f"bmm{s}_bf16_ms"] = timeit(bf16)
            if s == 4:
                p = torch.bmm(dys, xs).float().sum(0)
                r["bmm4_bf16_relerr"] = float((p - ref).norm() / ref.norm())
                r["addmm_relerr"] = float(((dy.t() @ x).float() - ref).norm() / ref.norm())
        best = min(v for k, v in r.items() if k.endswith("_ms") and isinstance(v, float))
        r["addmm_pflops"] = flop / r["addmm_ms"] / 1e12
        r["best_pflops"] = flop / best / 1e12
        res.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
