"""Ping-pong (algo 2) vs full-line (algo 4009) gemm.hip kernels on the GPT-2-XL NT
shapes below the full-line kernel's max(N, K) >= 4096 rule (the 1600 x 1600
attention projection, forward and dgrad), M = 32768, alternating arms.

    python tools/gemm_algo_ab.py   -> one JSON line per shape, algo and round
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e) / iters * 1000)
    return min(out), sorted(out)[1]


def main():
    from cluster_anywhere_amd.ops import gemm as G

    M = 32768
    for name, N, K in (("proj", 1600, 1600), ("qkv_fwd", 4800, 1600)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
        ref = x[:256].float() @ w.float().t() + b.float()
        bm, bn = G.tile_for(M, N, K)
        for rnd in range(2):
            for algo in (2, 4009):
                def f():
                    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                    return G.run_pp(x, w, c, 0, G.EPI_BF16, bm, bn, bias=b, algo=algo)
                y = f()
                err = ((y[:256].float() - ref).norm() / ref.norm()).item()
                mn, med = timeit(f)
                print(json.dumps({"shape": name, "N": N, "K": K, "algo": algo, "round": rnd, "us_min": round(mn, 1),
                                  "us_med": round(med, 1), "pfs": round(2.0 * M * N * K / med / 1e9, 3),
                                  "rel_err": round(err, 5)}), flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
