"""The k64 full-line kernel's DMA-placement variants on the GPT-2-XL NT shapes
(M = 32768, bias epilogue where the step has one): algo 1009 (4 phases, DMA in
phase 0), 2009 (phases 0-1), 3009 (phases 0-2), 4009 (2 phases, DMA in phase 0; the
training default). One JSON line per shape and round with the time of each.

    python tools/gemm_k64_variants.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ALGOS = (1009, 2009, 3009, 4009)


def timeit(fn, iters=20):
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
    return round(sorted(out)[1], 1)


def main():
    from cluster_anywhere_amd.ops import gemm as G

    M = 32768
    for name, N, K, bias in (("qkv_fwd", 4800, 1600, True), ("fc_fwd_plain", 6400, 1600, False),
                             ("fc2_fwd", 1600, 6400, True), ("fc_dgrad", 1600, 6400, False),
                             ("qkv_dgrad", 1600, 4800, False), ("proj", 1600, 1600, True)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1 if bias else None
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        bm, bn = G.tile_for(M, N, K)
        ref = x[:256].float() @ w.float().t() + (b.float() if bias else 0.0)
        for rnd in range(2):
            row = {"shape": name, "N": N, "K": K, "round": rnd}
            for algo in ALGOS:
                G.run_pp(x, w, c, 0, G.EPI_BF16, bm, bn, bias=b, algo=algo)
                err = ((c[:256].float() - ref).norm() / ref.norm()).item()
                assert err < 5e-3, (name, algo, err)
                row[str(algo)] = timeit(lambda: G.run_pp(x, w, c, 0, G.EPI_BF16, bm, bn, bias=b, algo=algo))
            print(json.dumps(row), flush=True)
        del x, w, c
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
