"""256 x 320 vs 256 x 256 full-line tiles (8 waves, 2 x 4) on the GPT-2-XL NT GEMMs
whose width both tiles divide (N = 6400: the fc forward and the fc2 dgrad), M = 32768,
alternating arms, one JSON line per shape and arm.

    python tools/gemm_tile_ab.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


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
    return min(out), sorted(out)[1]


def main():
    from cluster_anywhere_amd.ops import gemm as G

    M = 32768
    for name, N, K in (("fc_fwd_plain", 6400, 1600), ("fc2_dgrad_plain", 6400, 1600), ("fc_like_K6400", 6400, 6400)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        ref = x[:256].float() @ w.float().t()
        for rnd in range(2):
            for tile in ((256, 320), (256, 256)):
                y = G.gemm(x, w, tile=tile)
                err = ((y[:256].float() - ref).norm() / ref.norm()).item()
                mn, med = timeit(lambda: G.gemm(x, w, tile=tile))
                print(json.dumps({"shape": name, "N": N, "K": K, "tile": list(tile), "round": rnd,
                                  "us_min": round(mn, 1), "us_med": round(med, 1),
                                  "pfs": round(2.0 * M * N * K / med / 1e9, 3), "rel_err": round(err, 5)}), flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
