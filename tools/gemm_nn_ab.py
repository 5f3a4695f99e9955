"""NN kernel (gemm.hip algo 27: x @ W with W read as stored) vs the transpose + NT
path it replaces, on the GPT-2-XL input-gradient shapes (M = 32768 tokens), and the
NT kernel alone (what the transpose feeds). One JSON line per shape and round.

    python tools/gemm_nn_ab.py
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
    return round(sorted(out)[1], 1)


def main():
    from cluster_anywhere_amd.ops import gemm as G

    M = 32768
    # (name, N_out, K_in): dx [M, K_in] = dy [M, N_out] @ W [N_out, K_in]
    for name, n_out, k_in in (("qkv_dgrad", 4800, 1600), ("proj_dgrad", 1600, 1600), ("fc_dgrad", 6400, 1600),
                              ("fc2_fwd_from_T", 6400, 1600)):
        dy = torch.randn(M, n_out, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(n_out, k_in, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = G.transpose(w)
        ref = dy[:256].float() @ w.float()
        err = ((G.dgrad_w(dy, w)[:256].float() - ref).norm() / ref.norm()).item()
        for rnd in range(2):
            row = {"shape": name, "M": M, "N": k_in, "K": n_out, "round": rnd, "rel_err_nn": round(err, 5),
                   "nn_us": timeit(lambda: G.linear_nn64(dy, w)),
                   "transpose_plus_nt_us": timeit(lambda: G.dgrad(dy, G.transpose(w))),
                   "nt_only_us": timeit(lambda: G.dgrad(dy, wt)),
                   "transpose_us": timeit(lambda: G.transpose(w))}
            print(json.dumps(row), flush=True)
        del dy, w, wt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
