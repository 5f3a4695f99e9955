"""Our gemm.hip NT path vs hipBLASLt (torch's default heuristic and TunableOp's best
solution) on the plain (no-epilogue) NT GEMMs of the GPT-2-XL step, M = 32768.

    python tools/gemm_vs_blaslt.py [--tune]   -> one JSON line per shape and arm
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [  # name, N, K  (C[M,N] = A[M,K] B[N,K]^T)
    ("qkv_fwd", 4800, 1600), ("proj_fwd", 1600, 1600), ("fc_fwd_plain", 6400, 1600), ("fc2_fwd", 1600, 6400),
    ("qkv_dgrad", 1600, 4800), ("fc_dgrad", 1600, 6400), ("fc2_dgrad_plain", 6400, 1600),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best.append(s.elapsed_time(e) / iters * 1000)
    return min(best), sorted(best)[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--M", type=int, default=32768)
    a = ap.parse_args()
    from cluster_anywhere_amd.ops import gemm as G

    M = a.M
    if a.tune:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_max_tuning_duration(400)
        torch.cuda.tunable.set_filename("/tmp/tunable_r6.csv")
    for name, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        fl = 2.0 * M * N * K
        ref = F.linear(x.float()[:512], w.float())
        ours = G.linear_nt(x, w)
        err = ((ours[:512].float() - ref).norm() / ref.norm()).item()
        for arm, fn in (("ours", lambda: G.linear_nt(x, w)), ("blaslt", lambda: F.linear(x, w))):
            mn, med = timeit(fn)
            print(json.dumps({"shape": name, "N": N, "K": K, "arm": arm + ("_tuned" if a.tune and arm == "blaslt" else ""),
                              "us_min": round(mn, 1), "us_med": round(med, 1), "pfs": round(fl / med / 1e9, 3),
                              "rel_err_ours": round(err, 5)}), flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
