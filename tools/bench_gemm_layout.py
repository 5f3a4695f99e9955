#!/usr/bin/env python
"""Which operand layout makes the GPT-2-XL GEMMs fastest on hipBLASLt/gfx950?
For C[m,n] = sum_k A[m,k] B[k,n] time all four storage layouts of A and B
(row-major = k contiguous for A / n contiguous for B, or transposed)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    if os.environ.get("TUNED", "0") == "1":
        from cluster_anywhere_amd.ops.gemm_tuning import use_tuned_gemms
        use_tuned_gemms()
    M = 32768
    shapes = {  # name: (m, n, k)
        "qkv_wgrad": (4800, 1600, M), "proj_wgrad": (1600, 1600, M), "fc1_wgrad": (6400, 1600, M),
        "fc2_wgrad": (1600, 6400, M), "fc2_dgrad": (M, 6400, 1600), "fc1_dgrad": (M, 1600, 6400),
        "qkv_dgrad": (M, 1600, 4800), "proj_dgrad": (M, 1600, 1600), "fc1_fwd": (M, 6400, 1600),
    }
    for name, (m, n, k) in shapes.items():
        r = {"gemm": name, "m": m, "n": n, "k": k}
        for la in ("a_mk", "a_km"):
            A = torch.randn((m, k) if la == "a_mk" else (k, m), device="cuda", dtype=torch.bfloat16)
            Av = A if la == "a_mk" else A.t()
            for lb in ("b_kn", "b_nk"):
                B = torch.randn((k, n) if lb == "b_kn" else (n, k), device="cuda", dtype=torch.bfloat16)
                Bv = B if lb == "b_kn" else B.t()
                ms = timeit(lambda: torch.mm(Av, Bv))
                r[f"{la}/{lb}"] = round(2 * m * n * k / ms / 1e12, 3)  # PFLOP/s
                del B
            del A
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
