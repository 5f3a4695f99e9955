"""Llama-3-8B prefill GEMMs at 16384 tokens: hipBLASLt (F.linear on the nn.Linear
weight, the shipped tuned selections) vs gemm.hip reading the packed decode
weights (ops/gemm.py prefill_linear) per full-line variant, incl. the fused
SwiGLU / residual epilogues vs their unfused library equivalents.

    python tools/bench_prefill_gemm.py [--tokens 16384] > out.jsonl
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--algos", default="4009,9,1009,3009")
    a = ap.parse_args()
    from cluster_anywhere_amd.ops import gemm as G
    from cluster_anywhere_amd.ops import llm as L
    from cluster_anywhere_amd.ops.gemm_tuning import use_tuned_gemms

    use_tuned_gemms()
    M = a.tokens
    shapes = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 1), "gate_up": (28672, 4096, 5), "down": (4096, 14336, 1)}
    for name, (N, K, epi) in shapes.items():
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        r = torch.randn(M, N, device="cuda").bfloat16()
        fl = 2.0 * M * N * K
        if epi == 5:
            lib = lambda: L.silu_mul(F.linear(x, w))  # noqa: E731
        elif epi == 1:
            lib = lambda: torch.add(F.linear(x, w), r)  # noqa: E731
        else:
            lib = lambda: F.linear(x, w)  # noqa: E731
        us = timeit(lib)
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "impl": "hipblaslt+unfused", "us": round(us, 1),
                          "pfs": round(fl / us / 1e9, 3)}), flush=True)
        us = timeit(lambda: F.linear(x, w))
        print(json.dumps({"gemm": name, "impl": "hipblaslt gemm only", "us": round(us, 1),
                          "pfs": round(fl / us / 1e9, 3)}), flush=True)
        wp = L.pack_decode_weight(L.interleave_gate_up(w) if epi == 5 else w)
        for algo in [int(t) for t in a.algos.split(",")]:
            G.PREFILL_ALGO, G._PREFILL_ALGO_FORCED = algo, True
            out = r.clone()
            if epi == 5:
                fn = lambda: G.prefill_linear(x, wp, epi=G.EPI_SWIGLU)  # noqa: E731
            elif epi == 1:
                fn = lambda: G.prefill_linear(x, wp, out=out, accumulate=True)  # noqa: E731
            else:
                fn = lambda: G.prefill_linear(x, wp)  # noqa: E731
            us = timeit(fn)
            print(json.dumps({"gemm": name, "impl": f"gemm.hip algo {algo} packed", "us": round(us, 1),
                              "pfs": round(fl / us / 1e9, 3)}), flush=True)
        del x, w, r, wp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
