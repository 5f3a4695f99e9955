"""Weight-gradient GEMM timings at 32768 tokens (GPT-2-XL shapes): gemm.hip
stream-K / lockstep orders at several run counts vs hipBLASLt (torch.mm).

    python tools/wgrad_bench.py [--iters 20] > out.jsonl
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
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
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--ksweep", action="store_true", help="proj / fc wgrad at several token counts (fixed runs)")
    a = ap.parse_args()
    from cluster_anywhere_amd.ops import gemm as G

    if a.ksweep:
        for (M, N, runs) in ((1600, 1600, 245), (1600, 1600, 210), (6400, 1600, 250), (4800, 1600, 190)):
            for K in (8192, 32768):
                dy = torch.randn(K, M, device="cuda").bfloat16()
                x = torch.randn(K, N, device="cuda").bfloat16()
                c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                for ext in (True, False):
                    G.WGRAD_EXT = ext
                    med, mn = timeit(lambda: G.run_sk(dy, x, c, 2, True, runs), a.iters)
                    print(json.dumps({"M": M, "N": N, "K": K, "impl": "sk", "runs": runs, "ext": ext,
                                      "us_med": round(med, 1), "us_min": round(mn, 1),
                                      "pfs": round(2.0 * M * N * K / med / 1e9, 3)}), flush=True)
        return

    K = a.tokens
    cases = {(1600, 1600): [140, 175, 210, 245], (6400, 1600): [250], (4800, 1600): [190, 228]}
    for (M, N), runs_list in cases.items():
        dy = torch.randn(K, M, device="cuda").bfloat16()
        x = torch.randn(K, N, device="cuda").bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        med, mn = timeit(lambda: torch.mm(dy.t(), x, out=c), a.iters)
        print(json.dumps({"M": M, "N": N, "K": K, "impl": "hipblaslt", "us_med": round(med, 1),
                          "pfs": round(fl / med / 1e9, 3)}), flush=True)
        for runs in runs_list:
            for ls in (True, False):
                G.WGRAD_LOCKSTEP = ls
                med, mn = timeit(lambda: G.run_sk(dy, x, c, 2, False, runs), a.iters)
                print(json.dumps({"M": M, "N": N, "K": K, "impl": "sk", "runs": runs, "lockstep": ls,
                                  "us_med": round(med, 1), "us_min": round(mn, 1),
                                  "pfs": round(fl / med / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
