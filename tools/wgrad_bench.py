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
    ap.add_argument("--tn", action="store_true", help="TN full-line kernel (algo 25) vs stream-K vs hipBLASLt")
    ap.add_argument("--head", action="store_true", help="LM-head weight gradient (50432 x 1600, 16384-token chunk)")
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
    if a.head:
        M, N, Kc = 50432, 1600, 16384
        dy = torch.randn(Kc, M, device="cuda").bfloat16()
        x = torch.randn(Kc, N, device="cuda").bfloat16()
        c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * Kc
        rows = []
        for rnd in range(2):
            med, _ = timeit(lambda: G.run_sk(dy, x, c, 2, True), a.iters)
            rows.append(("sk", "auto", med))
            for (bm, S) in ((256, 1), (192, 1)):
                med, _ = timeit(lambda: G.run_tn(dy, x, c, True, bm, S), a.iters)
                rows.append(("tn64", f"{bm}x{S}", med))
        for impl, cfg, med in rows:
            print(json.dumps({"M": M, "N": N, "K": Kc, "impl": impl, "cfg": cfg, "us_med": round(med, 1),
                              "pfs": round(fl / med / 1e9, 3)}), flush=True)
        return
    if a.tn:
        plans = {(6400, 1600): [(256, 2), (256, 1)], (4800, 1600): [(192, 2), (256, 2), (192, 1)],
                 (1600, 1600): [(256, 7), (256, 6), (256, 5), (192, 5)]}
        sk = {(6400, 1600): 250, (4800, 1600): 190, (1600, 1600): 245}
        for (M, N), pl in plans.items():
            dy = torch.randn(K, M, device="cuda").bfloat16()
            x = torch.randn(K, N, device="cuda").bfloat16()
            c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
            fl = 2.0 * M * N * K
            rows = []
            for rnd in range(2):  # interleaved rounds
                med, _ = timeit(lambda: c.addmm_(dy.t(), x), a.iters)
                rows.append(("hipblaslt", None, med))
                med, _ = timeit(lambda: G.run_sk(dy, x, c, 2, True, sk[(M, N)]), a.iters)
                rows.append(("sk", sk[(M, N)], med))
                for (bm, S) in pl:
                    for ink in ((True, False) if S > 1 else (False,)):
                        med, _ = timeit(lambda: G.run_tn(dy, x, c, True, bm, S, ink), a.iters)
                        rows.append(("tn64" + ("_ink" if ink else ""), f"{bm}x{S}", med))
            for impl, cfg, med in rows:
                print(json.dumps({"M": M, "N": N, "K": K, "impl": impl, "cfg": cfg, "us_med": round(med, 1),
                                  "pfs": round(fl / med / 1e9, 3)}), flush=True)
        return
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
