"""gemm2.hip (256 x 160 tiles, 2 workgroups per CU, split-K tail) vs the
first-generation kernel (gemm.hip, 256 x 320 ping-pong) vs torch.matmul
(hipBLASLt) on the GPT-2-XL step shapes (M = 32768 tokens), random [-1, 1)
operands, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).

    python tools/bench_gemm2.py [--check] [--rounds 5] [--only fc,qkv] [--wgrad]
Prints one JSON line per shape."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import gemm as G  # noqa: E402
from cluster_anywhere_amd.ops._lib import kernels  # noqa: E402

dev = torch.device("cuda", 0)
T = 32768
# name: (N, K, epi)  for layout 0 (a[M,K] b[N,K])
SHAPES = {
    "qkv": (4800, 1600, 0),
    "proj": (1600, 1600, 0),
    "fc_gelu": (6400, 1600, 3),
    "fc2": (1600, 6400, 0),
    "dgrad_qkv": (1600, 4800, 0),
    "dgrad_proj": (1600, 1600, 0),
    "dgrad_fc2_dgelu": (6400, 1600, 4),
    "dgrad_fc": (1600, 6400, 0),
}
# weight gradients, layout 2: dW[M=N_out, N=K_in] = dy[T, N_out]^T x[T, K_in]
WGRAD = {"w_qkv": (4800, 1600), "w_proj": (1600, 1600), "w_fc": (6400, 1600), "w_fc2": (1600, 6400)}


def rnd(*shape):
    return (torch.rand(*shape, device=dev) * 2 - 1).bfloat16()


def timeit(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def check():
    out = []
    # layout 0, each epilogue, with and without the split tail (small M -> all-tail plan)
    for (M, N, K) in ((2048, 1600, 1024), (512, 320, 256), (32768 // 8, 1600, 1600), (1024, 480, 96),
                      (256, 160, 32), (256, 160, 64)):
        a, b = rnd(M, K), rnd(N, K) * 0.05
        bias = rnd(N)
        ref = a.float() @ b.float().t()
        for ms in (1, 4):
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            G.run2(a, b, c, 0, 0, bias=bias, max_split=ms)
            out.append({"M": M, "N": N, "K": K, "epi": 0, "split": G.plan2(M, N, K, dev, ms)[1],
                        "rel": rel(c, ref + bias.float())})
            u, z = torch.empty_like(c), torch.empty_like(c)
            G.run2(a, b, u, 0, 3, bias=bias, zout=z, max_split=ms)
            zr = ref + bias.float()
            out.append({"M": M, "N": N, "K": K, "epi": 3, "rel_z": rel(z, zr),
                        "rel_u": rel(u, torch.nn.functional.gelu(z.float(), approximate="tanh"))})
            db = torch.zeros(N, device=dev)
            zz = rnd(M, N)
            d = torch.empty_like(c)
            G.run2(a, b, d, 0, 4, z=zz, dbias=db, max_split=ms)
            zf = zz.float()
            t = torch.tanh(0.7978845608028654 * (zf + 0.044715 * zf ** 3))
            gp = 0.5 * (1 + t) + 0.5 * zf * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * zf * zf)
            out.append({"M": M, "N": N, "K": K, "epi": 4, "rel": rel(d, ref * gp), "rel_db": rel(db, (ref * gp).sum(0))})
            acc = rnd(M, N)
            acc0 = acc.float().clone()
            G.run2(a, b, acc, 0, 1, max_split=ms)
            out.append({"M": M, "N": N, "K": K, "epi": 1, "rel": rel(acc, acc0 + ref)})
    # ping-pong kernel with the split tail (M x 1600 tiles of 256 x 320 over the CUs)
    for (M, N, K) in ((32768, 1600, 1600), (8192, 1600, 2048), (32768 * 2 // 8, 4800, 1024)):
        a, b = rnd(M, K), rnd(N, K) * 0.05
        bias = rnd(N)
        ref = a.float() @ b.float().t() + bias.float()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        G.run_pp(a, b, c, 0, 0, 256, 320, bias=bias, algo=2)
        out.append({"pp_tail": G.tail_plan(M, N, K, 256, 320, dev, 2), "M": M, "N": N, "K": K, "rel": rel(c, ref)})
        db = torch.zeros(N, device=dev)
        zz = rnd(M, N)
        G.run_pp(a, b, c, 0, 4, 256, 320, z=zz, dbias=db, algo=2)
        zf = zz.float()
        t = torch.tanh(0.7978845608028654 * (zf + 0.044715 * zf ** 3))
        gp = 0.5 * (1 + t) + 0.5 * zf * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * zf * zf)
        r0 = (ref - bias.float()) * gp
        out.append({"pp_tail": G.tail_plan(M, N, K, 256, 320, dev, 2), "epi": 4, "M": M, "N": N, "K": K,
                    "rel": rel(c, r0), "rel_db": rel(db, r0.sum(0))})
        # repeat launches: tickets must have been reset by the last arrivers
        for _ in range(3):
            G.run_pp(a, b, c, 0, 0, 256, 320, bias=bias, algo=2)
        out.append({"pp_tail_repeat": True, "M": M, "N": N, "K": K, "rel": rel(c, ref)})
    # stream-K weight-gradient kernel (ragged M, accumulate), incl. repeat launches
    for (M, N, K) in ((1600, 1600, 32768), (4800, 1600, 8192), (6400, 320, 4096), (200, 640, 2048)):
        a, b = rnd(K, M), rnd(K, N)
        ref = a.float().t() @ b.float()
        c0 = rnd(M, N)
        for rep in range(3):
            c = c0.clone()
            G.run_sk(a, b, c, 2, True)
            out.append({"sk": rep, "M": M, "N": N, "K": K, "rel": rel(c, c0.float() + ref)})
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        G.run_sk(a, b, c, 2, False)
        out.append({"sk_store": True, "M": M, "N": N, "K": K, "rel": rel(c, ref)})
    # layout 2 (weight gradient) with ragged M
    for (M, N, K) in ((1600, 1600, 2048), (4800, 320, 1024), (200, 160, 512)):
        a, b = rnd(K, M), rnd(K, N)
        ref = a.float().t() @ b.float()
        for ms in (1, 8):
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            G.run2(a, b, c, 2, 0, max_split=ms)
            out.append({"layout": 2, "M": M, "N": N, "K": K, "split": G.plan2(M, N, K, dev, ms)[1], "rel": rel(c, ref)})
    bad = 0
    for r in out:
        worst = max(v for k, v in r.items() if k.startswith("rel"))
        r["ok"] = worst < 1.5e-2
        bad += not r["ok"]
        print(json.dumps(r), flush=True)
    return bad


def bench(rounds, only, wgrad):
    res = {}
    todo = dict(SHAPES)
    if only:
        todo = {k: v for k, v in todo.items() if k in only}
    for name, (N, K, epi) in todo.items():
        a, b = rnd(T, K), rnd(N, K) * 0.05
        bias = rnd(N)
        c = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        z = rnd(T, N) if epi in (3, 4) else None
        db = torch.zeros(N, device=dev) if epi == 4 else None
        flops = 2.0 * T * N * K

        def old():
            kernels().gemm_bf16(a, b, c, 0, epi, 256, 320, bias if epi in (0, 3) else None,
                                z if epi == 4 else None, z if epi == 3 else None, db, 1, None, False, 2)

        def tail():
            G.run_pp(a, b, c, 0, epi, 256, 320, bias=bias if epi in (0, 3) else None,
                     z=z if epi == 4 else None, zout=z if epi == 3 else None, dbias=db, algo=2)

        def new():
            G.run2(a, b, c, 0, epi, bias=bias if epi in (0, 3) else None,
                   z=z if epi == 4 else None, zout=z if epi == 3 else None, dbias=db)

        def lib():
            torch.matmul(a, b.t(), out=c)

        arms = {"old": old, "old_tail": tail, "new": new, "hipblaslt": lib}
        t = {k: [] for k in arms}
        for _ in range(rounds):
            for k, f in arms.items():
                t[k].append(timeit(f))
        r = {"shape": name, "M": T, "N": N, "K": K, "epi": epi, "plan": G.plan2(T, N, K, dev)[:3],
             "tail_plan": G.tail_plan(T, N, K, 256, 320, dev, 2)}
        for k in arms:
            med = sorted(t[k])[len(t[k]) // 2]
            r[k + "_us"] = round(med, 1)
            r[k + "_pfs"] = round(flops / med / 1e9, 3)
        res[name] = r
        print(json.dumps(r), flush=True)
    if wgrad:
        for name, (M, N) in WGRAD.items():
            dy, x = rnd(T, M), rnd(T, N)
            out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
            flops = 2.0 * T * M * N
            arms = {}
            tiles = -(-M // 256) * (N // 320)
            arms["sk256"] = lambda: G.run_sk(dy, x, out, 2, True, runs=256)
            for S in (1, 2, 3, 4, 7, 8):
                if tiles * S <= 512 and (1024 % S == 0 or S in (3, 7)):
                    arms[f"split{S}"] = (lambda S=S: G.run_sk(dy, x, out, 2, True, runs=tiles * S))
            arms["auto"] = lambda: G.run_sk(dy, x, out, 2, True)
            arms["hipblaslt_addmm"] = lambda: out.addmm_(dy.t(), x)
            t = {k: [] for k in arms}
            for _ in range(rounds):
                for k, f in arms.items():
                    t[k].append(timeit(f, reps=5))
            r = {"shape": name, "M": M, "N": N, "K": T, "auto_runs": G.sk_runs(M, N, T, dev)}
            for k in arms:
                med = sorted(t[k])[len(t[k]) // 2]
                r[k + "_us"] = round(med, 1)
                r[k + "_pfs"] = round(flops / med / 1e9, 3)
            print(json.dumps(r), flush=True)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--wgrad", action="store_true")
    ap.add_argument("--no-bench", action="store_true")
    args = ap.parse_args()
    kernels()
    if args.check:
        bad = check()
        if bad:
            print(f"{bad} numerics failures", flush=True)
            sys.exit(1)
    if not args.no_bench:
        bench(args.rounds, [s for s in args.only.split(",") if s], args.wgrad)
