"""GEMM shape sweep for the GPT-2-XL training step: times every GEMM the step
issues (fwd ``x @ W^T + b``, bwd ``dY @ W``, weight-grad ``dW += dY^T @ X``)
under the default hipBLASLt heuristic and, with ``--tune``, under torch's
TunableOp search (hipBLASLt + rocBLAS solutions per shape). Writes the tuned
solution table to ``--tunable-file`` so the training step can load it.

    python tools/bench_gemm.py --tokens 32768 [--tune --tunable-file tunableop/gemm.csv]
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.nn.functional as F


def shapes(d, vocab):
    # (name, N, K): out[M,N] = x[M,K] @ W[N,K]^T
    return [("qkv", 3 * d, d), ("proj", d, d), ("fc", 4 * d, d), ("fc2", d, 4 * d), ("lm", vocab, d)]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def run(tokens, d, vocab, only=None):
    dev = torch.device("cuda")
    rows = []
    tot_ms = 0.0
    for name, n, k in shapes(d, vocab):
        if only and name not in only:
            continue
        print(f"# {name} N={n} K={k}", flush=True)
        x = torch.randn(tokens, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
        # the step's fc GEMM has no bias (bias + GELU run fused in bias_gelu.hip)
        b = torch.randn(n, device=dev, dtype=torch.bfloat16) if name not in ("lm", "fc") else None
        dy = torch.randn(tokens, n, device=dev, dtype=torch.bfloat16)
        g = torch.zeros(n, k, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * tokens * n * k
        for role, fn in (("fwd", lambda: F.linear(x, w, b)),
                         ("dgrad", lambda: dy @ w),
                         # lm head (tied wte, plain autograd): dW = dY^T X without accumulate
                         ("wgrad", (lambda: dy.t() @ x) if name == "lm" else (lambda: g.addmm_(dy.t(), x)))):
            ms = bench(fn)
            tot_ms += ms
            rows.append({"gemm": name, "role": role, "M": tokens, "N": n, "K": k,
                         "ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)})
        del x, w, b, dy, g
        torch.cuda.empty_cache()
    return rows, tot_ms


def write_results(tn, path):
    """Dump the TunableOp table (validators + per-shape winners) in the CSV format
    ``torch.cuda.tunable.read_file`` accepts. This torch build has no
    ``tunable.write_file``, so it is written from ``get_validators/get_results``."""
    if hasattr(tn, "write_file"):
        tn.write_file(path)
        return
    with open(path, "w") as f:
        for k, v in tn.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for row in tn.get_results():
            f.write(",".join(str(c) for c in row) + "\n")
    print(f"# wrote {path}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--d", type=int, default=1600)
    ap.add_argument("--vocab", type=int, default=50304)
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--tunable-file", default="")
    ap.add_argument("--load", default="", help="start from an existing TunableOp results file")
    ap.add_argument("--only", default="", help="comma list of gemm names (qkv,proj,fc,fc2,lm)")
    ap.add_argument("--skip-default", action="store_true")
    args = ap.parse_args()
    only = [x for x in args.only.split(",") if x]

    def heartbeat():  # tuning one large shape can take minutes: keep the run visibly alive
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"# ... {time.time() - t0:.0f}s", flush=True)

    import threading

    threading.Thread(target=heartbeat, daemon=True).start()
    rows, tot = ([], 0.0) if args.skip_default else run(args.tokens, args.d, args.vocab, only)
    print(json.dumps({"mode": "default", "total_ms": round(tot, 2), "rows": rows}), flush=True)
    if args.tune:
        import torch.cuda.tunable as tn

        tn.enable(True)
        tn.tuning_enable(True)
        tn.set_max_tuning_duration(60)
        tn.set_max_tuning_iterations(20)
        if args.load:
            tn.read_file(args.load)
        if args.tunable_file:
            os.makedirs(os.path.dirname(os.path.abspath(args.tunable_file)), exist_ok=True)
            tn.set_filename(args.tunable_file, False)
        t0 = time.time()
        run(args.tokens, args.d, args.vocab, only)  # tuning pass
        tn.tuning_enable(False)
        if args.tunable_file:
            write_results(tn, args.tunable_file)
        rows2, tot2 = run(args.tokens, args.d, args.vocab, only)
        print(json.dumps({"mode": "tunableop", "tune_s": round(time.time() - t0, 1),
                          "total_ms": round(tot2, 2), "rows": rows2}), flush=True)


if __name__ == "__main__":
    main()
