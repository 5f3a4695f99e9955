"""Decode GEMM v3 (decode_gemm.hip) vs hipBLASLt (tuned selections) on Llama-3-8B's
decode shapes, batch 128, cache-cold
weights (rotated over >= 1 GB so each call streams from HBM, as in a decode step),
plus numerics vs fp32 (store, residual and SwiGLU epilogues, split and unsplit).
Prints one JSON line per shape."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import llm as L  # noqa: E402
from cluster_anywhere_amd.ops.gemm_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
M = int(os.environ.get("DECODE_M", "128"))
dev = torch.device("cuda", 0)


def timeit(fn, iters=40):
    """Per-call device time of ``fn`` replayed from a HIP graph (the decode path
    runs captured), so host launch cost is not measured."""
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(3):
        g.replay()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / (3 * iters) * 1e3


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def check():
    bad = 0
    g = torch.Generator(device=dev).manual_seed(0)
    for (m, n, k, splits) in ((128, 256, 512, 1), (128, 256, 512, 4), (7, 384, 1024, 2), (1, 128, 64, 1),
                              (100, 4096, 14336, None), (128, 6144, 4096, None)):
        x = torch.randn(m, k, device=dev, generator=g).bfloat16()
        w = (torch.randn(n, k, device=dev, generator=g) * 0.05).bfloat16()
        ref = x.float() @ w.float().t()
        y = L.decode_gemm(x, w, 0, splits=splits)
        r0 = rel(y, ref)
        res = torch.randn(m, n, device=dev, generator=g).bfloat16()
        y1 = L.decode_gemm(x, w, 1, residual=res, splits=splits)
        r1 = rel(y1, ref + res.float())
        wi = L.interleave_gate_up(w)
        y2 = L.decode_gemm(x, wi, 2, splits=splits)
        gg, uu = ref[:, : n // 2], ref[:, n // 2:]
        r2 = rel(y2, F.silu(gg) * uu)
        # repeat launches: the split tickets must be re-armed
        y3 = L.decode_gemm(x, w, 0, splits=splits)
        r3 = rel(y3, ref)
        # prepacked weights: plain and SwiGLU
        r4 = rel(L.decode_gemm(x, L.pack_decode_weight(w), 0, splits=splits, packed=True), ref)
        r5 = rel(L.decode_gemm(x, L.pack_decode_weight(wi), 2, splits=splits, packed=True), F.silu(gg) * uu)
        ok = max(r0, r1, r2, r3, r4, r5) < 1e-2
        bad += not ok
        print(json.dumps({"check": [m, n, k, splits], "store": round(r0, 5), "resid": round(r1, 5),
                          "swiglu": round(r2, 5), "repeat": round(r3, 5),
                          "packed": round(r4, 5), "packed_swiglu": round(r5, 5), "ok": ok}), flush=True)
    return bad


def bench():
    tot = {"hipblaslt": 0.0, "v3": 0.0, "v3p": 0.0}
    for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
                       ("lm_head", 128256, 4096)):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        nw = max(2, -(-(1 << 30) // (N * K * 2)))
        ws = [w] + [w.clone() for _ in range(nw - 1)]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % nw
            return ws[it[0]]

        a = timeit(lambda: F.linear(x, nxt()))
        c = timeit(lambda: L.decode_gemm(x, nxt()))
        wps = [L.pack_decode_weight(t) for t in ws]
        itp = [0]

        def nxtp():
            itp[0] = (itp[0] + 1) % nw
            return wps[itp[0]]

        d = timeit(lambda: L.decode_gemm(x, nxtp(), packed=True))
        row = {"gemm": name, "M": M, "N": N, "K": K, "splits": L.decode_gemm_splits(N, K),
               "hipblaslt_us": round(a, 1), "v3_us": round(c, 1), "v3p_us": round(d, 1),
               "v3_TBps": round(N * K * 2 / c / 1e6, 2), "hipblaslt_TBps": round(N * K * 2 / a / 1e6, 2)}
        if name == "gate_up":
            wsi = [L.interleave_gate_up(t) for t in ws]
            it2 = [0]

            def nxti():
                it2[0] = (it2[0] + 1) % nw
                return wsi[it2[0]]

            row["v3_swiglu_us"] = round(timeit(lambda: L.decode_gemm(x, nxti(), 2)), 1)
            del wps
            wpi = [L.pack_decode_weight(t) for t in wsi]
            row["v3p_swiglu_us"] = round(timeit(lambda: L.decode_gemm(x, wpi[it2[0] % nw], 2, packed=True)
                                                if not it2.__setitem__(0, it2[0] + 1) else None), 1)
            del wpi
            row["hipblaslt_plus_silu_us"] = round(timeit(lambda: L.silu_mul(F.linear(x, nxt()))), 1)
        if name != "lm_head":
            tot["hipblaslt"] += a
            tot["v3"] += c
            tot["v3p"] += d
        print(json.dumps(row), flush=True)
    print(json.dumps({"layer_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    torch.manual_seed(0)
    nbad = check()
    if "--ext" in sys.argv:  # the same checks with the separate reduce launch
        L.kernels().decode_gemm_config(1)
        nbad += check()
        L.kernels().decode_gemm_config(0)
    if nbad:
        print(f"{nbad} numerics failures", flush=True)
        sys.exit(1)
    if "--check" not in sys.argv:
        bench()
    if "--sweep" in sys.argv:
        for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            nw = max(2, -(-(1 << 30) // (N * K * 2)))
            wps = [L.pack_decode_weight(w)] + [L.pack_decode_weight(w) for _ in range(nw - 1)]
            for ext in (0, 1):
                # ext 1: split-K partials combined by a separate reduce launch
                L.kernels().decode_gemm_config(ext)
                out = {"sweep": name, "ext_reduce": ext}
                for sp in (1, 2, 3, 4, 6, 8, 16):
                    if K % (64 * sp) or (N // 128) * sp > 1024:
                        continue
                    it = [0]

                    def nx():
                        it[0] = (it[0] + 1) % nw
                        return wps[it[0]]
                    out[sp] = round(timeit(lambda: L.decode_gemm(x, nx(), splits=sp, packed=True)), 1)
                print(json.dumps(out), flush=True)
            L.kernels().decode_gemm_config(0)
            del wps
