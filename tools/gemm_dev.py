"""Correctness + speed of the hand-written MFMA GEMM (csrc/kernels/gemm.hip)
against fp32 torch (numerics) and torch.matmul / hipBLASLt (speed), on the
GPT-2-XL training shapes (M = 32768 tokens)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from cluster_anywhere_amd.ops._lib import kernels  # noqa: E402

K_ = kernels()
dev = "cuda"


def ref(layout, a, b):
    a32, b32 = a.float(), b.float()
    if layout == 0:
        return a32 @ b32.t()
    if layout == 1:
        return a32 @ b32
    return a32.t() @ b32


def run(layout, a, b, bm, bn, epi=0, bias=None, splitk=1, out=None, algo=1):
    M = a.shape[1] if layout == 2 else a.shape[0]
    N = b.shape[0] if layout == 0 else b.shape[1]
    c = out if out is not None else torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ws = torch.empty(splitk * M * N, device=dev, dtype=torch.float32) if splitk > 1 else None
    K_.gemm_bf16(a, b, c, layout, epi, bm, bn, bias, None, None, None, splitk, ws, False, algo)
    return c


def mk(layout, M, N, K):
    g = torch.Generator(device=dev).manual_seed(0)
    if layout == 0:
        a, b = torch.randn(M, K, device=dev, generator=g), torch.randn(N, K, device=dev, generator=g)
    elif layout == 1:
        a, b = torch.randn(M, K, device=dev, generator=g), torch.randn(K, N, device=dev, generator=g)
    else:
        a, b = torch.randn(K, M, device=dev, generator=g), torch.randn(K, N, device=dev, generator=g)
    return a.bfloat16(), b.bfloat16()


def check():
    res = []
    for layout in (0, 1, 2):
        for (bm, bn) in ((256, 256), (256, 320), (128, 320)):
            M, N, K = 2 * bm, 2 * bn, 448
            a, b = mk(layout, M, N, K)
            r = ref(layout, a, b)
            for algo in (0, 1, 2, 3, 4):
                c = run(layout, a, b, bm, bn, algo=algo).float()
                err = ((c - r).abs().max() / r.abs().max()).item()
                res.append({"layout": layout, "tile": [bm, bn], "algo": algo, "rel_err": err})
                print(json.dumps(res[-1]), flush=True)
                assert err < 2e-2, res[-1]
    return res


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


SHAPES = [  # name, layout, M, N, K   (C[M,N], reduction K)
    ("qkv_fwd", 0, 32768, 4800, 1600), ("proj_fwd", 0, 32768, 1600, 1600),
    ("fc_fwd", 0, 32768, 6400, 1600), ("fc2_fwd", 0, 32768, 1600, 6400),
    ("qkv_dgrad", 1, 32768, 1600, 4800), ("proj_dgrad", 1, 32768, 1600, 1600),
    ("fc_dgrad", 1, 32768, 1600, 6400), ("fc2_dgrad", 1, 32768, 6400, 1600),
    ("qkv_wgrad", 2, 4800, 1600, 32768), ("fc_wgrad", 2, 6400, 1600, 32768),
]


def speed_vs_tuned():
    """Per-role comparison against the shipped hipBLASLt selections (what the step
    would otherwise run): forward NT and input-gradient (ours: NT against W^T)."""
    from cluster_anywhere_amd.ops.gemm_tuning import use_tuned_gemms
    from cluster_anywhere_amd.ops import gemm as G

    use_tuned_gemms()
    for name, M, N, K in [("qkv", 32768, 4800, 1600), ("proj", 32768, 1600, 1600),
                          ("fc", 32768, 6400, 1600), ("fc2", 32768, 1600, 6400)]:
        x, w = mk(0, M, N, K)
        fl = 2.0 * M * N * K
        dy = torch.randn(M, N, device=dev).bfloat16()
        wt = G.transpose(w)
        row = {"gemm": name, "fwd_hipblaslt": fl / bench(lambda: x @ w.t()) / 1e15,
               "fwd_ours": fl / bench(lambda: G.linear_nt(x, w)) / 1e15,
               "dgrad_hipblaslt": fl / bench(lambda: dy @ w) / 1e15,
               "dgrad_ours": fl / bench(lambda: G.dgrad(dy, wt)) / 1e15,
               "transpose_us": bench(lambda: G.transpose(w)) * 1e6}
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)


def speed(tiles=((256, 256), (256, 320), (128, 320))):
    for name, layout, M, N, K in SHAPES:
        a, b = mk(layout, M, N, K)
        fl = 2.0 * M * N * K
        if layout == 0:
            tfn = lambda: a @ b.t()
        elif layout == 1:
            tfn = lambda: a @ b
        else:
            tfn = lambda: a.t() @ b
        row = {"gemm": name, "M": M, "N": N, "K": K, "torch_pfs": round(fl / bench(tfn) / 1e15, 3)}
        for bm, bn in tiles:
            if M % bm or N % bn:
                continue
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            for algo in ALGOS:
                t = bench(lambda: run(layout, a, b, bm, bn, out=c, algo=algo))
                row[f"a{algo}_{bm}x{bn}"] = round(fl / t / 1e15, 3)
        print(json.dumps(row), flush=True)


ALGOS = (2, 4)

def ablate():
    layout, M, N, K = 0, 32768, 6400, 1600
    a, b = mk(layout, M, N, K)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    names = {0: "full", 1: "noDMA", 2: "noLDSread", 3: "noDMA+noRead", 4: "noMFMA", 5: "noDMA+noMFMA",
             6: "noRead+noMFMA", 7: "loop+epi", 8: "noEpiStore", 15: "loop-only",
             16: "hotDMA", 32: "noVmWait", 48: "hot+noWait", 24: "hot+noEpi"}
    for base in (2,):
        row = {"algo": base}
        for abl in [0, 1, 2, 3, 8, 16, 32, 48, 24]:
            t = bench(lambda: run(layout, a, b, 256, 320, out=c, algo=abl * 10 + base))
            row[names[abl]] = round(t * 1e6, 1)
        row["full_pfs"] = round(fl / row["full"] / 1e9, 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    if "--tuned" in sys.argv:
        speed_vs_tuned()
        sys.exit(0)
    if "--ablate" in sys.argv:
        ablate()
        sys.exit(0)
    check()
    if "--check" not in sys.argv:
        speed()
