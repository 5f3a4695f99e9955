"""Persistent async-epilogue GEMM (algo 8) vs the per-tile ping-pong kernel
(algo 2, with its split-K tail where planned) on the GPT-2-XL step shapes.
python tools/bench_pst.py  -> one JSON line per (shape, epilogue)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from cluster_anywhere_amd.ops import gemm as G
    from cluster_anywhere_amd.ops import kernels

    k = kernels()
    shapes = [("qkv_fwd", 32768, 4800, 1600, "bias"), ("proj_fwd", 32768, 1600, 1600, "bias"),
              ("fc_fwd", 32768, 6400, 1600, "gelu"), ("proj_dgrad", 32768, 1600, 1600, "plain"),
              ("fc2_fwd", 32768, 1600, 6400, "bias"), ("qkv_dgrad", 32768, 1600, 4800, "plain")]
    for name, M, N, K, epi in shapes:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16() if epi != "plain" else None
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        zo = torch.empty_like(c) if epi == "gelu" else None
        e = G.EPI_BIAS_GELU if epi == "gelu" else G.EPI_BF16

        def pp():
            full, S = G.tail_plan(M, N, K, 256, 320, c.device, 2)
            ws = cnt = None
            if S > 1:
                ws, cnt = G._workspace(c.device, ((M // 256) * (N // 320) - full) * S * 256 * 320,
                                       (M // 256) * (N // 320) - full)
            k.gemm_bf16(x, w, c, 0, e, 256, 320, b, None, zo, None, 1, None, False, 2, ws, cnt, full, S)

        def pst():
            k.gemm_bf16(x, w, c, 0, e, 256, 320, b, None, zo, None, 1, None, False, 8, None, None, 0, 1)

        res = {"shape": name, "M": M, "N": N, "K": K, "epi": epi}
        outs = {}
        for nm, fn in (("pp", pp), ("pst", pst), ("pp2", pp), ("pst2", pst)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 20
            res[nm + "_us"] = round(us, 1)
            res[nm + "_pfs"] = round(2 * M * N * K / us / 1e9, 3)
            outs[nm[:3] if nm.startswith("ps") else nm[:2]] = c.clone()
        res["equal"] = bool(torch.equal(outs["pp"], outs["pst"]))
        print(json.dumps(res), flush=True)
        del x, w, c, zo


if __name__ == "__main__":
    main()
