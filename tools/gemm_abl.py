"""Timing ablations of the production GEMM (algo 2 = gemm_pp_kernel, one phase,
DMA two K-steps ahead) on GPT-2-XL's fc shape: each ABL bit removes one component
(1: in-loop DMA, 2: LDS fragment reads, 4: MFMAs, 8: epilogue global stores,
16: every K-step re-reads the first K-slice, L2-hot). Results are timing only
(outputs are wrong by design). Prints one JSON line per variant."""
import json
import sys

import torch

sys.path.insert(0, ".")
from cluster_anywhere_amd.ops.gemm import gemm  # noqa: E402

M, N, K = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (32768, 6400, 1600)))
BASE = int(sys.argv[4]) if len(sys.argv) >= 5 else 2  # 2: gemm_pp (KS 32), 0: gemm_kernel (BK 64)
ONLY = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) >= 6 else None
a = torch.randn(M, K, device="cuda").bfloat16()
b = torch.randn(N, K, device="cuda").bfloat16()


def t(algo, iters=20):
    for _ in range(3):
        gemm(a, b, 0, algo=algo, tile=(256, 320))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        gemm(a, b, 0, algo=algo, tile=(256, 320))
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


base = t(BASE)
for abl, what in ((0, "full"), (1, "no in-loop DMA"), (2, "no LDS frag reads"), (4, "no MFMA"),
                  (8, "no epilogue stores"), (16, "L2-hot K-slice"), (3, "MFMA + barriers only"),
                  (5, "frag reads + barriers only"), (6, "DMA + barriers only"), (24, "L2-hot, no epilogue")):
    if ONLY is not None and abl not in ONLY:
        continue
    us = t(BASE + 10 * abl) if abl else base
    print(json.dumps({"shape": [M, N, K], "base_algo": BASE, "abl": abl, "what": what, "us": round(us, 1),
                      "pfs": round(2 * M * N * K / us / 1e9, 3)}), flush=True)
