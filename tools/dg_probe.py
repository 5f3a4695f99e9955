"""What bounds the decode GEMM (decode_gemm.hip) on the Llama-3-8B gate_up shape:
per-call device time (HIP-graph replay, weights rotated over >= 1 GB so every call
streams from HBM) over the slab count (N / 128 workgroups, one per CU, no split),
the batch rows M (the X image is staged for all 128 rows either way: M = 1 reads
one row 128 times) and the ring depths (CAAMD_DG_RING is read once per process,
so the script is run once per ring setting).

    CAAMD_DG_RING=0 python tools/dg_probe.py  -> one JSON line per (N, M)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import llm as L  # noqa: E402
from tools.bench_decode_gemm3 import timeit  # noqa: E402

dev = torch.device("cuda", 0)
K = 4096
ring = os.environ.get("CAAMD_DG_RING", "0")
for N in (28672, 14336, 7168):
    for M in (128, 1):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        nw = max(2, -(-(1 << 30) // (N * K * 2)))
        wps = [L.pack_decode_weight(w.roll(i, 0)) for i in range(nw)]
        it = [0]

        def nx():
            it[0] = (it[0] + 1) % nw
            return wps[it[0]]

        us = timeit(lambda: L.decode_gemm(x, nx(), 0, splits=1, packed=True))
        print(json.dumps({"ring": ring, "N": N, "K": K, "M": M, "slabs": N // 128, "us": round(us, 2),
                          "TBps": round(N * K * 2 / us / 1e6, 2),
                          "us_per_step": round(us / (K // 64), 3)}), flush=True)
        del wps, w
        torch.cuda.empty_cache()
