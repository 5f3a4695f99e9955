"""Is the full-line GEMM's output store bound per CU or by the chip? One round of tiles
(N 6400 = 20 n-tiles, K 1600) on 60, 120 and 240 CUs (M = 3, 6, 12 x 256 rows), each
timed with the plain bf16 epilogue (algo 4009) and with the epilogue compiled out
(algo 4089). If the store is bound by HBM for the whole chip, the epilogue's share
shrinks with fewer CUs storing at once; if each CU's own store path is the bound, it
stays put.

    python tools/gemm_epi_occupancy.py   -> one JSON line per (CUs, arm, round)
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.gemm_algo_ab import timeit  # noqa: E402


def main():
    from cluster_anywhere_amd.ops import gemm as G

    N, K = 6400, 1600
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    for rnd in range(2):
        for mt in (3, 6, 12):
            M = 256 * mt
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row = {"tiles": mt * 20, "M": M, "round": rnd}
            for algo in (4009, 4089):
                mn, med = timeit(lambda: G.run_pp(x, w, c, 0, G.EPI_BF16, 256, 320, algo=algo), iters=200)
                row[str(algo)] = round(med, 2)
            row["epilogue_us"] = round(row["4009"] - row["4089"], 2)
            row["store_GBps_per_cu"] = round(256 * 320 * 2 / (row["epilogue_us"] * 1e3), 1) if row["epilogue_us"] > 0 else None
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
