"""What the fused epilogues cost on the full-line kernel (gemm.hip algo 4009):
GPT-2-XL fc shape (M 32768, N 6400, K 1600) with the plain bf16, bias+GELU and
dGELU epilogues, each also with the epilogue compiled out (ABL 8, algo 4089: the
main loop alone), alternating arms. (Round 6 also timed a dGELU variant with the
second half's Z loads issued early, algo 4649, bitwise equal and 11 us faster: it is
now the production epilogue, profiles/gemm_epi_ab_r6.jsonl.)

    python tools/gemm_epi_ab.py   -> one JSON line per epilogue, arm and round
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

    M, N, K = 32768, 6400, 1600
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
    z = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    zout = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(N, device="cuda", dtype=torch.float32)
    arms = {
        "plain": dict(epi=G.EPI_BF16),
        "bias_gelu": dict(epi=G.EPI_BIAS_GELU, bias=b, zout=zout),
        "dgelu": dict(epi=G.EPI_DGELU, z=z, dbias=db),
    }
    ref = (x[:256].float() @ w.float().t())
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for name, kw in arms.items():
            for algo in (4009, 4089):
                kw2 = dict(kw)
                epi = kw2.pop("epi")

                def f():
                    return G.run_pp(x, w, c, 0, epi, 256, 320, algo=algo, **kw2)
                f()
                err = None
                if name == "plain" and algo == 4009:
                    err = round(((c[:256].float() - ref).norm() / ref.norm()).item(), 5)
                mn, med = timeit(f)
                print(json.dumps({"epi": name, "algo": algo, "round": rnd, "us_min": round(mn, 1),
                                  "us_med": round(med, 1), "pfs": round(2.0 * M * N * K / med / 1e9, 3),
                                  "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
