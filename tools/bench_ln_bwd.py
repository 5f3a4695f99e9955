#!/usr/bin/env python
"""LayerNorm backward variants on the GPT-2-XL shape [32768, 1600] (+ residual
grad): correctness vs an fp32 torch reference and time per call / effective
HBM bandwidth for each (variant, grid cap)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import kernels  # noqa: E402


def main():
    C = kernels()
    R, D = 32768, 1600
    torch.manual_seed(0)
    x = torch.randn(R, D, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(R, D, device="cuda", dtype=torch.bfloat16)
    dres = torch.randn(R, D, device="cuda", dtype=torch.bfloat16)
    g = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    b = (0.1 * torch.randn(D, device="cuda")).bfloat16()
    y, mean, rstd, _ = C.layernorm_fwd(x, None, g, b, 1e-5)
    xr = x.float().requires_grad_(True)
    gr, br = g.float().requires_grad_(True), b.float().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-5)
    yr.backward(dy.float())
    ref_dx = xr.grad + dres.float()
    for variant, blocks in ((0, 0), (2, 0), (2, 1024), (2, 4096), (3, 0), (3, 4096), (3, 8192)):
        C.ln_bwd_config(variant, blocks)
        dx, dg, db = C.layernorm_bwd(dy, x, g, mean, rstd, dres)
        err = float((dx.float() - ref_dx).abs().max())
        gerr = float((dg.float() - gr.grad).abs().max() / gr.grad.abs().max())
        berr = float((db.float() - br.grad).abs().max() / br.grad.abs().max())
        for _ in range(3):
            C.layernorm_bwd(dy, x, g, mean, rstd, dres)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            C.layernorm_bwd(dy, x, g, mean, rstd, dres)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 50 * 1e3
        print(json.dumps({"variant": variant, "max_blocks": blocks, "us": round(us, 1),
                          "TB_s": round(4 * R * D * 2 / us / 1e6, 2), "dx_maxerr": err, "dgamma_relerr": gerr,
                          "dbeta_relerr": berr}),
              flush=True)
    # the training step's form: + the column sums of dx (the residual branch's bias
    # gradient) accumulated into a main-grad vector, dgamma / dbeta into main grads
    dxsum = torch.zeros(D, device="cuda", dtype=torch.bfloat16)
    gm = torch.zeros(D, device="cuda", dtype=torch.bfloat16)
    bm = torch.zeros(D, device="cuda", dtype=torch.bfloat16)
    caps = [int(c) for c in os.environ.get("LN_BWD_CAPS", "0,4096,1024").split(",")]
    for variant, blocks in [(v, c) for c in caps for v in (3, 2)] + [(3, 0)]:
        C.ln_bwd_config(variant, blocks)
        dxsum.zero_()
        dx = C.layernorm_bwd(dy, x, g, mean, rstd, dres, dxsum, gm, bm)[0]
        err = float((dx.float() - ref_dx).abs().max())
        serr = float((dxsum.float() - ref_dx.sum(0)).abs().max() / ref_dx.sum(0).abs().max())
        for _ in range(3):
            C.layernorm_bwd(dy, x, g, mean, rstd, dres, dxsum, gm, bm)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            C.layernorm_bwd(dy, x, g, mean, rstd, dres, dxsum, gm, bm)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 50 * 1e3
        print(json.dumps({"path": "dxsum", "variant": variant, "max_blocks": blocks, "us": round(us, 1),
                          "TB_s": round(4 * R * D * 2 / us / 1e6, 2), "dx_maxerr": err, "dxsum_relerr": serr}),
              flush=True)
    C.ln_bwd_config(3, 0)  # the library default


if __name__ == "__main__":
    main()
