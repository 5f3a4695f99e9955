#!/usr/bin/env python
"""Tune the hipBLASLt/rocBLAS solutions of the Llama decode GEMMs (TunableOp) for
the batch buckets the engine replays, and write the winners to a CSV that
``ops.gemm_tuning`` ships (``cluster_anywhere_amd/tuning/gemm_gfx950_*.csv``).

    CAAMD_TUNE_GEMMS=gpurun_out/gemm_llama.csv python tools/tune_llm_gemms.py --buckets 128 64

The decode projections at batch 128 are skinny (M = 128, K = 4096 / 14336): the
library default tiles M by 32 and re-reads every weight panel four times.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--buckets", type=int, nargs="+", default=[128])
    a = ap.parse_args()
    if not os.environ.get("CAAMD_TUNE_GEMMS"):
        raise SystemExit("set CAAMD_TUNE_GEMMS=<output csv>")
    import torch
    import torch.nn.functional as F

    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig
    from cluster_anywhere_amd.ops.gemm_tuning import dump_tuned, use_tuned_gemms

    use_tuned_gemms()
    cfg = LlamaConfig.named(a.model)
    with torch.device("cuda"):
        m = Llama(cfg).to(torch.bfloat16)
    L0 = m.layers[0]
    d = cfg.d_model if hasattr(cfg, "d_model") else L0.w_qkv.shape[1]
    t0 = time.time()
    for B in a.buckets:
        x = torch.randn(B, d, device="cuda", dtype=torch.bfloat16)
        for w in (L0.w_qkv, L0.w_o, L0.w_gate_up):
            F.linear(x if w.shape[1] == d else x.new_empty(B, w.shape[1]).normal_(), w)
        F.linear(torch.randn(B, L0.w_down.shape[1], device="cuda", dtype=torch.bfloat16), L0.w_down)
        head = m.embed if m.lm_head is None else m.lm_head
        F.linear(x, head)
        torch.cuda.synchronize()
        print(f"bucket {B} tuned ({time.time() - t0:.0f}s)", flush=True)
    dump_tuned()
    print("wrote", os.environ["CAAMD_TUNE_GEMMS"], flush=True)


if __name__ == "__main__":
    main()
