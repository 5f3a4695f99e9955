"""Fused softmax cross-entropy kernel (xent_fused_) on the GPT-2-XL LM-head chunk
[16384, 50304] (vocab 50257): time per call and effective bandwidth (read + write of
the logits). CAAMD_XENT_TPB selects the block size (read once per process)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import kernels  # noqa: E402


def main():
    rows, V, stride = 16384, 50257, 50304
    torch.manual_seed(0)
    base = (3 * torch.randn(rows, stride, device="cuda")).bfloat16()
    tgt = torch.randint(0, V, (rows,), device="cuda")
    scale = torch.tensor([1.0 / rows], device="cuda")
    lg = base.clone()
    for _ in range(3):
        lg.copy_(base)
        kernels().xent_fused_(lg, tgt, scale, V)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        lg.copy_(base)
        s.record()
        kernels().xent_fused_(lg, tgt, scale, V)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1000)
    us = sorted(ts)[len(ts) // 2]
    print(json.dumps({"tpb": os.environ.get("CAAMD_XENT_TPB", "512"), "us": round(us, 1),
                      "TB_s": round(2 * rows * stride * 2 / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
