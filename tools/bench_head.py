"""LM head + loss at the GPT-2-XL step shape: materialised logits (hipBLASLt GEMMs +
xent kernels) vs the chunked fused head (ops/loss.linear_cross_entropy).

python tools/bench_head.py [--tokens 32768] [--chunk 16384]
Prints one JSON line per variant: ms per fwd+bwd and peak memory over the call.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--dim", type=int, default=1600)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--vpad", type=int, default=50432)
    ap.add_argument("--chunks", default="16384,8192,32768")
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import cluster_anywhere_amd.ops.loss as L

    torch.manual_seed(0)
    h = (torch.randn(args.tokens, args.dim, device="cuda") * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(args.vpad, args.dim, device="cuda") * 0.02).bfloat16().requires_grad_()
    w.main_grad = torch.zeros_like(w)
    tgt = torch.randint(0, args.vocab, (args.tokens,), device="cuda")

    def run(fused, chunk):
        L.FUSED_HEAD = fused
        loss = L.linear_cross_entropy(h, w, tgt, args.vocab, chunk=chunk)
        loss.backward()
        h.grad = None
        w.grad = None

    variants = [("materialised", False, 0)] + [(f"fused_c{c}", True, int(c)) for c in args.chunks.split(",")]
    for name, fused, chunk in variants:
        for _ in range(2):
            run(fused, chunk)
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run(fused, chunk)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        flops = 3 * 2 * args.tokens * args.dim * args.vpad
        print(json.dumps({"variant": name, "ms": round(ms, 3), "pfs": round(flops / ms / 1e12, 3),
                          "peak_extra_gb": round((torch.cuda.max_memory_allocated() - base) / 1e9, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
