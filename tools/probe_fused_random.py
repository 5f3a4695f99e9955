"""Where a fresh process's ``FusedResNet.random`` time goes on the GPU (the Data actor's
model set-up): each stage synchronised and timed, first call in the process vs a
second call (kernel code-object loading is a first-launch cost).

    python tools/probe_fused_random.py   -> one JSON line per call
"""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def staged(dev):
    from cluster_anywhere_amd.models.resnet import FusedResNet

    out = {}
    t = time.perf_counter()

    def mark(k):
        nonlocal t
        torch.cuda.synchronize(dev)
        now = time.perf_counter()
        out[k] = round((now - t) * 1e3, 2)
        t = now

    flat = torch.randn(23_454_912, device=dev)
    mark("randn_ms")
    views = list(torch.split(flat, [flat.numel() // 53] * 53 + [flat.numel() % 53]))
    torch._foreach_mul_(views, [math.sqrt(2.0 / 64)] * len(views))
    mark("foreach_mul_ms")
    fb = flat.to(torch.bfloat16)
    mark("cast_ms")
    w = fb[: 256 * 64 * 9].view(256, 64, 3, 3).contiguous(memory_format=torch.channels_last)
    mark("channels_last_copy_ms")
    z = torch.zeros(2048, device=dev, dtype=torch.bfloat16)
    mark("zeros_ms")
    torch.nn.functional.pad(w.permute(0, 2, 3, 1), (0, 8)).contiguous()
    mark("pad_ms")
    t0 = time.perf_counter()
    m = FusedResNet.random("resnet50", torch.bfloat16, dev)
    torch.cuda.synchronize(dev)
    out["fused_random_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    del m, z
    return out


def main():
    t0 = time.perf_counter()
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    torch.empty(1, device=dev)
    torch.cuda.synchronize()
    init_ms = round((time.perf_counter() - t0) * 1e3, 1)
    for call in range(2):
        r = staged(dev)
        r.update({"call": call, "cuda_init_ms": init_ms if call == 0 else None})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
