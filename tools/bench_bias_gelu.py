"""Time the fused bias+GELU forward at the GPT-2-XL MLP shape (32768 x 6400 bf16)
and check it against the fp32 PyTorch reference."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cluster_anywhere_amd.ops import kernels  # noqa: E402


def main():
    C = kernels()
    R, N = 32768, 6400
    torch.manual_seed(0)
    h = torch.randn(R, N, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    y = C.bias_gelu_fwd(h, b)
    ref = torch.nn.functional.gelu(h.float() + b.float(), approximate="tanh")
    err = float((y.float() - ref).abs().max())
    for _ in range(3):
        C.bias_gelu_fwd(h, b)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        C.bias_gelu_fwd(h, b)
    e.record()
    e.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    print(json.dumps({"kernel": "bias_gelu_fwd", "shape": [R, N], "us": round(us, 1),
                      "TB_s": round(2 * R * N * 2 / us / 1e6, 2), "maxerr": err}))


if __name__ == "__main__":
    main()
