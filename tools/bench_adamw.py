"""Fused AdamW over a GPT-2-XL-sized flat buffer (1.56 B params: fp32 master, m, v,
bf16 grad, bf16 weight copy) for each kernel variant (adamw_config: bit 0
non-temporal loads/stores, bit 1 two vectors per thread per iteration).
python tools/bench_adamw.py -> one JSON line per variant (ms, TB/s)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from cluster_anywhere_amd.ops import kernels

    k = kernels()
    n = 1_557_611_200 // 64 * 64
    p = torch.randn(n, device="cuda")
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    g = (torch.randn(n, device="cuda") * 1e-3).bfloat16()
    pbf = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    ss = torch.zeros(1, device="cuda")
    res = {}
    for variant in (2, 0, 6, 4, 8, 12, 2, 0, 6, 4, 8, 12):
        k.adamw_config(variant)
        for _ in range(2):
            k.adamw_step(p, m, v, g, pbf, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1, 1.0, 0.0, None, None)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            k.adamw_step(p, m, v, g, pbf, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1, 1.0, 0.0, None, None)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        res.setdefault(variant, []).append(ms)
    k.adamw_config(0)
    for variant, ms in res.items():
        print(json.dumps({"variant": variant, "ms": [round(x, 3) for x in ms],
                          "tbps": round(n * 28 / min(ms) / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
