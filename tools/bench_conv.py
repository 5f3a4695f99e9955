"""Per-shape timing of the implicit-GEMM NHWC conv (csrc/kernels/conv.hip) over
every distinct ResNet-50 convolution at batch B, for each valid tile, against
MIOpen (channels_last F.conv2d + the bias/act epilogue kernel it needs).

python tools/bench_conv.py [--batch 512] [--iters 20]
One JSON line per shape: us per call per variant, TF/s, and the share of the
network's conv time (weighted by how often the shape occurs).
"""
import argparse
import json
import os
import sys
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def shapes(hw=224):
    from cluster_anywhere_amd.models.resnet import resnet

    net = resnet("resnet50")
    out = OrderedDict()

    def add(h, conv, res):
        k = conv.kernel_size[0]
        s, p = conv.stride[0], conv.padding[0]
        cin = max(8, conv.in_channels)
        key = (h, cin, conv.out_channels, k, s, p, res)
        out[key] = out.get(key, 0) + 1
        return (h + 2 * p - k) // s + 1

    h = add(hw, net.conv1, False)
    h = (h + 2 - 3) // 2 + 1
    for b in net.blocks:
        h_in = h
        convs = b.convs()
        for i, (conv, _, _) in enumerate(convs):
            h = add(h, conv, i == len(convs) - 1)
        if b.down is not None:
            add(h_in, b.down[0], False)
    return out


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tiles", default="0,1,2")
    args = ap.parse_args()
    from cluster_anywhere_amd.ops import kernels
    from cluster_anywhere_amd.ops.vision import _zero_page, conv_tile, conv_weight_nhwc

    k = kernels()
    B = args.batch
    tot = {"own": 0.0, "miopen": 0.0}
    for (h, cin, cout, ks, s, p, res), cnt in shapes().items():
        ho = (h + 2 * p - ks) // s + 1
        x = torch.randn(B, h, h, cin, device="cuda").bfloat16()
        w4 = (torch.randn(cout, cin, ks, ks, device="cuda") / (cin * ks * ks) ** 0.5).bfloat16()
        w2 = conv_weight_nhwc(w4.float(), cin).bfloat16()
        b = torch.zeros(cout, device="cuda").bfloat16()
        r = torch.randn(B, ho, ho, cout, device="cuda").bfloat16() if res else None
        flops = 2.0 * B * ho * ho * cout * cin * ks * ks
        row = {"shape": [B, h, cin, cout, ks, s, res], "count": cnt}
        best = None
        for t in (int(v) for v in args.tiles.split(",")):
            if cout % (64 if t == 1 else 128):
                continue
            us = timeit(lambda: k.conv2d_nhwc(x, w2, b, r, ks, s, p, True, t, _zero_page(x.device)), args.iters)
            row[f"tile{t}_us"] = round(us, 1)
            best = us if best is None else min(best, us)
        row["auto_tile"] = conv_tile(B * ho * ho, cout, cin * ks * ks, res)
        auto_us = row[f"tile{row['auto_tile']}_us"]
        xc = x.permute(0, 3, 1, 2)  # channels_last view of the NHWC tensor
        wc = w4.contiguous(memory_format=torch.channels_last)
        rc = r.permute(0, 3, 1, 2) if r is not None else None

        def lib():
            y = F.conv2d(xc, wc, None, s, p)
            return k.bias_act_(y, b, rc, True)

        mi = timeit(lib, args.iters)
        row.update(miopen_us=round(mi, 1), auto_tflops=round(flops / auto_us / 1e6, 1),
                   best_tflops=round(flops / best / 1e6, 1), miopen_tflops=round(flops / mi / 1e6, 1))
        tot["own"] += cnt * auto_us
        tot["miopen"] += cnt * mi
        print(json.dumps(row), flush=True)
        del x, r
    print(json.dumps({"total_us": {k_: round(v, 1) for k_, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
