"""ResNet-50 inference on one MI355X, without the Data pipeline: HIP-graph
forward (uint8 in HBM -> class ids), and the full host-batch path
(numpy -> pinned staging -> HBM -> graph). Separates GPU speed from pipeline
overheads in tools/bench_data.py.

    python tools/bench_resnet.py --batch-size 512 --iters 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cluster_anywhere_amd.models.resnet import ResNetPredictor, resnet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--model", default="resnet50")
    args = ap.parse_args()
    bs = args.batch_size
    gflop = resnet(args.model).flops_per_image(224) / 1e9
    p = ResNetPredictor(args.model, batch_size=bs)
    res = {"model": args.model, "batch_size": bs}

    def timed(fn, n):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n

    dt = timed(lambda: p.graph.replay(), args.iters)
    res["graph_ms"] = round(dt * 1e3, 2)
    res["graph_img_s"] = round(bs / dt, 1)
    res["graph_tflops"] = round(bs * gflop / dt / 1e3, 1)
    dt = timed(lambda: p._run(p.static_in), args.iters)
    res["eager_img_s"] = round(bs / dt, 1)
    imgs = np.random.randint(0, 256, (bs, 224, 224, 3), dtype=np.uint8)
    dt = timed(lambda: p(imgs), args.iters)
    res["host_path_img_s"] = round(bs / dt, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
