#!/usr/bin/env python
"""Data GPU throughput benchmark (BASELINE.json secondary metric: "Ray Data
streaming map_batches ResNet-50 inference, N GPU actors").

    python tools/bench_data.py --gpus 1 --rows 60000 [--batch-size 512]

Pipeline (one driver process; N GPU actors on this node):
  read (synthetic uint8 224x224x3 images, CPU tasks) ->
  map_batches(ResNet50Actor, num_gpus=1, concurrency=N, batch_size=B) ->
  iter_batches (driver consumes the predicted class ids).
Each actor runs the BN-folded bf16 channels_last ResNet-50 as one HIP-graph
replay per batch, with the uint8 batch staged host->HBM through a pinned buffer
on a side stream and normalised by a HIP kernel. The timed region covers the
whole streaming execution of ``--rows`` rows, INCLUDING building the GPU actor
pool (model init + HIP-graph capture; a dataset execution owns its pool); a
warm-up execution first loads the kernels/libraries. Also reported: time to the
first output batch and the steady-state rows/s after it.
Rank 0 prints one JSON line; ``value`` = rows/s over all N GPUs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_images(batch, hw=224):
    ids = batch["id"]
    if os.environ.get("CAAMD_BENCH_DATA_TRACE") == "1":
        print("READ " + json.dumps({"id0": int(ids[0]), "t": time.time(), "pid": os.getpid()}), flush=True)
    img = np.empty((len(ids), hw, hw, 3), dtype=np.uint8)
    img[:] = (ids % 251).astype(np.uint8)[:, None, None, None]
    return {"image": img, "id": ids}


class StubActor:
    """``--stub``: no model, no GPU -- the actor only touches its batch (one byte
    per image) so the run measures the read -> object store -> actor -> driver
    plumbing that the GPU actors sit on (the host-side ceiling of the pipeline)."""

    def __init__(self, **_):
        if os.environ.get("CAAMD_BENCH_DATA_TRACE") == "1":
            print("ACTOR_TIMES " + json.dumps({"enter": time.time(), "pid": os.getpid()}), flush=True)

    def __call__(self, batch):
        return {"id": batch["id"], "label": batch["image"][:, 0, 0, 0].astype(np.int64)}


class ResNet50Actor:
    def __init__(self, model="resnet50", batch_size=512, hw=224):
        t_enter = time.time()
        from cluster_anywhere_amd.models.resnet import ResNetPredictor

        self.p = ResNetPredictor(model, batch_size=batch_size, hw=hw)
        if os.environ.get("CAAMD_BENCH_DATA_TRACE") == "1":  # start-up timeline (worker log -> driver)
            print("ACTOR_TIMES " + json.dumps({"enter": t_enter, "ready": time.time(), "pid": os.getpid(),
                                               **{k: round(v, 3) for k, v in self.p.init_profile.items()}}),
                  flush=True)

    def __call__(self, batch):
        if os.environ.get("CAAMD_BENCH_DATA_TRACE") == "1" and not getattr(self, "_traced", False):
            self._traced = True
            t = time.time()
            out = {"id": batch["id"], "label": self.p(batch["image"])}
            print("ACTOR_FIRST_CALL " + json.dumps({"t": t, "done": time.time(), "pid": os.getpid()}), flush=True)
            return out
        return {"id": batch["id"], "label": self.p(batch["image"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--rows", type=int, default=204800)
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--read-blocks", type=int, default=0)
    ap.add_argument("--cpus", type=int, default=0)
    ap.add_argument("--actors-per-gpu", type=int, default=3,
                    help=">1 shares each GPU between actors (fractional num_gpus) so one's H2D "
                         "copy / host work overlaps another's graph replay")
    ap.add_argument("--stub", action="store_true", help="GPU-less stub actors (plumbing ceiling, see StubActor)")
    ap.add_argument("--timeline", default="", help="write a chrome trace + per-function summary here")
    ap.add_argument("--preserve-order", action="store_true",
                    help="deliver blocks in input order (off by default, as in the reference's DataContext)")
    args = ap.parse_args()
    import torch

    import cluster_anywhere_amd as ray
    from cluster_anywhere_amd import data

    gpu = torch.cuda.is_available()
    data.DataContext.get_current().execution_preserve_order = args.preserve_order
    ncpu = args.cpus or min(os.cpu_count() or 8, 16 * max(1, args.gpus))
    ray.init(num_cpus=ncpu, num_gpus=args.gpus if gpu and not args.stub else 0,
             object_store_memory=min(64 << 30, max(4 << 30, args.batch_size * args.hw * args.hw * 3 * 64)))
    # whole batches per block: a block of batch_size+1 rows would cost the actor a
    # second (padded) graph replay for its 1-row remainder
    per = args.batch_size * max(1, args.gpus)
    args.rows = max(per, (args.rows // per) * per)
    blocks = args.read_blocks or max(1, args.rows // args.batch_size)

    def pipeline(n):
        ds = data.range(n, override_num_blocks=max(1, min(blocks, n // args.batch_size or 1)))
        ds = ds.map_batches(make_images, batch_size=args.batch_size, fn_kwargs={"hw": args.hw})
        apg = max(1, args.actors_per_gpu)
        ds = ds.map_batches(StubActor if args.stub else ResNet50Actor, batch_size=args.batch_size,
                            num_gpus=(1.0 / apg) if gpu and not args.stub else 0,
                            **({"num_cpus": min(0.25, ncpu / (2.0 * args.gpus * max(1, args.actors_per_gpu)))}
                               if args.stub else {}),
                            concurrency=max(1, args.gpus) * apg, zero_copy_batch=True,
                            fn_constructor_kwargs={"model": args.model, "batch_size": args.batch_size,
                                                   "hw": args.hw})
        return ds

    # warm-up: builds the actor pool (model init + HIP graph capture)
    ds = pipeline(args.batch_size * max(1, args.gpus) * 2)
    warm = sum(len(b["label"]) for b in ds.iter_batches(batch_size=None))
    t0 = time.perf_counter()
    if os.environ.get("CAAMD_BENCH_DATA_TRACE") == "1":
        print("T0 " + json.dumps({"t0": time.time()}), flush=True)
    ds = pipeline(args.rows)
    n, n_first, t_first = 0, 0, None
    for b in ds.iter_batches(batch_size=None):
        if t_first is None:  # the actor pool is built per execution: model init + graph capture
            t_first, n_first = time.perf_counter(), len(b["label"])
            if os.environ.get("CAAMD_BENCH_DATA_TRACE") == "1":
                print("FIRST " + json.dumps({"t_first": time.time()}), flush=True)
        n += len(b["label"])
    dt = time.perf_counter() - t0
    t_end = time.perf_counter()
    assert n == args.rows, (n, args.rows)
    rps = n / dt
    from cluster_anywhere_amd.models.resnet import resnet

    gflop = 0.0 if args.stub else resnet(args.model).flops_per_image(args.hw) / 1e9
    stats = ds.stats()
    print(json.dumps({
        "metric": "Data GPU rows/sec (map_batches ResNet-50 inference)",
        "value": round(rps, 1), "unit": "rows/s", "n_gpus": args.gpus, "rows": n, "warmup_rows": warm,
        "seconds": round(dt, 3), "higher_is_better": True, "scaling": "strong",
        "dtype": "bf16" if gpu else "fp32", "data": "synthetic uint8 224x224x3 images, random-init weights",
        "config": {"model": "stub (no model, no GPU)" if args.stub else args.model, "batch_size": args.batch_size,
                   "hw": args.hw, "read_blocks": blocks,
                   "actors": args.gpus * max(1, args.actors_per_gpu), "cpus": ncpu,
                   "preserve_order": args.preserve_order},
        "model_tflops_per_gpu": round(rps * gflop / 1e3 / max(1, args.gpus), 1),
        "time_to_first_batch_s": round(t_first - t0, 3),
        "steady_state_rows_per_s": round((n - n_first) / max(1e-9, t_end - t_first), 1),
    }), flush=True)
    print(stats, flush=True)
    if args.timeline:
        ev = ray.timeline()
        with open(args.timeline, "w") as f:
            json.dump(ev, f)
        agg = {}
        for e in ev:
            if e.get("ph") == "X":
                a = agg.setdefault(e.get("name", "?"), [0, 0.0])
                a[0] += 1
                a[1] += e.get("dur", 0) / 1e3
        for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"timeline {k}: {c} calls, {ms:.0f} ms total, {ms / max(c, 1):.1f} ms avg", flush=True)
    ray.shutdown()


if __name__ == "__main__":
    main()
