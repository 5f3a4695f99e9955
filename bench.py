#!/usr/bin/env python
"""Headline benchmark: TorchTrainer DDP training throughput (tokens/s) of GPT-2-XL
on MI355X (BASELINE.json / BASELINE.md).

    python bench.py --gpus 1 --steps 10 --warmup 3          # 1 GPU
    python bench.py --gpus 8 --steps 10 --warmup 3          # 8 GPUs, no launcher needed
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 10 --warmup 3

Default ``--mode actor`` (the reference's architecture, python/ray/train/
_internal/backend_executor.py:69 + worker_group.py:102): this process is the
driver and never touches a GPU. ``TorchTrainer.fit()`` reserves a PACK placement
group of N one-GPU bundles, starts N ``_TrainWorker`` actors (fresh processes,
one per MI355X), runs ``TorchConfig.on_start`` in each (RCCL process group over
xGMI) and then ``train_loop_per_worker`` on every rank. When a torch.distributed
launcher started N copies of this script, rank 0 becomes the driver and the other
launcher ranks exit at once (they hold no GPU), so the same actor worker group is
what gets measured either way. ``--mode spmd`` keeps the launcher's processes as
the ranks (``TorchTrainer`` SPMD mode).

The per-rank step is the framework's fused data-parallel step: flat bf16 weights
+ fp32 master, bucketed RCCL gradient reduction overlapped with backward (ZeRO-1
reduce-scatter / all-gather overlapped with the next forward when N>1), one fused
HIP AdamW launch, hand-written HIP GEMM / LayerNorm / bias-GELU / cross-entropy /
MFMA flash-attention kernels. Synthetic tokens, random init, fixed work per GPU
(weak scaling). The K timed steps are bracketed by barrier + synchronize, time =
max over ranks; one JSON line is printed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

_LAUNCHER_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                  "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=("actor", "spmd"), default=os.environ.get("CAAMD_BENCH_MODE", "actor"))
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--micro-batch", type=int, default=int(os.environ.get("CAAMD_MBS", "32")))
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--zero", type=int, default=int(os.environ.get("CAAMD_ZERO", "1")),
                    help="1 = ZeRO-1 sharded optimizer when world > 1")
    ap.add_argument("--cpu", action="store_true", help=argparse.SUPPRESS)  # gloo/CPU rehearsal (tests)
    return ap.parse_args(argv)


def train_loop_per_worker(cfg):
    import torch
    import torch.distributed as dist

    from cluster_anywhere_amd import train
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config
    from cluster_anywhere_amd.train.loop import DataParallelStep
    from cluster_anywhere_amd.train.torch import get_device

    ctx = train.get_context()
    world, rank = ctx.get_world_size(), ctx.get_world_rank()
    device = get_device()
    on_gpu = device.type == "cuda"
    torch.manual_seed(1234)
    mcfg = GPT2Config.named(cfg["model"])
    with torch.device(device):  # random init straight in HBM (no 6 GB host copy per rank)
        model = GPT2(mcfg)
    step = DataParallelStep(model, lr=1e-4, weight_decay=0.1, max_grad_norm=1.0,
                            bucket_cap_mb=cfg["bucket_mb"], zero=bool(cfg["zero"]) and world > 1)
    B, T = cfg["micro_batch"], cfg["seq_len"]
    gen = torch.Generator(device=device)
    gen.manual_seed(rank + 1)

    def batch():
        x = torch.randint(0, mcfg.vocab_size, (B, T + 1), device=device, generator=gen)
        return x[:, :-1], x[:, 1:]

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        if on_gpu:
            torch.cuda.synchronize()

    for _ in range(cfg["warmup"]):
        step(*batch())
    sync()
    t0 = time.perf_counter()
    last = None
    for _ in range(cfg["steps"]):
        last = step(*batch())
    sync()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    train.report({
        "dt": dt, "loss": float(last.item()), "world": world, "params": model.num_params(),
        "flops_per_token": model.flops_per_token(T), "zero": step.zero, "pid": os.getpid(),
        "peak_mem_gb": (torch.cuda.max_memory_allocated(device) / 2**30) if on_gpu else 0.0,
    })


def _fit(args, cfg):
    from cluster_anywhere_amd.train import RunConfig, ScalingConfig
    from cluster_anywhere_amd.train.torch import TorchConfig, TorchTrainer

    trainer = TorchTrainer(
        train_loop_per_worker, train_loop_config=cfg,
        torch_config=TorchConfig(backend="gloo" if args.cpu else None),
        scaling_config=ScalingConfig(num_workers=args.gpus, use_gpu=not args.cpu,
                                     placement_strategy="PACK"),
        run_config=RunConfig(name=f"bench_gpt2xl_n{args.gpus}_{args.mode}",
                             storage_path=os.environ.get("CAAMD_STORAGE_PATH", "/tmp/caamd_results")))
    return trainer.fit()


def run(argv=None):
    args = parse(argv)
    launched = "WORLD_SIZE" in os.environ and ("LOCAL_RANK" in os.environ or "TORCHELASTIC_RUN_ID" in os.environ)
    launcher_rank = int(os.environ.get("RANK", "0")) if launched else 0
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cfg = {"model": args.model, "micro_batch": args.micro_batch, "seq_len": args.seq_len,
           "warmup": args.warmup, "steps": args.steps, "bucket_mb": args.bucket_mb, "zero": args.zero}

    if args.mode == "actor":
        if launched and launcher_rank != 0:
            return None  # the driver (launcher rank 0) owns every GPU through its actors
        for k in _LAUNCHER_VARS:
            os.environ.pop(k, None)
        for k in [k for k in os.environ if k.startswith("TORCHELASTIC_")]:
            os.environ.pop(k, None)
        import cluster_anywhere_amd as ray

        if args.cpu:
            ray.init(num_cpus=max(4, args.gpus + 2), num_gpus=0, include_dashboard=False)
        else:
            from cluster_anywhere_amd.core.api import detect_gpus

            n = len(detect_gpus())
            if n < args.gpus:
                raise SystemExit(f"--gpus {args.gpus}: only {n} GPU(s) visible on this node")
            ray.init(num_gpus=n, include_dashboard=False)
        try:
            m = _fit(args, cfg).metrics
        finally:
            ray.shutdown()
    else:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if args.gpus > 1 and world != args.gpus:
            raise SystemExit(f"--mode spmd --gpus {args.gpus} needs a torch.distributed launcher "
                             f"with WORLD_SIZE={args.gpus} (or use the default --mode actor)")
        for k, v in (("WORLD_SIZE", "1"), ("RANK", "0"), ("LOCAL_RANK", "0"),
                     ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", os.environ.get("MASTER_PORT", "29533"))):
            os.environ.setdefault(k, v)
        m = _fit(args, cfg).metrics
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
        if launcher_rank != 0:
            return None

    world = m["world"]
    tokens = args.micro_batch * args.seq_len * args.steps * world
    tps = tokens / m["dt"]
    out = {
        "metric": "TorchTrainer DDP tokens/sec (GPT-2-XL)",
        "value": round(tps, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(m["dt"] / args.steps * 1000, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32" if args.cpu else "bf16",
        "data": "synthetic random tokens, random-init weights",
        "config": {
            "model": args.model,
            "params": m["params"],
            "global_batch": args.micro_batch * world,
            "micro_batch_per_gpu": args.micro_batch,
            "seq_len": args.seq_len,
            "parallelism": f"dp{world}" + ("-zero1" if m["zero"] else ""),
            "mode": args.mode,
            "optimizer": "fused AdamW (fp32 master, bf16 weights/grads), grad clip 1.0",
        },
        "mfu_bf16_dense": round(tps / world * m["flops_per_token"] / 2.5e15, 4),
        "final_loss": round(m["loss"], 4),
        "peak_mem_gb": round(m["peak_mem_gb"], 1),
    }
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    run()
