#!/usr/bin/env python
"""Headline benchmark: TorchTrainer DDP training throughput (tokens/s) of GPT-2-XL
on MI355X (BASELINE.json / BASELINE.md).

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 10 --warmup 3

Every rank runs ``TorchTrainer.fit()`` in SPMD mode (the trainer detects the
torch.distributed launch and runs ``train_loop_per_worker`` on this rank, with
the RCCL process group over xGMI). The loop uses the framework's fused data-
parallel step: flat bf16 weights + fp32 master, bucketed RCCL gradient
reduction overlapped with backward (ZeRO-1 reduce-scatter/all-gather when N>1),
one fused HIP AdamW launch, hand-written HIP LayerNorm / bias-GELU /
cross-entropy / MFMA flash-attention kernels. Synthetic tokens, random init,
fixed work per GPU (weak scaling). The K timed steps are bracketed by barrier +
synchronize, time = max over ranks; rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--micro-batch", type=int, default=int(os.environ.get("CAAMD_MBS", "32")))
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--zero", type=int, default=int(os.environ.get("CAAMD_ZERO", "1")),
                    help="1 = ZeRO-1 sharded optimizer when world > 1")
    return ap.parse_args()


def train_loop_per_worker(cfg):
    import torch
    import torch.distributed as dist

    from cluster_anywhere_amd import train
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config
    from cluster_anywhere_amd.train.loop import DataParallelStep

    ctx = train.get_context()
    world, rank = ctx.get_world_size(), ctx.get_world_rank()
    device = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(1234)
    mcfg = GPT2Config.named(cfg["model"])
    model = GPT2(mcfg).to(device)
    step = DataParallelStep(model, lr=1e-4, weight_decay=0.1, max_grad_norm=1.0,
                            bucket_cap_mb=cfg["bucket_mb"], zero=bool(cfg["zero"]) and world > 1)
    B, T = cfg["micro_batch"], cfg["seq_len"]
    gen = torch.Generator(device=device)
    gen.manual_seed(rank + 1)

    def batch():
        x = torch.randint(0, mcfg.vocab_size, (B, T + 1), device=device, generator=gen)
        return x[:, :-1], x[:, 1:]

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
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
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    if rank == 0 and os.environ.get("CAAMD_TUNE_GEMMS"):
        from cluster_anywhere_amd.ops.gemm_tuning import dump_tuned

        dump_tuned()  # online-tuned table for this shape set (see ops/gemm_tuning.py)
    train.report({
        "dt": dt, "loss": float(last.item()), "world": world, "params": model.num_params(),
        "flops_per_token": model.flops_per_token(T), "zero": step.zero,
        "peak_mem_gb": torch.cuda.max_memory_allocated(device) / 2**30,
    })


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} needs a torch.distributed launcher with WORLD_SIZE={args.gpus}")
    import torch

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (torch.cuda.is_available() is False)")
    # single GPU without a launcher: this process is rank 0 of a world of 1
    for k, v in (("WORLD_SIZE", "1"), ("RANK", "0"), ("LOCAL_RANK", "0"),
                 ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", os.environ.get("MASTER_PORT", "29533"))):
        os.environ.setdefault(k, v)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    os.environ.setdefault("CAAMD_STORAGE_PATH", "/tmp/caamd_results")

    from cluster_anywhere_amd.train import RunConfig, ScalingConfig
    from cluster_anywhere_amd.train.torch import TorchTrainer

    cfg = {"model": args.model, "micro_batch": args.micro_batch, "seq_len": args.seq_len,
           "warmup": args.warmup, "steps": args.steps, "bucket_mb": args.bucket_mb, "zero": args.zero}
    trainer = TorchTrainer(train_loop_per_worker, train_loop_config=cfg,
                           scaling_config=ScalingConfig(num_workers=args.gpus, use_gpu=True),
                           run_config=RunConfig(name=f"bench_gpt2xl_n{args.gpus}"))
    result = trainer.fit()
    m = result.metrics
    rank = int(os.environ["RANK"])
    world = m["world"]
    if rank == 0:
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
            "dtype": "bf16",
            "data": "synthetic random tokens, random-init weights",
            "config": {
                "model": args.model,
                "params": m["params"],
                "global_batch": args.micro_batch * world,
                "micro_batch_per_gpu": args.micro_batch,
                "seq_len": args.seq_len,
                "parallelism": f"dp{world}" + ("-zero1" if m["zero"] else ""),
                "optimizer": "fused AdamW (fp32 master, bf16 weights/grads), grad clip 1.0",
            },
            "mfu_bf16_dense": round(tps / world * m["flops_per_token"] / 2.5e15, 4),
            "final_loss": round(m["loss"], 4),
            "peak_mem_gb": round(m["peak_mem_gb"], 1),
        }
        print(json.dumps(out), flush=True)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
