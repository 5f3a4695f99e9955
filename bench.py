#!/usr/bin/env python
"""Headline benchmark: TorchTrainer-style DDP training throughput (tokens/s) of
GPT-2-XL on MI355X (BASELINE.json / BASELINE.md).

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 10 --warmup 3

Each rank runs the per-worker training loop of ``cluster_anywhere_amd.train``
(flat bf16 weights + fp32 master, bucketed RCCL all-reduce overlapped with
backward, fused HIP AdamW/LayerNorm/GELU/cross-entropy kernels, synthetic
tokens, random init). Work per GPU is fixed (weak scaling). Rank 0 prints one
JSON line; time = max over ranks of K timed steps between barriers.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--micro-batch", type=int, default=int(os.environ.get("CAAMD_MBS", "8")))
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--zero", type=int, default=int(os.environ.get("CAAMD_ZERO", "1")),
                    help="1 = ZeRO-1 sharded optimizer when world > 1")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(
            f"--gpus {args.gpus} needs a torch.distributed launcher with WORLD_SIZE={args.gpus}"
        )
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (torch.cuda.is_available() is False)")
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=device)

    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config
    from cluster_anywhere_amd.train.loop import DataParallelStep

    torch.manual_seed(1234)
    cfg = GPT2Config.named(args.model)
    model = GPT2(cfg).to(device)
    step = DataParallelStep(
        model,
        lr=1e-4,
        weight_decay=0.1,
        max_grad_norm=1.0,
        bucket_cap_mb=args.bucket_mb,
        zero=bool(args.zero) and world > 1,
    )
    B, T = args.micro_batch, args.seq_len
    gen = torch.Generator(device=device)
    gen.manual_seed(rank + 1)

    def batch():
        x = torch.randint(0, cfg.vocab_size, (B, T + 1), device=device, generator=gen)
        return x[:, :-1], x[:, 1:]

    for _ in range(args.warmup):
        step(*batch())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = step(*batch())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    loss = float(last.item()) if last is not None else float("nan")
    tokens = B * T * args.steps * world
    tps = tokens / dt
    ms = dt / args.steps * 1000
    flops_tok = model.flops_per_token(T)
    mfu = tps / world * flops_tok / 2.5e15
    if rank == 0:
        out = {
            "metric": "TorchTrainer DDP tokens/sec (GPT-2-XL)",
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic random tokens, random-init weights",
            "config": {
                "model": args.model,
                "params": model.num_params(),
                "global_batch": B * world,
                "micro_batch_per_gpu": B,
                "seq_len": T,
                "parallelism": f"dp{world}" + ("-zero1" if step.zero else ""),
                "optimizer": "fused AdamW (fp32 master, bf16 weights/grads), grad clip 1.0",
            },
            "mfu_bf16_dense": round(mfu, 4),
            "final_loss": round(loss, 4),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
