#!/usr/bin/env python
"""RLlib throughput benchmark (BASELINE.json config "RLlib PPO Atari, GPU Learners +
CPU rollout actors"): PPO on FakeAtari-v0 (84x84x4 uint8 frames, Atari-shaped,
synthetic dynamics — no ALE ROMs offline) with the Nature-CNN actor-critic.

    python tools/bench_rllib.py --runners 8 --envs-per-runner 4 --iters 5

Env runners are CPU actors; the learner runs on the GPU (GAE HIP kernel, flat
buffers + fused AdamW). Reports env steps sampled+trained per second over the
timed iterations (after one warm-up iteration), split into sample / learn time.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runners", type=int, default=8)
    ap.add_argument("--envs-per-runner", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--train-batch", type=int, default=4000)
    ap.add_argument("--minibatch", type=int, default=500)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--runner-gpus", type=float, default=0.0,
                    help="num_gpus_per_env_runner: runners act on a GPU share (weights over HIP IPC)")
    ap.add_argument("--seconds", type=float, default=0.0,
                    help="run timed iterations until at least this many seconds passed (>= --iters)")
    args = ap.parse_args()
    import torch

    import cluster_anywhere_amd as ray
    from cluster_anywhere_amd import rllib

    gpu = torch.cuda.is_available() and args.gpus > 0
    # the local learner uses the GPU outside the scheduler; runner shares are booked against it
    ray.init(num_cpus=args.runners + 2, num_gpus=args.gpus if gpu else 0)
    cfg = (rllib.PPOConfig().environment("FakeAtari-v0")
           .env_runners(num_env_runners=args.runners, num_envs_per_env_runner=args.envs_per_runner,
                        num_gpus_per_env_runner=args.runner_gpus if gpu else 0)
           .learners(num_learners=0, num_gpus_per_learner=1 if gpu else 0)
           .training(train_batch_size=args.train_batch, minibatch_size=args.minibatch,
                     num_epochs=args.epochs, lr=2.5e-4, lambda_=0.95, clip_param=0.1, entropy_coeff=0.01)
           .debugging(seed=0))
    algo = cfg.build()
    algo.train()  # warm-up: actor start, kernel loads
    t0 = time.perf_counter()
    s0 = algo.env_steps_sampled
    samp = learn = 0.0
    it = 0
    last = t0
    while it < args.iters or time.perf_counter() - t0 < args.seconds:
        r = algo.train()
        it += 1
        samp += r.get("timers", {}).get("sample_s", 0.0)
        learn += r.get("timers", {}).get("learn_s", 0.0)
        if time.perf_counter() - last > 10:
            last = time.perf_counter()
            print(json.dumps({"progress_s": round(last - t0, 1), "iters": it,
                              "env_steps_per_s": round((algo.env_steps_sampled - s0) / (last - t0), 1),
                              "episode_return_mean": r["env_runners"].get("episode_return_mean")}), flush=True)
    args.iters = it
    dt = time.perf_counter() - t0
    steps = algo.env_steps_sampled - s0
    print(json.dumps({
        "metric": "RLlib PPO env steps/sec (FakeAtari 84x84x4, Nature-CNN)", "value": round(steps / dt, 1),
        "unit": "env_steps/s", "n_gpus": args.gpus if gpu else 0, "iters": args.iters, "seconds": round(dt, 2),
        "higher_is_better": True, "data": "synthetic Atari-shaped env, random-init weights",
        "config": {"runners": args.runners, "envs_per_runner": args.envs_per_runner,
                   "train_batch_size": args.train_batch, "minibatch_size": args.minibatch,
                   "num_epochs": args.epochs, "learner_device": "cuda" if gpu else "cpu",
                   "runner_device": "cuda" if gpu and args.runner_gpus else "cpu",
                   "weights_transport": "ipc" if algo._ipc_weights() else "object store"},
        "sample_s": round(samp, 2), "learn_s": round(learn, 2),
        "learner_samples_per_s": round(steps * args.epochs / max(learn, 1e-9), 1),
    }), flush=True)
    algo.stop()
    ray.shutdown()


if __name__ == "__main__":
    main()
