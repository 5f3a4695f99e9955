"""Core-runtime microbenchmarks: the metric set of the reference's
``ray microbenchmark`` (python/ray/_private/ray_perf.py; published numbers in
release/perf_metrics/microbenchmark.json, quoted in BASELINE.md), plus compiled-
graph round trips over our native shm channels.

    python tools/microbenchmark.py [--only substr] [--seconds 1.0] [--json out.json]

Each metric: 0.5 s warm-up, then R rounds of ``--seconds`` each; prints
"name  mean ± sd /s  (ref X, ratio)". CPU-only (pure runtime plumbing).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import cluster_anywhere_amd as ray  # noqa: E402

REF = os.path.join("/root/reference/release/perf_metrics/microbenchmark.json")
REF_NAMES = {
    "single client get calls (Plasma Store)": "single_client_get_calls_Plasma_Store",
    "single client put calls (Plasma Store)": "single_client_put_calls_Plasma_Store",
    "multi client put calls (Plasma Store)": "multi_client_put_calls_Plasma_Store",
    "single client put gigabytes": "single_client_put_gigabytes",
    "multi client put gigabytes": "multi_client_put_gigabytes",
    "single client tasks and get batch": "single_client_tasks_and_get_batch",
    "single client wait 1k refs": "single_client_wait_1k_refs",
    "single client tasks sync": "single_client_tasks_sync",
    "single client tasks async": "single_client_tasks_async",
    "multi client tasks async": "multi_client_tasks_async",
    "1:1 actor calls sync": "1_1_actor_calls_sync",
    "1:1 actor calls async": "1_1_actor_calls_async",
    "1:1 actor calls concurrent": "1_1_actor_calls_concurrent",
    "1:n actor calls async": "1_n_actor_calls_async",
    "n:n actor calls async": "n_n_actor_calls_async",
    "1:1 async-actor calls sync": "1_1_async_actor_calls_sync",
    "1:1 async-actor calls async": "1_1_async_actor_calls_async",
}


def _ref_numbers():
    try:
        with open(REF) as f:
            d = json.load(f)
        return {k: v[0] for k, v in d.items() if isinstance(v, list)}
    except (OSError, ValueError):
        return {}


@ray.remote
def small_value():
    return b"ok"


@ray.remote
class Actor:
    def small_value(self):
        return b"ok"

    def small_value_batch(self, n):
        ray.get([small_value.remote() for _ in range(n)])


@ray.remote
class AsyncActor:
    async def small_value(self):
        return b"ok"


@ray.remote
class Client:
    def __init__(self, servers):
        self.servers = servers if isinstance(servers, list) else [servers]

    def small_value_batch(self, n):
        refs = []
        for s in self.servers:
            refs += [s.small_value.remote() for _ in range(n)]
        ray.get(refs)


@ray.remote
def do_put_small():
    for _ in range(100):
        ray.put(0)


@ray.remote
def do_put():
    for _ in range(10):
        ray.put(np.zeros(10 * 1024 * 1024, dtype=np.int64))


@ray.remote
class Echo:
    def echo(self, x):
        return x


class Bench:
    def __init__(self, seconds, rounds, only):
        self.seconds, self.rounds, self.only = seconds, rounds, only
        self.results = []
        self.ref = _ref_numbers()

    def run(self, name, fn, multiplier=1.0):
        if self.only and self.only not in name:
            return
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 0.5:
            fn()
            n += 1
        step = max(1, n // 5)
        rates = []
        for _ in range(self.rounds):
            t0 = time.perf_counter()
            c = 0
            while time.perf_counter() - t0 < self.seconds:
                for _ in range(step):
                    fn()
                c += step
            rates.append(multiplier * c / (time.perf_counter() - t0))
        mean, sd = float(np.mean(rates)), float(np.std(rates))
        ref = self.ref.get(REF_NAMES.get(name, ""))
        extra = f"  (ref {ref:.1f}, x{mean / ref:.2f})" if ref else ""
        print(f"{name:48s} {mean:12.1f} ± {sd:8.1f} /s{extra}", flush=True)
        self.results.append({"name": name, "per_second": round(mean, 2), "sd": round(sd, 2),
                             "reference": ref, "ratio": round(mean / ref, 3) if ref else None})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    ncpu = multiprocessing.cpu_count()
    ray.init(num_cpus=max(8, ncpu), object_store_memory=4 << 30)
    b = Bench(args.seconds, args.rounds, args.only)

    value = ray.put(0)
    b.run("single client get calls (Plasma Store)", lambda: ray.get(value))
    b.run("single client put calls (Plasma Store)", lambda: ray.put(0))
    b.run("multi client put calls (Plasma Store)",
          lambda: ray.get([do_put_small.remote() for _ in range(10)]), 1000)
    arr = np.zeros(100 * 1024 * 1024, dtype=np.int64)
    b.run("single client put gigabytes", lambda: ray.put(arr), 8 * 0.1)
    del arr
    b.run("single client tasks and get batch",
          lambda: ray.get([small_value.remote() for _ in range(1000)]))
    b.run("multi client put gigabytes", lambda: ray.get([do_put.remote() for _ in range(10)]), 10 * 8 * 0.1)

    def wait_1k():
        pending = [small_value.remote() for _ in range(1000)]
        while pending:
            _, pending = ray.wait(pending)

    b.run("single client wait 1k refs", wait_1k)
    b.run("single client tasks sync", lambda: ray.get(small_value.remote()))
    b.run("single client tasks async", lambda: ray.get([small_value.remote() for _ in range(1000)]), 1000)
    m, n = 4, 2000
    actors = [Actor.remote() for _ in range(m)]
    b.run("multi client tasks async", lambda: ray.get([a.small_value_batch.remote(n) for a in actors]), n * m)
    a = Actor.remote()
    b.run("1:1 actor calls sync", lambda: ray.get(a.small_value.remote()))
    b.run("1:1 actor calls async", lambda: ray.get([a.small_value.remote() for _ in range(1000)]), 1000)
    ac = Actor.options(max_concurrency=16).remote()
    b.run("1:1 actor calls concurrent", lambda: ray.get([ac.small_value.remote() for _ in range(1000)]), 1000)
    k = max(2, ncpu // 2)
    servers = [Actor.remote() for _ in range(k)]
    client = Client.remote(servers)
    b.run("1:n actor calls async", lambda: ray.get(client.small_value_batch.remote(1000)), 1000 * k)
    clients = [Client.remote(servers[i % k]) for i in range(m)]
    b.run("n:n actor calls async", lambda: ray.get([c.small_value_batch.remote(1000) for c in clients]), 1000 * m)
    aa = AsyncActor.remote()
    b.run("1:1 async-actor calls sync", lambda: ray.get(aa.small_value.remote()))
    b.run("1:1 async-actor calls async", lambda: ray.get([aa.small_value.remote() for _ in range(1000)]), 1000)

    # compiled graph over shm channels vs the same call through task submission
    from cluster_anywhere_amd.dag import InputNode

    e = Echo.remote()
    with InputNode() as inp:
        dag = e.echo.bind(inp)
    cdag = dag.experimental_compile()
    b.run("compiled graph 1:1 actor round trip sync", lambda: ray.get(cdag.execute(b"x")))
    b.run("compiled graph 1:1 actor calls pipelined",
          lambda: [ray.get(r) for r in [cdag.execute(b"x") for _ in range(100)]], 100)
    cdag.teardown()
    ray.shutdown()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(b.results, f, indent=1)


if __name__ == "__main__":
    main()
