"""Actor workers do not count against the per-node pooled-worker soft cap
(reference: src/ray/raylet/worker_pool.cc soft limit applies to task workers;
dedicated actor workers are always started). Regression: with 1 CPU the cap is 4
workers, and 6 zero-CPU actors used to starve every later task of a worker."""
import cluster_anywhere_amd as ray


@ray.remote(num_cpus=0)
class Holder:
    def ping(self):
        return 1


@ray.remote
def task(x):
    return x + 1


def test_actors_do_not_starve_task_workers():
    ray.init(num_cpus=1)
    try:
        hs = [Holder.remote() for _ in range(6)]
        assert ray.get([h.ping.remote() for h in hs]) == [1] * 6
        assert ray.get([task.remote(i) for i in range(4)], timeout=60) == [1, 2, 3, 4]
    finally:
        ray.shutdown()
