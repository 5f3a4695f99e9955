"""Core runtime tests that start their own cluster (local mode, fractional GPUs,
worker output to the driver, GPU ids after placement-group removal) -- kept apart
from test_core.py's module-scoped cluster, so a parallel runner that interleaves
modules never asks for a second init while that cluster is up (reference:
python/ray/tests/test_basic.py, test_actor_resources.py, test_output.py)."""
import os
import time

import cluster_anywhere_amd as ray


@ray.remote
def add(a, b):
    return a + b


def test_local_mode():
    ray.shutdown()
    ray.init(local_mode=True)
    try:
        assert ray.get(add.remote(2, 3)) == 5

        @ray.remote
        class A:
            def f(self):
                return 7

        assert ray.get(A.remote().f.remote()) == 7
    finally:
        ray.shutdown()


def test_fractional_gpu_packing():
    """num_gpus=0.5 actors pack two per device; whole-GPU work waits for a free one
    (reference: fractional GPU resources, accelerators/amd_gpu.py)."""
    import cluster_anywhere_amd as ray

    ray.init(num_cpus=8, num_gpus=2)
    try:
        @ray.remote(num_gpus=0.5, num_cpus=0)
        class Half:
            def ids(self):
                import os

                return tuple(int(x) for x in os.environ["CAAMD_GPU_IDS"].split(","))  # physical ids

        @ray.remote(num_gpus=1, num_cpus=0)
        def whole():
            import os

            return tuple(int(x) for x in os.environ["CAAMD_GPU_IDS"].split(","))

        hs = [Half.remote() for _ in range(2)]
        ids = ray.get([h.ids.remote() for h in hs])
        assert all(len(i) == 1 for i in ids)
        from collections import Counter

        c = Counter(i[0] for i in ids)
        assert max(c.values()) == 2                      # packed, not spread
        w = ray.get(whole.remote(), timeout=30)          # the other GPU is still whole
        assert len(w) == 1 and w[0] not in c
        ready, _ = ray.wait([Half.remote().ids.remote()], timeout=30)
        assert ready
    finally:
        ray.shutdown()


def test_worker_output_streams_to_driver(capsys):
    """print() inside tasks shows up on the driver (reference: log_to_driver)."""
    import time

    import cluster_anywhere_amd as ray

    ray.init(num_cpus=2)
    try:
        @ray.remote
        def chatty(i):
            print(f"hello-from-task-{i}", flush=True)
            return i

        assert ray.get([chatty.remote(i) for i in range(3)]) == [0, 1, 2]
        deadline = time.time() + 10
        seen = ""
        while time.time() < deadline:
            seen += capsys.readouterr().out
            if all(f"hello-from-task-{i}" in seen for i in range(3)):
                break
            time.sleep(0.1)
        assert all(f"hello-from-task-{i}" in seen for i in range(3)), seen
        assert "(pid=" in seen
    finally:
        ray.shutdown()


def test_gpu_ids_return_when_placement_group_removed():
    """Removing a PG whose GPU actor is alive hands the device id back (a later
    fractional actor must still be placeable)."""
    import cluster_anywhere_amd as ray
    from cluster_anywhere_amd.util import placement_group, remove_placement_group
    from cluster_anywhere_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy

    ray.init(num_cpus=4, num_gpus=1)
    try:
        @ray.remote(num_gpus=1, num_cpus=0)
        class G:
            def f(self):
                return 1

        pg = placement_group([{"CPU": 1, "GPU": 1}])
        ray.get(pg.ready())
        a = G.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg, 0)).remote()
        assert ray.get(a.f.remote()) == 1
        ray.kill(a)
        remove_placement_group(pg)

        @ray.remote(num_gpus=0.4, num_cpus=0)
        class H:
            def f(self):
                return 3

        assert ray.get(H.remote().f.remote(), timeout=30) == 3
    finally:
        ray.shutdown()
