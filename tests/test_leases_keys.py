"""Leases for every task class (reference: scheduling keys of
src/ray/core_worker/transport/direct_task_transport.cc, raylet local dispatch
src/ray/raylet/local_task_manager.h:58): GPU tasks lease GPU-pinned workers (the
ids stay with the lease and come back with it), placement-group tasks lease
against their bundle, runtime-env tasks lease workers of that env's pool.
CPU-only box: the GPUs are logical (ids 0..1)."""
import os
import time

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.core import context
from cluster_anywhere_amd.util.placement_group import placement_group, remove_placement_group
from cluster_anywhere_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4, num_gpus=2, object_store_memory=256 << 20)
    yield
    ray.shutdown()


def _leased():
    return context.worker.leases.n_leased_tasks


def _wait_resources(key, want, timeout=10.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if abs(ray.available_resources().get(key, 0.0) - want) < 1e-6:
            return True
        time.sleep(0.05)
    return False


@ray.remote(num_gpus=1, num_cpus=0)
def gpu_task(i):
    t0 = time.time()
    time.sleep(0.02)
    return i, os.environ.get("CAAMD_GPU_IDS"), ray.get_gpu_ids(), os.getpid(), t0, time.time()


def _max_overlap(spans):
    ev = sorted([(a, 1) for a, _ in spans] + [(b, -1) for _, b in spans])
    cur = best = 0
    for _, d in ev:
        cur += d
        best = max(best, cur)
    return best


def test_gpu_tasks_run_on_leases_with_pinned_gpus(cluster):
    before = _leased()
    out = ray.get([gpu_task.remote(i) for i in range(40)])
    assert [o[0] for o in out] == list(range(40))
    assert _leased() - before >= 30  # all but the first went through GPU leases
    assert all(o[1] in ("0", "1") and len(o[2]) == 1 for o in out)  # one GPU per task
    # a worker keeps one GPU for its whole life: pid -> single GPU id
    by_pid = {}
    for o in out:
        by_pid.setdefault(o[3], set()).add(o[1])
    assert all(len(v) == 1 for v in by_pid.values())
    assert _max_overlap([(o[4], o[5]) for o in out]) <= 2  # never more than the 2 GPUs
    assert _wait_resources("GPU", 2.0)  # the leases gave their GPUs back


@ray.remote(num_gpus=0.5, num_cpus=0)
def half_gpu(i):
    t0 = time.time()
    time.sleep(0.05)
    return os.environ.get("CAAMD_GPU_IDS"), t0, time.time()


def test_fractional_gpu_leases_pack(cluster):
    before = _leased()
    out = ray.get([half_gpu.remote(i) for i in range(24)])
    assert _leased() - before >= 16
    assert _max_overlap([(a, b) for _, a, b in out]) <= 4  # two per GPU at most
    assert {g for g, _, _ in out} <= {"0", "1"}
    assert _wait_resources("GPU", 2.0)


def test_placement_group_tasks_lease_their_bundle(cluster):
    pg = placement_group([{"CPU": 1}, {"CPU": 1}], strategy="PACK")
    assert pg.wait(10)

    @ray.remote(num_cpus=1)
    def in_pg(i):
        from cluster_anywhere_amd.util.placement_group import get_current_placement_group

        cur = get_current_placement_group()
        time.sleep(0.01)
        return i, cur.id if cur is not None else None, time.time()

    before = _leased()
    strat = PlacementGroupSchedulingStrategy(pg, placement_group_bundle_index=-1)
    out = ray.get([in_pg.options(scheduling_strategy=strat).remote(i) for i in range(30)])
    assert [o[0] for o in out] == list(range(30))
    assert all(o[1] == pg.id for o in out)
    assert _leased() - before >= 20
    # bundle-indexed tasks lease against their own bundle
    s0 = PlacementGroupSchedulingStrategy(pg, placement_group_bundle_index=0)
    assert ray.get([in_pg.options(scheduling_strategy=s0).remote(i) for i in range(10)])[9][0] == 9
    remove_placement_group(pg)
    assert _wait_resources("CPU", 4.0)


@ray.remote
def env_task(i):
    return i, os.environ.get("CAAMD_TEST_ENV"), os.getpid()


def test_runtime_env_tasks_lease_env_pools(cluster):
    before = _leased()
    a = env_task.options(runtime_env={"env_vars": {"CAAMD_TEST_ENV": "a"}})
    b = env_task.options(runtime_env={"env_vars": {"CAAMD_TEST_ENV": "b"}})
    ra = [a.remote(i) for i in range(30)]
    rb = [b.remote(i) for i in range(30)]
    oa, ob = ray.get(ra), ray.get(rb)
    assert all(o[1] == "a" for o in oa) and all(o[1] == "b" for o in ob)
    assert not ({o[2] for o in oa} & {o[2] for o in ob})  # separate worker pools
    assert _leased() - before >= 40
    # plain tasks after env tasks do not see the env
    assert ray.get(env_task.remote(0))[1] is None
