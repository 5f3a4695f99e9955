"""Synchronous HyperBand, HyperBandForBOHB + TuneBOHB, PB2 and
ResourceChangingScheduler (reference: python/ray/tune/tests/test_trial_scheduler.py,
test_trial_scheduler_pbt.py, test_trial_scheduler_resource_changing.py)."""
import math
import os

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import tune
from cluster_anywhere_amd.train import Checkpoint


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8, include_dashboard=False)
    yield
    ray.shutdown()


def ckpt_trial(config):
    """Resumable trainable: acc grows by q per iteration; checkpoints its step."""
    import json
    import tempfile

    start = 0
    ck = tune.get_checkpoint()
    if ck is not None:
        with open(os.path.join(ck.path, "s.json")) as f:
            start = json.load(f)["i"]
    for i in range(start, 60):
        d = tempfile.mkdtemp()
        with open(os.path.join(d, "s.json"), "w") as f:
            json.dump({"i": i + 1}, f)
        tune.report({"acc": config["q"] * (i + 1), "res": tune.get_trial_resources().get("CPU", 0)},
                    checkpoint=Checkpoint.from_directory(d))


def test_sync_hyperband_brackets(cluster, tmp_path):
    # unit check of the bracket arithmetic: max_t 27, eta 3 -> s_max 3, brackets of 27/12/6/4
    hb = tune.HyperBandScheduler(max_t=27, reduction_factor=3)
    assert hb.s_max == 3
    sizes = []
    for s in (3, 2, 1, 0):
        sizes.append(int(math.ceil((hb.s_max + 1) / (s + 1) * 3 ** s)))
    assert sizes == [27, 12, 6, 4]
    sched = tune.HyperBandScheduler(max_t=9, reduction_factor=3)
    qs = [0.1, 0.2, 0.3, 0.5, 0.7, 1.0, 1.5, 2.0, 3.0]
    grid = tune.Tuner(ckpt_trial, param_space={"q": tune.grid_search(qs)},
                      tune_config=tune.TuneConfig(metric="acc", mode="max", scheduler=sched),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="hb")).fit()
    iters = {r.config["q"]: r.metrics["training_iteration"] for r in grid}
    assert iters[3.0] == 9          # the best trial reaches max_t through every rung
    assert min(iters.values()) < 9  # successive halving stopped the weak ones
    # promoted trials resumed from checkpoints: no trial ran a milestone twice
    assert all(v <= 9 for v in iters.values())


def test_hb_bohb_with_tunebohb(cluster, tmp_path):
    search = tune.TuneBOHB(seed=0, random_fraction=0.0, min_points_in_model=2)
    sched = tune.HyperBandForBOHB(max_t=9, reduction_factor=3)
    grid = tune.Tuner(ckpt_trial, param_space={"q": tune.uniform(0.0, 3.0)},
                      tune_config=tune.TuneConfig(metric="acc", mode="max", scheduler=sched,
                                                  search_alg=search, num_samples=14),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="bohb")).fit()
    assert len(grid) == 14
    assert sum(len(v) for v in search.obs.values()) >= 9  # milestones fed the density models
    best = grid.get_best_result()
    assert best.config["q"] > 1.5


def test_pb2_explores_inside_bounds(cluster, tmp_path):
    # bottom half, checked every 2 iterations: a trial is ranked against whatever the
    # others last reported, so under a loaded CI box (trials running one after another)
    # a bottom-quartile check every 3 iterations could miss every time
    sched = tune.PB2(perturbation_interval=2, hyperparam_bounds={"q": [0.1, 3.0]}, seed=1,
                     quantile_fraction=0.5)
    grid = tune.Tuner(ckpt_trial, param_space={"q": tune.uniform(0.1, 1.0)},
                      tune_config=tune.TuneConfig(metric="acc", mode="max", scheduler=sched, num_samples=4),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="pb2",
                                                stop={"training_iteration": 15})).fit()
    assert sched.num_perturbations >= 1
    assert all(0.1 <= r.config["q"] <= 3.0 for r in grid)
    assert len(sched.data) > 0


def test_resource_changing_scheduler(cluster, tmp_path):
    def alloc(controller, trial, result, scheduler):
        return {"CPU": 2} if result["training_iteration"] >= 3 else None

    sched = tune.ResourceChangingScheduler(resources_allocation_function=alloc)
    grid = tune.Tuner(ckpt_trial, param_space={"q": 1.0},
                      tune_config=tune.TuneConfig(metric="acc", mode="max", scheduler=sched),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="rcs",
                                                stop={"training_iteration": 8})).fit()
    r = grid[0]
    assert r.metrics["training_iteration"] == 8
    assert r.metrics["res"] == 2  # the relaunched trial sees its new resources
