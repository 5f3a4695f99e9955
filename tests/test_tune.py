"""Tune: search spaces, searchers, schedulers, stoppers, function / class /
Trainer trainables, PBT exploitation, failure retries and Tuner.restore
(reference: python/ray/tune/tests/test_tuner.py, test_sample.py,
test_trial_scheduler.py, test_trial_scheduler_pbt.py, test_tuner_restore.py)."""
import json
import os
import random
import tempfile

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import train, tune
from cluster_anywhere_amd.tune.search.sample import generate_variants


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


# ------------------------------------------------------------------ pure units
def test_search_space_sampling():
    space = {"lr": tune.loguniform(1e-4, 1e-1), "bs": tune.choice([16, 32]), "n": tune.randint(1, 5),
             "q": tune.quniform(0, 1, 0.25), "g": tune.grid_search(["a", "b", "c"]),
             "nested": {"x": tune.uniform(-1, 1), "y": tune.sample_from(lambda spec: spec.config["n"] * 2)}}
    vs = list(generate_variants(space, num_samples=4, seed=0))
    assert len(vs) == 12
    assert sorted({v["g"] for v in vs}) == ["a", "b", "c"]
    for v in vs:
        assert 1e-4 <= v["lr"] <= 1e-1 and v["bs"] in (16, 32) and 1 <= v["n"] < 5
        assert v["q"] in (0.0, 0.25, 0.5, 0.75, 1.0)
        assert -1 <= v["nested"]["x"] <= 1 and v["nested"]["y"] == v["n"] * 2


def test_grid_product():
    vs = list(generate_variants({"a": tune.grid_search([1, 2]), "b": tune.grid_search([3, 4, 5])}))
    assert sorted((v["a"], v["b"]) for v in vs) == [(a, b) for a in (1, 2) for b in (3, 4, 5)]


class _T:
    def __init__(self, tid):
        self.trial_id = tid
        self.latest_checkpoint = None
        self.config = {}


def test_asha_stops_bad_trials():
    s = tune.ASHAScheduler(metric="acc", mode="max", max_t=100, grace_period=1, reduction_factor=2)
    good, decisions = [], []
    for i in range(8):
        decisions.append(s.on_trial_result(_T(str(i)), {"training_iteration": 1, "acc": i}))
    # later (better) trials continue; once enough results exist, worse ones are cut
    assert decisions[-1] == "CONTINUE"
    assert "STOP" not in decisions[:1]
    assert s.on_trial_result(_T("bad"), {"training_iteration": 1, "acc": -5}) == "STOP"
    assert s.on_trial_result(_T("x"), {"training_iteration": 100, "acc": 99}) == "STOP"


def test_median_stopping():
    s = tune.MedianStoppingRule(metric="m", mode="max", time_attr="training_iteration", grace_period=1,
                                min_samples_required=2)
    for i in range(3):
        for t in range(1, 4):
            s.on_trial_result(_T(str(i)), {"training_iteration": t, "m": 10 + i})
    assert s.on_trial_result(_T("low"), {"training_iteration": 2, "m": 0}) == "STOP"


def test_stoppers():
    st = tune.stopper.make_stopper({"training_iteration": 3}) if hasattr(tune, "stopper") else None
    from cluster_anywhere_amd.tune.stopper import make_stopper

    st = make_stopper({"training_iteration": 3})
    assert not st("t", {"training_iteration": 2}) and st("t", {"training_iteration": 3})
    p = tune.TrialPlateauStopper("loss", std=0.01, num_results=3, grace_period=3)
    assert not any(p("t", {"loss": v}) for v in (5.0, 3.0))
    assert not p("t", {"loss": 1.0})
    assert p("u", {"loss": 1.0}) is False
    for _ in range(3):
        r = p("u", {"loss": 1.0})
    assert r
    c = tune.CombinedStopper(tune.MaximumIterationStopper(2), tune.FunctionStopper(lambda t, r: r.get("x") == 1))
    assert c("t", {"x": 1}) and c("t", {"training_iteration": 2}) and not c("t", {"training_iteration": 1})


def test_repeater_and_limiter():
    base = tune.BasicVariantGenerator()
    rep = tune.Repeater(base, repeat=3)
    rep.set_search_properties("m", "max", {"a": tune.grid_search([1, 2])})
    got = [rep.suggest(str(i)) for i in range(7)]
    assert [g["a"] for g in got[:6]] == [1, 1, 1, 2, 2, 2]
    assert [g["__trial_index__"] for g in got[:3]] == [0, 1, 2]
    assert got[6] == tune.Searcher.FINISHED
    lim = tune.ConcurrencyLimiter(tune.BasicVariantGenerator(), max_concurrent=1)
    lim.set_search_properties("m", "max", {"a": tune.grid_search([1, 2])})
    assert lim.suggest("1")["a"] == 1 and lim.suggest("2") is None
    lim.on_trial_complete("1", {})
    assert lim.suggest("2")["a"] == 2


# ------------------------------------------------------------- end to end
def quadratic(config):
    for i in range(5):
        tune.report({"score": -(config["x"] - 3) ** 2 + i * 0.01, "step": i})


def test_tuner_function_grid(cluster, tmp_path):
    tuner = tune.Tuner(quadratic, param_space={"x": tune.grid_search([0, 1, 2, 3, 4, 5])},
                       tune_config=tune.TuneConfig(metric="score", mode="max"),
                       run_config=tune.RunConfig(name="quad", storage_path=str(tmp_path)))
    grid = tuner.fit()
    assert len(grid) == 6 and grid.num_errors == 0
    best = grid.get_best_result()
    assert best.config["x"] == 3 and best.metrics["training_iteration"] == 5
    df = grid.get_dataframe()
    assert len(df) == 6 and "config/x" in df.columns
    assert os.path.exists(os.path.join(best.path, "result.json"))
    assert os.path.exists(os.path.join(best.path, "progress.csv"))
    assert json.load(open(os.path.join(best.path, "params.json")))["x"] == 3
    assert len(best.metrics_dataframe) == 5


def long_trial(config):
    for i in range(50):
        tune.report({"acc": config["q"] * (i + 1), "training_iteration": i + 1})


def test_tuner_asha_and_stop(cluster, tmp_path):
    sched = tune.ASHAScheduler(max_t=20, grace_period=2, reduction_factor=2)
    # best-first grid: trials report in lock-step (report() waits for the controller),
    # so later, weaker arrivals at each rung meet a recorded cutoff and are stopped
    tuner = tune.Tuner(long_trial, param_space={"q": tune.grid_search([3.0, 2.0, 1.0, 0.5, 0.2, 0.1])},
                       tune_config=tune.TuneConfig(metric="acc", mode="max", scheduler=sched),
                       run_config=tune.RunConfig(storage_path=str(tmp_path), name="asha"))
    grid = tuner.fit()
    iters = {r.config["q"]: r.metrics["training_iteration"] for r in grid}
    assert max(iters.values()) <= 20
    assert iters[3.0] == 20  # best trial runs to max_t
    assert min(iters.values()) < 20  # somebody got cut early
    # dict stop criterion
    grid2 = tune.Tuner(long_trial, param_space={"q": 1.0},
                       run_config=tune.RunConfig(storage_path=str(tmp_path), name="stop",
                                                 stop={"training_iteration": 7})).fit()
    assert grid2[0].metrics["training_iteration"] == 7


class Counter(tune.Trainable):
    def setup(self, config):
        self.v = 0
        self.inc = config["inc"]

    def step(self):
        self.v += self.inc
        return {"v": self.v, "done": self.v >= 10 * self.inc}

    def save_checkpoint(self, d):
        return {"v": self.v}

    def load_checkpoint(self, st):
        self.v = st["v"]


def test_class_trainable_checkpoints(cluster, tmp_path):
    grid = tune.Tuner(Counter, param_space={"inc": tune.grid_search([1, 2])},
                      tune_config=tune.TuneConfig(metric="v", mode="max"),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="cls",
                                                checkpoint_config=tune.CheckpointConfig(
                                                    checkpoint_frequency=3, checkpoint_at_end=True))).fit()
    best = grid.get_best_result()
    assert best.metrics["v"] == 20 and best.metrics["training_iteration"] == 10
    assert best.checkpoint is not None
    meta = json.load(open(os.path.join(best.checkpoint.path, "_trainable_meta.json")))
    assert meta["iteration"] == 10


def ckpt_trial(config):
    start = 0
    ck = tune.get_checkpoint()
    if ck is not None:
        with ck.as_directory() as d:
            start = json.load(open(os.path.join(d, "s.json")))["i"] + 1
    for i in range(start, 6):
        if i == 3 and not os.path.exists(config["marker"]):
            open(config["marker"], "w").close()
            raise RuntimeError("boom")
        with tempfile.TemporaryDirectory() as d:
            json.dump({"i": i}, open(os.path.join(d, "s.json"), "w"))
            tune.report({"i": i, "resumed_from": start}, checkpoint=train.Checkpoint.from_directory(d))


def test_trial_failure_retry_from_checkpoint(cluster, tmp_path):
    marker = str(tmp_path / "marker")
    grid = tune.Tuner(ckpt_trial, param_space={"marker": marker},
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="ft",
                                                failure_config=tune.FailureConfig(max_failures=1))).fit()
    r = grid[0]
    assert r.error is None
    assert r.metrics["i"] == 5 and r.metrics["resumed_from"] == 3
    # without retries the error surfaces in the grid
    os.remove(marker)
    grid = tune.Tuner(ckpt_trial, param_space={"marker": marker},
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="ft2")).fit()
    assert grid.num_errors == 1 and "boom" in str(grid.errors[0])


def pbt_trial(config):
    step = 0
    score = 0.0
    ck = tune.get_checkpoint()
    if ck is not None:
        with ck.as_directory() as d:
            st = json.load(open(os.path.join(d, "s.json")))
            step, score = st["step"], st["score"]
    import time

    while step < 12:
        time.sleep(0.05)
        step += 1
        score += config["lr"]
        with tempfile.TemporaryDirectory() as d:
            json.dump({"step": step, "score": score}, open(os.path.join(d, "s.json"), "w"))
            tune.report({"score": score, "lr": config["lr"], "training_iteration": step},
                        checkpoint=train.Checkpoint.from_directory(d))


def test_pbt_exploits(cluster, tmp_path):
    pbt = tune.PopulationBasedTraining(perturbation_interval=3, hyperparam_mutations={"lr": [0.01, 0.1, 1.0]},
                                       quantile_fraction=0.5, resample_probability=0.0, seed=0)
    grid = tune.Tuner(pbt_trial, param_space={"lr": tune.grid_search([0.01, 1.0])},
                      tune_config=tune.TuneConfig(metric="score", mode="max", scheduler=pbt),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="pbt")).fit()
    assert pbt.num_perturbations >= 1
    scores = sorted(r.metrics["score"] for r in grid)
    # the weak trial inherited the strong one's progress: both end well above 12 * 0.01
    assert scores[0] > 1.0
    # log_config: the exploited trial's schedule is on disk and replays (reference:
    # test_trial_scheduler_pbt.py PopulationBasedTrainingReplay)
    exp = os.path.join(str(tmp_path), "pbt")
    policies = [f for f in os.listdir(exp) if f.startswith("pbt_policy_")]
    assert policies
    rows = [json.loads(ln) for ln in open(os.path.join(exp, policies[0]))]
    assert len(rows[-1]) == 6 and rows[-1][1] == policies[0][len("pbt_policy_"):-4]
    replay = tune.schedulers.PopulationBasedTrainingReplay(os.path.join(exp, policies[0]))
    assert replay.config is not None and replay.schedule
    res = tune.Tuner(pbt_trial, tune_config=tune.TuneConfig(metric="score", mode="max", scheduler=replay),
                     run_config=tune.RunConfig(storage_path=str(tmp_path), name="replay")).fit()
    assert replay.num_perturbations == len(rows) and res[0].metrics["lr"] == rows[-1][5]["lr"]
    with pytest.raises(ValueError):
        tune.schedulers.PopulationBasedTrainingReplay(str(tmp_path / "missing.txt"))


def slow_trial(config):
    import time

    for i in range(config["n"]):
        time.sleep(0.05)
        tune.report({"i": i})


class _Interrupt(tune.Callback):
    def __init__(self, marker):
        self.marker = marker

    def on_trial_result(self, iteration, trials, trial, result, **info):
        if not os.path.exists(self.marker):
            open(self.marker, "w").close()
            raise KeyboardInterrupt


def test_tuner_restore(cluster, tmp_path):
    exp = str(tmp_path / "res")
    tuner = tune.Tuner(slow_trial, param_space={"n": tune.grid_search([3, 4])},
                       tune_config=tune.TuneConfig(max_concurrent_trials=1),
                       run_config=tune.RunConfig(storage_path=str(tmp_path), name="res",
                                                 callbacks=[_Interrupt(str(tmp_path / "m"))]))
    with pytest.raises(KeyboardInterrupt):
        tuner.fit()
    assert tune.Tuner.can_restore(exp)
    st = json.load(open(os.path.join(exp, "experiment_state.json")))
    assert any(t["status"] == "PAUSED" for t in st["trials"])
    grid = tune.Tuner.restore(exp, slow_trial).fit()
    done = {r.config["n"]: r.metrics.get("i") for r in grid}
    assert done == {3: 2, 4: 3}


def test_tune_run_and_with_parameters(cluster, tmp_path):
    data = list(range(100))

    def fn(config, data=None):
        tune.report({"s": sum(data) * config["k"]})

    ana = tune.run(tune.with_parameters(fn, data=data), config={"k": tune.grid_search([1, 2])},
                   metric="s", mode="max", storage_path=str(tmp_path), name="run",
                   resources_per_trial={"cpu": 1})
    assert ana.best_config["k"] == 2 and ana.best_result["s"] == 9900
    assert len(ana.trials) == 2


def test_tuner_over_torch_trainer(cluster, tmp_path):
    from cluster_anywhere_amd.train import ScalingConfig
    from cluster_anywhere_amd.train.torch import TorchTrainer

    def loop(config):
        import torch.distributed as dist

        for i in range(2):
            train.report({"v": config["a"] * 10 + i, "world": dist.get_world_size()})

    trainer = TorchTrainer(loop, train_loop_config={"a": 0}, scaling_config=ScalingConfig(num_workers=2))
    grid = tune.Tuner(trainer, param_space={"train_loop_config": {"a": tune.grid_search([1, 2])}},
                      tune_config=tune.TuneConfig(metric="v", mode="max"),
                      run_config=tune.RunConfig(storage_path=str(tmp_path), name="tt")).fit()
    assert grid.num_errors == 0
    best = grid.get_best_result()
    assert best.metrics["v"] == 21 and best.metrics["world"] == 2
