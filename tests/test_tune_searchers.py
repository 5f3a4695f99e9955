"""Native model-based searchers (OptunaSearch / HyperOptSearch = TPE, BayesOptSearch
= GP): each must find a known optimum faster than random search on the same budget,
and OptunaSearch must run inside a Tuner. Parity with the optuna / hyperopt /
bayes_opt libraries themselves is unpinned (not importable here)."""
import math

import numpy as np
import pytest

from cluster_anywhere_amd import tune


def _objective(cfg):
    # optimum at x = 0.3, log10(lr) = -3, act = "gelu"
    v = -(cfg["x"] - 0.3) ** 2 - 0.1 * (math.log10(cfg["lr"]) + 3) ** 2
    return v + (0.0 if cfg.get("act", "gelu") == "gelu" else -1.0)


SPACE = {"x": tune.uniform(-2.0, 2.0), "lr": tune.loguniform(1e-6, 1e-1), "act": tune.choice(["relu", "gelu", "tanh"]),
         "fixed": 7, "nested": {"k": tune.randint(1, 5)}}


def _drive(searcher, n, mode="max", space=SPACE):
    searcher.set_search_properties("score", mode, space, num_samples=n)
    best = -1e9
    for i in range(n):
        cfg = searcher.suggest(str(i))
        assert cfg["fixed"] == 7 and 1 <= cfg["nested"]["k"] < 5
        s = _objective(cfg)
        best = max(best, s)
        searcher.on_trial_complete(str(i), {"score": s if mode == "max" else -s, "config": cfg})
    assert searcher.suggest("done") == tune.Searcher.FINISHED
    return best


def _random_best(n, seed):
    rng = np.random.default_rng(seed)
    best = -1e9
    for _ in range(n):
        cfg = {"x": rng.uniform(-2, 2), "lr": 10 ** rng.uniform(-6, -1), "act": rng.choice(["relu", "gelu", "tanh"])}
        best = max(best, _objective(cfg))
    return best


@pytest.mark.parametrize("make", [lambda s: tune.OptunaSearch(seed=s), lambda s: tune.HyperOptSearch(random_state_seed=s, n_initial_points=10)])
def test_tpe_beats_random(make):
    ours = [_drive(make(s), 60) for s in range(3)]
    rand = [_random_best(60, s) for s in range(3)]
    assert np.median(ours) > np.median(rand)
    assert max(ours) > -0.02


def test_tpe_min_mode():
    s = tune.OptunaSearch(seed=0)
    assert _drive(s, 50, mode="min") > -0.1


def test_bayesopt_beats_random():
    space = {"x": tune.uniform(-2.0, 2.0), "lr": tune.loguniform(1e-6, 1e-1), "fixed": 7,
             "nested": {"k": tune.randint(1, 5)}}
    ours = [_drive(tune.BayesOptSearch(random_state=s, random_search_steps=5), 25, space=space) for s in range(2)]
    rand = [_random_best(25, s) for s in range(2)]
    assert min(ours) > max(rand) - 0.05
    assert max(ours) > -0.01
    with pytest.raises(ValueError):
        tune.BayesOptSearch(space={"a": tune.choice([1, 2])})


def test_points_to_evaluate_and_rewards():
    s = tune.OptunaSearch(space={"x": tune.uniform(0, 1)}, metric="m", mode="max",
                          points_to_evaluate=[{"x": 0.25}, {"x": 0.75}], evaluated_rewards=[1.0, 0.0])
    assert len(s.y) == 2 and s.X[0] == [0.25]
    s2 = tune.HyperOptSearch(space={"x": tune.uniform(0, 1)}, metric="m", mode="max", points_to_evaluate=[{"x": 0.5}])
    assert s2.suggest("a")["x"] == 0.5


def test_optuna_in_tuner(tmp_path):
    import cluster_anywhere_amd as ray

    ray.init(num_cpus=2, ignore_reinit_error=True)
    try:
        def trainable(config):
            tune.report({"score": -(config["x"] - 0.5) ** 2})

        tuner = tune.Tuner(trainable, param_space={"x": tune.uniform(0, 1)},
                           tune_config=tune.TuneConfig(metric="score", mode="max", num_samples=12,
                                                       search_alg=tune.OptunaSearch(seed=1)),
                           run_config=tune.RunConfig(storage_path=str(tmp_path), name="optuna"))
        res = tuner.fit()
        assert len(res) == 12
        assert res.get_best_result().metrics["score"] > -0.05
    finally:
        ray.shutdown()
