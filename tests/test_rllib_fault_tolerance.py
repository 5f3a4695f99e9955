"""RLlib keeps training through dead EnvRunner and Learner actors (reference:
rllib/env/env_runner_group.py:138,181-187 over rllib/utils/actor_manager.py:198 —
``restart_failed_env_runners`` defaults to True; rllib/algorithms/tests/
test_worker_failures.py). Processes are SIGKILLed, not ``ray.kill``ed."""
import math
import os
import signal
import threading
import time

import pytest
import torch

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import rllib
from cluster_anywhere_amd.rllib.callbacks import RLlibCallback


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8)
    yield
    ray.shutdown()


def _pid(actor):
    return ray.get(actor.__ray_call__.remote(lambda self: os.getpid()))


class _Recorder(RLlibCallback):
    recreated = []

    def on_env_runners_recreated(self, *, algorithm, env_runner_group, env_runner_indices, **kwargs):
        type(self).recreated.append(list(env_runner_indices))


def _ppo(num_runners=2, num_learners=0):
    return (rllib.PPOConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=num_runners, num_envs_per_env_runner=4)
            .learners(num_learners=num_learners)
            .training(lr=3e-4, train_batch_size=800, minibatch_size=200, num_epochs=2,
                      model={"fcnet_hiddens": [32, 32]})
            .callbacks(_Recorder).debugging(seed=0))


def test_env_runner_sigkilled_mid_train_is_restored(cluster):
    _Recorder.recreated = []
    algo = _ppo().build()
    try:
        r = algo.train()
        g = algo.env_runner_group
        victim = _pid(g.remote[1])
        killer = threading.Timer(0.05, lambda: os.kill(victim, signal.SIGKILL))
        killer.start()
        steps = r["num_env_steps_sampled_lifetime"]
        for _ in range(3):
            r = algo.train()  # the kill lands inside one of these
            assert r["num_env_steps_sampled_lifetime"] > steps
            steps = r["num_env_steps_sampled_lifetime"]
        killer.join()
        assert g.num_restarts >= 1 and _Recorder.recreated and 1 in _Recorder.recreated[0]
        assert all(g.healthy)
        assert _pid(g.remote[1]) != victim
        # the replacement samples with the current weights
        w = algo.learner_group.get_module_state()
        rw = ray.get(g.remote[1].get_weights.remote())
        for k in w:
            assert torch.allclose(w[k].cpu(), rw[k].cpu())
    finally:
        algo.stop()


def test_ignore_env_runner_failures_without_restart(cluster):
    algo = _ppo(num_runners=2).fault_tolerance(restart_failed_env_runners=False,
                                              ignore_env_runner_failures=True).build()
    try:
        algo.train()
        g = algo.env_runner_group
        os.kill(_pid(g.remote[0]), signal.SIGKILL)
        r = algo.train()
        assert g.healthy == [False, True] and g.num_restarts == 0
        assert r["num_env_steps_sampled_lifetime"] > 0
    finally:
        algo.stop()


def test_env_runner_failure_raises_when_not_tolerated(cluster):
    from cluster_anywhere_amd.exceptions import RayActorError

    algo = _ppo(num_runners=2).fault_tolerance(restart_failed_env_runners=False).build()
    try:
        algo.train()
        os.kill(_pid(algo.env_runner_group.remote[0]), signal.SIGKILL)
        time.sleep(0.5)
        with pytest.raises((RayActorError, RuntimeError)):
            algo.train()
    finally:
        algo.stop()


def test_impala_async_sampling_survives_runner_death(cluster):
    cfg = (rllib.get_algorithm_class("IMPALA").get_default_config().environment("CartPole-v1")
           .env_runners(num_env_runners=2, num_envs_per_env_runner=4, rollout_fragment_length=50)
           .training(lr=1e-3, model={"fcnet_hiddens": [32, 32]}).debugging(seed=0))
    algo = cfg.build()
    try:
        algo.train()
        g = algo.env_runner_group
        os.kill(_pid(g.remote[0]), signal.SIGKILL)
        for _ in range(6):
            r = algo.train()
        assert g.num_restarts >= 1 and all(g.healthy)
        assert r["num_env_steps_sampled_lifetime"] > 0
    finally:
        algo.stop()


@pytest.mark.parametrize("victim", [1, 0])
def test_learner_sigkilled_group_restarts_from_last_state(cluster, victim):
    """victim 0: the rank whose get_state snapshot the group keeps dies -- the
    snapshot is owned by the driver and outlives it."""
    algo = _ppo(num_runners=1, num_learners=2).build()
    try:
        algo.train()
        lg = algo.learner_group
        before = lg.get_state()
        os.kill(_pid(lg.actors[victim]), signal.SIGKILL)
        time.sleep(0.3)
        r = algo.train()
        assert lg.num_restarts == 1
        assert math.isfinite(r["learners"]["default_policy"]["total_loss"])
        states = ray.get([a.call.remote("get_module_state") for a in lg.actors])
        for k in states[0]:
            assert torch.allclose(states[0][k], states[1][k], atol=1e-6)
        assert lg.get_state()["num_updates"] > before["num_updates"]
    finally:
        algo.stop()
