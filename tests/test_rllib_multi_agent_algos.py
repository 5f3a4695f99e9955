"""Multi-agent beyond PPO: IMPALA / APPO / DQN / SAC over per-module learners, and
recurrent (LSTM) multi-agent PPO (reference: rllib/core/rl_module/multi_rl_module.py:49
under impala.py:588, appo.py:358, dqn.py:610; test model:
rllib/examples/multi_agent/multi_agent_cartpole.py, two-agent learning checks)."""
import math

import numpy as np
import pytest

from cluster_anywhere_amd import rllib
from cluster_anywhere_amd.rllib.env import Box
from cluster_anywhere_amd.rllib.env.multi_agent_env import CooperativeMatchEnv, MultiAgentEnv, make_multi_agent
from cluster_anywhere_amd.rllib.env.multi_agent_env_runner import MultiAgentEnvRunner


def _map(aid, ep, **k):
    return "p" + str(aid)


class TwoAgentTarget(MultiAgentEnv):
    """Continuous contextual task for two agents: each sees a target in [-1, 1]
    and is paid ``-(action - target)^2``; agent "b" must play the NEGATED target.
    10 steps: a uniform-random policy returns about -6.7 per agent, the optimum 0."""

    def __init__(self, config=None):
        self.possible_agents = ["a", "b"]
        self.agents = list(self.possible_agents)
        self.observation_spaces = {a: Box(-1.0, 1.0, (1,)) for a in self.agents}
        self.action_spaces = {a: Box(-1.0, 1.0, (1,)) for a in self.agents}
        self.rng = np.random.default_rng(0)

    def _obs(self):
        self.tg = self.rng.uniform(-1, 1, size=2).astype(np.float32)
        return {"a": self.tg[:1].copy(), "b": self.tg[1:].copy()}

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.t = 0
        return self._obs(), {}

    def step(self, action_dict):
        ra = -float((np.asarray(action_dict["a"]).reshape(-1)[0] - self.tg[0]) ** 2)
        rb = -float((np.asarray(action_dict["b"]).reshape(-1)[0] + self.tg[1]) ** 2)
        self.t += 1
        done = self.t >= 10
        return self._obs(), {"a": ra, "b": rb}, {"a": done, "b": done, "__all__": done}, {"__all__": False}, {}


def _coop(cfg):
    return (cfg.environment(CooperativeMatchEnv).multi_agent(policies=["pa", "pb"], policy_mapping_fn=_map)
            .reporting(metrics_num_episodes_for_smoothing=20).debugging(seed=0))


def _learn(algo, iters, target, key="episode_return_mean"):
    best = -math.inf
    for _ in range(iters):
        r = algo.train()
        best = max(best, r["env_runners"][key])
        if best > target:
            break
    return best, r


@pytest.mark.parametrize("name", ["IMPALA", "APPO"])
def test_impala_appo_multi_agent_learn(name):
    cfg = _coop(rllib.get_algorithm_class(name).get_default_config()
                .env_runners(num_envs_per_env_runner=8, rollout_fragment_length=20)
                .training(lr=3e-3, model={"fcnet_hiddens": [32]}, entropy_coeff=0.0))
    algo = cfg.build()
    best, r = _learn(algo, 300, 35)
    # random play returns 20 (team reward), optimal play 40
    assert best > 35, best
    assert set(r["learners"]) == {"pa", "pb"}
    assert all(math.isfinite(s["total_loss"]) for s in r["learners"].values())
    st = algo.learner_group.get_module_state()
    k = next(iter(st["pa"]))
    assert not np.allclose(st["pa"][k].numpy(), st["pb"][k].numpy())
    algo.stop()


def test_dqn_multi_agent_learns_with_per_module_replay():
    cfg = _coop(rllib.DQNConfig().env_runners(num_envs_per_env_runner=4, rollout_fragment_length=4)
                .training(lr=1e-3, train_batch_size=64, num_steps_sampled_before_learning_starts=200,
                          target_network_update_freq=200, epsilon=[(0, 1.0), (2000, 0.02)], training_intensity=32,
                          gamma=0.5, model={"fcnet_hiddens": [32]}))
    algo = cfg.build()
    assert set(algo.buffers) == {"pa", "pb"} and algo.buffer is None
    best, r = _learn(algo, 600, 35)
    assert best > 35, best
    assert set(r["learners"]) == {"pa", "pb"} and "epsilon" in r["learners"]["pa"]
    # every sampled agent step of a module went into that module's buffer
    assert len(algo.buffers["pa"]) == len(algo.buffers["pb"]) == min(algo.env_steps_sampled, 50_000)
    algo.stop()


def test_sac_multi_agent_learns_continuous():
    cfg = (rllib.SACConfig().environment(TwoAgentTarget)
           .env_runners(num_envs_per_env_runner=4, rollout_fragment_length=5)
           .multi_agent(policies=["pa", "pb"], policy_mapping_fn=_map)
           .training(num_steps_sampled_before_learning_starts=200, train_batch_size=128, gamma=0.5,
                     training_intensity=16, actor_lr=3e-3, critic_lr=3e-3, alpha_lr=3e-3,
                     model={"policy_hiddens": [32], "q_hiddens": [32]})
           .reporting(metrics_num_episodes_for_smoothing=20).debugging(seed=0))
    algo = cfg.build()
    best = {"pa": -math.inf, "pb": -math.inf}
    for _ in range(150):
        r = algo.train()
        for m, v in r["env_runners"].get("module_episode_returns_mean", {}).items():
            best[m] = max(best[m], v)
        if min(best.values()) > -2.5:
            break
    assert min(best.values()) > -2.5, best  # uniform-random play: about -6.7 per agent (returns include exploration)
    assert set(r["learners"]) == {"pa", "pb"} and all(math.isfinite(s["qf_loss"]) for s in r["learners"].values())
    # the two modules learned opposite mappings
    a = float(np.asarray(algo.compute_single_action(np.array([0.5], np.float32), policy_id="pa")).reshape(-1)[0])
    b = float(np.asarray(algo.compute_single_action(np.array([0.5], np.float32), policy_id="pb")).reshape(-1)[0])
    assert a > 0.2 and b < -0.2, (a, b)
    algo.stop()


def test_off_policy_runner_transitions():
    """need_next_obs mode: next_obs continues the agent's own observation stream,
    a fragment cut keeps bootstrapping (terminated False), episode ends terminate."""
    cfg = (rllib.DQNConfig().environment(CooperativeMatchEnv, env_config={"episode_len": 6})
           .env_runners(num_envs_per_env_runner=1, rollout_fragment_length=4)
           .multi_agent(policies=["pa", "pb"], policy_mapping_fn=_map))
    r = MultiAgentEnvRunner(cfg.runner_config(), 0)
    f1 = r.sample()["policy_batches"]["pa"]
    assert f1["obs"].shape == (4, 1, 4) and f1["next_obs"].shape == (4, 1, 4)
    assert np.array_equal(f1["next_obs"][:3, 0], f1["obs"][1:, 0])
    assert not f1["terminateds"].any()  # cut at step 4 of a 6-step episode: not terminal
    assert (f1["rewards"] <= 2.0).all()  # no value folded into the rewards
    f2 = r.sample()["policy_batches"]["pa"]
    # the previous fragment's bootstrap obs is the first obs of the next fragment
    assert np.array_equal(f1["next_obs"][3, 0], f2["obs"][0, 0])
    # steps 5-6 end the episode (terminal), a new episode starts in the same fragment
    assert f2["mask"].sum() == 4 and f2["terminateds"].sum() == 1


def test_recurrent_ppo_multi_agent_learns_memory_task():
    env_cls = make_multi_agent("RepeatAfterMe-v0")
    cfg = (rllib.PPOConfig().environment(env_cls, env_config={"num_agents": 2})
           .env_runners(num_envs_per_env_runner=8, rollout_fragment_length=40)
           .multi_agent(policies=["p0", "p1"], policy_mapping_fn=_map)
           .training(lr=3e-3, train_batch_size=640, minibatch_size=160, num_epochs=6, gamma=0.5, lambda_=0.9,
                     vf_loss_coeff=0.5, model={"fcnet_hiddens": [64], "use_lstm": True, "lstm_cell_size": 64,
                                               "max_seq_len": 20})
           .reporting(metrics_num_episodes_for_smoothing=16).debugging(seed=0))
    algo = cfg.build()
    lrn = algo.learner_group.local.learners["p0"]
    frag = algo.env_runner_group.sample()[0]["policy_batches"]["p0"]
    assert frag["state_in_h"].shape[0] % 20 == 0 and "mask" in frag
    b = lrn.postprocess(frag)
    assert b["obs"].shape[1] == 20 and b["loss_mask"].shape == b["resets"].shape
    best = {"p0": 0.0, "p1": 0.0}
    for _ in range(25):
        r = algo.train()
        for m, v in r["env_runners"]["module_episode_returns_mean"].items():
            best[m] = max(best[m], v)
        if min(best.values()) > 16:
            break
    assert min(best.values()) > 16, best  # chance is ~9.5 per agent, the optimum 19
    algo.stop()


def test_multi_agent_refusals():
    from cluster_anywhere_amd.rllib.algorithms.cql import CQLConfig

    with pytest.raises(NotImplementedError, match="multi-agent"):
        CQLConfig().environment(CooperativeMatchEnv).multi_agent(policies=["pa"], policy_mapping_fn=_map).validate()
    with pytest.raises(NotImplementedError, match="recurrent"):
        (rllib.DQNConfig().environment(CooperativeMatchEnv)
         .multi_agent(policies=["pa", "pb"], policy_mapping_fn=_map)
         .training(model={"use_lstm": True}).validate())


@pytest.mark.parametrize("algo_name", ["IMPALA", "APPO"])
def test_recurrent_impala_appo_multi_agent_learn_memory_task(algo_name):
    """LSTM modules per agent under V-trace: each agent-segment column is unrolled
    from the state its runner recorded at the column's first step."""
    env_cls = make_multi_agent("RepeatAfterMe-v0")
    cfg = (getattr(rllib, algo_name + "Config")().environment(env_cls, env_config={"num_agents": 2})
           .env_runners(num_envs_per_env_runner=8, rollout_fragment_length=40)
           .multi_agent(policies=["p0", "p1"], policy_mapping_fn=_map)
           .training(lr=3e-3, train_batch_size=320, gamma=0.5, vf_loss_coeff=0.5, entropy_coeff=0.0,
                     model={"fcnet_hiddens": [64], "use_lstm": True, "lstm_cell_size": 64, "max_seq_len": 20})
           .reporting(metrics_num_episodes_for_smoothing=16).debugging(seed=0))
    algo = cfg.build()
    best = {"p0": 0.0, "p1": 0.0}
    for _ in range(150):
        r = algo.train()
        for m, v in r["env_runners"]["module_episode_returns_mean"].items():
            best[m] = max(best[m], v)
        if min(best.values()) > 16:
            break
    assert min(best.values()) > 16, best  # chance is ~9.5 per agent, the optimum 19
    algo.stop()
