"""RLlib offline I/O (reference: rllib/offline/offline_env_runner.py,
offline_data.py, offline_prelearner.py, estimators/): PPO env runners record
CartPole episodes to Parquet (whole episodes per file), BC trains from that
directory by streaming it through a Data pipeline (the driver holds one batch,
never the dataset), and the off-policy estimators are checked against a hand
computation (and against the identity: target == behaviour policy => IS / WIS
reproduce the behaviour return exactly)."""
import glob
import math
import os

import numpy as np
import pyarrow.parquet as pq
import pytest
import torch

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import rllib
from cluster_anywhere_amd.rllib.offline import (DirectMethod, DoublyRobust, ImportanceSampling,
                                                WeightedImportanceSampling)


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _ppo(out_dir, runners=1):
    return (rllib.PPOConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=runners, num_envs_per_env_runner=4, rollout_fragment_length=100)
            .training(lr=3e-4, train_batch_size=400, minibatch_size=100, num_epochs=2,
                      model={"fcnet_hiddens": [32, 32]})
            .offline_data(output=str(out_dir), output_max_rows_per_file=500)
            .debugging(seed=0))


def _read_all(d):
    files = sorted(glob.glob(os.path.join(d, "*.parquet")))
    assert files
    return files, [pq.read_table(f).to_pydict() for f in files]


def test_record_episodes_then_stream_bc_and_ope(cluster, tmp_path):
    rec = tmp_path / "rec"
    algo = _ppo(rec).build()
    # behaviour data from FIXED weights: sample without training in between
    for _ in range(6):
        algo.env_runner_group.sample()
    files = algo.env_runner_group.flush_output()
    assert files and all(f.endswith(".parquet") for f in files)
    files, tables = _read_all(str(rec))
    n_rows = 0
    for t in tables:
        n_rows += len(t["t"])
        eps = {}
        for e, step, te, tr, p in zip(t["eps_id"], t["t"], t["terminateds"], t["truncateds"], t["action_prob"]):
            eps.setdefault(e, []).append((step, te, tr))
            assert 0.0 < p <= 1.0
        for e, steps in eps.items():  # whole episodes per file, steps 0..n-1, only the last one done
            assert [s for s, _, _ in steps] == list(range(len(steps)))
            assert all(not (te or tr) for _, te, tr in steps[:-1]) and (steps[-1][1] or steps[-1][2])
    assert n_rows >= 6 * 400 * 0.5

    # ---- off-policy estimates, target == behaviour: IS and WIS give back the behaviour value
    algo.algo_config.input_ = str(rec)
    algo.algo_config.off_policy_estimation_methods = {"is": {"type": ImportanceSampling},
                                                      "wis": {"type": "wis"}}
    est = algo.estimate_off_policy()
    for name in ("is", "wis"):
        assert math.isclose(est[name]["v_target"], est[name]["v_behavior"], rel_tol=1e-4), est[name]
    assert est["is"]["num_episodes"] > 10
    algo.stop()

    # ---- BC streams the recorded directory
    bc = (rllib.BCConfig().environment("CartPole-v1").offline_data(input_=str(rec), shuffle_buffer_rows=256)
          .training(lr=1e-3, train_batch_size=128, model={"fcnet_hiddens": [32, 32]})
          .evaluation(off_policy_estimation_methods={"is": {"type": ImportanceSampling},
                                                     "wis": {"type": WeightedImportanceSampling},
                                                     "dm": {"type": DirectMethod, "q_model_config": {"n_iters": 60}},
                                                     "dr": {"type": DoublyRobust, "q_model_config": {"n_iters": 60}}})
          .debugging(seed=0))
    b = bc.build()
    assert b.offline_data.streaming and b.offline_data.memory is None
    first = b.train()["learners"]["default_policy"]["policy_loss"]
    for _ in range(int(3 * n_rows / 128)):  # ~3 epochs
        r = b.train()
    last = r["learners"]["default_policy"]["policy_loss"]
    assert b.offline_data.epochs >= 2
    assert float(last) < float(first)

    # ---- hand computation of IS / WIS for the BC policy on the recorded episodes
    module = b.get_module()
    gamma = b.algo_config.gamma
    per_is, per_b, rhos, rews = [], [], [], []
    for t in tables:
        obs = np.asarray(t["obs"], np.float32).reshape(len(t["t"]), -1)
        with torch.no_grad():
            logits = module.forward_train({"obs": torch.from_numpy(obs)})["action_dist_inputs"].double()
        pi_all = torch.softmax(logits, -1).numpy()
        by_ep = {}
        for i, e in enumerate(t["eps_id"]):
            by_ep.setdefault(e, []).append(i)
        for e, idx in by_ep.items():
            idx = sorted(idx, key=lambda i: t["t"][i])
            rho, acc, vt, vb = 1.0, [], 0.0, 0.0
            for k, i in enumerate(idx):
                a = int(t["actions"][i])
                rho *= pi_all[i, a] / t["action_prob"][i]
                vt += gamma ** k * rho * t["rewards"][i]
                vb += gamma ** k * t["rewards"][i]
                acc.append(rho)
            per_is.append(vt)
            per_b.append(vb)
            rhos.append(acc)
            rews.append([t["rewards"][i] for i in idx])
    est = b.estimate_off_policy()
    assert math.isclose(est["is"]["v_target"], float(np.mean(per_is)), rel_tol=1e-4)
    assert math.isclose(est["is"]["v_behavior"], float(np.mean(per_b)), rel_tol=1e-6)
    L = max(len(x) for x in rhos)
    w = [np.mean([x[k] for x in rhos if len(x) > k]) for k in range(L)]
    wis = np.mean([sum(gamma ** k * x[k] / w[k] * r[k] for k in range(len(x))) for x, r in zip(rhos, rews)])
    assert math.isclose(est["wis"]["v_target"], float(wis), rel_tol=1e-4)
    for name in ("dm", "dr"):
        assert math.isfinite(est[name]["v_target"]) and est[name]["v_target"] > 0
    b.stop()
