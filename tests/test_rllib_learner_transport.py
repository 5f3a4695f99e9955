"""Train-batch hand-off to learner actors (LearnerGroup ``learner_batch_transport``):
the object-store ("shm") and HIP-IPC paths train exactly like the per-shard pickle
path (BASELINE config 4: hipIpc sample-batch hand-off). CPU: pickle vs shm with two
gloo learners; GPU: ipc vs pickle with two learners sharing one GPU (gloo group)."""
import numpy as np
import pytest
import torch

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.rllib.core.learner import Learner, LearnerGroup


class _Lin(torch.nn.Module):
    def __init__(self, obs_space=None, act_space=None):
        super().__init__()
        torch.manual_seed(0)
        self.l = torch.nn.Linear(8, 1)

    def get_state(self):
        return {k: v.detach().cpu() for k, v in self.state_dict().items()}

    def set_state(self, st):
        self.load_state_dict(st)


def _factory(obs_space, act_space):
    return _Lin()


class _MSE(Learner):
    def compute_loss(self, batch):
        pred = self.module.l(batch["x"].float()).squeeze(-1)
        loss = ((pred - batch["y"].float()) ** 2).mean()
        return {"default": loss}, {"loss": loss.detach()}


def _batch(n=64):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((n, 8)).astype(np.float32)
    return {"x": x, "y": (x @ np.arange(8, dtype=np.float32)).astype(np.float32)}


def _train(transport, cfg_extra=None, updates=3, num_learners=2):
    cfg = {"num_learners": num_learners, "lr": 1e-2, "seed": 0, "learner_batch_transport": transport,
           "num_gpus_per_learner": 0, **(cfg_extra or {})}
    g = LearnerGroup(_MSE, cfg, _factory, None, None)
    try:
        assert g.batch_transport(_batch()) == transport
        for _ in range(updates):
            st = g.update(_batch(), minibatch_size=32, num_epochs=2, shuffle=False)
        states = ray.get([a.call.remote("get_module_state") for a in g.actors])
        return st, states
    finally:
        g.stop()


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6)
    yield
    ray.shutdown()


def test_shm_transport_matches_pickle(cluster):
    st_p, w_p = _train("pickle")
    st_s, w_s = _train("shm")
    assert abs(st_p["loss"] - st_s["loss"]) < 1e-6
    for a, b in zip(w_p, w_s):
        for k in a:
            assert torch.equal(a[k], b[k])
    for k in w_s[0]:  # data-parallel replicas stay in sync
        assert torch.equal(w_s[0][k], w_s[1][k])


def test_auto_transport_on_cpu_is_shm(cluster):
    g = LearnerGroup(_MSE, {"num_learners": 2, "num_gpus_per_learner": 0}, _factory, None, None)
    try:
        assert g.batch_transport(_batch()) == "shm"
        assert g.batch_transport({"m": _batch()}) == "shm"  # nested multi-module batches
    finally:
        g.stop()
