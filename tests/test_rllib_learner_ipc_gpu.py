"""HIP-IPC sample-batch hand-off between GPU learners (LearnerGroup "ipc"): rank 0
stages the batch in its HBM once, the other learner copies its shard out of rank
0's memory through a HIP IPC handle; the trained weights equal the pickle path's."""
import pytest
import torch

import cluster_anywhere_amd as ray

from test_rllib_learner_transport import _train

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cluster():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    ray.init(num_cpus=4, num_gpus=1)
    yield
    ray.shutdown()


def test_ipc_transport_matches_pickle(cluster):
    extra = {"num_gpus_per_learner": 0.5, "learner_dist_backend": "gloo"}  # two learners share the GPU
    st_p, w_p = _train("pickle", extra)
    st_i, w_i = _train("ipc", extra)
    assert abs(st_p["loss"] - st_i["loss"]) < 1e-5
    for a, b in zip(w_p, w_i):
        for k in a:
            torch.testing.assert_close(a[k], b[k], rtol=1e-6, atol=1e-6)


def test_ipc_transport_three_learners_matches_pickle(cluster):
    """with n >= 3 learners one IPC share of rank 0's staged
    batch is read by n - 1 peers; rank 0 keeps it until every update_shard returned
    (release_staged), so no peer copies out of freed / reused HBM."""
    extra = {"num_gpus_per_learner": 0.3, "learner_dist_backend": "gloo"}
    st_p, w_p = _train("pickle", extra, num_learners=3)
    st_i, w_i = _train("ipc", extra, num_learners=3)
    assert abs(st_p["loss"] - st_i["loss"]) < 1e-5
    for a, b in zip(w_p, w_i):
        for k in a:
            torch.testing.assert_close(a[k], b[k], rtol=1e-6, atol=1e-6)
