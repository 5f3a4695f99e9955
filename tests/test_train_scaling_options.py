"""``ScalingConfig.accelerator_type`` and ``trainer_resources`` (reference:
python/ray/air/config.py:156-161 trainer bundle first in the placement-group
factory, :209-215 ``accelerator_type:<X>`` requested per worker bundle;
tests modelled on train/tests/test_base_trainer.py / test_backend.py resource
checks). Two nodes on one machine: the head without an accelerator, a second node
advertising ``accelerator_type:AMD-Instinct-MI355X-OAM``."""
import os

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import train
from cluster_anywhere_amd.train import RunConfig, ScalingConfig
from cluster_anywhere_amd.train.torch import TorchConfig, TorchTrainer
from cluster_anywhere_amd.util.accelerators import AMD_INSTINCT_MI355X

ACC = f"accelerator_type:{AMD_INSTINCT_MI355X}"


def test_scaling_config_bundles():
    sc = ScalingConfig(num_workers=2, accelerator_type=AMD_INSTINCT_MI355X, trainer_resources={"CPU": 2})
    b = sc.as_placement_group_bundles()
    assert b[0] == {"CPU": 2.0}
    assert b[1] == b[2] == {"CPU": 1.0, ACC: 0.001}
    assert sc.total_resources == {"CPU": 4.0, ACC: 0.002}
    # defaults: no coordinator bundle when there are workers
    assert ScalingConfig(num_workers=3).as_placement_group_bundles() == [{"CPU": 1.0}] * 3


def test_detect_accelerator_type_env(monkeypatch):
    from cluster_anywhere_amd.core.api import accelerator_resources, detect_accelerator_type

    monkeypatch.setenv("CAAMD_ACCELERATOR_TYPE", AMD_INSTINCT_MI355X)
    assert detect_accelerator_type() == AMD_INSTINCT_MI355X
    assert accelerator_resources([0]) == {ACC: 1.0}
    assert accelerator_resources([]) == {}


@pytest.fixture
def accel_cluster(tmp_path):
    from cluster_anywhere_amd.cluster_utils import Cluster

    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 4})
    try:
        node = c.add_node(num_cpus=4, resources={ACC: 1.0})
        c.connect()
        c.wait_for_nodes()
        yield node, str(tmp_path)
    finally:
        ray.shutdown()
        c.shutdown()


def _make_loop():
    # defined inside a function: pickled by value (the node processes of the
    # Cluster do not have tests/ on their path)
    def loop(cfg=None):
        import torch
        import torch.distributed as dist

        import cluster_anywhere_amd as r
        from cluster_anywhere_amd import train as t_

        rt = r.get_runtime_context()
        avail = r.available_resources().get("CPU", 0.0)
        mine = rt.get_node_id()
        on_acc = any(n["NodeID"] == mine and any(k.startswith("accelerator_type:") for k in n["Resources"])
                     for n in r.nodes())
        t = torch.tensor([1.0, float(on_acc)])
        dist.all_reduce(t)
        t_.report({"node": mine, "cpu_free": avail, "world": float(t[0]), "ranks_on_acc": float(t[1])})

    return loop


def test_accelerator_type_schedules_on_labelled_node(accel_cluster):
    node, tmp = accel_cluster
    acc_nodes = [n["NodeID"] for n in ray.nodes() if n["Resources"].get(ACC)]
    assert len(acc_nodes) == 1
    trainer = TorchTrainer(
        _make_loop(), torch_config=TorchConfig(backend="gloo"),
        scaling_config=ScalingConfig(num_workers=2, accelerator_type=AMD_INSTINCT_MI355X,
                                     trainer_resources={"CPU": 1}),
        run_config=RunConfig(name="acc", storage_path=tmp))
    res = trainer.fit()
    assert res.error is None
    assert res.metrics["node"] == acc_nodes[0]
    assert res.metrics["world"] == 2.0
    # 8 CPUs in the cluster: 2 workers + the coordinator's 1 reserved while training
    assert res.metrics["cpu_free"] <= 8 - 3 + 1e-6
    # every rank ran on the accelerator node
    assert res.metrics["ranks_on_acc"] == 2.0


def test_unknown_accelerator_type_is_not_scheduled(accel_cluster, monkeypatch):
    node, tmp = accel_cluster
    monkeypatch.setenv("CAAMD_TRAIN_PG_TIMEOUT", "3")
    trainer = TorchTrainer(
        _make_loop(), torch_config=TorchConfig(backend="gloo"),
        scaling_config=ScalingConfig(num_workers=1, accelerator_type="AMD-Instinct-MI999X"),
        run_config=RunConfig(name="noacc", storage_path=tmp))
    res = None
    with pytest.raises(Exception, match="could not reserve"):
        res = trainer.fit()
        if res.error is not None:
            raise res.error
