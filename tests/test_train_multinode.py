"""Multi-node TorchTrainer rendezvous on CPU (reference:
python/ray/train/torch/config.py:66 -- MASTER_ADDR is the rank-0 worker's node IP).

A head at 127.0.0.1 and a node agent that registers as 127.0.0.2 (both loopback
addresses on one machine): every worker learns its node's IP (CAAMD_NODE_IP), the
trainer rendezvouses at rank 0's node address, and a gloo all-reduce across the two
"nodes" succeeds."""
import os
import subprocess
import sys
import time

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import train
from cluster_anywhere_amd.train import ScalingConfig
from cluster_anywhere_amd.train.torch import TorchTrainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def two_ip_nodes(tmp_path):
    ctx = ray.init(num_cpus=2, _listen_tcp="127.0.0.1:0")
    env = dict(os.environ, PYTHONPATH=ROOT)
    agent = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address",
                              ctx["gcs_address"], "--num-cpus", "2", "--num-gpus", "0",
                              "--node-ip-address", "127.0.0.2", "--object-store-memory", str(128 << 20)], env=env)
    deadline = time.time() + 60
    while time.time() < deadline and sum(n["Alive"] for n in ray.nodes()) < 2:
        time.sleep(0.1)
    assert sum(n["Alive"] for n in ray.nodes()) == 2
    yield str(tmp_path)
    agent.kill()
    agent.wait()
    ray.shutdown()


def _loop():
    import torch
    import torch.distributed as dist

    ctx = train.get_context()
    t = torch.tensor([float(ctx.get_world_rank() + 1)])
    dist.all_reduce(t)
    train.report({"sum": float(t.item()), "master": os.environ["MASTER_ADDR"],
                  "node_ip": os.environ.get("CAAMD_NODE_IP"), "rank": ctx.get_world_rank()})


def test_rendezvous_uses_rank0_node_ip(two_ip_nodes):
    assert {n["NodeManagerAddress"] for n in ray.nodes()} == {"127.0.0.1", "127.0.0.2"}
    trainer = TorchTrainer(_loop, scaling_config=ScalingConfig(num_workers=2, placement_strategy="STRICT_SPREAD"),
                           run_config=train.RunConfig(storage_path=two_ip_nodes, name="mn"))
    res = trainer.fit()
    assert res.error is None
    m = res.metrics
    assert m["sum"] == 3.0
    # rank 0 reports; MASTER_ADDR is rank 0's own node address
    assert m["rank"] == 0 and m["master"] == m["node_ip"]
    assert m["node_ip"] in ("127.0.0.1", "127.0.0.2")


def test_master_addr_is_not_loopback_default(two_ip_nodes):
    """Workers packed onto the 127.0.0.2 node (the head has 2 CPUs, the packed group
    needs 2 + 1 of the agent's): rank 0 sits on the agent, so MASTER_ADDR must be
    127.0.0.2 -- the old hard-coded 127.0.0.1 fails this."""
    @ray.remote(num_cpus=2)
    class Hog:  # keeps the head node's CPUs busy so the group lands on the agent
        def ok(self):
            return os.environ.get("CAAMD_NODE_IP")

    h = Hog.remote()
    assert ray.get(h.ok.remote()) == "127.0.0.1"
    trainer = TorchTrainer(_loop, scaling_config=ScalingConfig(num_workers=2, placement_strategy="PACK"),
                           run_config=train.RunConfig(storage_path=two_ip_nodes, name="mn2"))
    res = trainer.fit()
    assert res.error is None
    assert res.metrics["node_ip"] == "127.0.0.2" and res.metrics["master"] == "127.0.0.2"
    assert res.metrics["sum"] == 3.0


def test_rccl_transport_parser():
    from cluster_anywhere_amd.train.torch import rccl_transports

    lines = ["host:1:2 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC",
             "host:1:2 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC",
             "host:1:2 [0] NCCL INFO Channel 00/0 : 1[1] -> 0[0] via SHM/direct/direct",
             "host:1:2 [0] NCCL INFO Channel 02/0 : 0[0] -> 8[0] [send] via NET/IB/0",
             "host:1:2 [0] NCCL INFO Connected all rings"]
    assert rccl_transports(lines) == {"P2P/IPC": 2, "SHM/direct/direct": 1, "NET": 1}
