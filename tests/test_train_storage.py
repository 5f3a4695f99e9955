"""Train run storage (reference: python/ray/train/_internal/storage.py:193,297,358,514):
``RunConfig(storage_path, storage_filesystem)`` is honoured -- pyarrow filesystems,
fsspec filesystems and URIs; workers upload their (node-local) checkpoint
directories into the experiment on the storage filesystem; results and restores
read them back through it, including a worker on a node other than the driver's."""
import os
import subprocess
import sys
import tempfile
import time

import pyarrow.fs as pafs
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import train
from cluster_anywhere_amd.train import Checkpoint, ScalingConfig
from cluster_anywhere_amd.train.storage import StorageContext, get_fs_and_path
from cluster_anywhere_amd.train.torch import TorchTrainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_storage_context_with_fsspec_memory_filesystem(tmp_path):
    import fsspec

    mem = fsspec.filesystem("memory")
    st = StorageContext("/bucket/runs", "exp", storage_filesystem=mem)
    assert not st.local and st.experiment_fs_path == "/bucket/runs/exp"
    st.create_experiment_dir()
    src = tmp_path / "w0"
    src.mkdir()
    (src / "model.bin").write_bytes(b"\x01" * 1000)
    (src / "sub").mkdir()
    (src / "sub" / "opt.txt").write_text("adam")
    p = st.persist_checkpoint(str(src), "checkpoint_000000")
    assert p == "/bucket/runs/exp/checkpoint_000000"
    assert mem.cat_file("/bucket/runs/exp/checkpoint_000000/model.bin") == b"\x01" * 1000
    assert st.list_checkpoints() == ["checkpoint_000000"]
    ck = Checkpoint(p, filesystem=st.storage_filesystem)
    ck.set_metadata({"step": 7})
    assert ck.get_metadata() == {"step": 7}
    with ck.as_directory() as d:
        assert open(os.path.join(d, "sub", "opt.txt")).read() == "adam"
    out = ck.to_directory(str(tmp_path / "dl"))
    assert open(os.path.join(out, "model.bin"), "rb").read() == b"\x01" * 1000
    st.write_text("result.json", '{"a": 1}\n')
    st.delete(p)
    assert st.list_checkpoints() == []


def test_uri_and_plain_paths_resolve(tmp_path):
    fs, path = get_fs_and_path(f"file://{tmp_path}/x")
    assert isinstance(fs, pafs.LocalFileSystem) and path.endswith("/x")
    fs, path = get_fs_and_path(str(tmp_path / "y"))
    assert isinstance(fs, pafs.LocalFileSystem) and os.path.isabs(path)


def _loop(cfg):
    ctx = train.get_context()
    start = 0
    ck = train.get_checkpoint()
    if ck is not None:
        with ck.as_directory() as d:
            start = int(open(os.path.join(d, "step.txt")).read()) + 1
    for step in range(start, start + 2):
        d = tempfile.mkdtemp(prefix="worker_local_")  # node-local directory of THIS worker
        with open(os.path.join(d, f"rank{ctx.get_world_rank()}.txt"), "w") as f:
            f.write(f"{os.environ.get('CAAMD_NODE_IP', '?')}")
        if ctx.get_world_rank() == 0:
            with open(os.path.join(d, "step.txt"), "w") as f:
                f.write(str(step))
        train.report({"step": step, "start": start, "node_ip": os.environ.get("CAAMD_NODE_IP")},
                     checkpoint=Checkpoint.from_directory(d))


@pytest.fixture
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_trainer_persists_to_subtree_filesystem_and_resumes(cluster, tmp_path):
    base = tmp_path / "bucket"
    base.mkdir()
    fs = pafs.SubTreeFileSystem(str(base), pafs.LocalFileSystem())
    rc = train.RunConfig(name="exp", storage_path="runs", storage_filesystem=fs,
                         checkpoint_config=train.CheckpointConfig(num_to_keep=1))
    res = TorchTrainer(_loop, scaling_config=ScalingConfig(num_workers=2), run_config=rc).fit()
    assert res.error is None and res.metrics["step"] == 1
    assert res.path == "runs/exp" and res.filesystem is fs
    ckdir = base / "runs" / "exp" / res.checkpoint.path.rsplit("/", 1)[1]
    # every rank's shard was uploaded into the one checkpoint directory; top-1 retention
    assert sorted(os.listdir(ckdir)) == ["rank0.txt", "rank1.txt", "step.txt"]
    assert sorted(os.listdir(base / "runs" / "exp")) == ["checkpoint_000001", "result.json"]
    assert res.checkpoint.filesystem is fs
    # resume from the storage checkpoint (downloaded by the workers)
    rc2 = train.RunConfig(name="exp2", storage_path="runs", storage_filesystem=fs)
    res2 = TorchTrainer(_loop, scaling_config=ScalingConfig(num_workers=2), run_config=rc2,
                        resume_from_checkpoint=res.checkpoint).fit()
    assert res2.metrics["start"] == 2 and res2.metrics["step"] == 3
    r = train.Result.from_path("runs/exp", storage_filesystem=fs)
    assert r.metrics["step"] == 1 and r.checkpoint.path.endswith("checkpoint_000001")


@pytest.fixture
def two_nodes(tmp_path):
    ctx = ray.init(num_cpus=1, _listen_tcp="127.0.0.1:0")
    env = dict(os.environ, PYTHONPATH=ROOT)
    agent = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address",
                              ctx["gcs_address"], "--num-cpus", "2", "--num-gpus", "0", "--resources",
                              '{"side": 2}', "--node-ip-address", "127.0.0.2", "--object-store-memory",
                              str(128 << 20)], env=env)
    deadline = time.time() + 60
    while time.time() < deadline and sum(n["Alive"] for n in ray.nodes()) < 2:
        time.sleep(0.1)
    assert sum(n["Alive"] for n in ray.nodes()) == 2
    yield
    agent.kill()
    agent.wait()
    ray.shutdown()


def test_checkpoint_written_on_the_other_node_restores(two_nodes, tmp_path):
    """Workers pinned to the non-driver node ("side") write node-local checkpoints that
    reach the storage filesystem; a second run there restores from them."""
    base = tmp_path / "store"
    base.mkdir()
    fs = pafs.SubTreeFileSystem(str(base), pafs.LocalFileSystem())
    sc = ScalingConfig(num_workers=1, resources_per_worker={"CPU": 1, "side": 1})
    res = TorchTrainer(_loop, scaling_config=sc,
                       run_config=train.RunConfig(name="mn", storage_path="r", storage_filesystem=fs)).fit()
    assert res.metrics["node_ip"] == "127.0.0.2"
    assert os.path.exists(base / "r" / "mn" / "checkpoint_000001" / "step.txt")
    res2 = TorchTrainer(_loop, scaling_config=sc, resume_from_checkpoint=res.checkpoint,
                        run_config=train.RunConfig(name="mn2", storage_path="r", storage_filesystem=fs)).fit()
    assert res2.metrics["start"] == 2 and res2.metrics["node_ip"] == "127.0.0.2"


def test_tune_experiment_mirrors_to_storage_and_restores(cluster, tmp_path):
    from cluster_anywhere_amd import tune

    base = tmp_path / "tb"
    base.mkdir()
    fs = pafs.SubTreeFileSystem(str(base), pafs.LocalFileSystem())

    def trainable(config):
        for i in range(3):
            tune.report({"score": config["x"] * (i + 1)})

    os.environ["CAAMD_TUNE_STAGING_DIR"] = str(tmp_path / "staging")
    try:
        grid = tune.Tuner(trainable, param_space={"x": tune.grid_search([1, 2])},
                          tune_config=tune.TuneConfig(metric="score", mode="max"),
                          run_config=tune.RunConfig(name="texp", storage_path="tune_runs",
                                                    storage_filesystem=fs)).fit()
        assert grid.get_best_result().metrics["score"] == 6
        assert grid.storage_path == "tune_runs/texp"
        assert (base / "tune_runs" / "texp" / "experiment_state.json").exists()
        assert tune.Tuner.can_restore("tune_runs/texp", storage_filesystem=fs)
        import shutil

        shutil.rmtree(tmp_path / "staging")  # restore must come from the storage filesystem
        t2 = tune.Tuner.restore("tune_runs/texp", trainable, storage_filesystem=fs)
        g2 = t2.fit()
        assert g2.get_best_result().metrics["score"] == 6 and len(g2) == 2
    finally:
        os.environ.pop("CAAMD_TUNE_STAGING_DIR", None)
