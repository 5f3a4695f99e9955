"""TorchTrainer on CPU (gloo, 2 workers): metrics, checkpoints, resume and
fault tolerance (reference: python/ray/train/tests/test_torch_trainer.py,
test_backend.py, test_new_persistence.py)."""
import os
import tempfile

import pytest
import torch

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import train
from cluster_anywhere_amd.train import (Checkpoint, CheckpointConfig, FailureConfig, RunConfig,
                                        ScalingConfig)
from cluster_anywhere_amd.train.torch import TorchTrainer, prepare_model


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def loop(config):
    import torch.distributed as dist

    ctx = train.get_context()
    torch.manual_seed(0)
    model = prepare_model(torch.nn.Linear(4, 1))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    start = 0
    ck = train.get_checkpoint()
    if ck is not None:
        with ck.as_directory() as d:
            st = torch.load(os.path.join(d, "state.pt"), weights_only=True)
            start = st["epoch"] + 1
            (model.module if hasattr(model, "module") else model).load_state_dict(st["model"])
    x = torch.randn(64, 4)
    y = x.sum(1, keepdim=True)
    for epoch in range(start, config["epochs"]):
        loss = ((model(x) - y) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        if config.get("crash_at") == epoch and not os.path.exists(config["marker"]):
            open(config["marker"], "w").close()
            os._exit(1)
        with tempfile.TemporaryDirectory() as d:
            if ctx.get_world_rank() == 0:
                m = model.module if hasattr(model, "module") else model
                torch.save({"epoch": epoch, "model": m.state_dict()}, os.path.join(d, "state.pt"))
            train.report({"loss": loss.item(), "epoch": epoch, "world": dist.get_world_size()},
                         checkpoint=Checkpoint.from_directory(d))


def test_torch_trainer_ddp_gloo(cluster, tmp_path):
    t = TorchTrainer(loop, train_loop_config={"epochs": 4},
                     scaling_config=ScalingConfig(num_workers=2),
                     run_config=RunConfig(name="ddp", storage_path=str(tmp_path),
                                          checkpoint_config=CheckpointConfig(num_to_keep=2)))
    r = t.fit()
    assert r.error is None
    assert r.metrics["world"] == 2 and r.metrics["epoch"] == 3
    assert r.checkpoint is not None and os.path.exists(os.path.join(r.checkpoint.path, "state.pt"))
    assert len(r.metrics_dataframe) == 4
    ckpts = sorted(d for d in os.listdir(r.path) if d.startswith("checkpoint_"))
    assert len(ckpts) == 2  # num_to_keep


def test_torch_trainer_fault_tolerance(cluster, tmp_path):
    marker = str(tmp_path / "crashed")
    t = TorchTrainer(loop, train_loop_config={"epochs": 4, "crash_at": 2, "marker": marker},
                     scaling_config=ScalingConfig(num_workers=2),
                     run_config=RunConfig(name="ft", storage_path=str(tmp_path),
                                          failure_config=FailureConfig(max_failures=1)))
    r = t.fit()
    assert os.path.exists(marker)
    assert r.metrics["epoch"] == 3
    # resumed from the epoch-1 checkpoint: epochs 0,1 then (restart) 2,3
    assert [m["epoch"] for m in r.metrics_dataframe.to_dict("records")] == [0, 1, 2, 3]


def test_trainer_error_surfaces(cluster, tmp_path):
    def bad(config):
        raise ValueError("boom in loop")

    t = TorchTrainer(bad, scaling_config=ScalingConfig(num_workers=1),
                     run_config=RunConfig(name="bad", storage_path=str(tmp_path)))
    with pytest.raises(train.TrainingFailedError):
        t.fit()


def test_resume_from_checkpoint(cluster, tmp_path):
    t = TorchTrainer(loop, train_loop_config={"epochs": 2},
                     scaling_config=ScalingConfig(num_workers=1),
                     run_config=RunConfig(name="a", storage_path=str(tmp_path)))
    r = t.fit()
    t2 = TorchTrainer(loop, train_loop_config={"epochs": 4}, resume_from_checkpoint=r.checkpoint,
                      scaling_config=ScalingConfig(num_workers=1),
                      run_config=RunConfig(name="b", storage_path=str(tmp_path)))
    r2 = t2.fit()
    assert [m["epoch"] for m in r2.metrics_dataframe.to_dict("records")] == [2, 3]


def test_accelerate_amp_bf16_and_fp16_scaler():
    """accelerate(amp=True): prepare_model runs forward under autocast and returns
    fp32 outputs; fp16 AMP steps through a loss scaler (reference
    train_loop_utils.py:278)."""
    import torch

    from cluster_anywhere_amd.train import torch as tt

    torch.manual_seed(0)
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    m.load_state_dict(ref.state_dict())
    try:
        tt.accelerate(amp=True)
        pm = tt.prepare_model(m, move_to_device=False, parallel_strategy=None)
        x = torch.randn(8, 16)
        seen = []
        h = pm[0].register_forward_hook(lambda mod, i, o: seen.append(o.dtype))
        y = pm(x)
        h.remove()
        assert seen == [torch.bfloat16] and y.dtype == torch.float32
        opt = tt.prepare_optimizer(torch.optim.SGD(pm.parameters(), lr=0.1))
        loss = y.square().mean()
        tt.backward(loss)
        yr = ref(x)
        yr.square().mean().backward()
        g, gr = pm[0].weight.grad, ref[0].weight.grad
        assert torch.allclose(g, gr, rtol=0.1, atol=2e-2)
        opt.step()
        # fp16: scaled backward, scaler-driven step
        tt.accelerate(amp=True, amp_dtype=torch.float16)
        opt2 = tt.prepare_optimizer(torch.optim.SGD(ref.parameters(), lr=0.1))
        assert hasattr(opt2, "scaler")
        ref.zero_grad()
        tt.backward(ref(x).square().mean())
        opt2.step()
    finally:
        tt.accelerate(amp=False)
