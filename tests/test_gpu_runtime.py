"""Runtime on a real MI355X: GPU actors (ROCR_VISIBLE_DEVICES isolation, HIP
kernels inside workers), GPU tensors through the object store, and TorchTrainer
in actor mode driving the fused GPT-2 step on the GPU."""
import time

import pytest
import torch

import cluster_anywhere_amd as ray

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_gpu_actor_runs_hip_kernels(cluster):
    @ray.remote(num_gpus=1)
    class G:
        def info(self):
            import os

            import torch

            from cluster_anywhere_amd.ops import layer_norm

            x = torch.randn(16, 1600, device="cuda", dtype=torch.bfloat16)
            g = torch.ones(1600, device="cuda", dtype=torch.bfloat16)
            b = torch.zeros(1600, device="cuda", dtype=torch.bfloat16)
            y = layer_norm(x, g, b)
            ref = torch.nn.functional.layer_norm(x.float(), (1600,))
            err = (y.float() - ref).abs().max().item()
            return (torch.cuda.device_count(), os.environ.get("ROCR_VISIBLE_DEVICES"),
                    ray.get_gpu_ids(), err)

    n, vis, ids, err = ray.get(G.remote().info.remote(), timeout=300)
    assert n == 1 and vis is not None and len(ids) == 1
    assert err < 0.05


def test_gpu_tensor_roundtrip(cluster):
    @ray.remote(num_gpus=1)
    def make():
        import torch

        return torch.arange(1000, device="cuda", dtype=torch.float32)

    t = ray.get(make.remote(), timeout=300)
    assert t.is_cuda and float(t.sum()) == sum(range(1000))


def test_torch_trainer_gpu_actor_mode(cluster, tmp_path):
    from cluster_anywhere_amd import train
    from cluster_anywhere_amd.train import RunConfig, ScalingConfig
    from cluster_anywhere_amd.train.torch import TorchTrainer, get_device, prepare_data_parallel_step

    def loop(cfg):
        import torch

        from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config

        torch.manual_seed(0)
        mc = GPT2Config.named("gpt2-tiny")
        step = prepare_data_parallel_step(GPT2(mc), lr=1e-3)
        dev = get_device()
        x = torch.randint(0, mc.vocab_size, (4, 65), device=dev)
        for i in range(cfg["steps"]):
            loss = step(x[:, :-1], x[:, 1:])
            train.report({"loss": float(loss), "device": str(dev)})

    r = TorchTrainer(loop, train_loop_config={"steps": 20},
                     scaling_config=ScalingConfig(num_workers=1, use_gpu=True),
                     run_config=RunConfig(name="gpu", storage_path=str(tmp_path))).fit()
    df = r.metrics_dataframe
    assert r.metrics["device"].startswith("cuda")
    assert df["loss"].iloc[-1] < df["loss"].iloc[0] - 1.0


def test_gpu_object_ipc_zero_copy(cluster):
    """tensor_transport="ipc": the consumer maps the producer's HBM allocation
    (a later in-place update by the producer is visible to the consumer)."""

    @ray.remote(num_gpus=0.4)
    class Producer:
        def __init__(self):
            import torch

            self.t = torch.zeros(1 << 20, device="cuda", dtype=torch.float32)

        @ray.method(tensor_transport="ipc")
        def get(self):
            return self.t

        def bump(self):
            import torch

            self.t.add_(1.0)
            torch.cuda.synchronize()
            return True

    @ray.remote(num_gpus=0.4)
    class Consumer:
        def hold(self, t):
            self.t = t
            return (t.is_cuda, float(self.t.sum()))

        def first(self):
            import torch

            torch.cuda.synchronize()
            return float(self.t[0])

        def drop(self):
            import gc

            import torch

            self.t = None
            gc.collect()
            torch.cuda.synchronize()
            return True

    p, c = Producer.remote(), Consumer.remote()
    ref = p.get.remote()
    assert ray.get(c.hold.remote(ref), timeout=300) == (True, 0.0)
    assert ray.get(p.bump.remote(), timeout=60)
    assert ray.get(c.first.remote(), timeout=60) == 1.0
    # the driver (same node, GPU visible) maps it too
    t = ray.get(ref, timeout=60)
    assert t.is_cuda and float(t[0]) == 1.0
    # explicit put with ipc transport
    x = torch.arange(64, device="cuda", dtype=torch.float32)
    r2 = ray.put(x, _tensor_transport="ipc")
    assert ray.get(c.hold.remote(r2), timeout=60) == (True, float(sum(range(64))))
    # readers release their IPC views BEFORE the producer goes away (the producer's
    # HBM backs them); a read after the producer died fails loudly instead of
    # mapping freed memory
    # (a SIGKILLed reader never releases its mapping: let it drop its views first)
    assert ray.get(c.drop.remote(), timeout=60)
    ray.kill(c)
    del t
    torch.cuda.synchronize()
    ray.kill(p)
    time.sleep(1.0)
    with pytest.raises(ray.exceptions.ObjectLostError):
        ray.get(ref, timeout=60)


def test_collective_rccl_single_rank(cluster):
    """util.collective over RCCL (backend 'nccl') in a GPU actor."""

    @ray.remote(num_gpus=0.1)
    class M:
        def run(self):
            import torch

            import cluster_anywhere_amd.util.collective as col

            col.init_collective_group(1, 0, backend="rccl", group_name="r1")
            t = torch.full((1024,), 2.0, device="cuda")
            col.allreduce(t, group_name="r1")
            col.broadcast(t, 0, group_name="r1")
            col.barrier("r1")
            col.destroy_collective_group("r1")
            return float(t.sum())

    assert ray.get(M.remote().run.remote(), timeout=120) == 2048.0


def test_compiled_dag_ipc_gpu_edge(cluster):
    """Compiled graph with a HIP-IPC tensor edge: the producer's HBM buffers are
    mapped once by the consumer (two actors sharing the GPU); values stay exact
    across pipelined executions (buffer reuse is safe)."""
    from cluster_anywhere_amd.dag import InputNode

    @ray.remote(num_gpus=0.4)
    class Prod:
        def make(self, x):
            import torch

            return {"t": torch.arange(1 << 16, device="cuda", dtype=torch.float32) * x, "tag": x}

    @ray.remote(num_gpus=0.4)
    class Cons:
        def use(self, d):
            t = d["t"]
            assert t.is_cuda
            return float(t.sum()), d["tag"]

    p, c = Prod.remote(), Cons.remote()
    with InputNode() as inp:
        dag = c.use.bind(p.make.bind(inp).with_tensor_transport("ipc"))
    cdag = dag.experimental_compile(_max_inflight_executions=4)
    try:
        base = float(sum(range(1 << 16)))
        refs = [cdag.execute(float(i)) for i in range(4)]
        outs = [ray.get(r, timeout=120) for r in refs]
        for i in range(4, 24):
            outs.append(ray.get(cdag.execute(float(i)), timeout=120))
        for i, (s, tag) in enumerate(outs):
            assert tag == float(i) and s == pytest.approx(base * i, rel=1e-6)
    finally:
        cdag.teardown()
    ray.kill(c)
    ray.kill(p)


def test_compiled_dag_ipc_asyncio_overlap(cluster):
    """asyncio execution + overlap_gpu_communication over HIP-IPC edges: the
    producer's copy into the shared HBM buffer runs on its comm stream and the ring
    message is published by its writer thread once the copy's event completed; the
    consumer's copy-out runs on its comm stream and is waited for only before its
    next read of the edge. 8 executions in flight from one event loop; every value
    exact (no buffer reused early)."""
    import asyncio

    from cluster_anywhere_amd.dag import InputNode

    @ray.remote(num_gpus=0.3)
    class Prod:
        def make(self, x):
            import torch

            t = torch.arange(1 << 20, device="cuda", dtype=torch.float32) * x
            torch.cuda._sleep(2_000_000)  # compute still running when the loop moves on
            return {"t": t + 0.0, "tag": x}

    @ray.remote(num_gpus=0.3)
    class Mid:
        def step(self, d):
            return {"t": d["t"] * 2.0, "tag": d["tag"]}

    @ray.remote(num_gpus=0.3)
    class Cons:
        def use(self, d):
            t = d["t"]
            assert t.is_cuda
            return float(t.double().sum()), d["tag"]

    p, m, c = Prod.remote(), Mid.remote(), Cons.remote()
    with InputNode() as inp:
        x = p.make.bind(inp).with_tensor_transport("ipc")
        y = m.step.bind(x).with_tensor_transport("ipc")
        dag = c.use.bind(y)
    cdag = dag.experimental_compile(enable_asyncio=True, _max_inflight_executions=8,
                                    _overlap_gpu_communication=True)
    base = float(sum(range(1 << 20)))

    async def main():
        futs = [await cdag.execute_async(float(i)) for i in range(8)]
        outs = list(await asyncio.gather(*futs))

        async def one(i):
            return await (await cdag.execute_async(float(i)))

        outs += await asyncio.gather(*[one(i) for i in range(8, 40)])
        return outs

    try:
        outs = asyncio.run(main())
        for i, (s, tag) in enumerate(outs):
            assert tag == float(i) and s == pytest.approx(2.0 * base * i, rel=1e-6)
    finally:
        cdag.teardown()
    for a in (c, m, p):
        ray.kill(a)
