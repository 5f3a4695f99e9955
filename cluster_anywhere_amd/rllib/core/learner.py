"""Learner / LearnerGroup (reference: rllib/core/learner/learner.py,
learner_group.py, torch/torch_learner.py).

A Learner keeps its RLModule's parameters in ONE flat fp32 buffer
(``FlatParamSpace``), so the optimizer is one fused AdamW launch
(``adamw.hip``, with device-side global-norm clipping) and data-parallel
learners all-reduce one contiguous gradient buffer over RCCL (gloo on CPU).
``LearnerGroup`` runs either a local learner or ``num_learners`` learner actors
(one GPU each), sharding every train batch across them."""
from __future__ import annotations

import os
import socket
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import torch

from ...ops.optim import FusedAdamW
from ...ops.rl_encoder import accumulate_into_grad
from ...parallel.flat import FlatParamSpace


def _to_tensor(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device, non_blocking=True)
    t = torch.from_numpy(np.ascontiguousarray(x))
    if device.type == "cuda":
        t = t.pin_memory().to(device, non_blocking=True)
    return t


def _mean_stats(agg: Dict[str, list]) -> Dict[str, float]:
    """Per-minibatch stats stay on the device until the end of ``update``: one host
    sync per update instead of one per statistic per minibatch."""
    keys = list(agg)
    tens = [k for k in keys if agg[k] and isinstance(agg[k][0], torch.Tensor)]
    out = {k: float(np.mean([float(x) for x in agg[k]])) for k in keys if k not in tens}
    if tens:
        means = torch.stack([torch.stack([x.detach().float().reshape(()) for x in agg[k]]).mean() for k in tens])
        out.update(zip(tens, means.tolist()))
    return out


class Learner:
    # Subclasses whose compute_loss is free of host syncs and host-side mutable state
    # opt in to running forward+backward of each minibatch as ONE HIP-graph replay.
    graph_capturable = False

    def __init__(self, config: Dict[str, Any], module_factory: Callable, obs_space, act_space,
                 device: Optional[str] = None, rank: int = 0, world: int = 1):
        self.config = config
        if device is None:
            device = "cuda" if torch.cuda.is_available() and config.get("num_gpus_per_learner", 1) > 0 else "cpu"
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        if config.get("seed") is not None:
            torch.manual_seed(config["seed"])
        self.module = module_factory(obs_space, act_space).to(self.device)
        if world > 1:  # data-parallel replicas start from rank 0's weights
            import torch.distributed as dist

            with torch.no_grad():
                for t in list(self.module.parameters()) + list(self.module.buffers()):
                    dist.broadcast(t.data, 0)
        self.obs_space, self.act_space = obs_space, act_space
        self.build()
        self.optimizers: Dict[str, FusedAdamW] = {}
        self.flats: Dict[str, FlatParamSpace] = {}
        for name, params_module in self.param_groups().items():
            flat = FlatParamSpace(params_module, dtype=torch.float32, master_fp32=False,
                                  decay_rule=lambda n, p: False)
            flat.master = flat.param_buffer  # fp32 params are the master weights
            self.flats[name] = flat
            self.optimizers[name] = FusedAdamW(flat, lr=self.lr_for(name), betas=(0.9, 0.999),
                                               eps=config.get("adam_eps", 1e-7), weight_decay=0.0,
                                               max_grad_norm=config.get("grad_clip") or 0.0)
        self.num_updates = 0
        self._graphs: Dict[tuple, tuple] = {}
        self._graph_off = not (self.graph_capturable and self.device.type == "cuda" and world == 1
                               and len(self.flats) == 1 and config.get("learner_cuda_graph", True))

    # ---------------------------------------------------------------- hooks
    def build(self):
        pass

    def param_groups(self) -> Dict[str, torch.nn.Module]:
        return {"default": self.module}

    def lr_for(self, name: str) -> float:
        return self.config.get("lr", 5e-5)

    def compute_loss(self, batch: Dict[str, torch.Tensor]) -> (Dict[str, torch.Tensor], Dict[str, float]):
        """Returns ({param_group: loss}, stats)."""
        raise NotImplementedError

    def after_update(self):
        pass

    # --------------------------------------------------------------- update
    def _allreduce(self, flat: FlatParamSpace):
        if self.world > 1:
            import torch.distributed as dist

            dist.all_reduce(flat.grad_buffer)

    def update_once(self, batch: Dict[str, torch.Tensor]) -> Dict[str, float]:
        losses, stats = self.compute_loss(batch)
        names = list(losses)
        if len(names) == 1:  # .grad of every parameter is a view of the flat grad buffer
            flat = self.flats[names[0]]
            flat.zero_grad()
            with accumulate_into_grad():  # encoder kernels add wgrads straight into .grad
                losses[names[0]].backward()
            self._allreduce(flat)
            self.optimizers[names[0]].step(inv_world=1.0 / self.world)
            self.num_updates += 1
            self.after_update()
            return stats
        for i, name in enumerate(names):
            flat = self.flats[name]
            flat.zero_grad()
            # each group's loss only differentiates w.r.t. its own parameters
            params = [s.param for s in flat.slots]
            grads = torch.autograd.grad(losses[name], params, retain_graph=i < len(names) - 1, allow_unused=True)
            with torch.no_grad():
                for s, g in zip(flat.slots, grads):
                    if g is not None:
                        flat.grad_buffer[s.offset: s.offset + s.numel].copy_(g.reshape(-1))
            self._allreduce(flat)
            self.optimizers[name].step(inv_world=1.0 / self.world)
        self.num_updates += 1
        self.after_update()
        return stats

    def update(self, batch: Dict[str, Any], minibatch_size: Optional[int] = None,
               num_epochs: int = 1, shuffle: bool = True) -> Dict[str, float]:
        b = {k: _to_tensor(v, self.device) for k, v in batch.items()}
        n = next(iter(b.values())).shape[0]
        mbs = min(minibatch_size or n, n)
        agg: Dict[str, list] = {}
        for _ in range(num_epochs):
            perm = torch.randperm(n, device=self.device) if shuffle else torch.arange(n, device=self.device)
            for s in range(0, n - mbs + 1, mbs):
                idx = perm[s: s + mbs]
                st = None
                if not self._graph_off:
                    st = self._update_graphed(b, idx)
                if st is None:
                    st = self.update_once({k: v[idx] for k, v in b.items()})
                for k, v in st.items():
                    agg.setdefault(k, []).append(v)
        return _mean_stats(agg)

    # ------------------------------------------------------- HIP-graph step
    def _update_graphed(self, b: Dict[str, torch.Tensor], idx: torch.Tensor) -> Optional[Dict[str, Any]]:
        """forward + backward of one minibatch as a single graph replay (captured
        once per minibatch shape; inputs gathered straight into the graph's static
        buffers); the fused AdamW step stays eager (its step count / lr change).
        Returns None (and turns graphs off) if the loss cannot be captured."""
        key = tuple(sorted((k, (idx.shape[0],) + tuple(v.shape[1:]), v.dtype) for k, v in b.items()))
        ent = self._graphs.get(key)
        if ent is None:
            try:
                ent = self._capture(b, idx, key)
            except Exception as e:  # noqa: BLE001 - any capture problem -> eager path
                import warnings

                warnings.warn(f"learner HIP-graph capture failed ({type(e).__name__}: {e}); running eagerly")
                self._graph_off = True
                torch.cuda.synchronize(self.device)
                return None
        static_in, graph, stacked, keys, name = ent
        for k, v in b.items():
            torch.index_select(v, 0, idx, out=static_in[k])
        graph.replay()
        self.optimizers[name].step(inv_world=1.0)
        self.num_updates += 1
        self.after_update()
        st = stacked.clone()
        return {k: st[i] for i, k in enumerate(keys)}

    def _capture(self, b, idx, key):
        name = next(iter(self.flats))
        flat = self.flats[name]
        static_in = {k: v[idx].clone() for k, v in b.items()}
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):  # warm-up (allocator / kernel selection) outside the capture
            for _ in range(2):
                flat.zero_grad()
                losses, _ = self.compute_loss(static_in)
                with accumulate_into_grad():
                    losses[name].backward()
                # drop the warm-up graph: a live graph keeps the parameters' AccumulateGrad
                # nodes (bound to the stream they were created on) for the capture to reuse,
                # and autograd then warns of a stream mismatch that can break the capture
                del losses
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        import gc

        gc.collect()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=side):
            flat.grad_buffer.zero_()
            losses, stats = self.compute_loss(static_in)
            with accumulate_into_grad():
                losses[name].backward()
            keys = list(stats)
            if not all(isinstance(stats[k], torch.Tensor) for k in keys):
                raise TypeError("compute_loss stats must be tensors to be captured")
            stacked = torch.stack([stats[k].detach().float().reshape(()) for k in keys])
        ent = (static_in, graph, stacked, keys, name)
        self._graphs[key] = ent
        return ent

    # ---------------------------------------------------------------- state
    def get_module_state(self, on_device: bool = False):
        """CPU state dict; ``on_device``: a detached snapshot on the learner's device
        (for HIP-IPC weight broadcast to GPU env runners: no host copy)."""
        if on_device:
            return {k: v.detach().clone() for k, v in self.module.state_dict().items()}
        return self.module.get_state()

    def get_state(self):
        return {"module": self.module.get_state(),
                "optim": {k: {kk: (vv.cpu() if isinstance(vv, torch.Tensor) else vv)
                              for kk, vv in o.state_dict().items()} for k, o in self.optimizers.items()},
                "num_updates": self.num_updates}

    def set_state(self, st):
        self.module.set_state(st["module"])
        for k, o in self.optimizers.items():
            if k in st.get("optim", {}):
                sd = {kk: (vv.to(self.device) if isinstance(vv, torch.Tensor) else vv)
                      for kk, vv in st["optim"][k].items()}
                sd["master"] = self.flats[k].param_buffer.clone()
                o.load_state_dict(sd)
        self.num_updates = st.get("num_updates", 0)
        return True


class MultiLearner:
    """One inner Learner per trained module of a multi-agent setup (reference
    role: the multi-module Learner of rllib/core/learner/learner.py). Every
    module keeps its own flat fp32 parameter buffer and fused AdamW; batches,
    stats and states are dicts keyed by module id. ``MultiLearner.of(cls)``
    makes the class for a given algorithm learner (e.g. ``PPOLearner``)."""

    inner_cls = Learner

    @classmethod
    def of(cls, inner_cls):
        return type(f"Multi{inner_cls.__name__}", (cls,), {"inner_cls": inner_cls})

    def __init__(self, config, module_factories: Dict[str, Callable], obs_spaces: Dict, act_spaces: Dict,
                 device: Optional[str] = None, rank: int = 0, world: int = 1):
        self.config = config
        self.learners: Dict[str, Learner] = {}
        for j, mid in enumerate(sorted(module_factories)):
            c = dict(config)
            if c.get("seed") is not None:
                c["seed"] = c["seed"] + 7919 * j  # distinct initial weights per module
            self.learners[mid] = self.inner_cls(c, module_factories[mid], obs_spaces[mid], act_spaces[mid],
                                                device, rank, world)
        self.device = next(iter(self.learners.values())).device if self.learners else torch.device("cpu")

    @property
    def module(self):
        from .multi_rl_module import MultiRLModule

        return MultiRLModule({m: l.module for m, l in self.learners.items()})

    def postprocess(self, frags: Dict[str, Dict]) -> Dict[str, Dict]:
        return {m: self.learners[m].postprocess(f) for m, f in frags.items() if m in self.learners}

    def update(self, batch: Dict[str, Dict], minibatch_size=None, num_epochs=1, shuffle=True):
        return {m: self.learners[m].update(b, minibatch_size, num_epochs, shuffle)
                for m, b in batch.items() if m in self.learners}

    def update_kl(self, kls: Dict[str, float]):
        return {m: self.learners[m].update_kl(k) for m, k in kls.items() if m in self.learners}

    def get_module_state(self):
        return {m: l.get_module_state() for m, l in self.learners.items()}

    def get_state(self):
        return {m: l.get_state() for m, l in self.learners.items()}

    def set_state(self, st):
        for m, s in st.items():
            if m in self.learners:
                self.learners[m].set_state(s)
        return True

    def __getattr__(self, name):
        """Any other learner method (``train_on``, ``learn_fragments``,
        ``update_target`` ...): called per module. A first argument keyed by module
        ids is split so each module gets its own entry; otherwise the call is
        broadcast. Returns ``{module_id: result}``."""
        if name.startswith("_") or not callable(getattr(self.inner_cls, name, None)):
            raise AttributeError(name)

        def call(*args, **kw):
            learners = self.__dict__.get("learners", {})
            if args and isinstance(args[0], dict) and args[0] and set(args[0]) <= set(learners):
                return {m: getattr(learners[m], name)(a, *args[1:], **kw) for m, a in args[0].items()}
            return {m: getattr(l, name)(*args, **kw) for m, l in learners.items()}

        return call


def _shard_nested(batch, i, n):
    if isinstance(batch, dict):
        return {k: _shard_nested(v, i, n) for k, v in batch.items()}
    per = batch.shape[0] // n
    return batch[i * per:(i + 1) * per]


def _mean_nested(results):
    if isinstance(results[0], dict):
        return {k: _mean_nested([r[k] for r in results]) for k in results[0]}
    return float(np.mean(results))


class _LearnerActor:
    def __init__(self, learner_cls, config, module_factory, obs_space, act_space, rank, world, addr, port):
        if world > 1:
            import torch.distributed as dist

            os.environ.update({"MASTER_ADDR": addr, "MASTER_PORT": str(port), "RANK": str(rank),
                               "WORLD_SIZE": str(world)})
            backend = config.get("learner_dist_backend") or ("nccl" if torch.cuda.is_available() else "gloo")
            if torch.cuda.is_available():
                gpus = [int(g) for g in os.environ.get("CAAMD_GPU_IDS", "").split(",") if g]
                torch.cuda.set_device(gpus[0] if gpus else 0)
            dist.init_process_group(backend, rank=rank, world_size=world)
        dev = None
        if torch.cuda.is_available():
            gpus = [int(g) for g in os.environ.get("CAAMD_GPU_IDS", "").split(",") if g]
            dev = f"cuda:{gpus[0]}" if gpus and os.environ.get("CAAMD_NOSET_ROCR_VISIBLE_DEVICES") else "cuda"
        self.learner = learner_cls(config, module_factory, obs_space, act_space, dev, rank, world)

    def call(self, method, *args, **kwargs):
        return getattr(self.learner, method)(*args, **kwargs)

    def info(self):
        from ...runtime_context import get_runtime_context

        return {"node": get_runtime_context().get_node_id(), "cuda": self.learner.device.type == "cuda"}

    # -- sample-batch hand-off (LearnerGroup.update) -------------------------------
    def stage_ipc(self, batch):
        """Rank 0 of the HIP-IPC hand-off: the whole train batch (an object-store
        argument, host) goes to THIS learner's HBM once; returns ``[ref]`` whose GPU
        tensors the other learners of the node map through HIP IPC handles."""
        from ...core import api as core

        self._staged = {k: _to_tensor(v, self.learner.device) for k, v in batch.items()}
        return [core.put(self._staged, _tensor_transport="ipc")]

    def update_shard(self, staged, i, n, mbs, num_epochs, shuffle):
        """Train on shard ``i`` of ``n``: of rank 0's staged HBM batch (``staged``
        None on rank 0 itself; the IPC-mapped dict elsewhere, copied device to
        device into this learner's own memory) or of a host batch (``host=True``
        path, ``update_shard_host``)."""
        b = self._staged if staged is None else staged
        per = next(iter(b.values())).shape[0] // n
        shard = {k: v[i * per:(i + 1) * per] for k, v in b.items()}
        if staged is not None:
            shard = {k: v.to(self.learner.device, copy=True) for k, v in shard.items()}
        del b, staged
        # rank 0 keeps _staged: peers may still be copying their shards out of it
        # (one IPC share read by n-1 consumers); the group releases it once every
        # update_shard returned (release_staged), or the next stage_ipc replaces it
        return self.learner.update(shard, mbs, num_epochs, shuffle)

    def release_staged(self):
        self._staged = None
        return True

    def update_shard_host(self, batch, i, n, mbs, num_epochs, shuffle):
        return self.learner.update(_shard_nested(batch, i, n), mbs, num_epochs, shuffle)



def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class LearnerGroup:
    """The local learner (``num_learners == 0``) or N learner actors training one
    module data-parallel (gloo / RCCL process group).

    Learner actors are restarted (``restart_failed_learners``, up to
    ``max_num_learner_restarts``): a call that finds an actor dead tears the whole
    group down (its process group is broken), starts a new one on a fresh
    rendezvous port, restores the last learner state this group saw (the state of
    the last completed update: module weights, optimizer moments, update count)
    and runs the call again. The state to restore is rank 0's ``get_state``
    result, kept as an object-store ref owned by the group, after the first update
    and then every
    ``learner_checkpoint_interval`` updates (default 10: a restart may replay up
    to that many updates; 1 = after every update), never pulled to the driver.

    Train batches reach the learner actors (``learner_batch_transport``):
    ``"ipc"`` (default when every learner is a GPU learner on one node; BASELINE
    config 4's hipIpc sample-batch hand-off): the batch is put into the object
    store once, rank 0 copies it host->HBM once, and the other learners copy their
    shards HBM->HBM out of rank 0's memory through HIP IPC handles; ``"shm"``
    (default otherwise): put once, every learner slices its shard out of the
    shared-memory object; ``"pickle"``: one pickled shard per learner."""

    def __init__(self, learner_cls, config: Dict[str, Any], module_factory, obs_space, act_space):
        self.n = config.get("num_learners", 0)
        self.local = None
        self.actors = []
        self.restart_failed = bool(config.get("restart_failed_learners", True))
        self.max_restarts = int(config.get("max_num_learner_restarts", 100))
        self.ckpt_every = max(1, int(config.get("learner_checkpoint_interval", 10)))
        self.num_restarts = 0
        self._last_state = None
        self._updates = 0
        self._info = []
        self._spec = (learner_cls, config, module_factory, obs_space, act_space)
        if self.n == 0:
            self.local = learner_cls(config, module_factory, obs_space, act_space)
        else:
            self._start()

    def _start(self):
        from ...core import api as core
        from ...core.actor import ActorClass

        learner_cls, config, module_factory, obs_space, act_space = self._spec
        A = ActorClass(_LearnerActor, {})
        port = _free_port()
        gpus = config.get("num_gpus_per_learner", 1) if core.cluster_resources().get("GPU", 0) > 0 else 0
        self.actors = [A.options(num_cpus=config.get("num_cpus_per_learner", 1), num_gpus=gpus,
                                 runtime_env={"env_vars": {"CAAMD_NOSET_ROCR_VISIBLE_DEVICES": "1",
                                                           "HSA_ENABLE_IPC_MODE_LEGACY": "0"}})
                       .remote(learner_cls, config, module_factory, obs_space, act_space, i, self.n,
                               "127.0.0.1", port) for i in range(self.n)]
        self._info = core.get([a.info.remote() for a in self.actors])

    def _restart(self, err):
        import logging

        from ...core import api as core

        if not self.restart_failed or self.num_restarts >= self.max_restarts:
            raise err
        self.num_restarts += 1
        logging.getLogger(__name__).warning("learner actor failed (%s); restarting the learner group "
                                            "(restart %d)", err, self.num_restarts)
        for a in self.actors:
            try:
                core.kill(a)
            except Exception:  # noqa: BLE001
                pass
        self._start()
        if self._last_state is not None:
            # an object-store ref (rank 0's snapshot) or a state dict (set_state)
            core.get([a.call.remote("set_state", self._last_state) for a in self.actors])

    def _run(self, make_calls):
        """``make_calls()`` -> refs, one per learner actor; their results. Restarts
        the group and retries when an actor died (also while making the calls)."""
        from ...core import api as core
        from ...exceptions import RayActorError, WorkerCrashedError

        while True:
            try:
                return core.get(make_calls())
            except (RayActorError, WorkerCrashedError) as e:
                self._restart(e)

    def _checkpoint(self, force: bool = False):
        """Snapshot the state to restore after a restart: rank 0 puts it into the
        object store and the group keeps the ref (first update, then every
        ``ckpt_every`` updates)."""
        if self.restart_failed and self.local is None:
            self._updates += 1
            if force or self._last_state is None or self._updates % self.ckpt_every == 0:
                from ...core import api as core

                # the RETURN value of rank 0's get_state: owned by this process (it
                # outlives the actor), kept as a ref and never deserialised here
                ref = self.actors[0].call.remote("get_state")
                core.wait([ref], num_returns=1)
                self._last_state = ref

    def _shard(self, batch, i):
        return _shard_nested(batch, i, self.n)

    def batch_transport(self, batch=None) -> str:
        t = self._spec[1].get("learner_batch_transport")
        flat = batch is None or all(not isinstance(v, dict) for v in batch.values())
        if t == "ipc" and not flat:
            t = "shm"  # multi-module (nested) batches: shared-memory hand-off
        if t:
            return t
        one_node = len({i["node"] for i in self._info}) == 1
        return "ipc" if (flat and one_node and self._info and all(i["cuda"] for i in self._info)) else "shm"

    def update(self, batch, minibatch_size=None, num_epochs=1, shuffle=True):
        if self.local is not None:
            return self.local.update(batch, minibatch_size, num_epochs, shuffle)
        from ...core import api as core

        mbs = None if minibatch_size is None else max(1, minibatch_size // self.n)
        t = self.batch_transport(batch)
        if t == "pickle":
            res = self._run(lambda: [a.call.remote("update", self._shard(batch, i), mbs, num_epochs, shuffle)
                                     for i, a in enumerate(self.actors)])
        else:
            bref = core.put(batch)  # one host copy for every learner

            def calls():
                if t == "ipc":
                    staged = core.get(self.actors[0].stage_ipc.remote(bref))[0]
                    return [a.update_shard.remote(None if i == 0 else staged, i, self.n, mbs, num_epochs, shuffle)
                            for i, a in enumerate(self.actors)]
                return [a.update_shard_host.remote(bref, i, self.n, mbs, num_epochs, shuffle)
                        for i, a in enumerate(self.actors)]

            res = self._run(calls)
            if t == "ipc":
                try:  # every peer's update_shard has returned: rank 0 may free the batch
                    self.actors[0].release_staged.remote()
                except Exception:
                    pass
        self._checkpoint()
        return _mean_nested(res)

    def call(self, method, *args, **kwargs):
        """Run a learner method on the local learner / all learner actors (rank 0's result)."""
        if self.local is not None:
            return getattr(self.local, method)(*args, **kwargs)
        out = self._run(lambda: [a.call.remote(method, *args, **kwargs) for a in self.actors])[0]
        if method.startswith(("learn", "update", "train")):
            self._checkpoint()
        return out

    def get_module_state(self, on_device: bool = False):
        if on_device and self.local is not None:
            return self.local.get_module_state(on_device=True)
        return self.call("get_module_state")

    def get_state(self):
        return self.call("get_state")

    def set_state(self, st):
        if self.local is not None:
            return self.local.set_state(st)
        self._run(lambda: [a.call.remote("set_state", st) for a in self.actors])
        if self.restart_failed:
            self._last_state = st
            self._updates = 0

    def stop(self):
        from ...core import api as core

        for a in self.actors:
            try:
                core.kill(a)
            except Exception:
                pass
