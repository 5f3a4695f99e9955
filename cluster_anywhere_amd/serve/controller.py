"""Serve controller actor (reference: python/ray/serve/_private/controller.py,
deployment_state.py, application_state.py, autoscaling_state.py).

A named, detached, threaded actor that owns every application's deployments
and replicas. A reconcile thread (every 100 ms):
  * starts replicas up to the target count and promotes them to RUNNING once
    their ``ready()`` completes,
  * drains + kills surplus replicas (graceful ``prepare_for_shutdown``),
  * health-checks RUNNING replicas and replaces dead ones,
  * runs the autoscaling policy from replica-reported ongoing requests.
Handles and the HTTP proxy read ``(version, replicas)`` snapshots; the version
bumps on every membership change so clients refresh only when needed.

Fault tolerance (reference: controller.py:123-124, 509 ``_recover_state_from_
checkpoint``; api.py:101 ``max_restarts=-1``): the controller is restarted by the
core on death, and every application / deployment change is checkpointed to the
internal KV (namespace ``serve``). Replicas and proxies are detached named
actors, so they outlive the controller and keep serving; a restarted controller
reads the checkpoint, re-attaches to the replicas by name (promoting each after a
``ready()`` round trip) and starts replacements only for the ones that are gone."""
from __future__ import annotations

import threading
import time
import traceback
import uuid
from typing import Any, Dict, List, Optional

from ..core import api as core
from .config import DeploymentConfig

CONTROLLER_NAME = "SERVE_CONTROLLER"
NAMESPACE = "serve"
CHECKPOINT_KEY = b"serve:controller_checkpoint"
REPLICA_PREFIX = "SERVE_REPLICA::"
REPLICA_PG_PREFIX = "SERVE_REPLICA_PG::"


class _ReplicaState:
    def __init__(self, tag, handle):
        self.tag = tag
        self.handle = handle
        self.state = "STARTING"
        self.ready_ref = handle.ready.remote()
        self.health_ref = None
        self.health_sent = 0.0
        self.metrics = {"ongoing": 0, "models": []}
        self.metrics_ref = None
        self.started = time.time()
        self.stop_ref = None
        self.node_id: Optional[str] = None  # known at start (max_replicas_per_node) or from metrics
        self.pg = None  # per-replica placement group (placement_group_bundles)


class _DeploymentState:
    def __init__(self, app: str, name: str, target, init_args, init_kwargs, config: DeploymentConfig):
        self.app = app
        self.name = name
        self.target = target
        self.init_args = init_args
        self.init_kwargs = init_kwargs
        self.config = config
        self.target_replicas = config.initial_replicas()
        self.replicas: List[_ReplicaState] = []
        self.version = 0
        self.counter = 0
        self.error: Optional[str] = None
        self.scale_since: Optional[float] = None
        self.scale_dir = 0
        self.metric_hist: List[tuple] = []
        self.deleting = False

    def running(self):
        return [r for r in self.replicas if r.state == "RUNNING"]

    def status(self):
        if self.error:
            return "DEPLOY_FAILED"
        run = len(self.running())
        if run == self.target_replicas and all(r.state == "RUNNING" for r in self.replicas):
            return "HEALTHY"
        return "UPDATING" if run < self.target_replicas else "DOWNSCALING"


class ServeController:
    def __init__(self, http_options=None):
        self.apps: Dict[str, Dict[str, Any]] = {}  # name -> {route_prefix, ingress, deployments{}}
        self.lock = threading.RLock()
        self.http_options = http_options
        self.proxy = None
        self.proxy_port = None
        self._orphans: List[_DeploymentState] = []
        self._ckpt_sig = None
        self.recovered = False
        self.alive = True
        self._recover_from_checkpoint()
        self.thread = threading.Thread(target=self._loop, name="serve-reconcile", daemon=True)
        self.thread.start()

    # --------------------------------------------------------- checkpointing
    def _signature(self):
        return (tuple(sorted((n, dn, st.version, st.target_replicas, tuple(r.tag for r in st.replicas))
                             for n, a in self.apps.items() for dn, st in a["deployments"].items())),
                self.proxy_port, getattr(self, "grpc_port", None), repr(getattr(self, "deploy_config", None)))

    def _checkpoint(self, force: bool = False):
        """Write the controller state to the internal KV when it changed."""
        from ..core import serialization
        from ..experimental import internal_kv

        with self.lock:
            sig = self._signature()
            if not force and sig == self._ckpt_sig:
                return
            state = {"apps": {}, "proxy_port": self.proxy_port, "grpc_port": getattr(self, "grpc_port", None),
                     "deploy_config": getattr(self, "deploy_config", None)}
            for n, a in self.apps.items():
                deps = {}
                for dn, st in a["deployments"].items():
                    deps[dn] = {"target": st.target, "args": st.init_args, "kwargs": st.init_kwargs,
                                "config": st.config, "target_replicas": st.target_replicas, "counter": st.counter,
                                "replicas": [r.tag for r in st.replicas if r.state in ("STARTING", "RUNNING")]}
                state["apps"][n] = {"route_prefix": a["route_prefix"], "ingress": a["ingress"],
                                    "created": a.get("created", time.time()), "deployments": deps}
            blob = serialization.dumps_function(state)
            self._ckpt_sig = sig
        internal_kv._internal_kv_put(CHECKPOINT_KEY, blob, namespace=NAMESPACE)

    def _recover_from_checkpoint(self):
        from ..core import serialization
        from ..experimental import internal_kv

        try:
            blob = internal_kv._internal_kv_get(CHECKPOINT_KEY, namespace=NAMESPACE)
        except Exception:
            blob = None
        if not blob:
            return
        state = serialization.loads_function(blob)
        for n, a in state["apps"].items():
            deps = {}
            for dn, d in a["deployments"].items():
                st = _DeploymentState(n, dn, d["target"], d["args"], d["kwargs"], d["config"])
                st.target_replicas = d["target_replicas"]
                st.counter = d["counter"]
                for tag in d["replicas"]:
                    try:
                        h = core.get_actor(REPLICA_PREFIX + tag, namespace=NAMESPACE)
                    except ValueError:
                        continue  # gone with the old controller's node / killed: replaced below
                    r = _ReplicaState(tag, h)  # STARTING until ready() answers
                    if d["config"].placement_group_bundles:
                        try:
                            from ..util.placement_group import get_placement_group

                            r.pg = get_placement_group(REPLICA_PG_PREFIX + tag)
                        except Exception:
                            pass
                    st.replicas.append(r)
                deps[dn] = st
            self.apps[n] = {"route_prefix": a["route_prefix"], "ingress": a["ingress"],
                            "deployments": deps, "created": a["created"]}
        for attr, name, port_key in (("proxy", "SERVE_PROXY", "proxy_port"),
                                     ("grpc_proxy", "SERVE_GRPC_PROXY", "grpc_port")):
            try:
                setattr(self, attr, core.get_actor(name, namespace=NAMESPACE))
                setattr(self, "proxy_port" if attr == "proxy" else "grpc_port", state.get(port_key))
            except ValueError:
                pass
        self.deploy_config = state.get("deploy_config")
        self.recovered = True

    def is_recovered(self):
        return self.recovered

    def pid(self):
        import os

        return os.getpid()

    # ------------------------------------------------------------- public API
    def deploy_application(self, name: str, route_prefix: Optional[str], ingress: str,
                           deployments: List[Dict]):
        with self.lock:
            old = self.apps.get(name)
            new_deps = {}
            for d in deployments:
                cfg: DeploymentConfig = d["config"]
                prev = old["deployments"].get(d["name"]) if old else None
                if prev is not None and prev.config.version is not None and prev.config.version == cfg.version \
                        and prev.target is not None:
                    # same code version: in-place reconfigure / rescale
                    if cfg.user_config != prev.config.user_config:
                        for r in prev.replicas:
                            r.handle.reconfigure.remote(cfg.user_config)
                    prev.config = cfg
                    if cfg.autoscaling_config is None:
                        prev.target_replicas = cfg.initial_replicas()
                    new_deps[d["name"]] = prev
                    continue
                if prev is not None:
                    prev.deleting = True  # old replicas drain below
                    self._orphans.append(prev)
                new_deps[d["name"]] = _DeploymentState(name, d["name"], d["target"], d["args"], d["kwargs"], cfg)
            if old:
                for dn, st in old["deployments"].items():
                    if dn not in new_deps:
                        st.deleting = True
                        self._orphans.append(st)
            self.apps[name] = {"route_prefix": route_prefix, "ingress": ingress, "deployments": new_deps,
                               "created": time.time()}
        self._checkpoint(force=True)
        return True

    def delete_application(self, name: str):
        with self.lock:
            app = self.apps.pop(name, None)
            if app:
                for st in app["deployments"].values():
                    st.deleting = True
                    self._orphans.append(st)
        self._checkpoint(force=True)
        return True

    def get_replicas(self, app: str, deployment: str):
        with self.lock:
            a = self.apps.get(app)
            if a is None or deployment not in a["deployments"]:
                return None
            st = a["deployments"][deployment]
            return (st.version, [(r.tag, r.handle, list(r.metrics.get("models", []))) for r in st.running()],
                    st.config.max_ongoing_requests, st.config.max_queued_requests)

    def get_routes(self):
        with self.lock:
            return {a["route_prefix"]: (name, a["ingress"]) for name, a in self.apps.items()
                    if a["route_prefix"] is not None}

    def get_ingress(self, app: str):
        with self.lock:
            a = self.apps.get(app)
            return a["ingress"] if a else None

    def list_apps(self):
        with self.lock:
            return list(self.apps.keys())

    def status(self):
        with self.lock:
            out = {}
            for name, a in self.apps.items():
                deps = {}
                for dn, st in a["deployments"].items():
                    deps[dn] = {"status": st.status(), "target_replicas": st.target_replicas,
                                "running_replicas": len(st.running()),
                                "replica_states": {r.tag: r.state for r in st.replicas},
                                "replica_nodes": {r.tag: r.node_id for r in st.replicas},
                                "message": st.error or getattr(st, "pending_reason", None) or ""}
                sts = [d["status"] for d in deps.values()]
                if any(s == "DEPLOY_FAILED" for s in sts):
                    ast = "DEPLOY_FAILED"
                elif all(s == "HEALTHY" for s in sts):
                    ast = "RUNNING"
                else:
                    ast = "DEPLOYING"
                out[name] = {"status": ast, "route_prefix": a["route_prefix"], "deployments": deps}
            return out

    def set_proxy(self, proxy, port):
        self.proxy, self.proxy_port = proxy, port
        self._checkpoint(force=True)
        return True

    def get_proxy(self):
        return self.proxy, self.proxy_port

    def set_grpc_proxy(self, proxy, port):
        self.grpc_proxy, self.grpc_port = proxy, port
        self._checkpoint(force=True)
        return True

    def get_grpc_proxy(self):
        return getattr(self, "grpc_proxy", None), getattr(self, "grpc_port", None)

    def set_deploy_config(self, cfg: Optional[dict]):
        """Last config applied by ``serve deploy`` (returned by ``serve config``)."""
        self.deploy_config = cfg
        self._checkpoint(force=True)
        return True

    def get_deploy_config(self):
        return getattr(self, "deploy_config", None)

    def record_handle_metrics(self, app, deployment, queued, router_id: str = ""):
        """Requests waiting in a handle router's queue (no replica slot free): counted
        by the autoscaler on top of the replicas' ongoing requests (reference:
        autoscaling_state.py, handle queued metrics)."""
        with self.lock:
            a = self.apps.get(app)
            if a and deployment in a["deployments"]:
                st = a["deployments"][deployment]
                q = getattr(st, "router_queued", None)
                if q is None:
                    q = st.router_queued = {}
                q[router_id] = (int(queued), time.time())
        return True

    def shutdown(self):
        with self.lock:
            for name in list(self.apps):
                self.delete_application(name)
        deadline = time.time() + 10
        while time.time() < deadline:
            with self.lock:
                if not self._orphans:
                    break
            time.sleep(0.05)
        for attr in ("proxy", "grpc_proxy"):
            p = getattr(self, attr, None)
            if p is not None:
                try:
                    core.kill(p)
                except Exception:
                    pass
                setattr(self, attr, None)
        self.alive = False
        try:
            from ..experimental import internal_kv

            internal_kv._internal_kv_del(CHECKPOINT_KEY, namespace=NAMESPACE)
        except Exception:
            pass
        return True

    # --------------------------------------------------------------- reconcile
    def _loop(self):
        while self.alive:
            try:
                with self.lock:
                    for a in list(self.apps.values()):
                        for st in a["deployments"].values():
                            self._reconcile(st)
                    for st in list(self._orphans):
                        self._reconcile(st)
                        if not st.replicas:
                            self._orphans.remove(st)
                if self.alive:
                    self._checkpoint()
            except Exception:  # keep the control loop alive
                traceback.print_exc()
            time.sleep(0.1)

    def _pick_node(self, st: _DeploymentState, opts: Dict[str, Any]) -> Optional[str]:
        """``max_replicas_per_node``: an alive node holding fewer than that many live
        replicas of this deployment whose free resources fit the replica actor (the
        emptiest such node first), or None (the replica waits; reference:
        deployment_scheduler.py:143-176 -- there an implicit per-node resource of 1.0
        of which each replica takes 1 / max_replicas_per_node)."""
        cap = st.config.max_replicas_per_node
        count: Dict[str, int] = {}
        for r in st.replicas:
            if r.state in ("STARTING", "RUNNING") and r.node_id:
                count[r.node_id] = count.get(r.node_id, 0) + 1
        need = {"CPU": float(opts.get("num_cpus", 0) or 0), "GPU": float(opts.get("num_gpus", 0) or 0)}
        for k, v in (opts.get("resources") or {}).items():
            need[k] = float(v)
        try:
            avail = core.available_resources_per_node()
        except Exception:
            avail = {}
        best = None
        for n in core.nodes():
            if not n.get("Alive", True):
                continue
            nid = n["NodeID"]
            c = count.get(nid, 0)
            if c >= cap:
                continue
            free = avail.get(nid, n.get("Resources", {}))
            if any(v > 0 and free.get(k, 0.0) + 1e-9 < v for k, v in need.items()):
                continue
            if best is None or c < best[0]:
                best = (c, nid)
        return best[1] if best else None

    def _start_replica(self, st: _DeploymentState):
        from ..core.actor import ActorClass
        from .replica import ServeReplica

        cfg = st.config
        tag = f"{st.app}#{st.name}#{uuid.uuid4().hex[:6]}"
        opts = dict(cfg.ray_actor_options or {})
        node = pg = None
        if cfg.max_replicas_per_node:
            node = self._pick_node(st, opts)
            if node is None:
                st.pending_reason = (f"no node can take another replica (max_replicas_per_node="
                                     f"{cfg.max_replicas_per_node})")
                return False
            from ..util.scheduling_strategies import NodeAffinitySchedulingStrategy

            opts["scheduling_strategy"] = NodeAffinitySchedulingStrategy(node, soft=False)
        elif cfg.placement_group_bundles:
            # one gang per replica, the replica actor in bundle 0, its tasks / child
            # actors (e.g. the ranks of a multi-GPU model) in the PG's other bundles
            # (reference: deployment_scheduler.py:143-176, replica.py placement group)
            from ..util.placement_group import placement_group
            from ..util.scheduling_strategies import PlacementGroupSchedulingStrategy

            pg = placement_group(cfg.placement_group_bundles, strategy=cfg.placement_group_strategy or "PACK",
                                 name=REPLICA_PG_PREFIX + tag, lifetime="detached")
            opts["scheduling_strategy"] = PlacementGroupSchedulingStrategy(
                pg, placement_group_bundle_index=0, placement_group_capture_child_tasks=True)
        st.pending_reason = None
        st.counter += 1
        opts.setdefault("num_cpus", 0)
        opts["max_concurrency"] = max(16, st.config.max_ongoing_requests * 2)
        opts["max_restarts"] = 0
        # detached + named: replicas outlive a controller crash and the restarted
        # controller finds them again by name (_recover_from_checkpoint)
        opts["name"] = REPLICA_PREFIX + tag
        opts["namespace"] = NAMESPACE
        opts["lifetime"] = "detached"
        Replica = ActorClass(ServeReplica, {})
        h = Replica.options(**opts).remote(st.app, st.name, tag, st.target, st.init_args, st.init_kwargs,
                                           st.config.user_config, st.config.max_ongoing_requests)
        r = _ReplicaState(tag, h)
        r.node_id, r.pg = node, pg
        st.replicas.append(r)
        return True

    def _stop_replica(self, st: _DeploymentState, r: _ReplicaState):
        if r.state != "STOPPING":
            r.state = "STOPPING"
            st.version += 1
            r.stop_ref = r.handle.prepare_for_shutdown.remote(st.config.graceful_shutdown_timeout_s,
                                                             st.config.graceful_shutdown_wait_loop_s)
            r.stop_deadline = time.time() + st.config.graceful_shutdown_timeout_s + 2

    def _reconcile(self, st: _DeploymentState):
        from ..exceptions import RayActorError, RayError

        now = time.time()
        # promote / fail starting replicas
        for r in list(st.replicas):
            if r.state == "STARTING":
                ready, _ = core.wait([r.ready_ref], timeout=0)
                if ready:
                    try:
                        core.get(r.ready_ref)
                        r.state = "RUNNING"
                        st.version += 1
                        st.error = None
                    except RayError as e:
                        st.error = f"replica {r.tag} failed to start: {e}"
                        st.replicas.remove(r)
                        self._kill(r)
            elif r.state == "STOPPING":
                ready, _ = core.wait([r.stop_ref], timeout=0)
                if ready or now > r.stop_deadline:
                    st.replicas.remove(r)
                    self._kill(r)
        target = 0 if st.deleting else st.target_replicas
        live = [r for r in st.replicas if r.state in ("STARTING", "RUNNING")]
        if len(live) < target and not (st.error and len(live) == 0 and st.counter > 3 * max(1, target)):
            for _ in range(target - len(live)):
                if not self._start_replica(st):
                    break  # no node may take one now (max_replicas_per_node): retried next pass
        elif len(live) > target:
            # drain the least loaded / newest replicas first
            order = sorted(live, key=lambda r: (r.state == "RUNNING", -r.started))
            for r in order[: len(live) - target]:
                if r.state == "STARTING":
                    st.replicas.remove(r)
                    self._kill(r)
                else:
                    self._stop_replica(st, r)
        # health checks + metrics
        for r in st.running():
            if r.health_ref is not None:
                ready, _ = core.wait([r.health_ref], timeout=0)
                if ready:
                    try:
                        core.get(r.health_ref)
                        r.health_ref = None
                    except RayError:
                        r.state = "DEAD"
                elif now - r.health_sent > st.config.health_check_timeout_s:
                    r.state = "DEAD"
            elif now - r.health_sent > st.config.health_check_period_s:
                r.health_ref = r.handle.check_health.remote()
                r.health_sent = now
            if r.state == "DEAD":
                st.replicas.remove(r)
                st.version += 1
                self._kill(r)
                continue
            if r.metrics_ref is not None:
                ready, _ = core.wait([r.metrics_ref], timeout=0)
                if ready:
                    try:
                        m = core.get(r.metrics_ref)
                        models_changed = m.get("models") != r.metrics.get("models")
                        r.metrics = m
                        if m.get("node_id"):
                            r.node_id = m["node_id"]
                        if models_changed:
                            st.version += 1
                    except RayError:
                        pass
                    r.metrics_ref = None
            else:
                interval = st.config.autoscaling_config.metrics_interval_s if st.config.autoscaling_config else 0.5
                if now - r.metrics.get("_sent", 0) > interval:
                    r.metrics["_sent"] = now
                    r.metrics_ref = r.handle.get_metrics.remote()
        if st.config.autoscaling_config is not None and not st.deleting:
            self._autoscale(st, now)

    def _autoscale(self, st: _DeploymentState, now: float):
        cfg = st.config.autoscaling_config
        run = st.running()
        queued = sum(n for n, t in getattr(st, "router_queued", {}).values() if now - t < 2.0)
        total = sum(r.metrics.get("ongoing", 0) for r in run) + queued
        st.metric_hist.append((now, total))
        st.metric_hist = [(t, v) for t, v in st.metric_hist if now - t <= cfg.look_back_period_s]
        avg = sum(v for _, v in st.metric_hist) / max(1, len(st.metric_hist))
        desired = cfg.desired(avg, max(1, len(run)) if run else st.target_replicas)
        if desired == st.target_replicas:
            st.scale_since, st.scale_dir = None, 0
            return
        d = 1 if desired > st.target_replicas else -1
        if st.scale_dir != d:
            st.scale_dir, st.scale_since = d, now
            return
        delay = cfg.upscale_delay_s if d > 0 else cfg.downscale_delay_s
        if now - st.scale_since >= delay:
            st.target_replicas = desired
            st.scale_since, st.scale_dir = None, 0

    def _kill(self, r: _ReplicaState):
        try:
            core.kill(r.handle)
        except Exception:
            pass
        if r.pg is not None:
            try:
                from ..util.placement_group import remove_placement_group

                remove_placement_group(r.pg)
            except Exception:
                pass
            r.pg = None
