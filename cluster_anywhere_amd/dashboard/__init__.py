"""Dashboard HTTP server: cluster/state REST endpoints, job submission API and
Prometheus metrics (reference: python/ray/dashboard/ — head.py,
modules/job/job_head.py (/api/jobs/), modules/state/state_head.py
(/api/v0/...), modules/reporter (metrics export)).

Runs as a uvicorn thread inside the head process (``core/head_main.py``) or the
driver that hosts the head (``init(include_dashboard=True)``)."""
from __future__ import annotations

import json
import os
import socket
import threading
import time
from typing import Any, Callable, Dict, Optional

from .job_manager import JobManager

_server = None


def _state_fn(head=None) -> Callable[[str], Any]:
    if head is not None:
        return lambda what, arg=None: head.call_sync(lambda: head.state(what, arg))
    from ..core.api import _state

    return lambda what, arg=None: _state(what, arg)


def render_prometheus(state: Callable) -> str:
    lines = []
    nodes = state("nodes")
    lines += ["# HELP ray_cluster_active_nodes Alive nodes", "# TYPE ray_cluster_active_nodes gauge",
              f"ray_cluster_active_nodes {sum(1 for n in nodes if n['Alive'])}"]
    total, avail = state("cluster_resources"), state("available_resources")
    lines += ["# HELP ray_resources Cluster resources", "# TYPE ray_resources gauge"]
    for k, v in sorted(total.items()):
        if k.startswith("node:"):
            continue
        lines.append(f'ray_resources{{Name="{k}",State="TOTAL"}} {v}')
        lines.append(f'ray_resources{{Name="{k}",State="AVAILABLE"}} {avail.get(k, 0.0)}')
    counts: Dict[str, int] = {}
    for t in state("tasks"):
        counts[t.get("state", "?")] = counts.get(t.get("state", "?"), 0) + 1
    lines += ["# HELP ray_tasks Tasks by state", "# TYPE ray_tasks gauge"]
    lines += [f'ray_tasks{{State="{k}"}} {v}' for k, v in sorted(counts.items())]
    acounts: Dict[str, int] = {}
    for a in state("actors"):
        acounts[a.get("state", "?")] = acounts.get(a.get("state", "?"), 0) + 1
    lines += ["# HELP ray_actors Actors by state", "# TYPE ray_actors gauge"]
    lines += [f'ray_actors{{State="{k}"}} {v}' for k, v in sorted(acounts.items())]
    st = state("store")
    if isinstance(st, dict):
        lines += ["# TYPE ray_object_store_memory gauge",
                  f'ray_object_store_memory{{Type="USED"}} {st.get("used", 0)}',
                  f'ray_object_store_memory{{Type="CAPACITY"}} {st.get("capacity", 0)}']
    from .reporter import prometheus_lines

    lines += prometheus_lines(nodes)
    for name, m in sorted(state("metrics").items()):
        kind = m["kind"]
        lines.append(f"# HELP {name} {m['desc']}")
        lines.append(f"# TYPE {name} {kind}")
        for key, val in m["series"].items():
            lab = ",".join(f'{k}="{v}"' for k, v in zip(m["tag_keys"], key))
            if kind != "histogram":
                lines.append(f"{name}{{{lab}}} {val}" if lab else f"{name} {val}")
                continue
            buckets, ssum, cnt = val
            acc = 0
            for b, c in zip(m["boundaries"] + [float("inf")], buckets):
                acc += c
                le = "+Inf" if b == float("inf") else repr(float(b))
                sep = "," if lab else ""
                lines.append(f'{name}_bucket{{{lab}{sep}le="{le}"}} {acc}')
            lines.append(f"{name}_sum{{{lab}}} {ssum}")
            lines.append(f"{name}_count{{{lab}}} {cnt}")
    return "\n".join(lines) + "\n"


def build_app(state: Callable, jobs: JobManager, session_dir: Optional[str] = None, serve_agent=None):
    from starlette.applications import Starlette
    from starlette.requests import Request
    from starlette.responses import HTMLResponse, JSONResponse, PlainTextResponse, Response
    from starlette.routing import Route

    def j(x, status=200):
        return JSONResponse(json.loads(json.dumps(x, default=str)), status_code=status)

    async def version(req):
        from .. import __version__

        return j({"version": __version__, "ray_version": "2.42.0-mi355x", "session_name": "caamd"})

    async def cluster_status(req):
        return j({"result": True, "data": {"clusterStatus": {
            "total": state("cluster_resources"), "available": state("available_resources"),
            "nodes": state("nodes")}}})

    def lister(what):
        async def h(req):
            rows = state(what)
            return j({"result": True, "data": {"result": {"result": rows, "total": len(rows)}}})

        return h

    async def metrics(req):
        return PlainTextResponse(render_prometheus(state), media_type="text/plain; version=0.0.4")

    async def submit(req: Request):
        body = await req.json()
        try:
            sid = jobs.submit(body["entrypoint"], body.get("submission_id") or body.get("job_id"),
                              body.get("runtime_env"), body.get("metadata"),
                              body.get("entrypoint_num_cpus"), body.get("entrypoint_num_gpus"))
        except ValueError as e:
            return j({"error": str(e)}, 400)
        return j({"submission_id": sid, "job_id": sid})

    async def list_jobs(req):
        return j(jobs.list())

    async def job_info(req):
        info = jobs.info(req.path_params["sid"])
        return j(info) if info else j({"error": "not found"}, 404)

    async def job_logs(req):
        logs = jobs.logs(req.path_params["sid"])
        return j({"logs": logs}) if logs is not None else j({"error": "not found"}, 404)

    async def job_stop(req):
        return j({"stopped": jobs.stop(req.path_params["sid"])})

    async def job_delete(req):
        return j({"deleted": jobs.delete(req.path_params["sid"])})

    async def timeline(req):
        from ..core.api import _timeline_events

        return j(_timeline_events(state("events")))

    async def ui(req):
        # single-page UI over the REST endpoints below (reference: dashboard/client)
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ui.html")) as f:
            return HTMLResponse(f.read())

    def _log_dir():
        return session_dir if session_dir and os.path.isdir(session_dir) else None

    async def list_logs(req):
        d = _log_dir()
        files = []
        if d:
            for root, _, names in os.walk(d):
                for n in sorted(names):
                    if n.endswith((".log", ".out", ".err")):
                        p = os.path.join(root, n)
                        files.append({"name": os.path.relpath(p, d), "size": os.path.getsize(p)})
        return j({"files": files})

    async def log_file(req):
        d = _log_dir()
        name = req.query_params.get("name", "")
        lines = int(req.query_params.get("lines", "1000"))
        if not d or not name:
            return j({"error": "not found"}, 404)
        p = os.path.realpath(os.path.join(d, name))
        if not p.startswith(os.path.realpath(d) + os.sep) or not os.path.isfile(p):
            return j({"error": "not found"}, 404)  # no escaping the session directory
        with open(p, errors="replace") as f:
            text = "".join(f.readlines()[-lines:])
        return j({"name": name, "text": text})

    async def serve_apps(req: Request):
        """Serve REST API (dashboard/serve_agent.py): PUT deploys a ServeDeploySchema,
        GET returns the instance details, DELETE shuts Serve down."""
        import asyncio

        if serve_agent is None:
            return j({"error": "Serve REST API unavailable (no cluster address)"}, 503)
        body = None
        if req.method == "PUT":
            try:
                body = await req.json()
            except Exception:
                return j({"error": "body must be a ServeDeploySchema JSON object"}, 400)
        op = {"GET": "get", "PUT": "put", "DELETE": "delete"}[req.method]
        r = await asyncio.get_running_loop().run_in_executor(None, serve_agent.request, op, body)
        if not r.get("ok"):
            return j({"error": r.get("error"), "trace": r.get("trace")}, r.get("status", 500))
        return j(r.get("body") or {}) if op == "get" else Response(status_code=200)

    routes = [Route("/", ui),
              Route("/api/serve/applications/", serve_apps, methods=["GET", "PUT", "DELETE"]), Route("/ui", ui), Route("/api/v0/logs", list_logs),
              Route("/api/v0/logs/file", log_file),
              Route("/api/version", version), Route("/api/cluster_status", cluster_status),
              Route("/api/v0/nodes", lister("nodes")), Route("/api/v0/actors", lister("actors")),
              Route("/api/v0/tasks", lister("tasks")), Route("/api/v0/objects", lister("objects")),
              Route("/api/v0/workers", lister("workers")),
              Route("/api/v0/placement_groups", lister("placement_groups")),
              Route("/api/timeline", timeline), Route("/metrics", metrics),
              Route("/api/jobs/", submit, methods=["POST"]), Route("/api/jobs/", list_jobs, methods=["GET"]),
              Route("/api/jobs/{sid}", job_info, methods=["GET"]),
              Route("/api/jobs/{sid}", job_delete, methods=["DELETE"]),
              Route("/api/jobs/{sid}/logs", job_logs), Route("/api/jobs/{sid}/stop", job_stop, methods=["POST"])]
    return Starlette(routes=routes)


def start_dashboard(host: str = "127.0.0.1", port: int = 8265, head=None, control_address: Optional[str] = None,
                    session_dir: Optional[str] = None) -> str:
    """Start the dashboard thread; returns its URL."""
    global _server
    import uvicorn

    if port == 0:
        s = socket.socket()
        s.bind((host, 0))
        port = s.getsockname()[1]
        s.close()
    state = _state_fn(head)
    if control_address is None:
        control_address = head.sock_path if head is not None else os.environ.get("CAAMD_ADDRESS", "auto")
    if session_dir is None:
        session_dir = head.session_dir if head is not None else "/tmp/caamd"
    jobs = JobManager(control_address, os.path.join(session_dir, "jobs"))
    from .serve_agent import ServeAgentClient

    serve_agent = ServeAgentClient(control_address) if control_address and control_address != "auto" else None
    app = build_app(state, jobs, session_dir, serve_agent)
    cfg = uvicorn.Config(app, host=host, port=port, log_level="warning", lifespan="off", access_log=False)
    server = uvicorn.Server(cfg)
    t = threading.Thread(target=server.run, name="caamd-dashboard", daemon=True)
    t.start()
    deadline = time.time() + 30
    while not server.started and time.time() < deadline:
        time.sleep(0.02)
    _server = (server, jobs, serve_agent)
    return f"http://{host}:{port}"


def stop_dashboard():
    global _server
    if _server is not None:
        _server[0].should_exit = True
        _server[1].stop_all()
        if _server[2] is not None:
            _server[2].close()
        _server = None
