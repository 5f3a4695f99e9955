"""Serve REST API of the dashboard: ``PUT / GET / DELETE /api/serve/applications/``
(reference: ``python/ray/dashboard/modules/serve/serve_rest_api_impl.py:116-157``,
``python/ray/serve/_private/...sdk``).

The dashboard lives in the head process (or the driver that hosts the head), which
is not a driver of the cluster. Serve calls need one, so the first REST request
starts a helper DRIVER process (``python -m cluster_anywhere_amd.dashboard.serve_agent
<address>``) that attaches to the cluster and answers JSON-line requests on its
stdin / stdout; later requests reuse it (one at a time, under a lock). If it dies it
is restarted on the next request.

* ``PUT``: body = a ``ServeDeploySchema`` (declarative: applications absent from
  it are deleted), deployed with ``serve.schema.deploy_config``.
* ``GET``: ``ServeInstanceDetails``-shaped JSON -- ``applications: {name: {name,
  route_prefix, status, deployments: {...}, deployed_app_config}}``, ``http_options``,
  ``proxy_location``, ``proxies``, ``deploy_mode``.
* ``DELETE``: ``serve.shutdown()``.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time
from typing import Any, Dict, Optional


class ServeAgentClient:
    def __init__(self, address: str, timeout_s: float = 300.0):
        self.address = address
        self.timeout_s = timeout_s
        self.proc: Optional[subprocess.Popen] = None
        self.lock = threading.Lock()

    def _ensure(self):
        if self.proc is not None and self.proc.poll() is None:
            return
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ)
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        self.proc = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.dashboard.serve_agent", self.address],
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                     env=env, text=True, bufsize=1)

    def request(self, op: str, body: Optional[Dict] = None) -> Dict[str, Any]:
        with self.lock:
            for attempt in range(2):
                self._ensure()
                try:
                    self.proc.stdin.write(json.dumps({"op": op, "body": body}) + "\n")
                    self.proc.stdin.flush()
                    line = self._readline(self.timeout_s)
                except TimeoutError:
                    # a deploy hung in the agent: kill it (the next request starts a
                    # fresh one) instead of holding the lock for every later call
                    self.close()
                    return {"ok": False, "status": 504,
                            "error": f"serve agent did not answer within {self.timeout_s}s"}
                except (BrokenPipeError, OSError):
                    line = ""
                if line:
                    return json.loads(line)
                self.close()  # died: restart once
            return {"ok": False, "status": 503, "error": "serve agent unavailable"}

    def _readline(self, timeout_s: float) -> str:
        """One reply line, waiting at most ``timeout_s`` (select on the pipe)."""
        import select

        f = self.proc.stdout
        deadline = time.time() + timeout_s
        buf = ""
        fd = f.fileno()
        while True:
            left = deadline - time.time()
            if left <= 0:
                raise TimeoutError
            r, _, _ = select.select([fd], [], [], left)
            if not r:
                raise TimeoutError
            chunk = os.read(fd, 1 << 16).decode()
            if not chunk:
                return buf  # EOF: the agent died
            buf += chunk
            if "\n" in buf:  # one request in flight at a time: nothing follows the reply
                return buf.split("\n", 1)[0] + "\n"

    def close(self):
        p, self.proc = self.proc, None
        if p is not None:
            try:
                p.kill()
                p.wait(timeout=5)
            except Exception:
                pass


# ------------------------------------------------------------------ agent process
def _details() -> Dict[str, Any]:
    from ..core import api as core
    from ..serve import api

    from ..exceptions import RayActorError

    empty = {"controller_info": {}, "proxy_location": None, "http_options": None, "grpc_options": None,
             "proxies": {}, "deploy_mode": "UNSET", "applications": {}}
    ctl = api._get_controller(create=False)
    if ctl is None:
        return empty
    try:
        raw = core.get(ctl.status.remote(), timeout=30)
        cfg = core.get(ctl.get_deploy_config.remote(), timeout=30) or {}
        proxy, port = core.get(ctl.get_proxy.remote(), timeout=30)
    except RayActorError:  # the controller is gone or going (right after a DELETE): no Serve instance
        return empty
    app_cfg = {a["name"]: a for a in cfg.get("applications", [])}
    apps = {}
    for name, a in raw.items():
        apps[name] = {"name": name, "route_prefix": a["route_prefix"], "docs_path": None, "status": a["status"],
                      "message": "", "deployed_app_config": app_cfg.get(name),
                      "source": "declarative" if name in app_cfg else "imperative",
                      "deployments": {dn: {"name": dn, "status": d["status"], "message": d["message"],
                                           "target_num_replicas": d["target_replicas"],
                                           "running_replicas": d["running_replicas"],
                                           "replica_states": d["replica_states"]}
                                      for dn, d in a["deployments"].items()}}
    return {"controller_info": {"actor_name": "SERVE_CONTROLLER_ACTOR"},
            "proxy_location": cfg.get("proxy_location", "HeadOnly"),
            "http_options": cfg.get("http_options") or ({"host": "0.0.0.0", "port": port} if port else None),
            "grpc_options": cfg.get("grpc_options"),
            "proxies": {"head": {"status": "HEALTHY", "port": port}} if proxy is not None else {},
            "deploy_mode": "MULTI_APP" if cfg else "UNSET", "applications": apps}


def _handle(req: Dict[str, Any]) -> Dict[str, Any]:
    op = req.get("op")
    if op == "get":
        return {"ok": True, "status": 200, "body": _details()}
    if op == "put":
        from pydantic import ValidationError

        from ..serve.schema import ServeDeploySchema, deploy_config

        try:
            cfg = ServeDeploySchema.model_validate(req.get("body") or {})
        except ValidationError as e:
            return {"ok": False, "status": 400, "error": str(e)}
        deploy_config(cfg)
        return {"ok": True, "status": 200, "body": {"applications": [a.name for a in cfg.applications]}}
    if op == "delete":
        from ..serve import api

        api.shutdown()
        return {"ok": True, "status": 200, "body": {}}
    return {"ok": False, "status": 400, "error": f"unknown op {op!r}"}


def main(argv=None):
    import traceback

    import cluster_anywhere_amd as ray

    address = (argv or sys.argv[1:])[0]
    # responses go to the ORIGINAL stdout; everything else that prints (the runtime,
    # user code imported by a deploy) lands on stderr instead of corrupting the protocol
    out = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    ray.init(address=address, include_dashboard=False, log_to_driver=False)
    for line in sys.stdin:
        try:
            resp = _handle(json.loads(line))
        except Exception as e:  # report, keep serving
            resp = {"ok": False, "status": 500, "error": f"{type(e).__name__}: {e}",
                    "trace": traceback.format_exc(limit=5)}
        out.write(json.dumps(resp, default=str) + "\n")
        out.flush()


if __name__ == "__main__":
    main()
