"""``serve`` command line (reference: python/ray/serve/scripts.py:320 — ``deploy``,
``run``, ``build``, ``config``, ``status``, ``shutdown``, ``start``).

    python -m cluster_anywhere_amd serve run app_module:app        # or a config.yaml
    python -m cluster_anywhere_amd serve build app_module:app -o serve.yaml
    python -m cluster_anywhere_amd serve deploy serve.yaml --address 127.0.0.1:6380
    python -m cluster_anywhere_amd serve status | config | shutdown -y

``deploy`` / ``status`` / ``config`` / ``shutdown`` attach to a running cluster
(``--address``, default ``auto``); ``run`` starts a local cluster when none is
running and, unless ``--non-blocking``, serves until interrupted.
"""
from __future__ import annotations

import argparse
import sys
import time

import yaml


def _init(address, must_exist=True):
    import cluster_anywhere_amd as ray

    if ray.is_initialized():
        return ray
    try:
        ray.init(address=address or "auto", include_dashboard=False)
    except Exception:
        if must_exist:
            raise
        ray.init(include_dashboard=False)
    return ray


def _load_config(path):
    from .schema import ServeDeploySchema

    with open(path) as f:
        return ServeDeploySchema.model_validate(yaml.safe_load(f))


def _is_http(address) -> bool:
    return bool(address) and str(address).startswith(("http://", "https://"))


def _rest(address: str, method: str, body=None):
    """The dashboard's Serve REST API (``/api/serve/applications/``)."""
    import json
    import urllib.error
    import urllib.request

    data = None if body is None else json.dumps(body).encode()
    req = urllib.request.Request(address.rstrip("/") + "/api/serve/applications/", data=data, method=method,
                                 headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=600) as r:
            raw = r.read()
    except urllib.error.HTTPError as e:
        raise SystemExit(f"Serve REST {method} failed ({e.code}): {e.read().decode(errors='replace')[:2000]}")
    return json.loads(raw) if raw else {}


def cmd_deploy(a):
    from .schema import deploy_config

    cfg = _load_config(a.config_file)
    if _is_http(a.address):  # through the dashboard (reference: serve deploy --address http://...)
        _rest(a.address, "PUT", cfg.model_dump(mode="json"))
        print(f"Sent deploy request for {len(cfg.applications)} application(s): "
              + ", ".join(x.name for x in cfg.applications))
        return 0
    _init(a.address)
    deploy_config(cfg)
    print(f"Sent deploy request for {len(cfg.applications)} application(s): "
          + ", ".join(x.name for x in cfg.applications))
    return 0


def cmd_run(a):
    from . import api
    from .schema import ServeApplicationSchema, ServeDeploySchema, deploy_config

    target = a.config_or_import_path
    if target.endswith((".yaml", ".yml")):
        cfg = _load_config(target)
    else:
        args = dict(kv.split("=", 1) for kv in a.arguments)
        cfg = ServeDeploySchema(applications=[ServeApplicationSchema(
            name=a.name, route_prefix=a.route_prefix, import_path=target, args=args)])
    _init(a.address, must_exist=False)
    deploy_config(cfg)
    print(f"Deployed {', '.join(x.name for x in cfg.applications)}; HTTP port {api.http_port()}", flush=True)
    if a.non_blocking:
        return 0
    try:
        while True:
            time.sleep(1)
    except KeyboardInterrupt:
        pass
    api.shutdown()
    return 0


def cmd_build(a):
    from .schema import build_config

    cfg = build_config(a.import_paths, app_names=a.app_names)
    text = yaml.safe_dump(cfg, sort_keys=False)
    if a.output_path:
        with open(a.output_path, "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text)
    return 0


def _status_dict():
    from . import api

    st = api.status()
    apps = {}
    for n, s in st.applications.items():
        apps[n] = {"status": s.status, "route_prefix": s.route_prefix,
                   "deployments": {dn: {"status": d.status, "replica_states": dict(d.replica_states),
                                        "message": d.message} for dn, d in s.deployments.items()}}
    return {"proxies": dict(st.proxies), "applications": apps}


def cmd_status(a):
    if _is_http(a.address):
        d = _rest(a.address, "GET")
        st = {"proxies": {k: v.get("status") for k, v in (d.get("proxies") or {}).items()},
              "applications": {n: {"status": x["status"], "route_prefix": x["route_prefix"],
                                   "deployments": {dn: {"status": dd["status"],
                                                        "replica_states": dd.get("replica_states", {})}
                                                   for dn, dd in x["deployments"].items()}}
                               for n, x in (d.get("applications") or {}).items()}}
        sys.stdout.write(yaml.safe_dump(st, sort_keys=False))
        return 0
    _init(a.address)
    sys.stdout.write(yaml.safe_dump(_status_dict(), sort_keys=False))
    return 0


def cmd_config(a):
    from ..core import api as core
    from . import api

    _init(a.address)
    ctl = api._get_controller(create=False)
    cfg = core.get(ctl.get_deploy_config.remote()) if ctl is not None else None
    if not cfg:
        print("No config has been deployed.")
        return 0
    apps = cfg.get("applications", [])
    if a.name:
        apps = [x for x in apps if x["name"] == a.name]
    for i, app in enumerate(apps):
        if i:
            sys.stdout.write("---\n")
        sys.stdout.write(yaml.safe_dump(app, sort_keys=False))
    return 0


def cmd_shutdown(a):
    from . import api

    if not a.yes:
        print("Pass -y/--yes to shut down Serve on the cluster.")
        return 1
    if _is_http(a.address):
        _rest(a.address, "DELETE")
        print("Serve shut down.")
        return 0
    _init(a.address)
    api.shutdown()
    print("Serve shut down.")
    return 0


def cmd_start(a):
    from . import api

    _init(a.address)
    grpc = {"port": a.grpc_port, "grpc_servicer_functions": a.grpc_servicer_functions} \
        if a.grpc_servicer_functions else None
    api.start(http_options={"host": a.http_host, "port": a.http_port}, grpc_options=grpc,
              proxy_location=a.proxy_location)
    print(f"Serve started: HTTP {api.http_port()}" + (f", gRPC {api.grpc_port()}" if grpc else ""))
    return 0


def add_parser(sub):
    p = sub.add_parser("serve", help="deploy and manage Serve applications")
    ssub = p.add_subparsers(dest="serve_cmd", required=True)
    x = ssub.add_parser("deploy")
    x.add_argument("config_file")
    x.add_argument("-a", "--address", default=None)
    x.set_defaults(fn=cmd_deploy)
    x = ssub.add_parser("run")
    x.add_argument("config_or_import_path")
    x.add_argument("arguments", nargs="*", help="key=value application-builder arguments")
    x.add_argument("-a", "--address", default=None)
    x.add_argument("--name", default="default")
    x.add_argument("--route-prefix", default="/")
    x.add_argument("--non-blocking", action="store_true")
    x.set_defaults(fn=cmd_run)
    x = ssub.add_parser("build")
    x.add_argument("import_paths", nargs="+")
    x.add_argument("-o", "--output-path", default=None)
    x.add_argument("--app-names", nargs="*", default=None)
    x.set_defaults(fn=cmd_build)
    for name, fn in (("status", cmd_status), ("config", cmd_config)):
        x = ssub.add_parser(name)
        x.add_argument("-a", "--address", default=None)
        x.add_argument("--name", default=None)
        x.set_defaults(fn=fn)
    x = ssub.add_parser("shutdown")
    x.add_argument("-a", "--address", default=None)
    x.add_argument("-y", "--yes", action="store_true")
    x.set_defaults(fn=cmd_shutdown)
    x = ssub.add_parser("start")
    x.add_argument("-a", "--address", default=None)
    x.add_argument("--http-host", default="127.0.0.1")
    x.add_argument("--http-port", type=int, default=8000)
    x.add_argument("--grpc-port", type=int, default=9000)
    x.add_argument("--grpc-servicer-functions", nargs="*", default=[])
    x.add_argument("--proxy-location", default="HeadOnly")
    x.set_defaults(fn=cmd_start)
    return p


def main(argv=None):
    ap = argparse.ArgumentParser(prog="serve")
    sub = ap.add_subparsers(dest="cmd", required=True)
    add_parser(sub)
    a = ap.parse_args(["serve"] + list(argv if argv is not None else sys.argv[1:]))
    return a.fn(a) or 0


if __name__ == "__main__":
    sys.exit(main())
