"""Standalone head process (reference: ``ray start --head`` -> gcs_server +
raylet + dashboard processes; here one process: the Head event loop (GCS +
head-node raylet), the head node's object server, and the dashboard thread).

Writes ``<temp>/caamd/latest_address`` (TCP control address for node agents
and remote drivers) and ``<temp>/caamd/head.json`` (pid, addresses, dashboard
URL) so ``init(address="auto")`` and the CLI can find it."""
from __future__ import annotations

import argparse
import json
import os
import signal
import tempfile
import threading
import time
import uuid


def embedded(cfg_json: str):
    """Head process owned by one driver (``init()`` default): configuration comes
    from the driver as JSON; prints its addresses on stdout and exits when the
    driver process goes away (or on SIGTERM from ``shutdown()``)."""
    import sys

    cfg = json.loads(cfg_json)
    for p in reversed(cfg.get("sys_path", [])):
        if p not in sys.path:
            sys.path.insert(0, p)
    from .head import Head

    head = Head(cfg["session_dir"], bytes.fromhex(cfg["node_id"]), cfg["resources"], cfg["store_name"],
                int(cfg["store_bytes"]), cfg["gpus"], namespace=cfg.get("namespace") or "default",
                worker_env=cfg.get("worker_env") or {}, listen_tcp=cfg.get("listen_tcp"),
                labels=cfg.get("labels"), gcs_storage=cfg.get("gcs_storage"),
                spill_config=cfg.get("spill_config"))
    head.start()
    print(json.dumps({"pid": os.getpid(), "unix": head.sock_path, "address": head.tcp_address,
                      "session_dir": head.session_dir, "node_id": head.head_hex}), flush=True)
    parent = int(cfg.get("parent_pid", os.getppid()))
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, signal.SIG_IGN)  # the driver's Ctrl-C is the driver's business
    while not stop.is_set():
        stop.wait(0.5)
        if os.getppid() != parent:
            break  # the driver died without shutdown(): take the session down with it
    head.shutdown()


def _previous_session(gcs_storage):
    """The session a previous head on this GCS storage ran, if it can be resumed:
    its object-store arena still exists and its process is gone."""
    if not gcs_storage:
        return None
    from .gcs_persist import peek_session

    prev = peek_session(gcs_storage)
    if not prev:
        return None
    if not os.path.exists("/dev/shm" + prev["store_name"]):
        return None
    try:
        os.kill(int(prev["pid"]), 0)
        return None  # that head is still running: never share an arena between two heads
    except ProcessLookupError:
        pass
    except PermissionError:
        return None
    return prev


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=6380)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--num-cpus", type=float, default=None)
    ap.add_argument("--num-gpus", type=int, default=None)
    ap.add_argument("--resources", default="{}")
    ap.add_argument("--object-store-memory", type=int, default=None)
    ap.add_argument("--dashboard-host", default="127.0.0.1")
    ap.add_argument("--dashboard-port", type=int, default=8265)
    ap.add_argument("--include-dashboard", default="true")
    ap.add_argument("--temp-dir", default=None)
    ap.add_argument("--labels", default="{}", help="node labels (JSON)")
    ap.add_argument("--gcs-storage", default=None,
                    help="durable GCS table log (head fault tolerance): a head restarted with the same "
                         "path restores the KV, function table, jobs, detached actors and placement groups")
    ap.add_argument("--system-config", default=None, help="JSON _system_config (object_spilling_config)")
    a = ap.parse_args(argv)

    from .api import _default_cpus, _default_store_bytes, _mem_bytes, detect_gpus
    from .head import Head

    root = a.temp_dir or os.path.join(tempfile.gettempdir(), "caamd")
    sess = f"session_{time.strftime('%Y%m%d-%H%M%S')}_{os.getpid()}_{uuid.uuid4().hex[:6]}"
    session_dir = os.path.join(root, sess)
    gpus = list(range(a.num_gpus)) if a.num_gpus is not None else detect_gpus()
    res = {"CPU": float(a.num_cpus if a.num_cpus is not None else _default_cpus()), "memory": float(_mem_bytes())}
    if gpus:
        res["GPU"] = float(len(gpus))
        from .api import accelerator_resources

        res.update(accelerator_resources(gpus))
    store_bytes = int(a.object_store_memory or _default_store_bytes())
    res["object_store_memory"] = float(store_bytes)
    res[f"node:{a.host}"] = 1.0
    res["node:__internal_head__"] = 1.0
    res.update({k: float(v) for k, v in json.loads(a.resources).items()})
    store_name = f"/caamd_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    node_id = os.urandom(16)
    port = a.port
    reattach = False
    prev = _previous_session(a.gcs_storage)
    if prev is not None:
        # the node outlived the previous head (its arena is still there and the old
        # head process is gone): come back as the same node, on the same addresses,
        # so its workers / actors / drivers reconnect and re-register
        session_dir, store_name, store_bytes = prev["session_dir"], prev["store_name"], int(prev["store_bytes"])
        node_id = bytes.fromhex(prev["node_id"])
        res["object_store_memory"] = float(store_bytes)
        if prev.get("tcp_address"):
            port = int(prev["tcp_address"].rsplit(":", 1)[1])
        reattach = True
    head = Head(session_dir, node_id, res, store_name, store_bytes, gpus,
                listen_tcp=f"{a.host}:{port}", labels=json.loads(a.labels), gcs_storage=a.gcs_storage,
                reattach=reattach, reconnect_s=float(os.environ.get("CAAMD_HEAD_RECONNECT_S", "60")),
                spill_config=json.loads(a.system_config).get("object_spilling_config") if a.system_config else None)
    head.start()
    url = None
    if a.include_dashboard.lower() in ("1", "true", "yes"):
        from ..dashboard import start_dashboard

        url = start_dashboard(a.dashboard_host, a.dashboard_port, head=head, control_address=head.sock_path)
    os.makedirs(root, exist_ok=True)
    info = {"pid": os.getpid(), "address": head.tcp_address, "unix": head.sock_path, "dashboard": url,
            "session_dir": session_dir, "node_id": head.head_hex}
    with open(os.path.join(root, "head.json"), "w") as f:
        json.dump(info, f)
    with open(os.path.join(root, "latest_address"), "w") as f:
        f.write(head.sock_path)
    print(json.dumps(info), flush=True)
    stop = threading.Event()

    def on_sig(*_):
        stop.set()

    signal.signal(signal.SIGTERM, on_sig)
    signal.signal(signal.SIGINT, on_sig)
    while not stop.is_set():
        stop.wait(0.5)
    try:
        from ..dashboard import stop_dashboard

        stop_dashboard()
    finally:
        head.shutdown()
        try:
            os.unlink(os.path.join(root, "head.json"))
        except OSError:
            pass


if __name__ == "__main__":
    import sys

    if len(sys.argv) > 2 and sys.argv[1] == "--embedded":
        embedded(sys.argv[2])
    else:
        main()
