"""Per-node agent (the raylet role for non-head nodes; reference:
src/ray/raylet/main.cc, node_manager.cc, worker_pool.cc).

``python -m cluster_anywhere_amd.core.node_agent --address HEAD:PORT``:
creates this node's shared-memory object store and object server, registers
the node's resources (CPUs, MI355X GPUs from the KFD topology, custom
resources) with the head over TCP, then starts worker processes on the head's
request and frees objects the head garbage-collects. Exits (taking its
workers with it) when the head connection drops."""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
import uuid


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--num-cpus", type=float, default=None)
    ap.add_argument("--num-gpus", type=int, default=None)
    ap.add_argument("--resources", default="{}")
    ap.add_argument("--object-store-memory", type=int, default=None)
    ap.add_argument("--node-ip-address", default="127.0.0.1")
    ap.add_argument("--node-id", default=None)
    ap.add_argument("--labels", default="{}", help="node labels (JSON)")
    a = ap.parse_args(argv)

    from .. import _native
    from .api import _default_cpus, _default_store_bytes, _mem_bytes, detect_gpus, store_segment_name
    from .object_server import ObjectServer
    from .protocol import ConnectionClosed, connect

    node_hex = a.node_id or os.urandom(16).hex()
    gpus = list(range(a.num_gpus)) if a.num_gpus is not None else detect_gpus()
    res = {"CPU": float(a.num_cpus if a.num_cpus is not None else _default_cpus()), "memory": float(_mem_bytes())}
    if gpus:
        res["GPU"] = float(len(gpus))
        from .api import accelerator_resources

        res.update(accelerator_resources(gpus))
    store_bytes = int(a.object_store_memory or _default_store_bytes())
    res["object_store_memory"] = float(store_bytes)
    res.update({k: float(v) for k, v in json.loads(a.resources).items()})
    store_name = store_segment_name(node=True)
    store = _native.ObjectStore(store_name, store_bytes, 1 << 18, True)
    store.prefault_async(int(os.environ.get("CAAMD_OBJECT_STORE_PREFAULT_BYTES", str(2 << 30))))
    osrv = ObjectServer(store, a.node_ip_address)
    reg = {"resources": res, "gpu_ids": gpus, "store_name": store_name,
           "obj_addr": osrv.address(a.node_ip_address), "address": a.node_ip_address, "pid": os.getpid(),
           "labels": json.loads(a.labels)}
    conn = connect(a.address)
    conn.send(("register", "node", os.urandom(16), os.getpid(), node_hex, reg))
    msg = conn.recv()
    assert msg[0] == "registered", msg
    reconnect_s = float(msg[1].get("reconnect_s") or 0)

    def reconnect():
        """The head went away: a restarted head (same GCS storage, same address)
        takes this node back with its store and running workers (reference: raylets
        re-registering with a restarted GCS)."""
        deadline = time.time() + reconnect_s
        while time.time() < deadline:
            try:
                c = connect(a.address)
                c.send(("register", "node", os.urandom(16), os.getpid(), node_hex, dict(reg, reattach=True)))
                m = c.recv()
                if m[0] == "registered":
                    return c
            except (ConnectionClosed, OSError):
                pass
            time.sleep(0.3)
        return None
    session_dir = msg[1]["session_dir"]
    log_dir = os.path.join(session_dir, f"node-{node_hex[:8]}")
    os.makedirs(log_dir, exist_ok=True)
    procs = []
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

    def cleanup(*_):
        for p in procs:
            try:
                p.kill()
            except Exception:
                pass
        try:
            store.unlink()
        except Exception:
            pass
        os._exit(0)

    signal.signal(signal.SIGTERM, cleanup)
    print(f"node {node_hex} joined {a.address} with {res}", flush=True)
    # physical metrics of this node, pushed to the head (dashboard/reporter.py)
    link = {"conn": conn}

    def push_stats(st):
        try:
            link["conn"].send(("node_stats", st))
        except Exception:
            pass

    from ..dashboard.reporter import NodeReporter

    NodeReporter(push_stats, session_dir).start()
    try:
        while True:
            try:
                m = conn.recv()
            except (ConnectionClosed, OSError):
                nc = reconnect() if reconnect_s > 0 else None
                if nc is None:
                    break
                conn = link["conn"] = nc
                continue
            if m[0] == "spawn":
                _, wid, gpu_ids, extra = m
                e = dict(os.environ)
                e.update(extra)
                e["CAAMD_HEAD"] = a.address
                e["CAAMD_WORKER_ID"] = wid
                e["CAAMD_NODE_ID"] = node_hex
                e["CAAMD_NODE_IP"] = a.node_ip_address
                e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
                log = open(os.path.join(log_dir, f"worker-{wid[:8]}.log"), "ab")
                procs.append(subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.worker_main"],
                                              env=e, stdout=log, stderr=subprocess.STDOUT,
                                              stdin=subprocess.DEVNULL))
                log.close()
                procs[:] = [p for p in procs if p.poll() is None]
            elif m[0] == "free":
                for oid in m[1]:
                    try:
                        store.remove(oid)
                    except Exception:
                        pass
            elif m[0] == "shutdown":
                break
    finally:
        cleanup()


if __name__ == "__main__":
    main()
