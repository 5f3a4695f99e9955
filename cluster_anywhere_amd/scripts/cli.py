"""Command line interface (reference: python/ray/scripts/scripts.py — ``ray
start/stop/status/submit/timeline/memory/list/summary``, and
python/ray/dashboard/modules/job/cli.py — ``ray job submit/status/logs/stop/list``).

    python -m cluster_anywhere_amd start --head [--port 6380] [--num-cpus N] [--num-gpus G]
    python -m cluster_anywhere_amd start --address HOST:PORT [--num-cpus N] [--resources '{"x":1}']
    python -m cluster_anywhere_amd status | stop | timeline [-o file]
    python -m cluster_anywhere_amd list actors|tasks|nodes|objects|workers|placement-groups|jobs
    python -m cluster_anywhere_amd summary tasks|actors
    python -m cluster_anywhere_amd job submit [--submission-id ID] [--no-wait] -- <entrypoint>
    python -m cluster_anywhere_amd job status|logs|stop ID ; job list
    python -m cluster_anywhere_amd up|down|get-head-ip|attach cluster.yaml ; exec cluster.yaml <cmd>
    python -m cluster_anywhere_amd submit cluster.yaml script.py [args] ; rsync-up|rsync-down cluster.yaml SRC DST
    python -m cluster_anywhere_amd memory [--top N] ; logs [GLOB] [--tail N]
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _root(temp_dir=None):
    return temp_dir or os.path.join(tempfile.gettempdir(), "caamd")


def _head_info(temp_dir=None):
    p = os.path.join(_root(temp_dir), "head.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    return e


def cmd_start(a):
    root = _root(a.temp_dir)
    os.makedirs(root, exist_ok=True)
    if a.head:
        argv = [sys.executable, "-m", "cluster_anywhere_amd.core.head_main", "--port", str(a.port),
                "--host", a.node_ip_address, "--dashboard-port", str(a.dashboard_port),
                "--include-dashboard", a.include_dashboard, "--resources", a.resources]
        if a.temp_dir:
            argv += ["--temp-dir", a.temp_dir]
        if a.gcs_storage:
            argv += ["--gcs-storage", a.gcs_storage]
        if a.system_config:
            argv += ["--system-config", a.system_config]
    elif a.address:
        argv = [sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address", a.address,
                "--resources", a.resources, "--node-ip-address", a.node_ip_address]
    else:
        print("start needs --head or --address", file=sys.stderr)
        return 2
    if a.num_cpus is not None:
        argv += ["--num-cpus", str(a.num_cpus)]
    if a.num_gpus is not None:
        argv += ["--num-gpus", str(a.num_gpus)]
    if a.object_store_memory:
        argv += ["--object-store-memory", str(a.object_store_memory)]
    if a.block:
        return subprocess.call(argv, env=_env())
    log = open(os.path.join(root, "head.out" if a.head else f"node-{int(time.time())}.out"), "ab")
    p = subprocess.Popen(argv, env=_env(), stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                         start_new_session=True)
    with open(os.path.join(root, "pids"), "a") as f:
        f.write(f"{p.pid}\n")
    if a.head:
        deadline = time.time() + 60
        while time.time() < deadline:
            info = _head_info(a.temp_dir)
            if info and info["pid"] == p.pid:
                print(f"Started head: address={info['address']} dashboard={info['dashboard']}")
                print(f"Join other nodes with: python -m cluster_anywhere_amd start --address {info['address']}")
                return 0
            if p.poll() is not None:
                print("head failed to start; see", os.path.join(root, "head.out"), file=sys.stderr)
                return 1
            time.sleep(0.1)
        return 1
    print(f"Started node agent pid={p.pid} joining {a.address}")
    return 0


def cmd_stop(a):
    root = _root(a.temp_dir)
    p = os.path.join(root, "pids")
    n = 0
    if os.path.exists(p):
        with open(p) as f:
            pids = [int(x) for x in f.read().split() if x.strip().isdigit()]
        for pid in reversed(pids):  # node agents first, head last
            try:
                os.kill(pid, signal.SIGTERM)
                n += 1
            except ProcessLookupError:
                pass
        os.unlink(p)
    print(f"Stopped {n} process(es).")
    return 0


def _connect(a):
    import cluster_anywhere_amd as ray

    addr = a.address or os.environ.get("CAAMD_ADDRESS") or os.environ.get("RAY_ADDRESS") or "auto"
    ray.init(address=addr, _temp_dir=getattr(a, "temp_dir", None))
    return ray


def cmd_status(a):
    ray = _connect(a)
    nodes = ray.nodes()
    total, avail = ray.cluster_resources(), ray.available_resources()
    print(f"======== Cluster status ========\nNodes: {sum(n['Alive'] for n in nodes)} alive, "
          f"{sum(not n['Alive'] for n in nodes)} dead")
    for n in nodes:
        print(f"  {n['NodeID'][:12]}  {'ALIVE' if n['Alive'] else 'DEAD '}  {n['NodeManagerAddress']}")
    print("Resources:")
    for k in sorted(total):
        if k.startswith("node:"):
            continue
        used = total[k] - avail.get(k, 0.0)
        print(f"  {used:g}/{total[k]:g} {k}")
    ray.shutdown()
    return 0


def cmd_list(a):
    from ..util import state

    ray = _connect(a)
    fn = {"actors": state.list_actors, "tasks": state.list_tasks, "nodes": state.list_nodes,
          "objects": state.list_objects, "workers": state.list_workers,
          "placement-groups": state.list_placement_groups, "jobs": state.list_jobs}[a.what]
    rows = fn(limit=a.limit)
    print(json.dumps(rows, indent=1, default=str))
    ray.shutdown()
    return 0


def cmd_summary(a):
    from ..util import state

    ray = _connect(a)
    fn = state.summarize_tasks if a.what == "tasks" else state.summarize_actors
    print(json.dumps(fn(), indent=1, default=str))
    ray.shutdown()
    return 0


def cmd_timeline(a):
    ray = _connect(a)
    out = a.output or f"timeline-{int(time.time())}.json"
    ray.timeline(out)
    print(f"Trace written to {out} (open in chrome://tracing or Perfetto)")
    ray.shutdown()
    return 0


def _job_client(a):
    from ..job_submission import JobSubmissionClient

    addr = a.address
    if addr is None:
        info = _head_info()
        addr = info["dashboard"] if info else "http://127.0.0.1:8265"
    return JobSubmissionClient(addr)


def cmd_job(a):
    c = _job_client(a)
    if a.job_cmd == "submit":
        ep = " ".join(a.entrypoint[1:] if a.entrypoint and a.entrypoint[0] == "--" else a.entrypoint)
        renv = json.loads(a.runtime_env_json) if a.runtime_env_json else None
        if a.working_dir:
            renv = dict(renv or {}, working_dir=os.path.abspath(a.working_dir))
        sid = c.submit_job(entrypoint=ep, submission_id=a.submission_id, runtime_env=renv)
        print(f"Job '{sid}' submitted successfully")
        if a.no_wait:
            return 0
        for chunk in c.tail_job_logs(sid):
            sys.stdout.write(chunk)
        st = c.get_job_status(sid)
        print(f"Job '{sid}' {st.value.lower()}")
        return 0 if st.value == "SUCCEEDED" else 1
    if a.job_cmd == "status":
        print(c.get_job_status(a.job_id).value)
    elif a.job_cmd == "logs":
        sys.stdout.write(c.get_job_logs(a.job_id))
    elif a.job_cmd == "stop":
        print("stopped" if c.stop_job(a.job_id) else "not running")
    elif a.job_cmd == "list":
        for j in c.list_jobs():
            print(f"{j.submission_id}  {j.status.value:10s}  {j.entrypoint}")
    return 0


def _launcher_cfg(a):
    from ..autoscaler import commands

    return commands.load_cluster_config(a.cluster_config)


def cmd_up(a):
    from ..autoscaler import commands

    st = commands.create_or_update_cluster(a.cluster_config, no_restart=a.no_restart)
    print(f"Cluster {st['cluster_name']!r} is up: address={st['address']}")
    print(f"  run on it:   python -m cluster_anywhere_amd exec {a.cluster_config} '<cmd>'")
    print(f"  tear down:   python -m cluster_anywhere_amd down {a.cluster_config}")
    return 0


def cmd_down(a):
    from ..autoscaler import commands

    commands.teardown_cluster(a.cluster_config, workers_only=a.workers_only)
    print("Cluster torn down." if not a.workers_only else "Worker nodes terminated.")
    return 0


def cmd_exec(a):
    from ..autoscaler import commands

    return commands.exec_cluster(a.cluster_config, " ".join(a.cmd)).returncode


def cmd_submit(a):
    from ..autoscaler import commands

    return commands.submit(a.cluster_config, a.script, a.script_args).returncode


def cmd_get_head_ip(a):
    from ..autoscaler import commands

    print(commands.get_head_node_ip(a.cluster_config))
    return 0


def cmd_rsync(a):
    from ..autoscaler import commands

    commands.rsync(a.cluster_config, a.source, a.target, down=a.cmd == "rsync-down")
    return 0


def cmd_attach(a):
    from ..autoscaler import commands

    cfg = _launcher_cfg(a)
    st = commands._load_state(cfg["cluster_name"])
    if st is None:
        print("cluster is not running", file=sys.stderr)
        return 1
    if st["provider"] == "local":
        return subprocess.call([os.environ.get("SHELL", "bash")], env=dict(os.environ, CAAMD_ADDRESS=st["address"]))
    auth = cfg.get("auth", {})
    tgt = f"{auth['ssh_user']}@{st['head_ip']}" if auth.get("ssh_user") else st["head_ip"]
    return subprocess.call(["ssh", "-t", tgt])


def cmd_memory(a):
    """Object-store usage by node and the largest live objects (reference: ``ray memory``)."""
    from ..util import state

    ray = _connect(a)
    objs = state.list_objects(limit=100000)
    per_node = {}
    for o in objs:
        n = o.get("node_id") or o.get("node") or "inline"
        sz = int(o.get("object_size") or o.get("size") or 0)
        c, b = per_node.get(n, (0, 0))
        per_node[n] = (c + 1, b + sz)
    print("======== Object references ========")
    print(f"{'node':34s} {'objects':>8s} {'bytes':>14s}")
    for n, (c, b) in sorted(per_node.items(), key=lambda kv: -kv[1][1]):
        print(f"{str(n)[:34]:34s} {c:8d} {b:14d}")
    top = sorted(objs, key=lambda o: -int(o.get("object_size") or o.get("size") or 0))[: a.top]
    if top:
        print(f"\nLargest {len(top)} objects:")
        for o in top:
            print(f"  {str(o.get('object_id', ''))[:48]:48s} {int(o.get('object_size') or o.get('size') or 0):14d}"
                  f"  refs={o.get('ref_count', '?')}")
    total = ray.cluster_resources().get("object_store_memory", 0)
    print(f"\nObject store capacity: {int(total)} bytes")
    ray.shutdown()
    return 0


def cmd_logs(a):
    """List the session's log files, or print one (``--tail`` lines; reference: ``ray logs``)."""
    import fnmatch

    ray = _connect(a)
    from ..core.api import _session

    sdir = _session.get("session_dir")
    ray.shutdown()
    if not sdir or not os.path.isdir(sdir):
        print("no session directory", file=sys.stderr)
        return 1
    files = sorted(f for f in os.listdir(sdir) if f.endswith((".log", ".out", ".err")))
    if a.glob:
        files = [f for f in files if fnmatch.fnmatch(f, a.glob)]
    if not a.glob or len(files) != 1:
        for f in files:
            print(f"{os.path.getsize(os.path.join(sdir, f)):10d}  {f}")
        return 0
    with open(os.path.join(sdir, files[0]), errors="replace") as fh:
        lines = fh.readlines()
    sys.stdout.writelines(lines[-a.tail:] if a.tail else lines)
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(prog="cluster_anywhere_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("start")
    s.add_argument("--head", action="store_true")
    s.add_argument("--address", default=None)
    s.add_argument("--port", type=int, default=6380)
    s.add_argument("--num-cpus", type=float, default=None)
    s.add_argument("--num-gpus", type=int, default=None)
    s.add_argument("--resources", default="{}")
    s.add_argument("--object-store-memory", type=int, default=None)
    s.add_argument("--node-ip-address", default="127.0.0.1")
    s.add_argument("--dashboard-port", type=int, default=8265)
    s.add_argument("--include-dashboard", default="true")
    s.add_argument("--temp-dir", default=None)
    s.add_argument("--gcs-storage", default=None,
                   help="head fault tolerance: durable GCS table log reloaded by a head restarted on it")
    s.add_argument("--system-config", default=None,
                   help='JSON, e.g. {"object_spilling_config": {"type": "filesystem", '
                        '"params": {"directory_path": ["/mnt/a", "/mnt/b"]}}}')
    s.add_argument("--block", action="store_true")
    s.set_defaults(fn=cmd_start)
    s = sub.add_parser("stop")
    s.add_argument("--temp-dir", default=None)
    s.set_defaults(fn=cmd_stop)
    for name, fn in (("status", cmd_status), ("timeline", cmd_timeline)):
        s = sub.add_parser(name)
        s.add_argument("--address", default=None)
        s.add_argument("--temp-dir", default=None)
        s.add_argument("-o", "--output", default=None)
        s.set_defaults(fn=fn)
    s = sub.add_parser("list")
    s.add_argument("what", choices=["actors", "tasks", "nodes", "objects", "workers", "placement-groups", "jobs"])
    s.add_argument("--address", default=None)
    s.add_argument("--limit", type=int, default=100)
    s.set_defaults(fn=cmd_list)
    s = sub.add_parser("summary")
    s.add_argument("what", choices=["tasks", "actors"])
    s.add_argument("--address", default=None)
    s.set_defaults(fn=cmd_summary)
    j = sub.add_parser("job")
    jsub = j.add_subparsers(dest="job_cmd", required=True)
    js = jsub.add_parser("submit")
    js.add_argument("--address", default=None)
    js.add_argument("--submission-id", default=None)
    js.add_argument("--runtime-env-json", default=None)
    js.add_argument("--working-dir", default=None)
    js.add_argument("--no-wait", action="store_true")
    js.add_argument("entrypoint", nargs=argparse.REMAINDER)
    for name in ("status", "logs", "stop"):
        x = jsub.add_parser(name)
        x.add_argument("job_id")
        x.add_argument("--address", default=None)
    x = jsub.add_parser("list")
    x.add_argument("--address", default=None)
    j.set_defaults(fn=cmd_job)
    for name, fn in (("up", cmd_up), ("down", cmd_down), ("get-head-ip", cmd_get_head_ip), ("attach", cmd_attach)):
        x = sub.add_parser(name)
        x.add_argument("cluster_config")
        if name == "up":
            x.add_argument("--no-restart", action="store_true")
            x.add_argument("-y", "--yes", action="store_true")
        if name == "down":
            x.add_argument("--workers-only", action="store_true")
            x.add_argument("-y", "--yes", action="store_true")
        x.set_defaults(fn=fn)
    x = sub.add_parser("exec")
    x.add_argument("cluster_config")
    x.add_argument("cmd", nargs=argparse.REMAINDER)
    x.set_defaults(fn=cmd_exec)
    x = sub.add_parser("submit")
    x.add_argument("cluster_config")
    x.add_argument("script")
    x.add_argument("script_args", nargs=argparse.REMAINDER)
    x.set_defaults(fn=cmd_submit)
    for name in ("rsync-up", "rsync-down"):
        x = sub.add_parser(name)
        x.add_argument("cluster_config")
        x.add_argument("source")
        x.add_argument("target")
        x.set_defaults(fn=cmd_rsync, cmd=name)
    x = sub.add_parser("memory")
    x.add_argument("--address", default=None)
    x.add_argument("--top", type=int, default=10)
    x.set_defaults(fn=cmd_memory)
    x = sub.add_parser("logs")
    x.add_argument("glob", nargs="?", default=None)
    x.add_argument("--address", default=None)
    x.add_argument("--tail", type=int, default=0)
    x.set_defaults(fn=cmd_logs)
    from ..serve.scripts import add_parser as add_serve_parser

    add_serve_parser(sub)
    a = ap.parse_args(argv)
    return a.fn(a) or 0


if __name__ == "__main__":
    sys.exit(main())
