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

    ray.init(address=a.address or "auto", _temp_dir=getattr(a, "temp_dir", None))
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
    from ..serve.scripts import add_parser as add_serve_parser

    add_serve_parser(sub)
    a = ap.parse_args(argv)
    return a.fn(a) or 0


if __name__ == "__main__":
    sys.exit(main())
