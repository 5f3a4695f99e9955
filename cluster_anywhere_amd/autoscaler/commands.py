"""Cluster launcher: ``up`` / ``down`` / ``exec`` / ``submit`` / ``rsync`` /
``get-head-ip`` from one YAML file (reference roles:
python/ray/autoscaler/_private/commands.py ``create_or_update_cluster`` :221,
``teardown_cluster`` :429, ``exec_cluster``, ``rsync``, ``get_head_node_ip``,
and the on-prem "local" provider with ``head_ip`` / ``worker_ips``).

Config (a subset of the reference schema)::

    cluster_name: demo
    provider:
      type: local              # this host: head + worker node agents as processes,
                               # min_workers kept by an autoscaler monitor process
      # type: ssh              # on-prem machines reached over ssh
      # head_ip: 10.0.0.1
      # worker_ips: [10.0.0.2, 10.0.0.3]
    auth: {ssh_user: ubuntu, ssh_private_key: ~/.ssh/id_rsa}       # ssh only
    head_node_type: head
    available_node_types:
      head:   {resources: {CPU: 8, GPU: 8}}
      cpu:    {resources: {CPU: 4}, min_workers: 1, max_workers: 4}
    initialization_commands: []     # before setup, on every node
    setup_commands: []              # on every node
    head_setup_commands: []
    worker_setup_commands: []
    file_mounts: {remote_path: local_path}
    head_start_ray_commands: [...]  # default: start --head
    worker_start_ray_commands: [...]  # default: start --address $HEAD_ADDRESS
    idle_timeout_minutes: 5

State of a launched cluster (address, pids) lives in
``$TMPDIR/caamd-clusters/<cluster_name>.json``.
"""
from __future__ import annotations

import json
import os
import shlex
import shutil
import signal
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HEAD_PORT = 6380


def _env(extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e.update(extra or {})
    return e


def load_cluster_config(path_or_dict) -> dict:
    if isinstance(path_or_dict, str):
        import yaml

        with open(path_or_dict) as f:
            cfg = yaml.safe_load(f)
    else:
        cfg = json.loads(json.dumps(path_or_dict))
    cfg.setdefault("cluster_name", "default")
    prov = cfg.setdefault("provider", {"type": "local"})
    if prov.get("type") not in ("local", "ssh"):
        raise ValueError(f"provider type {prov.get('type')!r} is not supported here (local, ssh)")
    types = cfg.setdefault("available_node_types", {"head": {"resources": {}}})
    cfg.setdefault("head_node_type", next(iter(types)))
    if cfg["head_node_type"] not in types:
        raise ValueError(f"head_node_type {cfg['head_node_type']!r} is not in available_node_types")
    for k in ("initialization_commands", "setup_commands", "head_setup_commands", "worker_setup_commands"):
        cfg.setdefault(k, [])
    cfg.setdefault("file_mounts", {})
    return cfg


def _state_dir() -> str:
    d = os.path.join(tempfile.gettempdir(), "caamd-clusters")
    os.makedirs(d, exist_ok=True)
    return d


def _state_path(name: str) -> str:
    return os.path.join(_state_dir(), f"{name}.json")


def _load_state(name: str) -> Optional[dict]:
    p = _state_path(name)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


# ------------------------------------------------------------ command runners
class LocalCommandRunner:
    """Runs commands on this host (reference: LocalCommandRunner / the docker-less
    path of command_runner.py)."""

    def __init__(self, env: Optional[Dict[str, str]] = None):
        self.env = env or {}

    def run(self, cmd: str, capture: bool = False, check: bool = True) -> subprocess.CompletedProcess:
        r = subprocess.run(["bash", "-c", cmd], env=_env(self.env), capture_output=capture, text=True)
        if check and r.returncode != 0:
            raise RuntimeError(f"command failed ({r.returncode}): {cmd}\n{r.stderr if capture else ''}")
        return r

    def rsync(self, src: str, dst: str, down: bool = False):
        a, b = (dst, src) if down else (src, dst)
        if os.path.abspath(a) == os.path.abspath(b):
            return
        os.makedirs(os.path.dirname(os.path.abspath(b)) or ".", exist_ok=True)
        if os.path.isdir(a):
            shutil.copytree(a, b, dirs_exist_ok=True)
        else:
            shutil.copy2(a, b)


class SSHCommandRunner:
    """Runs commands on an on-prem machine over ssh (reference: SSHCommandRunner)."""

    def __init__(self, ip: str, user: Optional[str] = None, key: Optional[str] = None,
                 env: Optional[Dict[str, str]] = None):
        self.ip, self.user, self.key = ip, user, key
        self.env = env or {}

    def _target(self):
        return f"{self.user}@{self.ip}" if self.user else self.ip

    def _ssh(self) -> List[str]:
        opts = ["-o", "StrictHostKeyChecking=no", "-o", "UserKnownHostsFile=/dev/null", "-o", "LogLevel=ERROR",
                "-o", "ConnectTimeout=10"]
        if self.key:
            opts += ["-i", os.path.expanduser(self.key)]
        return opts

    def run(self, cmd: str, capture: bool = False, check: bool = True) -> subprocess.CompletedProcess:
        exports = " ".join(f"export {k}={shlex.quote(v)};" for k, v in self.env.items())
        r = subprocess.run(["ssh"] + self._ssh() + [self._target(), f"bash -lc {shlex.quote(exports + cmd)}"],
                           capture_output=capture, text=True)
        if check and r.returncode != 0:
            raise RuntimeError(f"ssh {self.ip} failed ({r.returncode}): {cmd}")
        return r

    def rsync(self, src: str, dst: str, down: bool = False):
        remote = f"{self._target()}:{dst if not down else src}"
        args = ["-e", "ssh " + " ".join(self._ssh()), "-az"]
        if down:
            subprocess.run(["rsync"] + args + [remote, dst], check=True)
        else:
            subprocess.run(["rsync"] + args + [src, remote], check=True)


def _runner(cfg, ip: Optional[str], env=None):
    if cfg["provider"]["type"] == "local" or ip in (None, "127.0.0.1", "localhost"):
        return LocalCommandRunner(env)
    auth = cfg.get("auth", {})
    return SSHCommandRunner(ip, auth.get("ssh_user"), auth.get("ssh_private_key"), env)


def _res_args(resources: Dict[str, float]) -> str:
    out = []
    if "CPU" in resources:
        out += ["--num-cpus", str(resources["CPU"])]
    if "GPU" in resources:
        out += ["--num-gpus", str(int(resources["GPU"]))]
    custom = {k: v for k, v in resources.items() if k not in ("CPU", "GPU", "memory")}
    if custom:
        out += ["--resources", shlex.quote(json.dumps(custom))]
    return " ".join(out)


def _py() -> str:
    return f"{shlex.quote(sys.executable)} -m cluster_anywhere_amd"


def _setup_node(cfg, runner, head: bool):
    for remote, local in (cfg.get("file_mounts") or {}).items():
        runner.rsync(os.path.expanduser(local), os.path.expanduser(remote))
    cmds = list(cfg["initialization_commands"]) + list(cfg["setup_commands"])
    cmds += list(cfg["head_setup_commands"] if head else cfg["worker_setup_commands"])
    for c in cmds:
        runner.run(c)


# ------------------------------------------------------------------ commands
def create_or_update_cluster(config, *, no_restart: bool = False) -> dict:
    """Start (or restart) the head and the minimum workers; returns the state."""
    cfg = load_cluster_config(config)
    name = cfg["cluster_name"]
    st = _load_state(name)
    if st is not None and not no_restart:
        teardown_cluster(cfg)
        st = None
    if st is not None:
        return st
    prov = cfg["provider"]
    types = cfg["available_node_types"]
    head_t = cfg["head_node_type"]
    temp_dir = os.path.join(_state_dir(), name)
    state = {"cluster_name": name, "provider": prov["type"], "temp_dir": temp_dir, "monitor_pid": None,
             "workers": []}
    if prov["type"] == "local":
        os.makedirs(temp_dir, exist_ok=True)
        runner = LocalCommandRunner()
        _setup_node(cfg, runner, head=True)
        port = int(prov.get("head_port", 0) or 0) or _free_port()
        head_cmds = cfg.get("head_start_ray_commands") or [
            f"{_py()} start --head --port {port} --temp-dir {shlex.quote(temp_dir)} --include-dashboard false "
            + _res_args(types[head_t].get("resources", {}))]
        for c in head_cmds:
            runner.run(c)
        info = _wait_head(temp_dir)
        state.update(address=info["address"], head_ip="127.0.0.1", head_pid=info["pid"])
        # worker types (all but the head) go to an autoscaler monitor process that
        # launches min_workers now and scales within [min, max] afterwards
        wtypes = {k: v for k, v in types.items() if k != head_t}
        if wtypes:
            acfg = {"max_workers": cfg.get("max_workers", 8), "available_node_types": wtypes,
                    "idle_timeout_minutes": cfg.get("idle_timeout_minutes", 5.0)}
            path = os.path.join(temp_dir, "autoscaler.json")
            with open(path, "w") as f:
                json.dump(acfg, f)
            log = open(os.path.join(temp_dir, "monitor.out"), "ab")
            p = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.autoscaler.monitor", "--address",
                                  info["address"], "--config", path, "--interval", "1.0"],
                                 env=_env(), stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                                 start_new_session=True)
            log.close()
            state["monitor_pid"] = p.pid
    else:
        head_ip = prov["head_ip"]
        port = int(prov.get("head_port", HEAD_PORT))
        runner = _runner(cfg, head_ip)
        _setup_node(cfg, runner, head=True)
        for c in cfg.get("head_start_ray_commands") or [
                f"python -m cluster_anywhere_amd stop; python -m cluster_anywhere_amd start --head "
                f"--port {port} --node-ip-address {head_ip} " + _res_args(types[head_t].get("resources", {}))]:
            runner.run(c)
        address = f"{head_ip}:{port}"
        state.update(address=address, head_ip=head_ip)
        wt = next((v for k, v in types.items() if k != head_t), {"resources": {}})
        for ip in prov.get("worker_ips", []):
            wr = _runner(cfg, ip, env={"CAAMD_HEAD_ADDRESS": address})
            _setup_node(cfg, wr, head=False)
            for c in cfg.get("worker_start_ray_commands") or [
                    f"python -m cluster_anywhere_amd stop; python -m cluster_anywhere_amd start "
                    f"--address {address} --node-ip-address {ip} " + _res_args(wt.get("resources", {}))]:
                wr.run(c.replace("$HEAD_ADDRESS", address))
            state["workers"].append(ip)
    with open(_state_path(name), "w") as f:
        json.dump(state, f)
    return state


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait_head(temp_dir: str, timeout: float = 60.0) -> dict:
    deadline = time.time() + timeout
    p = os.path.join(temp_dir, "head.json")
    while time.time() < deadline:
        if os.path.exists(p):
            try:
                with open(p) as f:
                    return json.load(f)
            except ValueError:
                pass
        time.sleep(0.1)
    raise TimeoutError(f"head did not come up (see {temp_dir}/head.out)")


def _kill(pid: Optional[int], sig=signal.SIGTERM, wait: float = 10.0):
    if not pid:
        return
    try:
        os.kill(pid, sig)
    except ProcessLookupError:
        return
    deadline = time.time() + wait
    while time.time() < deadline:
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            return
        try:  # reap if it is our child
            if os.waitpid(pid, os.WNOHANG)[0] == pid:
                return
        except ChildProcessError:
            pass
        time.sleep(0.05)
    try:
        os.kill(pid, signal.SIGKILL)
    except ProcessLookupError:
        pass


def teardown_cluster(config, *, workers_only: bool = False) -> None:
    cfg = load_cluster_config(config)
    name = cfg["cluster_name"]
    st = _load_state(name)
    if st is None:
        return
    if st["provider"] == "local":
        _kill(st.get("monitor_pid"))  # its SIGTERM handler terminates the worker node agents
        if not workers_only:
            LocalCommandRunner().run(f"{_py()} stop --temp-dir {shlex.quote(st['temp_dir'])}", check=False)
            _kill(st.get("head_pid"))
    else:
        for ip in st.get("workers", []):
            _runner(cfg, ip).run("python -m cluster_anywhere_amd stop", check=False)
        if not workers_only:
            _runner(cfg, st["head_ip"]).run("python -m cluster_anywhere_amd stop", check=False)
    if not workers_only:
        os.unlink(_state_path(name))


def get_head_node_ip(config) -> str:
    cfg = load_cluster_config(config)
    st = _load_state(cfg["cluster_name"])
    if st is None:
        raise RuntimeError(f"cluster {cfg['cluster_name']!r} is not running (run `up` first)")
    return st["head_ip"]


def exec_cluster(config, cmd: str, capture: bool = False) -> subprocess.CompletedProcess:
    """Run ``cmd`` on the head node with the cluster address exported
    (``CAAMD_ADDRESS``: ``init(address="auto")`` connects to it)."""
    cfg = load_cluster_config(config)
    st = _load_state(cfg["cluster_name"])
    if st is None:
        raise RuntimeError(f"cluster {cfg['cluster_name']!r} is not running (run `up` first)")
    env = {"CAAMD_ADDRESS": st["address"]}
    return _runner(cfg, st["head_ip"], env).run(cmd, capture=capture, check=False)


def rsync(config, source: str, target: str, down: bool = False) -> None:
    cfg = load_cluster_config(config)
    st = _load_state(cfg["cluster_name"])
    if st is None:
        raise RuntimeError(f"cluster {cfg['cluster_name']!r} is not running (run `up` first)")
    _runner(cfg, st["head_ip"]).rsync(source, target, down=down)


def submit(config, script: str, args: Optional[List[str]] = None, capture: bool = False):
    cfg = load_cluster_config(config)
    st = _load_state(cfg["cluster_name"])
    if st is None:
        raise RuntimeError(f"cluster {cfg['cluster_name']!r} is not running (run `up` first)")
    target = os.path.join(st.get("temp_dir") or "/tmp", os.path.basename(script))
    if st["provider"] == "ssh":
        target = f"~/{os.path.basename(script)}"
    rsync(cfg, script, target)
    return exec_cluster(cfg, f"{shlex.quote(sys.executable) if st['provider'] == 'local' else 'python'} "
                             f"{target} " + " ".join(shlex.quote(a) for a in args or []), capture=capture)
