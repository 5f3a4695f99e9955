"""Cluster launcher (reference: autoscaler/_private/commands.py
create_or_update_cluster / teardown_cluster / exec_cluster / rsync / submit,
and the `ray up/down/exec/submit/memory/logs` CLI) with the local provider:
head + min_workers node agents kept by an autoscaler monitor process."""
import os
import subprocess
import sys
import time

import pytest
import yaml

from cluster_anywhere_amd.autoscaler import commands

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    e.pop("CAAMD_ADDRESS", None)
    return e


def _cli(*args, timeout=120):
    return subprocess.run([sys.executable, "-m", "cluster_anywhere_amd", *args], env=_env(), capture_output=True,
                          text=True, timeout=timeout)


@pytest.fixture
def cfg_path(tmp_path):
    marker = tmp_path / "setup.txt"
    cfg = {"cluster_name": f"t{os.getpid()}", "provider": {"type": "local"}, "head_node_type": "head",
           "available_node_types": {"head": {"resources": {"CPU": 2}},
                                    "extra": {"resources": {"CPU": 1, "extra": 1}, "min_workers": 1,
                                              "max_workers": 2}},
           "setup_commands": [f"echo ok > {marker}"],
           "file_mounts": {str(tmp_path / "mounted.txt"): str(tmp_path / "src.txt")}}
    (tmp_path / "src.txt").write_text("payload")
    p = tmp_path / "cluster.yaml"
    p.write_text(yaml.safe_dump(cfg))
    yield str(p)
    commands.teardown_cluster(str(p))


def test_up_exec_submit_down(cfg_path, tmp_path):
    r = _cli("up", cfg_path, "-y")
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "setup.txt").read_text().strip() == "ok"
    assert (tmp_path / "mounted.txt").read_text() == "payload"
    assert _cli("get-head-ip", cfg_path).stdout.strip() == "127.0.0.1"
    probe = ("import time, cluster_anywhere_amd as ray; ray.init(); t = time.time()\n"
             "while ray.cluster_resources().get('extra') != 1.0 and time.time() - t < 60: time.sleep(0.2)\n"
             "print('NODES', len([n for n in ray.nodes() if n['Alive']]), ray.cluster_resources().get('extra'))")
    script = tmp_path / "probe.py"
    script.write_text(probe)
    r = _cli("submit", cfg_path, str(script))
    assert "NODES 2 1.0" in r.stdout, (r.stdout, r.stderr)
    r = _cli("exec", cfg_path, "python -m cluster_anywhere_amd memory")
    assert "Object store capacity" in r.stdout, r.stderr
    r = _cli("exec", cfg_path, "python -m cluster_anywhere_amd logs")
    assert r.returncode == 0
    (tmp_path / "up.txt").write_text("x")
    assert _cli("rsync-up", cfg_path, str(tmp_path / "up.txt"), str(tmp_path / "copied" / "up.txt")).returncode == 0
    assert (tmp_path / "copied" / "up.txt").read_text() == "x"
    st = commands._load_state(commands.load_cluster_config(cfg_path)["cluster_name"])
    mon, head = st["monitor_pid"], st["head_pid"]
    r = _cli("down", cfg_path, "-y")
    assert r.returncode == 0, r.stderr
    time.sleep(0.5)
    for pid in (mon, head):
        try:
            os.kill(pid, 0)
            alive = open(f"/proc/{pid}/stat").read().split(")")[1].split()[0] not in ("Z", "X")
        except (ProcessLookupError, FileNotFoundError):
            alive = False
        assert not alive, pid
    assert commands._load_state(commands.load_cluster_config(cfg_path)["cluster_name"]) is None


def test_config_validation():
    with pytest.raises(ValueError, match="provider type"):
        commands.load_cluster_config({"provider": {"type": "aws"}})
    with pytest.raises(ValueError, match="head_node_type"):
        commands.load_cluster_config({"head_node_type": "x", "available_node_types": {"h": {"resources": {}}}})
