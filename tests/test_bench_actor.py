"""The headline bench's multi-worker path, rehearsed on CPU with gloo.

``bench.py --gpus N`` runs the GPT-2 step through the framework's own actor
worker group (PACK placement group -> N ``_TrainWorker`` actors -> process group
-> ZeRO-1 step). These tests run exactly that code path with ``--cpu`` (gloo,
world 2, gpt2-tiny), both stand-alone and under ``torch.distributed.run`` (the
way the round-end driver launches N>1), and check the one-JSON-line contract.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--cpu", "--model", "gpt2-tiny", "--micro-batch", "2", "--seq-len", "32", "--steps", "2",
        "--warmup", "1"]


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["CAAMD_STORAGE_PATH"] = "/tmp/caamd_bench_test"
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    return env


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{") and '"metric"' in l]


def test_bench_actor_mode_world2_cpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == 2 and j["steps"] == 2 and j["warmup"] == 1
    assert j["config"]["parallelism"] == "dp2-zero1"
    assert j["config"]["mode"] == "actor"
    assert j["value"] > 0 and j["ms_per_step"] > 0
    assert j["config"]["global_batch"] == 4


def test_bench_actor_mode_under_launcher_prints_once():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29641",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2


def test_bench_spmd_mode_under_launcher():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29643",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", "spmd", *TINY]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert lines[0]["config"]["parallelism"] == "dp2-zero1"


def test_bench_actor_mode_world8_cpu():
    """The N=8 scaling run's code path (dp8-zero1 through the actor worker group),
    rehearsed with gloo on CPU: shard alignment to 8 x world, bucket cuts and the
    weight all-gather order at the world size of a full MI355X node."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", *TINY],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == 8 and j["config"]["parallelism"] == "dp8-zero1"
    assert j["config"]["global_batch"] == 16 and j["value"] > 0


def test_bench_actor_mode_under_launcher_world8():
    """Exactly the driver's N=8 launch line (torch.distributed.run, 8 procs, 127.0.0.1),
    CPU/gloo: one JSON line, dp8."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", "29647",
           os.path.join(ROOT, "bench.py"), "--gpus", "8", *TINY]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 8 and lines[0]["config"]["parallelism"] == "dp8-zero1"
