"""ray.air namespace, RuntimeEnv / JobConfig (reference: python/ray/air/__init__.py,
runtime_env/runtime_env.py, job_config.py)."""
import os
import time

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.exceptions import RuntimeEnvSetupError
from cluster_anywhere_amd.job_config import JobConfig
from cluster_anywhere_amd.runtime_env import RuntimeEnv, RuntimeEnvConfig, missing_packages


def test_air_reexports():
    from cluster_anywhere_amd import air, train

    assert air.ScalingConfig is train.ScalingConfig and air.Result is train.Result
    rr = air.ResourceRequest([{"CPU": 1, "GPU": 1}, {"CPU": 2}])
    assert rr.required_resources() == {"CPU": 3, "GPU": 1} and rr.head_bundle == {"CPU": 1, "GPU": 1}
    assert rr == air.ResourceRequest([{"CPU": 1, "GPU": 1}, {"CPU": 2}])
    assert callable(air.session.report)


def test_runtime_env_validation():
    env = RuntimeEnv(env_vars={"A": "1"}, working_dir="/tmp", pip=["numpy>=1.0", "scipy"])
    assert env.env_vars() == {"A": "1"} and env.pip_config() == {"packages": ["numpy>=1.0", "scipy"]}
    assert RuntimeEnv.deserialize(env.serialize()) == env
    with pytest.raises(TypeError):
        RuntimeEnv(env_vars={"A": 1})
    with pytest.raises(ValueError):
        RuntimeEnv(bogus=1)
    assert missing_packages(["numpy", "definitely-not-a-package-xyz==1.0"]) == ["definitely-not-a-package-xyz==1.0"]
    assert RuntimeEnvConfig(setup_timeout_seconds=10)["setup_timeout_seconds"] == 10


def test_job_config_runtime_env_and_namespace():
    jc = JobConfig(runtime_env={"env_vars": {"JOBCFG_VAR": "hello"}}, ray_namespace="jc_ns")
    jc.set_metadata("k", "v")
    assert JobConfig.from_json(jc.to_json()).metadata == {"k": "v"}
    ray.init(num_cpus=2, job_config=jc)
    try:
        @ray.remote
        def read():
            return os.environ.get("JOBCFG_VAR")

        assert ray.get(read.remote()) == "hello"
        assert ray.get_runtime_context().namespace == "jc_ns"

        @ray.remote
        def f():
            return 1

        # not installable offline: the install fails and the task reports it
        with pytest.raises(RuntimeEnvSetupError):
            ray.get(f.options(runtime_env={"pip": ["definitely-not-a-package-xyz"]}).remote(), timeout=300)
        assert ray.get(f.options(runtime_env={"pip": ["numpy"]}).remote()) == 1  # satisfied: no env built
    finally:
        ray.shutdown()


def _build_wheel(tmp_path, version="1.2.3"):
    import subprocess
    import sys

    src = tmp_path / "src"
    pkg = src / "caamd_rtenv_probe"
    pkg.mkdir(parents=True)
    (pkg / "__init__.py").write_text(f'VERSION = "{version}"\n')
    (src / "setup.py").write_text(
        "from setuptools import setup\n"
        f"setup(name='caamd_rtenv_probe', version='{version}', packages=['caamd_rtenv_probe'])\n")
    wheels = tmp_path / "wheels"
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-index", "--no-deps", "--no-build-isolation",
                        "-w", str(wheels), str(src)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return str(wheels)


def test_pip_runtime_env_installs_offline(tmp_path, monkeypatch):
    """runtime_env={"pip": ...} installs a local wheel into a cached virtualenv and
    the task runs inside it, while the driver cannot import the package (reference:
    _private/runtime_env/pip.py:45,216, uri_cache.py:9)."""
    import importlib.util

    from cluster_anywhere_amd.runtime_env import pip as rpip

    monkeypatch.setenv("CAAMD_RUNTIME_ENV_DIR", str(tmp_path / "envs"))
    wheels = _build_wheel(tmp_path)
    assert importlib.util.find_spec("caamd_rtenv_probe") is None
    ray.init(num_cpus=2)
    try:
        @ray.remote
        def probe():
            import sys

            import caamd_rtenv_probe

            return caamd_rtenv_probe.VERSION, sys.prefix

        env = {"pip": {"packages": ["caamd_rtenv_probe==1.2.3"], "find_links": [wheels]}}
        ver, prefix = ray.get(probe.options(runtime_env=env).remote(), timeout=300)
        assert ver == "1.2.3" and prefix.startswith(str(tmp_path / "envs"))
        # the env is cached: the second use starts no build
        envs = rpip._cache().entries()
        assert len(envs) == 1
        t0 = time.time()
        assert ray.get(probe.options(runtime_env=env).remote(), timeout=120)[0] == "1.2.3"
        # actors take the env too
        @ray.remote
        class A:
            def v(self):
                import caamd_rtenv_probe

                return caamd_rtenv_probe.VERSION

        a = A.options(runtime_env=env).remote()
        assert ray.get(a.v.remote(), timeout=120) == "1.2.3"
        # the driver's interpreter is untouched
        assert importlib.util.find_spec("caamd_rtenv_probe") is None
        # a version that is not among the local wheels fails with RuntimeEnvSetupError
        bad = {"pip": {"packages": ["caamd_rtenv_probe==9.9"], "find_links": [wheels]}}
        with pytest.raises(RuntimeEnvSetupError):
            ray.get(probe.options(runtime_env=bad).remote(), timeout=300)
        assert time.time() - t0 < 300
    finally:
        ray.shutdown()


def test_uri_cache_evicts_least_recently_used(tmp_path):
    from cluster_anywhere_amd.runtime_env.pip import _MARKER, URICache

    root = tmp_path / "pip"
    for i, name in enumerate(["a", "b", "c"]):
        d = root / name
        d.mkdir(parents=True)
        (d / "blob").write_bytes(b"x" * 1000)
        (d / _MARKER).write_text("{}")
        os.utime(d / _MARKER, (1000 + i, 1000 + i))
    c = URICache(str(root), max_bytes=2100)
    c.touch(str(root / "a"))  # a becomes the most recently used
    gone = c.evict()
    assert gone == [str(root / "b")]
    assert sorted(n for n in os.listdir(root) if not n.endswith(".lock")) == ["a", "c"]


def test_uri_cache_skips_envs_with_live_users(tmp_path):
    """An env some live process registered as its user (a worker running in it,
    possibly under another head) is never evicted; stale registrations are dropped."""
    import subprocess
    import sys

    from cluster_anywhere_amd.runtime_env.pip import _MARKER, URICache, live_users, mark_in_use

    root = tmp_path / "pip"
    for i, name in enumerate(["a", "b", "c"]):
        d = root / name
        d.mkdir(parents=True)
        (d / "blob").write_bytes(b"x" * 1000)
        (d / _MARKER).write_text("{}")
        os.utime(d / _MARKER, (1000 + i, 1000 + i))
    mark_in_use(str(root / "a"))  # this process uses the oldest env
    dead = subprocess.Popen([sys.executable, "-c", "pass"])
    dead.wait()
    mark_in_use(str(root / "b"), dead.pid)  # a user that has exited
    assert live_users(str(root / "a")) == [os.getpid()]
    c = URICache(str(root), max_bytes=2100)
    assert c.evict() == [str(root / "b")]
    assert live_users(str(root / "b")) == []
    assert os.path.isdir(root / "a")
