"""ray.air namespace, RuntimeEnv / JobConfig (reference: python/ray/air/__init__.py,
runtime_env/runtime_env.py, job_config.py)."""
import os

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

        with pytest.raises(RuntimeEnvSetupError):
            f.options(runtime_env={"pip": ["definitely-not-a-package-xyz"]}).remote()
        assert ray.get(f.options(runtime_env={"pip": ["numpy"]}).remote()) == 1
    finally:
        ray.shutdown()
