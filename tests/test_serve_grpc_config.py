"""Serve gRPC ingress, the declarative config schema and the ``serve`` CLI
(reference test model: python/ray/serve/tests/test_grpc.py, test_config_files/,
test_cli.py, test_schema.py)."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time
import urllib.error
import urllib.request

import grpc
import pytest
import yaml

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import serve
from cluster_anywhere_amd.serve import _serve_api_pb2 as api_pb2
from cluster_anywhere_amd.serve.schema import ServeDeploySchema, build_config, deploy_config

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _grpc_user_pb2 as pb2  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _get(url):
    try:
        return json.loads(urllib.request.urlopen(url, timeout=30).read())
    except urllib.error.HTTPError as e:
        raise AssertionError(e.read()[-3000:].decode(errors="replace"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@serve.deployment
class GrpcDeployment:
    def __call__(self, req):
        if req.name == "boom":
            raise ValueError("boom requested")
        return pb2.UserDefinedResponse(greeting=f"Hello {req.name}", num_x2=req.num * 2)

    def Multiplexing(self, req):
        return pb2.UserDefinedResponse(greeting=f"model={serve.get_multiplexed_model_id()}")

    def Streaming(self, req):
        for i in range(3):
            yield pb2.UserDefinedResponse(greeting=f"{req.name}-{i}", num_x2=i)


@pytest.fixture(scope="module")
def app_module(tmp_path_factory):
    """The app module must be importable BEFORE the cluster starts: workers inherit
    the driver's code search path when they are spawned (as in the reference)."""
    tmp = tmp_path_factory.mktemp("serve_cfg")
    name = f"serve_cfg_app_{os.getpid()}"
    (tmp / f"{name}.py").write_text(APP_MODULE)
    sys.path.insert(0, str(tmp))
    yield name, tmp
    sys.path.remove(str(tmp))


@pytest.fixture(scope="module")
def cluster(app_module):
    ray.init(num_cpus=6, include_dashboard=False)
    yield
    serve.shutdown()
    ray.shutdown()


def test_grpc_proxy_unary_stream_multiplex_and_errors(cluster):
    serve.start(grpc_options=serve.gRPCOptions(
        port=0, grpc_servicer_functions=["_grpc_user_pb2.add_UserDefinedServiceServicer_to_server"]),
        proxy_location="Disabled")
    serve.run(GrpcDeployment.bind(), name="grpcapp", route_prefix=None)
    ch = grpc.insecure_channel(f"127.0.0.1:{serve.grpc_port()}")
    stub = pb2.UserDefinedServiceStub(ch)
    md = (("application", "grpcapp"),)
    r = stub.__call__(pb2.UserDefinedMessage(name="amd", num=21), metadata=md, timeout=30)
    assert r.greeting == "Hello amd" and r.num_x2 == 42
    r = stub.__call__(pb2.UserDefinedMessage(name="solo", num=1), timeout=30)  # only app: no metadata needed
    assert r.greeting == "Hello solo"
    r = stub.Multiplexing(pb2.UserDefinedMessage(), metadata=md + (("multiplexed_model_id", "m7"),), timeout=30)
    assert r.greeting == "model=m7"
    outs = list(stub.Streaming(pb2.UserDefinedMessage(name="s"), metadata=md, timeout=30))
    assert [o.greeting for o in outs] == ["s-0", "s-1", "s-2"]
    with pytest.raises(grpc.RpcError) as e:
        stub.__call__(pb2.UserDefinedMessage(name="boom"), metadata=md, timeout=30)
    assert e.value.code() == grpc.StatusCode.INTERNAL and "boom requested" in e.value.details()
    with pytest.raises(grpc.RpcError) as e:
        stub.__call__(pb2.UserDefinedMessage(name="x"), metadata=(("application", "nope"),), timeout=30)
    assert e.value.code() == grpc.StatusCode.NOT_FOUND
    api = api_pb2.RayServeAPIServiceStub(ch)
    assert list(api.ListApplications(api_pb2.ListApplicationsRequest(), timeout=30).application_names) == \
        ["grpcapp"]
    assert api.Healthz(api_pb2.HealthzRequest(), timeout=30).message == "success"
    serve.delete("grpcapp")


APP_MODULE = textwrap.dedent('''
    from cluster_anywhere_amd import serve

    @serve.deployment
    class Doubler:
        def __init__(self):
            self.factor = 2

        def reconfigure(self, cfg):
            self.factor = cfg.get("factor", 2)

        def __call__(self, x):
            return x * self.factor

    @serve.deployment
    class Ingress:
        def __init__(self, doubler, greeting="hi"):
            self.doubler = doubler
            self.greeting = greeting

        async def __call__(self, request):
            x = int(request.query_params.get("x", "1"))
            return {"greeting": self.greeting, "y": await self.doubler.remote(x)}

    app = Ingress.bind(Doubler.bind())

    def builder(args):
        return Ingress.bind(Doubler.bind(), greeting=args.get("greeting", "built"))
''')


def test_schema_validation():
    ok = {"applications": [{"name": "a", "route_prefix": "/a", "import_path": "m:app"}]}
    ServeDeploySchema.model_validate(ok)
    bad = [
        {"applications": [{"name": "a", "import_path": "m:app"}, {"name": "a", "route_prefix": "/b",
                                                                  "import_path": "m:app"}]},
        {"applications": [{"name": "a", "route_prefix": "a", "import_path": "m:app"}]},
        {"applications": [{"name": "a", "import_path": "m:app", "deployments": [
            {"name": "D", "num_replicas": 2, "autoscaling_config": {"max_replicas": 3}}]}]},
        {"applications": [{"name": "a", "import_path": "m:app", "bogus": 1}]},
    ]
    for b in bad:
        with pytest.raises(Exception):
            ServeDeploySchema.model_validate(b)


def test_deploy_config_overrides_and_redeploy(cluster, app_module):
    mod, _ = app_module
    port = _free_port()
    cfg = {"http_options": {"port": port}, "applications": [
        {"name": "calc", "route_prefix": "/calc", "import_path": f"{mod}:app",
         "deployments": [{"name": "Doubler", "num_replicas": 2, "user_config": {"factor": 5}}]},
        {"name": "built", "route_prefix": "/built", "import_path": f"{mod}:builder", "args": {"greeting": "yo"}}]}
    deploy_config(cfg)
    st = serve.status().applications
    assert st["calc"].status == "RUNNING" and st["calc"].deployments["Doubler"].running_replicas == 2
    hp = serve.http_port()
    out = _get(f"http://127.0.0.1:{hp}/calc?x=3")
    assert out == {"greeting": "hi", "y": 15}
    out = _get(f"http://127.0.0.1:{hp}/built?x=2")
    assert out == {"greeting": "yo", "y": 4}
    # redeploy: only "calc", new factor -> "built" is deleted, calc reconfigured
    cfg["applications"] = cfg["applications"][:1]
    cfg["applications"][0]["deployments"][0]["user_config"] = {"factor": 10}
    deploy_config(cfg)
    assert "built" not in serve.status().applications
    out = _get(f"http://127.0.0.1:{hp}/calc?x=3")
    assert out["y"] == 30
    from cluster_anywhere_amd.serve import scripts

    assert scripts.main(["config"]) == 0
    assert scripts.main(["status"]) == 0
    serve.delete("calc")


def test_build_config_and_cli_build(app_module):
    mod, tmp = app_module
    cfg = build_config([f"{mod}:app"])
    assert cfg["applications"][0]["import_path"] == f"{mod}:app"
    names = [d["name"] for d in cfg["applications"][0]["deployments"]]
    assert set(names) == {"Ingress", "Doubler"}
    out = tmp / "serve.yaml"
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, str(tmp)]))
    subprocess.run([sys.executable, "-m", "cluster_anywhere_amd", "serve", "build", f"{mod}:app", "-o", str(out)],
                   check=True, env=env, cwd=str(tmp), timeout=120)
    parsed = ServeDeploySchema.model_validate(yaml.safe_load(out.read_text()))
    assert parsed.applications[0].name == "default"


def test_cli_deploy_status_shutdown_against_a_cluster(app_module):
    from cluster_anywhere_amd.cluster_utils import Cluster

    mod, tmp = app_module
    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 4})
    try:
        port = _free_port()
        (tmp / "cfg.yaml").write_text(yaml.safe_dump({"http_options": {"port": port}, "applications": [
            {"name": "cli", "route_prefix": "/", "import_path": f"{mod}:app",
             "deployments": [{"name": "Doubler", "user_config": {"factor": 3}}]}]}))
        env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, str(tmp)]))
        run = lambda *a: subprocess.run([sys.executable, "-m", "cluster_anywhere_amd", "serve", *a,  # noqa: E731
                                         "-a", c.address], env=env, cwd=str(tmp), timeout=180,
                                        capture_output=True, text=True)
        r = run("deploy", "cfg.yaml")
        assert r.returncode == 0, r.stderr[-2000:]
        deadline = time.time() + 60
        while True:
            try:
                out = json.loads(urllib.request.urlopen(f"http://127.0.0.1:{port}/?x=4", timeout=10).read())
                break
            except Exception:
                if time.time() > deadline:
                    raise
                time.sleep(0.3)
        assert out["y"] == 12
        r = run("status")
        st = yaml.safe_load(r.stdout)
        assert st["applications"]["cli"]["status"] == "RUNNING"
        r = run("config")
        assert yaml.safe_load(r.stdout)["name"] == "cli"
        r = run("shutdown", "-y")
        assert r.returncode == 0, r.stderr[-2000:]
    finally:
        c.shutdown()
