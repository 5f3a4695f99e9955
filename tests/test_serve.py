"""Serve: deployments, handles + composition, HTTP proxy, FastAPI ingress,
@serve.batch, streaming, multiplexing, user_config, autoscaling, replica
failure recovery (reference: python/ray/serve/tests/test_api.py,
test_handle_api.py, test_batching.py, test_multiplex.py,
test_autoscaling_policy.py, test_streaming_response.py)."""
import asyncio
import json
import os
import time
import urllib.request

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import serve


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8)
    serve.start(http_options={"port": 0})
    yield
    serve.shutdown()
    ray.shutdown()


def _http(path, data=None, headers=None):
    port = serve.http_port()
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=data, headers=headers or {})
    with urllib.request.urlopen(req, timeout=30) as r:
        return r.status, r.read()


@serve.deployment
def hello(request):
    return "hello " + request.query_params.get("name", "world")


def test_function_deployment_http(cluster):
    h = serve.run(hello.bind(), name="hello", route_prefix="/hello")
    assert _http("/hello?name=mi355x") == (200, b"hello mi355x")
    assert _http("/-/healthz") == (200, b"success")
    st = serve.status()
    assert st.applications["hello"].status == "RUNNING"
    serve.delete("hello")
    assert "hello" not in serve.status().applications


@serve.deployment(num_replicas=2)
class Adder:
    def __init__(self, inc):
        self.inc = inc

    def __call__(self, x):
        return x + self.inc

    def pid(self):
        return os.getpid()


@serve.deployment
class Pipeline:
    def __init__(self, a, b):
        self.a, self.b = a, b

    async def __call__(self, x):
        y = await self.a.remote(x)
        return await self.b.remote(y)


def test_composition_and_routing(cluster):
    app = Pipeline.bind(Adder.bind(1), Adder.options(name="Adder2").bind(10))
    h = serve.run(app, name="pipe", route_prefix=None)
    assert h.remote(5).result() == 16
    assert [r.result() for r in [h.remote(i) for i in range(20)]] == [i + 11 for i in range(20)]
    # both replicas of a deployment receive traffic
    ah = serve.get_deployment_handle("Adder", "pipe")
    pids = {ah.pid.remote().result() for _ in range(30)}
    assert len(pids) == 2
    # responses can be passed into other calls unresolved
    assert ah.remote(ah.remote(1)).result() == 3
    serve.delete("pipe")


@serve.deployment(max_ongoing_requests=32)
class Batcher:
    def __init__(self):
        self.sizes = []

    @serve.batch(max_batch_size=8, batch_wait_timeout_s=0.05)
    async def __call__(self, xs):
        self.sizes.append(len(xs))
        return [x * 2 for x in xs]

    def sizes_seen(self):
        return self.sizes


def test_batching(cluster):
    h = serve.run(Batcher.bind(), name="batch", route_prefix=None)
    rs = [h.remote(i) for i in range(16)]
    assert [r.result() for r in rs] == [2 * i for i in range(16)]
    sizes = h.sizes_seen.remote().result()
    assert max(sizes) > 1 and sum(sizes) == 16
    serve.delete("batch")


@serve.deployment
class Streamer:
    def __call__(self, n):
        for i in range(n):
            yield i

    async def agen(self, n):
        for i in range(n):
            await asyncio.sleep(0.001)
            yield f"tok{i}"


def test_streaming(cluster):
    h = serve.run(Streamer.bind(), name="stream", route_prefix=None)
    assert list(h.options(stream=True).remote(5)) == [0, 1, 2, 3, 4]
    assert list(h.options(stream=True, method_name="agen").remote(3)) == ["tok0", "tok1", "tok2"]
    serve.delete("stream")


@serve.deployment(num_replicas=2)
class Multi:
    @serve.multiplexed(max_num_models_per_replica=2)
    async def get_model(self, model_id):
        return {"id": model_id, "pid": os.getpid()}

    async def __call__(self, x):
        m = await self.get_model(serve.get_multiplexed_model_id())
        return m["id"], m["pid"], x


def test_multiplexing(cluster):
    h = serve.run(Multi.bind(), name="mux", route_prefix=None)
    r = h.options(multiplexed_model_id="m1").remote(1).result()
    assert r[0] == "m1"
    time.sleep(1.2)  # replica reports its loaded models to the controller
    pids = {h.options(multiplexed_model_id="m1").remote(i).result()[1] for i in range(10)}
    assert pids == {r[1]}
    serve.delete("mux")


@serve.deployment(user_config={"threshold": 1})
class Configurable:
    def __init__(self):
        self.t = None

    def reconfigure(self, cfg):
        self.t = cfg["threshold"]

    def __call__(self, _):
        return self.t


def test_user_config_update(cluster):
    h = serve.run(Configurable.options(version="v1").bind(), name="cfg", route_prefix=None)
    assert h.remote(0).result() == 1
    h = serve.run(Configurable.options(version="v1", user_config={"threshold": 7}).bind(), name="cfg",
                  route_prefix=None)
    deadline = time.time() + 10
    while h.remote(0).result() != 7 and time.time() < deadline:
        time.sleep(0.05)
    assert h.remote(0).result() == 7
    serve.delete("cfg")


def test_fastapi_ingress(cluster):
    from fastapi import FastAPI

    api = FastAPI()

    @serve.deployment
    @serve.ingress(api)
    class Api:
        def __init__(self, greeting):
            self.greeting = greeting

        @api.get("/hi/{name}")
        def hi(self, name: str):
            return {"msg": f"{self.greeting} {name}"}

        @api.post("/sum")
        async def sum_(self, body: dict):
            return {"sum": sum(body["xs"])}

    serve.run(Api.bind("hey"), name="api", route_prefix="/api")
    st, body = _http("/api/hi/amd")
    assert st == 200 and json.loads(body) == {"msg": "hey amd"}
    st, body = _http("/api/sum", data=json.dumps({"xs": [1, 2, 3]}).encode(),
                     headers={"content-type": "application/json"})
    assert json.loads(body) == {"sum": 6}
    serve.delete("api")


@serve.deployment(autoscaling_config={"min_replicas": 1, "max_replicas": 3, "target_ongoing_requests": 1,
                                      "upscale_delay_s": 0.2, "downscale_delay_s": 0.5,
                                      "metrics_interval_s": 0.1, "look_back_period_s": 0.5},
                  max_ongoing_requests=10)
class Slow:
    async def __call__(self, t):
        await asyncio.sleep(t)
        return os.getpid()


def test_autoscaling(cluster):
    h = serve.run(Slow.bind(), name="auto", route_prefix=None)
    assert serve.status().applications["auto"].deployments["Slow"].running_replicas == 1
    rs = [h.remote(3.0) for _ in range(8)]
    deadline = time.time() + 20
    peak = 1
    while time.time() < deadline:
        peak = max(peak, serve.status().applications["auto"].deployments["Slow"].target_replicas)
        if peak >= 2:
            break
        time.sleep(0.1)
    assert peak >= 2
    [r.result() for r in rs]
    deadline = time.time() + 20
    while time.time() < deadline:
        if serve.status().applications["auto"].deployments["Slow"].target_replicas == 1:
            break
        time.sleep(0.2)
    assert serve.status().applications["auto"].deployments["Slow"].target_replicas == 1
    serve.delete("auto")


@serve.deployment(health_check_period_s=0.2, health_check_timeout_s=2)
class Fragile:
    def __call__(self, die=False):
        if die:
            os._exit(1)
        return os.getpid()


def test_replica_failure_recovery(cluster):
    h = serve.run(Fragile.bind(), name="frag", route_prefix=None)
    pid = h.remote().result()
    with pytest.raises(Exception):
        h.remote(True).result(_retries=0)
    deadline = time.time() + 30
    new = None
    while time.time() < deadline:
        try:
            new = h.remote().result(timeout_s=5)
            if new != pid:
                break
        except Exception:
            time.sleep(0.2)
    assert new is not None and new != pid
    serve.delete("frag")


def test_llm_openai_app(cluster, tmp_path):
    from cluster_anywhere_amd.serve.llm import LLMConfig, build_openai_app

    app = build_openai_app({"llm_configs": [LLMConfig(model_id="llama-tiny",
                                                      engine_kwargs={"max_model_len": 256})]})
    serve.run(app, name="llm", route_prefix="/llm")
    st, body = _http("/llm/v1/models")
    assert json.loads(body)["data"][0]["id"] == "llama-tiny"
    req = {"model": "llama-tiny", "prompt": "hello", "max_tokens": 7}
    st, body = _http("/llm/v1/completions", data=json.dumps(req).encode(),
                     headers={"content-type": "application/json"})
    r = json.loads(body)
    assert st == 200 and r["usage"]["completion_tokens"] == 7 and r["usage"]["prompt_tokens"] == 6
    # concurrent requests share the engine (continuous batching) and stay deterministic (greedy)
    h = serve.get_deployment_handle("LLMServer:llama-tiny", "llm")
    outs = [h.generate.remote(dict(req)) for _ in range(6)]
    ids = [o.result()["choices"][0]["token_ids"] for o in outs]
    assert all(i == r["choices"][0]["token_ids"] for i in ids)
    # streaming deltas concatenate to the full completion
    deltas = list(h.options(stream=True, method_name="stream").remote(dict(req)))
    assert sum((d["token_ids"] for d in deltas), []) == ids[0]
    st, body = _http("/llm/v1/chat/completions", data=json.dumps(
        {"model": "llama-tiny", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 3}).encode(),
        headers={"content-type": "application/json"})
    assert json.loads(body)["usage"]["completion_tokens"] == 3
    _check_sse_streams_before_done("/llm/v1/completions",
                                   {"model": "llama-tiny", "prompt": "hello", "max_tokens": 96, "ignore_eos": True,
                                    "stream": True}, lambda c: c["choices"][0]["text"])
    _check_sse_streams_before_done("/llm/v1/chat/completions",
                                   {"model": "llama-tiny", "messages": [{"role": "user", "content": "hi"}],
                                    "max_tokens": 96, "ignore_eos": True, "stream": True},
                                   lambda c: c["choices"][0]["delta"].get("content", ""))
    serve.delete("llm")


def _check_sse_streams_before_done(path, req, text_of):
    """The first SSE event reaches the client while the generation is still running
    (not collected and sent at the end): its arrival is well before the [DONE]."""
    port = serve.http_port()
    r = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=json.dumps(req).encode(),
                               headers={"content-type": "application/json"})
    t0 = time.time()
    events, t_first = [], None
    with urllib.request.urlopen(r, timeout=60) as resp:
        assert resp.headers.get("content-type", "").startswith("text/event-stream")
        for raw in resp:
            line = raw.decode().strip()
            if not line.startswith("data: "):
                continue
            if t_first is None:
                t_first = time.time() - t0
            if line == "data: [DONE]":
                break
            events.append(json.loads(line[6:]))
    t_done = time.time() - t0
    assert len(events) > 10, events[:3]
    assert t_first < 0.5 * t_done, (t_first, t_done)
    assert sum(len(text_of(e)) for e in events) > 0


@serve.deployment(num_replicas=2)
class Stateful:
    def __init__(self):
        self.n = 0

    def __call__(self, request):
        self.n += 1
        return f"ok {os.getpid()}"


def test_controller_crash_recovery(cluster):
    """The controller checkpoints to the internal KV, restarts without limit and
    re-attaches to its (detached, named) replicas: HTTP keeps being served while it
    is down and after it comes back, with the same replicas (reference:
    serve/_private/controller.py:509 _recover_state_from_checkpoint)."""
    from cluster_anywhere_amd.serve.controller import CONTROLLER_NAME, NAMESPACE

    serve.run(Stateful.bind(), name="ft", route_prefix="/ft")
    assert _http("/ft")[0] == 200
    before = serve.status().applications["ft"].deployments["Stateful"].replica_states
    assert len(before) == 2
    ctl = ray.get_actor(CONTROLLER_NAME, namespace=NAMESPACE)
    old_pid = ray.get(ctl.pid.remote())
    ray.kill(ctl, no_restart=False)
    # the proxy and replicas do not depend on the controller for the data path
    served = 0
    t_end = time.time() + 3
    while time.time() < t_end:
        assert _http("/ft")[0] == 200
        served += 1
    assert served > 0
    ctl = ray.get_actor(CONTROLLER_NAME, namespace=NAMESPACE)
    deadline = time.time() + 60
    while time.time() < deadline:
        try:
            if ray.get(ctl.is_recovered.remote(), timeout=10):
                break
        except Exception:
            pass
        time.sleep(0.2)
    assert ray.get(ctl.is_recovered.remote())
    assert ray.get(ctl.pid.remote()) != old_pid  # a new controller process
    deadline = time.time() + 30
    while time.time() < deadline:
        st = serve.status().applications.get("ft")
        if st and st.status == "RUNNING":
            break
        time.sleep(0.1)
    after = serve.status().applications["ft"].deployments["Stateful"].replica_states
    assert set(after) == set(before), (before, after)  # same replicas, re-attached
    assert _http("/ft")[0] == 200
    # the recovered controller keeps managing the app
    serve.delete("ft")
    assert "ft" not in serve.status().applications
