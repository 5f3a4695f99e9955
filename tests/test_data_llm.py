"""``data.llm`` batch processors (reference: python/ray/llm/tests/batch/ —
test_processor_base.py, stages/test_base.py, test_chat_template_stage.py,
test_tokenize_stage.py, test_http_request_stage.py, test_prepare_image_stage.py).

CPU: the engine stage runs llama-tiny in fp32 with the byte tokenizer; the HTTP
stage talks to a local HTTP server (there is no network)."""
import asyncio
import base64
import io
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data as rd
from cluster_anywhere_amd.data.llm import (EngineProcessorConfig, HttpRequestProcessorConfig, ProcessorConfig,
                                           build_llm_processor)
from cluster_anywhere_amd.llm.batch import (ChatTemplateStage, DetokenizeStage, Processor, StatefulStage,
                                            StatefulStageUDF, TokenizeStage)
from cluster_anywhere_amd.llm.batch.stages import PrepareImageUDF


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _drain(udf, batch):
    async def go():
        return [o async for o in udf(batch)]
    return asyncio.new_event_loop().run_until_complete(go())


# ------------------------------------------------------------ stage base
class _Reverse(StatefulStageUDF):
    """Emits rows in reverse order (the wrapper must realign them)."""

    def __init__(self, data_column, factor=1):
        super().__init__(data_column)
        self.factor = factor

    async def udf(self, rows):
        for r in reversed(rows):
            yield {self.IDX_IN_BATCH_COLUMN: r[self.IDX_IN_BATCH_COLUMN], "y": r["x"] * self.factor}

    @property
    def expected_input_keys(self):
        return ["x"]


class _Stage(StatefulStage):
    fn: type = _Reverse


def test_stage_udf_realigns_out_of_order_rows():
    out = _drain(_Reverse("__data", 3), {"__data": [{"x": 1, "k": "a"}, {"x": 2, "k": "b"}]})
    rows = [o["__data"][0] for o in out]
    assert rows == [{"x": 2, "k": "b", "y": 6}, {"x": 1, "k": "a", "y": 3}]


def test_stage_udf_errors():
    with pytest.raises(ValueError, match="Required input keys"):
        _drain(_Reverse("__data"), {"__data": [{"z": 1}]})
    with pytest.raises(ValueError, match="reserved"):
        _drain(_Reverse("__data"), {"__data": [{"x": 1, "__idx_in_batch": 0}]})

    class Dup(StatefulStageUDF):
        async def udf(self, rows):
            for _ in range(2):
                yield {self.IDX_IN_BATCH_COLUMN: 0}

    with pytest.raises(ValueError, match="more than once"):
        _drain(Dup("__data"), {"__data": [{"x": 1}]})

    class Drop(StatefulStageUDF):
        async def udf(self, rows):
            yield {self.IDX_IN_BATCH_COLUMN: 0}

    with pytest.raises(ValueError, match="never produced"):
        _drain(Drop("__data"), {"__data": [{"x": 1}, {"x": 2}]})


def test_stage_map_batches_kwargs():
    st = _Stage(fn_constructor_kwargs={"factor": 2}, map_batches_kwargs={"concurrency": 3, "batch_size": 5})
    kw = st.get_dataset_map_batches_kwargs(batch_size=8, data_column="__data")
    assert kw["batch_size"] == 8 and kw["concurrency"] == 3
    assert kw["fn_constructor_kwargs"] == {"factor": 2, "data_column": "__data"}
    bad = _Stage(fn_constructor_kwargs={"data_column": "x"})
    with pytest.raises(ValueError, match="data_column"):
        bad.get_dataset_map_batches_kwargs(batch_size=8, data_column="__data")


def test_processor_pipeline_and_stage_names(cluster):
    cfg = ProcessorConfig(batch_size=4)
    proc = Processor(cfg, [_Stage(fn_constructor_kwargs={"factor": 2}), _Stage(fn_constructor_kwargs={})],
                     preprocess=lambda r: {"x": r["id"] + 1},
                     postprocess=lambda r: {"id": r["id"], "y": r["y"], "x": r["x"]})
    assert proc.list_stage_names() == ["_Stage", "_Stage_2"]
    assert proc.get_stage_by_name("_Stage_2").fn is _Reverse
    with pytest.raises(ValueError):
        proc.get_stage_by_name("nope")
    rows = sorted(proc(rd.range(10)).take_all(), key=lambda r: r["id"])
    # the second stage overwrites y with x * 1 (later stages win on shared keys)
    assert rows == [{"id": i, "x": i + 1, "y": i + 1} for i in range(10)]


def test_builder_registry_and_override():
    with pytest.raises(ValueError, match="not registered"):
        build_llm_processor(ProcessorConfig(batch_size=1))
    seen = []
    proc = build_llm_processor(EngineProcessorConfig(batch_size=2, detokenize=False),
                               override_stage_config_fn=lambda n, s: seen.append(n))
    assert seen == ["ChatTemplateStage", "TokenizeStage", "EngineStage"]
    assert proc.list_stage_names() == seen


# ------------------------------------------------------------ text stages
def test_chat_template_tokenize_detokenize_roundtrip(cluster):
    cfg = ProcessorConfig(batch_size=3)
    proc = Processor(cfg, [ChatTemplateStage(), TokenizeStage(),
                           _Copy(fn_constructor_kwargs={}), DetokenizeStage()],
                     preprocess=lambda r: {"messages": [{"role": "system", "content": "be brief"},
                                                        {"role": "user", "content": f"q{r['id']}"}]},
                     postprocess=lambda r: {"id": r["id"], "prompt": r["prompt"], "text": r["generated_text"],
                                            "n": len(r["tokenized_prompt"])})
    rows = sorted(proc(rd.range(7)).take_all(), key=lambda r: r["id"])
    for r in rows:
        want = f"<|system|>be brief\n<|user|>q{r['id']}\n<|assistant|>"
        assert r["prompt"] == want
        assert r["text"] == want  # detokenize(tokenize(p)) == p; BOS dropped
        assert r["n"] == len(want.encode()) + 1


class _CopyUDF(StatefulStageUDF):
    async def udf(self, rows):
        for r in rows:
            yield {self.IDX_IN_BATCH_COLUMN: r[self.IDX_IN_BATCH_COLUMN],
                   "generated_tokens": list(r["tokenized_prompt"])}


class _Copy(StatefulStage):
    fn: type = _CopyUDF


# ------------------------------------------------------------ HTTP stage
class _Handler(BaseHTTPRequestHandler):
    fails = {}
    lock = threading.Lock()

    def do_POST(self):
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        key = body.get("id")
        with self.lock:
            n = self.fails.get(key, 0)
            if key is not None and key % 5 == 0 and n == 0:  # every 5th row: one 503 first
                self.fails[key] = 1
                self.send_response(503)
                self.end_headers()
                return
        out = json.dumps({"echo": body, "auth": self.headers.get("Authorization"),
                          "choices": [{"message": {"content": f"answer {key}"}}]}).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(out)))
        self.end_headers()
        self.wfile.write(out)

    def log_message(self, *a):
        pass


@pytest.fixture(scope="module")
def server():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield f"http://127.0.0.1:{srv.server_address[1]}/v1/chat/completions"
    srv.shutdown()


def test_http_request_processor(cluster, server):
    cfg = HttpRequestProcessorConfig(url=server, headers={"Authorization": "Bearer t"}, batch_size=4,
                                     concurrency=2, qps=200)
    proc = build_llm_processor(
        cfg, preprocess=lambda r: dict(model="m", id=r["id"],
                                       messages=[{"role": "user", "content": f"{r['id']} ** 3 = ?"}]),
        postprocess=lambda r: dict(id=r["id"], resp=r["choices"][0]["message"]["content"], auth=r["auth"],
                                   sent=r["echo"]["messages"][0]["content"]))
    rows = sorted(proc(rd.range(12)).take_all(), key=lambda r: r["id"])
    assert [r["resp"] for r in rows] == [f"answer {i}" for i in range(12)]
    assert all(r["auth"] == "Bearer t" for r in rows)
    assert rows[3]["sent"] == "3 ** 3 = ?"
    assert _Handler.fails  # 503s happened and were retried


# ------------------------------------------------------------ image stage
def test_prepare_image_stage(tmp_path):
    from PIL import Image

    img = Image.new("RGB", (8, 6), (255, 0, 0))
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    url = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
    p = tmp_path / "x.png"
    img.save(p)
    msgs = [{"role": "user", "content": [{"type": "text", "text": "what?"},
                                         {"type": "image_url", "image_url": {"url": url}},
                                         {"type": "image", "image": str(p)}]}]
    out = _drain(PrepareImageUDF("__data", resize=[4, 4]), {"__data": [{"messages": msgs}, {"messages": []}]})
    rows = [o["__data"][0] for o in out]
    assert rows[0]["image_sizes"] == [(4, 4), (4, 4)] and rows[0]["image"][0].mode == "RGB"
    assert rows[1]["image"] == []
    assert PrepareImageUDF.extract_image_info(msgs) == [url, str(p)]


# ------------------------------------------------------------ engine stage
def test_engine_processor_matches_engine_greedy(cluster):
    from cluster_anywhere_amd.llm import SamplingParams
    from cluster_anywhere_amd.llm.build import build_engine

    cfg = EngineProcessorConfig(model="llama-tiny", batch_size=3, concurrency=1,
                                sampling_params=dict(max_tokens=6, temperature=0.0, ignore_eos=True),
                                engine_kwargs=dict(max_model_len=256))
    proc = build_llm_processor(
        cfg, preprocess=lambda r: dict(messages=[{"role": "user", "content": f"count to {r['id']}"}],
                                       sampling_params=dict(max_tokens=4 + r["id"] % 3)),
        postprocess=lambda r: dict(id=r["id"], toks=list(r["generated_tokens"]), text=r["generated_text"],
                                   prompt=r["prompt"], n=r["num_generated_tokens"]))
    rows = sorted(proc(rd.range(5)).take_all(), key=lambda r: r["id"])
    eng, tok = build_engine("llama-tiny", engine_kwargs=dict(max_model_len=256), device="cpu")
    for r in rows:
        n = 4 + r["id"] % 3
        ref = eng.generate([tok.encode(r["prompt"])], SamplingParams(max_tokens=n, ignore_eos=True))[0]
        assert [int(t) for t in r["toks"]] == ref.output_token_ids and r["n"] == n
        assert r["text"] == tok.decode(ref.output_token_ids)
