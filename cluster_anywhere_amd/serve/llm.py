"""Serve LLM: an OpenAI-compatible LLM deployment over the native engine
(reference: python/ray/serve/llm.py, python/ray/llm/_internal/serve/
deployments/llm/llm_server.py, routers/router.py).

``LLMServer`` (one replica per GPU, ``num_gpus=1``) owns an ``AsyncLLMEngine``;
``build_openai_app`` wires ``/v1/completions``, ``/v1/chat/completions`` and
``/v1/models`` through a FastAPI ingress (``LLMRouter``) that load-balances to
the LLMServer replicas via handles (streaming with ``stream=True``)."""

import json
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

from .deployment import Application, deployment, ingress


@dataclass
class LLMConfig:
    model_id: str = "llama-tiny"
    model_source: Optional[str] = None  # local HF checkpoint dir; None -> random init of model_id preset
    tokenizer_source: Optional[str] = None
    dtype: str = "bfloat16"
    engine_kwargs: Dict[str, Any] = field(default_factory=dict)
    deployment_config: Dict[str, Any] = field(default_factory=dict)
    accelerator_type: Optional[str] = None
    seed: int = 0


def _build_engine(cfg: LLMConfig):
    from ..llm.async_engine import AsyncLLMEngine
    from ..llm.build import build_engine

    eng, tok = build_engine(cfg.model_id, cfg.model_source, cfg.tokenizer_source, cfg.dtype,
                            cfg.engine_kwargs, cfg.seed)
    return AsyncLLMEngine(eng), tok


def _sampling(body: Dict):
    from ..llm import SamplingParams

    stop = body.get("stop_token_ids") or []
    return SamplingParams(max_tokens=int(body.get("max_tokens", 16)), temperature=float(body.get("temperature", 0.0)),
                          top_p=float(body.get("top_p", 1.0)), top_k=int(body.get("top_k", -1)),
                          stop_token_ids=list(stop), ignore_eos=bool(body.get("ignore_eos", False)),
                          seed=body.get("seed"))


class LLMServer:
    """One engine replica. ``generate`` returns a completion dict;
    ``stream`` yields text deltas."""

    def __init__(self, llm_config: Union[LLMConfig, Dict]):
        if isinstance(llm_config, dict):
            llm_config = LLMConfig(**llm_config)
        self.config = llm_config
        self.engine, self.tokenizer = _build_engine(llm_config)
        self.model_id = llm_config.model_id

    def _prompt_ids(self, body: Dict) -> List[int]:
        if "prompt_token_ids" in body:
            return list(body["prompt_token_ids"])
        if "messages" in body:
            text = self.tokenizer.apply_chat_template(list(body["messages"]), tokenize=False,
                                                      add_generation_prompt=True)
        else:
            text = body.get("prompt", "")
        return self.tokenizer.encode(text)

    async def generate(self, body: Dict) -> Dict:
        ids = self._prompt_ids(body)
        final = None
        async for o in self.engine.generate(ids, _sampling(body)):
            final = o
        text = self.tokenizer.decode(final.output_token_ids)
        return {"id": f"cmpl-{uuid.uuid4().hex[:12]}", "object": "text_completion", "created": int(time.time()),
                "model": self.model_id,
                "choices": [{"index": 0, "text": text, "token_ids": final.output_token_ids,
                             "finish_reason": final.finish_reason}],
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(final.output_token_ids),
                          "total_tokens": len(ids) + len(final.output_token_ids)}}

    async def stream(self, body: Dict):
        ids = self._prompt_ids(body)
        sent = 0
        async for o in self.engine.generate(ids, _sampling(body)):
            new = o.output_token_ids[sent:]
            sent = len(o.output_token_ids)
            yield {"token_ids": new, "text": self.tokenizer.decode(new), "finish_reason": o.finish_reason}

    def stats(self):
        return dict(self.engine.engine.stats)

    def check_health(self):
        if self.engine.error is not None:
            raise RuntimeError(f"engine failed: {self.engine.error}")


def _sse(obj) -> str:
    return "data: " + json.dumps(obj) + "\n\n"


def _router_cls():
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse, StreamingResponse

    api = FastAPI()

    @ingress(api)
    class LLMRouter:
        def __init__(self, servers: Dict[str, Any]):
            self.servers = servers

        def _server(self, body):
            mid = body.get("model") or next(iter(self.servers))
            if mid not in self.servers:
                return None
            return self.servers[mid]

        @api.get("/v1/models")
        async def models(self):
            return {"object": "list", "data": [{"id": m, "object": "model", "owned_by": "cluster_anywhere_amd"}
                                                for m in self.servers]}

        @api.post("/v1/completions")
        async def completions(self, request: Request):
            body = await request.json()
            h = self._server(body)
            if h is None:
                return JSONResponse({"error": f"unknown model {body.get('model')}"}, status_code=404)
            if body.get("stream"):
                cid, created = f"cmpl-{uuid.uuid4().hex[:12]}", int(time.time())
                model = body.get("model") or next(iter(self.servers))

                async def sse():
                    # one SSE event per engine step, written as soon as the replica yields it
                    async for d in h.options(stream=True, method_name="stream").remote(body):
                        yield _sse({"id": cid, "object": "text_completion", "created": created, "model": model,
                                    "choices": [{"index": 0, "text": d["text"], "token_ids": d["token_ids"],
                                                 "finish_reason": d["finish_reason"]}]})
                    yield "data: [DONE]\n\n"

                return StreamingResponse(sse(), media_type="text/event-stream")
            return await h.generate.remote(body)

        @api.post("/v1/chat/completions")
        async def chat(self, request: Request):
            body = await request.json()
            h = self._server(body)
            if h is None:
                return JSONResponse({"error": f"unknown model {body.get('model')}"}, status_code=404)
            if body.get("stream"):
                cid, created = f"chatcmpl-{uuid.uuid4().hex[:12]}", int(time.time())
                model = body.get("model") or next(iter(self.servers))

                async def sse():
                    head = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model}
                    yield _sse(dict(head, choices=[{"index": 0, "delta": {"role": "assistant"},
                                                    "finish_reason": None}]))
                    async for d in h.options(stream=True, method_name="stream").remote(body):
                        yield _sse(dict(head, choices=[{"index": 0, "delta": {"content": d["text"]},
                                                        "finish_reason": d["finish_reason"]}]))
                    yield "data: [DONE]\n\n"

                return StreamingResponse(sse(), media_type="text/event-stream")
            r = await h.generate.remote(body)
            c = r["choices"][0]
            return {"id": r["id"].replace("cmpl", "chatcmpl"), "object": "chat.completion", "created": r["created"],
                    "model": r["model"], "usage": r["usage"],
                    "choices": [{"index": 0, "message": {"role": "assistant", "content": c["text"]},
                                 "finish_reason": c["finish_reason"]}]}

    return LLMRouter


def build_llm_deployment(llm_config: LLMConfig, *, name_prefix: str = "LLMServer:") -> Application:
    import torch

    dc = {"max_ongoing_requests": 256}
    dc.update(llm_config.deployment_config or {})
    opts = dict(dc.pop("ray_actor_options", {}))
    if torch.cuda.is_available() or opts.get("num_gpus"):
        opts.setdefault("num_gpus", 1)
    d = deployment(LLMServer, name=f"{name_prefix}{llm_config.model_id}")
    return d.options(ray_actor_options=opts, **dc).bind(llm_config)


def build_openai_app(llm_serving_args) -> Application:
    """``llm_serving_args``: an :class:`LLMServingArgs`, ``{"llm_configs": [...]}`` or
    a list of configs."""
    if isinstance(llm_serving_args, dict):
        configs = llm_serving_args.get("llm_configs")
    elif hasattr(llm_serving_args, "llm_configs"):
        configs = llm_serving_args.llm_configs
    else:
        configs = llm_serving_args
    configs = [c if isinstance(c, LLMConfig) else LLMConfig(**c) for c in configs]
    servers = {c.model_id: build_llm_deployment(c) for c in configs}
    Router = deployment(_router_cls(), name="LLMRouter")
    return Router.bind(servers)


# ---- reference names (python/ray/serve/llm.py:19-63) -------------------------------
VLLMDeployment = LLMServer  # the engine deployment class (the in-tree engine, not vLLM)


def LLMModelRouterDeployment(*args, **kwargs):
    """The OpenAI-compatible router deployment class (FastAPI ingress), built lazily
    so importing serve.llm does not import FastAPI."""
    return _router_cls()(*args, **kwargs)


@dataclass
class LLMServingArgs:
    llm_configs: List[Union[LLMConfig, Dict[str, Any]]] = field(default_factory=list)


def build_vllm_deployment(llm_config: LLMConfig) -> Application:
    return build_llm_deployment(llm_config)
