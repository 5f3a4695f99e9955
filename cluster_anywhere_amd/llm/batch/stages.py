"""Batch-LLM stages: stateful ``map_batches`` UDFs composed by a :class:`Processor`.

Reference roles: ``python/ray/llm/_internal/batch/stages/base.py`` (row-wrapping
pre/post-process, ``StatefulStageUDF`` — row-aligned async UDF over the
processor's data column — and ``StatefulStage`` at :233), ``chat_template_stage.py``,
``tokenize_stage.py`` (tokenize + detokenize), ``http_request_stage.py`` and
``prepare_image_stage.py``; the reference's engine stage delegates to vLLM.
Here the engine stage drives the in-tree paged-KV engine (:mod:`..engine`,
gfx950 decode kernels, HIP graphs) inside a GPU actor of the data executor.

Row contract (same as the reference): every stage reads the rows of the
``data_column`` (a column of dicts), runs its UDF over the batch and merges the
UDF's per-row outputs back into those dicts; outputs may arrive out of order
and are matched by ``__idx_in_batch``; every input row must be produced exactly
once.
"""
from __future__ import annotations

import asyncio
import base64
import io
import logging
import os
import time
from typing import Any, AsyncIterator, Callable, Dict, List, Optional, Type

import numpy as np
from pydantic import BaseModel, ConfigDict, Field

logger = logging.getLogger(__name__)


def _plain(v):
    """numpy containers coming out of columnar blocks -> plain Python."""
    if isinstance(v, np.ndarray):
        return [_plain(x) for x in v.tolist()] if v.dtype == object else v.tolist()
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, np.generic):
        return v.item()
    return v


def wrap_preprocess(fn: Callable, data_column: str) -> Callable:
    """Row -> {data_column: row + fn(row)} (reference: stages/base.py:12)."""

    def _preprocess(row: Dict[str, Any]) -> Dict[str, Any]:
        data = dict(row)
        data.update(fn(row))
        return {data_column: data}

    return _preprocess


def wrap_postprocess(fn: Callable, data_column: str) -> Callable:
    """{data_column: row} -> fn(row): the user picks the output columns."""

    def _postprocess(row: Dict[str, Any]) -> Dict[str, Any]:
        if data_column not in row:
            raise ValueError(f"[Internal] {data_column} not found in row {row}")
        return fn(row[data_column])

    return _postprocess


class StatefulStageUDF:
    """Row-aligned async UDF over the processor's data column
    (reference: stages/base.py:65)."""

    IDX_IN_BATCH_COLUMN: str = "__idx_in_batch"

    def __init__(self, data_column: str):
        self.data_column = data_column

    async def __call__(self, batch: Dict[str, Any]) -> AsyncIterator[Dict[str, Any]]:
        if not batch or self.data_column not in batch:
            if not batch:
                return
            raise ValueError(f"[Internal] {self.data_column} not found in batch {list(batch)}")
        col = batch[self.data_column]
        inputs = [dict(r) for r in (col.tolist() if hasattr(col, "tolist") else col)]
        if not inputs:
            return
        self.validate_inputs(inputs)
        for i, row in enumerate(inputs):
            row[self.IDX_IN_BATCH_COLUMN] = i
        left = set(range(len(inputs)))
        # one row per yield: the executor coalesces them into output blocks, so a
        # slow row never holds back the rows finished before it
        async for out in self.udf(inputs):
            if self.IDX_IN_BATCH_COLUMN not in out:
                raise ValueError(f"The output of the UDF must contain the column {self.IDX_IN_BATCH_COLUMN}.")
            i = out.pop(self.IDX_IN_BATCH_COLUMN)
            if i not in left:
                raise ValueError(f"The row {i} is outputed twice. This is likely due to the UDF is not one-to-one.")
            left.remove(i)
            row = inputs[i]
            row.pop(self.IDX_IN_BATCH_COLUMN, None)
            row.update(out)
            yield {self.data_column: [row]}
        if left:
            raise ValueError(f"The rows {sorted(left)} are not outputed.")

    def validate_inputs(self, inputs: List[Dict[str, Any]]):
        need = set(self.expected_input_keys)
        for row in inputs:
            keys = set(row)
            if self.IDX_IN_BATCH_COLUMN in keys:
                raise ValueError(f"The input column {self.IDX_IN_BATCH_COLUMN} is reserved for internal use.")
            missing = need - keys
            if missing:
                raise ValueError(f"Required input keys {missing} not found at the input of "
                                 f"{type(self).__name__}. Input keys: {keys}")

    @property
    def expected_input_keys(self) -> List[str]:
        return []

    async def udf(self, rows: List[Dict[str, Any]]) -> AsyncIterator[Dict[str, Any]]:
        raise NotImplementedError("StageUDF must implement the udf method")
        yield  # pragma: no cover


class StatefulStage(BaseModel):
    """One processor stage: the UDF class, its constructor kwargs and the
    ``map_batches`` kwargs (concurrency, GPUs ...) (reference: stages/base.py:233)."""

    model_config = ConfigDict(arbitrary_types_allowed=True, validate_assignment=True)

    fn: Type[StatefulStageUDF] = Field(description="The stateful UDF class of this stage.")
    fn_constructor_kwargs: Dict[str, Any] = Field(default_factory=dict)
    map_batches_kwargs: Dict[str, Any] = Field(default_factory=lambda: dict(concurrency=1))

    def get_dataset_map_batches_kwargs(self, batch_size: int, data_column: str) -> Dict[str, Any]:
        kw = dict(self.map_batches_kwargs)
        if kw.get("batch_size", batch_size) != batch_size:
            logger.warning("batch_size is set to %d in map_batches_kwargs, but it will be overridden by the "
                           "batch size configured by the processor %d.", kw["batch_size"], batch_size)
        kw["batch_size"] = batch_size
        ctor = dict(self.fn_constructor_kwargs)
        if "data_column" in ctor:
            raise ValueError("'data_column' cannot be used as in fn_constructor_kwargs.")
        ctor["data_column"] = data_column
        kw["fn_constructor_kwargs"] = ctor
        kw.setdefault("num_cpus", 0.25)  # light host stages; the engine stage sets its own
        return kw


# ------------------------------------------------------------ text stages
class ChatTemplateUDF(StatefulStageUDF):
    def __init__(self, data_column: str, model: Optional[str] = None, chat_template: Optional[str] = None):
        from ..tokenizer import load_tokenizer

        super().__init__(data_column)
        self.tokenizer = load_tokenizer(model)
        self.chat_template = chat_template

    async def udf(self, batch):
        prompts = self.tokenizer.apply_chat_template([_plain(r["messages"]) for r in batch], tokenize=False,
                                                     add_generation_prompt=True,
                                                     chat_template=self.chat_template)
        assert len(prompts) == len(batch)
        for row, prompt in zip(batch, prompts):
            yield {self.IDX_IN_BATCH_COLUMN: row[self.IDX_IN_BATCH_COLUMN], "prompt": prompt}

    @property
    def expected_input_keys(self):
        return ["messages"]


class ChatTemplateStage(StatefulStage):
    fn: Type[StatefulStageUDF] = ChatTemplateUDF


class TokenizeUDF(StatefulStageUDF):
    def __init__(self, data_column: str, model: Optional[str] = None):
        from ..tokenizer import load_tokenizer

        super().__init__(data_column)
        self.tokenizer = load_tokenizer(model)

    async def udf(self, batch):
        ids = self.tokenizer([str(r["prompt"]) for r in batch])["input_ids"]
        for row, toks in zip(batch, ids):
            yield {self.IDX_IN_BATCH_COLUMN: row[self.IDX_IN_BATCH_COLUMN], "tokenized_prompt": list(toks)}

    @property
    def expected_input_keys(self):
        return ["prompt"]


class TokenizeStage(StatefulStage):
    fn: Type[StatefulStageUDF] = TokenizeUDF


class DetokenizeUDF(StatefulStageUDF):
    def __init__(self, data_column: str, model: Optional[str] = None):
        from ..tokenizer import load_tokenizer

        super().__init__(data_column)
        self.tokenizer = load_tokenizer(model)

    async def udf(self, batch):
        texts = self.tokenizer.batch_decode([_plain(r["generated_tokens"]) for r in batch],
                                            skip_special_tokens=True)
        for row, text in zip(batch, texts):
            yield {self.IDX_IN_BATCH_COLUMN: row[self.IDX_IN_BATCH_COLUMN], "generated_text": text}

    @property
    def expected_input_keys(self):
        return ["generated_tokens"]


class DetokenizeStage(StatefulStage):
    fn: Type[StatefulStageUDF] = DetokenizeUDF


# ------------------------------------------------------------ HTTP stage
class HttpRequestUDF(StatefulStageUDF):
    """POST every row (as its JSON body) to ``url`` and merge the JSON response
    into the row (reference: http_request_stage.py:12). Requests of a batch run
    concurrently (``max_concurrent``), paced to ``qps`` when set; 429 / 5xx /
    connection errors are retried with exponential backoff ``max_retries`` times."""

    def __init__(self, data_column: str, url: str, additional_header: Optional[Dict[str, Any]] = None,
                 qps: Optional[float] = None, max_concurrent: int = 64, max_retries: int = 3,
                 base_retry_wait_s: float = 0.5, timeout_s: float = 300.0):
        super().__init__(data_column)
        self.url = url
        self.headers = {"Content-Type": "application/json", **(additional_header or {})}
        self.qps = qps
        self.max_concurrent = max(1, int(max_concurrent))
        self.max_retries = max_retries
        self.base_wait = base_retry_wait_s
        self.timeout_s = timeout_s

    async def _post(self, session, body):
        import aiohttp

        for attempt in range(self.max_retries + 1):
            try:
                async with session.post(self.url, headers=self.headers, json=body) as resp:
                    if resp.status == 429 or resp.status >= 500:
                        if attempt < self.max_retries:
                            await asyncio.sleep(self.base_wait * (2 ** attempt))
                            continue
                    resp.raise_for_status()
                    return await resp.json(content_type=None)
            except (aiohttp.ClientConnectionError, asyncio.TimeoutError):
                if attempt >= self.max_retries:
                    raise
                await asyncio.sleep(self.base_wait * (2 ** attempt))
        raise RuntimeError("unreachable")

    async def udf(self, batch):
        import aiohttp

        sem = asyncio.Semaphore(self.max_concurrent)
        t0 = time.monotonic()

        async def one(k, row, session):
            if self.qps:
                delay = t0 + k / float(self.qps) - time.monotonic()
                if delay > 0:
                    await asyncio.sleep(delay)
            body = {key: _plain(v) for key, v in row.items() if key != self.IDX_IN_BATCH_COLUMN}
            async with sem:
                out = await self._post(session, body)
            if isinstance(out, dict) and self.IDX_IN_BATCH_COLUMN in out:
                raise ValueError(f"The response of the HTTP request must not contain the column "
                                 f"{self.IDX_IN_BATCH_COLUMN}.")
            res = dict(out) if isinstance(out, dict) else {"http_response": out}
            res[self.IDX_IN_BATCH_COLUMN] = row[self.IDX_IN_BATCH_COLUMN]
            return res

        timeout = aiohttp.ClientTimeout(total=self.timeout_s)
        async with aiohttp.ClientSession(timeout=timeout) as session:
            tasks = [asyncio.ensure_future(one(k, row, session)) for k, row in enumerate(batch)]
            try:
                for fut in asyncio.as_completed(tasks):
                    yield await fut
            finally:
                for t in tasks:
                    t.cancel()


class HttpRequestStage(StatefulStage):
    fn: Type[StatefulStageUDF] = HttpRequestUDF


# ------------------------------------------------------------ image stage
def _load_image(src):
    from PIL import Image

    if isinstance(src, Image.Image):
        return src
    if isinstance(src, (bytes, bytearray)):
        return Image.open(io.BytesIO(src))
    if isinstance(src, str):
        if src.startswith("data:"):
            head, _, data = src.partition(",")
            raw = base64.b64decode(data) if ";base64" in head else data.encode()
            return Image.open(io.BytesIO(raw))
        if src.startswith(("http://", "https://")):
            import urllib.request

            with urllib.request.urlopen(src, timeout=30) as r:
                return Image.open(io.BytesIO(r.read()))
        path = src[len("file://"):] if src.startswith("file://") else src
        if os.path.exists(path):
            return Image.open(path)
    raise ValueError(f"cannot load image from {str(src)[:80]!r}: expected a PIL image, bytes, a data URL, "
                     "an http(s) URL or a local path")


class PrepareImageUDF(StatefulStageUDF):
    """Collect the images of each row's chat messages (``{"type": "image", "image": ...}``
    or ``{"type": "image_url", "image_url": {"url": ...}}`` parts), load them as RGB
    PIL images (optionally resized to ``resize``) and add ``image`` / ``image_sizes``
    (reference: prepare_image_stage.py:306). Loading runs in a thread pool."""

    def __init__(self, data_column: str, resize: Optional[List[int]] = None):
        super().__init__(data_column)
        self.resize = tuple(resize) if resize else None

    @staticmethod
    def extract_image_info(messages) -> List[Any]:
        out = []
        for m in messages:
            content = m.get("content")
            if not isinstance(content, list):
                continue
            for part in content:
                if not isinstance(part, dict) or part.get("type") not in ("image", "image_url"):
                    continue
                if part["type"] == "image":
                    out.append(part.get("image"))
                else:
                    iu = part.get("image_url")
                    out.append(iu.get("url") if isinstance(iu, dict) else iu)
        return out

    def _prep(self, src):
        img = _load_image(src).convert("RGB")
        if self.resize:
            img = img.resize(self.resize)
        return img

    async def udf(self, batch):
        loop = asyncio.get_running_loop()
        for row in batch:
            srcs = self.extract_image_info(_plain(row["messages"]))
            imgs = await asyncio.gather(*(loop.run_in_executor(None, self._prep, s) for s in srcs))
            yield {self.IDX_IN_BATCH_COLUMN: row[self.IDX_IN_BATCH_COLUMN], "image": list(imgs),
                   "image_sizes": [(im.width, im.height) for im in imgs]}

    @property
    def expected_input_keys(self):
        return ["messages"]


class PrepareImageStage(StatefulStage):
    fn: Type[StatefulStageUDF] = PrepareImageUDF


# ------------------------------------------------------------ engine stage
_SAMPLING_KEYS = ("max_tokens", "temperature", "top_p", "top_k", "stop_token_ids", "ignore_eos", "seed")


class EngineUDF(StatefulStageUDF):
    """Generate with the in-tree engine: one engine per actor (one GPU), every
    row of the batch added as a request and scheduled by continuous batching;
    rows are yielded as their sequences finish. Inputs: ``tokenized_prompt``
    (or ``prompt``, tokenized here) and optional per-row ``sampling_params``.
    Outputs: ``generated_tokens``, ``num_input_tokens``, ``num_generated_tokens``,
    ``finish_reason``, ``time_taken_llm``."""

    def __init__(self, data_column: str, model: str = "llama-tiny", model_source: Optional[str] = None,
                 tokenizer_source: Optional[str] = None, dtype: str = "bfloat16",
                 engine_kwargs: Optional[Dict[str, Any]] = None, sampling_params: Optional[Dict] = None,
                 seed: int = 0):
        from ..build import build_engine

        super().__init__(data_column)
        self.engine, self.tokenizer = build_engine(model, model_source, tokenizer_source, dtype,
                                                   engine_kwargs, seed)
        self.default_sampling = dict(sampling_params or {})

    def _params(self, row):
        from ..engine import SamplingParams

        sp = dict(self.default_sampling)
        sp.update({k: v for k, v in (_plain(row.get("sampling_params")) or {}).items() if k in _SAMPLING_KEYS})
        return SamplingParams(**{k: v for k, v in sp.items() if k in _SAMPLING_KEYS})

    async def udf(self, batch):
        eng = self.engine
        t0 = time.time()
        rid_row = {}
        for row in batch:
            ids = row.get("tokenized_prompt")
            ids = _plain(ids) if ids is not None else self.tokenizer.encode(str(row["prompt"]))
            rid = eng.add_request([int(t) for t in ids], self._params(row))
            rid_row[rid] = (row[self.IDX_IN_BATCH_COLUMN], len(ids))
        while rid_row:
            for o in eng.step():
                if o.finished and o.request_id in rid_row:
                    idx, n_in = rid_row.pop(o.request_id)
                    yield {self.IDX_IN_BATCH_COLUMN: idx, "generated_tokens": list(o.output_token_ids),
                           "num_input_tokens": n_in, "num_generated_tokens": len(o.output_token_ids),
                           "finish_reason": o.finish_reason, "time_taken_llm": time.time() - t0}
            await asyncio.sleep(0)
            if rid_row and not eng.has_unfinished():
                raise RuntimeError(f"engine went idle with {len(rid_row)} rows unfinished")

    @property
    def expected_input_keys(self):
        return []

    def validate_inputs(self, inputs):
        super().validate_inputs(inputs)
        for r in inputs:
            if "tokenized_prompt" not in r and "prompt" not in r:
                raise ValueError("EngineUDF needs 'tokenized_prompt' or 'prompt' in every row; "
                                 f"got keys {set(r)}")


class EngineStage(StatefulStage):
    fn: Type[StatefulStageUDF] = EngineUDF
