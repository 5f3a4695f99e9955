"""Batch-LLM stages: stateful ``map_batches`` UDFs composed by a :class:`Processor`.

Reference roles: ``python/ray/llm/_internal/batch/stages/base.py`` (the stage
UDF / stage description pair), ``chat_template_stage.py``,
``tokenize_stage.py`` (tokenize + detokenize), ``http_request_stage.py`` and
``prepare_image_stage.py``; the reference's engine stage delegates to vLLM.
Here the engine stage drives the in-tree paged-KV engine (:mod:`..engine`,
gfx950 decode kernels, HIP graphs) inside a GPU actor of the data executor.

Row contract (public, shared with the reference): a stage reads the dicts of
the ``data_column``, its UDF yields one output per input row tagged with the
row's ``__idx_in_batch``, in any order, and the output is merged into the row.
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


class _PackRow:
    """Pre-processing map: the user's row function runs on the raw row and its
    output is folded into a copy of that row, which becomes the single value of
    the processor's data column (every stage reads and writes that column)."""

    def __init__(self, fn: Callable, data_column: str):
        self.fn, self.col = fn, data_column

    def __call__(self, row: Dict[str, Any]) -> Dict[str, Any]:
        packed = dict(row)
        packed.update(self.fn(row))
        return {self.col: packed}


class _UnpackRow:
    """Post-processing map: the user's function sees the data-column dict and
    decides the output columns."""

    def __init__(self, fn: Callable, data_column: str):
        self.fn, self.col = fn, data_column

    def __call__(self, row: Dict[str, Any]) -> Dict[str, Any]:
        try:
            packed = row[self.col]
        except KeyError:
            raise ValueError(f"postprocess: row has no {self.col!r} column (columns: {sorted(row)})") from None
        return self.fn(packed)


def wrap_preprocess(fn: Callable, data_column: str) -> Callable:
    return _PackRow(fn, data_column)


def wrap_postprocess(fn: Callable, data_column: str) -> Callable:
    return _UnpackRow(fn, data_column)


class _Ledger:
    """Which rows of one batch a stage UDF still owes. Positions are handed out
    as the row tag; an output is accepted once per position."""

    __slots__ = ("rows", "owed", "left", "stage")

    def __init__(self, rows: List[Dict[str, Any]], stage: str):
        self.rows = rows
        self.owed = bytearray(b"\x01") * len(rows)
        self.left = len(rows)
        self.stage = stage

    def settle(self, tag: Any, out: Dict[str, Any]) -> Dict[str, Any]:
        if not isinstance(tag, (int, np.integer)) or not 0 <= int(tag) < len(self.rows):
            raise ValueError(f"{self.stage}: output tag {tag!r} names no row of this batch")
        pos = int(tag)
        if not self.owed[pos]:
            raise ValueError(f"{self.stage}: row {pos} was produced more than once "
                             "(a stage UDF maps every input row to exactly one output row)")
        self.owed[pos] = 0
        self.left -= 1
        merged = self.rows[pos]
        merged.update(out)
        return merged

    def unsettled(self) -> List[int]:
        return [i for i, o in enumerate(self.owed) if o]


class StatefulStageUDF:
    """Base of a processor stage: a stateful, async ``map_batches`` callable.

    Subclasses implement ``udf(rows)``, an async generator over the batch's
    data-column dicts that yields one dict per input row, carrying the row's tag
    under ``IDX_IN_BATCH_COLUMN`` (outputs may come in any order). The base class
    tags the rows, checks the contract and merges every output into its input row
    (output keys win), handing each finished row downstream at once so a slow row
    does not hold back the others. Role reference: stages/base.py:65."""

    IDX_IN_BATCH_COLUMN: str = "__idx_in_batch"

    def __init__(self, data_column: str):
        self.data_column = data_column

    def _rows_of(self, batch: Dict[str, Any]) -> List[Dict[str, Any]]:
        if self.data_column not in batch:
            raise ValueError(f"{type(self).__name__}: batch has no {self.data_column!r} column "
                             f"(columns: {sorted(batch)})")
        col = batch[self.data_column]
        return [dict(r) for r in (col.tolist() if hasattr(col, "tolist") else col)]

    async def __call__(self, batch: Dict[str, Any]) -> AsyncIterator[Dict[str, Any]]:
        if not batch:
            return
        rows = self._rows_of(batch)
        if not rows:
            return
        self.validate_inputs(rows)
        tag = self.IDX_IN_BATCH_COLUMN
        for pos, r in enumerate(rows):
            r[tag] = pos
        ledger = _Ledger(rows, type(self).__name__)
        async for out in self.udf(rows):
            if tag not in out:
                raise ValueError(f"{ledger.stage}: every output row must carry its input tag "
                                 f"{tag!r} (got keys {sorted(out)})")
            pos = out.pop(tag)
            merged = ledger.settle(pos, out)
            merged.pop(tag, None)
            yield {self.data_column: [merged]}
        if ledger.left:
            raise ValueError(f"{ledger.stage}: generator ended with {ledger.left} row(s) never produced: "
                             f"{ledger.unsettled()[:16]}")

    def validate_inputs(self, inputs: List[Dict[str, Any]]):
        want = self.expected_input_keys
        tag = self.IDX_IN_BATCH_COLUMN
        for r in inputs:
            if tag in r:
                raise ValueError(f"{type(self).__name__}: input rows may not use the key {tag!r}; "
                                 "it is reserved for the stage's row tags")
            gaps = [k for k in want if k not in r]
            if gaps:
                raise ValueError(f"{type(self).__name__}: Required input keys missing: {gaps} "
                                 f"(row has {sorted(r)})")

    @property
    def expected_input_keys(self) -> List[str]:
        return []

    async def udf(self, rows: List[Dict[str, Any]]) -> AsyncIterator[Dict[str, Any]]:
        raise NotImplementedError(f"{type(self).__name__} must define udf(rows)")
        yield  # pragma: no cover


class StatefulStage(BaseModel):
    """A stage description: which UDF class runs, its constructor kwargs and the
    ``map_batches`` options it runs with (actors, CPUs / GPUs). The processor
    owns ``batch_size`` and ``data_column``. Role reference: stages/base.py:233."""

    model_config = ConfigDict(arbitrary_types_allowed=True, validate_assignment=True)

    fn: Type[StatefulStageUDF] = Field(description="UDF class of this stage.")
    fn_constructor_kwargs: Dict[str, Any] = Field(default_factory=dict)
    map_batches_kwargs: Dict[str, Any] = Field(default_factory=lambda: dict(concurrency=1))

    def get_dataset_map_batches_kwargs(self, batch_size: int, data_column: str) -> Dict[str, Any]:
        if "data_column" in self.fn_constructor_kwargs:
            raise ValueError(f"{type(self).__name__}: fn_constructor_kwargs may not set 'data_column'; "
                             "the processor passes its own")
        user_bs = self.map_batches_kwargs.get("batch_size")
        if user_bs not in (None, batch_size):
            logger.warning("%s: map_batches_kwargs batch_size=%s ignored, the processor runs batches of %d",
                           type(self).__name__, user_bs, batch_size)
        opts = {"num_cpus": 0.25}  # host-side stages are light; the engine stage sets its own
        opts.update(self.map_batches_kwargs)
        opts["batch_size"] = batch_size
        opts["fn_constructor_kwargs"] = {**self.fn_constructor_kwargs, "data_column": data_column}
        return opts


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
