"""Asyncio front-end of the engine: a single stepping thread owns the GPU,
request coroutines receive their tokens through per-request asyncio queues.
(reference: vLLM's AsyncLLMEngine, used by python/ray/llm/_internal/serve.)"""
from __future__ import annotations

import asyncio
import threading
import traceback
from typing import AsyncIterator, Dict, List, Optional

from .engine import LLMEngine, RequestOutput, SamplingParams


class AsyncLLMEngine:
    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self.queues: Dict[str, tuple] = {}
        self.wake = threading.Event()
        self.alive = True
        self.error: Optional[BaseException] = None
        self.thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self.thread.start()

    def _loop(self):
        while self.alive:
            if not self.engine.has_unfinished():
                self.wake.wait(0.05)
                self.wake.clear()
                continue
            try:
                outs = self.engine.step()
            except BaseException as e:  # noqa
                traceback.print_exc()
                self.error = e
                for rid, (loop, q) in list(self.queues.items()):
                    loop.call_soon_threadsafe(q.put_nowait, e)
                self.queues.clear()
                continue
            for o in outs:
                ent = self.queues.get(o.request_id)
                if ent is None:
                    continue
                loop, q = ent
                loop.call_soon_threadsafe(q.put_nowait, o)
                if o.finished:
                    self.queues.pop(o.request_id, None)

    async def generate(self, prompt_token_ids: List[int], params: Optional[SamplingParams] = None,
                       request_id: Optional[str] = None) -> AsyncIterator[RequestOutput]:
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        rid = self.engine.add_request(prompt_token_ids, params, request_id)
        self.queues[rid] = (loop, q)
        self.wake.set()
        try:
            while True:
                o = await q.get()
                if isinstance(o, BaseException):
                    raise o
                yield o
                if o.finished:
                    break
        finally:
            if rid in self.queues:  # cancelled / disconnected client
                self.queues.pop(rid, None)
                self.engine.abort_request(rid)

    def shutdown(self):
        self.alive = False
        self.wake.set()
