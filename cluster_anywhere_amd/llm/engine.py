"""Continuous-batching LLM engine with a paged KV cache (the serving engine
behind ``serve.llm``; reference: python/ray/llm/_internal/serve/deployments/
llm/vllm/ delegates to vLLM — this is a native MI355X engine instead).

* KV cache: per layer ``[num_blocks, KVH, block_size, D]`` bf16, sized from the
  HBM left after the weights (``gpu_memory_utilization`` of 288 GB).
* Scheduler (every ``step()``): admit waiting requests into a batched prefill
  (bounded by ``max_num_batched_tokens`` / ``max_num_seqs`` / free blocks),
  otherwise one decode token for every running sequence; if the cache runs out
  the newest sequence is preempted (blocks freed, re-prefilled later).
* Decode forward is captured once per batch-size bucket in a HIP graph (static
  input buffers, ``max_ctx = max_model_len``) and replayed; prefill runs eagerly.
* Sampling: greedy / temperature / top-k / top-p on the GPU.
"""
from __future__ import annotations

import itertools
import math
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch


@dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 0.0
    top_p: float = 1.0
    top_k: int = -1
    stop_token_ids: List[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None


@dataclass
class RequestOutput:
    request_id: str
    prompt_token_ids: List[int]
    output_token_ids: List[int]
    finished: bool
    finish_reason: Optional[str] = None
    metrics: Dict[str, float] = field(default_factory=dict)


class _Seq:
    def __init__(self, rid, prompt, params, arrival):
        self.rid = rid
        self.prompt = list(prompt)
        self.out: List[int] = []
        self.params = params
        self.blocks: List[int] = []
        self.arrival = arrival
        self.first_token_time = None
        self.finish_reason = None

    @property
    def tokens(self):
        return self.prompt + self.out

    @property
    def last_token(self):
        return self.out[-1] if self.out else self.prompt[-1]

    @property
    def ctx(self):
        return len(self.prompt) + len(self.out)


class BlockAllocator:
    def __init__(self, num_blocks: int):
        self.free = list(range(num_blocks - 1, -1, -1))
        self.num_blocks = num_blocks

    def allocate(self, n: int) -> Optional[List[int]]:
        if n > len(self.free):
            return None
        return [self.free.pop() for _ in range(n)]

    def release(self, blocks: List[int]):
        self.free.extend(reversed(blocks))

    @property
    def num_free(self):
        return len(self.free)


class LLMEngine:
    def __init__(self, model, *, block_size: int = 16, max_num_seqs: int = 256, max_model_len: int = 4096,
                 max_num_batched_tokens: int = 16384, num_blocks: Optional[int] = None,
                 gpu_memory_utilization: float = 0.9, eos_token_id: Optional[int] = None,
                 use_graphs: bool = True, device=None):
        self.model = model
        cfg = model.cfg
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        self.dtype = next(model.parameters()).dtype
        self.bs = block_size
        self.max_num_seqs = max_num_seqs
        self.max_model_len = min(max_model_len, cfg.max_position)
        self.max_blocks_per_seq = (self.max_model_len + block_size - 1) // block_size
        self.max_num_batched_tokens = max_num_batched_tokens
        self.eos = eos_token_id
        per_block = 2 * cfg.n_layer * cfg.n_kv_head * block_size * cfg.head_dim * 2  # bytes, K+V bf16
        # decode-GEMM weight copies (fused SwiGLU, packed streams) before the cache takes the rest of HBM
        self.decode_gemm = bool(self.device.type == "cuda" and hasattr(model, "prepare_decode")
                                and model.prepare_decode())
        if num_blocks is None:
            if self.device.type == "cuda":
                free, total = torch.cuda.mem_get_info(self.device)
                budget = free - (1 - gpu_memory_utilization) * total
                num_blocks = max(16, int(budget // per_block))
            else:
                num_blocks = 256
        self.num_blocks = num_blocks
        shape = (num_blocks, cfg.n_kv_head, block_size, cfg.head_dim)
        self.k_caches = [torch.zeros(shape, dtype=self.dtype, device=self.device) for _ in range(cfg.n_layer)]
        self.v_caches = [torch.zeros(shape, dtype=self.dtype, device=self.device) for _ in range(cfg.n_layer)]
        self.alloc = BlockAllocator(num_blocks)
        self.waiting: deque = deque()
        self.running: List[_Seq] = []
        self.seqs: Dict[str, _Seq] = {}
        self._ids = itertools.count()
        self.lock = threading.RLock()
        self.use_graphs = use_graphs and self.device.type == "cuda"
        if self.device.type == "cuda":
            from ..ops.gemm_tuning import use_tuned_gemms

            use_tuned_gemms()  # shipped per-shape hipBLASLt selections (prefill GEMMs)
        self.graphs: Dict[int, tuple] = {}
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "preemptions": 0, "steps": 0}
        # (batch size, seconds) of every decode step: forward + sampling, host included
        self.decode_times: List[tuple] = []
        self._pinned: Dict[int, Dict[str, torch.Tensor]] = {}
        # one-step-ahead decode (greedy batches on HIP graphs): step t + 1 is launched
        # with step t's argmax still on the GPU, and step t's tokens are read back and
        # processed while t + 1 runs, so the host work of a step (reading tokens,
        # appending, building the next inputs) overlaps the GPU (CAAMD_LLM_ASYNC=0: off)
        import os as _os

        self._async = self.use_graphs and _os.environ.get("CAAMD_LLM_ASYNC", "1") != "0"
        self._inflight: Optional[dict] = None
        self._async_flip = 0
        self._last_finish: Optional[float] = None
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(0)

    # ------------------------------------------------------------ requests
    def add_request(self, prompt_token_ids: List[int], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None) -> str:
        params = params or SamplingParams()
        if len(prompt_token_ids) == 0:
            raise ValueError("empty prompt")
        if len(prompt_token_ids) + params.max_tokens > self.max_model_len:
            raise ValueError(f"prompt ({len(prompt_token_ids)}) + max_tokens ({params.max_tokens}) exceeds "
                             f"max_model_len {self.max_model_len}")
        rid = request_id or f"req-{next(self._ids)}"
        s = _Seq(rid, prompt_token_ids, params, time.time())
        with self.lock:
            self.seqs[rid] = s
            self.waiting.append(s)
        return rid

    def abort_request(self, rid: str):
        with self.lock:
            s = self.seqs.pop(rid, None)
            if s is None:
                return
            if s in self.running:
                self.running.remove(s)
            try:
                self.waiting.remove(s)
            except ValueError:
                pass
            self.alloc.release(s.blocks)
            s.blocks = []

    def has_unfinished(self) -> bool:
        with self.lock:
            return bool(self.waiting or self.running)

    # ------------------------------------------------------------ scheduling
    def _blocks_needed(self, n_tokens):
        return (n_tokens + self.bs - 1) // self.bs

    def _schedule_prefill(self) -> List[_Seq]:
        batch, tokens = [], 0
        while self.waiting and len(self.running) + len(batch) < self.max_num_seqs:
            s = self.waiting[0]
            n = s.ctx  # recompute of a preempted sequence re-prefills prompt + outputs
            if batch and tokens + n > self.max_num_batched_tokens:
                break
            need = self._blocks_needed(n + 1) - len(s.blocks)
            got = self.alloc.allocate(need) if need > 0 else []
            if got is None:
                break
            s.blocks.extend(got)
            self.waiting.popleft()
            batch.append(s)
            tokens += n
        return batch

    def _ensure_decode_blocks(self):
        for s in list(self.running):
            if s not in self.running:
                continue
            need = self._blocks_needed(s.ctx + 1) - len(s.blocks)
            while need > 0:
                got = self.alloc.allocate(need)
                if got is not None:
                    s.blocks.extend(got)
                    break
                victim = self.running[-1]
                self._preempt(victim)
                if victim is s:
                    break

    def _preempt(self, s: _Seq):
        self.running.remove(s)
        self.alloc.release(s.blocks)
        s.blocks = []
        self.waiting.appendleft(s)
        self.stats["preemptions"] += 1

    # ------------------------------------------------------------ execution
    def _slots(self, s: _Seq, start: int, end: int) -> List[int]:
        return [s.blocks[p // self.bs] * self.bs + p % self.bs for p in range(start, end)]

    def _run_prefill(self, batch: List[_Seq]) -> torch.Tensor:
        import numpy as np

        T = max(s.ctx for s in batch)
        B = len(batch)
        # numpy-vectorised inputs (the per-token Python slot lists took milliseconds per
        # 8k-token chunk while the GPU waited)
        toks = np.zeros((B, T), np.int64)
        pos = np.zeros((B, T), np.int32)
        slots = np.full((B, T), -1, np.int32)
        last = np.zeros(B, np.int64)
        ar = np.arange(T, dtype=np.int32)
        for i, s in enumerate(batch):
            n = s.ctx
            toks[i, : len(s.prompt)] = s.prompt
            if s.out:
                toks[i, len(s.prompt): n] = s.out
            pos[i, :n] = ar[:n]
            blk = np.asarray(s.blocks, np.int32)
            slots[i, :n] = blk[ar[:n] // self.bs] * self.bs + ar[:n] % self.bs
            last[i] = n - 1
        dev = self.device
        logits = self.model.prefill(torch.from_numpy(toks).to(dev, non_blocking=True),
                                    torch.from_numpy(pos).to(dev, non_blocking=True),
                                    torch.from_numpy(slots).reshape(-1).to(dev, non_blocking=True),
                                    self.k_caches, self.v_caches, torch.from_numpy(last).to(dev, non_blocking=True))
        self.stats["prefill_tokens"] += sum(s.ctx for s in batch)
        return logits

    def _decode_inputs(self, batch: List[_Seq], B: int, pending: int = 0, key=None):
        """Decode inputs built with numpy in (pinned, reused) host buffers: no
        per-sequence tensor construction, and the H2D copies are truly async.
        ``pending``: tokens already generated on the GPU but not yet appended (the
        one-step-ahead path); ``key`` selects the pinned buffer set (that path
        alternates two, so a set is never rewritten while its copies are queued)."""
        import numpy as np

        key = B if key is None else key
        buf = self._pinned.get(key)
        if buf is None:
            pin = self.device.type == "cuda"
            buf = self._pinned[key] = {
                "toks": torch.zeros(B, dtype=torch.long, pin_memory=pin),
                "pos": torch.zeros(B, dtype=torch.int32, pin_memory=pin),
                "slots": torch.full((B,), -1, dtype=torch.int32, pin_memory=pin),
                "ctx": torch.zeros(B, dtype=torch.int32, pin_memory=pin),
                "bt": torch.zeros(B, self.max_blocks_per_seq, dtype=torch.int32, pin_memory=pin)}
        n = len(batch)
        toks, pos, slots, ctx, bt = (buf[k].numpy() for k in ("toks", "pos", "slots", "ctx", "bt"))
        c = np.fromiter((s.ctx for s in batch), np.int32, n) + pending
        p = c - 1  # position of the newest (not yet cached) token
        if not pending:
            toks[:n] = np.fromiter((s.last_token for s in batch), np.int64, n)
        toks[n:] = 0
        pos[:n], pos[n:] = p, 0
        ctx[:n], ctx[n:] = c, 0
        bt[:n] = 0
        for i, s in enumerate(batch):
            bt[i, : len(s.blocks)] = s.blocks
        slots[:n] = bt[np.arange(n), p // self.bs] * self.bs + p % self.bs
        slots[n:] = -1
        return buf["toks"], buf["pos"], buf["slots"], buf["bt"], buf["ctx"]

    def _bucket(self, n):
        b = 1
        while b < n:
            b *= 2
        return min(b, max(self.max_num_seqs, n))

    def _graph_for(self, B: int):
        g = self.graphs.get(B)
        if g is not None:
            return g
        dev = self.device
        st = {"toks": torch.zeros(B, dtype=torch.long, device=dev),
              "pos": torch.zeros(B, dtype=torch.int32, device=dev),
              "slots": torch.full((B,), -1, dtype=torch.int32, device=dev),
              "bt": torch.zeros(B, self.max_blocks_per_seq, dtype=torch.int32, device=dev),
              "ctx": torch.ones(B, dtype=torch.int32, device=dev)}

        def fwd():
            return self.model.decode(st["toks"], st["pos"], st["slots"], self.k_caches, self.v_caches, st["bt"],
                                     st["ctx"], self.max_model_len)

        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                fwd()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = fwd()
        g = (graph, st, out)
        self.graphs[B] = g
        return g

    def _run_decode(self, batch: List[_Seq]) -> torch.Tensor:
        n = len(batch)
        self.stats["decode_tokens"] += n
        if self.use_graphs:
            B = self._bucket(n)
            graph, st, out = self._graph_for(B)
            toks, pos, slots, bt, ctx = self._decode_inputs(batch, B)
            st["toks"].copy_(toks, non_blocking=True)
            st["pos"].copy_(pos, non_blocking=True)
            st["slots"].copy_(slots, non_blocking=True)
            st["bt"].copy_(bt, non_blocking=True)
            st["ctx"].copy_(ctx, non_blocking=True)
            graph.replay()
            return out[:n]
        toks, pos, slots, bt, ctx = (t.clone() for t in self._decode_inputs(batch, n))
        dev = self.device
        max_ctx = max(s.ctx for s in batch)
        return self.model.decode(toks.to(dev), pos.to(dev), slots.to(dev), self.k_caches, self.v_caches,
                                 bt.to(dev), ctx.to(dev), max_ctx)

    # ------------------------------------------------------- one step ahead
    def _async_ok(self, batch: List[_Seq]) -> bool:
        from ..ops._lib import kernels

        return (self._async and len(batch) <= self.max_num_seqs and all(s.params.temperature <= 0 for s in batch)
                and hasattr(kernels(), "argmax_rows"))

    def _launch_ahead(self, prev: Optional[dict]) -> Optional[dict]:
        """Launch one greedy decode step for the running sequences without waiting
        for ``prev`` (the step in flight, if any): its tokens are gathered on the GPU
        as this step's input. Returns the in-flight record, or None when the step
        cannot be launched ahead (a cache block is missing, or nothing would run)."""
        from ..ops._lib import kernels

        pending = 1 if prev is not None else 0
        # sequences that reach max_tokens with prev's token are done: no further step
        batch = [s for s in self.running if len(s.out) + pending < s.params.max_tokens]
        if not batch or not self._async_ok(batch):
            return None
        for s in batch:  # blocks for the token this step writes (position ctx - 1 + pending)
            need = self._blocks_needed(s.ctx + pending + 1) - len(s.blocks)
            if need > 0:
                got = self.alloc.allocate(need)
                if got is None:
                    return None
                s.blocks.extend(got)
        n = len(batch)
        B = self._bucket(n)
        graph, st, out = self._graph_for(B)
        self._async_flip ^= 1
        toks, pos, slots, bt, ctx = self._decode_inputs(batch, B, pending, key=(B, self._async_flip))
        dev = self.device
        if prev is not None:
            where = {id(s): i for i, s in enumerate(prev["batch"])}
            if any(id(s) not in where for s in batch):  # (cannot happen: joins only after a drain)
                return None
            idx = [where[id(s)] for s in batch]
            if idx == list(range(n)):
                st["toks"][:n].copy_(prev["toks_dev"][:n])
            else:
                st["toks"][:n].copy_(prev["toks_dev"][torch.tensor(idx, device=dev)])
        else:
            st["toks"].copy_(toks, non_blocking=True)
        st["pos"].copy_(pos, non_blocking=True)
        st["slots"].copy_(slots, non_blocking=True)
        st["bt"].copy_(bt, non_blocking=True)
        st["ctx"].copy_(ctx, non_blocking=True)
        graph.replay()
        toks_dev = kernels().argmax_rows(out[:n])
        host = self._pinned.get(("out", B, self._async_flip))
        if host is None:  # (setdefault would allocate pinned memory on every step)
            host = self._pinned[("out", B, self._async_flip)] = torch.empty(B, dtype=torch.long, pin_memory=True)
        host[:n].copy_(toks_dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.stats["decode_tokens"] += n
        return {"batch": batch, "toks_dev": toks_dev, "host": host, "event": ev}

    def _finish_ahead(self, inf: dict) -> List[RequestOutput]:
        """Read back an in-flight step's tokens and append them; sequences that
        finished (or were aborted) in the meantime drop their extra token."""
        inf["event"].synchronize()
        batch = inf["batch"]
        toks = inf["host"][: len(batch)].tolist()
        now_p = time.perf_counter()
        if self._last_finish is not None:
            self.decode_times.append((len(batch), now_p - self._last_finish))
        self._last_finish = now_p
        live = {id(x) for x in self.running}
        keep = [(s, t) for s, t in zip(batch, toks) if s.finish_reason is None and id(s) in live]
        if not keep:
            return []
        return self._append([s for s, _ in keep], [t for _, t in keep], time.time())

    def _sample(self, logits: torch.Tensor, batch: List[_Seq]) -> List[int]:
        temps = [s.params.temperature for s in batch]
        if all(t <= 0 for t in temps) and logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 2:
            # greedy: row argmax on the bf16 logits in one HIP launch (no fp32 copy)
            from ..ops._lib import kernels

            return kernels().argmax_rows(logits).tolist()
        logits = logits.float()
        if all(t <= 0 for t in temps):
            return logits.argmax(-1).tolist()
        out = logits.argmax(-1)
        for i, s in enumerate(batch):
            p = s.params
            if p.temperature <= 0:
                continue
            row = logits[i] / p.temperature
            if p.top_k and p.top_k > 0:
                kth = torch.topk(row, min(p.top_k, row.numel())).values[-1]
                row = torch.where(row < kth, torch.full_like(row, -float("inf")), row)
            probs = torch.softmax(row, -1)
            if p.top_p < 1.0:
                sp, si = torch.sort(probs, descending=True)
                keep = torch.cumsum(sp, 0) - sp < p.top_p
                sp = torch.where(keep, sp, torch.zeros_like(sp))
                probs = torch.zeros_like(probs).scatter_(0, si, sp)
            gen = self._gen
            if p.seed is not None:
                gen = torch.Generator(device=logits.device)
                gen.manual_seed(p.seed + len(s.out))
            out[i] = torch.multinomial(probs / probs.sum(), 1, generator=gen)[0]
        return out.tolist()

    def _append(self, batch: List[_Seq], toks: List[int], now: float) -> List[RequestOutput]:
        outs = []
        for s, t in zip(batch, toks):
            s.out.append(int(t))
            if s.first_token_time is None:
                s.first_token_time = now
            p = s.params
            reason = None
            if not p.ignore_eos and self.eos is not None and t == self.eos:
                reason = "stop"
            elif t in p.stop_token_ids:
                reason = "stop"
            elif len(s.out) >= p.max_tokens:
                reason = "length"
            if reason is not None:
                s.finish_reason = reason
                self.running.remove(s)
                self.alloc.release(s.blocks)
                s.blocks = []
                self.seqs.pop(s.rid, None)
            outs.append(RequestOutput(s.rid, s.prompt, list(s.out), reason is not None, reason,
                                      {"arrival": s.arrival, "first_token": s.first_token_time,
                                       "now": now}))
        return outs

    def step(self) -> List[RequestOutput]:
        """One scheduler iteration: a prefill batch or one decode token for
        every running sequence. Returns the sequences that produced a token."""
        with self.lock:
            self.stats["steps"] += 1
            if self._inflight is not None:
                inf, self._inflight = self._inflight, None
                # keep one step ahead while no waiting request could be admitted
                admit = bool(self.waiting) and len(self.running) < self.max_num_seqs
                if not admit:
                    self._inflight = self._launch_ahead(inf)
                outs = self._finish_ahead(inf)
                if self._inflight is not None and all(s.finish_reason is not None
                                                      for s in self._inflight["batch"]):
                    # every sequence of the step launched ahead has finished (e.g. all on
                    # stop tokens): nothing will read it -- drain it now, so it is not
                    # finished inside the next request's first step (a bogus decode-time
                    # entry spanning the idle gap)
                    self._inflight["event"].synchronize()
                    self._inflight = None
                if self._inflight is None:
                    self._last_finish = None
                return outs
            batch = self._schedule_prefill()
            if batch:
                logits = self._run_prefill(batch)
                toks = self._sample(logits, batch)
                self.running.extend(batch)
                return self._append(batch, toks, time.time())
            if not self.running:
                return []
            self._ensure_decode_blocks()
            batch = list(self.running)
            if not batch:
                return []
            if self._async_ok(batch) and not (self.waiting and len(self.running) < self.max_num_seqs):
                self._inflight = self._launch_ahead(None)
                if self._inflight is not None:
                    self._last_finish = time.perf_counter()
                    return []
            t0 = time.perf_counter()
            logits = self._run_decode(batch)
            toks = self._sample(logits, batch)
            self.decode_times.append((len(batch), time.perf_counter() - t0))
            return self._append(batch, toks, time.time())

    def generate(self, prompts: List[List[int]], params: Optional[SamplingParams] = None) -> List[RequestOutput]:
        """Offline batch generation (all prompts scheduled with continuous batching)."""
        ids = [self.add_request(p, params) for p in prompts]
        final: Dict[str, RequestOutput] = {}
        while self.has_unfinished():
            for o in self.step():
                if o.finished:
                    final[o.request_id] = o
        return [final[i] for i in ids]
