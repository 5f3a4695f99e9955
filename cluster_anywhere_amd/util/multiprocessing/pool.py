"""``multiprocessing.Pool`` API over a pool of actors (reference:
python/ray/util/multiprocessing/pool.py — ``Pool`` :545, ``PoolActor.run_batch``
:532, ``AsyncResult`` :220, ``IMapIterator`` :420).

Each pool process is an actor; work is shipped in chunks (``run_batch`` runs a
list of ``(args, kwargs)`` calls and returns one list), so per-item scheduling
cost is paid once per chunk. ``maxtasksperchild`` retires an actor after that
many chunks and starts a fresh one (re-running the initializer). Ordered
results for ``map``/``imap``; ``imap_unordered`` yields chunks as they finish.

A chunk whose actor dies (OOM kill, node loss, a crashed initializer) is run again
on a fresh actor, up to ``_CHUNK_ATTEMPTS`` times, so a lost pool process costs a
re-run, not the whole map (the pool's functions are stateless, as stdlib requires).
"""
from __future__ import annotations

import threading
from multiprocessing import TimeoutError
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple


_CHUNK_ATTEMPTS = 4


class _Chunk:
    """One submitted batch: what to re-run if its actor dies."""

    __slots__ = ("ref", "func", "batch", "slot", "handle")

    def __init__(self, ref, func, batch, slot, handle):
        self.ref, self.func, self.batch, self.slot, self.handle = ref, func, batch, slot, handle


class PoolTaskError(Exception):
    def __init__(self, underlying: BaseException):
        super().__init__(repr(underlying))
        self.underlying = underlying


class _PoolActor:
    def __init__(self, initializer=None, initargs=None):
        if initializer is not None:
            initializer(*(initargs or ()))

    def ping(self):
        return True

    def run_batch(self, func, batch):
        out = []
        for args, kwargs in batch:
            try:
                out.append(func(*args, **(kwargs or {})))
            except Exception as e:  # noqa: BLE001 — delivered to the caller
                out.append(PoolTaskError(e))
        return out


class AsyncResult:
    """Result of ``apply_async`` / ``map_async`` (stdlib semantics)."""

    def __init__(self, pool, chunks, callback=None, error_callback=None, single_result=False):
        self._pool = pool
        self._chunks = chunks
        self._single = single_result
        self._callback, self._error_callback = callback, error_callback
        self._event = threading.Event()
        self._value: Any = None
        self._error: Optional[BaseException] = None
        threading.Thread(target=self._collect, daemon=True).start()

    def _collect(self):
        try:
            chunks = [self._pool._resolve(c) for c in self._chunks]
            flat = [x for c in chunks for x in c]
            err = next((x for x in flat if isinstance(x, PoolTaskError)), None)
            if err is not None:
                self._error = err.underlying
            else:
                self._value = flat[0] if self._single else flat
        except BaseException as e:  # noqa: BLE001
            self._error = e
        self._event.set()
        try:
            if self._error is None and self._callback is not None:
                self._callback(self._value)
            elif self._error is not None and self._error_callback is not None:
                self._error_callback(self._error)
        except Exception:
            pass

    def ready(self) -> bool:
        return self._event.is_set()

    def successful(self) -> bool:
        if not self.ready():
            raise ValueError(f"{self!r} not ready")
        return self._error is None

    def wait(self, timeout: Optional[float] = None) -> None:
        self._event.wait(timeout)

    def get(self, timeout: Optional[float] = None):
        if not self._event.wait(timeout):
            raise TimeoutError
        if self._error is not None:
            raise self._error
        return self._value


class Pool:
    def __init__(self, processes: Optional[int] = None, initializer: Optional[Callable] = None,
                 initargs: Optional[Iterable] = None, maxtasksperchild: Optional[int] = None,
                 context: Any = None, ray_address: Optional[str] = None,
                 ray_remote_args: Optional[Dict[str, Any]] = None):
        from ...core import api

        if not api.is_initialized():
            if ray_address is not None:
                api.init(address=ray_address)
            else:
                api.init(num_cpus=processes)
        cpus = int(api.cluster_resources().get("CPU", 1))
        processes = processes or cpus
        if processes <= 0:
            raise ValueError("Processes in the pool must be >0.")
        self._initializer, self._initargs = initializer, tuple(initargs or ())
        self._maxtasks = maxtasksperchild or -1
        self._remote_args = dict(ray_remote_args or {})
        self._closed = False
        self._terminated = False
        self._lock = threading.Lock()
        self._cls = api.remote(**self._remote_args)(_PoolActor) if self._remote_args else api.remote(_PoolActor)
        self._actors: List[list] = [self._new_actor() for _ in range(processes)]
        self._next = 0
        api.get([a.ping.remote() for a, _ in self._actors])

    def _new_actor(self):
        return [self._cls.remote(self._initializer, self._initargs), 0]

    @property
    def _processes(self) -> int:
        return len(self._actors)

    def _submit(self, func, batch, retry: bool = False) -> _Chunk:
        with self._lock:
            if self._closed and not retry:
                raise ValueError("Pool not running")
            if self._terminated:
                raise ValueError("Pool terminated")
            i = self._next
            self._next = (self._next + 1) % len(self._actors)
            entry = self._actors[i]
            handle = entry[0]
            ref = handle.run_batch.remote(func, batch)
            entry[1] += 1
            if self._maxtasks > 0 and entry[1] >= self._maxtasks:
                handle.__ray_terminate__.remote()  # runs after its queued batches
                self._actors[i] = self._new_actor()
            return _Chunk(ref, func, batch, i, handle)

    def _resolve(self, chunk: _Chunk, timeout: Optional[float] = None) -> list:
        """The chunk's result list; a chunk whose actor died is re-run on a fresh one."""
        from ...core.api import get
        from ...exceptions import ActorDiedError, ActorUnavailableError

        for attempt in range(_CHUNK_ATTEMPTS):
            try:
                return get(chunk.ref, timeout=timeout)
            except (ActorDiedError, ActorUnavailableError):
                if attempt == _CHUNK_ATTEMPTS - 1 or self._terminated:
                    raise
                with self._lock:
                    entry = self._actors[chunk.slot]
                    if entry[0] is chunk.handle:  # not replaced yet (by maxtasksperchild or another chunk)
                        self._actors[chunk.slot] = self._new_actor()
                chunk = self._submit(chunk.func, chunk.batch, retry=True)
        raise AssertionError("unreachable")

    def _chunks(self, func, iterable, chunksize, star):
        items = list(iterable)
        if chunksize is None:
            chunksize, extra = divmod(len(items), self._processes * 4)
            chunksize += 1 if extra else 0
        chunksize = max(1, chunksize)
        refs = []
        for s in range(0, len(items), chunksize):
            batch = [((tuple(x) if star else (x,)), None) for x in items[s:s + chunksize]]
            refs.append(self._submit(func, batch))
        return refs

    # -- stdlib API -------------------------------------------------------------
    def apply(self, func: Callable, args: Optional[Tuple] = None, kwargs: Optional[Dict] = None):
        return self.apply_async(func, args, kwargs).get()

    def apply_async(self, func, args=None, kwargs=None, callback=None, error_callback=None) -> AsyncResult:
        chunk = self._submit(func, [(tuple(args or ()), kwargs)])
        return AsyncResult(self, [chunk], callback, error_callback, single_result=True)

    def map(self, func: Callable, iterable: Iterable, chunksize: Optional[int] = None) -> list:
        return self.map_async(func, iterable, chunksize).get()

    def map_async(self, func, iterable, chunksize=None, callback=None, error_callback=None) -> AsyncResult:
        return AsyncResult(self, self._chunks(func, iterable, chunksize, False), callback, error_callback)

    def starmap(self, func, iterable, chunksize=None) -> list:
        return self.starmap_async(func, iterable, chunksize).get()

    def starmap_async(self, func, iterable, chunksize=None, callback=None, error_callback=None) -> AsyncResult:
        return AsyncResult(self, self._chunks(func, iterable, chunksize, True), callback, error_callback)

    def imap(self, func: Callable, iterable: Iterable, chunksize: int = 1):
        for chunk in self._chunks(func, iterable, chunksize, False):
            for x in self._resolve(chunk):
                if isinstance(x, PoolTaskError):
                    raise x.underlying
                yield x

    def imap_unordered(self, func: Callable, iterable: Iterable, chunksize: int = 1):
        from ...core.api import wait

        pending = {c.ref: c for c in self._chunks(func, iterable, chunksize, False)}
        while pending:
            done, _ = wait(list(pending), num_returns=1)
            for x in self._resolve(pending.pop(done[0])):
                if isinstance(x, PoolTaskError):
                    raise x.underlying
                yield x

    def close(self):
        self._closed = True

    def terminate(self):
        from ...core.api import kill

        self._closed = True
        self._terminated = True
        for a, _ in self._actors:
            try:
                kill(a)
            except Exception:
                pass
        self._actors = []

    def join(self):
        from ...core.api import get

        if not self._closed:
            raise ValueError("Pool is still running")
        get([a.ping.remote() for a, _ in self._actors])

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.terminate()
