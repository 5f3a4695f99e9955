"""Drop-in ``multiprocessing.Pool`` on cluster actors (reference:
python/ray/util/multiprocessing/pool.py)."""
from .pool import AsyncResult, Pool, PoolTaskError, TimeoutError

__all__ = ["Pool", "AsyncResult", "PoolTaskError", "TimeoutError"]
