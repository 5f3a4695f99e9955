"""Entry point of a worker process (reference: python/ray/_private/workers/default_worker.py).

Spawned by the head/node with CAAMD_HEAD (control address), CAAMD_WORKER_ID,
CAAMD_NODE_ID, CAAMD_GPU_IDS (and ROCR_VISIBLE_DEVICES for GPU workers, set
before any HIP initialisation), optional CAAMD_RUNTIME_ENV (json).
"""
from __future__ import annotations

import ctypes
import json
import os
import signal
import sys


def _die_with_parent():
    try:
        libc = ctypes.CDLL("libc.so.6")
        PR_SET_PDEATHSIG = 1
        libc.prctl(PR_SET_PDEATHSIG, signal.SIGKILL)
    except Exception:
        pass


def _apply_runtime_env(renv: dict):
    wd = renv.get("working_dir")
    if wd:
        if os.path.isdir(wd):
            os.chdir(wd)
            sys.path.insert(0, wd)
    for m in renv.get("py_modules") or []:
        p = m if os.path.isdir(m) else os.path.dirname(m)
        if p not in sys.path:
            sys.path.insert(0, p)


def main():
    if float(os.environ.get("CAAMD_HEAD_RECONNECT_S", "0") or 0) <= 0:
        _die_with_parent()
    # else: the worker outlives a head crash and re-attaches to the restarted head
    # (it exits on its own if none comes back within the reconnect window)
    for p in reversed(os.environ.get("CAAMD_SYS_PATH", "").split(os.pathsep)):
        if p and p not in sys.path:
            sys.path.insert(1, p)
    renv = os.environ.get("CAAMD_RUNTIME_ENV")
    if renv:
        _apply_runtime_env(json.loads(renv))
    from . import context
    from .worker import CoreWorker

    cw = CoreWorker(os.environ["CAAMD_HEAD"], "worker", bytes.fromhex(os.environ["CAAMD_WORKER_ID"]),
                    os.environ.get("CAAMD_NODE_ID", ""),
                    extra={"gpu_ids": [int(g) for g in os.environ.get("CAAMD_GPU_IDS", "").split(",") if g]})
    context.worker = cw
    lc = os.environ.get("CAAMD_LOGGING_CONFIG")
    if lc:  # init(logging_config=...) of the driver that started this cluster
        from .._compat import LoggingConfig

        LoggingConfig._from_env(lc)._apply()
    try:
        cw.run_worker_loop()
    finally:
        context.worker = None
        try:
            cw.close()
        except Exception:
            pass
        os._exit(0)


if __name__ == "__main__":
    main()
