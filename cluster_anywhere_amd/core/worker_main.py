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


def _loaded_hip_runtime():
    """Path of the HIP runtime this process already mapped (torch's own copy), so the
    prewarm calls into the same library instance torch uses."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.rsplit(None, 1)[-1]
                if path.endswith("/libamdhip64.so") or "/libamdhip64.so." in path:
                    return path
    except OSError:
        pass
    return None


def _prewarm_hip():
    """A worker leased GPUs (CAAMD_GPU_IDS) initialises HIP on a thread while it
    registers with the head and receives its actor / task (~0.1 s), instead of inside
    the user's first CUDA call (0.2-0.37 s for a Data ResNet actor, PERF.md "Data
    start-up"). The runtime and the device context come up through ctypes calls into
    torch's own libamdhip64 (``hipInit`` / ``hipFree(0)``: ctypes drops the GIL, so the
    worker's main thread keeps running; ``torch.cuda.init()`` holds the GIL for all of
    it), then ``torch.cuda.init()`` finishes the torch side. Only when torch is already
    in the process (forked from the zygote, so importing it costs nothing) and a device
    is visible (counting devices does not initialise HIP); torch's lazy-init lock makes
    the user's own calls wait for it. Only for workers isolated to their GPUs
    (ROCR_VISIBLE_DEVICES set by the head, so device 0 is the leased one); Train
    worker groups see the whole node and are left alone. CAAMD_WORKER_HIP_PREWARM=0
    turns it off."""
    if os.environ.get("CAAMD_WORKER_HIP_PREWARM", "1") == "0" or not os.environ.get("CAAMD_GPU_IDS"):
        return
    if os.environ.get("CAAMD_NOSET_ROCR_VISIBLE_DEVICES") or not os.environ.get("ROCR_VISIBLE_DEVICES"):
        # every GPU of the node visible (Train worker groups, for RCCL P2P): device 0 is
        # not this worker's device, and a context there would be one per worker
        return
    torch = sys.modules.get("torch")
    if torch is None:
        return
    try:
        if torch.cuda.device_count() < 1:
            return
    except Exception:
        return

    def run():
        path = _loaded_hip_runtime()
        if path:
            try:
                hip = ctypes.CDLL(path)
                if hip.hipInit(0) == 0:
                    hip.hipFree(ctypes.c_void_p(0))  # the current device's context
            except Exception:
                pass
        try:
            torch.cuda.init()
        except Exception:
            pass

    import threading

    threading.Thread(target=run, name="caamd-hip-prewarm", daemon=True).start()


def main():
    if float(os.environ.get("CAAMD_HEAD_RECONNECT_S", "0") or 0) <= 0:
        _die_with_parent()
    _prewarm_hip()
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
