"""GPU workers prewarm HIP on a thread at start-up (core/worker_main.py _prewarm_hip;
PERF.md round 6 "Data start-up"). CPU checks: the runtime lookup finds torch's own
libamdhip64 once torch is imported, and the prewarm starts no thread when it must not
(no GPU lease, opted out, or no visible device)."""
import threading

import torch  # noqa: F401  (the prewarm only runs where torch is already imported)

from cluster_anywhere_amd.core import worker_main as wm


def _prewarm_threads():
    return [t for t in threading.enumerate() if t.name == "caamd-hip-prewarm"]


def test_loaded_hip_runtime_is_torchs_copy():
    path = wm._loaded_hip_runtime()
    assert path is None or ("libamdhip64.so" in path and "torch" in path)


def test_prewarm_skips_without_lease_or_device(monkeypatch):
    before = len(_prewarm_threads())
    monkeypatch.delenv("CAAMD_GPU_IDS", raising=False)
    wm._prewarm_hip()  # no GPU lease
    monkeypatch.setenv("CAAMD_GPU_IDS", "0")
    monkeypatch.setenv("CAAMD_WORKER_HIP_PREWARM", "0")
    wm._prewarm_hip()  # opted out
    monkeypatch.setenv("CAAMD_WORKER_HIP_PREWARM", "1")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    wm._prewarm_hip()  # leased, but every GPU visible (no isolation)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0")
    monkeypatch.setenv("CAAMD_NOSET_ROCR_VISIBLE_DEVICES", "1")
    wm._prewarm_hip()  # Train worker group (NOSET)
    monkeypatch.delenv("CAAMD_NOSET_ROCR_VISIBLE_DEVICES")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    wm._prewarm_hip()  # isolated, but no device visible
    assert len(_prewarm_threads()) == before
