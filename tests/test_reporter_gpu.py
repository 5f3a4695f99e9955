"""The node reporter reads real MI355X telemetry (amdsmi, sysfs fallback): non-zero
GFX utilisation on the GPU this process keeps busy, HBM used / total."""
import threading
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_reporter_sees_busy_gpu():
    from cluster_anywhere_amd.dashboard import reporter

    gpus = reporter.sample_gpus()
    assert gpus, "no AMD GPU visible to amdsmi or sysfs"
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            for _ in range(20):
                a @ a
            torch.cuda.synchronize()

    th = threading.Thread(target=spin, daemon=True)
    th.start()
    try:
        time.sleep(0.5)
        best = {}
        for _ in range(20):
            for g in reporter.sample_gpus():
                u = g.get("utilization_gpu") or 0.0
                best[g["index"]] = max(best.get(g["index"], 0.0), u)
            time.sleep(0.1)
    finally:
        stop.set()
        th.join(timeout=30)
    print("reporter gpus:", reporter.sample_gpus(), "max utilisation:", best)
    assert max(best.values()) > 0.0
    g0 = max(reporter.sample_gpus(), key=lambda g: g.get("memory_used", 0))
    assert g0.get("memory_total", 0) > 200 << 30 and g0.get("memory_used", 0) > 100 << 20
