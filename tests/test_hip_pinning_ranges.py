"""arena_contains: a buffer counts as registered only inside ONE registered chunk
(cluster_anywhere_amd/core/hip_pinning.py); CPU-only, the chunk table is planted."""
import numpy as np

from cluster_anywhere_amd.core import hip_pinning as hp


def test_arena_contains_single_chunk_only(monkeypatch):
    buf = np.zeros(4096, np.uint8)
    base = buf.__array_interface__["data"][0]
    monkeypatch.setattr(hp, "_chunks", [(base, base + 2048), (base + 2048, base + 4096)])
    monkeypatch.setattr(hp, "_starts", [base, base + 2048])
    assert hp.arena_contains(buf[:2048])
    assert hp.arena_contains(buf[2048:])
    assert hp.arena_contains(buf[100:200])
    assert not hp.arena_contains(buf[2000:2100])  # straddles two registrations
    assert not hp.arena_contains(np.zeros(16, np.uint8))  # outside the arena


def test_arena_contains_nothing_registered(monkeypatch):
    monkeypatch.setattr(hp, "_chunks", [])
    monkeypatch.setattr(hp, "_starts", [])
    assert not hp.arena_contains(np.zeros(16, np.uint8))
