"""Stale object-store segments (owner pid gone) are unlinked when a new head
starts; segments of live pids, segments a live process still maps (a dead head's
arena that its workers hold for a restarted head) and unrelated files stay (reference role:
python/ray/_private/node.py cleans up the previous session's plasma files)."""
import mmap
import os
import subprocess
import sys

from cluster_anywhere_amd.core.api import _sweep_stale_stores


def test_sweep_removes_only_dead_owner_segments():
    dead = subprocess.run([sys.executable, "-c", "import os; print(os.getpid())"], capture_output=True,
                          text=True).stdout.strip()
    stale = f"/dev/shm/caamd_{dead}_0123abcd"
    stale_node = f"/dev/shm/caamd_node_{dead}_4567cdef"
    live = f"/dev/shm/caamd_{os.getpid()}_89abcdef"
    other = "/dev/shm/caamd_not_a_store_test"
    for p in (stale, stale_node, live, other):
        with open(p, "wb") as f:
            f.write(b"x")
    mapped = f"/dev/shm/caamd_{dead}_fedcba98"  # dead owner, but a live process maps it
    with open(mapped, "wb") as f:
        f.write(b"x" * 4096)
    f = open(mapped, "r+b")
    mm = mmap.mmap(f.fileno(), 4096)
    try:
        assert _sweep_stale_stores() >= 2
        assert not os.path.exists(stale) and not os.path.exists(stale_node)
        assert os.path.exists(live) and os.path.exists(other) and os.path.exists(mapped)
    finally:
        mm.close()
        f.close()
        for p in (stale, stale_node, live, other, mapped):
            if os.path.exists(p):
                os.unlink(p)
