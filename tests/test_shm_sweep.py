"""Stale object-store segments (owner pid gone) are unlinked when a new head
starts; segments of live pids, segments a live process still maps (a dead head's
arena that its workers hold for a restarted head), segments of another PID
namespace (another container sharing /dev/shm) and unrelated files stay (reference
role: python/ray/_private/node.py cleans up the previous session's plasma files)."""
import mmap
import os
import subprocess
import sys

from cluster_anywhere_amd.core.api import _pid_ns, _sweep_stale_stores, store_segment_name


def test_segment_names_carry_the_pid_namespace():
    n = store_segment_name()
    assert n.startswith(f"/caamd_{os.getpid()}_{_pid_ns()}_")
    assert store_segment_name(node=True).startswith(f"/caamd_node_{os.getpid()}_{_pid_ns()}_")


def test_sweep_removes_only_dead_owner_segments_of_this_namespace():
    dead = subprocess.run([sys.executable, "-c", "import os; print(os.getpid())"], capture_output=True,
                          text=True).stdout.strip()
    ns = _pid_ns()
    foreign_ns = format(int(ns, 16) + 1, "x")
    stale = f"/dev/shm/caamd_{dead}_{ns}_0123abcd"
    stale_node = f"/dev/shm/caamd_node_{dead}_{ns}_4567cdef"
    live = f"/dev/shm/caamd_{os.getpid()}_{ns}_89abcdef"
    other = "/dev/shm/caamd_not_a_store_test"
    foreign = f"/dev/shm/caamd_{dead}_{foreign_ns}_13579bdf"  # another container's live arena
    legacy = f"/dev/shm/caamd_{dead}_2468ace0"  # no namespace in the name: never judged
    for p in (stale, stale_node, live, other, foreign, legacy):
        with open(p, "wb") as f:
            f.write(b"x")
    mapped = f"/dev/shm/caamd_{dead}_{ns}_fedcba98"  # dead owner, but a live process maps it
    with open(mapped, "wb") as f:
        f.write(b"x" * 4096)
    f = open(mapped, "r+b")
    mm = mmap.mmap(f.fileno(), 4096)
    try:
        assert _sweep_stale_stores() >= 2
        assert not os.path.exists(stale) and not os.path.exists(stale_node)
        for p in (live, other, mapped, foreign, legacy):
            assert os.path.exists(p), p
    finally:
        mm.close()
        f.close()
        for p in (stale, stale_node, live, other, mapped, foreign, legacy):
            if os.path.exists(p):
                os.unlink(p)
