"""The node-wide copy-thread budget of the native object store survives a putter
that dies mid-copy: its claim slot names its pid, and the next large put reclaims
the slot of a dead pid instead of leaking those threads for the life of the store
(before: one shared counter, decremented only by the putter's own destructor)."""
import os
import subprocess
import sys
import uuid

import numpy as np

from cluster_anywhere_amd import _native


def _dead_pid() -> int:
    return int(subprocess.run([sys.executable, "-c", "import os; print(os.getpid())"], capture_output=True,
                              text=True).stdout.strip())


def test_dead_putter_claim_is_reclaimed():
    name = f"/caamd_test_budget_{uuid.uuid4().hex[:8]}"
    st = _native.ObjectStore(name, 256 << 20, 1 << 10, True)
    try:
        assert st.copy_threads_claimed() == 0
        st._debug_plant_claim(_dead_pid(), 64)  # a SIGKILLed putter's claim: the whole budget
        st._debug_plant_claim(os.getpid(), 0)   # a live claim of zero threads stays
        assert st.copy_threads_claimed() == 64
        data = np.ones(96 << 20, dtype=np.uint8)
        off = st.create(b"x" * 24, data.nbytes, 0)
        assert off >= 0
        st.copy_in(off, data, 4)
        assert st.copy_threads_claimed() == 0  # the dead claim was reclaimed, ours released
        view = np.frombuffer(st.buffer(off, data.nbytes), dtype=np.uint8)
        assert view[-1] == 1
    finally:
        st.unlink()
