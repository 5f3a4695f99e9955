"""Per-shape GEMM kernel selection for the plain library GEMMs (hipBLASLt /
rocBLAS) of the training step.

hipBLASLt's default heuristic picks a mediocre kernel for several GPT-2-XL
shapes on gfx950 (e.g. the 1600x1600 projection weight-gradient, 49 output
tiles of 256x256 on a 256-CU chip, runs at ~500 TF/s). ``tools/bench_gemm.py
--tune`` searches every hipBLASLt and rocBLAS solution for each shape the step
issues (torch TunableOp) on an MI355X; the winning solution ids are shipped in
``cluster_anywhere_amd/tuning/*.csv`` and loaded here with tuning DISABLED — so
a run only looks kernels up, it never benchmarks. Shapes not in the table use
the library default. The table is validated by TunableOp against the torch /
HIP / hipBLASLt / rocBLAS versions and the GPU arch it was tuned on; on any
mismatch it is ignored (library default kernels, same numerics).
"""
from __future__ import annotations

import glob
import os

_DONE = False
TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def tables():
    return sorted(glob.glob(os.path.join(TUNING_DIR, "gemm_gfx950_*.csv")))


def use_tuned_gemms() -> bool:
    """Enable the shipped GEMM selections (idempotent). ``CAAMD_TUNED_GEMMS=0`` disables."""
    global _DONE
    if _DONE:
        return True
    if os.environ.get("CAAMD_TUNED_GEMMS", "1") == "0":
        return False
    import torch

    if not torch.cuda.is_available() or not tables():
        return False
    import torch.cuda.tunable as tn

    tn.enable(True)
    tn.tuning_enable(False)
    try:
        tn.write_file_on_exit(False)
    except Exception:
        pass
    ok = False
    for t in tables():
        try:
            ok = bool(tn.read_file(t)) or ok
        except Exception:
            pass
    _DONE = True
    return ok
