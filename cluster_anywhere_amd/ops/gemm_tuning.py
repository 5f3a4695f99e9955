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
    # CAAMD_TUNE_GEMMS=<csv>: online-tune every shape the run issues that the
    # shipped tables miss (exact shapes/layouts/bias epilogues of the real step),
    # then write shipped + new winners to <csv> at exit (merge it into tuning/).
    out = os.environ.get("CAAMD_TUNE_GEMMS", "")
    tn.tuning_enable(bool(out))
    if out:
        tn.set_max_tuning_duration(60)
        tn.set_max_tuning_iterations(20)
    ok = False
    for t in tables():
        try:
            ok = bool(tn.read_file(t)) or ok
        except Exception:
            pass
    if out:
        tn.set_filename(out, False)

        def _beat():  # tuning a shape can take a minute: keep the run visibly alive
            import sys
            import time

            t0 = time.time()
            while True:
                time.sleep(30)
                print(f"# gemm tuning ... {time.time() - t0:.0f}s", file=sys.stderr, flush=True)

        import threading

        threading.Thread(target=_beat, daemon=True).start()
    _DONE = True
    return ok


def dump_tuned() -> None:
    """Write shipped + newly tuned winners to ``$CAAMD_TUNE_GEMMS`` (no-op otherwise)."""
    out = os.environ.get("CAAMD_TUNE_GEMMS", "")
    if not out or not _DONE:
        return
    import importlib.util

    import torch.cuda.tunable as tn

    path = os.path.join(os.path.dirname(os.path.dirname(TUNING_DIR)), "tools", "bench_gemm.py")
    spec = importlib.util.spec_from_file_location("_caamd_bench_gemm", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    mod.write_results(tn, out)
