"""Every tensor entry point of the HIP extension runs under a device guard on
its tensors' GPU and refuses tensors on different GPUs (csrc/kernels/bindings.cpp
GUARDED / DeviceSel). The selection rule is exercised on the CPU through
``_C._select_device``; the guarded bindings themselves run in the GPU suite."""
import importlib
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ext():
    import torch  # noqa: F401  (loads the HIP runtime the extension links against)

    try:
        return importlib.import_module("cluster_anywhere_amd._C")
    except ImportError as e:  # pragma: no cover - the build check runs first
        pytest.skip(f"extension not built: {e}")


def test_select_device_rule():
    C = _ext()
    assert C._select_device([]) == -1
    assert C._select_device([(False, -1), (False, -1)]) == -1       # CPU-only arguments: no guard
    assert C._select_device([(False, -1), (True, 3), (True, 3)]) == 3
    with pytest.raises(RuntimeError, match="different GPUs"):
        C._select_device([(True, 0), (False, -1), (True, 1)])


def test_every_tensor_binding_is_guarded():
    src = open(os.path.join(ROOT, "csrc", "kernels", "bindings.cpp")).read()
    mod = src[src.index("PYBIND11_MODULE(_C, m)"):]
    defs = re.findall(r'm\.def\("([A-Za-z0-9_]+)",\s*([^,)]+)', mod)
    assert len(defs) > 30
    unguarded = [n for n, target in defs if target.strip().startswith("&") and not n.startswith("_")]
    assert not unguarded, f"bindings registered without GUARDED(): {unguarded}"
