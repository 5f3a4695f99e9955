"""Time bias_grad_ (column sums of dy [32768, 1600]) on the in-tree extension or
another build (BG_SO=path, same-box A/B)."""
import importlib.machinery
import importlib.util
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import kernels  # noqa: E402

C = kernels()
if os.environ.get("BG_SO"):
    _ld = importlib.machinery.ExtensionFileLoader("caamd_ab._C", os.environ["BG_SO"])
    _spec = importlib.util.spec_from_loader("caamd_ab._C", _ld)
    C = importlib.util.module_from_spec(_spec)
    _ld.exec_module(C)
dy = torch.randn(32768, 1600, device="cuda").to(torch.bfloat16)
out = torch.zeros(1600, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    C.bias_grad_(dy, out, True)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(50):
    C.bias_grad_(dy, out, True)
e.record()
torch.cuda.synchronize()
print(json.dumps({"so": os.environ.get("BG_SO", "tree"), "us": round(s.elapsed_time(e) / 50 * 1e3, 1)}))
