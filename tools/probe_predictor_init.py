"""Time a fresh ResNetPredictor's construction phases (what a new Data GPU actor
pays before its first batch): CUDA init, random init, BN fold + weight packing,
HIP-graph capture; then the first and second batch."""
import json
import os
import sys
import time

t0 = time.perf_counter()
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t1 = time.perf_counter()
from cluster_anywhere_amd.models.resnet import ResNetPredictor  # noqa: E402

t2 = time.perf_counter()
p = ResNetPredictor("resnet50", batch_size=512)
t3 = time.perf_counter()
import numpy as np  # noqa: E402

x = np.full((512, 224, 224, 3), 7, dtype=np.uint8)
a = time.perf_counter()
p(x)
b = time.perf_counter()
p(x)
c = time.perf_counter()
print(json.dumps({"import_torch_s": round(t1 - t0, 3), "import_pkg_s": round(t2 - t1, 3),
                  "construct_s": round(t3 - t2, 3), **{k: round(v, 3) for k, v in p.init_profile.items()},
                  "first_batch_s": round(b - a, 3), "second_batch_s": round(c - b, 3)}), flush=True)
