#!/usr/bin/env python
"""Phase breakdown of a GPU map_batches actor's start-up (what bounds Data's
time-to-first-batch): CUDA init, model init, BN folding, arena pinning, warm-up
runs and HIP-graph capture of ResNetPredictor, in a fresh process."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t_start = time.perf_counter()
import torch  # noqa: E402

t_torch = time.perf_counter()
from cluster_anywhere_amd.models.resnet import ResNetPredictor  # noqa: E402

p = ResNetPredictor("resnet50", batch_size=int(sys.argv[1]) if len(sys.argv) > 1 else 512)
import numpy as np  # noqa: E402

x = np.zeros((p.bs, 224, 224, 3), np.uint8)
t0 = time.perf_counter()
p(x)
torch.cuda.synchronize()
print(json.dumps({"import_torch_s": round(t_torch - t_start, 3), **{k: round(v, 3) for k, v in p.init_profile.items()},
                  "first_call_s": round(time.perf_counter() - t0, 3)}), flush=True)

# the same start-up inside a GPU actor of a running cluster (arena pinning included)
import cluster_anywhere_amd as ray  # noqa: E402

ray.init(num_cpus=4, num_gpus=1, object_store_memory=5 << 30)


@ray.remote(num_gpus=1)
class _A:
    def __init__(self):
        self.t_enter = time.time()
        self.p = ResNetPredictor("resnet50", batch_size=512)

    def prof(self):
        return dict(self.p.init_profile, t_enter=self.t_enter)


t_submit = time.time()
a = _A.remote()
prof = ray.get(a.prof.remote())
print(json.dumps({"actor_ready_s": round(time.time() - t_submit, 3),
                  "actor_process_start_s": round(prof.pop("t_enter") - t_submit, 3),
                  **{k: round(v, 3) for k, v in prof.items()}}), flush=True)
ray.shutdown()
