"""Start-up components of a fresh GPU process (the Data ResNet actor's critical path),
each in its own child process so every number is a cold start:

  torch_cuda_init   torch.cuda.init() + a first allocation
  hip_init_thread   hipInit + hipSetDevice + hipFree(0) through ctypes on a thread
                    (ctypes drops the GIL), then torch.cuda.init()
  cpu_build_resnet  ResNet-50 random init + BN fold on the CPU (torch, 1 and 4 threads)
  predictor         ResNetPredictor(...) end to end (its init_profile)

    python tools/actor_init_probe.py   -> one JSON line per probe
"""
from __future__ import annotations

import ast
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBES = {
    "torch_cuda_init": r"""
import time; t0=time.perf_counter()
import torch; t1=time.perf_counter()
torch.cuda.init(); x=torch.empty(1, device='cuda'); torch.cuda.synchronize(); t2=time.perf_counter()
print({'import_torch_s': t1-t0, 'cuda_init_s': t2-t1})
""",
    "hip_init_thread": r"""
import time, threading, ctypes; t0=time.perf_counter()
import torch; t1=time.perf_counter()
hip = ctypes.CDLL('libamdhip64.so')
done = {}
def f():
    a=time.perf_counter(); hip.hipInit(0); hip.hipSetDevice(0); hip.hipFree(ctypes.c_void_p(0)); done['hip_s']=time.perf_counter()-a
th=threading.Thread(target=f); th.start()
a=time.perf_counter(); s=0.0
while th.is_alive():  # the main thread keeps running Python meanwhile
    s+=1.0
main_spin_s=time.perf_counter()-a
th.join(); t2=time.perf_counter()
torch.cuda.init(); x=torch.empty(1, device='cuda'); torch.cuda.synchronize(); t3=time.perf_counter()
print({'import_torch_s': t1-t0, 'hip_thread_s': done['hip_s'], 'main_thread_ran_s': main_spin_s, 'torch_init_after_s': t3-t2})
""",
    "cpu_build_resnet_1t": r"""
import time, torch; torch.set_num_threads(1)
import sys; sys.path.insert(0, %r)
from cluster_anywhere_amd.models.resnet import resnet
t0=time.perf_counter(); net=resnet('resnet50').eval(); t1=time.perf_counter()
ws=[]
for m in net.modules():
    if isinstance(m, torch.nn.BatchNorm2d):
        ws.append(m.weight/torch.sqrt(m.running_var+m.eps))
t2=time.perf_counter()
print({'cpu_init_s': t1-t0, 'fold_stats_s': t2-t1})
""" % ROOT,
    "cpu_build_resnet_4t": r"""
import time, torch; torch.set_num_threads(4)
import sys; sys.path.insert(0, %r)
from cluster_anywhere_amd.models.resnet import resnet
t0=time.perf_counter(); net=resnet('resnet50').eval(); t1=time.perf_counter()
print({'cpu_init_s': t1-t0})
""" % ROOT,
    "predictor": r"""
import time, sys; t0=time.perf_counter()
import torch; sys.path.insert(0, %r)
from cluster_anywhere_amd.models.resnet import ResNetPredictor
t1=time.perf_counter()
p=ResNetPredictor('resnet50', batch_size=512, hw=224)
t2=time.perf_counter()
print({'import_s': t1-t0, 'predictor_s': t2-t1, **{k: round(v, 3) for k, v in p.init_profile.items()}})
""" % ROOT,
}


def main():
    names = sys.argv[1:] or list(PROBES)
    for rnd in range(2):
        for n in names:
            r = subprocess.run([sys.executable, "-c", PROBES[n]], capture_output=True, text=True, timeout=120)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            out = ast.literal_eval(line[-1]) if line else {"error": r.stderr[-500:]}
            print(json.dumps({"probe": n, "round": rnd, **{k: (round(v, 3) if isinstance(v, float) else v)
                                                              for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
