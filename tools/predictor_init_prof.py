#!/usr/bin/env python
"""Start-up phases of ResNetPredictor (the Data bench's actor constructor):
first construction in a fresh process vs a second one in the same process (no
first-time library / code-object loads), plus a first-call breakdown per op."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t0 = time.perf_counter()
import torch  # noqa: E402

t1 = time.perf_counter()
from cluster_anywhere_amd.models.resnet import ResNetPredictor, resnet  # noqa: E402

t2 = time.perf_counter()
print(json.dumps({"import_torch_s": round(t1 - t0, 3), "import_resnet_s": round(t2 - t1, 3)}), flush=True)
if os.environ.get("BREAKDOWN") == "1":
    import torch.nn.functional as F

    from cluster_anywhere_amd.ops.vision import IMAGENET_MEAN, IMAGENET_STD, maxpool3s2_nhwc, normalize_pad8

    ph = {}

    def mark(name, t):
        torch.cuda.synchronize()
        ph[name] = round(time.perf_counter() - t, 4)
        return time.perf_counter()

    t = time.perf_counter()
    torch.cuda.init()
    torch.zeros(1, device="cuda")
    t = mark("cuda_init", t)
    with torch.device("cuda"):
        net = resnet("resnet50").eval()
    t = mark("model_init", t)
    m = net.fuse_for_inference(torch.bfloat16, torch.device("cuda"))
    t = mark("fuse", t)
    x = torch.zeros((8, 224, 224, 3), dtype=torch.uint8, device="cuda")
    x8 = normalize_pad8(x, IMAGENET_MEAN, IMAGENET_STD)
    t = mark("normalize", t)
    y = m.stem.own(x8)
    t = mark("stem", t)
    y = maxpool3s2_nhwc(y)
    t = mark("maxpool", t)
    for convs, down in m.blocks:
        idt = y if down is None else down.own(y)
        z = y
        for c in convs[:-1]:
            z = c.own(z)
        y = convs[-1].own(z, residual=idt)
    t = mark("blocks", t)
    v = y.mean(dim=(1, 2))
    t = mark("mean", t)
    lg = F.linear(v, m.fc_w, m.fc_b)
    t = mark("linear", t)
    lg.argmax(dim=1)
    t = mark("argmax", t)
    xs = torch.zeros((512, 224, 224, 3), dtype=torch.uint8, device="cuda")
    t = mark("alloc_in", t)
    g = torch.cuda.CUDAGraph()
    t = time.perf_counter()
    with torch.cuda.graph(g):
        out = m.predict_uint8(xs).argmax(dim=1)
        t_rec = time.perf_counter()
    ph["capture_record"] = round(t_rec - t, 4)
    t = mark("capture_total", t)
    g.replay()
    t = mark("replay1", t)
    print(json.dumps(ph), flush=True)
else:
    for i in range(2):
        p = ResNetPredictor("resnet50", batch_size=512, hw=224)
        print(json.dumps({"construction": i, **{k: round(v, 3) for k, v in p.init_profile.items()}}), flush=True)
        del p
        torch.cuda.empty_cache()
