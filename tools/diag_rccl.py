"""Standalone check of a directly-constructed RCCL process group (world 1), with a
progress line after every step (diagnoses util.collective's RCCL path)."""
import datetime
import os
import sys
import time

import torch
import torch.distributed as dist

t0 = time.time()


def say(m):
    print(f"[{time.time() - t0:6.1f}s] {m}", flush=True)


mode = sys.argv[1] if len(sys.argv) > 1 else "eager"
torch.cuda.set_device(0)
say("device set")
store = dist.TCPStore("127.0.0.1", 0, 1, True, datetime.timedelta(seconds=60), wait_for_workers=False)
say(f"store on port {store.port}")
opts = dist.ProcessGroupNCCL.Options()
opts._timeout = datetime.timedelta(seconds=60)
opts.group_name = "diag"
pg = dist.ProcessGroupNCCL(store, 0, 1, opts)
say("pg constructed")
if mode == "eager":
    pg.eager_connect_single_device(torch.device("cuda", 0))
    say("eager connect done")
t = torch.full((1024,), 2.0, device="cuda")
o = dist.AllreduceOptions()
o.reduceOp = dist.ReduceOp.SUM
pg.allreduce([t], o).wait()
torch.cuda.synchronize()
say(f"allreduce ok sum={float(t.sum())}")
b = dist.BroadcastOptions()
b.rootRank = 0
b.rootTensor = 0
pg.broadcast([t], b).wait()
torch.cuda.synchronize()
say("broadcast ok")
pg.shutdown()
say("shutdown ok")
