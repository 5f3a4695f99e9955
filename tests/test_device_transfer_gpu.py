"""Side-stream host->HBM prefetch must not hand a dropped batch's HBM to the next
copy while compute still reads it (reference: python/ray/train/torch/
train_loop_utils.py:688-703, ``record_stream`` on every moved tensor).

Each consumer below queues ``torch.cuda._sleep`` on the compute stream before it
reads a batch, then drops the batch at once: without ``record_stream`` the next
prefetch copy (side stream, not delayed) reuses the freed block and the delayed
read sees the NEXT batch's values."""
import numpy as np
import pytest
import torch

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data as rd

pytestmark = pytest.mark.gpu

ROWS, WIDTH, BS = 64, 1 << 16, 8  # 8 batches of 8 x 65536 float32 (2 MiB each)
SLEEP = 5_000_000  # GPU cycles per batch (a few ms)


def _consume_delayed(batches, key):
    """Sum every batch AFTER a GPU-side delay, dropping the batch right away."""
    sums = []
    for b in batches:
        t = b[key] if isinstance(b, dict) else b[0]
        torch.cuda._sleep(SLEEP)
        sums.append(t.double().sum(dim=1))  # queued behind the sleep
        del t, b
    torch.cuda.synchronize()
    return torch.cat(sums).cpu().numpy()


def test_side_stream_mover_records_on_compute_stream():
    from cluster_anywhere_amd.util.device_transfer import SideStreamMover

    dev = torch.device("cuda", 0)
    host = [torch.full((BS, WIDTH), float(i), dtype=torch.float32).pin_memory() for i in range(ROWS // BS)]
    mover = SideStreamMover(dev)

    def gen():
        nxt = None
        for hb in host:
            ready = mover.hand_over(nxt) if nxt is not None else None
            nxt = mover.stage(hb)
            if ready is not None:
                yield {"x": ready}
        yield {"x": mover.hand_over(nxt)}

    got = _consume_delayed(gen(), "x")
    want = np.repeat(np.arange(ROWS // BS, dtype=np.float64) * WIDTH, BS)
    np.testing.assert_array_equal(got, want)
    mover.close()


def test_train_device_loader_no_reuse_race():
    from torch.utils.data import DataLoader, TensorDataset

    from cluster_anywhere_amd.train.torch import _DeviceLoader

    x = torch.arange(ROWS, dtype=torch.float32)[:, None].expand(ROWS, WIDTH).contiguous()
    dl = DataLoader(TensorDataset(x), batch_size=BS, pin_memory=True)
    got = _consume_delayed(_DeviceLoader(dl, torch.device("cuda", 0)), None)
    np.testing.assert_array_equal(got, np.arange(ROWS, dtype=np.float64) * WIDTH)


def test_iter_torch_batches_no_reuse_race():
    ray.init(num_cpus=2, num_gpus=1)
    try:
        arr = np.repeat(np.arange(ROWS, dtype=np.float32)[:, None], WIDTH, axis=1)
        ds = rd.from_numpy(arr).repartition(ROWS // BS)
        got = _consume_delayed(ds.iter_torch_batches(batch_size=BS, device="cuda:0"), "data")
        np.testing.assert_array_equal(np.sort(got), np.arange(ROWS, dtype=np.float64) * WIDTH)
        assert len(np.unique(got)) == ROWS
    finally:
        ray.shutdown()
