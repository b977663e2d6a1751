"""Multi-process (world_size 2, gloo, CPU) check of the image tiling + gather path used by bench.py
on N GPUs: each rank renders its row bands (oracle CPU renderer stands in for the device), the
bands are all-gathered and reassembled on rank 0, and the result equals the single-process render
bit for bit (the RNG is keyed by the global pixel index)."""
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle as O
from _rt import PKG

W, H, SPP, BAND = 37, 29, 3, 4


def _load_dist():
    spec = importlib.util.spec_from_file_location("rt_dist", os.path.join(PKG, "dist.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rtdist = _load_dist()
    gat = rtdist.ImageGather(W, H, BAND, rank, world, torch.device("cpu"))
    rows = rtdist.local_rows(H, BAND, rank, world)
    sc = O.Scene()
    acc = np.zeros((H, W, 4), np.float32)
    full = np.zeros((H, W), np.uint32)
    # render this rank's bands only (contiguous row runs)
    runs, start = [], rows[0]
    for a, b in zip(rows, rows[1:] + [None]):
        if b != a + 1:
            runs.append((start, a + 1))
            start = b
    for (r0, r1) in runs:
        a, rgba, _ = sc.render(W, H, SPP, seed=4, rows=(r0, r1), accum=acc)
        full[r0:r1] = rgba[r0:r1]
    gat.local_view().copy_(torch.from_numpy(full[rows].view(np.int32).ravel()))
    img = gat.gather()
    if rank == 0:
        np.save(out_path, img.numpy().view(np.uint32).reshape(H, W))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_band_gather_equals_single_process(tmp_path, world):
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    img = np.load(out)
    _, ref, _ = O.Scene().render(W, H, SPP, seed=4)
    assert np.array_equal(img, ref)


def test_local_rows_partition():
    d = _load_dist()
    for (H_, band, n) in [(1080, 8, 8), (29, 4, 3), (7, 8, 2), (2160, 8, 5)]:
        allr = sorted(sum((d.local_rows(H_, band, r, n) for r in range(n)), []))
        assert allr == list(range(H_))
