"""Multi-process row bands on the GPU: the bench.py / dist.py path (one process per rank, each rendering
its row bands of MC/Renderer.cpp:100-110's loop with the HIP kernels, the RGBA8 bands all-gathered and
reassembled on rank 0), run with two ranks on the box's one GPU.  Two ranks cannot share a device under
RCCL, so the gather runs over gloo on host copies of the bands; the bands themselves come from the HIP
library.  The reassembled frame must equal the one-rank frame bit for bit."""
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W, H, SPP, BAND = 96, 70, 6, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _worker(rank, world, port, out_dir, scene_kind):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpu-based-ray-tracer_amd")
    rt = _load("rt_amd_w%d" % rank, os.path.join(pkg, "__init__.py"))
    rtdist = _load("rt_dist_w%d" % rank, os.path.join(pkg, "dist.py"))
    if scene_kind == "c5":
        raw = np.load(os.path.join(os.path.dirname(__file__), "golden", "bvh_scene.npz"))["raw_bunny"]
        scene = rt.Scene.cornell_c5(raw)
    else:
        scene = rt.Scene.cornell()
    c = rt.Context(0)
    c.upload(scene)
    c.resize(W, H, BAND, rank, world)
    cam, _, _ = rt.camera_default(W, H)
    rgba, _ = c.render(cam, SPP, seed=11)
    gat = rtdist.ImageGather(W, H, BAND, rank, world, torch.device("cpu"))
    assert gat.n_local == rgba.shape[0]
    gat.local_view().copy_(torch.from_numpy(np.ascontiguousarray(rgba).view(np.int32).ravel()))
    img = gat.gather()
    if rank == 0:
        c.resize(W, H, BAND, 0, 1)
        one, _ = c.render(cam, SPP, seed=11)
        np.save(os.path.join(out_dir, "gathered.npy"), img.numpy().view(np.uint32).reshape(H, W))
        np.save(os.path.join(out_dir, "one.npy"), np.ascontiguousarray(one).view(np.uint32).reshape(H, W))
    c.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scene_kind", ["cornell", "c5"])
def test_two_process_row_bands_equal_one_rank(tmp_path, scene_kind):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), scene_kind), nprocs=2, join=True)
    g = np.load(tmp_path / "gathered.npy")
    one = np.load(tmp_path / "one.npy")
    assert np.array_equal(g, one)
