"""Several GPUs, one frame, behind the C-ABI (rt_group_*, include/rt_capi.h): the row bands of
Renderer::Render's row loop (MC/Renderer.cpp:100-110) dealt over the members, each member's band set
rendered on its own device and stream, the RGBA8 bands gathered to member 0 and reassembled.

One GPU box: members may share a device (the copy gather; RCCL takes one rank per GPU), and a
one-member group exercises the RCCL gather (ncclCommInitAll + ncclGather with one rank).  The image is
compared bit for bit with the one-context render, which the parity tests compare with the oracle.
The 8-GPU RCCL gather itself is not run here (driver-run scaling bench only)."""
import os

import numpy as np
import pytest

from _rt import rt


def test_group_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available() or os.path.exists("/dev/kfd"):
        pytest.skip("GPU present")
    with pytest.raises(rt.RtError):
        rt.Group([0, 0])


def single(W, H, spp, seed=3, first_frame=1, ctx=None):
    c = ctx or rt.Context(0)
    if ctx is None:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
    cam, _, _ = rt.camera_default(W, H)
    rgba, acc = c.render(cam, spp, first_frame=first_frame, seed=seed)
    return c, rgba, acc


@pytest.mark.gpu
@pytest.mark.parametrize("devices,band,W,H", [([0, 0], 8, 96, 72), ([0, 0, 0], 8, 83, 61), ([0, 0, 0, 0], 4, 64, 50),
                                             ([0] * 8, 8, 40, 1080)])
def test_group_copy_gather_equals_one_device(devices, band, W, H):
    """members on one GPU (copy gather), ragged band counts: RGBA8 and accumulation bitwise equal; eight members
    over C4's 1080 rows (135 bands: seven members own 17, one 16)"""
    c, rgba1, acc1 = single(W, H, 8)
    c.close()
    g = rt.Group(devices)
    g.upload(rt.Scene.cornell())
    g.resize(W, H, band)
    cam, _, _ = rt.camera_default(W, H)
    rgba = g.render(cam, 8, seed=3)
    assert g.stats().gather == 0 and g.stats().n == len(devices)
    assert np.array_equal(rgba, rgba1)
    assert np.array_equal(g.accumulation().view(np.uint32), acc1.view(np.uint32))
    g.close()


@pytest.mark.gpu
def test_group_one_member_rccl_gather():
    """a one-member group on device 0 takes the RCCL path (one rank): same frame"""
    W, H = 72, 40
    c, rgba1, _ = single(W, H, 4)
    c.close()
    g = rt.Group([0])
    g.upload(rt.Scene.cornell())
    g.resize(W, H)
    cam, _, _ = rt.camera_default(W, H)
    rgba = g.render(cam, 4, seed=3)
    st = g.stats()
    assert st.n == 1 and st.gather in (0, 1)
    if st.gather == 0:
        pytest.skip("RCCL communicator not available on this box (copy gather used)")
    assert np.array_equal(rgba, rgba1)
    assert st.last_ms > 0 and st.max_member_kernel_ms > 0
    g.close()


@pytest.mark.gpu
def test_group_incremental_and_device_frame():
    """Render(+4 spp) twice == one 8-spp render; the assembled frame on member 0's device is the host copy"""
    import torch
    W, H = 64, 48
    c, rgba1, acc1 = single(W, H, 8, seed=5)
    c.close()
    g = rt.Group([0, 0])
    g.upload(rt.Scene.cornell())
    g.resize(W, H, 8)
    cam, _, _ = rt.camera_default(W, H)
    g.render(cam, 4, first_frame=1, seed=5, fetch=False)
    rgba = g.render(cam, 4, first_frame=5, seed=5)
    assert np.array_equal(rgba, rgba1)
    assert np.array_equal(g.accumulation().view(np.uint32), acc1.view(np.uint32))
    ptr = g.frame_device()
    t = torch.empty((H, W), dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(W * H * 4), 3) == 0   # D2D
    assert np.array_equal(t.cpu().numpy().view(np.uint32), rgba)
    g.close()
