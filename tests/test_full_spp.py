"""The benchmarked Cornell configurations at their FULL spp: C2 784x784x256 and C4
1920x1080x1024 (the bench.py workload), seed 0, RR 0.8, frames 1..spp -- the reference's accumulation over
every frame (MC/Renderer.cpp:114-133), its average, clamp and RGBA8 pack.

Golden vectors: tests/golden/full_c2.npz, full_c4.npz from oracle/_ref/ref_harness (the reference's own MC/
BVH, triangle, material and camera code compiled from /root/reference, the Philox words injected into its
mt19937; oracle/gen_golden.py `full`): the SHA-256 of the whole float4 accumulation and RGBA8 frame, and
every 16th row of the accumulation.

CPU: the oracle (the restatement) reproduces committed rows at full spp bit for bit.
GPU: the C-ABI renders both frames in the bench's launch shape (one rt_render of all frames from frame 1:
frame chunks, pre-pass segments and parts as the bench runs them) and the accumulation and RGBA8 frame
hash to the reference's."""
import hashlib
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt


def fixture(name):
    return np.load(os.path.join(O.GOLDEN, f"full_{name}.npz"))


def test_fixture_shapes():
    for name, (W, H, spp) in (("c2", (784, 784, 256)), ("c4", (1920, 1080, 1024))):
        z = fixture(name)
        assert (int(z["W"]), int(z["H"]), int(z["spp"]), int(z["seed"]), int(z["first_frame"])) == (W, H, spp, 0, 1)
        assert np.array_equal(z["rows"], np.arange(0, H, 16))
        assert z["accum_rows"].shape == (len(z["rows"]), W, 3)
        # the alpha channel accumulates 1 per frame: the 8-bit alpha is 255 everywhere
        assert np.all((z["rgba_rows"] >> 24) == 255)
        assert int(z["stats"][4]) == W * H * spp and int(z["stats"][3]) == 0   # samples; no harness overflow


@pytest.mark.parametrize("name,row", [("c2", 400), ("c4", 544)])
def test_oracle_reproduces_full_spp_rows(name, row):
    """The restatement at full spp on one committed row (a row through the boxes), bit for bit."""
    z = fixture(name)
    W, H, spp = int(z["W"]), int(z["H"]), int(z["spp"])
    k = int(np.where(z["rows"] == row)[0][0])
    acc, rgba, _ = O.Scene().render(W, H, spp, seed=0, rr=0.8, threads=min(8, os.cpu_count() or 1), rows=(row, row + 1))
    assert np.array_equal(acc[row, :, :3].view(np.uint32), z["accum_rows"][k].view(np.uint32))
    assert np.array_equal(rgba[row], z["rgba_rows"][k])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c2", "c4"])
def test_full_spp_frame_matches_reference(name):
    z = fixture(name)
    W, H, spp = int(z["W"]), int(z["H"]), int(z["spp"])
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, first_frame=1, seed=0, rr=0.8)
        st = c.stats()
        assert st.kernel == 1 and st.overflow_lost == 0 and st.kernel_reason == rt.KERNEL_REASON_DEFAULT
    finally:
        c.close()
    rows = acc[z["rows"], :, :3]
    same = np.all(rows.view(np.uint32) == z["accum_rows"].view(np.uint32), axis=-1)
    assert same.all(), f"{same.mean():.6%} of the committed rows' pixels bitwise equal"
    assert np.array_equal(rgba[z["rows"]], z["rgba_rows"])
    assert hashlib.sha256(np.ascontiguousarray(acc).tobytes()).hexdigest() == str(z["sha_accum"])
    assert hashlib.sha256(np.ascontiguousarray(rgba).tobytes()).hexdigest() == str(z["sha_rgba"])
