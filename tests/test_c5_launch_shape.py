"""C5 in the launch shape that produces its benchmark figure: the Cornell box + the
79,488-triangle bunny on the vertex kernel's BVH variant (rt_stats.kernel == 3) with the split scene's
camera pre-pass, rendering many frames in one rt_render -- and, when the parked-sample and camera-record
budget is smaller than the render, as several passes over consecutive frame ranges (rt_capi.cpp: the
pass split, each later pass's first_frame, the pre-pass records of every pass).  The reference
accumulates every frame into one float4 buffer (MC/Renderer.cpp:114-133) and traverses its two-level
BVH (MC/BVH.h:72-101); the GPU frame must hash to the reference's whatever the pass count.

Golden vectors: tests/golden/full_c5.npz (3840x2160x256, seed 0, RR 0.8, frames 1..256) from
oracle/_ref/ref_harness -- the reference's own MC/ BVH, triangle, material and camera code compiled from
/root/reference, the Philox words injected into its mt19937 and re-filled at the top of a shading call
for paths longer than one engine fill (oracle/ref/mt_inject.h) -- via `oracle/gen_golden.py full_c5`:
the SHA-256 of the float4 accumulation and of the RGBA8 frame, and every 64th accumulation row.
tests/golden/full_c5_4096.npz is the same at C5's full 4096 spp on every 64th row (`gen_golden.py full_c5_4096`:
the harness renders only those rows -- the whole frame would take ~11 h on 8 cores); its SHA-256 covers those
rows.  tests/golden/full_c5_4096_mid.npz, _o16.npz and _o48.npz (round 6) hold the rows 32, 96, ..., 16, 80, ... and
48, 112, ..., so the 4096-spp frame is pinned on every 16th row; _o8, _o24, _o40 and _o56 (late round 6) the rows
8, 24, 40 and 56 off, every 8th row with all of them; _o4, _o12, ..., _o60 the rows 4 off those, every 4th row.  The GPU renders the whole frame in the benchmark's launch shape (ten passes at
the default budget) and compares the rows of both."""
import hashlib
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

FIXTURES = [n for n in ("full_c5", "full_c5_4096") if os.path.exists(os.path.join(O.GOLDEN, f"{n}.npz"))]
EXTRA_4096 = ("full_c5_4096_mid", "full_c5_4096_o16", "full_c5_4096_o48", "full_c5_4096_o8", "full_c5_4096_o24", "full_c5_4096_o40",
              "full_c5_4096_o56") + tuple(f"full_c5_4096_o{o}" for o in range(4, 64, 8))
ROW_OFFSET = {"full_c5_4096_mid": 32, **{f"full_c5_4096_o{o}": o for o in range(4, 64, 4) if o != 32}}


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64 if a.dtype == np.float64 else a.dtype)


@pytest.fixture(scope="module")
def bunny_raw():
    return np.load(os.path.join(O.GOLDEN, "bvh_scene.npz"))["raw_bunny"]


@pytest.fixture(scope="module")
def scene(bunny_raw):
    return rt.Scene.cornell_c5(bunny_raw)


def test_fixture_present_and_shaped():
    assert "full_c5" in FIXTURES
    for name in FIXTURES + list(EXTRA_4096):
        if not os.path.exists(os.path.join(O.GOLDEN, f"{name}.npz")):
            continue
        z = np.load(os.path.join(O.GOLDEN, f"{name}.npz"))
        W, H, spp = int(z["W"]), int(z["H"]), int(z["spp"])
        assert (W, H, int(z["seed"]), int(z["first_frame"])) == (3840, 2160, 0, 1) and spp in (256, 4096)
        assert np.array_equal(z["rows"], np.arange(ROW_OFFSET.get(name, 0), H, 64))
        assert z["accum_rows"].shape == (len(z["rows"]), W, 3)
        assert np.all((z["rgba_rows"] >> 24) == 255)
        # samples; no harness overflow (every path read the injected stream, however long)
        assert int(z["stats"][4]) == W * H * spp and int(z["stats"][3]) == 0


def test_oracle_reproduces_a_full_c5_row(bunny_raw):
    """The restatement renders one committed row (through the bunny) at 256 spp bit for bit."""
    z = np.load(os.path.join(O.GOLDEN, "full_c5.npz"))
    W, H, spp = int(z["W"]), int(z["H"]), int(z["spp"])
    row = 640
    k = int(np.where(z["rows"] == row)[0][0])
    meshes = O.cornell_meshes() + [("c5", rt.c5_mesh(bunny_raw), np.array([0.7, 0.7, 0.7], np.float32), np.zeros(3, np.float32))]
    acc, rgba, _ = O.Scene(meshes).render(W, H, spp, seed=0, rr=0.8, threads=min(8, os.cpu_count() or 1), rows=(row, row + 1))
    assert np.array_equal(bits(acc[row, :, :3]), bits(z["accum_rows"][k]))
    assert np.array_equal(rgba[row], z["rgba_rows"][k])


def _context(monkeypatch, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    return rt.Context(0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("budget_mb,min_passes", [(None, 1), (16000, 4)], ids=["default-budget", "forced-passes"])
def test_c5_frame_in_launch_shape(scene, monkeypatch, name, budget_mb, min_passes):
    """One rt_render of every frame, as bench_configs.py times C5: with the default budget (256 spp: one pass;
    4096 spp: ten), and with a budget that forces at least four passes (each pass its own pre-pass over its
    frame range, first_frame continuing the accumulation)."""
    z = np.load(os.path.join(O.GOLDEN, f"{name}.npz"))
    W, H, spp = int(z["W"]), int(z["H"]), int(z["spp"])
    env = {} if budget_mb is None else {"RT_LBUF_BUDGET_MB": budget_mb}
    c = _context(monkeypatch, **env)
    try:
        c.upload(scene)
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, first_frame=1, seed=0, rr=0.8)
        st = c.stats()
        print(f"{name} budget {budget_mb}: kernel {st.kernel} passes {st.n_passes} pre-pass {st.last_prepass_ms:.1f} ms "
              f"path {st.last_main_ms:.1f} ms resampled {st.resampled}")
        assert st.kernel == 3 and st.overflow_lost == 0 and st.kernel_reason == rt.KERNEL_REASON_DEFAULT
        assert st.n_passes >= min_passes
        if budget_mb is None and spp == 256:
            assert st.n_passes == 1
        assert st.last_prepass_ms > 0.0   # the split scene's camera pre-pass ran (in every pass)
    finally:
        c.close()
    zs = [z]
    if name == "full_c5_4096":
        # the same frame's rows 32, 96, ..., 16, 80, ... / 48, 112, ... and 8 / 24 / 40 / 56 and 4 / 12 / ... / 60 off (round 6): every 4th row
        zs += [np.load(os.path.join(O.GOLDEN, f"{x}.npz")) for x in EXTRA_4096 if os.path.exists(os.path.join(O.GOLDEN, f"{x}.npz"))]
    for z in zs:
        rows = acc[z["rows"], :, :3]
        same = np.all(bits(rows) == bits(z["accum_rows"]), axis=-1)
        assert same.all(), f"{same.mean():.6%} of the committed rows' pixels bitwise equal"
        assert np.array_equal(rgba[z["rows"]], z["rgba_rows"])
        rows_only = bool(z["rows_only"]) if "rows_only" in z.files else False
        sel_acc = np.ascontiguousarray(acc[z["rows"]] if rows_only else acc)
        sel_rgba = np.ascontiguousarray(rgba[z["rows"]] if rows_only else rgba)
        assert hashlib.sha256(sel_acc.tobytes()).hexdigest() == str(z["sha_accum"])
        assert hashlib.sha256(sel_rgba.tobytes()).hexdigest() == str(z["sha_rgba"])


@pytest.mark.gpu
def test_bvh_variant_ring_overflow_across_passes(scene, bunny_raw, monkeypatch):
    """Kernel 3 at RR 0.9 (a reference UI setting, MC/mainloop.cpp:96-100) with a 4-level fold ring and a
    parked-sample budget that splits the render into several passes: every pass lists the samples whose path
    outgrew the ring and resample_kernel renders them again into their parked slots.  Bitwise vs the oracle."""
    W, H, spp, seed, rr = 96, 54, 48, 2, 0.9
    c = _context(monkeypatch, RT_STACK_DEPTH=4, RT_LBUF_BUDGET_MB=2)
    try:
        c.upload(scene)
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        rgba, acc = c.render(cam, spp, seed=seed, rr=rr)
        st = c.stats()
        print(f"passes {st.n_passes} resampled {st.resampled} of {W * H * spp}")
        assert st.kernel == 3 and st.stack_depth == 4
        assert st.n_passes >= 3 and st.resampled > 100 and st.overflow_lost == 0
        assert st.last_prepass_ms > 0.0
    finally:
        c.close()
    meshes = O.cornell_meshes() + [("c5", rt.c5_mesh(bunny_raw), np.array([0.7, 0.7, 0.7], np.float32), np.zeros(3, np.float32))]
    oacc, orgba, _ = O.Scene(meshes).render(W, H, spp, seed=seed, rr=rr, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(bits(acc), bits(oacc))
    assert np.array_equal(rgba, orgba)
