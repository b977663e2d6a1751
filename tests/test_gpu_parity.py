"""GPU parity: the HIP megakernel (through the C-ABI) against the reference's golden vectors and the
oracle.  Tolerance (north star): per-pixel RMSE < 1e-4 of clamp(accum/spp, 0, 1) at matched spp;
the EXACT mode is held to more than that: its float4 accumulation must be bitwise identical to the
reference's.  FAST mode is held to the RMSE tolerance."""
import os

import numpy as np
import pytest

import _oracle as O
from _rt import rt

pytestmark = pytest.mark.gpu
G = O.GOLDEN
RMSE_TOL = 1e-4


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64 if a.dtype == np.float64 else a.dtype)


def rmse(acc, ref, spp):
    a = np.clip(acc[..., :3] / np.float32(spp), 0, 1).astype(np.float64)
    b = np.clip(ref[..., :3] / np.float32(spp), 0, 1).astype(np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.fixture(scope="module")
def ctx():
    c = rt.Context(0)
    c.upload(rt.Scene.cornell())
    yield c
    c.close()


def render(ctx, W, H, spp, seed=0, rr=0.8, exact=True, band=8, rank=0, nranks=1, first_frame=1):
    ctx.resize(W, H, band, rank, nranks)
    cam, _, _ = rt.camera_default(W, H)
    return ctx.render(cam, spp, first_frame=first_frame, seed=seed, rr=rr, exact=exact)


def test_device_arithmetic_is_ieee(ctx):
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(0, 7, 200000), rng.uniform(1e-6, 1e6, 200000), [0.5, 1.0, 2.0, 6.2831855]]).astype(np.float32)
    out = ctx.math_selftest(x)
    assert np.array_equal(bits(out[:, 0]), bits(np.sqrt(x)))                        # correctly rounded sqrtf
    assert np.array_equal(bits(out[:, 1]), bits(np.float32(1.0) / x))                # correctly rounded f32 division
    r = out[:, 4:6].copy().view(np.float64).ravel()
    assert np.array_equal(bits(r), bits(1.0 / x.astype(np.float64)))                 # f64 reciprocal
    # hemisphere angle phi = 2*PI*U in [0, 2*PI]: cos/sin equal glibc's cosf/sinf bit for bit
    phi = x[x <= np.float32(6.2831855)]
    c, s = O.libm_trig(phi)
    sel = x <= np.float32(6.2831855)
    assert np.array_equal(bits(out[sel, 2]), bits(c))
    assert np.array_equal(bits(out[sel, 3]), bits(s))


def test_device_trig_equals_glibc_on_0_2pi(ctx):
    # a strided sweep over every float bit pattern in [0, 2*PI] (phi = 2*PI*U, MC/WhittedMaterial.h:80)
    top = np.uint32(np.float32(6.2831855).view(np.uint32))
    for start in (0, 31, 62):
        b = np.arange(start, int(top) + 1, 97, dtype=np.uint32)
        x = b.view(np.float32)
        out = ctx.math_selftest(x)
        c, s = O.libm_trig(x)
        assert np.array_equal(bits(out[:, 2]), bits(c)) and np.array_equal(bits(out[:, 3]), bits(s))


def test_closest_hit_matches_reference(ctx):
    z = np.load(os.path.join(G, "rays_cornell.npz"))
    tri, t = ctx.trace(z["org"], z["dir"])
    assert np.array_equal(tri, z["tri"])
    hit = z["hit"] == 1
    assert np.array_equal(bits(t[hit]), bits(z["t"][hit]))


@pytest.mark.parametrize("key", ["64x64_spp1_s0_rr0.8", "64x64_spp16_s0_rr0.8", "64x64_spp256_s0_rr0.8",
                                 "128x128_spp16_s7_rr0.8", "40x30_spp8_s123_rr0.5", "33x17_spp4_s5_rr0.9"])
def test_image_matches_reference_golden(ctx, key):
    z = np.load(os.path.join(G, "images_cornell.npz"))
    wh, spp, s, rr = key.split("_")
    W, H = map(int, wh.split("x"))
    spp = int(spp[3:])
    rgba, acc = render(ctx, W, H, spp, seed=int(s[1:]), rr=float(rr[2:]))
    g_acc, g_rgba = z[f"accum_{key}"], z[f"rgba_{key}"]
    e = rmse(acc, g_acc, spp)
    same = np.mean(np.all(bits(acc) == bits(g_acc), axis=-1))
    d8 = np.abs(rgba.view(np.uint8).astype(int) - g_rgba.view(np.uint8).astype(int)).max()
    print(f"{key}: rmse {e:.3e} bitwise-identical pixels {same:.4%} max |d8| {d8}")
    assert e < RMSE_TOL
    assert same == 1.0   # bit-identical accumulation


def test_fast_mode_within_tolerance(ctx):
    _, a = render(ctx, 64, 64, 64, exact=True)
    _, b = render(ctx, 64, 64, 64, exact=False)
    assert rmse(a, b, 64) < 1e-5


def test_incremental_frames_equal_batched(ctx):
    _, a = render(ctx, 48, 40, 5, seed=11)
    ctx.resize(48, 40)
    cam, _, _ = rt.camera_default(48, 40)
    for f in range(1, 6):
        rgba, acc = ctx.render(cam, 1, first_frame=f, seed=11)
    assert np.array_equal(bits(acc), bits(a))


def test_row_band_split_reassembles_bitwise(ctx):
    W, H, spp = 70, 45, 4
    rgba1, acc1 = render(ctx, W, H, spp, seed=3)
    full = np.zeros_like(acc1)
    for r in range(3):
        rgba, acc = render(ctx, W, H, spp, seed=3, band=8, rank=r, nranks=3)
        rows = ctx.local_to_global_rows()
        full[rows] = acc
    assert np.array_equal(bits(full), bits(acc1))


def test_row_band_split_reassembles_bitwise_bvh_variant():
    """The same split on the C5 scene (the vertex kernel's BVH variant), frame chunks included."""
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell_c5(np.load(os.path.join(os.path.dirname(__file__), "golden", "bvh_scene.npz"))["raw_bunny"]))
        W, H, spp = 64, 40, 12
        rgba1, acc1 = render(c, W, H, spp, seed=9)
        assert c.stats().kernel == 3
        full = np.zeros_like(acc1)
        for r in range(3):
            rgba, acc = render(c, W, H, spp, seed=9, band=8, rank=r, nranks=3)
            full[c.local_to_global_rows()] = acc
        assert np.array_equal(bits(full), bits(acc1))
    finally:
        c.close()


def test_matches_oracle_at_larger_size(ctx):
    W, H, spp = 192, 160, 32
    rgba, acc = render(ctx, W, H, spp, seed=5)
    sc = O.Scene()
    oacc, orgba, _ = sc.render(W, H, spp, seed=5)
    e = rmse(acc, oacc, spp)
    same = np.mean(np.all(bits(acc) == bits(oacc), axis=-1))
    print(f"oracle {W}x{H}x{spp}: rmse {e:.3e} identical {same:.4%}")
    assert e < RMSE_TOL and same == 1.0


@pytest.mark.parametrize("rr", [0.5, 0.8, 0.9])
def test_roulette_settings_match_oracle(ctx, rr):
    """The reference UI's three Russian-roulette survival probabilities (MC/mainloop.cpp:96-110) on a
    256x192x32 frame against the CPU restatement: bitwise accumulation and RGBA8 (at 0.9 paths average
    ten vertices, so the fold ring and its drain run deep)."""
    W, H, spp = 256, 192, 32
    rgba, acc = render(ctx, W, H, spp, seed=3, rr=rr)
    oacc, orgba, _ = O.Scene().render(W, H, spp, seed=3, rr=rr, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(bits(acc), bits(oacc))
    assert np.array_equal(rgba, orgba)


def test_counters_and_no_stack_overflow(ctx):
    ctx.resize(64, 64)
    cam, _, _ = rt.camera_default(64, 64)
    ctx.render(cam, 16, exact=True, count=True, fetch=False)
    st = ctx.stats()
    assert st.samples == 64 * 64 * 16 and st.stack_overflows == 0
    assert 4.0 < st.rays / st.samples < 7.5
    assert st.node_tests > st.rays and st.tri_tests > 0 and st.last_kernel_ms > 0


def test_exact_modes_agree_bitwise(ctx):
    # scene in LDS or HBM, fold stack in LDS or HBM: the same IEEE operations, the same bits
    W, H, spp = 96, 80, 24
    ctx.resize(W, H)
    cam, _, _ = rt.camera_default(W, H)
    ref = None
    for kw in (dict(), dict(global_scene=True), dict(global_stack=True), dict(global_scene=True, global_stack=True)):
        rgba, acc = ctx.render(cam, spp, seed=9, **kw)
        if ref is None:
            ref = acc
        assert np.array_equal(bits(acc), bits(ref)), kw


def test_frame_chunks_are_bitwise_neutral(monkeypatch):
    """Splitting a pixel's frames into work items (the megakernel: chunk 0 accumulates, later chunks park
    their samples for the in-order finalize pass) leaves the accumulation bit-identical, from frame 1 and
    from a later first frame."""
    W, H, spp = 40, 24, 37
    out = {}
    monkeypatch.setenv("RT_VERTEX", "0")
    for chunks in ("1", "5", "37"):
        monkeypatch.setenv("RT_CHUNKS", chunks)
        c = rt.Context(0)
        try:
            c.upload(rt.Scene.cornell())
            c.resize(W, H)
            cam, _, _ = rt.camera_default(W, H)
            _, a = c.render(cam, 20, seed=3)
            _, b = c.render(cam, spp - 20, first_frame=21, seed=3)
            assert c.stats().n_chunks == min(int(chunks), spp - 20)
            assert c.stats().kernel == 0   # the megakernel
            out[chunks] = (a, b)
        finally:
            c.close()
    for k in ("5", "37"):
        assert np.array_equal(bits(out[k][0]), bits(out["1"][0]))
        assert np.array_equal(bits(out[k][1]), bits(out["1"][1]))
    monkeypatch.delenv("RT_VERTEX")
    monkeypatch.delenv("RT_CHUNKS")
    # the vertex kernel: its camera pre-pass groups a tile's frames in segments of up to 64 frames (70
    # frames: 2 segments per tile, the last of 6), and the path kernel takes each segment in up to 4 parts
    # (16 frames' worth) when a pass has few tiles (here 8).  RT_SEG_PARTS_OFF=1 shortens the segments instead
    # (16 frames: 5 segments per tile, the last of 6, one part each); both give the megakernel's bits
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        _, v = c.render(cam, 70, seed=3)
        assert c.stats().kernel == 1 and c.stats().n_chunks == 2
    finally:
        c.close()
    monkeypatch.setenv("RT_SEG_PARTS_OFF", "1")
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        _, v8 = c.render(cam, 70, seed=3)
        assert c.stats().kernel == 1 and c.stats().n_chunks == 5
    finally:
        c.close()
    monkeypatch.delenv("RT_SEG_PARTS_OFF")
    assert np.array_equal(bits(v8), bits(v))
    # parts as fine as one frame's worth of records (RT_SEG_PART_LF=0; 64 parts per segment) and as many
    # as the split allows (RT_SEG_MIN_PARTS): the same bits
    monkeypatch.setenv("RT_SEG_MIN_PARTS", "100000")
    monkeypatch.setenv("RT_SEG_PART_LF", "0")
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        _, v1 = c.render(cam, 70, seed=3)
        assert c.stats().kernel == 1 and c.stats().n_chunks == 2
    finally:
        c.close()
    monkeypatch.delenv("RT_SEG_MIN_PARTS")
    monkeypatch.delenv("RT_SEG_PART_LF")
    assert np.array_equal(bits(v1), bits(v))
    # one work queue and no finer tail (the default: 8 per-XCD queues, most of them dry at once on this small
    # frame, and the list's last parts split 8x): the same bits
    monkeypatch.setenv("RT_WORK_QUEUES", "1")
    monkeypatch.setenv("RT_SEG_TAIL_EXTRA", "0")
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        _, vq = c.render(cam, 70, seed=3)
    finally:
        c.close()
    monkeypatch.delenv("RT_WORK_QUEUES")
    monkeypatch.delenv("RT_SEG_TAIL_EXTRA")
    assert np.array_equal(bits(vq), bits(v))
    monkeypatch.setenv("RT_VERTEX", "0")
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        _, m = c.render(cam, 70, seed=3)
    finally:
        c.close()
    monkeypatch.delenv("RT_VERTEX")
    assert np.array_equal(bits(v), bits(m))
    # a parked-sample budget below one launch's needs splits the render into passes over frame ranges
    monkeypatch.setenv("RT_LBUF_BUDGET_MB", "1")
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(96, 64)
        cam, _, _ = rt.camera_default(96, 64)
        _, a = c.render(cam, 100, seed=3)
        st = c.stats()
        assert st.n_passes > 1
    finally:
        c.close()
    monkeypatch.delenv("RT_LBUF_BUDGET_MB")
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(96, 64)
        _, b = c.render(cam, 100, seed=3)
        assert c.stats().n_passes == 1
    finally:
        c.close()
    assert np.array_equal(bits(a), bits(b))


@pytest.mark.parametrize("W,H,first,n", [(784, 784, 1, 4),        # C2 at full size
                                         (1920, 1080, 1, 2),      # C4 at full size
                                         (1920, 1080, 1021, 4)])  # C4's last frames (RNG counter, divisor)
def test_full_size_matches_oracle(ctx, W, H, first, n):
    """SURVEY.md §8(d) parity gate (ii): the configuration's full resolution against the CPU restatement,
    at a few frames (the oracle runs multithreaded on the host).  Bitwise accumulation and RGBA8."""
    ctx.resize(W, H)
    ctx.reset_accumulation()
    cam, _, _ = rt.camera_default(W, H)
    rgba, acc = ctx.render(cam, n, first_frame=first, seed=0)
    oacc, orgba, _ = O.Scene().render(W, H, n, seed=0, first_frame=first, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(bits(acc), bits(oacc))
    assert np.array_equal(rgba, orgba)


def test_coherent_trace_equals_bvh_traversal(monkeypatch):
    """Small scenes trace every ray through their distinct leaf boxes; RT_BRUTE=0 walks the BVH instead.
    Same bits either way: a jittered frame, and a pixel-centre G-buffer frame whose centre ray is
    exactly +z (a non-finite reciprocal direction, which sends its wave through the BVH rounds)."""
    out = {}
    for brute in ("1", "0"):
        monkeypatch.setenv("RT_BRUTE", brute)
        c = rt.Context(0)
        try:
            c.upload(rt.Scene.cornell())
            c.resize(96, 64)
            cam, _, _ = rt.camera_default(96, 64)
            _, a = c.render(cam, 16, seed=9)
            c.resize(65, 65)
            cam, proj, view = rt.camera_look_ex(65, 65, (2.78, 2.73, -8.0), (0.0, 0.0, 1.0))
            _, g = c.render_denoised(cam, proj, view, 1, rt.denoise_params(), seed=9)
            gb = c.gbuffer()
            out[brute] = (a, g, gb["color"], gb["position"], gb["normal"], gb["prim"])
        finally:
            c.close()
    for x, y in zip(out["1"], out["0"]):
        assert np.array_equal(bits(x), bits(y))


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [True, False])
def test_vertex_kernel_equals_megakernel(monkeypatch, exact):
    """Small scenes render with the vertex-synchronous kernel (rt_coherent.hip); RT_VERTEX=0 runs the
    general megakernel, RT_FORCE_WALK=1 sends every ray of the vertex kernel through its per-lane BVH
    walk (the path of rays with a non-finite reciprocal direction).  Same bits in EXACT and FAST mode,
    with and without frame chunks, with the fold levels' materials in the direct term's sign bits (the
    default) or in their own array (RT_RING_PACK=0)."""
    out = {}
    for name, env in (("vertex", {}), ("mega", {"RT_VERTEX": "0"}), ("walk", {"RT_FORCE_WALK": "1"}),
                      ("vertex_chunks", {"RT_CHUNKS": "3"}), ("ring_mat_array", {"RT_RING_PACK": "0"})):
        for k in ("RT_VERTEX", "RT_FORCE_WALK", "RT_CHUNKS", "RT_RING_PACK"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        c = rt.Context(0)
        try:
            c.upload(rt.Scene.cornell())
            c.resize(80, 56)
            cam, _, _ = rt.camera_default(80, 56)
            rgba, a = c.render(cam, 24, seed=5, exact=exact)
            out[name] = (rgba, a)
        finally:
            c.close()
    for name in ("mega", "walk", "vertex_chunks", "ring_mat_array"):
        assert np.array_equal(out[name][0], out["vertex"][0]), name
        assert np.array_equal(bits(out[name][1]), bits(out["vertex"][1])), name


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["cornell_bvh", "c5"])
@pytest.mark.parametrize("exact", [True, False])
def test_vertex_bvh_kernel_equals_megakernel(monkeypatch, scene, exact):
    """Scenes without decisive leaf boxes render with the vertex kernel's BVH variant (the scene in HBM,
    two rays per lane walking the stackless BVH): the Cornell box with RT_BRUTE=0 and the C5 scene
    (Cornell + 79k-triangle mesh).  RT_VERTEX_BVH=0 runs the megakernel; same bits, with and without
    frame chunks."""
    out = {}
    for name, env in (("vertex", {}), ("mega", {"RT_VERTEX_BVH": "0"}), ("vertex_chunks", {"RT_CHUNKS": "3"})):
        for k in ("RT_VERTEX", "RT_VERTEX_BVH", "RT_BRUTE", "RT_CHUNKS"):
            monkeypatch.delenv(k, raising=False)
        if scene == "cornell_bvh":
            monkeypatch.setenv("RT_BRUTE", "0")
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        c = rt.Context(0)
        try:
            if scene == "c5":
                c.upload(rt.Scene.cornell_c5(np.load(os.path.join(os.path.dirname(__file__), "golden", "bvh_scene.npz"))["raw_bunny"]))
            else:
                c.upload(rt.Scene.cornell())
            c.resize(72, 48)
            cam, _, _ = rt.camera_default(72, 48)
            rgba, a = c.render(cam, 16, seed=7, exact=exact)
            out[name] = (rgba, a, c.stats().kernel)
        finally:
            c.close()
    assert out["vertex"][2] == 3 and out["mega"][2] == 0
    for name in ("mega", "vertex_chunks"):
        assert np.array_equal(out[name][0], out["vertex"][0]), name
        assert np.array_equal(bits(out[name][1]), bits(out["vertex"][1])), name


@pytest.mark.gpu
@pytest.mark.parametrize("view", [((2.78, 2.73, -8.0), (0.0, 0.0, 1.0), 35.0),      # the usual view, centred
                                  ((2.78, 1.0, 2.8), (0.0, 1.0, 0.0), 90.0),       # inside the box, up at the light
                                  ((0.3, 0.3, 0.3), (0.6, 0.35, 0.7), 110.0),      # a corner, very wide
                                  ((4.2, 0.8, 4.0), (-0.3, 0.05, -0.9), 20.0),     # inside the tall block's box, narrow
                                  ((2.78, 9.0, 2.8), (0.0, -1.0, 0.001), 60.0)])   # above the ceiling, looking down
def test_prepass_tile_cull_views(view):
    """The camera pre-pass tests only the leaf boxes its tile's frustum meets (rt_coherent.hip
    tile_box_mask): over cameras inside and outside the box, wide and narrow, looking along an axis, the
    vertex kernel's image equals the megakernel's (which tests every box for every ray) bit for bit."""
    pos, fwd, fov = view
    W, H, spp = 200, 120, 6
    cam = rt.camera_look(W, H, pos, fwd, vfov=fov)
    out = []
    for vertex in ("1", "0"):
        os.environ["RT_VERTEX"] = vertex
        try:
            c = rt.Context(0)
            try:
                c.upload(rt.Scene.cornell())
                c.resize(W, H)
                _, acc = c.render(cam, spp, seed=7)
                out.append((acc, c.stats().kernel))
            finally:
                c.close()
        finally:
            os.environ.pop("RT_VERTEX", None)
    assert out[0][1] == 1 and out[1][1] == 0
    assert np.array_equal(bits(out[0][0]), bits(out[1][0]))
