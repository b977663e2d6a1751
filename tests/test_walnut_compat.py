"""The Walnut drop-in (include/rt/walnut/Camera.h, Renderer.h): the reference's own layer, MC/mainloop.cpp,
builds against it with no edit but its two include lines (here: an include path that maps "Camera.h" /
"Renderer.h" to the drop-in), and runs.

CPU: the layer file compiles UNCHANGED from /root/reference against the drop-in and test-only Walnut / ImGui
/ glm stubs (tests/walnut_stub/), and links with librt_hip.so (tests/_walnut_build.py).
GPU: the driver clicks the layer's buttons (Render Offline, RR 50 %, Render in Real-Time) and holds W with the
right mouse button for one update; every frame the layer displays (Walnut::Image::SetData of
GetFinalImage(), MC/Renderer.cpp:112 and MC/mainloop.cpp:55-58) must equal the same render through the
C-ABI bit for bit -- the seeds follow the drop-in Renderer's epochs (Reaccumulate starts a fresh stream),
the roulette value the button set, and the moved camera UpdateCamera's WASD step (MC/Camera.cpp:49-53)."""
import os
import subprocess

import numpy as np
import pytest

import _walnut_build as WB
from _rt import rt

W, H = 64, 48


@pytest.mark.skipif(not os.path.exists(WB.MAINLOOP), reason="needs /root/reference (the reference's layer file)")
def test_reference_layer_compiles_against_the_dropin(tmp_path):
    out = WB.build(str(tmp_path / "walnut_mainloop"))
    assert out is not None and os.path.exists(out)


def read(path):
    raw = np.fromfile(path, np.uint32)
    w, h = int(raw[0]), int(raw[1])
    return raw[2:].reshape(h, w)


def render(cam, frames, seed, rr):
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        rgba, _ = c.render(cam, frames, seed=seed, rr=rr)
        return rgba
    finally:
        c.close()


@pytest.mark.gpu
def test_reference_layer_runs_on_the_dropin(tmp_path):
    if not os.path.exists(WB.BIN):
        pytest.skip("tests/_bin/walnut_mainloop not built (build() builds it where /root/reference exists)")
    assert not WB.headers_changed(WB.BIN), "tests/_bin/walnut_mainloop predates the drop-in headers: rerun build()"
    prefix = str(tmp_path / "frame")
    r = subprocess.run([WB.BIN, prefix], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    cam, _, _ = rt.camera_default(W, H)
    # Render Offline: Reaccumulate (epoch 1) + 1 spp at RR 0.8
    assert np.array_equal(read(prefix + "_0.bin"), render(cam, 1, seed=1, rr=0.8))
    # RR 50 % (Reaccumulate, epoch 2) then Render Offline (epoch 3): 1 spp at RR 0.5
    f1 = read(prefix + "_1.bin")
    assert np.array_equal(f1, render(cam, 1, seed=3, rr=0.5))
    # Render in Real-Time: one more accumulated spp
    assert np.array_equal(read(prefix + "_2.bin"), render(cam, 2, seed=3, rr=0.5))
    # W held with the right button for dt = 0.05: position += (5 * dt) * forward (MC/Camera.cpp:49-53), the
    # camera moved so the layer Reaccumulates (epoch 4); two real-time frames
    s = np.float32(5.0) * np.float32(0.05)
    fwd = np.array(rt.DEFAULT_CAMERA_FORWARD, np.float32)
    pos = np.array(rt.DEFAULT_CAMERA_POSITION, np.float32) + s * fwd
    moved = rt.camera_look(W, H, tuple(float(v) for v in pos), tuple(float(v) for v in fwd))
    f3 = read(prefix + "_3.bin")
    assert np.array_equal(f3, render(moved, 2, seed=4, rr=0.5))
    assert not np.array_equal(f3, render(cam, 2, seed=4, rr=0.5))
    assert "1 spp" in r.stdout.splitlines()   # the layer's own spp counter (GetSPP)


# ------------------------------------------------------------------ the scene-extension spelling (C5)
def test_scene_extension_compiles_against_the_dropin(tmp_path):
    """tests/walnut_stub/c5_scene.cpp extends the scene the reference's way -- Whitted::WhittedMaterial,
    `renderer.Add(new Whitted::TriangleMesh(path, white))`, `GenerateBVH()` (MC/Renderer.h:78-86,
    MC/TriangleMesh.h:148-186, MC/WhittedMaterial.h:24-42) -- and compiles against include/rt/walnut/*.h."""
    out = WB.build_c5(str(tmp_path / "walnut_c5_scene"))
    assert os.path.exists(out)


@pytest.mark.gpu
def test_scene_extension_builds_c5(tmp_path):
    """C5 built through the drop-in's Whitted:: types: the flattened tree is the reference's
    (the SHA-256 digest of tests/golden/c5_scene.npz, from the reference's own TriangleMesh + BVH code) and 16
    frames through Renderer::Render give the reference's 96x54x16 accumulation bit for bit."""
    import importlib.util
    import _oracle as O
    if not os.path.exists(WB.C5_BIN):
        pytest.skip("tests/_bin/walnut_c5_scene not built (build() builds it)")
    assert not WB.headers_changed(WB.C5_BIN), "tests/_bin/walnut_c5_scene predates the drop-in headers: rerun build()"
    fx = np.load(os.path.join(O.GOLDEN, "c5_scene.npz"))
    bunny = np.load(os.path.join(O.GOLDEN, "bvh_scene.npz"))["raw_bunny"]
    obj = str(tmp_path / "c5_bunny.obj")
    rt.write_obj(obj, rt.c5_mesh(bunny))
    prefix = str(tmp_path / "c5")
    r = subprocess.run([WB.C5_BIN, obj, prefix], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "entities 7" in r.stdout and "16 spp" in r.stdout, r.stdout
    raw = np.fromfile(prefix + "_scene.bin", np.uint8)
    nn, nt = raw[:8].view(np.uint32)
    off = 8
    def take(dt, n):
        nonlocal off
        v = raw[off:off + 4 * n].view(dt)
        off += 4 * n
        return v
    nf = take(np.float32, 7 * nn).reshape(nn, 7); ni = take(np.int32, 5 * nn).reshape(nn, 5)
    tf = take(np.float32, 13 * nt).reshape(nt, 13); ti = take(np.int32, 2 * nt).reshape(nt, 2)
    spec = importlib.util.spec_from_file_location("gg", os.path.join(O.ORACLE_DIR, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    nodes = np.zeros(nn, gg.NODE_DT)
    nodes["mn"], nodes["mx"], nodes["area"] = nf[:, 0:3], nf[:, 3:6], nf[:, 6]
    for k, col in (("left", 0), ("right", 1), ("tri", 2), ("mesh", 3), ("top", 4)):
        nodes[k] = ni[:, col]
    tris = np.zeros(nt, gg.TRI_DT)
    for k, sl in (("a", slice(0, 3)), ("b", slice(3, 6)), ("c", slice(6, 9)), ("n", slice(9, 12))):
        tris[k] = tf[:, sl]
    tris["mesh"] = ti[:, 0]
    assert nn == int(fx["n_nodes"]) and nt == int(fx["n_tris"])
    assert gg.scene_digest(nodes, tris) == str(fx["digest"])
    acc = np.fromfile(prefix + "_accum.bin", np.float32).reshape(54, 96, 4)
    assert np.array_equal(acc.view(np.uint32), fx["accum_96x54_spp16_s0"].view(np.uint32))
