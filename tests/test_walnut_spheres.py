"""The reference's Entity extension point through the C++ drop-in: Whitted::Entity with the
virtual interface of MC/Entity.h:19-55, Whitted::Sphere (MC/Sphere.h:16-108) accepted by Renderer::Add +
GenerateBVH and rendered on the GPU, and the Renderer's public `bvh` / `entities` members (MC/Renderer.h:200-201).
tests/walnut_stub/spheres.cpp compiles against include/rt/walnut/*.h and uses them the reference's way.

Fixture: tests/golden/cornell_spheres.npz, from the reference's own Sphere / BVH / TriangleMesh code
(oracle/gen_golden.py spheres; see tests/test_spheres.py).
CPU: the entities on their own -- GetArea, Get3DAABB, IsEmissive of each sphere against the reference's entity
table, and Sphere::GetIntersectionRecord (host) against the reference's closest hits on that sphere, bitwise.
GPU: renderer.bvh->traverse_BVH_from_root over the fixture's rays (hit, entity, double t, location, normal) and
the 128x128x64 image through Renderer::Render, bitwise."""
import os
import subprocess

import numpy as np
import pytest

import _oracle as O
import _walnut_build as WB

FX = os.path.join(O.GOLDEN, "cornell_spheres.npz")
REC_DT = np.dtype([("hit", "<i4"), ("entity", "<i4"), ("t", "<f8"), ("loc", "<f4", 3), ("n", "<f4", 3)])


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


@pytest.fixture(scope="module")
def fx():
    return np.load(FX)


def _gg():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gg", os.path.join(O.ORACLE_DIR, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    return gg


def _inputs(tmp_path, fx):
    sp = np.concatenate([fx["spheres_center"], fx["spheres_radius"][:, None], fx["spheres_material"][:, None].astype(np.float32)], 1)
    sp.astype("<f4").tofile(tmp_path / "spheres.in")
    np.concatenate([fx["org"], fx["dir"]], 1).astype("<f4").tofile(tmp_path / "rays.in")
    return str(tmp_path / "spheres.in"), str(tmp_path / "rays.in")


def _hit_entity(fx):
    gg = _gg()
    tris = fx["tris"].view(gg.TRI_DT)
    ent = np.full(len(fx["tri"]), -1, np.int32)
    hit = fx["hit"] == 1
    ent[hit] = tris["mesh"][fx["tri"][hit]]
    return ent


def test_entity_interface_of_spheres(tmp_path, fx):
    exe = WB.build_spheres(str(tmp_path / "walnut_spheres"))
    si, ri = _inputs(tmp_path, fx)
    r = subprocess.run([exe, "entities", si, ri, str(tmp_path / "out")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    ns, nr = len(fx["spheres_radius"]), len(fx["org"])
    raw = np.fromfile(tmp_path / "out", np.uint8)
    ent = raw[:ns * 44].view("<f4").reshape(ns, 11)
    recs = raw[ns * 44:].view(REC_DT).reshape(nr, ns)
    meshes = fx["meshes"].view(_gg().MESH_DT)[6:]   # the entities after the six Cornell meshes, in Add order
    assert np.array_equal(bits(ent[:, 0]), bits(meshes["total_area"]))    # 4 * PI * r^2 (MC/Sphere.h:22)
    assert np.array_equal(bits(ent[:, 1:4]), bits(meshes["mn"]))          # AABB_3D{c + r, c - r}
    assert np.array_equal(bits(ent[:, 4:7]), bits(meshes["mx"]))
    assert np.array_equal(ent[:, 7].astype(np.int32), meshes["emissive"])
    # Sphere::GetIntersectionRecord on its own: where the reference's closest hit is sphere k, sphere k's own
    # record is that hit, bit for bit
    he = _hit_entity(fx)
    n_checked = 0
    for k in range(ns):
        sel = he == 6 + k
        r_k = recs[sel, k]
        assert np.all(r_k["hit"] == 1)
        assert np.array_equal(bits(r_k["t"]), bits(fx["t"][sel]))
        assert np.array_equal(bits(r_k["loc"]), bits(fx["loc"][sel]))
        assert np.array_equal(bits(r_k["n"]), bits(fx["n"][sel]))
        n_checked += int(sel.sum())
    assert n_checked > 1000


@pytest.mark.gpu
def test_spheres_render_through_the_dropin(tmp_path, fx):
    if not os.path.exists(WB.SPHERES_BIN):
        pytest.skip("tests/_bin/walnut_spheres not built (build() builds it)")
    assert not WB.headers_changed(WB.SPHERES_BIN), "tests/_bin/walnut_spheres predates the drop-in headers: rerun build()"
    si, ri = _inputs(tmp_path, fx)
    out = str(tmp_path / "render")
    r = subprocess.run([WB.SPHERES_BIN, "render", si, ri, out, "128", "128", "64"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "entities 10" in r.stdout and "64 spp" in r.stdout, r.stdout
    rec = np.fromfile(out, REC_DT)
    hit = fx["hit"] == 1
    assert np.array_equal(rec["hit"] == 1, hit)
    assert np.array_equal(rec["entity"][hit], _hit_entity(fx)[hit])
    for k in ("t", "loc", "n"):
        assert np.array_equal(bits(rec[k][hit]), bits(fx[k][hit])), k
    acc = np.fromfile(out + ".accum", np.float32).reshape(128, 128, 4)
    assert np.array_equal(bits(acc), bits(fx["accum_128x128_spp64_s0_rr0.8"]))
