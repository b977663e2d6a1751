#!/usr/bin/env python3
"""oracle/gen_golden.py -- TEST INFRASTRUCTURE ONLY: regenerate tests/golden/*.npz.

Runs oracle/_ref/ref_harness (the reference's own BVH / triangle / material / camera / OBJ-loader
code compiled from /root/reference by `make -C oracle ref`) on seeded synthetic inputs and stores
inputs + outputs as small .npz fixtures.  Only data is stored: no reference source text.
Container-only (needs /root/reference); the GPU box uses the committed fixtures.

    python oracle/gen_golden.py            # all fixtures
    python oracle/gen_golden.py bvh        # only the BVH Ray Tracer (C3) fixtures
    python oracle/gen_golden.py dn         # only the Denoiser project fixtures
    python oracle/gen_golden.py c1         # only the C1 (Whitted two-sphere world) fixtures
    python oracle/gen_golden.py optics     # only the Renderer optics helpers (mirror / Snell / Fresnel)
    python oracle/gen_golden.py c5         # only the C5 (Cornell + 79,488-triangle bunny) fixtures
    python oracle/gen_golden.py spheres    # only the Cornell + Whitted::Sphere fixtures (cornell_spheres.npz)
    python oracle/gen_golden.py stat       # only the shipped-mt19937 statistical fixture
    python oracle/gen_golden.py full       # C2 and C4 at their full spp (full_c2 / full_c4: one of them)
    python oracle/gen_golden.py full_c5    # C5 (Cornell + 79k-triangle bunny) at 3840x2160x256 (~10 min)
    python oracle/gen_golden.py full_c5_4096  # C5 at its full 4096 spp, every 64th row (~10 min)
    python oracle/gen_golden.py full_c5_4096_mid  # the same frame's rows 32, 96, ... (round 6)
    python oracle/gen_golden.py full_c5_4096_o16  # ... rows 16, 80, ...; full_c5_4096_o48: rows 48, 112, ... (round 6)
    python oracle/gen_golden.py full_c5_4096_o8   # ... rows 8, 72, ...; _o24, _o40, _o56 likewise (round 6: every 8th row)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(REPO, "tests", "golden")
HARNESS = os.path.join(HERE, "_ref", "ref_harness")
REF = os.environ.get("RT_REFERENCE", "/root/reference")
CORNELL_DIR = os.path.join(REF, "Monte Carlo Path Tracer", "8599RayTracerGUI", "src", "cornellbox")
MESH_NAMES = ["floor", "shortbox", "tallbox", "left", "right", "light"]
# Renderer::Renderer materials, MC/Renderer.cpp:28-41 (red, green, white, light)
ALBEDO = np.array([[0.63, 0.065, 0.05], [0.1, 0.5, 0.1], [0.7, 0.7, 0.7], [0.7, 0.7, 0.7]], np.float32)
EMISSION = np.array([[0, 0, 0], [0, 0, 0], [0, 0, 0], [47.8, 38.6, 31.1]], np.float32)
MESH_MATERIAL = [2, 2, 2, 0, 1, 3]

NODE_DT = np.dtype([("mn", "<f4", 3), ("mx", "<f4", 3), ("area", "<f4"), ("left", "<i4"), ("right", "<i4"),
                    ("tri", "<i4"), ("mesh", "<i4"), ("top", "<i4")])
TRI_DT = np.dtype([("a", "<f4", 3), ("b", "<f4", 3), ("c", "<f4", 3), ("n", "<f4", 3), ("area", "<f4"),
                   ("mesh", "<i4"), ("material", "<i4")])
MESH_DT = np.dtype([("total_area", "<f4"), ("mn", "<f4", 3), ("mx", "<f4", 3), ("material", "<i4"), ("emissive", "<i4")])
HIT_DT = np.dtype([("hit", "<i4"), ("tri", "<i4"), ("mat", "<i4"), ("t", "<f8"), ("loc", "<f4", 3), ("n", "<f4", 3)])


def run(*args):
    r = subprocess.run([HARNESS] + [str(a) for a in args], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"harness {args[0]} failed: {r.returncode} {r.stderr}")
    print(" ", r.stdout.strip())


def tmp(name):
    return os.path.join(TMP, name)


def gen_scene():
    raw = {}
    for n in MESH_NAMES:
        run("objraw", os.path.join(CORNELL_DIR, n + ".obj"), tmp(n + ".raw"))
        raw[n] = np.fromfile(tmp(n + ".raw"), "<f4").reshape(-1, 9)
    run("scene", CORNELL_DIR, "", tmp("nodes"), tmp("tris"), tmp("meshes"))
    nodes = np.fromfile(tmp("nodes"), NODE_DT)
    tris = np.fromfile(tmp("tris"), TRI_DT)
    meshes = np.fromfile(tmp("meshes"), MESH_DT)
    out = {f"raw_{n}": raw[n] for n in MESH_NAMES}
    out.update(albedo=ALBEDO, emission=EMISSION, mesh_material=np.array(MESH_MATERIAL, np.int32),
               nodes=nodes.view(np.uint8), tris=tris.view(np.uint8), meshes=meshes.view(np.uint8))
    np.savez_compressed(os.path.join(GOLDEN, "cornell_scene.npz"), **out)
    return tris


def gen_rays(tris, rng):
    n = 4096
    cam = np.array([2.81432, 4.20749, -9.11751], np.float32)
    lo, hi = np.array([0, 0, 0], np.float32), np.array([5.56, 5.488, 5.592], np.float32)
    o, d = [], []
    # (a) camera rays towards random points of the box
    k = 1200
    tgt = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    o.append(np.repeat(cam[None], k, 0)); d.append(tgt - cam)
    # (b) random interior origins, random directions
    k = 1200
    o.append(rng.uniform(lo, hi, (k, 3)).astype(np.float32)); d.append(rng.normal(size=(k, 3)).astype(np.float32))
    # (c) axis-aligned / signed-zero directions (slab NaN / inf paths)
    k = 600
    oo = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    dd = np.zeros((k, 3), np.float32)
    ax = rng.integers(0, 3, k)
    dd[np.arange(k), ax] = rng.choice([-1.0, 1.0], k)
    negz = rng.random((k, 3)) < 0.5
    dd = np.where((dd == 0) & negz, np.float32(-0.0), dd)
    o.append(oo); d.append(dd)
    # (d) origins exactly on walls / light plane / box tops
    k = 500
    oo = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    which = rng.integers(0, 4, k)
    oo[which == 0, 1] = 0.0
    oo[which == 1, 1] = np.float32(5.487)
    oo[which == 2, 0] = 0.0
    oo[which == 3, 2] = np.float32(5.592)
    o.append(oo); d.append(rng.normal(size=(k, 3)).astype(np.float32))
    # (e) towards triangle vertices and edge midpoints (shared-edge / tie cases)
    k = n - sum(len(x) for x in o)
    ti = rng.integers(0, len(tris), k)
    w = rng.integers(0, 4, k)
    a, b, c = tris["a"][ti], tris["b"][ti], tris["c"][ti]
    tgt = np.where((w == 0)[:, None], a, np.where((w == 1)[:, None], b, np.where((w == 2)[:, None], 0.5 * (a + b), 0.5 * (b + c))))
    src = np.where((rng.random(k) < 0.5)[:, None], cam[None], rng.uniform(lo, hi, (k, 3)).astype(np.float32))
    o.append(src.astype(np.float32)); d.append((tgt - src).astype(np.float32))
    o = np.concatenate(o).astype(np.float32)
    d = np.concatenate(d).astype(np.float32)
    np.concatenate([o, d], 1).astype("<f4").tofile(tmp("rays.in"))
    run("rays", CORNELL_DIR, "", tmp("rays.in"), tmp("rays.out"))
    res = np.fromfile(tmp("rays.out"), HIT_DT)
    np.savez_compressed(os.path.join(GOLDEN, "rays_cornell.npz"), org=o, dir=d, hit=res["hit"], tri=res["tri"],
                        mat=res["mat"], t=res["t"], loc=res["loc"], n=res["n"])


def gen_mt(rng):
    cases = []
    k = 3000
    v = rng.normal(size=(k, 3, 3)).astype(np.float32)
    org = rng.normal(size=(k, 3)).astype(np.float32) * 3
    tgt = (v.mean(1) + rng.normal(size=(k, 3)) * 0.6).astype(np.float32)
    cases.append(np.concatenate([v.reshape(k, 9), org, tgt - org], 1))
    # degenerate triangles, parallel rays, rays through vertices/edges, zero direction
    k = 600
    v = rng.normal(size=(k, 3, 3)).astype(np.float32)
    v[:200, 2] = v[:200, 1]                       # zero area
    org = rng.normal(size=(k, 3)).astype(np.float32) * 3
    d = rng.normal(size=(k, 3)).astype(np.float32)
    e1 = v[:, 1] - v[:, 0]
    d[200:300] = e1[200:300]                       # parallel to an edge of the plane
    d[300:400] = (v[300:400, 0] - org[300:400])    # through vertex a
    d[400:500] = (0.5 * (v[400:500, 1] + v[400:500, 2]) - org[400:500])   # through edge midpoint
    d[500:550] = 0.0                               # zero direction
    d[550:600] = -(v[550:600].mean(1) - org[550:600])   # pointing away (t < 0)
    cases.append(np.concatenate([v.reshape(k, 9), org, d], 1))
    # axis-aligned Cornell-like quads, rays from the camera
    k = 400
    cam = np.array([2.81432, 4.20749, -9.11751], np.float32)
    a = np.zeros((k, 3), np.float32); b = np.zeros((k, 3), np.float32); c = np.zeros((k, 3), np.float32)
    a[:, 0] = rng.uniform(0, 2, k); b[:, 0] = a[:, 0] + 3; c[:, 0] = a[:, 0]
    a[:, 2] = rng.uniform(0, 2, k); b[:, 2] = a[:, 2]; c[:, 2] = a[:, 2] + 3
    tgt = (a + b + c) / 3 + rng.normal(size=(k, 3)).astype(np.float32) * 0.8
    tgt[:, 1] = 0
    cases.append(np.concatenate([a, b, c, np.repeat(cam[None], k, 0), tgt - cam], 1))
    cases = np.concatenate(cases).astype("<f4")
    cases.tofile(tmp("mt.in"))
    run("mt", tmp("mt.in"), tmp("mt.out"))
    res = np.fromfile(tmp("mt.out"), np.dtype([("hit", "<i4"), ("t", "<f8")]))
    np.savez_compressed(os.path.join(GOLDEN, "mt_cases.npz"), cases=cases, hit=res["hit"], t=res["t"])


def gen_aabb(rng):
    k = 4000
    mn = rng.normal(size=(k, 3)).astype(np.float32)
    ext = np.abs(rng.normal(size=(k, 3))).astype(np.float32)
    ext[:500, rng.integers(0, 3)] = 0.0            # flat boxes (axis-aligned walls)
    mx = mn + ext
    o = (rng.normal(size=(k, 3)) * 3).astype(np.float32)
    d = rng.normal(size=(k, 3)).astype(np.float32)
    # signed zero and axis-aligned directions; origins on slab planes -> 0*inf = NaN
    d[1000:1600, 0] = 0.0
    d[1300:1600, 0] = -0.0
    d[1600:2000, 1] = 0.0
    d[1600:1800, 2] = -0.0
    o[1000:1400, 0] = mn[1000:1400, 0]
    o[1600:1700, 1] = mx[1600:1700, 1]
    o[2000:2200] = (mn[2000:2200] + mx[2000:2200]) / 2      # inside
    d[2200:2300] = 0.0                                      # zero direction
    d[2300:2400] = np.float32(1e-30) * np.sign(d[2300:2400])  # tiny directions (huge reciprocals)
    cases = np.concatenate([mn, mx, o, d], 1).astype("<f4")
    cases.tofile(tmp("aabb.in"))
    run("aabb", tmp("aabb.in"), tmp("aabb.out"))
    hit = np.fromfile(tmp("aabb.out"), "<i4")
    np.savez_compressed(os.path.join(GOLDEN, "aabb_cases.npz"), cases=cases, hit=hit)


def gen_light(rng):
    k = 3000
    u = rng.integers(0, 2**32, (k, 3), dtype=np.uint64).astype(np.uint32)
    edge = np.array([0, 1, 0x7FFFFFFF, 0x80000000, 0xFFFFFF7F, 0xFFFFFF80, 0xFFFFFFFF], np.uint32)
    u[:300] = rng.choice(edge, (300, 3))
    u.astype("<u4").tofile(tmp("light.in"))
    run("light", CORNELL_DIR, tmp("light.in"), tmp("light.out"))
    res = np.fromfile(tmp("light.out"), np.dtype([("loc", "<f4", 3), ("n", "<f4", 3), ("emission", "<f4", 3), ("pdf", "<f4")]))
    np.savez_compressed(os.path.join(GOLDEN, "light_cases.npz"), u=u, loc=res["loc"], n=res["n"], emission=res["emission"], pdf=res["pdf"])


def gen_material(rng):
    k = 3000
    n = rng.normal(size=(k, 3)).astype(np.float32)
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    n[:300] = axes[rng.integers(0, 6, 300)]
    n[300:400, 1] = n[300:400, 0]          # |n.x| == |n.y| tie
    n = n.astype(np.float32)
    wi = rng.normal(size=(k, 3)).astype(np.float32)
    u = rng.integers(0, 2**32, (k, 2), dtype=np.uint64).astype(np.uint32)
    edge = np.array([0, 1, 0x80000000, 0xFFFFFF7F, 0xFFFFFF80, 0xFFFFFFFF], np.uint32)
    u[:200] = rng.choice(edge, (200, 2))
    alb = rng.integers(0, 3, k).astype(np.uint32)
    rec = np.concatenate([n.view(np.uint32), wi.view(np.uint32), u, alb[:, None]], 1).astype("<u4")
    rec.tofile(tmp("mat.in"))
    run("material", tmp("mat.in"), tmp("mat.out"))
    res = np.fromfile(tmp("mat.out"), np.dtype([("raw", "<f4", 3), ("dir", "<f4", 3), ("brdf", "<f4", 3), ("pdf", "<f4")]))
    np.savez_compressed(os.path.join(GOLDEN, "material_cases.npz"), n=n, wi=wi, u=u, albedo_index=alb,
                        raw=res["raw"], dir=res["dir"], brdf=res["brdf"], pdf=res["pdf"])


def gen_camera():
    out = {}
    for (W, H, frame, seed) in [(16, 16, 1, 0), (12, 9, 3, 42), (4, 4, 1, 7), (17, 13, 2, 0)]:
        run("camera", W, H, frame, seed, tmp("cam"))
        b = np.fromfile(tmp("cam"), np.uint8)
        mats = b[:256].view("<f4").reshape(4, 4, 4)
        vec = b[256:280].view("<f4")
        inj = b[280:284].view("<i4")[0]
        dirs = b[284:].view("<f4").reshape(-1, 3)
        key = f"{W}x{H}_f{frame}_s{seed}"
        out[f"mats_{key}"] = mats
        out[f"dirs_{key}"] = dirs
        out[f"vec_{key}"] = vec
        assert inj == 1
    for (W, H) in [(784, 784), (1920, 1080), (3840, 2160), (1280, 960), (640, 480), (64, 64), (128, 128), (40, 30)]:
        run("camera", W, H, 1, 0, tmp("cam"))
        b = np.fromfile(tmp("cam"), np.uint8)
        out[f"mats_{W}x{H}"] = b[:256].view("<f4").reshape(4, 4, 4)
    np.savez_compressed(os.path.join(GOLDEN, "camera.npz"), **out)


def gen_images():
    out = {}
    for (W, H, spp, seed, rr) in [(64, 64, 1, 0, 0.8), (64, 64, 16, 0, 0.8), (64, 64, 256, 0, 0.8), (128, 128, 16, 7, 0.8),
                                  (40, 30, 8, 123, 0.5), (33, 17, 4, 5, 0.9)]:
        run("image", CORNELL_DIR, "", W, H, spp, seed, rr, os.cpu_count() or 8, tmp("acc"), tmp("rgba"), tmp("stats"))
        key = f"{W}x{H}_spp{spp}_s{seed}_rr{rr}"
        out[f"accum_{key}"] = np.fromfile(tmp("acc"), "<f4").reshape(H, W, 4)
        out[f"rgba_{key}"] = np.fromfile(tmp("rgba"), "<u4").reshape(H, W)
        out[f"stats_{key}"] = np.fromfile(tmp("stats"), "<u8")
    np.savez_compressed(os.path.join(GOLDEN, "images_cornell.npz"), **out)


# Cornell + Whitted::Sphere entities (MC/Sphere.h:16-108 through Renderer::Add + GenerateBVH):
# (center, radius, material of {red, green, white, light}); a white sphere on the floor, a green one above the
# short box, a white one half inside the tall box (its surface crosses the box's faces: ties and near-ties with
# triangles), and an emissive one (the light's material: after the light mesh, so SamplingAreaLight still picks
# the mesh) near the ceiling
SPHERES = [((3.9, 1.0, 1.2), 0.9, 2), ((1.5, 2.3, 1.3), 0.6, 1), ((3.4, 3.3, 3.3), 0.5, 2), ((4.6, 4.7, 4.3), 0.35, 3)]


def sphere_extra():
    return ",".join(f"sphere:{c[0]!r}:{c[1]!r}:{c[2]!r}:{r!r}:{m}" for (c, r, m) in SPHERES)


def gen_spheres(rng):
    """tests/golden/cornell_spheres.npz: the reference's own Sphere / BVH / TriangleMesh code (ref_harness) on the
    Cornell box + SPHERES -- the flattened two-level tree, 4096 closest hits, and images at 128x128x64 (the
    VERDICT's case) and two more shapes / roulette settings."""
    extra = sphere_extra()
    run("scene", CORNELL_DIR, extra, tmp("snodes"), tmp("stris"), tmp("smeshes"))
    nodes = np.fromfile(tmp("snodes"), NODE_DT)
    tris = np.fromfile(tmp("stris"), TRI_DT)
    meshes = np.fromfile(tmp("smeshes"), MESH_DT)
    cam = np.array([2.81432, 4.20749, -9.11751], np.float32)
    lo, hi = np.array([0, 0, 0], np.float32), np.array([5.56, 5.488, 5.592], np.float32)
    cen = np.array([c for (c, _, _) in SPHERES], np.float32)
    rad = np.array([r for (_, r, _) in SPHERES], np.float32)
    o, d = [], []
    k = 1200   # camera rays into the box
    tgt = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    o.append(np.repeat(cam[None], k, 0)); d.append(tgt - cam)
    k = 1200   # interior origins, random directions
    o.append(rng.uniform(lo, hi, (k, 3)).astype(np.float32)); d.append(rng.normal(size=(k, 3)).astype(np.float32))
    k = 800    # aimed at sphere centers, from the camera and from inside the box
    si = rng.integers(0, len(SPHERES), k)
    src = np.where((rng.random(k) < 0.5)[:, None], cam[None], rng.uniform(lo, hi, (k, 3)).astype(np.float32))
    o.append(src.astype(np.float32)); d.append((cen[si] - src).astype(np.float32))
    k = 896    # grazing: aimed at points on (or just off) the silhouettes
    si = rng.integers(0, len(SPHERES), k)
    src = np.where((rng.random(k) < 0.5)[:, None], cam[None], rng.uniform(lo, hi, (k, 3)).astype(np.float32))
    v = (cen[si] - src).astype(np.float32)
    perp = np.cross(v, rng.normal(size=(k, 3)).astype(np.float32))
    perp /= np.linalg.norm(perp, axis=1, keepdims=True) + 1e-30
    scale = rad[si] * rng.choice([0.999, 1.0, 1.0001, 0.5], k).astype(np.float32)
    o.append(src.astype(np.float32)); d.append((cen[si] + perp * scale[:, None] - src).astype(np.float32))
    o = np.concatenate(o).astype(np.float32)
    d = np.concatenate(d).astype(np.float32)
    np.concatenate([o, d], 1).astype("<f4").tofile(tmp("srays.in"))
    run("rays", CORNELL_DIR, extra, tmp("srays.in"), tmp("srays.out"))
    res = np.fromfile(tmp("srays.out"), HIT_DT)
    out = dict(spheres_center=cen, spheres_radius=rad, spheres_material=np.array([m for (_, _, m) in SPHERES], np.int32),
               nodes=nodes.view(np.uint8), tris=tris.view(np.uint8), meshes=meshes.view(np.uint8),
               org=o, dir=d, hit=res["hit"], tri=res["tri"], mat=res["mat"], t=res["t"], loc=res["loc"], n=res["n"])
    for (W, H, spp, seed, rr) in [(128, 128, 64, 0, 0.8), (96, 72, 16, 3, 0.5), (64, 48, 32, 11, 0.9)]:
        run("image", CORNELL_DIR, extra, W, H, spp, seed, rr, os.cpu_count() or 8, tmp("acc"), tmp("rgba"), tmp("stats"))
        key = f"{W}x{H}_spp{spp}_s{seed}_rr{rr}"
        out[f"accum_{key}"] = np.fromfile(tmp("acc"), "<f4").reshape(H, W, 4)
        out[f"rgba_{key}"] = np.fromfile(tmp("rgba"), "<u4").reshape(H, W)
        out[f"stats_{key}"] = np.fromfile(tmp("stats"), "<u8")
    np.savez_compressed(os.path.join(GOLDEN, "cornell_spheres.npz"), **out)
    print(f"  spheres: {len(nodes)} nodes, {len(tris)} slots, {int(res['hit'].sum())} hits of {len(o)} rays, "
          f"{int((np.isin(res['tri'], [i for i, t in enumerate(tris) if t['n'][0] == 0 and t['n'][1] == 0 and t['n'][2] == 0])).sum())} on spheres")


FULL_CONFIGS = [("c2", 784, 784, 256), ("c4", 1920, 1080, 1024)]
FULL_ROW_STRIDE = 16


def gen_full(which=None):
    """The benchmarked Cornell configurations at their FULL spp: C2 784x784x256 and
    C4 1920x1080x1024, seed 0, RR 0.8, frames 1..spp (MC/Renderer.cpp:114-133 accumulation over all frames).
    Stores the SHA-256 of the float4 accumulation and of the RGBA8 frame, and every 16th row of the
    accumulation's rgb (rows 0, 16, 32, ...), from which bench.py and the GPU tests compute RMSE / bitwise
    fractions.  C4 takes about 5 minutes on 8 cores."""
    import hashlib
    for (name, W, H, spp) in FULL_CONFIGS:
        if which not in (None, name):
            continue
        run("image", CORNELL_DIR, "", W, H, spp, 0, 0.8, os.cpu_count() or 8, tmp("acc"), tmp("rgba"), tmp("stats"))
        acc = np.fromfile(tmp("acc"), "<f4").reshape(H, W, 4)
        rgba = np.fromfile(tmp("rgba"), "<u4").reshape(H, W)
        rows = np.arange(0, H, FULL_ROW_STRIDE)
        np.savez_compressed(os.path.join(GOLDEN, f"full_{name}.npz"), W=np.int64(W), H=np.int64(H), spp=np.int64(spp),
                            seed=np.int64(0), rr=np.float32(0.8), first_frame=np.int64(1),
                            sha_accum=np.array(hashlib.sha256(acc.tobytes()).hexdigest()),
                            sha_rgba=np.array(hashlib.sha256(rgba.tobytes()).hexdigest()),
                            rows=rows.astype(np.int64), accum_rows=np.ascontiguousarray(acc[rows, :, :3]),
                            rgba_rows=np.ascontiguousarray(rgba[rows]), stats=np.fromfile(tmp("stats"), "<u8"))


C5_FULL_ROW_STRIDE = 64


def c5_obj():
    """The C5 OBJ (the bunny subdivided 1:4 twice, written x100), as gen_c5 makes it."""
    rt = load_pkg()
    bunny = np.load(os.path.join(GOLDEN, "bvh_scene.npz"))["raw_bunny"]
    raw = rt.c5_mesh(bunny)
    obj = tmp("c5_bunny.obj")
    rt.write_obj(obj, raw)
    return obj


def gen_full_c5(spp=256, row_stride=1, row_offset=0):
    """C5's launch shape: the Cornell box + the 79,488-triangle bunny at 3840x2160,
    seed 0, RR 0.8, frames 1..spp, through the reference's own TriangleMesh + BVH (MC/Renderer.cpp:114-133
    accumulation over all frames; MC/BVH.h:72-101 traversal).  2.1 G samples at 256 spp: long enough that
    some paths exceed the 624 words of one engine fill, so the harness re-fills the injected stream at the
    top of a shading call (mt_inject.h refill_if_near).  Stores the SHA-256 of the float4 accumulation and
    of the RGBA8 frame, and every 64th row of the accumulation's rgb.  row_offset (round 6): the rows
    y % 64 == row_offset instead, a second fixture of the same frame (full_c5_4096_mid: the rows halfway between)."""
    import hashlib
    import time
    W, H = 3840, 2160
    obj = c5_obj()
    t0 = time.time()
    extra = ([C5_FULL_ROW_STRIDE] + ([row_offset] if row_offset else [])) if row_stride > 1 else []
    run("image", CORNELL_DIR, obj, W, H, spp, 0, 0.8, os.cpu_count() or 8, tmp("acc"), tmp("rgba"), tmp("stats"), *extra)
    secs = time.time() - t0
    acc = np.fromfile(tmp("acc"), "<f4").reshape(H, W, 4)
    rgba = np.fromfile(tmp("rgba"), "<u4").reshape(H, W)
    rows = np.arange(row_offset, H, C5_FULL_ROW_STRIDE)
    name = ("full_c5" if spp == 256 else f"full_c5_{spp}") + ({0: "", 32: "_mid"}.get(row_offset, f"_o{row_offset}"))
    # (rows only: the SHA-256 of the committed rows' accumulation and RGBA8 instead of the whole frame's)
    sel_acc, sel_rgba = (acc, rgba) if row_stride == 1 else (np.ascontiguousarray(acc[rows]), np.ascontiguousarray(rgba[rows]))
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), W=np.int64(W), H=np.int64(H), spp=np.int64(spp),
                        seed=np.int64(0), rr=np.float32(0.8), first_frame=np.int64(1), rows_only=np.bool_(row_stride > 1),
                        sha_accum=np.array(hashlib.sha256(sel_acc.tobytes()).hexdigest()),
                        sha_rgba=np.array(hashlib.sha256(sel_rgba.tobytes()).hexdigest()),
                        rows=rows.astype(np.int64), accum_rows=np.ascontiguousarray(acc[rows, :, :3]),
                        rgba_rows=np.ascontiguousarray(rgba[rows]), stats=np.fromfile(tmp("stats"), "<u8"),
                        harness_seconds=np.float64(secs), harness_threads=np.int64(os.cpu_count() or 8))


def gen_stat():
    """The reference with its SHIPPED random stream (serial std::mt19937 seeded 5489, MSVC 32-bit
    distribution, camera draws then pixel loop per frame): the statistical gate of SURVEY.md 8(d)."""
    W, H, spp, rr = 64, 64, 1024, 0.8
    run("image_mt", CORNELL_DIR, W, H, spp, rr, tmp("mt_acc"))
    acc = np.fromfile(tmp("mt_acc"), "<f4").reshape(H, W, 4)
    np.savez_compressed(os.path.join(GOLDEN, "stat_mt19937.npz"), accum=acc, W=np.int64(W), H=np.int64(H), spp=np.int64(spp),
                        rr=np.float32(rr))


# ------------------------------------------------------------------ BVH Ray Tracer (config C3)
BV_DIR = os.path.join(REF, "BVH Ray Tracer", "8599RayTracerGUI", "src")
HARNESS_BV = os.path.join(HERE, "_ref", "ref_whitted_bvh")
BV_NODE_FIELDS = ("mn", "mx", "left", "right", "tri", "mesh", "top")   # area: not part of the BV build


def run_bv(*args):
    r = subprocess.run([HARNESS_BV] + [str(a) for a in args], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"ref_whitted_bvh {args[0]} failed: {r.returncode} {r.stderr}")
    print(" ", r.stdout.strip())


def bv_objs():
    return os.path.join(BV_DIR, "stanford_bunny.obj"), os.path.join(BV_DIR, "utah_teapot.obj")


def scene_digest(nodes, tris):
    """SHA-256 over the flattened topology and geometry (the fields both builds define)."""
    import hashlib
    h = hashlib.sha256()
    for f in BV_NODE_FIELDS:
        h.update(np.ascontiguousarray(nodes[f]).tobytes())
    for f in ("a", "b", "c", "n", "mesh"):
        h.update(np.ascontiguousarray(tris[f]).tobytes())
    return h.hexdigest()


def gen_bvh_scene():
    bunny, teapot = bv_objs()
    raw = {}
    for name, path in (("bunny", bunny), ("teapot", teapot)):
        run("objraw", path, tmp(name + ".raw"))
        raw[name] = np.fromfile(tmp(name + ".raw"), "<f4").reshape(-1, 9)
    run_bv("scene", bunny, teapot, tmp("bv_nodes"), tmp("bv_tris"))
    nodes = np.fromfile(tmp("bv_nodes"), NODE_DT)
    tris = np.fromfile(tmp("bv_tris"), TRI_DT)
    np.savez_compressed(os.path.join(GOLDEN, "bvh_scene.npz"), raw_bunny=raw["bunny"], raw_teapot=raw["teapot"],
                        n_nodes=np.int64(len(nodes)), n_tris=np.int64(len(tris)), digest=np.array(scene_digest(nodes, tris)),
                        nodes_head=nodes[:512].view(np.uint8), tris_head=tris[:256].view(np.uint8))
    return nodes, tris


def gen_bvh_rays(nodes, tris, rng):
    n = 4096
    cam = np.array([-1, 5, 10], np.float32)
    lo, hi = nodes["mn"][0], nodes["mx"][0]
    o, d = [], []
    k = 1500   # camera rays at the objects
    tgt = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    o.append(np.repeat(cam[None], k, 0)); d.append(tgt - cam)
    k = 1000   # random origins around the objects
    o.append(rng.uniform(lo - 2, hi + 2, (k, 3)).astype(np.float32)); d.append(rng.normal(size=(k, 3)).astype(np.float32))
    k = 500    # towards the point lights from surface-ish points (shadow rays)
    ti = rng.integers(0, len(tris), k)
    src = ((tris["a"][ti] + tris["b"][ti] + tris["c"][ti]) / 3).astype(np.float32)
    light = np.where((rng.random(k) < 0.5)[:, None], np.array([-20, 70, 20], np.float32), np.array([20, 70, 20], np.float32))
    o.append(src); d.append((light - src).astype(np.float32))
    k = 300    # axis-aligned directions
    oo = rng.uniform(lo - 1, hi + 1, (k, 3)).astype(np.float32)
    dd = np.zeros((k, 3), np.float32)
    dd[np.arange(k), rng.integers(0, 3, k)] = rng.choice([-1.0, 1.0], k)
    o.append(oo); d.append(dd)
    k = n - sum(len(x) for x in o)   # through vertices and edge midpoints (shared edges, ties)
    ti = rng.integers(0, len(tris), k)
    w = rng.integers(0, 3, k)
    a, b, c = tris["a"][ti], tris["b"][ti], tris["c"][ti]
    tgt = np.where((w == 0)[:, None], a, np.where((w == 1)[:, None], 0.5 * (a + b), 0.5 * (b + c)))
    o.append(np.repeat(cam[None], k, 0)); d.append((tgt - cam).astype(np.float32))
    o = np.concatenate(o).astype(np.float32)
    d = np.concatenate(d).astype(np.float32)
    np.concatenate([o, d], 1).astype("<f4").tofile(tmp("bv_rays.in"))
    bunny, teapot = bv_objs()
    run_bv("rays", bunny, teapot, tmp("bv_rays.in"), tmp("bv_rays.out"))
    res = np.fromfile(tmp("bv_rays.out"), HIT_DT)
    np.savez_compressed(os.path.join(GOLDEN, "bvh_rays.npz"), org=o, dir=d, hit=res["hit"], tri=res["tri"], t=res["t"],
                        loc=res["loc"], n=res["n"])


def gen_bvh_images():
    import hashlib
    bunny, teapot = bv_objs()
    out = {}
    for (W, H) in [(16, 12), (1280, 960)]:
        run_bv("camera", W, H, tmp("bv_cam"))
        b = np.fromfile(tmp("bv_cam"), np.uint8)
        out[f"mats_{W}x{H}"] = b[:256].view("<f4").reshape(4, 4, 4)
        out[f"vec_{W}x{H}"] = b[256:280].view("<f4")
        if W * H <= 4096:
            out[f"dirs_{W}x{H}"] = b[280:].view("<f4").reshape(-1, 3)
    for (W, H, spp) in [(160, 120, 3), (97, 61, 2), (1280, 960, 64)]:
        run_bv("image", bunny, teapot, W, H, spp, os.cpu_count() or 8, tmp("acc"), tmp("rgba"), tmp("stats"))
        acc = np.fromfile(tmp("acc"), "<f4").reshape(H, W, 4)
        rgba = np.fromfile(tmp("rgba"), "<u4").reshape(H, W)
        key = f"{W}x{H}_spp{spp}"
        if W * H <= 20000:
            out[f"accum_{key}"] = acc
            out[f"rgba_{key}"] = rgba
        out[f"sha_accum_{key}"] = np.array(hashlib.sha256(acc.tobytes()).hexdigest())
        out[f"sha_rgba_{key}"] = np.array(hashlib.sha256(rgba.tobytes()).hexdigest())
        out[f"stats_{key}"] = np.fromfile(tmp("stats"), "<u8")
    np.savez_compressed(os.path.join(GOLDEN, "bvh_images.npz"), **out)


# ------------------------------------------------------------------ Cornell box + synthesized mesh (config C5)
def load_pkg():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rt_amd", os.path.join(REPO, "cpu-based-ray-tracer_amd", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def gen_c5(rng):
    """C5: the Cornell box + the 79,488-triangle subdivided bunny, added through the reference's own
    TriangleMesh(OBJ, white) + BVH (build_cornell's `extra`).  The OBJ is generated from the committed
    raw bunny (bvh_scene.npz) by the package's c5_mesh(); its values round-trip exactly through stof."""
    import hashlib
    rt = load_pkg()
    bunny = np.load(os.path.join(GOLDEN, "bvh_scene.npz"))["raw_bunny"]
    raw = rt.c5_mesh(bunny)
    obj = tmp("c5_bunny.obj")
    rt.write_obj(obj, raw)
    run("objraw", obj, tmp("c5.raw"))
    assert np.array_equal(np.fromfile(tmp("c5.raw"), "<f4").reshape(-1, 9).view(np.uint32), raw.view(np.uint32))
    run("scene", CORNELL_DIR, obj, tmp("c5_nodes"), tmp("c5_tris"), tmp("c5_meshes"))
    nodes = np.fromfile(tmp("c5_nodes"), NODE_DT)
    tris = np.fromfile(tmp("c5_tris"), TRI_DT)
    out = dict(n_nodes=np.int64(len(nodes)), n_tris=np.int64(len(tris)), digest=np.array(scene_digest(nodes, tris)),
               nodes_head=nodes[:512].view(np.uint8), tris_head=tris[:256].view(np.uint8),
               raw_sha=np.array(hashlib.sha256(raw.tobytes()).hexdigest()))
    # closest-hit rays: camera rays at the bunny, interior rays, rays grazing bunny vertices/edges
    n = 4096
    cam = np.array([2.81432, 4.20749, -9.11751], np.float32)
    lo, hi = raw.reshape(-1, 3).min(0) * np.float32(0.01), raw.reshape(-1, 3).max(0) * np.float32(0.01)
    o, d = [], []
    k = 1500
    o.append(np.repeat(cam[None], k, 0)); d.append(rng.uniform(lo, hi, (k, 3)).astype(np.float32) - cam)
    k = 1500
    room_lo, room_hi = np.array([0, 0, 0], np.float32), np.array([5.56, 5.488, 5.592], np.float32)
    o.append(rng.uniform(room_lo, room_hi, (k, 3)).astype(np.float32)); d.append(rng.normal(size=(k, 3)).astype(np.float32))
    k = n - 3000
    bt = tris[tris["mesh"] == 6]
    ti = rng.integers(0, len(bt), k)
    w = rng.integers(0, 3, k)
    a, b, c = bt["a"][ti], bt["b"][ti], bt["c"][ti]
    tgt = np.where((w == 0)[:, None], a, np.where((w == 1)[:, None], 0.5 * (a + b), (a + b + c) / 3)).astype(np.float32)
    src = rng.uniform(room_lo, room_hi, (k, 3)).astype(np.float32)
    o.append(src); d.append((tgt - src).astype(np.float32))
    o = np.concatenate(o).astype(np.float32)
    d = np.concatenate(d).astype(np.float32)
    np.concatenate([o, d], 1).astype("<f4").tofile(tmp("c5_rays.in"))
    run("rays", CORNELL_DIR, obj, tmp("c5_rays.in"), tmp("c5_rays.out"))
    res = np.fromfile(tmp("c5_rays.out"), HIT_DT)
    out.update(ray_org=o, ray_dir=d, ray_hit=res["hit"], ray_tri=res["tri"], ray_t=res["t"])
    # images: a small one stored whole, the full C5 frame (3840x2160) at 1 spp by SHA-256, and the
    # per-sample work counters at 480x270
    for (W, H, spp, seed) in [(96, 54, 16, 0), (3840, 2160, 1, 0), (480, 270, 4, 3)]:
        run("image", CORNELL_DIR, obj, W, H, spp, seed, 0.8, os.cpu_count() or 8, tmp("acc"), tmp("rgba"), tmp("stats"))
        acc = np.fromfile(tmp("acc"), "<f4").reshape(H, W, 4)
        rgba = np.fromfile(tmp("rgba"), "<u4").reshape(H, W)
        key = f"{W}x{H}_spp{spp}_s{seed}"
        if W * H <= 20000:
            out[f"accum_{key}"] = acc
            out[f"rgba_{key}"] = rgba
        out[f"sha_accum_{key}"] = np.array(hashlib.sha256(acc.tobytes()).hexdigest())
        out[f"sha_rgba_{key}"] = np.array(hashlib.sha256(rgba.tobytes()).hexdigest())
        out[f"stats_{key}"] = np.fromfile(tmp("stats"), "<u8")
    np.savez_compressed(os.path.join(GOLDEN, "c5_scene.npz"), **out)


# ------------------------------------------------------------------ Whitted Style Ray Tracer (config C1)
HARNESS_WH = os.path.join(HERE, "_ref", "ref_whitted_spheres")
WH_HIT_DT = np.dtype([("ent", "<i4"), ("tri", "<i4"), ("t", "<f4"), ("b2", "<f4"), ("b3", "<f4")])


def gen_optics(rng):
    """The Renderer's optics helpers (mirror_reflection_direction, snell_refraction_direction,
    accurate_fresnel_reflectance: WH/Renderer.h:41-107, the same code as MC/Renderer.h:93-161) on unit incident
    directions and normals from outside and inside, grazing and perpendicular incidence, and total internal
    reflection, for the drop-in Renderer's public surface (tests/test_walnut_queries.py)."""
    n = 4096
    def unit(k):
        v = rng.normal(size=(k, 3))
        return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)
    I, N = unit(n), unit(n)
    eta = rng.choice(np.array([1.0, 1.00029, 1.333, 1.5, 1.6, 2.42, 0.75], np.float32), n).astype(np.float32)
    # exact edge cases: I perpendicular to N (cos 0: "inside"), I = -N, I = N, axis-aligned normals
    I[:4] = [[1, 0, 0], [0, -1, 0], [0, 1, 0], [0.6, -0.8, 0]]
    N[:4] = [[0, 1, 0], [0, 1, 0], [0, 1, 0], [0, 1, 0]]
    cases = np.concatenate([I, N, eta[:, None]], 1).astype("<f4")
    cases.tofile(tmp("optics.in"))
    run_wh("optics", tmp("optics.in"), tmp("optics.out"))
    res = np.fromfile(tmp("optics.out"), "<f4").reshape(n, 7)
    np.savez_compressed(os.path.join(GOLDEN, "optics_cases.npz"), cases=cases, mirror=res[:, 0:3], snell=res[:, 3:6], fresnel=res[:, 6])


def run_wh(*args):
    r = subprocess.run([HARNESS_WH] + [str(a) for a in args], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"ref_whitted_spheres {args[0]} failed: {r.returncode} {r.stderr}")
    print(" ", r.stdout.strip())


def gen_c1(rng):
    """C1: the two-sphere Whitted world through the reference's own Sphere / TriangleMesh / Camera code
    (shading recursion restated, see oracle/ref/ref_whitted_spheres.cpp)."""
    import hashlib
    out = {}
    for (W, H) in [(16, 12), (640, 480), (160, 120)]:
        run_wh("camera", W, H, tmp("wh_cam"))
        b = np.fromfile(tmp("wh_cam"), np.uint8)
        out[f"mats_{W}x{H}"] = b[:256].view("<f4").reshape(4, 4, 4)
        out[f"vec_{W}x{H}"] = b[256:280].view("<f4")
        if W * H <= 4096:
            out[f"dirs_{W}x{H}"] = b[280:].view("<f4").reshape(-1, 3)
    # closest hits: camera rays at the objects, random rays (incl. from inside the glass sphere),
    # rays at the chessboard's vertices and shared diagonal (ties between its two triangles)
    n = 4096
    cam = np.array([0, 0, 6], np.float32)
    o, d = [], []
    k = 1500
    tgt = rng.uniform([-6, -3.5, -17], [6, 3, -5], (k, 3)).astype(np.float32)
    o.append(np.repeat(cam[None], k, 0)); d.append(tgt - cam)
    k = 1000
    o.append(rng.uniform([-6, -2.9, -17], [6, 4, -4], (k, 3)).astype(np.float32)); d.append(rng.normal(size=(k, 3)).astype(np.float32))
    k = 600   # from inside the glass sphere (center (0.5, -0.5, -8), r 1.5)
    dirv = rng.normal(size=(k, 3)); dirv /= np.linalg.norm(dirv, axis=1, keepdims=True)
    o.append((np.array([0.5, -0.5, -8]) + dirv * rng.uniform(0, 1.4, (k, 1))).astype(np.float32))
    d.append(rng.normal(size=(k, 3)).astype(np.float32))
    k = n - 3100
    board = np.array([[-5, -3, -6], [5, -3, -6], [5, -3, -16], [-5, -3, -16]], np.float32)
    w = rng.random(k)
    a, b = board[1], board[3]   # the shared edge of triangles (0,1,3) and (1,2,3)
    tgt = np.where((rng.random(k) < 0.5)[:, None], (a[None] * w[:, None] + b[None] * (1 - w[:, None])), board[rng.integers(0, 4, k)])
    o.append(np.repeat(cam[None], k, 0)); d.append((tgt - cam).astype(np.float32))
    o = np.concatenate(o).astype(np.float32)
    d = np.concatenate(d).astype(np.float32)
    np.concatenate([o, d], 1).astype("<f4").tofile(tmp("wh_rays.in"))
    run_wh("rays", tmp("wh_rays.in"), tmp("wh_rays.out"))
    res = np.fromfile(tmp("wh_rays.out"), WH_HIT_DT)
    out.update(ray_org=o, ray_dir=d, ray_ent=res["ent"], ray_tri=res["tri"], ray_t=res["t"], ray_b2=res["b2"], ray_b3=res["b3"])
    # glibc powf on specular-lobe arguments (x in [0, 1], exponent 25)
    x = np.concatenate([rng.random(20000), rng.random(2000) ** 0.01, [0.0, 1.0, 0.5]]).astype(np.float32)
    pin = np.stack([x, np.full_like(x, 25.0)], 1).astype("<f4")
    pin.tofile(tmp("pow.in"))
    run_wh("pow", tmp("pow.in"), tmp("pow.out"))
    out.update(pow_x=x, pow_y=np.float32(25.0), pow_out=np.fromfile(tmp("pow.out"), "<f4"))
    for (W, H, spp) in [(640, 480, 1), (160, 120, 3), (97, 61, 2)]:
        run_wh("image", W, H, spp, os.cpu_count() or 8, tmp("acc"), tmp("rgba"), tmp("stats"))
        acc = np.fromfile(tmp("acc"), "<f4").reshape(H, W, 4)
        rgba = np.fromfile(tmp("rgba"), "<u4").reshape(H, W)
        key = f"{W}x{H}_spp{spp}"
        out[f"accum_{key}"] = acc
        out[f"rgba_{key}"] = rgba
        out[f"sha_accum_{key}"] = np.array(hashlib.sha256(acc.tobytes()).hexdigest())
        out[f"sha_rgba_{key}"] = np.array(hashlib.sha256(rgba.tobytes()).hexdigest())
        out[f"stats_{key}"] = np.fromfile(tmp("stats"), "<u8")
    np.savez_compressed(os.path.join(GOLDEN, "c1_spheres.npz"), **out)


# ------------------------------------------------------------------ the Denoiser project
HARNESS_DN = os.path.join(HERE, "_ref", "ref_denoiser")
DN_DIR = os.path.join(REF, "Denoiser", "8599RayTracerGUI", "src", "cornellbox")
# (name, W, H, frames, seed, step_x, jbf_half, temporal_half, tolerance, weighting, immediate_clamp)
DN_CASES = [("full", 96, 72, 4, 0, 0.05, 3, 3, 1.0, 0.2, 1),
            ("temporal", 96, 72, 3, 5, 0.08, 0, 7, 2.0, 0.1, 1),
            ("jbf16", 64, 48, 2, 9, 0.0, 16, 0, 1.0, 0.2, 0)]


def gen_dn():
    """Frames of the Denoiser project through the reference's own Denoising::Denoiser (DN/Denoiser.h,
    compiled as is) and its DN/ geometry + camera code (shading glue restated, oracle/ref/ref_denoiser.cpp)."""
    out = {}
    for (name, W, H, n, seed, step, jh, th, tol, wgt, clamp) in DN_CASES:
        r = subprocess.run([HARNESS_DN, "frames", DN_DIR, str(W), str(H), str(n), str(seed), repr(step), str(jh), str(th), repr(tol),
                            repr(wgt), str(clamp), str(os.cpu_count() or 8), tmp("dn.bin")], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"ref_denoiser failed: {r.stderr}")
        print(" ", r.stdout.strip())
        b = np.fromfile(tmp("dn.bin"), np.uint8)
        npx = W * H
        off = 0

        def take(dt, count):
            nonlocal off
            nb = np.dtype(dt).itemsize * count
            v = b[off:off + nb].view(dt)
            off += nb
            return v
        for k in range(n):
            key = f"{name}_f{k + 1}"
            out[f"{key}_color"] = take("<f4", 3 * npx).reshape(H, W, 3)
            out[f"{key}_pos"] = take("<f4", 3 * npx).reshape(H, W, 3)
            out[f"{key}_nrm"] = take("<f4", 3 * npx).reshape(H, W, 3)
            out[f"{key}_contrib"] = take("<i4", npx).reshape(H, W)
            out[f"{key}_prim"] = take("<i4", npx).reshape(H, W)
            out[f"{key}_proj"] = take("<f4", 16)
            out[f"{key}_view"] = take("<f4", 16)
            out[f"{key}_campos"] = take("<f4", 3)
            out[f"{key}_spatial"] = take("<f4", 3 * npx).reshape(H, W, 3)
            out[f"{key}_temporal"] = take("<f4", 3 * npx).reshape(H, W, 3)
            out[f"{key}_rgba"] = take("<u4", npx).reshape(H, W)
        assert off == b.size
        out[f"{name}_params"] = np.array([W, H, n, seed, jh, th, clamp], np.int64)
        out[f"{name}_fparams"] = np.array([step, tol, wgt], np.float32)
    np.savez_compressed(os.path.join(GOLDEN, "denoiser.npz"), **out)


def main():
    global TMP
    if not all(os.path.exists(h) for h in (HARNESS, HARNESS_BV, HARNESS_WH, HARNESS_DN)):
        subprocess.check_call(["make", "-C", HERE, "ref"])
    os.makedirs(GOLDEN, exist_ok=True)
    only = sys.argv[1] if len(sys.argv) > 1 else "all"
    with tempfile.TemporaryDirectory() as TMP:
        if only in ("all", "cornell"):
            rng = np.random.default_rng(20260101)
            tris = gen_scene()
            gen_rays(tris, rng)
            gen_mt(rng)
            gen_aabb(rng)
            gen_light(rng)
            gen_material(rng)
            gen_camera()
            gen_images()
        if only in ("all", "cornell", "stat"):
            gen_stat()
        if only in ("all", "bvh"):
            rng = np.random.default_rng(20261015)
            nodes, tris = gen_bvh_scene()
            gen_bvh_rays(nodes, tris, rng)
            gen_bvh_images()
        if only in ("all", "c1"):
            gen_c1(np.random.default_rng(20261017))
        if only in ("all", "c1", "optics"):
            gen_optics(np.random.default_rng(20261018))
        if only in ("all", "dn"):
            gen_dn()
        if only in ("all", "c5"):
            gen_c5(np.random.default_rng(20261016))
        if only in ("all", "spheres"):
            gen_spheres(np.random.default_rng(20261018))
        if only in ("all", "full", "full_c2", "full_c4"):
            gen_full(None if only in ("all", "full") else only[5:])
        if only == "full_c5":
            gen_full_c5(256)
        if only == "full_c5_4096":
            # C5's full spp on every 64th row (the whole frame would take ~11 h on 8 cores): 535 M samples, ~10 min
            gen_full_c5(4096, row_stride=C5_FULL_ROW_STRIDE)
        if only == "full_c5_4096_mid":
            gen_full_c5(4096, row_stride=C5_FULL_ROW_STRIDE, row_offset=C5_FULL_ROW_STRIDE // 2)
        if only.startswith("full_c5_4096_o"):
            # the rows off by 16 / 48 (16, 80, ... and 48, 112, ...): with full_c5_4096 and _mid, every 16th row; by 8, 24,
            # 40, 56 as well (full_c5_4096_o8 ...): every 8th row
            gen_full_c5(4096, row_stride=C5_FULL_ROW_STRIDE, row_offset=int(only[len("full_c5_4096_o"):]))
    print("golden fixtures written to", GOLDEN)


if __name__ == "__main__":
    sys.exit(main())
