"""Build the Walnut drop-in checks (tests/test_walnut_compat.py).

1. The reference's own layer file MC/mainloop.cpp, compiled UNCHANGED from /root/reference (copied to a
   scratch directory at build time only so that its quoted "Camera.h" / "Renderer.h" resolve through the
   include path instead of its own directory -- nothing of the reference is kept in this repository), against
   include/rt/walnut/*.h (the drop-in) and the test-only Walnut / ImGui / glm stubs of tests/walnut_stub/,
   linked with librt_hip.so and tests/walnut_stub/driver.cpp.  Needs /root/reference (this container); the GPU
   box runs the binary built here (tests/_bin/, git-ignored, shipped with the tree like the .so files).
2. tests/walnut_stub/c5_scene.cpp: configuration C5 built through the reference's scene-extension spelling
   (Whitted::WhittedMaterial, Whitted::TriangleMesh(path, material*), Add, GenerateBVH) against the same
   drop-in headers.  Needs no reference file.
3. tests/walnut_stub/queries.cpp: the drop-in Renderer's scene queries and optics helpers with the reference's
   signatures (MC/Renderer.h:88-180).  Needs no reference file.
4. tests/walnut_stub/spheres.cpp: Whitted::Sphere entities through Add / GenerateBVH and the Whitted::Entity
   interface (MC/Entity.h:19-55, MC/Sphere.h:16-108), the public bvh / entities members.  Needs no reference file."""
import glob
import hashlib
import os
import shutil
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAINLOOP = "/root/reference/Monte Carlo Path Tracer/8599RayTracerGUI/src/mainloop.cpp"
BIN = os.path.join(REPO, "tests", "_bin", "walnut_mainloop")
C5_BIN = os.path.join(REPO, "tests", "_bin", "walnut_c5_scene")
QUERIES_BIN = os.path.join(REPO, "tests", "_bin", "walnut_queries")
SPHERES_BIN = os.path.join(REPO, "tests", "_bin", "walnut_spheres")
STUB = os.path.join(REPO, "tests", "walnut_stub")
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")


def headers():
    """The drop-in headers a front-end compiles against: their layout is what the library checks (rt/Abi.h)."""
    inc = os.path.join(REPO, "include")
    return sorted(glob.glob(os.path.join(inc, "*.h")) + glob.glob(os.path.join(inc, "rt", "*.h")) +
                  glob.glob(os.path.join(inc, "rt", "walnut", "*.h")))


def headers_digest():
    h = hashlib.sha256()
    for p in headers():
        h.update(os.path.relpath(p, REPO).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stamp(out):
    return out + ".headers"


def stale(out):
    """Why `out` must be rebuilt, or None: it is missing, or older than a drop-in header or librt_hip.so.
    (The round-5 r05a SIGSEGV was a walnut_mainloop built against an older rt::Renderer than the library's.)"""
    if not os.path.exists(out):
        return "missing"
    t = os.path.getmtime(out)
    for p in headers() + [os.path.join(PKG, "librt_hip.so")]:
        if os.path.exists(p) and os.path.getmtime(p) > t:
            return os.path.relpath(p, REPO) + " is newer"
    return None


def headers_changed(out):
    """On a box that only runs the prebuilt binaries (mtimes need not survive the copy): whether the headers
    differ from the ones `out` was compiled against (the digest stored next to it at build time)."""
    try:
        with open(_stamp(out)) as f:
            return f.read().strip() != headers_digest()
    except OSError:
        return True


def _gxx(srcs, out):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-std=c++20", "-O1", "-Wall", "-Wno-unused-private-field", "-iquote", os.path.join(STUB, "dropin"),
           "-I", STUB, "-I", os.path.join(REPO, "include")] + srcs + ["-o", out,
           "-L", PKG, "-lrt_hip", "-Wl,-rpath," + PKG, "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    with open(_stamp(out), "w") as f:
        f.write(headers_digest() + "\n")
    return out


def build_c5(out=C5_BIN):
    return _gxx([os.path.join(STUB, "c5_scene.cpp")], out)


def build_queries(out=QUERIES_BIN):
    return _gxx([os.path.join(STUB, "queries.cpp")], out)


def build_spheres(out=SPHERES_BIN):
    return _gxx([os.path.join(STUB, "spheres.cpp")], out)


def build(out=BIN, force=True):
    """Build the three binaries.  force=False rebuilds only those that are stale (missing, or older than a
    drop-in header or librt_hip.so)."""
    d = os.path.dirname(out)
    for path, fn in ((os.path.join(d, os.path.basename(C5_BIN)), build_c5),
                     (os.path.join(d, os.path.basename(QUERIES_BIN)), build_queries),
                     (os.path.join(d, os.path.basename(SPHERES_BIN)), build_spheres)):
        if force or stale(path):
            fn(path)
    if not os.path.exists(MAINLOOP):
        return None
    if not force and not stale(out):
        return out
    tmp = tempfile.mkdtemp(prefix="rt_walnut_")
    try:
        src = os.path.join(tmp, "mainloop.cpp")
        shutil.copyfile(MAINLOOP, src)
        return _gxx([src, os.path.join(STUB, "driver.cpp")], out)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
