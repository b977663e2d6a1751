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
   signatures (MC/Renderer.h:88-180).  Needs no reference file."""
import os
import shutil
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAINLOOP = "/root/reference/Monte Carlo Path Tracer/8599RayTracerGUI/src/mainloop.cpp"
BIN = os.path.join(REPO, "tests", "_bin", "walnut_mainloop")
C5_BIN = os.path.join(REPO, "tests", "_bin", "walnut_c5_scene")
QUERIES_BIN = os.path.join(REPO, "tests", "_bin", "walnut_queries")
STUB = os.path.join(REPO, "tests", "walnut_stub")
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")


def _gxx(srcs, out):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-std=c++20", "-O1", "-Wall", "-Wno-unused-private-field", "-iquote", os.path.join(STUB, "dropin"),
           "-I", STUB, "-I", os.path.join(REPO, "include")] + srcs + ["-o", out,
           "-L", PKG, "-lrt_hip", "-Wl,-rpath," + PKG, "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


def build_c5(out=C5_BIN):
    return _gxx([os.path.join(STUB, "c5_scene.cpp")], out)


def build_queries(out=QUERIES_BIN):
    return _gxx([os.path.join(STUB, "queries.cpp")], out)


def build(out=BIN):
    build_c5(os.path.join(os.path.dirname(out), os.path.basename(C5_BIN)))
    build_queries(os.path.join(os.path.dirname(out), os.path.basename(QUERIES_BIN)))
    if not os.path.exists(MAINLOOP):
        return None
    tmp = tempfile.mkdtemp(prefix="rt_walnut_")
    try:
        src = os.path.join(tmp, "mainloop.cpp")
        shutil.copyfile(MAINLOOP, src)
        return _gxx([src, os.path.join(STUB, "driver.cpp")], out)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
