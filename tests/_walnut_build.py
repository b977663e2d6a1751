"""Build the Walnut drop-in check (tests/test_walnut_compat.py): the reference's own layer file
MC/mainloop.cpp, compiled UNCHANGED from /root/reference (copied to a scratch directory at build time only
so that its quoted "Camera.h" / "Renderer.h" resolve through the include path instead of its own
directory -- nothing of the reference is kept in this repository), against include/rt/walnut/*.h (the
drop-in) and the test-only Walnut / ImGui / glm stubs of tests/walnut_stub/, linked with librt_hip.so
and tests/walnut_stub/driver.cpp.  Needs /root/reference (this container); the GPU box runs the binary
built here (tests/_bin/, git-ignored, shipped with the tree like the .so files)."""
import os
import shutil
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAINLOOP = "/root/reference/Monte Carlo Path Tracer/8599RayTracerGUI/src/mainloop.cpp"
BIN = os.path.join(REPO, "tests", "_bin", "walnut_mainloop")


def build(out=BIN):
    if not os.path.exists(MAINLOOP):
        return None
    stub = os.path.join(REPO, "tests", "walnut_stub")
    pkg = os.path.join(REPO, "cpu-based-ray-tracer_amd")
    tmp = tempfile.mkdtemp(prefix="rt_walnut_")
    try:
        src = os.path.join(tmp, "mainloop.cpp")
        shutil.copyfile(MAINLOOP, src)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        cmd = ["g++", "-std=c++20", "-O1", "-Wall", "-Wno-unused-private-field", "-iquote", os.path.join(stub, "dropin"),
               "-I", stub, "-I", os.path.join(REPO, "include"), src, os.path.join(stub, "driver.cpp"), "-o", out,
               "-L", pkg, "-lrt_hip", "-Wl,-rpath," + pkg, "-Wl,-rpath-link,/opt/rocm/lib"]
        subprocess.run(cmd, check=True, capture_output=True, text=True)
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
