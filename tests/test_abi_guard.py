"""The C++ drop-in's layout guard (include/rt/Abi.h; DESIGN.md section 1, "The round-5 SIGSEGV").

rt::Renderer / rt::Camera / rt::WhittedRenderer / rt::DenoisingRenderer are allocated by the caller with the
sizeof of the header IT was compiled against, and constructed by librt_hip.so.  Round 5's walnut_mainloop,
built against a 200-byte rt::Renderer, ran against a library whose rt::Renderer was 264 bytes: the library's
member initialisers wrote 64 bytes past the caller's heap object and the process died with SIGSEGV.

Here a caller is compiled against a deliberately different layout (a copy of include/ with one member added,
or another RT_CXX_ABI_VERSION) and must get a clean rt::Error, with every byte past its object untouched.
CPU only: the guard runs before the library touches a device."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cpu-based-ray-tracer_amd")
LIB = os.path.join(PKG, "librt_hip.so")

CALLER = r'''
#include <cstdio>
#include <cstring>
#include <new>
#include "rt/Renderer.h"
#include "rt/WhittedRenderer.h"
#include "rt/DenoisingRenderer.h"

// construct T in a buffer with a canary tail; report the outcome and whether the library wrote past sizeof(T)
template <class T, class F>
static void probe(const char* name, F make)
{
    alignas(64) static unsigned char buf[sizeof(T) + 512];
    std::memset(buf, 0xAB, sizeof buf);
    const char* outcome = "constructed";
    std::string what;
    try {
        T* p = make(buf);
        p->~T();
    } catch (const rt::Error& e) {
        outcome = "rt::Error";
        what = e.what();
    }
    bool past = false;
    for (size_t i = sizeof(T); i < sizeof buf; ++i) past |= buf[i] != 0xAB;
    std::printf("%s|%s|%s|%s\n", name, outcome, past ? "WROTE_PAST" : "clean", what.c_str());
}

int main()
{
    probe<rt::Camera>("Camera", [](void* b) { return new (b) rt::Camera(45.0f, 0.1f, 100.0f); });
    probe<rt::Renderer>("Renderer", [](void* b) { return new (b) rt::Renderer(rt::Renderer::Settings{}, false); });
    probe<rt::DenoisingRenderer>("DenoisingRenderer", [](void* b) { return new (b) rt::DenoisingRenderer(); });
    probe<rt::WhittedRenderer>("WhittedRenderer", [](void* b) {
        return new (b) rt::WhittedRenderer(nullptr, rt::WhittedRenderer::Settings{});
    });
    return 0;
}
'''

ABI_MSG = "compiled against a different include/rt header"


def _compile_and_run(tmp_path, include_dir):
    src = tmp_path / "caller.cpp"
    src.write_text(CALLER)
    exe = tmp_path / "caller"
    subprocess.run(["g++", "-std=c++20", "-O1", "-I", str(include_dir), str(src), "-o", str(exe), "-L", PKG, "-lrt_hip",
                    "-Wl,-rpath," + PKG, "-Wl,-rpath-link,/opt/rocm/lib"], check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "")))
    assert r.returncode == 0, r.stderr[-2000:]
    out = {}
    for line in r.stdout.splitlines():
        name, outcome, past, what = line.split("|", 3)
        out[name] = (outcome, past, what)
    return out


def _patched_include(tmp_path, edits):
    inc = tmp_path / "include"
    shutil.copytree(os.path.join(REPO, "include"), inc)
    for rel, old, new in edits:
        p = inc / rel
        s = p.read_text()
        assert old in s, (rel, old)
        p.write_text(s.replace(old, new, 1))
    return inc


pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="librt_hip.so not built")


def test_matching_header_passes_the_guard(tmp_path):
    out = _compile_and_run(tmp_path, os.path.join(REPO, "include"))
    assert out["Camera"][:2] == ("constructed", "clean")
    for name in ("Renderer", "DenoisingRenderer", "WhittedRenderer"):
        outcome, past, what = out[name]
        assert past == "clean"
        # past the guard: without a GPU the library fails later (rt_create / the scene), never on the layout
        assert ABI_MSG not in what, what


@pytest.mark.parametrize("cls,rel,anchor", [
    ("Renderer", "rt/Renderer.h", "    std::vector<rt::Entity*> entities;           // MC/Renderer.h:201\n"),
    ("Camera", "rt/Camera.h", "    mutable std::vector<rt::vec3> ray_directions;\n"),
    ("DenoisingRenderer", "rt/DenoisingRenderer.h", "    uint32_t frame = 0;\n"),
    ("WhittedRenderer", "rt/WhittedRenderer.h", "    uint32_t frame_accumulating = 1;\n"),
])
def test_grown_layout_fails_loudly(tmp_path, cls, rel, anchor):
    inc = _patched_include(tmp_path, [(rel, anchor, anchor + "    double rt_test_extra_member_[8] = {};\n")])
    outcome, past, what = _compile_and_run(tmp_path, inc)[cls]
    assert outcome == "rt::Error" and ABI_MSG in what, what
    assert past == "clean"


def test_settings_layout_fails_loudly(tmp_path):
    anchor = "        uint32_t band = 8;          // rows per band of the multi-GPU split\n"
    inc = _patched_include(tmp_path, [("rt/Renderer.h", anchor, anchor + "        uint64_t rt_test_extra_setting = 0;\n")])
    outcome, past, what = _compile_and_run(tmp_path, inc)["Renderer"]
    assert outcome == "rt::Error" and ABI_MSG in what and "Settings" in what, what
    assert past == "clean"


def test_abi_version_mismatch_fails_loudly(tmp_path):
    txt = open(os.path.join(REPO, "include", "rt", "Abi.h")).read()
    line = next(ln for ln in txt.splitlines() if ln.startswith("#define RT_CXX_ABI_VERSION "))
    inc = _patched_include(tmp_path, [("rt/Abi.h", line + "\n", "#define RT_CXX_ABI_VERSION 999\n")])
    out = _compile_and_run(tmp_path, inc)
    for name in ("Camera", "Renderer", "DenoisingRenderer", "WhittedRenderer"):
        outcome, past, what = out[name]
        assert outcome == "rt::Error" and "C++ ABI 999" in what, (name, what)
        assert past == "clean"


def test_unguarded_constructors_are_not_exported():
    """A front-end built before the guard calls constructors without the tag; the library no longer exports
    them, so such a binary stops at symbol lookup instead of corrupting its heap (the r05a crash)."""
    r = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True)
    syms = r.stdout
    for old in ("_ZN2rt8RendererC1ERKNS0_8SettingsEb", "_ZN2rt8RendererC1Ev", "_ZN2rt6CameraC1Efff",
                "_ZN2rt17DenoisingRendererC1Ev", "_ZN2rt15WhittedRendererC1EP8rt_sceneRKNS_15WhittedSettingsE"):
        assert old not in syms, old
    assert "_ZN2rt8AbiGuardC1ERKNS_6AbiTagEmm" in syms or "_ZN2rt8AbiGuardC2ERKNS_6AbiTagEmm" in syms
