"""ctypes binding of oracle/liboracle.so -- the CPU restatement used as the checker.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
GOLDEN = os.path.join(REPO, "tests", "golden")

_lib = None


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("samples", "rays", "node_tests", "tri_tests", "draws", "shading_calls", "max_depth")]


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(ORACLE_DIR, f) for f in ("rt_oracle.cpp", "rt_oracle.h", "philox.h")]
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(s) for s in srcs):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"])
        L = C.CDLL(LIB)
        L.or_scene_new.restype = C.c_void_p
        L.or_scene_free.argtypes = [C.c_void_p]
        L.or_scene_add_mesh.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.or_scene_build.argtypes = [C.c_void_p]
        L.or_scene_num_tris.argtypes = [C.c_void_p]
        L.or_scene_num_nodes.argtypes = [C.c_void_p]
        L.or_scene_dump.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int32), C.POINTER(C.c_float), C.POINTER(C.c_int32)]
        L.or_trace.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_int32),
                               C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_double), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.or_mt.argtypes = [C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_int32), C.POINTER(C.c_double)]
        L.or_aabb.argtypes = [C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_int32)]
        L.or_camera_matrices.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_float)]
        L.or_camera_dirs.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.POINTER(C.c_float)]
        L.or_render.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_float, C.c_int,
                                C.c_uint32, C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.POINTER(Counters)]
        L.or_rng_u32.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        L.or_rng_u32.restype = C.c_uint32
        L.or_rng_float.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        L.or_rng_float.restype = C.c_float
        L.or_obj_positions.argtypes = [C.c_char_p, C.POINTER(C.c_float), C.c_int64]
        L.or_obj_positions.restype = C.c_int64
        L.or_light_sample.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_uint32), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                      C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.or_material_sample.argtypes = [C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.POINTER(C.c_float),
                                         C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.or_trig.argtypes = [C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.or_exp_acos.argtypes = [C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        _lib = L
    return _lib


def cornell_meshes():
    """Raw (pre-scale, de-indexed) Cornell positions + materials, from the committed fixture."""
    z = np.load(os.path.join(GOLDEN, "cornell_scene.npz"))
    names = ["floor", "shortbox", "tallbox", "left", "right", "light"]
    out = []
    for i, n in enumerate(names):
        m = int(z["mesh_material"][i])
        out.append((n, np.ascontiguousarray(z[f"raw_{n}"], np.float32), z["albedo"][m].astype(np.float32), z["emission"][m].astype(np.float32)))
    return out


class Scene:
    def __init__(self, meshes=None):
        L = lib()
        self.h = C.c_void_p(L.or_scene_new())
        for (_, raw, alb, em) in (meshes if meshes is not None else cornell_meshes()):
            raw = np.ascontiguousarray(raw, np.float32)
            L.or_scene_add_mesh(self.h, _p(raw, C.c_float), raw.shape[0], _p(np.ascontiguousarray(alb, np.float32), C.c_float),
                                _p(np.ascontiguousarray(em, np.float32), C.c_float))
        assert L.or_scene_build(self.h) == 0

    def __del__(self):
        try:
            lib().or_scene_free(self.h)
        except Exception:
            pass

    def dump(self):
        L = lib()
        nt = L.or_scene_num_tris(self.h)
        nn = L.or_scene_num_nodes(self.h)
        nf = np.zeros((nn, 7), np.float32); ni = np.zeros((nn, 5), np.int32)
        tf = np.zeros((nt, 13), np.float32); ti = np.zeros((nt, 2), np.int32)
        k = L.or_scene_dump(self.h, _p(nf, C.c_float), _p(ni, C.c_int32), _p(tf, C.c_float), _p(ti, C.c_int32))
        assert k == nn
        return nf, ni, tf, ti

    def trace(self, org, dirs):
        L = lib()
        org = np.ascontiguousarray(org, np.float32); dirs = np.ascontiguousarray(dirs, np.float32)
        n = org.shape[0]
        hit = np.zeros(n, np.int32); tri = np.zeros(n, np.int32); mat = np.zeros(n, np.int32)
        t = np.zeros(n, np.float64); loc = np.zeros((n, 3), np.float32); nrm = np.zeros((n, 3), np.float32)
        L.or_trace(self.h, n, _p(org, C.c_float), _p(dirs, C.c_float), _p(hit, C.c_int32), _p(tri, C.c_int32), _p(mat, C.c_int32),
                   _p(t, C.c_double), _p(loc, C.c_float), _p(nrm, C.c_float))
        return dict(hit=hit, tri=tri, mat=mat, t=t, loc=loc, n=nrm)

    def light_sample(self, u):
        u = np.ascontiguousarray(u, np.uint32)
        n = u.shape[0]
        loc = np.zeros((n, 3), np.float32); nrm = np.zeros((n, 3), np.float32); em = np.zeros((n, 3), np.float32); pdf = np.zeros(n, np.float32)
        lib().or_light_sample(self.h, n, _p(u, C.c_uint32), _p(loc, C.c_float), _p(nrm, C.c_float), _p(em, C.c_float), _p(pdf, C.c_float))
        return loc, nrm, em, pdf

    def render(self, W, H, spp, seed=0, rr=0.8, threads=0, first_frame=1, accum=None, rows=(0, 0)):
        L = lib()
        if accum is None:
            accum = np.zeros((H, W, 4), np.float32)
        rgba = np.zeros((H, W), np.uint32)
        cnt = Counters()
        rc = L.or_render(self.h, W, H, first_frame, spp, seed, rr, threads, rows[0], rows[1], _p(accum, C.c_float), _p(rgba, C.c_uint32), C.byref(cnt))
        assert rc == 0
        return accum, rgba, cnt


def mt(cases):
    cases = np.ascontiguousarray(cases, np.float32)
    n = cases.shape[0]
    hit = np.zeros(n, np.int32); t = np.zeros(n, np.float64)
    lib().or_mt(n, _p(cases, C.c_float), _p(hit, C.c_int32), _p(t, C.c_double))
    return hit, t


def aabb(cases):
    cases = np.ascontiguousarray(cases, np.float32)
    n = cases.shape[0]
    hit = np.zeros(n, np.int32)
    lib().or_aabb(n, _p(cases, C.c_float), _p(hit, C.c_int32))
    return hit


def camera_matrices(W, H):
    m = np.zeros(64, np.float32)
    lib().or_camera_matrices(W, H, _p(m, C.c_float))
    return m.reshape(4, 4, 4)


def camera_dirs(W, H, frame, seed):
    d = np.zeros((H * W, 3), np.float32)
    lib().or_camera_dirs(W, H, frame, seed, _p(d, C.c_float))
    return d


def rng_u32(seed, pixel, frame, dim):
    return lib().or_rng_u32(seed, pixel, frame, dim)


def material_sample(n, wi, u, albedo):
    n = np.ascontiguousarray(n, np.float32); wi = np.ascontiguousarray(wi, np.float32)
    u = np.ascontiguousarray(u, np.uint32); albedo = np.ascontiguousarray(albedo, np.float32)
    k = n.shape[0]
    raw = np.zeros((k, 3), np.float32); d = np.zeros((k, 3), np.float32); b = np.zeros((k, 3), np.float32); pdf = np.zeros(k, np.float32)
    lib().or_material_sample(k, _p(n, C.c_float), _p(wi, C.c_float), _p(u, C.c_uint32), _p(albedo, C.c_float),
                             _p(raw, C.c_float), _p(d, C.c_float), _p(b, C.c_float), _p(pdf, C.c_float))
    return raw, d, b, pdf


def libm_trig(x):
    x = np.ascontiguousarray(x, np.float32)
    c = np.zeros_like(x); s = np.zeros_like(x)
    lib().or_trig(x.shape[0], _p(x, C.c_float), _p(c, C.c_float), _p(s, C.c_float))
    return c, s


def libm_exp_acos(x):
    """the host libm's expf and acosf (glibc: what the reference's denoiser calls)"""
    x = np.ascontiguousarray(x, np.float32)
    e = np.zeros_like(x); a = np.zeros_like(x)
    lib().or_exp_acos(x.shape[0], _p(x, C.c_float), _p(e, C.c_float), _p(a, C.c_float))
    return e, a
