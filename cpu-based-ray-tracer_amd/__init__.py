"""cpu-based-ray-tracer_amd -- MI355X-native Monte Carlo path tracer (host binding).

Thin ctypes binding of the C-ABI in include/rt_capi.h (librt_hip.so, built in-tree by `make`).
The product path is the HIP megakernel; there is no CPU fallback: if the shared library is
missing or a call fails, an exception is raised.

Load it by path (the directory name is not a Python identifier):
    import importlib.util, os
    spec = importlib.util.spec_from_file_location("rt_amd", "cpu-based-ray-tracer_amd/__init__.py")
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "librt_hip.so")

# include/rt_capi.h RT_API_VERSION: the struct layouts (rt_stats, rt_scene_info, ...) this binding declares
API_VERSION = 4

RT_OK = 0
RT_ERR_OVERFLOW = -6
RENDER_EXACT = 1
RENDER_COUNT = 2
RENDER_GLOBAL_SCENE = 4
RENDER_GLOBAL_STACK = 8
RENDER_WHITTED = 16

_lib = None


class RtError(RuntimeError):
    pass


class Camera(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("inv_projection", C.c_float * 16), ("inv_view", C.c_float * 16)]


class DeviceCfg(C.Structure):
    _fields_ = [("device", C.c_int32), ("stream", C.c_void_p), ("flags", C.c_uint32)]


class RenderParams(C.Structure):
    _fields_ = [("first_frame", C.c_uint32), ("n_frames", C.c_uint32), ("seed", C.c_uint64), ("rr", C.c_float), ("flags", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("last_kernel_ms", C.c_float), ("node_tests", C.c_uint64), ("tri_tests", C.c_uint64), ("rays", C.c_uint64),
                ("stack_overflows", C.c_uint64), ("samples", C.c_uint64), ("grid", C.c_uint32), ("block", C.c_uint32),
                ("stack_depth", C.c_uint32), ("wave_rounds", C.c_uint64), ("wave_steps", C.c_uint64),
                ("wave_tri_tests", C.c_uint64), ("wave_service", C.c_uint64), ("wave_fold", C.c_uint64),
                ("cycles_service", C.c_uint64), ("cycles_queue", C.c_uint64), ("cycles_trace", C.c_uint64),
                ("service_lanes", C.c_uint64), ("last_denoise_ms", C.c_float), ("n_chunks", C.c_uint32),
                ("n_passes", C.c_uint32), ("kernel", C.c_uint32), ("resampled", C.c_uint64), ("overflow_lost", C.c_uint64),
                ("kernel_reason", C.c_uint32), ("last_prepass_ms", C.c_float), ("last_main_ms", C.c_float)]

class GroupStats(C.Structure):
    _fields_ = [("last_ms", C.c_float), ("max_member_kernel_ms", C.c_float), ("gather", C.c_uint32), ("n", C.c_uint32)]


_DIAGNOSTIC = {"rt_debug_counters", "rt_read_accumulation", "rt_scene_walk_orders", "rt_scene_whitted_orders",
               "rt_scene_whitted_orders_half"}   # may be absent from an older A/B build

KERNEL_NAMES = {0: "pt_megakernel", 1: "pt_coherent_kernel", 2: "whitted_kernel", 3: "pt_coherent_kernel"}
# rt_stats.kernel_reason (include/rt_capi.h RT_KERNEL_REASON_*)
KERNEL_REASON_DEFAULT, KERNEL_REASON_TABLES_LDS, KERNEL_REASON_MATERIALS, KERNEL_REASON_MODE, KERNEL_REASON_KNOB = 0, 1, 2, 3, 4
KERNEL_REASON_TRIANGLES, KERNEL_REASON_SPHERES = 5, 6


class DenoiseParams(C.Structure):
    """rt_denoise_params: the Denoiser project's filter settings (DN/Denoiser.h:333-358, DN/Renderer.cpp:108-241)."""
    _fields_ = [("jbf_half_size", C.c_int32), ("temporal_half_size", C.c_int32), ("tolerance", C.c_float),
                ("current_frame_weighting", C.c_float), ("immediate_clamp", C.c_int32), ("sigma_position", C.c_float),
                ("sigma_color", C.c_float), ("sigma_normal", C.c_float), ("sigma_coplanarity", C.c_float)]


class WorldMaterial(C.Structure):
    """rt_world_material: a Whitted Style Ray Tracer entity's material (WH/Entity.h:49-55)."""
    _fields_ = [("nature", C.c_int32), ("refractive_index", C.c_float), ("phong_diffuse", C.c_float), ("phong_specular", C.c_float),
                ("specular_size_factor", C.c_float), ("diffuse_color", C.c_float * 3)]


REFLECTIVE, REFLECTIVE_REFRACTIVE, DIFFUSE_GLOSSY = 0, 1, 2


class SceneInfo(C.Structure):
    _fields_ = [("n_meshes", C.c_uint32), ("n_tris", C.c_uint32), ("n_nodes", C.c_uint32), ("n_light_tris", C.c_uint32),
                ("max_depth", C.c_uint32), ("light_mesh", C.c_int32), ("light_area", C.c_float), ("device_bytes", C.c_uint64),
                ("n_leaf_boxes", C.c_uint32), ("n_light_skip", C.c_uint32),
                ("split_root", C.c_uint32), ("split_end", C.c_uint32), ("n_split_leaves", C.c_uint32), ("n_split_boxes", C.c_uint32),
                ("n_spheres", C.c_uint32)]


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def lib():
    """Load librt_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RtError(f"{LIB_PATH} not built: run `make -C {PKG_DIR}` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, i32, fp = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32, C.POINTER(C.c_float)
    sig = {
        "rt_api_version": (i32, []),
        "rt_scene_create": (i32, [C.POINTER(vp)]),
        "rt_scene_destroy": (None, [vp]),
        "rt_scene_add_cornell_box": (i32, [vp]),
        "rt_scene_add_obj": (i32, [vp, C.c_char_p, fp, fp, C.POINTER(i32)]),
        "rt_scene_add_mesh": (i32, [vp, fp, u64, fp, fp, C.POINTER(i32)]),
        "rt_scene_add_sphere": (i32, [vp, fp, C.c_float, fp, fp, C.POINTER(i32)]),
        "rt_scene_add_whitted_mesh": (i32, [vp, fp, u64, C.c_float, fp, fp, C.c_float, C.POINTER(i32)]),
        "rt_scene_add_whitted_obj": (i32, [vp, C.c_char_p, C.c_float, fp, fp, C.c_float, C.POINTER(i32)]),
        "rt_scene_add_point_light": (i32, [vp, fp, fp]),
        "rt_scene_set_sky": (i32, [vp, fp]),
        "rt_scene_add_bvh_tracer_scene": (i32, [vp, C.c_char_p, C.c_char_p]),
        "rt_scene_build": (i32, [vp]),
        "rt_scene_get_info": (i32, [vp, C.POINTER(SceneInfo)]),
        "rt_scene_export": (i32, [vp, fp, C.POINTER(i32), fp, C.POINTER(i32)]),
        "rt_camera_default": (i32, [u32, u32, C.POINTER(Camera), fp, fp]),
        "rt_camera_look": (i32, [u32, u32, fp, fp, C.c_float, C.c_float, C.c_float, C.POINTER(Camera)]),
        "rt_create": (i32, [C.POINTER(vp), C.POINTER(DeviceCfg)]),
        "rt_destroy": (None, [vp]),
        "rt_last_error": (C.c_char_p, [vp]),
        "rt_upload_scene": (i32, [vp, vp]),
        "rt_upload_scene_gpu_bvh": (i32, [vp, vp, fp]),
        "rt_scene_lbvh_host": (i32, [vp, fp, fp]),
        "rt_scene_walk_orders": (i32, [vp, fp, C.POINTER(C.c_uint64)]),
        "rt_scene_whitted_orders": (i32, [vp, fp, C.POINTER(C.c_uint64)]),
        "rt_scene_whitted_orders_half": (i32, [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
        "rt_debug_scene_arrays": (i32, [vp, fp, u32, fp, u32]),
        "rt_resize": (i32, [vp, u32, u32, u32, u32, u32]),
        "rt_local_rows": (u32, [vp]),
        "rt_render": (i32, [vp, C.POINTER(Camera), C.POINTER(RenderParams), C.POINTER(u32), fp]),
        "rt_device_buffers": (i32, [vp, C.POINTER(vp), C.POINTER(vp)]),
        "rt_copy_rgba_to_device": (i32, [vp, vp]),
        "rt_read_accumulation": (i32, [vp, C.POINTER(C.c_float)]),
        "rt_reset_accumulation": (i32, [vp]),
        "rt_synchronize": (i32, [vp]),
        "rt_get_stats": (i32, [vp, C.POINTER(Stats)]),
        "rt_debug_counters": (i32, [vp, C.POINTER(C.c_uint64), u32]),
        "rt_trace": (i32, [vp, u64, fp, fp, C.POINTER(i32), C.POINTER(C.c_double)]),
        "rt_math_selftest": (i32, [vp, u64, fp, fp]),
        "rt_debug_primitives": (i32, [vp, u64, fp, C.POINTER(i32), C.POINTER(C.c_double), u64, fp, C.POINTER(i32)]),
        "rt_world_material_default": (None, [C.POINTER(WorldMaterial)]),
        "rt_scene_add_world_sphere": (i32, [vp, fp, C.c_float, C.POINTER(WorldMaterial), C.POINTER(i32)]),
        "rt_scene_add_world_mesh": (i32, [vp, fp, u32, C.POINTER(u32), u32, fp, C.POINTER(WorldMaterial), C.POINTER(i32)]),
        "rt_scene_add_two_spheres_scene": (i32, [vp]),
        "rt_world_trace": (i32, [vp, u64, fp, fp, C.POINTER(i32), C.POINTER(i32), fp]),
        "rt_camera_look_ex": (i32, [u32, u32, fp, fp, C.c_float, C.c_float, C.c_float, C.POINTER(Camera), fp, fp]),
        "rt_denoise_params_default": (None, [C.POINTER(DenoiseParams)]),
        "rt_render_denoised": (i32, [vp, C.POINTER(Camera), fp, fp, u32, u64, C.c_float, C.POINTER(DenoiseParams), C.POINTER(u32), fp]),
        "rt_denoise_restart": (i32, [vp]),
        "rt_get_gbuffer": (i32, [vp, fp, fp, fp, C.POINTER(i32), fp]),
        "rt_group_create": (i32, [C.POINTER(vp), C.POINTER(i32), u32]),
        "rt_group_destroy": (None, [vp]),
        "rt_group_last_error": (C.c_char_p, [vp]),
        "rt_group_size": (u32, [vp]),
        "rt_group_member": (vp, [vp, u32]),
        "rt_group_upload_scene": (i32, [vp, vp]),
        "rt_group_resize": (i32, [vp, u32, u32, u32]),
        "rt_group_render": (i32, [vp, C.POINTER(Camera), C.POINTER(RenderParams), C.POINTER(u32)]),
        "rt_group_frame_device": (i32, [vp, C.POINTER(vp)]),
        "rt_group_read_accumulation": (i32, [vp, fp]),
        "rt_group_reset_accumulation": (i32, [vp]),
        "rt_group_synchronize": (i32, [vp]),
        "rt_group_get_stats": (i32, [vp, C.POINTER(GroupStats)]),
    }
    for name, (res, args) in sig.items():
        if (name in _DIAGNOSTIC or name.startswith("rt_group_")) and not hasattr(L, name):
            continue   # diagnostics / multi-GPU entry points absent from an older A/B build (the product
                       # library exports all: test_capi_cpu.test_library_exports_every_declared_symbol)
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    v = L.rt_api_version()
    if v != API_VERSION:
        # a library built from another header revision would read / write structs of another size
        raise RtError(f"{LIB_PATH}: C-ABI version {v}, this binding needs {API_VERSION} (rebuild with `make -C {PKG_DIR}`)")
    _lib = L
    return L



class Scene:
    """Host scene: meshes + reference-identical BVH build (rt_scene_*)."""

    def __init__(self):
        self.h = C.c_void_p()
        self._check(lib().rt_scene_create(C.byref(self.h)), "rt_scene_create")

    @staticmethod
    def _check(st, what):
        if st != RT_OK:
            raise RtError(f"{what} failed with status {st}")

    @classmethod
    def cornell(cls, extra=()):
        s = cls()
        s._check(lib().rt_scene_add_cornell_box(s.h), "rt_scene_add_cornell_box")
        for (raw, albedo, emission) in extra:
            s.add_mesh(raw, albedo, emission)
        s.build()
        return s

    @classmethod
    def cornell_c5(cls, bunny_raw):
        """Configuration C5: the Cornell box plus the synthesized 79,488-triangle bunny (c5_mesh)."""
        return cls.cornell(extra=[(c5_mesh(bunny_raw), (0.7, 0.7, 0.7), (0.0, 0.0, 0.0))])

    def add_mesh(self, raw, albedo, emission):
        raw = np.ascontiguousarray(raw, np.float32).reshape(-1, 9)
        mid = C.c_int32()
        self._check(lib().rt_scene_add_mesh(self.h, _fp(raw), raw.shape[0], _fp(np.asarray(albedo, np.float32)),
                                            _fp(np.asarray(emission, np.float32)), C.byref(mid)), "rt_scene_add_mesh")
        return mid.value

    def add_sphere(self, center, radius, albedo, emission=(0.0, 0.0, 0.0)):
        """Renderer::Add(new Whitted::Sphere(center, radius, material)) (MC/Sphere.h:16-108): an entity of the
        path-traced scene; returns its entity index."""
        eid = C.c_int32()
        self._check(lib().rt_scene_add_sphere(self.h, _fp(np.asarray(center, np.float32)), float(radius),
                                              _fp(np.asarray(albedo, np.float32)), _fp(np.asarray(emission, np.float32)),
                                              C.byref(eid)), "rt_scene_add_sphere")
        return eid.value

    def add_obj(self, path, albedo, emission):
        mid = C.c_int32()
        self._check(lib().rt_scene_add_obj(self.h, path.encode(), _fp(np.asarray(albedo, np.float32)),
                                           _fp(np.asarray(emission, np.float32)), C.byref(mid)), "rt_scene_add_obj")
        return mid.value

    # ---- Whitted-style scenes (the reference's BVH Ray Tracer, BV/Renderer.cpp:26-43)
    def add_whitted_mesh(self, raw, scale, offset, diffuse=(0.5, 0.5, 0.5), phong_diffuse=0.6):
        raw = np.ascontiguousarray(raw, np.float32).reshape(-1, 9)
        off = None if offset is None else _fp(np.asarray(offset, np.float32))
        mid = C.c_int32()
        self._check(lib().rt_scene_add_whitted_mesh(self.h, _fp(raw), raw.shape[0], float(scale), off, _fp(np.asarray(diffuse, np.float32)),
                                                    float(phong_diffuse), C.byref(mid)), "rt_scene_add_whitted_mesh")
        return mid.value

    def add_point_light(self, position, radiance=(1.0, 1.0, 1.0)):
        self._check(lib().rt_scene_add_point_light(self.h, _fp(np.asarray(position, np.float32)), _fp(np.asarray(radiance, np.float32))),
                    "rt_scene_add_point_light")

    def set_sky(self, rgb):
        self._check(lib().rt_scene_set_sky(self.h, _fp(np.asarray(rgb, np.float32))), "rt_scene_set_sky")

    @classmethod
    def bvh_tracer(cls, bunny_raw, teapot_raw):
        """The BVH Ray Tracer's Renderer::Renderer() scene from raw objl positions (BV/Renderer.cpp:26-43)."""
        s = cls()
        s.add_whitted_mesh(bunny_raw, 2.0, (-1.0, 6.1, 0.0))
        s.add_whitted_mesh(teapot_raw, 1.0, (-1.0, 3.0, 0.0))
        s.add_point_light((-20.0, 70.0, 20.0))
        s.add_point_light((20.0, 70.0, 20.0))
        return s.build()

    # ---- the Whitted Style Ray Tracer's world (config C1, WH/Renderer.cpp:27-49)
    @staticmethod
    def world_material(nature=DIFFUSE_GLOSSY, **kw):
        m = WorldMaterial()
        lib().rt_world_material_default(C.byref(m))
        m.nature = nature
        for k, v in kw.items():
            if k == "diffuse_color":
                m.diffuse_color[:] = [float(c) for c in v]
            else:
                setattr(m, k, float(v))
        return m

    def add_world_sphere(self, center, radius, material=None):
        mid = C.c_int32()
        self._check(lib().rt_scene_add_world_sphere(self.h, _fp(np.asarray(center, np.float32)), float(radius),
                                                    C.byref(material) if material is not None else None, C.byref(mid)),
                    "rt_scene_add_world_sphere")
        return mid.value

    def add_world_mesh(self, vertices, indices, uv, material=None):
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 3)
        i = np.ascontiguousarray(indices, np.uint32).reshape(-1, 3)
        t = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
        mid = C.c_int32()
        self._check(lib().rt_scene_add_world_mesh(self.h, _fp(v), v.shape[0], i.ctypes.data_as(C.POINTER(C.c_uint32)), i.shape[0], _fp(t),
                                                  C.byref(material) if material is not None else None, C.byref(mid)),
                    "rt_scene_add_world_mesh")
        return mid.value

    @classmethod
    def two_spheres(cls):
        """The Whitted Style Ray Tracer's Renderer::Renderer() world (WH/Renderer.cpp:27-49)."""
        s = cls()
        s._check(lib().rt_scene_add_two_spheres_scene(s.h), "rt_scene_add_two_spheres_scene")
        return s.build()

    def build(self):
        self._check(lib().rt_scene_build(self.h), "rt_scene_build")
        return self

    def info(self):
        i = SceneInfo()
        self._check(lib().rt_scene_get_info(self.h, C.byref(i)), "rt_scene_get_info")
        return i

    def lbvh_host(self):
        """The device build's tree, built on the host (rt_scene_lbvh_host): nodes (2n-1, 8) and triangle
        records (n, 16) as float32 arrays in the traversal layout."""
        n = self.info().n_tris
        nodes = np.zeros((2 * n - 1, 8), np.float32); tris = np.zeros((n, 16), np.float32)
        self._check(lib().rt_scene_lbvh_host(self.h, _fp(nodes), _fp(tris)), "rt_scene_lbvh_host")
        return nodes, tris

    def walk_orders(self, whitted=False):
        """The split subtree's 8 near-first pre-orders (rt_scene_walk_orders): (8, split_end - split_root, 8)
        float32 in the traversal layout, or None when the scene has no split; whitted=True: a Whitted scene's
        whole tree (rt_scene_whitted_orders, (8, n_nodes, 8))."""
        name = "rt_scene_whitted_orders" if whitted else "rt_scene_walk_orders"
        fn = getattr(lib(), name)
        n = C.c_uint64(0)
        self._check(fn(self.h, None, C.byref(n)), name)
        if n.value == 0:
            return None
        out = np.zeros(n.value, np.float32)
        self._check(fn(self.h, _fp(out), C.byref(n)), name)
        return out.reshape(8, -1, 8)

    def whitted_orders_half(self):
        """The Whitted orderings in 16-byte half-plane nodes (rt_scene_whitted_orders_half): (8, n_nodes, 4) uint32,
        or None."""
        n = C.c_uint64(0)
        self._check(lib().rt_scene_whitted_orders_half(self.h, None, C.byref(n)), "rt_scene_whitted_orders_half")
        if n.value == 0:
            return None
        out = np.zeros(n.value, np.uint32)
        self._check(lib().rt_scene_whitted_orders_half(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(n)),
                    "rt_scene_whitted_orders_half")
        return out.reshape(8, -1, 4)

    def export(self):
        i = self.info()
        nf = np.zeros((i.n_nodes, 7), np.float32); ni = np.zeros((i.n_nodes, 5), np.int32)
        tf = np.zeros((i.n_tris, 13), np.float32); ti = np.zeros((i.n_tris, 2), np.int32)
        self._check(lib().rt_scene_export(self.h, _fp(nf), ni.ctypes.data_as(C.POINTER(C.c_int32)), _fp(tf),
                                          ti.ctypes.data_as(C.POINTER(C.c_int32))), "rt_scene_export")
        return nf, ni, tf, ti

    def __del__(self):
        try:
            if self.h:
                lib().rt_scene_destroy(self.h)
                self.h = C.c_void_p()
        except Exception:
            pass


def subdivide_midpoint(raw, levels=1):
    """1:4 midpoint subdivision of a de-indexed triangle list (n, 9) float32, `levels` times.

    Each (a, b, c) becomes (a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca) with the float32
    midpoints m = (p + q) * 0.5 (commutative, so triangles sharing an edge share its midpoint and the
    mesh stays watertight); orientation is kept.  Used to synthesize the ~80k-triangle mesh of the C5
    configuration (SURVEY.md section 7 'Config 5', 8(d))."""
    t = np.ascontiguousarray(raw, np.float32).reshape(-1, 3, 3)
    half = np.float32(0.5)
    for _ in range(levels):
        a, b, c = t[:, 0], t[:, 1], t[:, 2]
        ab, bc, ca = (a + b) * half, (b + c) * half, (c + a) * half
        t = np.stack([np.stack([a, ab, ca], 1), np.stack([ab, b, bc], 1), np.stack([ca, bc, c], 1), np.stack([ab, bc, ca], 1)], 1)
        t = np.ascontiguousarray(t.reshape(-1, 3, 3), np.float32)
    return t.reshape(-1, 9)


def fit_mesh(raw, height, base_center, obj_units=100.0):
    """Uniformly scale a triangle list to `height` with its bounding-box bottom centre at `base_center`
    (world units), returned in OBJ units (world x `obj_units`) so that the reference's fixed 0.01 mesh
    scale (MC/TriangleMesh.h:150,170) restores world units.  float32 throughout, fixed operation order."""
    v = np.ascontiguousarray(raw, np.float32).reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    s = np.float32(height) / (hi[1] - lo[1])
    anchor = np.array([(lo[0] + hi[0]) * np.float32(0.5), lo[1], (lo[2] + hi[2]) * np.float32(0.5)], np.float32)
    w = (v - anchor) * s + np.asarray(base_center, np.float32)
    return np.ascontiguousarray((w * np.float32(obj_units)).reshape(-1, 9), np.float32)


def c5_mesh(bunny_raw):
    """The C5 asset: the Stanford bunny (raw objl positions) subdivided 1:4 twice
    (4,968 -> 79,488 triangles), 1.5 units tall, standing on the floor (y = 0) at x = 4.2, z = 1.2,
    clear of both boxes; white albedo 0.7 (added to the Cornell scene via Add + GenerateBVH,
    MC/Renderer.h:78-86)."""
    return fit_mesh(subdivide_midpoint(bunny_raw, 2), 1.5, (4.2, 0.0, 1.2))


def write_obj(path, raw):
    """De-indexed triangle list -> OBJ text whose values round-trip exactly through std::stof."""
    v = np.ascontiguousarray(raw, np.float32).reshape(-1, 3)
    with open(path, "w") as f:
        f.write("".join("v %.9g %.9g %.9g\n" % (x, y, z) for x, y, z in v.astype(np.float64)))
        f.write("".join("f %d %d %d\n" % (3 * i + 1, 3 * i + 2, 3 * i + 3) for i in range(v.shape[0] // 3)))


def camera_look(W, H, position, forward, vfov=35.0, near=0.1, far=100.0):
    cam = Camera()
    st = lib().rt_camera_look(W, H, _fp(np.asarray(position, np.float32)), _fp(np.asarray(forward, np.float32)), vfov, near, far,
                              C.byref(cam))
    if st != RT_OK:
        raise RtError(f"rt_camera_look failed {st}")
    return cam


def camera_look_ex(W, H, position, forward, vfov=35.0, near=0.1, far=100.0):
    """camera + its (non-inverted) projection and view matrices (column-major 16 floats each)."""
    cam = Camera()
    proj = np.zeros(16, np.float32); view = np.zeros(16, np.float32)
    st = lib().rt_camera_look_ex(W, H, _fp(np.asarray(position, np.float32)), _fp(np.asarray(forward, np.float32)), vfov, near, far,
                                 C.byref(cam), _fp(proj), _fp(view))
    if st != RT_OK:
        raise RtError(f"rt_camera_look_ex failed {st}")
    return cam, proj, view


DEFAULT_CAMERA_POSITION = (2.81432, 4.20749, -9.11751)     # MC/Camera.h:19-21, DN/Camera.h:19-20
DEFAULT_CAMERA_FORWARD = (0.00209191, -0.148299, 0.988941)


def denoise_params(**kw):
    """rt_denoise_params with the DN/Denoiser.h defaults, overridden by keyword."""
    p = DenoiseParams()
    lib().rt_denoise_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def camera_two_spheres(W, H):
    """The Whitted Style Ray Tracer's Camera{35, 0.1, 100} at (0, 0, 6) looking down -z (WH/Camera.h:17-19, WH/mainloop.cpp:23)."""
    return camera_look(W, H, (0.0, 0.0, 6.0), (0.0, 0.0, -1.0))


def camera_bvh_tracer(W, H):
    """The BVH Ray Tracer's Camera{35, 0.1, 100} at (-1, 5, 10) looking down -z (BV/Camera.h:19-20, BV/mainloop.cpp:22)."""
    return camera_look(W, H, (-1.0, 5.0, 10.0), (0.0, 0.0, -1.0))


def camera_default(W, H):
    cam = Camera()
    proj = np.zeros(16, np.float32); view = np.zeros(16, np.float32)
    st = lib().rt_camera_default(W, H, C.byref(cam), _fp(proj), _fp(view))
    if st != RT_OK:
        raise RtError(f"rt_camera_default failed {st}")
    return cam, proj, view


class Group:
    """Several GPUs rendering one frame (rt_group_*): member i renders the row bands b with b mod n == i on
    devices[i]; the RGBA8 band sets are gathered to member 0 (RCCL for distinct devices, copies otherwise)."""

    def __init__(self, devices):
        self.h = C.c_void_p()
        devs = (C.c_int32 * len(devices))(*devices)
        st = lib().rt_group_create(C.byref(self.h), devs, len(devices))
        if st != RT_OK:
            raise RtError(f"rt_group_create failed with status {st}")
        self.n = len(devices)
        self.W = self.H = 0

    def _check(self, st, what):
        if st != RT_OK:
            msg = lib().rt_group_last_error(self.h)
            raise RtError(f"{what} failed ({st}): {msg.decode() if msg else ''}")

    def upload(self, scene):
        self._check(lib().rt_group_upload_scene(self.h, scene.h), "rt_group_upload_scene")

    def resize(self, W, H, band=8):
        self._check(lib().rt_group_resize(self.h, W, H, band), "rt_group_resize")
        self.W, self.H = W, H

    def render(self, cam, n_frames, first_frame=1, seed=0, rr=0.8, exact=True, fetch=True):
        p = RenderParams(first_frame, n_frames, seed, rr, RENDER_EXACT if exact else 0)
        if fetch:
            rgba = np.zeros((self.H, self.W), np.uint32)
            self._check(lib().rt_group_render(self.h, C.byref(cam), C.byref(p), rgba.ctypes.data_as(C.POINTER(C.c_uint32))), "rt_group_render")
            return rgba
        self._check(lib().rt_group_render(self.h, C.byref(cam), C.byref(p), None), "rt_group_render")
        return None

    def accumulation(self):
        acc = np.zeros((self.H, self.W, 4), np.float32)
        self._check(lib().rt_group_read_accumulation(self.h, _fp(acc)), "rt_group_read_accumulation")
        return acc

    def frame_device(self):
        d = C.c_void_p()
        self._check(lib().rt_group_frame_device(self.h, C.byref(d)), "rt_group_frame_device")
        return d.value

    def sync(self):
        self._check(lib().rt_group_synchronize(self.h), "rt_group_synchronize")

    def stats(self):
        s = GroupStats()
        self._check(lib().rt_group_get_stats(self.h, C.byref(s)), "rt_group_get_stats")
        return s

    def member_stats(self, i):
        s = Stats()
        m = lib().rt_group_member(self.h, i)
        if lib().rt_get_stats(m, C.byref(s)) != RT_OK:
            raise RtError("rt_get_stats failed")
        return s

    def close(self):
        if self.h:
            lib().rt_group_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One GPU: device buffers, stream, megakernel launches (rt_create .. rt_destroy)."""

    def __init__(self, device=0, stream=None):
        self.h = C.c_void_p()
        cfg = DeviceCfg(device, C.c_void_p(stream) if stream else None, 0)
        st = lib().rt_create(C.byref(self.h), C.byref(cfg))
        if st != RT_OK:
            raise RtError(f"rt_create failed with status {st} (is a GPU visible?)")
        self.W = self.H = 0
        self.local_rows = 0

    def _check(self, st, what):
        if st != RT_OK:
            msg = lib().rt_last_error(self.h)
            raise RtError(f"{what} failed ({st}): {msg.decode() if msg else ''}")

    def upload(self, scene):
        self._check(lib().rt_upload_scene(self.h, scene.h), "rt_upload_scene")

    def upload_gpu_bvh(self, scene):
        """rt_upload_scene_gpu_bvh: the BVH built on the device (non-parity fast path); returns the build ms."""
        ms = C.c_float(0.0)
        self._check(lib().rt_upload_scene_gpu_bvh(self.h, scene.h, C.byref(ms)), "rt_upload_scene_gpu_bvh")
        return ms.value

    def debug_scene_arrays(self, n_nodes, n_tris):
        """The device's node (n_nodes, 8) and triangle (n_tris, 16) arrays (rt_debug_scene_arrays)."""
        nodes = np.zeros((n_nodes, 8), np.float32); tris = np.zeros((n_tris, 16), np.float32)
        self._check(lib().rt_debug_scene_arrays(self.h, _fp(nodes), nodes.size, _fp(tris), tris.size), "rt_debug_scene_arrays")
        return nodes, tris

    def resize(self, W, H, band=8, rank=0, nranks=1):
        self._check(lib().rt_resize(self.h, W, H, band, rank, nranks), "rt_resize")
        self.W, self.H = W, H
        self.band, self.rank, self.nranks = band, rank, nranks
        self.local_rows = lib().rt_local_rows(self.h)

    def render(self, cam, n_frames, first_frame=1, seed=0, rr=0.8, exact=True, count=False, fetch=True, global_scene=False,
               global_stack=False, whitted=False):
        flags = (RENDER_EXACT if exact else 0) | (RENDER_COUNT if count else 0) | (RENDER_GLOBAL_SCENE if global_scene else 0)
        flags |= (RENDER_GLOBAL_STACK if global_stack else 0) | (RENDER_WHITTED if whitted else 0)
        p = RenderParams(first_frame, n_frames, seed, rr, flags)
        if fetch:
            rgba = np.zeros((self.local_rows, self.W), np.uint32)
            acc = np.zeros((self.local_rows, self.W, 4), np.float32)
            self._check(lib().rt_render(self.h, C.byref(cam), C.byref(p), rgba.ctypes.data_as(C.POINTER(C.c_uint32)), _fp(acc)), "rt_render")
            return rgba, acc
        self._check(lib().rt_render(self.h, C.byref(cam), C.byref(p), None, None), "rt_render")
        return None

    def reset_accumulation(self):
        """Renderer::Reaccumulate (MC/Renderer.h:57-60): zero the accumulation buffer."""
        self._check(lib().rt_reset_accumulation(self.h), "rt_reset_accumulation")

    def stats(self):
        s = Stats()
        self._check(lib().rt_get_stats(self.h, C.byref(s)), "rt_get_stats")
        return s

    def debug_counters(self, n=32):
        """Raw device counters of the last render (diagnostics; rt_debug_counters)."""
        out = (C.c_uint64 * n)()
        self._check(lib().rt_debug_counters(self.h, out, n), "rt_debug_counters")
        return list(out)

    def sync(self):
        self._check(lib().rt_synchronize(self.h), "rt_synchronize")

    def device_buffers(self):
        a, r = C.c_void_p(), C.c_void_p()
        self._check(lib().rt_device_buffers(self.h, C.byref(a), C.byref(r)), "rt_device_buffers")
        return a.value, r.value

    def accumulation(self):
        """The local float4 accumulation after a synchronisation (rt_read_accumulation; RtError on an EXACT
        overflow of the renders since the last check)."""
        a = np.zeros((self.local_rows, self.W, 4), np.float32)
        self._check(lib().rt_read_accumulation(self.h, _fp(a)), "rt_read_accumulation")
        return a

    def copy_rgba_to_device(self, dst_ptr):
        self._check(lib().rt_copy_rgba_to_device(self.h, C.c_void_p(dst_ptr)), "rt_copy_rgba_to_device")

    def trace(self, org, dirs):
        org = np.ascontiguousarray(org, np.float32); dirs = np.ascontiguousarray(dirs, np.float32)
        n = org.shape[0]
        tri = np.zeros(n, np.int32); t = np.zeros(n, np.float64)
        self._check(lib().rt_trace(self.h, n, _fp(org), _fp(dirs), tri.ctypes.data_as(C.POINTER(C.c_int32)),
                                   t.ctypes.data_as(C.POINTER(C.c_double))), "rt_trace")
        return tri, t

    def render_denoised(self, cam, proj, view, frame, params, seed=0, rr=0.8, fetch=True):
        """One frame of the Denoiser project's Renderer::Render (G-buffer pass, JBF, temporal, pack)."""
        proj = np.ascontiguousarray(proj, np.float32); view = np.ascontiguousarray(view, np.float32)
        if fetch:
            rgba = np.zeros((self.H, self.W), np.uint32)
            col = np.zeros((self.H, self.W, 4), np.float32)
            self._check(lib().rt_render_denoised(self.h, C.byref(cam), _fp(proj), _fp(view), frame, seed, rr, C.byref(params),
                                                 rgba.ctypes.data_as(C.POINTER(C.c_uint32)), _fp(col)), "rt_render_denoised")
            return rgba, col
        self._check(lib().rt_render_denoised(self.h, C.byref(cam), _fp(proj), _fp(view), frame, seed, rr, C.byref(params), None, None),
                    "rt_render_denoised")
        return None

    def denoise_restart(self):
        self._check(lib().rt_denoise_restart(self.h), "rt_denoise_restart")

    def gbuffer(self):
        n = (self.H, self.W)
        col = np.zeros(n + (4,), np.float32); pos = np.zeros(n + (4,), np.float32); nrm = np.zeros(n + (4,), np.float32)
        prim = np.zeros(n, np.int32); spa = np.zeros(n + (4,), np.float32)
        self._check(lib().rt_get_gbuffer(self.h, _fp(col), _fp(pos), _fp(nrm), prim.ctypes.data_as(C.POINTER(C.c_int32)), _fp(spa)),
                    "rt_get_gbuffer")
        return dict(color=col, position=pos, normal=nrm, prim=prim, spatial=spa)

    def world_trace(self, org, dirs):
        org = np.ascontiguousarray(org, np.float32); dirs = np.ascontiguousarray(dirs, np.float32)
        n = org.shape[0]
        ent = np.zeros(n, np.int32); tri = np.zeros(n, np.int32); tb = np.zeros((n, 3), np.float32)
        self._check(lib().rt_world_trace(self.h, n, _fp(org), _fp(dirs), ent.ctypes.data_as(C.POINTER(C.c_int32)),
                                         tri.ctypes.data_as(C.POINTER(C.c_int32)), _fp(tb)), "rt_world_trace")
        return ent, tri, tb

    def debug_primitives(self, mt_cases, box_cases):
        """The kernels' Moller-Trumbore (float pre-screen + double test) and the three slab-test forms on the
        reference's fixture layouts (rt_debug_primitives): (mt_hit, mt_t, box_hit[n, 3])."""
        mt = np.ascontiguousarray(mt_cases, np.float32).reshape(-1, 15)
        bx = np.ascontiguousarray(box_cases, np.float32).reshape(-1, 12)
        mh = np.zeros(mt.shape[0], np.int32); mtt = np.zeros(mt.shape[0], np.float64); bh = np.zeros((bx.shape[0], 3), np.int32)
        self._check(lib().rt_debug_primitives(self.h, mt.shape[0], _fp(mt), mh.ctypes.data_as(C.POINTER(C.c_int32)),
                                              mtt.ctypes.data_as(C.POINTER(C.c_double)), bx.shape[0], _fp(bx),
                                              bh.ctypes.data_as(C.POINTER(C.c_int32))), "rt_debug_primitives")
        return mh, mtt, bh

    def math_selftest(self, x):
        x = np.ascontiguousarray(x, np.float32)
        out = np.zeros((x.shape[0], 9), np.float32)
        self._check(lib().rt_math_selftest(self.h, x.shape[0], _fp(x), _fp(out)), "rt_math_selftest")
        return out

    def local_to_global_rows(self):
        """global row index of every local row (row bands dealt round-robin)."""
        rows = []
        b = self.rank
        while b * self.band < self.H:
            rows.extend(range(b * self.band, min((b + 1) * self.band, self.H)))
            b += self.nranks
        return np.array(rows, np.int64)

    def close(self):
        if self.h:
            lib().rt_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
