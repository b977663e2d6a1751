/* rt_capi.h -- C-ABI of the MI355X path tracer (librt_hip.so).
 *
 * The drop-in boundary: the reference has no FFI; its hot path is the C++ call
 * Renderer::Render(const Camera&) (Monte Carlo Path Tracer/8599RayTracerGUI/src/Renderer.cpp:91-122)
 * driven by the Walnut layer (mainloop.cpp:139-148).  The C++20 host classes in include/rt/
 * (Renderer, Camera) keep that API and call the entry points below; other hosts (ctypes, cgo,
 * JNI) bind them directly.  Plain pointers and sizes only; no HIP/torch types;
 * integer status codes, no exceptions across the ABI; message via rt_last_error().
 *
 * Reference anchors, per entry point ("MC/" = Monte Carlo Path Tracer/8599RayTracerGUI/src/):
 *   rt_scene_add_obj / rt_scene_add_mesh  Whitted::TriangleMesh ctor + Renderer::Add        MC/TriangleMesh.h:148-186, MC/Renderer.h:78-81
 *   rt_scene_add_cornell_box              Renderer::Renderer() scene                        MC/Renderer.cpp:26-57
 *   rt_scene_build                        Renderer::GenerateBVH / BVH::build_BVH            MC/Renderer.h:83-86, MC/BVH.h:131-214
 *   rt_camera_default                     Camera(35,0.1,100) + ResizeViewport matrices      MC/Camera.cpp:87-112, MC/mainloop.cpp:22
 *   rt_resize                             Renderer::ResizeViewport                          MC/Renderer.cpp:59-89
 *   rt_render                             Renderer::Render x n_frames (+ RayGen_Shader)     MC/Renderer.cpp:91-134
 *   rt_reset_accumulation                 Renderer::Reaccumulate                            MC/Renderer.h:57-60
 *   rt_trace                              Renderer::ray_BVH_intersection_record             MC/Renderer.h:88-91
 *   rt_render + RT_RENDER_WHITTED         BVH Ray Tracer Renderer::Render / cast_Whitted_ray   BV/Renderer.cpp:69-233
 *   rt_scene_add_bvh_tracer_scene         BVH Ray Tracer Renderer::Renderer()                  BV/Renderer.cpp:26-43
 *   rt_render_denoised                    Denoiser project Renderer::Render (G-buffer, JBF,    DN/Renderer.cpp:101-311,
 *                                         temporal filter)                                   DN/Denoiser.h:133-328
 *   rt_scene_add_world_sphere / _mesh     Whitted Style Ray Tracer Sphere / TriangleMesh + World::Add
 *                                         (WH/Sphere.h:16-75, WH/TriangleMesh.h:47-155, WH/World.h:37-45)
 *   rt_scene_add_two_spheres_scene        Whitted Style Ray Tracer Renderer::Renderer()       WH/Renderer.cpp:27-49
 *   rt_render + RT_RENDER_WHITTED on a    Whitted Style Ray Tracer RayGen_Shader /           WH/Renderer.cpp:82-125,
 *     world scene                         cast_Whitted_ray                                   WH/Renderer.h:184-310
 */
#ifndef RT_CAPI_H
#define RT_CAPI_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 4): rt_stats grew last_prepass_ms / last_main_ms, rt_scene_info the light-skip and split fields,
 * rt_read_accumulation was added; a host built against another version must not pass its structs
 * 4 (round 6): rt_scene_add_sphere, rt_scene_info.n_spheres, RT_KERNEL_REASON_SPHERES */
#define RT_API_VERSION 4

typedef int32_t rt_status;
#define RT_OK 0
#define RT_ERR_INVALID (-1) /* bad argument / shape */
#define RT_ERR_HIP (-2)     /* a HIP runtime call failed (message has the hipError_t name) */
#define RT_ERR_IO (-3)      /* file not found / unparsable OBJ */
#define RT_ERR_STATE (-4)   /* call order (no scene uploaded, no viewport) */
#define RT_ERR_OOM (-5)     /* device allocation failed */
#define RT_ERR_OVERFLOW (-6) /* an EXACT render lost a path level (see rt_render): the image is not the reference's */

typedef struct rt_scene rt_scene; /* host-side scene builder */
typedef struct rt_ctx rt_ctx;     /* one device context (one GPU, one stream) */

/* ------------------------------------------------------------------ scene (host) */
rt_status rt_scene_create(rt_scene** out);
void rt_scene_destroy(rt_scene* s);
/* Cornell box of Renderer::Renderer(): floor, shortbox, tallbox (white), left (red), right (green), light */
rt_status rt_scene_add_cornell_box(rt_scene* s);
/* a TriangleMesh from an OBJ file (single mesh; positions scaled by 0.01 like the reference) */
rt_status rt_scene_add_obj(rt_scene* s, const char* path, const float albedo[3], const float emission[3], int32_t* mesh_id);
/* a TriangleMesh from de-indexed raw positions (9 floats per triangle, pre-scale, objl order) */
rt_status rt_scene_add_mesh(rt_scene* s, const float* raw_positions, uint64_t n_tris, const float albedo[3], const float emission[3],
                            int32_t* mesh_id);
/* Whitted-style scenes (the reference's "BVH Ray Tracer", BV/ = BVH Ray Tracer/8599RayTracerGUI/src/):
 * a TriangleMesh(file, mesh_scale, world_coordinates) (BV/TriangleMesh.h:113-151): vertex =
 * offset + scale * p (offset may be NULL: vertex = scale * p); every triangle Diffuse_Glossy with the
 * given diffuse color and phong_diffuse (BV/TriangleMesh.h:64-67,138-141) */
rt_status rt_scene_add_whitted_mesh(rt_scene* s, const float* raw_positions, uint64_t n_tris, float scale, const float offset[3],
                                    const float diffuse[3], float phong_diffuse, int32_t* mesh_id);
rt_status rt_scene_add_whitted_obj(rt_scene* s, const char* path, float scale, const float offset[3], const float diffuse[3],
                                   float phong_diffuse, int32_t* mesh_id);
/* Renderer::Add(std::unique_ptr<PointLightSource>) (BV/Renderer.h:88-97, BV/LightSource.h) */
rt_status rt_scene_add_point_light(rt_scene* s, const float position[3], const float radiance[3]);
/* Whitted miss color (default (0.2, 0.7, 0.8), BV/Renderer.h:189) */
rt_status rt_scene_set_sky(rt_scene* s, const float rgb[3]);
/* the BVH Ray Tracer's Renderer::Renderer() scene (BV/Renderer.cpp:26-43) from the two OBJ files */
rt_status rt_scene_add_bvh_tracer_scene(rt_scene* s, const char* bunny_obj, const char* teapot_obj);

/* The Whitted Style Ray Tracer's world (WH/ = Whitted Style Ray Tracer/8599RayTracerGUI/src/): entities
 * intersected brute force in insertion order, Whitted recursion to depth 5 with Fresnel reflection /
 * Snell refraction (WH/Renderer.h:184-310).  A scene holds either such a world or triangle meshes. */
#define RT_REFLECTIVE 0
#define RT_REFLECTIVE_REFRACTIVE 1
#define RT_DIFFUSE_GLOSSY 2
typedef struct {
    int32_t nature;               /* RT_REFLECTIVE / RT_REFLECTIVE_REFRACTIVE / RT_DIFFUSE_GLOSSY */
    float refractive_index;       /* WH/Entity.h defaults: 1.3 */
    float phong_diffuse;          /* 0.8 */
    float phong_specular;         /* 0.2 */
    float specular_size_factor;   /* 25 */
    float diffuse_color[3];       /* (0.2, 0.2, 0.2); triangle meshes use the chessboard texture instead
                                     (TriangleMesh::GetDiffuseColor, WH/TriangleMesh.h:79-84) */
} rt_world_material;
/* fills *m with the WH/Entity.h defaults */
void rt_world_material_default(rt_world_material* m);
rt_status rt_scene_add_world_sphere(rt_scene* s, const float center[3], float radius, const rt_world_material* m, int32_t* entity_id);
/* indexed mesh: n_vertices positions (3 floats) + texture coordinates (2 floats), 3 indices per triangle */
rt_status rt_scene_add_world_mesh(rt_scene* s, const float* vertices, uint32_t n_vertices, const uint32_t* indices, uint32_t n_tris,
                                  const float* uv, const rt_world_material* m, int32_t* entity_id);
/* Renderer::Renderer() of the Whitted Style Ray Tracer: diffuse + glass sphere, chessboard, two lights */
rt_status rt_scene_add_two_spheres_scene(rt_scene* s);
/* Whitted::Sphere(center, radius, material) + Renderer::Add (MC/Sphere.h:16-108, MC/Renderer.h:78-81): a sphere
 * entity of the PATH-TRACED scene (beside the triangle meshes; id = its entity index, the order of Add).  It is
 * a top-level leaf of the entity BVH with box AABB_3D{center + radius, center - radius} and area 4 PI radius^2;
 * rays meet it by the reference's float QuadraticFormula (MC/WhittedUtilities.h:36-60, MC/Sphere.h:62-97).  An
 * emissive sphere may not be the first emissive entity: the reference's Sphere::Sampling is empty (a TODO,
 * MC/Sphere.h:30-33), so SamplingAreaLight would read an unset record (rt_scene_build: RT_ERR_INVALID).  Scenes
 * with spheres render on the megakernel (rt_stats.kernel_reason RT_KERNEL_REASON_SPHERES). */
rt_status rt_scene_add_sphere(rt_scene* s, const float center[3], float radius, const float albedo[3], const float emission[3],
                              int32_t* entity_id);
rt_status rt_scene_build(rt_scene* s);

typedef struct {
    uint32_t n_meshes, n_tris, n_nodes, n_light_tris, max_depth;
    int32_t light_mesh;
    float light_area;
    uint64_t device_bytes; /* bytes the flattened scene occupies in HBM */
    uint32_t n_leaf_boxes; /* distinct leaf boxes of a small scene's coherent trace (0: BVH traversal) */
    uint32_t n_light_skip; /* (light triangle, triangle) pairs whose shadow-ray candidates the vertex kernel skips
                              (near-coplanar with the light; 0 when the scene's error bound does not hold) */
    uint32_t split_root;   /* split trace of a larger scene (the vertex kernel's BVH variant): the walked subtree
                              [split_root, split_end) of the DFS pre-order; 0 when the scene has none */
    uint32_t split_end;
    uint32_t n_split_leaves;   /* leaves outside that subtree, tested by their boxes (<= 32) */
    uint32_t n_split_boxes;    /* their distinct boxes */
    uint32_t n_spheres;        /* sphere entities (API 4); rt_scene_export: a sphere's slot has tri_f a = center,
                                  b = (radius, radius^2, 0), c = n = 0, area = its area, tri_i = (entity, -2) */
} rt_scene_info;
rt_status rt_scene_get_info(const rt_scene* s, rt_scene_info* info);
/* flattened DFS pre-order view for tests: node_f 7/node (min[3] max[3] mesh_area), node_i 5/node
 * (left right tri mesh top_level), tri_f 13/tri (a b c n area), tri_i 2/tri (mesh material) */
rt_status rt_scene_export(const rt_scene* s, float* node_f, int32_t* node_i, float* tri_f, int32_t* tri_i);
/* The scene's BVH built on the HOST in the device build's algorithm (tests of rt_upload_scene_gpu_bvh):
 * a Karras LBVH over the Morton codes of the triangle-box centroids, one triangle per leaf, in the
 * traversal layout -- nodes: 8 floats x (2 n_tris - 1), tris: 16 floats x n_tris.  Needs >= 2 triangles. */
rt_status rt_scene_lbvh_host(const rt_scene* s, float* nodes, float* tris);
/* A split scene's walked subtree in its 8 near-first pre-orders (one per ray-direction octant, bit 0 = d.x < 0,
 * bit 1 = d.y < 0, bit 2 = d.z < 0), for tests: 8 x (split_end - split_root) nodes of 8 floats in the traversal
 * layout (indices as in the DFS order; a skip pointer that leaves the subtree reads n_nodes).  *n_floats
 * receives the size (0: no split); out may be null to query it. */
rt_status rt_scene_walk_orders(const rt_scene* s, float* out, uint64_t* n_floats);
/* A Whitted scene's (point lights, config C3) whole tree in its 8 near-first pre-orders, for tests: 8 x n_nodes
 * nodes in the same layout (a skip pointer past the last node reads n_nodes; 0 floats: none).  The Whitted
 * kernel walks the ordering of a finite ray's octant (knob RT_WH_ORDER=0: the DFS order). */
rt_status rt_scene_whitted_orders(const rt_scene* s, float* out, uint64_t* n_floats);
/* The same orderings in the Whitted kernel's 16-byte nodes (round 6), for tests: 8 x n_nodes x 4 words -- (near.x |
 * far.x << 16, near.y | far.y << 16, near.z | far.z << 16, skip or 0x80000000 | triangle), each plane an IEEE half
 * rounded outward; *n_words receives the size (0: none). */
rt_status rt_scene_whitted_orders_half(const rt_scene* s, uint32_t* out, uint64_t* n_words);

/* ------------------------------------------------------------------ camera (host math) */
typedef struct {
    float position[3];
    float inv_projection[16]; /* column-major glm::mat4 */
    float inv_view[16];
} rt_camera;
/* the reference Camera (defaults MC/Camera.h:19-37, fov 35 deg, near 0.1, far 100) for a viewport;
 * optional proj/view (16 floats each, may be NULL) */
rt_status rt_camera_default(uint32_t width, uint32_t height, rt_camera* out, float* proj, float* view);
/* a camera at `position` looking along `forward` (up = +y), glm::lookAt / perspectiveFov */
rt_status rt_camera_look(uint32_t width, uint32_t height, const float position[3], const float forward[3], float vfov_deg,
                         float near_clip, float far_clip, rt_camera* out);
/* the same plus the (non-inverted) projection and view matrices (16 floats each, may be NULL), which
 * the Denoiser's temporal reprojection uses (DN/Renderer.cpp:254-256) */
rt_status rt_camera_look_ex(uint32_t width, uint32_t height, const float position[3], const float forward[3], float vfov_deg,
                            float near_clip, float far_clip, rt_camera* out, float* proj, float* view);

/* ------------------------------------------------------------------ device context */
typedef struct {
    int32_t device;  /* HIP device ordinal */
    void* stream;    /* hipStream_t to launch on (NULL: the context creates its own) */
    uint32_t flags;  /* reserved, 0 */
} rt_device_cfg;
rt_status rt_create(rt_ctx** out, const rt_device_cfg* cfg);
void rt_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);
rt_status rt_upload_scene(rt_ctx* ctx, const rt_scene* s);
/* rt_upload_scene with the BVH built on the DEVICE (rt_lbvh.hip, a non-parity fast path for large
 * meshes; the reference builds on the host, MC/BVH.h:131-214): a Karras linear BVH over 30-bit Morton
 * codes, one triangle per leaf, written in DFS order with skip pointers.  Closest-hit t values equal the
 * reference-tree render's (the Moller-Trumbore operations do not depend on the tree); a tie between two
 * triangles at one t resolves by this tree's DFS order instead of the reference's.  Renders use the
 * BVH-walking kernels (no leaf-box table).  build_ms (may be NULL) receives the build time on the
 * device.  Needs >= 2 triangles. */
rt_status rt_upload_scene_gpu_bvh(rt_ctx* ctx, const rt_scene* s, float* build_ms);
/* diagnostic: copy the device's node / triangle arrays (up to n_node_floats / n_tri_floats floats) */
rt_status rt_debug_scene_arrays(rt_ctx* ctx, float* nodes, uint32_t n_node_floats, float* tris, uint32_t n_tri_floats);
/* full image size; allocates the accumulation (float4) and RGBA8 buffers for this device's pixels.
 * Pixels are dealt in row bands of `band` rows round-robin over `nranks` (band=8, rank=0, nranks=1
 * for one GPU); rt_local_rows() returns how many rows this device owns. */
rt_status rt_resize(rt_ctx* ctx, uint32_t width, uint32_t height, uint32_t band, uint32_t rank, uint32_t nranks);
uint32_t rt_local_rows(const rt_ctx* ctx);

#define RT_RENDER_EXACT 1u /* fold the recursion inner-first (bit-faithful accumulation); else forward */
#define RT_RENDER_COUNT 2u /* collect node/triangle/ray counters (rt_get_stats) */
#define RT_RENDER_GLOBAL_SCENE 4u /* read the scene from HBM even when it fits in LDS (A/B) */
#define RT_RENDER_GLOBAL_STACK 8u /* keep the whole EXACT fold stack in HBM (A/B) */
#define RT_RENDER_WHITTED 16u /* Whitted-style shading with point lights and corner-of-pixel rays
                                 (BV/Renderer.cpp:109-233) instead of Monte Carlo path tracing; seed/rr unused */
typedef struct {
    uint32_t first_frame; /* 1-based frame index of the first sample (== reference frame_accumulating) */
    uint32_t n_frames;    /* samples per pixel rendered by this call */
    uint64_t seed;        /* RNG key */
    float rr;             /* Russian-roulette survival probability (MC/Renderer.h:199) */
    uint32_t flags;       /* RT_RENDER_* */
} rt_render_params;
/* Renders n_frames frames into the device accumulation buffer (reset when first_frame == 1) and
 * packs RGBA8.  Asynchronous on the context stream unless a host output pointer is given:
 * out_rgba (local rows x width u32, ABGR, may be NULL) / out_accum (local rows x width x 4 f32,
 * may be NULL) are filled after a stream synchronisation.  Local row r is global row
 * (rank + (r / band) * nranks) * band + r % band.
 *
 * Path length (RT_RENDER_EXACT): Renderer::shading recurses until Russian roulette stops it
 * (MC/Renderer.cpp:193); the kernels cut a path at 4096 vertices (probability rr^4096: 1e-397 at the
 * default 0.8, 1.3e-18 at 0.99).  The fold stack is sized from rr (1.5 x the depth a path exceeds with
 * probability 1e-12, 192..2048 levels); a deeper path is still exact -- the vertex kernel lists the
 * sample and renders it again with a 4096-level stack (rt_stats.resampled).  Only when a level cannot be
 * kept (the megakernel's stack, used for G-buffer/counter renders, or more than 2^20 overflows in one
 * pass) does the render fail: RT_ERR_OVERFLOW, returned by the call that synchronises with it (rt_render
 * with an output pointer, rt_synchronize, rt_read_accumulation, rt_get_stats).  The outcome accumulates over
 * asynchronous renders until such a call reads it, so an earlier render's loss is reported even when a
 * later render lost nothing. */
rt_status rt_render(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p, uint32_t* out_rgba, float* out_accum);
/* device pointers of the local accumulation (float4) and RGBA8 buffers */
rt_status rt_device_buffers(rt_ctx* ctx, void** d_accum, void** d_rgba);
/* copy the local float4 accumulation (local_rows x W x 4 floats) to host memory after synchronising with
 * the context's stream; returns RT_ERR_OVERFLOW like rt_synchronize (replaces reading
 * Renderer::temporal_accumulation_frame_data, MC/Renderer.h:194) */
rt_status rt_read_accumulation(rt_ctx* ctx, float* out_accum);
/* copy device RGBA8 to a caller device pointer (e.g. a torch tensor) on the context stream */
rt_status rt_copy_rgba_to_device(rt_ctx* ctx, void* dst);
rt_status rt_reset_accumulation(rt_ctx* ctx);
rt_status rt_synchronize(rt_ctx* ctx);

typedef struct {
    float last_kernel_ms;     /* the last rt_render's kernels, first to last (HIP events, same stream) */
    uint64_t node_tests;      /* RT_RENDER_COUNT only */
    uint64_t tri_tests;
    uint64_t rays;
    uint64_t stack_overflows; /* EXACT paths deeper than the fold stack / ring: resampled + overflow_lost */
    uint64_t samples;
    uint32_t grid, block, stack_depth;
    /* RT_RENDER_COUNT scheduling diagnostics: wave-level executions */
    uint64_t wave_rounds, wave_steps, wave_tri_tests, wave_service;
    /* RT_RENDER_COUNT: wave-level fold iterations; wave cycles (s_memtime) spent in service,
     * work-queue + camera-ray, and traversal rounds; lanes served per service round (sum) */
    uint64_t wave_fold, cycles_service, cycles_queue, cycles_trace, service_lanes;
    float last_denoise_ms;    /* rt_render_denoised: the joint bilateral + temporal kernels (HIP events) */
    uint32_t n_chunks;        /* frame chunks per pixel of the last rt_render's (last) launch: 1 unless the
                                 launch has few pixels per lane; last_kernel_ms covers the in-order finalize */
    uint32_t n_passes;        /* launches over consecutive frame ranges (bounded parked-sample memory) */
    uint32_t kernel;          /* the path kernel of the last rt_render: RT_KERNEL_* */
    uint64_t resampled;       /* EXACT: samples whose path outgrew the fold ring, rendered again exactly */
    uint64_t overflow_lost;   /* EXACT: levels / samples that could not be kept (non-zero => RT_ERR_OVERFLOW)
                                 -- both summed over the renders since the last synchronisation that checked them */
    uint32_t kernel_reason;   /* why `kernel` rendered the last path frame: RT_KERNEL_REASON_* (API 3; was a reserved
                                 zero in API 2) */
    float last_prepass_ms;    /* the vertex kernel's camera pre-pass (camera_prepass_kernel), summed over passes */
    float last_main_ms;       /* the path kernel proper (pt_coherent_kernel / pt_megakernel), summed over passes;
                                 last_kernel_ms spans these plus the resample and in-order finalize kernels */
} rt_stats;
#define RT_KERNEL_MEGA 0      /* pt_megakernel (rt_kernels.hip): any scene, counters, G-buffer frames */
#define RT_KERNEL_VERTEX 1    /* pt_coherent_kernel (rt_coherent.hip): small scenes, vertex-synchronous */
#define RT_KERNEL_WHITTED 2   /* whitted_kernel / whitted_world_kernel (rt_whitted.hip) */
#define RT_KERNEL_VERTEX_BVH 3   /* pt_coherent_kernel's BVH variant (rt_coherent.hip): other path scenes */
#define RT_KERNEL_REASON_DEFAULT 0       /* the kernel the scene calls for */
#define RT_KERNEL_REASON_TABLES_LDS 1    /* megakernel: the BVH variant stages the material and light tables (and a
                                            split scene's outside triangles) in LDS, and they exceed its 40 KB
                                            (about 2500 light triangles or 1280 materials); a large slowdown */
#define RT_KERNEL_REASON_MATERIALS 2     /* megakernel: 2^14 materials or more (the vertex kernel packs 14 bits) */
#define RT_KERNEL_REASON_MODE 3          /* megakernel: a work-counter render or a denoiser G-buffer frame */
#define RT_KERNEL_REASON_KNOB 4          /* a debug knob (RT_VERTEX / RT_VERTEX_BVH / RT_BRUTE) chose it */
#define RT_KERNEL_REASON_TRIANGLES 5     /* megakernel: 2^31 triangles or more (the BVH variant indexes triangles in 31 bits) */
#define RT_KERNEL_REASON_SPHERES 6       /* megakernel: the scene has sphere entities (rt_scene_add_sphere, API 4) */
rt_status rt_get_stats(rt_ctx* ctx, rt_stats* st);
/* diagnostic: the raw device counters of the last rt_render (up to 512 x u64; [16..23] = wave cycles per
 * section and [24..43] = wave-level event counts of the vertex kernel in RT_SECTIONS builds, [64..511]
 * candidate histograms in RT_SECTIONS >= 3 builds), after a stream synchronisation */
rt_status rt_debug_counters(rt_ctx* ctx, uint64_t* out, uint32_t n);

/* ------------------------------------------------------------------ several GPUs, one frame
 * A group of device contexts renders one frame together.  Replaces, across GPUs, the reference's
 * std::execution::par row loop of Renderer::Render (MC/Renderer.cpp:100-110): member i (rank i of
 * n) owns the row bands b with b mod n == i (bands of `band` rows, as rt_resize), renders them in one
 * launch on its own device and stream, and the RGBA8 band sets are gathered to member 0 and reassembled
 * into the full frame there.  The gather is RCCL (ncclGather over one communicator per member,
 * ncclCommInitAll, issued as one group) when the member devices are distinct, device-to-device copies
 * when a device repeats (RCCL takes one rank per GPU; e.g. n members on one GPU in tests) or when
 * RT_GROUP_GATHER=copy (a debug knob, read only with RT_DEBUG_KNOBS=1).  Every pixel is the same as in a one-device render: the random stream is keyed by
 * the global pixel. */
typedef struct rt_group rt_group;
rt_status rt_group_create(rt_group** out, const int32_t* devices, uint32_t n);
void rt_group_destroy(rt_group* g);
const char* rt_group_last_error(const rt_group* g);
uint32_t rt_group_size(const rt_group* g);
/* member i's context (rank i): stats, device buffers of its bands */
rt_ctx* rt_group_member(rt_group* g, uint32_t i);
rt_status rt_group_upload_scene(rt_group* g, const rt_scene* s);
rt_status rt_group_resize(rt_group* g, uint32_t width, uint32_t height, uint32_t band);
/* one Renderer::Render x n_frames on every member, then the gather.  Asynchronous unless out_rgba (width x
 * height u32, ABGR, row 0 = bottom) is given; the members' overflow status is checked at the
 * synchronisation (as rt_render) */
rt_status rt_group_render(rt_group* g, const rt_camera* cam, const rt_render_params* p, uint32_t* out_rgba);
/* the assembled RGBA8 frame on member 0's device (valid after rt_group_render's work completes) */
rt_status rt_group_frame_device(rt_group* g, void** d_rgba);
/* the accumulation (width x height x 4 f32, row 0 = bottom) gathered to the host */
rt_status rt_group_read_accumulation(rt_group* g, float* out_accum);
rt_status rt_group_reset_accumulation(rt_group* g);
rt_status rt_group_synchronize(rt_group* g);
typedef struct {
    float last_ms;            /* the last rt_group_render: member 0's stream, first launch to assembled frame */
    float max_member_kernel_ms; /* the slowest member's path-kernel time of that render */
    uint32_t gather;          /* 1 = RCCL, 0 = device-to-device copies */
    uint32_t n;               /* members */
} rt_group_stats;
rt_status rt_group_get_stats(rt_group* g, rt_group_stats* st);

/* ------------------------------------------------------------------ the Denoiser (DN/ = Denoiser/8599RayTracerGUI/src/)
 * One call = one Renderer::Render of the Denoiser project (DN/Renderer.cpp:101-283): a 1-spp path-traced
 * frame through the pixel centres that records the G-buffer (DN/Renderer.cpp:285-311), the joint
 * bilateral filter and the temporal filter of DN/Denoiser.h, and the RGBA8 pack.  Full frames on one
 * device (rt_resize with nranks == 1).  The history (previous frame's output, primitive ids and
 * matrices) lives in the context; rt_denoise_restart drops it (Renderer::RestartTemporal, DN/Renderer.h:74-77). */
typedef struct {
    int32_t jbf_half_size;            /* 0: joint bilateral filter off; the UI's 15/33/65 px kernels are 3/16/32 */
    int32_t temporal_half_size;       /* 0: temporal filter off; the UI's 7/15/33 px kernels are 3/7/16 */
    float tolerance;                  /* history clamp, in deviations (1, 2, 3) */
    float current_frame_weighting;    /* 0.05 / 0.1 / 0.2 / 0.5 */
    int32_t immediate_clamp;          /* clamp each frame's color to [0,1] before filtering (default 1) */
    float sigma_position, sigma_color, sigma_normal, sigma_coplanarity;   /* 32, 0.6, 0.1, 0.1 */
} rt_denoise_params;
/* DN/Denoiser.h member defaults (JBF half size 7, temporal 3, tolerance 1, weighting 0.2, sigmas) */
void rt_denoise_params_default(rt_denoise_params* p);
/* proj/view: this frame's camera matrices (rt_camera_look_ex); frame: the RNG frame index (1-based);
 * out_rgba (W x H u32) / out_color (W x H x 4 f32: the temporal output) may be NULL */
rt_status rt_render_denoised(rt_ctx* ctx, const rt_camera* cam, const float proj[16], const float view[16], uint32_t frame, uint64_t seed,
                             float rr, const rt_denoise_params* p, uint32_t* out_rgba, float* out_color);
rt_status rt_denoise_restart(rt_ctx* ctx);
/* the last denoised frame's buffers (W x H each; any pointer may be NULL): G-buffer color / world
 * position / normal (4 floats per pixel), primitive id (-1: primary ray missed), joint bilateral output */
rt_status rt_get_gbuffer(rt_ctx* ctx, float* color, float* position, float* normal, int32_t* prim, float* spatial);

/* closest hit of n rays (host arrays; tri = flattened triangle slot or -1, t = double distance) */
rt_status rt_trace(rt_ctx* ctx, uint64_t n, const float* org, const float* dir, int32_t* tri, double* t);
/* Renderer::SamplingAreaLight (MC/Renderer.h:163-180 -> TriangleMesh::Sampling -> BVH::Sampling_from_root,
 * MC/TriangleMesh.h:193-197, MC/BVH.h:103-129, MC/TriangleMesh.h:69-89) on the device, for n cases of three
 * given u32 draws (Walnut::Random::Float's words: area pick, triangle x, triangle y): the sampled location and
 * the light triangle's normal (3 floats each), the light's emission (3 floats) and the PDF 1 / total light
 * area (the overwrite of MC/BVH.h:105-106).  RT_ERR_STATE if the scene has no emissive mesh. */
rt_status rt_sample_light(rt_ctx* ctx, uint64_t n, const uint32_t* u, float* loc, float* normal, float* emission, float* pdf);
/* closest hit of n rays against a Whitted world (get_intersection_payload, WH/Renderer.h:109-140):
 * entity index or -1, mesh triangle slot or -1, and (t, barycentric 2, barycentric 3) as 3 floats */
rt_status rt_world_trace(rt_ctx* ctx, uint64_t n, const float* org, const float* dir, int32_t* entity, int32_t* tri, float* t_bary);
/* device checks of the primitives the kernels shortcut, on the reference's fixture layouts:
 * n_mt Moller-Trumbore cases of 15 floats (a, b, c, origin, direction; MC/TriangleMesh.h:19-45) ->
 * mt_hit (0/1) and mt_t (the double t on a hit, else 0) through the kernels' float pre-screen +
 * double test; n_box slab cases of 12 floats (min, max, origin, direction; MC/BoundingVolume.h:173-215)
 * -> box_hit, 3 per case: the std::max/min form, the finite-reciprocal IEEE form and the vertex
 * kernel's leaf-box form (-1 for the last two when the reciprocal direction is not finite).
 * Host arrays; any count may be 0. */
rt_status rt_debug_primitives(rt_ctx* ctx, uint64_t n_mt, const float* mt_cases, int32_t* mt_hit, double* mt_t, uint64_t n_box,
                              const float* box_cases, int32_t* box_hit);
/* device arithmetic self-test: for each x: sqrtf, 1/x, cos, sin (as the kernel evaluates them),
 * the double reciprocal's low/high words, the C1 specular lobe powf(x, 25), and the denoiser's expf(x)
 * and acosf(x) (glibc's algorithms, DN/Denoiser.h:195,203) -> 9 floats per input */
rt_status rt_math_selftest(rt_ctx* ctx, uint64_t n, const float* x, float* out);

int32_t rt_api_version(void);

#ifdef __cplusplus
}
#endif
#endif
