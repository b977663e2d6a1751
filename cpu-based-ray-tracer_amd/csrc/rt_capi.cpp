// rt_capi.cpp -- implementation of include/rt_capi.h (host side; compiled by hipcc, links the HIP runtime).
#include "rt_capi.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rt_kernels.h"
#include "rt_knobs.h"
#include "rt_scene.h"

struct rt_scene {
    rt::SceneBuilder builder;
    rt::FlatScene flat;
    bool built = false;
};

// device counters: [0, 64) work / overflow / section counters, [64, 512) diagnostic histograms
// (RT_SECTIONS >= 3 builds, rt_coherent.hip)
static constexpr uint32_t kCounterWords = 512;
// the work counters: [0] items / parts (one queue), [1] the pre-pass's list length, and from word 32 the path
// kernel's 8 part queues, 32 words (128 B) apart
static constexpr size_t kWorkCounterBytes = (32 + 8 * 32) * sizeof(uint32_t);

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    // scene
    float4 *d_nodes = nullptr, *d_tris = nullptr, *d_mats = nullptr, *d_lnodes = nullptr, *d_ltris = nullptr, *d_lboxes = nullptr;
    float4* d_sboxes = nullptr;   // split trace (FlatScene::sboxes): outside leaf boxes
    int32_t* d_stri = nullptr;    // split trace: outside slot -> triangle
    float4* d_wcopies = nullptr;  // split trace: near-first orderings of the walked subtree (FlatScene::wcopies)
    float4* d_worders = nullptr;  // Whitted scenes: near-first orderings of the whole tree (FlatScene::worders)
    uint4* d_worders_h = nullptr; // the same in 16-byte nodes, half planes rounded outward (FlatScene::worders_h)
    uint32_t split_root = 0, split_end = 0, n_sboxes = 0, n_sleaves = 0;
    float4* d_tabc = nullptr;                      // the triangles' vertices (the Whitted half-plane walk's exact leaf boxes)
    // fold-level materials in the direct term's sign bits (one 16-byte ring entry per level instead of an
    // entry plus a 4-byte material that misses L2 on its own line: C4 221 -> 133 B/sample of L2 -> fabric
    // traffic): RT_RING_PACK 0 off, 1 BVH variant only, 2 both variants
    uint32_t ring_pack = 2;
    bool bvh_prepass = true;     // split scenes: the BVH variant's paths start from the camera pre-pass (RT_BVH_PREPASS=0: off)
    bool pre_defer_walk = true;  // ... whose camera rays into the walked subtree are traced by the path kernel (RT_PRE_DEFER=0: walked there)
    float4 *d_wmats = nullptr, *d_plights = nullptr, *d_went = nullptr, *d_wtris = nullptr;
    rt_scene_header hdr{};
    bool has_scene = false;
    // image
    uint32_t W = 0, H = 0, band = 8, rank = 0, nranks = 1, local_rows = 0;
    float4* d_accum = nullptr;
    uint32_t* d_rgba = nullptr;
    // scratch
    uint32_t* d_counter = nullptr;
    unsigned long long* d_counters = nullptr;
    float4* d_stack_ld = nullptr;
    int32_t* d_stack_mat = nullptr;
    uint32_t stack_depth = 0;
    uint32_t stack_depth_force = 0;   // test knob (RT_STACK_DEPTH): a small fold ring forces overflows
    // EXACT: ring overflows listed by the vertex kernel and rendered again by resample_kernel
    uint4* d_ovf = nullptr;
    uint32_t ovf_cap = 1u << 20;
    float4* d_rs_stack = nullptr;
    int32_t* d_rs_mat = nullptr;
    uint32_t rs_threads = 1024;
    // counters[13] (lost levels / samples) and counters[14] (overflows listed and re-rendered) of the last render, copied
    // to pinned host memory at the end of rt_render and checked at the next synchronisation
    unsigned long long* h_ovf = nullptr;
    bool pending_check = false;
    uint32_t grid = 0, block = 256, total_threads = 0;   // grid of the EXACT kernel (sizes the fold stack)
    uint32_t n_cu = 0;
    int occ_global[2][2] = {{0, 0}, {0, 0}};              // blocks per CU, [exact][count], scene in HBM
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // per pass: events before the camera pre-pass, between it and the path kernel, after the path kernel
    std::vector<hipEvent_t> kev;
    uint32_t kev_used = 0;        // passes of the last render with kernel events
    bool kev_prepass = false;     // the last render ran the camera pre-pass
    rt_stats stats{};
    bool pending_stats = false;
    uint32_t last_flags = 0;
    // the Denoiser: this frame's G-buffer, filter outputs and the history (previous temporal output, ids, matrices)
    float4 *d_gb_color = nullptr, *d_gb_pos = nullptr, *d_gb_nrm = nullptr, *d_spatial = nullptr, *d_temporal = nullptr, *d_prev_color = nullptr;
    int32_t *d_gb_prim = nullptr, *d_prev_prim = nullptr;
    uint32_t *d_dn_rgba = nullptr;
    size_t dn_pixels = 0;
    bool have_prev = false;
    float prev_proj[16] = {}, prev_view[16] = {};
    hipEvent_t ev2 = nullptr, ev3 = nullptr;
    bool pending_denoise = false;
    bool gb_next = false, gb_clamp = true;   // rt_render_denoised -> rt_render: G-buffer mode
    // frame chunking (KParams::n_chunks): split when a launch has fewer than min_px_per_lane pixels
    // per lane, into about items_per_lane items per lane but no chunk shorter than min_chunk_frames
    // (tuned on MI355X at N=1 and on an 8-way row band; RT_CHUNKS forces a count)
    uint32_t force_chunks = 0, items_per_lane = 64, min_px_per_lane = 32, min_chunk_frames = 8;
    uint64_t lbuf_budget = 96ull << 30;   // bytes of parked samples (+ camera records) per launch; C4 needs 59 GB of 288
    bool lbuf_budget_env = false;         // RT_LBUF_BUDGET_MB given: else min(96 GB, 3/4 of free memory) per render
    float* d_lbuf = nullptr;
    uint32_t* d_sky = nullptr;    // pre-pass sky bits (KParams::sky_bits)
    size_t sky_words_alloc = 0;
    size_t lbuf_floats = 0;
    // the vertex kernel's camera pre-pass: surface-hit records, per-segment counts, the non-empty segments
    float4* d_crec = nullptr;
    size_t crec_quads = 0;
    uint2* d_seg_list = nullptr;
    size_t seg_words = 0;
    unsigned long long* d_tile_boxes = nullptr;   // the pre-pass's per-tile leaf-box masks
    size_t tile_words = 0;
    int lds_levels_force = -1;   // diagnostic: fold-stack levels in LDS (RT_LDS_LEVELS), occupancy permitting or not
    bool brute = true;   // small scenes: coherent trace over the distinct leaf boxes (RT_BRUTE=0 disables)
    bool direct_div2 = true;   // the direct term's two divisions on Markstein's path when in range (RT_DIRECT_DIV2=0: IEEE, A/B)
    bool sky_bits = true;   // the pre-pass's camera-ray misses as bits, not parked samples (RT_SKY_BITS=0 disables)
    bool force_walk = false;   // diagnostic: the vertex kernel's per-lane BVH walk for every ray (RT_FORCE_WALK=1)
    bool vertex = true;  // small scenes: the vertex-synchronous kernel, rt_coherent.hip (RT_VERTEX=0: the megakernel's coherent trace)
    bool lbuf_pm = false;   // diagnostic: the vertex kernel's parked samples pixel-major (RT_LBUF_PIXEL_MAJOR=1; -1 % C4/C5)
    bool split = true;   // larger scenes: the split trace when the scene has one (RT_SPLIT=0 disables)
    bool walk_order = true;   // split trace: walk the subtree's near-first ordering of the ray's octant (RT_WALK_ORDER=0: DFS)
    bool wh_order = true;     // Whitted kernel: walk the whole tree's near-first ordering of the ray's octant (RT_WH_ORDER=0: DFS)
    bool wh_half = false;     // ... in its 16-byte half-plane nodes (RT_WH_HALF=1 with a -DRT_WH_HALF=1 build: an A/B)
    bool seg_parts_off = false;   // A/B (RT_SEG_PARTS_OFF=1): short pre-pass segments, one path-kernel part each
    uint32_t seg_min_parts = 128; // A/B (RT_SEG_MIN_PARTS): path-kernel parts per wave the split aims for
    uint32_t seg_part_lf = 4;     // A/B (RT_SEG_PART_LF): log2 of the fewest frames' worth of records in a part
    uint32_t seg_tail_parts = 8;  // A/B (RT_SEG_TAIL_PARTS): each wave's last parts' worth of segments taken finer ...
    uint32_t seg_tail_extra = 3;  // A/B (RT_SEG_TAIL_EXTRA): ... in 2^extra times as many parts (0: no tail split)
    uint32_t n_work_queues = 8;   // A/B (RT_WORK_QUEUES, 1 or 8): counters handing out the path kernel's parts
    bool vertex_bvh = true;   // other scenes: the vertex kernel's BVH variant (RT_VERTEX_BVH=0: the megakernel)
    uint32_t lds_pad = 0;   // diagnostic: extra dynamic LDS bytes per workgroup (RT_LDS_PAD) to lower occupancy
    uint32_t thresh = 8, steps = 12;   // traversal scheduling (tuned on MI355X, profiles/) (RT_THRESH / RT_STEPS override)
    uint32_t vthresh = 32, vsteps = 8; // the same for the vertex kernel's BVH variant (C5 sweep)
    uint32_t sthresh = 12, ssteps = 12; // the BVH variant with the split trace: few lanes walk, so rounds run while
                                       // more than 12 of them do, 12 box tests per round.  Round 3 (C5 sweep 2 / 4 / 6 /
                                       // 8 / 12 / 16 / 32: 3003 / 3283 / 3399 / 3419-3427 / 3403 / 3261 / 2588 Msamples/s;
                                       // steps 4 / 8 / 12 / 16: 3336 / 3427 / 3466 / 3461, profiles/r03/ab/ab_c5_split.json)
                                       // chose 8; on the round-5 kernel (near-first SAH walk, shorter walks) 8 / 12 / 16 /
                                       // 20 / 24 / 32 give 87.7-88.4 / 85.8 / 86.4 / 88.5 / 92.0 / 102.5 ms at 3840x2160x64
                                       // (profiles/r05/ab/sweep_c5_thresh.jsonl)
};

namespace {

constexpr size_t kMaxLdsScene = 48 * 1024;   // scenes up to ~700 triangles live in LDS
// the vertex kernel's BVH variant: materials + light tables + split slots in LDS beside its 17 KB of lane
// state (~2500 light triangles; C5: 1.9 KB)
constexpr size_t kMaxBvhSmallLds = 40 * 1024;
constexpr uint32_t kStackDepth = 192;   // EXACT fold stack; RR 0.8 => P(depth > 192) ~ 2.5e-19 per sample
constexpr uint32_t kStackDepthMax = 2048;
// the vertex kernel's pending fold keeps its top ring position in 12 bits (rt_coherent.hip VS_PEND: top | count << 12)
static_assert(kStackDepthMax <= 4096, "the pending fold's ring position is 12 bits (rt_coherent.hip VS_PEND)");
constexpr uint32_t kResampleDepth = 4096;   // the kernels' path-length cap (P = rr^4096)

// levels of the EXACT fold stack / ring for survival probability rr: 1.5 x the depth a path exceeds with
// probability 1e-12 (the vertex kernel's ring also holds the previous path's draining fold), at least
// kStackDepth, at most kStackDepthMax.  Deeper paths are exact all the same: the vertex kernel lists
// them for resample_kernel; the megakernel reports RT_ERR_OVERFLOW.
uint32_t stack_levels_for(float rr)
{
    if (!(rr > 0.0f)) return kStackDepth;
    const double d = 1.5 * std::ceil(std::log(1e-12) / std::log((double)rr));
    return (uint32_t)std::min<double>(kStackDepthMax, std::max<double>(kStackDepth, d));
}

rt_status hip_fail(rt_ctx* c, hipError_t e, const char* what)
{
    if (c) c->err = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    return e == hipErrorOutOfMemory ? RT_ERR_OOM : RT_ERR_HIP;
}
#define HIPC(ctx, call)                                   \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
    } while (0)

template <class T> void dfree(T*& p) { if (p) { (void)hipFree((void*)p); p = nullptr; } }

template <class T, class S> rt_status upload(rt_ctx* c, T*& dst, const std::vector<S>& src)
{
    dfree(dst);
    if (src.empty()) return RT_OK;
    HIPC(c, hipMalloc((void**)&dst, src.size() * sizeof(S)));
    HIPC(c, hipMemcpy((void*)dst, src.data(), src.size() * sizeof(S), hipMemcpyHostToDevice));
    return RT_OK;
}

// after a stream synchronisation: an EXACT render that lost a fold level (megakernel stack) or a
// sample the overflow list could not hold fails instead of returning a wrong image
rt_status check_overflow(rt_ctx* c)
{
    if (!c->pending_check) return RT_OK;
    c->pending_check = false;
    // h_ovf holds the device totals since the last check (the last render's copy, after the stream
    // synchronised); they are cleared for the next renders
    c->stats.overflow_lost = c->h_ovf[0];
    c->stats.resampled = c->h_ovf[1];
    if (c->h_ovf[0] != 0 || c->h_ovf[1] != 0) {
        if (hipMemsetAsync(c->d_counters + 13, 0, 2 * sizeof(unsigned long long), c->stream) != hipSuccess) {
            c->err = "clearing the overflow counters failed";
            return RT_ERR_HIP;
        }
    }
    if (c->h_ovf[0] != 0) {
        c->err = "EXACT fold stack overflow: " + std::to_string(c->h_ovf[0]) + " path level(s) or sample(s) lost (stack depth " +
                 std::to_string(c->stack_depth) + ", rr too close to 1 for the megakernel's stack)";
        return RT_ERR_OVERFLOW;
    }
    return RT_OK;
}

uint32_t count_local_rows(uint32_t H, uint32_t band, uint32_t rank, uint32_t nranks)
{
    uint32_t n = 0;
    for (uint32_t b = rank; b * band < H; b += nranks) n += std::min(band, H - b * band);
    return n;
}

}  // namespace

extern "C" {

int32_t rt_api_version(void) { return RT_API_VERSION; }

// ------------------------------------------------------------------ scene
rt_status rt_scene_create(rt_scene** out)
{
    if (!out) return RT_ERR_INVALID;
    *out = new (std::nothrow) rt_scene;
    return *out ? RT_OK : RT_ERR_OOM;
}
void rt_scene_destroy(rt_scene* s) { delete s; }

rt_status rt_scene_add_cornell_box(rt_scene* s)
{
    if (!s) return RT_ERR_INVALID;
    s->builder.add_cornell_box();
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_mesh(rt_scene* s, const float* raw, uint64_t n_tris, const float albedo[3], const float emission[3], int32_t* mesh_id)
{
    if (!s || (!raw && n_tris) || !albedo || !emission || n_tris == 0) return RT_ERR_INVALID;
    rt::MeshDesc m;
    m.raw.assign(raw, raw + 9 * n_tris);
    m.material = rt::MaterialDesc{{albedo[0], albedo[1], albedo[2]}, {emission[0], emission[1], emission[2]}};
    m.name = "mesh" + std::to_string(s->builder.num_meshes());
    const int id = s->builder.add_mesh(std::move(m));
    if (mesh_id) *mesh_id = id;
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_sphere(rt_scene* s, const float center[3], float radius, const float albedo[3], const float emission[3],
                              int32_t* entity_id)
{
    if (!s || !center || !albedo || !emission || !(radius > 0.0f) || !std::isfinite(radius)) return RT_ERR_INVALID;
    const int id = s->builder.add_sphere(rt::F3{center[0], center[1], center[2]}, radius,
                                         rt::MaterialDesc{{albedo[0], albedo[1], albedo[2]}, {emission[0], emission[1], emission[2]}});
    if (entity_id) *entity_id = id;
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_obj(rt_scene* s, const char* path, const float albedo[3], const float emission[3], int32_t* mesh_id)
{
    if (!s || !path || !albedo || !emission) return RT_ERR_INVALID;
    rt::MeshDesc m;
    std::string err;
    if (!rt::SceneBuilder::load_obj_positions(path, m.raw, err) || m.raw.empty()) return RT_ERR_IO;
    m.material = rt::MaterialDesc{{albedo[0], albedo[1], albedo[2]}, {emission[0], emission[1], emission[2]}};
    m.name = path;
    const int id = s->builder.add_mesh(std::move(m));
    if (mesh_id) *mesh_id = id;
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_whitted_mesh(rt_scene* s, const float* raw, uint64_t n_tris, float scale, const float offset[3], const float diffuse[3],
                                    float phong_diffuse, int32_t* mesh_id)
{
    if (!s || !raw || n_tris == 0 || !diffuse) return RT_ERR_INVALID;
    rt::MeshDesc m;
    m.raw.assign(raw, raw + 9 * n_tris);
    m.material = rt::MaterialDesc{{diffuse[0], diffuse[1], diffuse[2]}, {0, 0, 0}, phong_diffuse};
    m.scale = scale;
    if (offset) { m.has_offset = true; m.offset = rt::F3{offset[0], offset[1], offset[2]}; }
    m.name = "whitted" + std::to_string(s->builder.num_meshes());
    const int id = s->builder.add_mesh(std::move(m));
    if (mesh_id) *mesh_id = id;
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_whitted_obj(rt_scene* s, const char* path, float scale, const float offset[3], const float diffuse[3], float phong_diffuse,
                                   int32_t* mesh_id)
{
    if (!s || !path || !diffuse) return RT_ERR_INVALID;
    std::vector<float> raw;
    std::string err;
    if (!rt::SceneBuilder::load_obj_positions(path, raw, err) || raw.empty()) return RT_ERR_IO;
    return rt_scene_add_whitted_mesh(s, raw.data(), raw.size() / 9, scale, offset, diffuse, phong_diffuse, mesh_id);
}

rt_status rt_scene_add_point_light(rt_scene* s, const float position[3], const float radiance[3])
{
    if (!s || !position || !radiance) return RT_ERR_INVALID;
    s->builder.add_point_light(rt::PointLight{{position[0], position[1], position[2]}, {radiance[0], radiance[1], radiance[2]}});
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_set_sky(rt_scene* s, const float rgb[3])
{
    if (!s || !rgb) return RT_ERR_INVALID;
    s->builder.set_sky(rt::F3{rgb[0], rgb[1], rgb[2]});
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_bvh_tracer_scene(rt_scene* s, const char* bunny_obj, const char* teapot_obj)
{
    // Renderer::Renderer(), BV/Renderer.cpp:26-43: bunny x2 at (-1, 6.1, 0), teapot x1 at (-1, 3, 0),
    // Diffuse_Glossy triangles with diffuse color 0.5 and phong_diffuse 0.6 (BV/TriangleMesh.h:64-67,138-141),
    // point lights (-20, 70, 20) and (20, 70, 20) of radiance 1
    if (!s || !bunny_obj || !teapot_obj) return RT_ERR_INVALID;
    const float grey[3] = {0.5f, 0.5f, 0.5f};
    const float ob[3] = {-1.0f, 6.1f, 0.0f}, ot[3] = {-1.0f, 3.0f, 0.0f};
    rt_status r;
    if ((r = rt_scene_add_whitted_obj(s, bunny_obj, 2.0f, ob, grey, 0.6f, nullptr)) != RT_OK) return r;
    if ((r = rt_scene_add_whitted_obj(s, teapot_obj, 1.0f, ot, grey, 0.6f, nullptr)) != RT_OK) return r;
    const float l0[3] = {-20.0f, 70.0f, 20.0f}, l1[3] = {20.0f, 70.0f, 20.0f}, one[3] = {1.0f, 1.0f, 1.0f};
    rt_scene_add_point_light(s, l0, one);
    rt_scene_add_point_light(s, l1, one);
    return RT_OK;
}

void rt_world_material_default(rt_world_material* m)
{
    if (!m) return;
    const rt::WorldEntity d;
    m->nature = d.nature; m->refractive_index = d.refractive_index; m->phong_diffuse = d.phong_diffuse;
    m->phong_specular = d.phong_specular; m->specular_size_factor = d.specular_size_factor;
    m->diffuse_color[0] = d.diffuse_color.x; m->diffuse_color[1] = d.diffuse_color.y; m->diffuse_color[2] = d.diffuse_color.z;
}

static bool world_material(rt::WorldEntity& e, const rt_world_material* m)
{
    if (!m) return true;   // WH/Entity.h defaults
    if (m->nature < 0 || m->nature > 2) return false;
    e.nature = m->nature; e.refractive_index = m->refractive_index; e.phong_diffuse = m->phong_diffuse;
    e.phong_specular = m->phong_specular; e.specular_size_factor = m->specular_size_factor;
    e.diffuse_color = rt::F3{m->diffuse_color[0], m->diffuse_color[1], m->diffuse_color[2]};
    return true;
}

rt_status rt_scene_add_world_sphere(rt_scene* s, const float center[3], float radius, const rt_world_material* m, int32_t* entity_id)
{
    if (!s || !center || !(radius > 0.0f)) return RT_ERR_INVALID;
    rt::WorldEntity e;
    e.kind = 0; e.center = rt::F3{center[0], center[1], center[2]}; e.radius = radius;
    if (!world_material(e, m)) return RT_ERR_INVALID;
    const int id = s->builder.add_world_entity(std::move(e));
    if (entity_id) *entity_id = id;
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_world_mesh(rt_scene* s, const float* vertices, uint32_t n_vertices, const uint32_t* indices, uint32_t n_tris,
                                  const float* uv, const rt_world_material* m, int32_t* entity_id)
{
    if (!s || !vertices || !indices || !uv || n_vertices == 0 || n_tris == 0) return RT_ERR_INVALID;
    rt::WorldEntity e;
    e.kind = 1;
    for (uint32_t i = 0; i < n_vertices; ++i) e.vertices.push_back(rt::F3{vertices[3 * i], vertices[3 * i + 1], vertices[3 * i + 2]});
    e.indices.assign(indices, indices + 3 * (size_t)n_tris);
    for (uint32_t i : e.indices) if (i >= n_vertices) return RT_ERR_INVALID;
    e.uv.assign(uv, uv + 2 * (size_t)n_vertices);
    if (!world_material(e, m)) return RT_ERR_INVALID;
    const int id = s->builder.add_world_entity(std::move(e));
    if (entity_id) *entity_id = id;
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_add_two_spheres_scene(rt_scene* s)
{
    if (!s) return RT_ERR_INVALID;
    s->builder.add_two_spheres_scene();
    s->built = false;
    return RT_OK;
}

rt_status rt_scene_build(rt_scene* s)
{
    if (!s) return RT_ERR_INVALID;
    std::string err;
    if (!s->builder.build(s->flat, err)) return RT_ERR_INVALID;
    s->built = true;
    return RT_OK;
}

rt_status rt_scene_get_info(const rt_scene* s, rt_scene_info* info)
{
    if (!s || !info || !s->built) return s && !s->built ? RT_ERR_STATE : RT_ERR_INVALID;
    const auto& h = s->flat.hdr;
    info->n_meshes = h.n_mats;
    info->n_tris = h.n_tris;
    info->n_nodes = h.n_nodes;
    info->n_light_tris = h.n_ltris;
    info->max_depth = h.max_depth;
    info->light_mesh = h.light_mesh;
    info->light_area = h.light_area;
    info->device_bytes = (s->flat.nodes.size() + s->flat.tris.size() + s->flat.mats.size() + s->flat.lnodes.size() + s->flat.ltris.size() +
                          s->flat.lboxes.size()) * 4;
    info->n_leaf_boxes = h.n_lboxes;
    uint32_t skip = 0;   // the light triangles' candidate-skip masks (rt_layout.h ltris word 3)
    for (size_t k = 0; k + 15 < s->flat.ltris.size(); k += 16) {
        uint32_t m;
        std::memcpy(&m, &s->flat.ltris[k + 3], 4);
        skip += (uint32_t)__builtin_popcount(m);
    }
    info->n_light_skip = skip;
    info->split_root = s->flat.split_root;
    info->split_end = s->flat.split_end;
    info->n_split_leaves = (uint32_t)s->flat.stri.size();
    info->n_split_boxes = (uint32_t)(s->flat.sboxes.size() / 8);
    info->n_spheres = h.n_spheres;
    return RT_OK;
}

rt_status rt_scene_export(const rt_scene* s, float* nf, int32_t* ni, float* tf, int32_t* ti)
{
    if (!s || !s->built) return RT_ERR_STATE;
    const auto& f = s->flat;
    if (nf) std::memcpy(nf, f.dbg_node_f.data(), f.dbg_node_f.size() * 4);
    if (ni) std::memcpy(ni, f.dbg_node_i.data(), f.dbg_node_i.size() * 4);
    if (tf) std::memcpy(tf, f.dbg_tri_f.data(), f.dbg_tri_f.size() * 4);
    if (ti) std::memcpy(ti, f.dbg_tri_i.data(), f.dbg_tri_i.size() * 4);
    return RT_OK;
}

rt_status rt_scene_walk_orders(const rt_scene* s, float* out, uint64_t* n_floats)
{
    if (!s || !s->built) return RT_ERR_STATE;
    if (!n_floats) return RT_ERR_INVALID;
    *n_floats = s->flat.wcopies.size();
    if (out && !s->flat.wcopies.empty()) std::memcpy(out, s->flat.wcopies.data(), s->flat.wcopies.size() * sizeof(float));
    return RT_OK;
}

rt_status rt_scene_whitted_orders(const rt_scene* s, float* out, uint64_t* n_floats)
{
    if (!s || !s->built) return RT_ERR_STATE;
    if (!n_floats) return RT_ERR_INVALID;
    *n_floats = s->flat.worders.size();
    if (out && !s->flat.worders.empty()) std::memcpy(out, s->flat.worders.data(), s->flat.worders.size() * sizeof(float));
    return RT_OK;
}

rt_status rt_scene_whitted_orders_half(const rt_scene* s, uint32_t* out, uint64_t* n_words)
{
    if (!s || !s->built) return RT_ERR_STATE;
    if (!n_words) return RT_ERR_INVALID;
    *n_words = s->flat.worders_h.size();
    if (out && !s->flat.worders_h.empty()) std::memcpy(out, s->flat.worders_h.data(), s->flat.worders_h.size() * sizeof(uint32_t));
    return RT_OK;
}

// ------------------------------------------------------------------ context
rt_status rt_create(rt_ctx** out, const rt_device_cfg* cfg)
{
    if (!out) return RT_ERR_INVALID;
    *out = nullptr;
    rt_ctx* c = new (std::nothrow) rt_ctx;
    if (!c) return RT_ERR_OOM;
    c->device = cfg ? cfg->device : 0;
    if (const char* e = rt_knob("RT_THRESH")) c->thresh = c->vthresh = c->sthresh = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = rt_knob("RT_STEPS")) c->steps = c->vsteps = c->ssteps = std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 10));
    if (const char* e = rt_knob("RT_LDS_LEVELS")) c->lds_levels_force = (int)std::strtol(e, nullptr, 10);
    if (const char* e = rt_knob("RT_BRUTE")) c->brute = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_SKY_BITS")) c->sky_bits = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_DIRECT_DIV2")) c->direct_div2 = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_VERTEX")) c->vertex = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_SPLIT")) c->split = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_WALK_ORDER")) c->walk_order = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_WH_ORDER")) c->wh_order = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_WH_HALF")) c->wh_half = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_SEG_PARTS_OFF")) c->seg_parts_off = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_SEG_MIN_PARTS")) c->seg_min_parts = (uint32_t)std::max(1ul, std::strtoul(e, nullptr, 10));
    if (const char* e = rt_knob("RT_SEG_PART_LF")) c->seg_part_lf = (uint32_t)std::min(6ul, std::strtoul(e, nullptr, 10));
    if (const char* e = rt_knob("RT_SEG_TAIL_PARTS")) c->seg_tail_parts = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = rt_knob("RT_SEG_TAIL_EXTRA")) c->seg_tail_extra = (uint32_t)std::min(6ul, std::strtoul(e, nullptr, 10));
    if (const char* e = rt_knob("RT_WORK_QUEUES")) c->n_work_queues = std::strtoul(e, nullptr, 10) >= 8 ? 8u : 1u;
    if (const char* e = rt_knob("RT_VERTEX_BVH")) c->vertex_bvh = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_LBUF_PIXEL_MAJOR")) c->lbuf_pm = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_FORCE_WALK")) c->force_walk = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_RING_PACK")) c->ring_pack = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = rt_knob("RT_BVH_PREPASS")) c->bvh_prepass = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_PRE_DEFER")) c->pre_defer_walk = std::strtoul(e, nullptr, 10) != 0;
    if (const char* e = rt_knob("RT_LDS_PAD")) c->lds_pad = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = rt_knob("RT_CHUNKS")) c->force_chunks = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = rt_knob("RT_ITEMS_PER_LANE")) c->items_per_lane = std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 10));
    if (const char* e = rt_knob("RT_MIN_PX_PER_LANE")) c->min_px_per_lane = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = rt_knob("RT_MIN_CHUNK_FRAMES")) c->min_chunk_frames = std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 10));
    if (const char* e = rt_knob("RT_LBUF_BUDGET_MB")) {
        c->lbuf_budget = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) << 20;
        c->lbuf_budget_env = true;
    }
    if (const char* e = rt_knob("RT_STACK_DEPTH")) c->stack_depth_force = std::min<uint32_t>(kStackDepthMax, (uint32_t)std::strtoul(e, nullptr, 10));
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) { rt_status s = hip_fail(c, e, "hipSetDevice"); std::fprintf(stderr, "rt_create: %s\n", c->err.c_str()); delete c; return s; }
    if (cfg && cfg->stream) {
        c->stream = (hipStream_t)cfg->stream;
    } else {
        e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e != hipSuccess) { rt_status s = hip_fail(c, e, "hipStreamCreate"); delete c; return s; }
        c->own_stream = true;
    }
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess || hipEventCreate(&c->ev2) != hipSuccess ||
        hipEventCreate(&c->ev3) != hipSuccess ||
        hipMalloc((void**)&c->d_counter, kWorkCounterBytes) != hipSuccess || hipMalloc((void**)&c->d_counters, kCounterWords * 8) != hipSuccess ||
        hipHostMalloc((void**)&c->h_ovf, 2 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
        c->err = "context allocation failed";
        rt_destroy(c);
        return RT_ERR_HIP;
    }
    if (hipMemset(c->d_counters, 0, kCounterWords * 8) != hipSuccess) { c->err = "hipMemset failed"; rt_destroy(c); return RT_ERR_HIP; }
    // persistent grid: every CU filled to the kernel's occupancy
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) { c->err = "hipGetDeviceProperties failed"; rt_destroy(c); return RT_ERR_HIP; }
    // all instantiations are sized by the most register-hungry one so one stack serves every mode;
    // the occupancy query is advisory only: the kernel has no grid barrier, a non-resident block
    // simply starts later and finds the queue drained
    c->n_cu = (uint32_t)prop.multiProcessorCount;
    int ex_max = 1;
    for (int ex = 0; ex < 2; ++ex)
        for (int cn = 0; cn < 2; ++cn) {
            int b = rt_megakernel_occupancy(ex, cn, false, 256, 0);
            c->occ_global[ex][cn] = b > 0 ? b : 2;
            if (ex) ex_max = std::max(ex_max, c->occ_global[ex][cn]);
        }
    ex_max = std::max({ex_max, rt_coherent_occupancy(true, false, true, 256, 0), rt_coherent_occupancy(true, true, false, 256, 0),
                       rt_coherent_occupancy(true, true, true, 256, 0)});
    c->block = 256;
    // the EXACT fold stack is sized for the largest grid any mode launches (LDS staging never
    // raises occupancy above the register-limited value)
    c->grid = c->n_cu * (uint32_t)ex_max;
    c->total_threads = c->grid * c->block;
    *out = c;
    return RT_OK;
}

void rt_destroy(rt_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    dfree(c->d_sboxes); dfree(c->d_stri); dfree(c->d_wcopies); dfree(c->d_worders);
    dfree(c->d_nodes); dfree(c->d_tris); dfree(c->d_mats); dfree(c->d_lnodes); dfree(c->d_ltris); dfree(c->d_lboxes); dfree(c->d_wmats); dfree(c->d_plights);
    dfree(c->d_tabc);
    dfree(c->d_went); dfree(c->d_wtris);
    dfree(c->d_gb_color); dfree(c->d_gb_pos); dfree(c->d_gb_nrm); dfree(c->d_spatial); dfree(c->d_temporal); dfree(c->d_prev_color);
    dfree(c->d_gb_prim); dfree(c->d_prev_prim); dfree(c->d_dn_rgba); dfree(c->d_lbuf); dfree(c->d_sky);
    dfree(c->d_crec); dfree(c->d_seg_list); dfree(c->d_tile_boxes);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    if (c->ev3) (void)hipEventDestroy(c->ev3);
    dfree(c->d_accum); dfree(c->d_rgba); dfree(c->d_counter); dfree(c->d_counters); dfree(c->d_stack_ld); dfree(c->d_stack_mat);
    dfree(c->d_ovf); dfree(c->d_rs_stack); dfree(c->d_rs_mat);
    if (c->h_ovf) (void)hipHostFree(c->h_ovf);
    for (hipEvent_t e : c->kev) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

rt_status rt_upload_scene(rt_ctx* c, const rt_scene* s)
{
    if (!c || !s) return RT_ERR_INVALID;
    if (!s->built) { c->err = "scene not built (rt_scene_build)"; return RT_ERR_STATE; }
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipStreamSynchronize(c->stream));
    rt_status r;
    if ((r = upload(c, c->d_nodes, s->flat.nodes)) != RT_OK) return r;
    if ((r = upload(c, c->d_tris, s->flat.tris)) != RT_OK) return r;
    if ((r = upload(c, c->d_mats, s->flat.mats)) != RT_OK) return r;
    if ((r = upload(c, c->d_lnodes, s->flat.lnodes)) != RT_OK) return r;
    if ((r = upload(c, c->d_ltris, s->flat.ltris)) != RT_OK) return r;
    if ((r = upload(c, c->d_lboxes, s->flat.lboxes)) != RT_OK) return r;
    if ((r = upload(c, c->d_sboxes, s->flat.sboxes)) != RT_OK) return r;
    if ((r = upload(c, c->d_stri, s->flat.stri)) != RT_OK) return r;
    {   // the near-first orderings (8 x the walked subtree's nodes: 40.7 MB at C5) only where the BVH variant walks them
        static const std::vector<float> kNone;
        const bool walks = c->vertex && c->vertex_bvh && c->split && c->walk_order && !c->force_walk;
        if ((r = upload(c, c->d_wcopies, walks ? s->flat.wcopies : kNone)) != RT_OK) return r;
        // (8 x the whole tree's nodes for a Whitted scene: 5.8 MB at C3)
        if ((r = upload(c, c->d_worders, c->wh_order ? s->flat.worders : kNone)) != RT_OK) return r;
        // (half of that in 16-byte nodes, when the Whitted walk takes them: 2.9 MB at C3)
        static const std::vector<uint32_t> kNoneU;
        if ((r = upload(c, c->d_worders_h, c->wh_order && c->wh_half ? s->flat.worders_h : kNoneU)) != RT_OK) return r;
    }
    c->split_root = s->flat.split_root;
    c->split_end = s->flat.split_end;
    c->n_sboxes = (uint32_t)(s->flat.sboxes.size() / 8);
    c->n_sleaves = (uint32_t)s->flat.stri.size();
    {   // the vertices, when the Whitted walk takes the half-plane orderings (RT_WH_HALF)
        static const std::vector<float> kNoneF;
        if ((r = upload(c, c->d_tabc, c->wh_order && c->wh_half ? s->flat.tabc : kNoneF)) != RT_OK) return r;
    }
    if ((r = upload(c, c->d_wmats, s->flat.wmats)) != RT_OK) return r;
    if ((r = upload(c, c->d_plights, s->flat.plights)) != RT_OK) return r;
    if ((r = upload(c, c->d_went, s->flat.went)) != RT_OK) return r;
    if ((r = upload(c, c->d_wtris, s->flat.wtris)) != RT_OK) return r;
    c->hdr = s->flat.hdr;
    c->has_scene = true;
    return RT_OK;
}

namespace {
// the LBVH build's inputs from a built scene: the vertices (9 floats) and the records (16 floats) of each
// triangle, in the host tree's DFS order (the build's order does not depend on it)
bool lbvh_inputs(const rt_scene* s, std::vector<float>& verts)
{
    const uint32_t n = s->flat.hdr.n_tris;
    if (n < 2 || s->flat.dbg_tri_f.size() < 13 * (size_t)n || s->flat.tris.size() < 16 * (size_t)n) return false;
    verts.resize(9 * (size_t)n);
    for (uint32_t i = 0; i < n; ++i) std::memcpy(&verts[9 * (size_t)i], &s->flat.dbg_tri_f[13 * (size_t)i], 9 * sizeof(float));
    return true;
}
}  // namespace

rt_status rt_scene_lbvh_host(const rt_scene* s, float* nodes, float* tris)
{
    if (!s || !nodes || !tris) return RT_ERR_INVALID;
    if (!s->built) return RT_ERR_STATE;
    std::vector<float> verts, nv, tv;
    if (!lbvh_inputs(s, verts)) return RT_ERR_INVALID;
    if (!lbvh_build_host(s->flat.hdr.n_tris, verts.data(), s->flat.tris.data(), nv, tv)) return RT_ERR_INVALID;
    std::memcpy(nodes, nv.data(), nv.size() * sizeof(float));
    std::memcpy(tris, tv.data(), tv.size() * sizeof(float));
    return RT_OK;
}

rt_status rt_upload_scene_gpu_bvh(rt_ctx* c, const rt_scene* s, float* build_ms)
{
    if (!c || !s) return RT_ERR_INVALID;
    if (!s->built) { c->err = "scene not built (rt_scene_build)"; return RT_ERR_STATE; }
    std::vector<float> verts;
    if (s->flat.hdr.n_spheres > 0) { c->err = "the GPU BVH build takes triangle meshes only (the scene has spheres)"; return RT_ERR_INVALID; }
    if (!lbvh_inputs(s, verts)) { c->err = "the GPU BVH build needs >= 2 triangles"; return RT_ERR_INVALID; }
    if (s->flat.hdr.n_tris >= (1u << 30)) { c->err = "the GPU BVH build takes < 2^30 triangles (node ids are int)"; return RT_ERR_INVALID; }
    rt_status r = rt_upload_scene(c, s);   // materials, light tables, ... (the host tree is replaced below)
    if (r != RT_OK) return r;
    const uint32_t n = s->flat.hdr.n_tris, m = 2 * n - 1;
    float* d_verts = nullptr;
    float4 *d_nodes = nullptr, *d_tris = nullptr;
    // the build is timed with its own events: the context's ev0/ev1 time renders, whose pending stats
    // (rt_get_stats) must not pick up the build's time
    hipEvent_t b0 = nullptr, b1 = nullptr;
    auto fail = [&](hipError_t e) {
        dfree(d_verts); dfree(d_nodes); dfree(d_tris);
        if (b0) (void)hipEventDestroy(b0);
        if (b1) (void)hipEventDestroy(b1);
        return hip_fail(c, e, "rt_upload_scene_gpu_bvh");
    };
    hipError_t e;
    if ((e = hipEventCreate(&b0)) != hipSuccess) return fail(e);
    if ((e = hipEventCreate(&b1)) != hipSuccess) return fail(e);
    if ((e = hipMalloc((void**)&d_verts, verts.size() * sizeof(float))) != hipSuccess) return fail(e);
    if ((e = hipMalloc((void**)&d_nodes, 2 * (size_t)m * sizeof(float4))) != hipSuccess) return fail(e);
    if ((e = hipMalloc((void**)&d_tris, 4 * (size_t)n * sizeof(float4))) != hipSuccess) return fail(e);
    if ((e = hipMemcpy(d_verts, verts.data(), verts.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess) return fail(e);
    if ((e = hipEventRecord(b0, c->stream)) != hipSuccess) return fail(e);
    if ((e = lbvh_build_device(n, d_verts, c->d_tris, d_nodes, d_tris, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipEventRecord(b1, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipEventSynchronize(b1)) != hipSuccess) return fail(e);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, b0, b1);
    if (build_ms) *build_ms = ms;
    (void)hipEventDestroy(b0);
    (void)hipEventDestroy(b1);
    dfree(d_verts);
    dfree(c->d_nodes); dfree(c->d_tris);
    c->d_nodes = d_nodes; c->d_tris = d_tris;
    // the BVH-walking kernels: no leaf-box table, no compact tree
    dfree(c->d_lboxes); dfree(c->d_tabc);
    dfree(c->d_sboxes); dfree(c->d_stri); dfree(c->d_wcopies); dfree(c->d_worders); dfree(c->d_worders_h);   // the split and orderings refer to the host tree's node order
    c->split_root = c->split_end = c->n_sboxes = c->n_sleaves = 0;
    c->hdr.n_nodes = m;
    c->hdr.n_lboxes = 0;
    c->hdr.has_vboxes = 0;
    return RT_OK;
}

rt_status rt_debug_scene_arrays(rt_ctx* c, float* nodes, uint32_t n_node_floats, float* tris, uint32_t n_tri_floats)
{
    if (!c) return RT_ERR_INVALID;
    if (!c->has_scene) return RT_ERR_STATE;
    HIPC(c, hipStreamSynchronize(c->stream));
    const size_t nn = std::min<size_t>(n_node_floats, 8 * (size_t)c->hdr.n_nodes), nt = std::min<size_t>(n_tri_floats, 16 * (size_t)c->hdr.n_tris);
    if (nodes && nn) HIPC(c, hipMemcpy(nodes, c->d_nodes, nn * sizeof(float), hipMemcpyDeviceToHost));
    if (tris && nt) HIPC(c, hipMemcpy(tris, c->d_tris, nt * sizeof(float), hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_resize(rt_ctx* c, uint32_t W, uint32_t H, uint32_t band, uint32_t rank, uint32_t nranks)
{
    if (!c || W == 0 || H == 0 || band == 0 || nranks == 0 || rank >= nranks) return RT_ERR_INVALID;
    if (W > 65536 || H > 65536) { c->err = "viewport too large"; return RT_ERR_INVALID; }
    HIPC(c, hipSetDevice(c->device));
    const uint32_t rows = count_local_rows(H, band, rank, nranks);
    if (W == c->W && H == c->H && band == c->band && rank == c->rank && nranks == c->nranks && c->d_accum) return RT_OK;
    HIPC(c, hipStreamSynchronize(c->stream));
    dfree(c->d_accum); dfree(c->d_rgba);
    c->W = W; c->H = H; c->band = band; c->rank = rank; c->nranks = nranks; c->local_rows = rows;
    const size_t npx = (size_t)std::max<uint32_t>(rows, 1) * W;
    HIPC(c, hipMalloc((void**)&c->d_accum, npx * sizeof(float4)));
    HIPC(c, hipMalloc((void**)&c->d_rgba, npx * sizeof(uint32_t)));
    HIPC(c, hipMemsetAsync(c->d_accum, 0, npx * sizeof(float4), c->stream));
    HIPC(c, hipMemsetAsync(c->d_rgba, 0, npx * sizeof(uint32_t), c->stream));
    return RT_OK;
}

uint32_t rt_local_rows(const rt_ctx* c) { return c ? c->local_rows : 0; }

rt_status rt_render(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, uint32_t* out_rgba, float* out_accum)
{
    if (!c || !cam || !p) return RT_ERR_INVALID;
    if (!c->has_scene) { c->err = "no scene uploaded"; return RT_ERR_STATE; }
    if (!c->d_accum) { c->err = "no viewport (rt_resize)"; return RT_ERR_STATE; }
    if (c->hdr.n_went > 0 && !(p->flags & RT_RENDER_WHITTED)) { c->err = "a Whitted world renders with RT_RENDER_WHITTED"; return RT_ERR_INVALID; }
    if (p->first_frame == 0) { c->err = "first_frame is 1-based"; return RT_ERR_INVALID; }
    // a survival probability >= 1 never terminates a path in a closed scene (the reference recurses
    // until its stack overflows); reject it, and NaN
    if (!(p->flags & RT_RENDER_WHITTED) && !(p->rr >= 0.0f && p->rr < 1.0f)) { c->err = "rr must be in [0, 1)"; return RT_ERR_INVALID; }
    HIPC(c, hipSetDevice(c->device));
    const bool whitted = (p->flags & RT_RENDER_WHITTED) != 0;
    if (whitted && c->hdr.n_spheres > 0) { c->err = "Whitted renders take triangle meshes (the path tracer's spheres: rt_scene_add_sphere)"; return RT_ERR_INVALID; }
    const bool exact = !whitted && (p->flags & RT_RENDER_EXACT) != 0, count = (p->flags & RT_RENDER_COUNT) != 0;
    if (exact) {
        // the fold stack / ring, sized from rr (reallocated when a render needs more levels)
        const uint32_t want = c->stack_depth_force ? std::max<uint32_t>(1, c->stack_depth_force) : stack_levels_for(p->rr);
        // (the vertex kernel indexes the ring in 32 bits: lane * depth + position, rt_coherent.hip RING_AT)
        if ((uint64_t)want * c->total_threads >= (1ull << 32)) { c->err = "fold ring index exceeds 32 bits"; return RT_ERR_INVALID; }
        if (!c->d_stack_ld || want > c->stack_depth || (c->stack_depth_force && want != c->stack_depth)) {
            HIPC(c, hipStreamSynchronize(c->stream));
            dfree(c->d_stack_ld); dfree(c->d_stack_mat);
            c->stack_depth = 0;
            HIPC(c, hipMalloc((void**)&c->d_stack_ld, (size_t)want * c->total_threads * sizeof(float4)));
            HIPC(c, hipMalloc((void**)&c->d_stack_mat, (size_t)want * c->total_threads * sizeof(int32_t)));
            c->stack_depth = want;
        }
        if (!c->d_ovf) {
            HIPC(c, hipMalloc((void**)&c->d_ovf, (size_t)c->ovf_cap * sizeof(uint4)));
            HIPC(c, hipMalloc((void**)&c->d_rs_stack, (size_t)kResampleDepth * c->rs_threads * sizeof(float4)));
            HIPC(c, hipMalloc((void**)&c->d_rs_mat, (size_t)kResampleDepth * c->rs_threads * sizeof(int32_t)));
        }
    }
    KParams P{};
    P.nodes = c->d_nodes; P.n_nodes = c->hdr.n_nodes;
    P.tris = c->d_tris; P.n_tris = c->hdr.n_tris;
    P.mats = c->d_mats; P.n_mats = c->hdr.n_mats;
    P.lnodes = c->d_lnodes; P.n_lnodes = c->hdr.n_lnodes;
    P.ltris = c->d_ltris; P.n_ltris = c->hdr.n_ltris;
    P.lboxes = c->d_lboxes; P.n_lboxes = c->brute ? c->hdr.n_lboxes : 0;
    if (c->split && c->split_root != 0 && P.n_lboxes == 0) {
        P.sboxes = c->d_sboxes; P.stri = c->d_stri; P.n_sboxes = c->n_sboxes;
        P.split_root = c->split_root; P.split_end = c->split_end; P.n_split_leaves = c->n_sleaves;
        // (not with the forced full walk: it walks the original order)
        if (c->walk_order && c->d_wcopies && !c->force_walk) {
            // offset so that node k of an ordering is at [2 * k] (k >= split_root; computed as an integer)
            P.wcopies = reinterpret_cast<const float4*>(reinterpret_cast<uintptr_t>(c->d_wcopies) - (uintptr_t)c->split_root * 2u * sizeof(float4));
            P.wcopy_stride = 2u * (c->split_end - c->split_root);
        }
    }
    P.worders = c->d_worders;
    P.worders_h = (c->d_worders && c->d_worders_h && c->hdr.has_vboxes && c->d_tabc) ? c->d_worders_h : nullptr;
    P.tabc = c->d_tabc;
    P.light_area = c->hdr.light_area;
    std::memcpy(P.light_emission, c->hdr.light_emission, sizeof P.light_emission);
    P.has_light = c->hdr.light_mesh >= 0 && c->hdr.n_ltris > 0;
    P.wmats = c->d_wmats; P.plights = c->d_plights; P.n_plights = c->hdr.n_plights;
    P.went = c->d_went; P.wtris = c->d_wtris; P.n_went = c->hdr.n_went;
    P.max_bounce_depth = c->hdr.max_bounce_depth; P.intersection_correction = c->hdr.intersection_correction;
    std::memcpy(P.sky, c->hdr.sky, sizeof P.sky);
    std::memcpy(P.cam_pos, cam->position, sizeof P.cam_pos);
    std::memcpy(P.iproj, cam->inv_projection, sizeof P.iproj);
    std::memcpy(P.iview, cam->inv_view, sizeof P.iview);
    P.W = c->W; P.H = c->H;
    P.first_frame = p->first_frame; P.n_frames = p->n_frames;
    P.seed = p->seed; P.rr = p->rr;
    {   // IEEE single divisions on the host: exactly the kernels' constants and correctly rounded reciprocals
        const float pdf = 1.0f / (2.0f * 3.141592653589793f);
        P.y_pdf = 1.0f / pdf;
        P.y_rr = p->rr > 0.0f ? 1.0f / p->rr : 0.0f;
        P.rr_fast = (p->rr >= 0x1p-20f && p->rr < 1.0f) ? 1u : 0u;
        P.wh_fast = (c->W >= 1u && c->W < (1u << 20) && c->H >= 1u && c->H < (1u << 20)) ? 1u : 0u;
        P.lpdf = 1.0f / c->hdr.light_area;
        P.y_lpdf = 1.0f / P.lpdf;
        // the direct term's (X / dist^2) / lpdf on Markstein's path (rt_coherent.hip): the light PDF must lie in
        // div_fast's verified divisor range [2^-20, 2^20) (rt_device.h div2_core); RT_DIRECT_DIV2=0 is the A/B
        P.lpdf_fast = (c->direct_div2 && P.lpdf >= 0x1p-20f && P.lpdf < 0x1p20f) ? 1u : 0u;
        P.y_w = 1.0f / (float)c->W; P.y_h = 1.0f / (float)c->H;
    }
    P.band = c->band; P.rank = c->rank; P.nranks = c->nranks; P.n_local_rows = c->local_rows;
    P.tiles_x = (c->W + 7) / 8;
    P.r_band = (float)(1.0 / (double)std::max<uint32_t>(1u, P.band));
    P.r_tiles_x = (float)(1.0 / (double)std::max<uint32_t>(1u, P.tiles_x));
    const uint64_t items = (uint64_t)((c->local_rows + 7) / 8) * P.tiles_x * 64;
    if (items >= 0xFFFFFFFFull) { c->err = "image too large for one launch"; return RT_ERR_INVALID; }
    P.n_items = (uint32_t)items;
    P.accum = c->d_accum; P.rgba = c->d_rgba;
    P.work_counter = c->d_counter;
    P.work_queues = c->d_counter + 32; P.n_work_queues = c->n_work_queues;
    P.stack_ld = c->d_stack_ld; P.stack_mat = c->d_stack_mat; P.stack_depth = exact ? c->stack_depth : 0;
    // read by the vertex kernel only; set below for its BVH variant (C5 198.6 vs 203.4 ms; the leaf-box
    // variant measured 0.6 % slower with it: C4 346.8 vs 344.5 ms)
    P.ring_pack = 0u;
    P.total_threads = c->total_threads;
    P.counters = c->d_counters;
    P.ovf_list = exact ? c->d_ovf : nullptr; P.ovf_cap = c->ovf_cap;
    P.rs_stack = c->d_rs_stack; P.rs_mat = c->d_rs_mat;
    P.thresh = c->thresh; P.steps = c->steps;
    P.force_walk = c->force_walk ? 1u : 0u;
    P.lds_pad = c->lds_pad;
    if (c->gb_next) {
        P.gb_color = c->d_gb_color; P.gb_pos = c->d_gb_pos; P.gb_nrm = c->d_gb_nrm; P.gb_prim = c->d_gb_prim; P.gb_clamp = c->gb_clamp;
    }
    // small scenes are staged into LDS (one copy per workgroup)
    const size_t lds_bytes = rt_scene_lds_bytes(P);
    const bool lds = (p->flags & RT_RENDER_GLOBAL_SCENE) == 0 && lds_bytes <= kMaxLdsScene;
    P.lds_scene_quads = lds ? (uint32_t)(lds_bytes / sizeof(float4)) : 0;
    // small scenes with decisive leaf boxes: the vertex-synchronous kernel (rt_coherent.hip)
    // any other path scene: its BVH variant, the scene in HBM (RT_VERTEX_BVH=0: the megakernel)
    // (the vertex kernel packs a material index in 14 bits beside the path's vertex count, rt_coherent.hip VS_MAT)
    const bool coh_box = c->vertex && P.n_lboxes > 0 && lds && !count && !c->gb_next && !whitted && P.n_mats < (1u << 14);
    // (the camera pre-pass's records carry a triangle index in 19 bits, rt_kernels.h crec: only the leaf-box
    // variant runs the pre-pass, and its scenes have <= 64 triangles; the BVH variant carries full indices)
    // (the BVH variant stages the materials and light tables in LDS with its lane state: a scene whose tables
    // exceed kMaxBvhSmallLds renders on the megakernel)
    const size_t bvh_small_bytes = (size_t)(2 * P.n_mats + P.n_lnodes + 4 * P.n_ltris + 3 * P.n_split_leaves) * sizeof(float4);
    // what keeps a path scene off the BVH variant, RT_KERNEL_REASON_DEFAULT when nothing does: ONE list of
    // predicates, so that every fallback to the megakernel reports its own reason (rt_stats.kernel_reason;
    // ADVICE r04/r05)
    const uint32_t bvh_block = [&]() -> uint32_t {
        if (count || c->gb_next) return RT_KERNEL_REASON_MODE;
        if (c->hdr.n_spheres > 0) return RT_KERNEL_REASON_SPHERES;   // the vertex kernel's leaves are triangles
        if (!c->vertex || !c->vertex_bvh) return RT_KERNEL_REASON_KNOB;
        if (P.n_tris >= (1u << 31)) return RT_KERNEL_REASON_TRIANGLES;
        if (P.n_mats >= (1u << 14)) return RT_KERNEL_REASON_MATERIALS;
        if (bvh_small_bytes > kMaxBvhSmallLds) return RT_KERNEL_REASON_TABLES_LDS;
        return RT_KERNEL_REASON_DEFAULT;
    }();
    const bool coh_bvh = !coh_box && !whitted && bvh_block == RT_KERNEL_REASON_DEFAULT;
    const bool coh = coh_box || coh_bvh;
    uint32_t reason = RT_KERNEL_REASON_DEFAULT;
    if (!coh && !whitted) reason = bvh_block;
    else if (coh_bvh && !c->brute && c->hdr.n_lboxes > 0) reason = RT_KERNEL_REASON_KNOB;   // RT_BRUTE=0: a small scene on the BVH variant
    // the camera pre-pass: the leaf-box variant always; the BVH variant for a split scene, whose camera rays are
    // traced like the path kernel's split phase (records carry the triangle in 19 bits, rt_kernels.h crec)
    const bool prepass = coh_box || (coh_bvh && c->bvh_prepass && P.split_root != 0u && P.n_tris < (1u << 19) - 1u);
    P.pre_defer_walk = c->pre_defer_walk ? 1u : 0u;
    auto occupancy = [&](size_t bytes) {
        return coh ? rt_coherent_occupancy(exact, coh_bvh, prepass, (int)c->block, bytes) : rt_megakernel_occupancy(exact, count, lds, (int)c->block, bytes);
    };
    const size_t lane_bytes = coh ? rt_coherent_lane_state_lds_bytes(exact, P.has_light != 0, coh_bvh) : rt_lane_state_lds_bytes(exact);
    if (coh_box) {   // the vertex kernel reads the leaf boxes with scalar loads and the nodes from HBM: neither is staged
        P.lds_scene_quads -= 2 * P.n_lboxes + 2 * P.n_nodes;
    }
    if (coh_bvh) {   // the BVH variant reads the nodes and triangles from HBM; the materials and the light
        // tables are in LDS (C5: 21 quads), the split's outside triangles (<= 32 x 3 quads) after them
        P.lds_scene_quads = (uint32_t)(bvh_small_bytes / sizeof(float4));
        P.ring_pack = (c->ring_pack >= 1 && c->hdr.n_mats <= 8) ? 1u : 0u;
        P.thresh = P.split_root != 0u ? c->sthresh : c->vthresh;
        P.steps = P.split_root != 0u ? c->ssteps : c->vsteps;
    }
    if (coh_box && exact) P.ring_pack = (c->ring_pack >= 2 && c->hdr.n_mats <= 8) ? 1u : 0u;
    // EXACT: as many fold-stack levels in LDS as fit beside the scene without costing occupancy
    // (4 workgroups of 256 lanes per CU = 40 KiB each), at most 8
    P.lds_levels = 0;
    if (exact && !coh && (p->flags & RT_RENDER_GLOBAL_STACK) == 0) {   // the vertex kernel's fold ring is in HBM
        const size_t used = (lds ? lds_bytes : 0) + lane_bytes + c->lds_pad;
        const int occ0 = occupancy(used);
        for (uint32_t lv = 8; lv > 0; --lv)
            if (occupancy(used + rt_stack_lds_bytes(lv)) >= occ0) { P.lds_levels = lv; break; }
    }
    if (exact && !coh && c->lds_levels_force >= 0) P.lds_levels = std::min<uint32_t>((uint32_t)c->lds_levels_force, P.stack_depth);
    size_t shmem = ((lds || coh_bvh) ? (size_t)P.lds_scene_quads * sizeof(float4) : 0) + (exact ? rt_stack_lds_bytes(P.lds_levels) : 0) + lane_bytes + c->lds_pad;
    int bpc = occupancy(shmem);
    c->stats.kernel_reason = reason;
    if (bpc <= 0) bpc = c->occ_global[exact][count];
    uint32_t grid = c->n_cu * (uint32_t)bpc;
    if (exact) grid = std::min(grid, c->grid);   // the fold stack holds c->total_threads lanes
    const uint64_t px_local = (uint64_t)c->local_rows * c->W;
    const uint64_t items_px = P.n_items;   // 8x8-tile-padded pixel items
    c->last_flags = p->flags;
    // (counters[13..14], the EXACT overflow outcome, are not reset here: they accumulate over renders
    // until a synchronisation point reads them (check_overflow), so an earlier asynchronous render's loss
    // is never masked by a later clean one)
    HIPC(c, hipMemsetAsync(c->d_counters, 0, 13 * 8, c->stream));
    HIPC(c, hipMemsetAsync(c->d_counters + 15, 0, (kCounterWords - 15) * 8, c->stream));
    c->kev_used = 0;
    c->kev_prepass = false;
    if (p->n_frames > 0 && c->local_rows > 0) {
        HIPC(c, hipEventRecord(c->ev0, c->stream));
        if (whitted && c->hdr.n_went > 0) {
            HIPC(c, rt_launch_whitted_world(P, count, c->stream, &grid));
        } else if (whitted) {
            HIPC(c, rt_launch_whitted(P, count, c->stream, &grid));
        } else {
            // Frame chunks: a lane renders one work item's frames in order, so a launch with few items
            // per lane waits on the costliest pixels' sequential frames (the tail; a row band of a
            // multi-GPU frame is 1 pixel per lane).  Each pixel's frames are split into chunks, about
            // items_per_lane items per lane: chunk 0 accumulates, later chunks park their samples
            // (12 B each) for the in-order finalize pass.  The parked samples of one launch are capped
            // by lbuf_budget; a longer render runs as several passes over consecutive frame ranges
            // (first_frame continues the accumulation, so passes are exact too).
            const uint64_t lanes = (uint64_t)grid * c->block;
            uint32_t want = 1;
            if (!c->gb_next && p->n_frames > 1 && px_local > 0) {
                if (c->force_chunks) want = std::min(c->force_chunks, p->n_frames);
                else if (px_local < (uint64_t)c->min_px_per_lane * lanes)
                    want = (uint32_t)std::min<uint64_t>({(uint64_t)p->n_frames, std::max<uint64_t>(1, p->n_frames / c->min_chunk_frames),
                                                         ((uint64_t)c->items_per_lane * lanes + px_local - 1) / px_local});
            }
            // the vertex kernel parks every frame (finalize accumulates them); the megakernel parks the
            // frames of chunks >= 1
            const bool park_all = coh;
            uint32_t passes = 1;
            if (!c->lbuf_budget_env) {
                // parked-sample budget from the device's free memory (the current buffer counts as free):
                // at most 96 GB, at most 3/4 of what is free
                size_t fr = 0, tot = 0;
                HIPC(c, hipMemGetInfo(&fr, &tot));
                c->lbuf_budget = std::max<uint64_t>(64ull << 20, std::min<uint64_t>(96ull << 30, (fr + c->lbuf_floats * sizeof(float) + c->crec_quads * sizeof(float4)) / 4 * 3));
            }
            if (want > 1 || park_all) {
                // the bytes one pass of nf frames allocates: parked samples (12 B, frames in 4-frame blocks) and,
                // for the leaf-box variant, the camera records (16 B per 8x8-padded tile pixel and frame, the
                // frames rounded up to whole pre-pass segments of min(64, the next power of two) frames)
                auto pass_bytes = [&](uint64_t nf) {
                    uint64_t b = 12ull * px_local * ((nf + 3) & ~3ull);
                    if (prepass) {
                        uint64_t sf = 1;
                        while (sf < nf && sf < 64) sf <<= 1;
                        b += 16ull * items_px * ((nf + sf - 1) / sf * sf);
                    }
                    return b;
                };
                const uint64_t nfr = p->n_frames;
                passes = (uint32_t)std::min<uint64_t>(nfr, std::max<uint64_t>(1, pass_bytes(nfr) / c->lbuf_budget));
                while (passes < nfr && pass_bytes((nfr + passes - 1) / passes) > c->lbuf_budget) ++passes;
            }
            uint32_t done = 0;
            for (uint32_t pass = 0; pass < passes; ++pass) {
                const uint32_t nf = (p->n_frames - done + (passes - pass) - 1) / (passes - pass);
                KParams Q = P;
                Q.first_frame = p->first_frame + done;
                Q.n_frames = nf;
                uint32_t n_chunks = std::min(want, nf);
                const uint32_t F = (nf + n_chunks - 1) / n_chunks;
                n_chunks = (nf + F - 1) / F;
                Q.n_chunks = n_chunks; Q.chunk_frames = F; Q.items_per_chunk = (uint32_t)items_px;
                Q.park_all = park_all ? 1u : 0u;
                Q.lbuf_pixel_major = park_all && c->lbuf_pm ? 1u : 0u;
                // the 32-bit work counter runs past n_items by the last refills (each wave takes 64 items
                // per atomic until it sees the queue empty, a few refills at most): keep 4 per wave of headroom
                if (items_px * n_chunks + lanes * 4ull >= 0xFFFFFFFFull) { c->err = "too many work items for one launch"; return RT_ERR_INVALID; }
                Q.n_items = (uint32_t)(items_px * n_chunks);
                if (n_chunks > 1 || park_all) {
                    // 4-frame blocks of 12 floats per pixel (rt_kernels.hip)
                    const size_t plane = (size_t)px_local * (((park_all ? nf : nf - F) + 3u) & ~3u);
                    if (3 * plane > c->lbuf_floats) {
                        HIPC(c, hipStreamSynchronize(c->stream));
                        dfree(c->d_lbuf);
                        c->lbuf_floats = 0;
                        HIPC(c, hipMalloc((void**)&c->d_lbuf, 3 * plane * sizeof(float)));
                        c->lbuf_floats = 3 * plane;
                    }
                    Q.lbuf = c->d_lbuf; Q.lbuf_stride = (size_t)px_local;
                }
                HIPC(c, hipMemsetAsync(c->d_counter, 0, kWorkCounterBytes, c->stream));
                HIPC(c, hipMemsetAsync(c->d_counters + 3, 0, sizeof(unsigned long long), c->stream));   // this pass's overflow list
                while (c->kev.size() < 3 * (size_t)(pass + 1)) {
                    hipEvent_t e = nullptr;
                    HIPC(c, hipEventCreate(&e));
                    c->kev.push_back(e);
                }
                HIPC(c, hipEventRecord(c->kev[3 * pass], c->stream));
                if (prepass) {
                    // the camera pre-pass: segments of one 8x8 tile x F frames (F a power of two <= 64, rt_kernels.h crec)
                    Q.n_tiles = P.tiles_x * ((c->local_rows + 7) / 8);
                    uint32_t lf = 0;
                    while ((1u << lf) < nf && lf < 6) ++lf;
                    // a wave of the path kernel takes parts of segments: aim at 128 parts per wave, so the
                    // launch's tail (the waves' last parts) stays short, also when a pass has few tiles (a rank's
                    // row bands of a multi-GPU frame).  The segments stay long (the pre-pass's per-segment
                    // work -- the tile's box list, the record counter -- is paid once per 64 frames) and the
                    // path kernel splits each into 2^ps parts of its records, as fine as 16 frames' worth (a
                    // 64-frame segment in 4 parts whenever fewer than 128 per wave would remain: C4 at N = 1
                    // and 2 -0.7 %, N = 4 and 8 and C5 unchanged against round 4's rule of 32 parts per wave
                    // as fine as 8 frames, profiles/r05/ab/ab_seg_parts_*.jsonl; 8-frame parts cost more per
                    // part than the shorter tail saves; one-segment-per-part with 8-frame segments cost the
                    // pre-pass 0.9 ms more, profiles/r03/numbers/band_split*.jsonl)
                    const uint64_t waves = (uint64_t)grid * (c->block / 64u);
                    uint32_t ps = 0;
                    while (lf > ps + c->seg_part_lf && ((uint64_t)Q.n_tiles * ((nf + (1u << lf) - 1u) >> lf) << ps) < (uint64_t)c->seg_min_parts * waves) ++ps;
                    if (c->seg_parts_off) { lf -= ps; ps = 0; }   // A/B: short segments, one part each
                    Q.seg_part_shift = ps;
                    // the launch's tail: the list's last segments (each wave's last seg_tail_parts parts' worth)
                    // in 2^seg_tail_extra times as many parts, no finer than one frame's worth of records
                    Q.seg_tail_shift = std::min(ps + c->seg_tail_extra, lf);
                    Q.seg_tail_n = (uint32_t)std::min<uint64_t>(((uint64_t)c->seg_tail_parts * waves) >> ps, 0xFFFFFFFFull);
                    if (c->seg_parts_off) { Q.seg_tail_shift = 0; Q.seg_tail_n = 0; }   // the A/B baseline has no finer tail either
                    Q.seg_frames = 1u << lf;
                    Q.seg_shift = 6 + lf;
                    const uint64_t nseg = (uint64_t)Q.n_tiles * ((nf + Q.seg_frames - 1) / Q.seg_frames);
                    if (nseg >= (1ull << (32 - Q.seg_shift))) { c->err = "too many samples for one pass"; return RT_ERR_INVALID; }
                    Q.n_segments = (uint32_t)nseg;
                    Q.r_n_tiles = (float)(1.0 / (double)std::max<uint32_t>(1u, Q.n_tiles));
                    // the path kernel's record decode divides segment, tile and local row by uniform divisors
                    // (and multiplies: every factor < 2^24 -- the image's W and H too -- and every product, a pixel
                    // index at most, < 2^32)
                    Q.div24 = (nseg < (1u << 24) && Q.n_tiles < (1u << 24) && c->local_rows < (1u << 24) && Q.band < (1u << 24) &&
                               Q.tiles_x < (1u << 24) && c->W < (1u << 24) && c->H < (1u << 24) && Q.nranks < (1u << 24) &&
                               (uint64_t)c->W * c->H < (1ull << 32) && Q.n_frames < (1u << 24)) ? 1u : 0u;
                    if ((nseg << Q.seg_shift) > c->crec_quads) {
                        HIPC(c, hipStreamSynchronize(c->stream));
                        dfree(c->d_crec);
                        c->crec_quads = 0;
                        HIPC(c, hipMalloc((void**)&c->d_crec, (size_t)(nseg << Q.seg_shift) * sizeof(float4)));
                        c->crec_quads = (size_t)(nseg << Q.seg_shift);
                    }
                    if (nseg > c->seg_words) {
                        HIPC(c, hipStreamSynchronize(c->stream));
                        dfree(c->d_seg_list);
                        c->seg_words = 0;
                        HIPC(c, hipMalloc((void**)&c->d_seg_list, (size_t)nseg * sizeof(uint2)));
                        c->seg_words = (size_t)nseg;
                    }
                    if (Q.n_tiles > c->tile_words) {
                        HIPC(c, hipStreamSynchronize(c->stream));
                        dfree(c->d_tile_boxes);
                        c->tile_words = 0;
                        HIPC(c, hipMalloc((void**)&c->d_tile_boxes, (size_t)Q.n_tiles * 8));
                        c->tile_words = Q.n_tiles;
                    }
                    // sky bits: with segments of >= 32 frames (a segment then owns whole 32-frame words) the pre-pass
                    // sets a bit for a camera-ray miss instead of parking the sky's radiance (RT_SKY_BITS=0: park it)
                    Q.sky_bits = nullptr; Q.sky_words = 0;
                    if (c->sky_bits && park_all && Q.seg_frames >= 32u) {
                        const uint32_t sw = (nf + 31u) / 32u;
                        const size_t need = (size_t)sw * px_local;
                        if (need > c->sky_words_alloc) {
                            HIPC(c, hipStreamSynchronize(c->stream));
                            dfree(c->d_sky);
                            c->sky_words_alloc = 0;
                            HIPC(c, hipMalloc((void**)&c->d_sky, need * sizeof(uint32_t)));
                            c->sky_words_alloc = need;
                        }
                        Q.sky_bits = c->d_sky; Q.sky_words = sw;
                    }
                    Q.crec = c->d_crec; Q.seg_list = c->d_seg_list; Q.seg_list_n = c->d_counter + 1;
                    Q.tile_boxes = c->d_tile_boxes;
                    Q.n_chunks = (uint32_t)(nseg / Q.n_tiles);
                    const size_t pre_lds = coh_bvh ? (size_t)3 * P.n_split_leaves * sizeof(float4) : (size_t)(4 * P.n_tris + 2 * P.n_mats) * sizeof(float4);
                    HIPC(c, rt_launch_camera_prepass(Q, coh_bvh, pre_lds, c->stream));
                }
                HIPC(c, hipEventRecord(c->kev[3 * pass + 1], c->stream));
                if (coh) HIPC(c, rt_launch_coherent(Q, exact, coh_bvh, prepass, grid, c->block, shmem, c->stream));
                else HIPC(c, rt_launch_megakernel(Q, exact, count, lds, grid, c->block, c->stream));
                HIPC(c, hipEventRecord(c->kev[3 * pass + 2], c->stream));
                // EXACT vertex kernel: the samples whose path outgrew the ring, rendered again into their
                // parked slots (exits at once when none was listed)
                if (coh && exact) HIPC(c, rt_launch_resample(Q, c->rs_threads, c->stream));
                HIPC(c, rt_launch_finalize_chunks(Q, (uint32_t)px_local, c->stream));
                c->stats.n_chunks = Q.n_chunks;
                done += nf;
            }
            c->stats.n_passes = passes;
            c->kev_used = passes;
            c->kev_prepass = prepass;
        }
        c->stats.grid = grid;
        c->stats.kernel = whitted ? RT_KERNEL_WHITTED : (coh_bvh ? RT_KERNEL_VERTEX_BVH : coh ? RT_KERNEL_VERTEX : RT_KERNEL_MEGA);
        HIPC(c, hipEventRecord(c->ev1, c->stream));
        c->pending_stats = true;
        if (exact && !whitted) {
            // overflow outcome (listed total, lost), checked at the next synchronisation
            HIPC(c, hipMemcpyAsync(c->h_ovf, c->d_counters + 13, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
            c->pending_check = true;
        }
    }
    c->stats.samples = (uint64_t)c->local_rows * c->W * p->n_frames;
    if (out_rgba || out_accum) {
        const size_t npx = (size_t)c->local_rows * c->W;
        if (out_rgba) HIPC(c, hipMemcpyAsync(out_rgba, c->d_rgba, npx * 4, hipMemcpyDeviceToHost, c->stream));
        if (out_accum) HIPC(c, hipMemcpyAsync(out_accum, c->d_accum, npx * 16, hipMemcpyDeviceToHost, c->stream));
        HIPC(c, hipStreamSynchronize(c->stream));
        return check_overflow(c);
    }
    return RT_OK;
}

void rt_denoise_params_default(rt_denoise_params* p)
{
    if (!p) return;
    // Denoising::Denoiser members, DN/Denoiser.h:333-358; RayGen_Shader clamps by default (DN/Renderer.h:37)
    p->jbf_half_size = 7; p->temporal_half_size = 3; p->tolerance = 1.0f; p->current_frame_weighting = 0.2f; p->immediate_clamp = 1;
    p->sigma_position = 32.0f; p->sigma_color = 0.6f; p->sigma_normal = 0.1f; p->sigma_coplanarity = 0.1f;
}

rt_status rt_denoise_restart(rt_ctx* c)
{
    if (!c) return RT_ERR_INVALID;
    c->have_prev = false;
    return RT_OK;
}

rt_status rt_render_denoised(rt_ctx* c, const rt_camera* cam, const float proj[16], const float view[16], uint32_t frame, uint64_t seed, float rr,
                             const rt_denoise_params* dp, uint32_t* out_rgba, float* out_color)
{
    if (!c || !cam || !proj || !view || !dp) return RT_ERR_INVALID;
    if (!c->has_scene || c->hdr.n_nodes == 0) { c->err = "no triangle scene uploaded"; return RT_ERR_STATE; }
    if (c->hdr.n_spheres > 0) { c->err = "the Denoiser project's G-buffer takes triangle meshes (the scene has spheres)"; return RT_ERR_INVALID; }
    if (!c->d_accum) { c->err = "no viewport (rt_resize)"; return RT_ERR_STATE; }
    if (c->nranks != 1) { c->err = "the denoiser filters whole frames: rt_resize with nranks == 1"; return RT_ERR_INVALID; }
    if (frame == 0) { c->err = "frame is 1-based"; return RT_ERR_INVALID; }
    if (!(rr >= 0.0f && rr < 1.0f)) { c->err = "rr must be in [0, 1)"; return RT_ERR_INVALID; }
    if (dp->jbf_half_size < 0 || dp->temporal_half_size < 0) { c->err = "negative filter size"; return RT_ERR_INVALID; }
    HIPC(c, hipSetDevice(c->device));
    const size_t npx = (size_t)c->W * c->H;
    if (c->dn_pixels != npx) {
        HIPC(c, hipStreamSynchronize(c->stream));
        dfree(c->d_gb_color); dfree(c->d_gb_pos); dfree(c->d_gb_nrm); dfree(c->d_spatial); dfree(c->d_temporal); dfree(c->d_prev_color);
        dfree(c->d_gb_prim); dfree(c->d_prev_prim); dfree(c->d_dn_rgba);
        float4** f4[6] = {&c->d_gb_color, &c->d_gb_pos, &c->d_gb_nrm, &c->d_spatial, &c->d_temporal, &c->d_prev_color};
        for (float4** q : f4) HIPC(c, hipMalloc((void**)q, npx * sizeof(float4)));
        HIPC(c, hipMalloc((void**)&c->d_gb_prim, npx * 4));
        HIPC(c, hipMalloc((void**)&c->d_prev_prim, npx * 4));
        HIPC(c, hipMalloc((void**)&c->d_dn_rgba, npx * 4));
        HIPC(c, hipMemsetAsync(c->d_gb_pos, 0, npx * sizeof(float4), c->stream));   // FrameBuffer::Reset value-initializes
        HIPC(c, hipMemsetAsync(c->d_gb_nrm, 0, npx * sizeof(float4), c->stream));
        c->dn_pixels = npx;
        c->have_prev = false;
    }
    // 1) the G-buffer frame: the megakernel in GB mode, one sample per pixel
    rt_render_params rp{frame, 1u, seed, rr, RT_RENDER_EXACT};
    c->gb_next = true;
    c->gb_clamp = dp->immediate_clamp != 0;
    rt_status st = rt_render(c, cam, &rp, nullptr, nullptr);
    c->gb_next = false;
    if (st != RT_OK) return st;
    // 2) joint bilateral + 3) temporal (+ pack)
    const bool temporal = dp->temporal_half_size > 0;
    DenoiseParams D{};
    D.W = (int)c->W; D.H = (int)c->H;
    D.color = c->d_gb_color; D.pos = c->d_gb_pos; D.nrm = c->d_gb_nrm; D.prim = c->d_gb_prim;
    D.spatial = dp->jbf_half_size > 0 ? c->d_spatial : c->d_gb_color;
    D.prev_color = c->d_prev_color; D.prev_prim = c->d_prev_prim;
    D.temporal = c->d_temporal; D.rgba = c->d_dn_rgba;
    D.jbf_half = dp->jbf_half_size; D.immediate_clamp = dp->immediate_clamp != 0;
    D.sigma_position = dp->sigma_position; D.sigma_color = dp->sigma_color; D.sigma_normal = dp->sigma_normal; D.sigma_coplanarity = dp->sigma_coplanarity;
    D.temporal_half = dp->temporal_half_size; D.tolerance = dp->tolerance; D.weighting = dp->current_frame_weighting;
    D.have_prev = temporal && c->have_prev;
    std::memcpy(D.prev_proj, c->prev_proj, sizeof D.prev_proj);
    std::memcpy(D.prev_view, c->prev_view, sizeof D.prev_view);
    HIPC(c, hipEventRecord(c->ev2, c->stream));
    HIPC(c, rt_launch_denoise(D, c->stream));
    HIPC(c, hipEventRecord(c->ev3, c->stream));
    c->pending_denoise = true;
    // the history: previous_frame_g_buffer = g_buffer (its color is the temporal output), DN/Denoiser.h:321-325
    if (temporal) {
        HIPC(c, hipMemcpyAsync(c->d_prev_color, c->d_temporal, npx * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
        HIPC(c, hipMemcpyAsync(c->d_prev_prim, c->d_gb_prim, npx * 4, hipMemcpyDeviceToDevice, c->stream));
        std::memcpy(c->prev_proj, proj, sizeof c->prev_proj);
        std::memcpy(c->prev_view, view, sizeof c->prev_view);
    }
    c->have_prev = temporal;   // disabling the filter drops the history (DN/Denoiser.h:237-243)
    HIPC(c, hipMemcpyAsync(c->d_rgba, c->d_dn_rgba, npx * 4, hipMemcpyDeviceToDevice, c->stream));
    if (out_rgba) HIPC(c, hipMemcpyAsync(out_rgba, c->d_dn_rgba, npx * 4, hipMemcpyDeviceToHost, c->stream));
    if (out_color) HIPC(c, hipMemcpyAsync(out_color, c->d_temporal, npx * 16, hipMemcpyDeviceToHost, c->stream));
    if (out_rgba || out_color) HIPC(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

rt_status rt_get_gbuffer(rt_ctx* c, float* color, float* position, float* normal, int32_t* prim, float* spatial)
{
    if (!c) return RT_ERR_INVALID;
    if (!c->dn_pixels) { c->err = "no denoised frame rendered"; return RT_ERR_STATE; }
    HIPC(c, hipSetDevice(c->device));
    const size_t n = c->dn_pixels;
    if (color) HIPC(c, hipMemcpyAsync(color, c->d_gb_color, n * 16, hipMemcpyDeviceToHost, c->stream));
    if (position) HIPC(c, hipMemcpyAsync(position, c->d_gb_pos, n * 16, hipMemcpyDeviceToHost, c->stream));
    if (normal) HIPC(c, hipMemcpyAsync(normal, c->d_gb_nrm, n * 16, hipMemcpyDeviceToHost, c->stream));
    if (prim) HIPC(c, hipMemcpyAsync(prim, c->d_gb_prim, n * 4, hipMemcpyDeviceToHost, c->stream));
    if (spatial) HIPC(c, hipMemcpyAsync(spatial, c->d_spatial, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

rt_status rt_device_buffers(rt_ctx* c, void** d_accum, void** d_rgba)
{
    if (!c) return RT_ERR_INVALID;
    if (d_accum) *d_accum = c->d_accum;
    if (d_rgba) *d_rgba = c->d_rgba;
    return RT_OK;
}

rt_status rt_read_accumulation(rt_ctx* c, float* out_accum)
{
    if (!c || !out_accum) return RT_ERR_INVALID;
    if (!c->d_accum) { c->err = "no viewport (rt_resize)"; return RT_ERR_STATE; }
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipStreamSynchronize(c->stream));
    const rt_status ov = check_overflow(c);
    if (c->local_rows > 0) HIPC(c, hipMemcpy(out_accum, c->d_accum, (size_t)c->local_rows * c->W * 16, hipMemcpyDeviceToHost));
    return ov;
}

rt_status rt_copy_rgba_to_device(rt_ctx* c, void* dst)
{
    if (!c || !dst) return RT_ERR_INVALID;
    HIPC(c, hipMemcpyAsync(dst, c->d_rgba, (size_t)c->local_rows * c->W * 4, hipMemcpyDeviceToDevice, c->stream));
    return RT_OK;
}

rt_status rt_reset_accumulation(rt_ctx* c)
{
    if (!c || !c->d_accum) return RT_ERR_STATE;
    HIPC(c, hipMemsetAsync(c->d_accum, 0, (size_t)std::max<uint32_t>(c->local_rows, 1) * c->W * sizeof(float4), c->stream));
    return RT_OK;
}

rt_status rt_synchronize(rt_ctx* c)
{
    if (!c) return RT_ERR_INVALID;
    HIPC(c, hipStreamSynchronize(c->stream));
    return check_overflow(c);
}

rt_status rt_debug_counters(rt_ctx* c, uint64_t* out, uint32_t n)
{
    if (!c || !out || n > kCounterWords) return RT_ERR_INVALID;
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(out, c->d_counters, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

rt_status rt_get_stats(rt_ctx* c, rt_stats* st)
{
    if (!c || !st) return RT_ERR_INVALID;
    if (c->pending_stats) {
        HIPC(c, hipEventSynchronize(c->ev1));
        float ms = 0.0f;
        HIPC(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->stats.last_kernel_ms = ms;
        float pre = 0.0f, main = 0.0f;
        for (uint32_t i = 0; i < c->kev_used && 3 * (size_t)i + 2 < c->kev.size(); ++i) {
            float a = 0.0f, b = 0.0f;
            HIPC(c, hipEventElapsedTime(&a, c->kev[3 * i], c->kev[3 * i + 1]));
            HIPC(c, hipEventElapsedTime(&b, c->kev[3 * i + 1], c->kev[3 * i + 2]));
            pre += a; main += b;
        }
        c->stats.last_prepass_ms = c->kev_prepass ? pre : 0.0f;
        c->stats.last_main_ms = main;
        unsigned long long h[16] = {};   // [3]: the last pass's overflow list; [13] lost, [14] listed in all passes
        HIPC(c, hipMemcpy(h, c->d_counters, sizeof h, hipMemcpyDeviceToHost));
        c->stats.node_tests = h[0]; c->stats.tri_tests = h[1]; c->stats.rays = h[2];
        c->stats.wave_rounds = h[4]; c->stats.wave_steps = h[5]; c->stats.wave_tri_tests = h[6]; c->stats.wave_service = h[7];
        c->stats.wave_fold = h[8]; c->stats.cycles_service = h[9]; c->stats.cycles_queue = h[10]; c->stats.cycles_trace = h[11];
        c->stats.service_lanes = h[12];
        c->pending_stats = false;
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    const rt_status ov = check_overflow(c);
    // the overflow outcome as of the last check (resampled + lost, summed since the check before it)
    c->stats.stack_overflows = c->stats.resampled + c->stats.overflow_lost;
    if (c->pending_denoise) {
        HIPC(c, hipEventSynchronize(c->ev3));
        float ms = 0.0f;
        HIPC(c, hipEventElapsedTime(&ms, c->ev2, c->ev3));
        c->stats.last_denoise_ms = ms;
        c->pending_denoise = false;
    }
    c->stats.block = c->block; c->stats.stack_depth = c->stack_depth;
    *st = c->stats;
    return ov;
}

rt_status rt_trace(rt_ctx* c, uint64_t n, const float* org, const float* dir, int32_t* tri, double* t)
{
    if (!c || (n && (!org || !dir || !tri || !t))) return RT_ERR_INVALID;
    if (!c->has_scene) { c->err = "no scene uploaded"; return RT_ERR_STATE; }
    if (n == 0) return RT_OK;
    if (n > 0x7FFFFFFFull) return RT_ERR_INVALID;
    HIPC(c, hipSetDevice(c->device));
    float *d_o = nullptr, *d_d = nullptr; int32_t* d_tri = nullptr; double* d_t = nullptr;
    auto cleanup = [&]() { dfree(d_o); dfree(d_d); dfree(d_tri); dfree(d_t); };
    hipError_t e;
    if ((e = hipMalloc((void**)&d_o, n * 12)) != hipSuccess || (e = hipMalloc((void**)&d_d, n * 12)) != hipSuccess ||
        (e = hipMalloc((void**)&d_tri, n * 4)) != hipSuccess || (e = hipMalloc((void**)&d_t, n * 8)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "hipMalloc(rt_trace)");
    }
    KParams P{};
    P.nodes = c->d_nodes; P.n_nodes = c->hdr.n_nodes; P.tris = c->d_tris;
    if ((e = hipMemcpyAsync(d_o, org, n * 12, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(d_d, dir, n * 12, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess ||
        (e = rt_launch_trace(P, (uint32_t)n, d_o, d_d, d_tri, d_t, c->stream)) != hipSuccess ||
        (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(tri, d_tri, n * 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(t, d_t, n * 8, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "rt_trace");
    }
    cleanup();
    c->pending_stats = true;   // last_kernel_ms = the trace kernel
    c->kev_used = 0;
    return RT_OK;
}

#if RT_WALK_STUDY
// the walk study (variant builds only, rt_kernels.hip walk_study_kernel): n rays walked through the split subtree's
// near-first orderings, K rays per lane, `steps` node tests per round; `reps` timed launches, their times in ms[]
rt_status rt_debug_walk_study(rt_ctx* c, uint64_t n, const float* org, const float* dir, uint32_t k, uint32_t steps, uint32_t reps,
                              int32_t* tri, double* t, float* ms, uint64_t* rounds)
{
    // k: rays per lane (1-4), | 0x100 for the refill kernel; 0x201: the (ray, round) count of a K = 1 lockstep run into
    // rounds[0] (its ms are not a rate)
    if (!c || !org || !dir || !tri || !t || !ms || n == 0 || n > 0x7FFFFFFFull || (k & 0xFFu) < 1 || (k & 0xFFu) > 4 ||
        ((k & ~0x1FFu) && k != 0x201u) || steps == 0 || reps == 0 || (k == 0x201u && !rounds))
        return RT_ERR_INVALID;
    if (!c->has_scene || c->split_root == 0 || !c->d_wcopies) { c->err = "the walk study needs a split scene with near-first orderings"; return RT_ERR_STATE; }
    HIPC(c, hipSetDevice(c->device));
    float *d_o = nullptr, *d_d = nullptr; int32_t* d_tri = nullptr; double* d_t = nullptr; uint32_t* d_ctr = nullptr;
    auto cleanup = [&]() { dfree(d_o); dfree(d_d); dfree(d_tri); dfree(d_t); dfree(d_ctr); };
    hipError_t e;
    if ((e = hipMalloc((void**)&d_o, n * 12)) != hipSuccess || (e = hipMalloc((void**)&d_d, n * 12)) != hipSuccess ||
        (e = hipMalloc((void**)&d_tri, n * 4)) != hipSuccess || (e = hipMalloc((void**)&d_t, n * 8)) != hipSuccess ||
        (e = hipMalloc((void**)&d_ctr, 512)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "hipMalloc(rt_debug_walk_study)");
    }
    KParams P{};
    P.nodes = c->d_nodes; P.n_nodes = c->hdr.n_nodes; P.tris = c->d_tris; P.n_tris = c->hdr.n_tris;
    P.split_root = c->split_root; P.split_end = c->split_end; P.steps = steps;
    P.wcopies = reinterpret_cast<const float4*>(reinterpret_cast<uintptr_t>(c->d_wcopies) - (uintptr_t)c->split_root * 2u * sizeof(float4));
    P.wcopy_stride = 2u * (c->split_end - c->split_root);
    P.counters = reinterpret_cast<decltype(P.counters)>(d_ctr);   // the refill kernel's ray counter
    if ((e = hipMemcpyAsync(d_o, org, n * 12, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(d_d, dir, n * 12, hipMemcpyHostToDevice, c->stream)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "rt_debug_walk_study");
    }
    for (uint32_t r = 0; r < reps; ++r) {
        if ((e = hipMemsetAsync(d_ctr, 0, 512, c->stream)) != hipSuccess || (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess ||
            (e = rt_launch_walk_study(P, (uint32_t)n, k, d_o, d_d, d_tri, d_t, c->stream)) != hipSuccess ||
            (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess || (e = hipEventSynchronize(c->ev1)) != hipSuccess ||
            (e = hipEventElapsedTime(&ms[r], c->ev0, c->ev1)) != hipSuccess) {
            cleanup(); return hip_fail(c, e, "rt_debug_walk_study");
        }
    }
    uint64_t cnt[64] = {};
    if ((e = hipMemcpyAsync(tri, d_tri, n * 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(t, d_t, n * 8, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(cnt, d_ctr, 512, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "rt_debug_walk_study");
    }
    if (k == 0x201u) {
        rounds[0] = 0;
        for (int i = 0; i < 8; ++i) rounds[0] += cnt[8 * i];
    }
    cleanup();
    return RT_OK;
}
#endif

rt_status rt_sample_light(rt_ctx* c, uint64_t n, const uint32_t* u, float* loc, float* normal, float* emission, float* pdf)
{
    if (!c || (n && (!u || !loc || !normal || !emission || !pdf))) return RT_ERR_INVALID;
    if (!c->has_scene) { c->err = "no scene uploaded"; return RT_ERR_STATE; }
    if (c->hdr.light_mesh < 0 || c->hdr.n_ltris == 0) { c->err = "the scene has no emissive mesh"; return RT_ERR_STATE; }
    if (n == 0) return RT_OK;
    if (n > 0x7FFFFFFFull) return RT_ERR_INVALID;
    HIPC(c, hipSetDevice(c->device));
    uint32_t* d_u = nullptr; float* d_out = nullptr;
    auto cleanup = [&]() { dfree(d_u); dfree(d_out); };
    KParams P{};
    P.lnodes = c->d_lnodes; P.n_lnodes = c->hdr.n_lnodes;
    P.ltris = c->d_ltris; P.n_ltris = c->hdr.n_ltris;
    P.light_area = c->hdr.light_area;
    std::memcpy(P.light_emission, c->hdr.light_emission, sizeof P.light_emission);
    P.lpdf = 1.0f / c->hdr.light_area;   // as rt_render (an IEEE single division)
    std::vector<float> out((size_t)n * 10);
    hipError_t e;
    if ((e = hipMalloc((void**)&d_u, n * 12)) != hipSuccess || (e = hipMalloc((void**)&d_out, n * 40)) != hipSuccess ||
        (e = hipMemcpyAsync(d_u, u, n * 12, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = rt_launch_light_sample(P, (uint32_t)n, d_u, d_out, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(out.data(), d_out, n * 40, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "rt_sample_light");
    }
    cleanup();
    for (uint64_t i = 0; i < n; ++i) {
        const float* o = &out[10 * i];
        for (int k = 0; k < 3; ++k) { loc[3 * i + k] = o[k]; normal[3 * i + k] = o[3 + k]; emission[3 * i + k] = o[6 + k]; }
        pdf[i] = o[9];
    }
    return RT_OK;
}

rt_status rt_world_trace(rt_ctx* c, uint64_t n, const float* org, const float* dir, int32_t* ent, int32_t* tri, float* tb)
{
    if (!c || (n && (!org || !dir || !ent || !tri || !tb))) return RT_ERR_INVALID;
    if (!c->has_scene || c->hdr.n_went == 0) { c->err = "no Whitted world uploaded"; return RT_ERR_STATE; }
    if (n == 0) return RT_OK;
    if (n > 0x7FFFFFFFull) return RT_ERR_INVALID;
    HIPC(c, hipSetDevice(c->device));
    float *d_o = nullptr, *d_d = nullptr, *d_tb = nullptr; int32_t *d_e = nullptr, *d_t = nullptr;
    auto cleanup = [&]() { dfree(d_o); dfree(d_d); dfree(d_tb); dfree(d_e); dfree(d_t); };
    KParams P{};
    P.went = c->d_went; P.wtris = c->d_wtris; P.n_went = c->hdr.n_went;
    hipError_t e;
    if ((e = hipMalloc((void**)&d_o, n * 12)) != hipSuccess || (e = hipMalloc((void**)&d_d, n * 12)) != hipSuccess ||
        (e = hipMalloc((void**)&d_tb, n * 12)) != hipSuccess || (e = hipMalloc((void**)&d_e, n * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&d_t, n * 4)) != hipSuccess ||
        (e = hipMemcpyAsync(d_o, org, n * 12, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(d_d, dir, n * 12, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = rt_launch_world_trace(P, (uint32_t)n, d_o, d_d, d_e, d_t, d_tb, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(ent, d_e, n * 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(tri, d_t, n * 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(tb, d_tb, n * 12, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "rt_world_trace");
    }
    cleanup();
    return RT_OK;
}

rt_status rt_debug_primitives(rt_ctx* c, uint64_t n_mt, const float* mt, int32_t* mt_hit, double* mt_t, uint64_t n_box, const float* box,
                              int32_t* box_hit)
{
    if (!c || (n_mt && (!mt || !mt_hit || !mt_t)) || (n_box && (!box || !box_hit))) return RT_ERR_INVALID;
    if (n_mt > 0x7FFFFFFFull || n_box > 0x7FFFFFFFull) return RT_ERR_INVALID;
    if (n_mt == 0 && n_box == 0) return RT_OK;
    HIPC(c, hipSetDevice(c->device));
    float *d_mt = nullptr, *d_box = nullptr; int32_t *d_mh = nullptr, *d_bh = nullptr; double* d_t = nullptr;
    auto cleanup = [&]() { dfree(d_mt); dfree(d_box); dfree(d_mh); dfree(d_bh); dfree(d_t); };
    hipError_t e = hipSuccess;
    if ((n_mt && ((e = hipMalloc((void**)&d_mt, n_mt * 60)) != hipSuccess || (e = hipMalloc((void**)&d_mh, n_mt * 4)) != hipSuccess ||
                  (e = hipMalloc((void**)&d_t, n_mt * 8)) != hipSuccess ||
                  (e = hipMemcpyAsync(d_mt, mt, n_mt * 60, hipMemcpyHostToDevice, c->stream)) != hipSuccess)) ||
        (n_box && ((e = hipMalloc((void**)&d_box, n_box * 48)) != hipSuccess || (e = hipMalloc((void**)&d_bh, n_box * 12)) != hipSuccess ||
                   (e = hipMemcpyAsync(d_box, box, n_box * 48, hipMemcpyHostToDevice, c->stream)) != hipSuccess)) ||
        (e = rt_launch_debug_primitives((uint32_t)n_mt, d_mt, d_mh, d_t, (uint32_t)n_box, d_box, d_bh, c->stream)) != hipSuccess ||
        (n_mt && ((e = hipMemcpyAsync(mt_hit, d_mh, n_mt * 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
                  (e = hipMemcpyAsync(mt_t, d_t, n_mt * 8, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)) ||
        (n_box && (e = hipMemcpyAsync(box_hit, d_bh, n_box * 12, hipMemcpyDeviceToHost, c->stream)) != hipSuccess) ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        cleanup(); return hip_fail(c, e, "rt_debug_primitives");
    }
    cleanup();
    return RT_OK;
}

rt_status rt_math_selftest(rt_ctx* c, uint64_t n, const float* x, float* out)
{
    if (!c || (n && (!x || !out))) return RT_ERR_INVALID;
    if (n == 0) return RT_OK;
    HIPC(c, hipSetDevice(c->device));
    float *d_x = nullptr, *d_out = nullptr;
    hipError_t e;
    if ((e = hipMalloc((void**)&d_x, n * 4)) != hipSuccess || (e = hipMalloc((void**)&d_out, n * 36)) != hipSuccess) {
        dfree(d_x); dfree(d_out); return hip_fail(c, e, "hipMalloc(selftest)");
    }
    if ((e = hipMemcpyAsync(d_x, x, n * 4, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = rt_launch_math((uint32_t)n, d_x, d_out, c->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(out, d_out, n * 36, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        dfree(d_x); dfree(d_out); return hip_fail(c, e, "rt_math_selftest");
    }
    dfree(d_x); dfree(d_out);
    return RT_OK;
}

}  // extern "C"
