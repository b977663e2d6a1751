// rt_kernels.h -- launch interface between the C-ABI layer (rt_capi.cpp) and the HIP kernels.
#ifndef RT_KERNELS_H
#define RT_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

struct KParams {
    // scene (rt_layout.h)
    const float4* nodes; uint32_t n_nodes;
    const float4* tris; uint32_t n_tris;
    const float4* mats; uint32_t n_mats;
    const float4* lnodes; uint32_t n_lnodes;
    const float4* ltris; uint32_t n_ltris;
    const float4* lboxes; uint32_t n_lboxes;   // small scenes: distinct leaf boxes + triangle masks (rt_layout.h)
    // split trace (larger scenes, the vertex kernel's BVH variant; rt_scene.h FlatScene::sboxes): the rays walk
    // only the subtree [split_root, split_end), the outside leaves are tested by their boxes (split_root = 0: off)
    const float4* sboxes; const int32_t* stri; uint32_t n_sboxes, split_root, split_end, n_split_leaves;
    // the subtree's near-first orderings (rt_scene.h FlatScene::wcopies; null: off): ordering o's node k at
    // wcopies[2 * k + o * wcopy_stride], k in [split_root, split_end) (the pointer is offset by -2 * split_root)
    // (each ordering's boxes are its octant's (near, far) planes: rt_device.h slab_nf_within)
    const float4* wcopies; uint32_t wcopy_stride;
    // Whitted scenes: the whole tree's near-first orderings (FlatScene::worders; null: the DFS walk), ordering
    // o's node k at worders[2 * (o * n_nodes + k)]
    const float4* worders;
    // the same orderings in 16-byte nodes with half planes rounded outward (FlatScene::worders_h; null: off), ordering
    // o's node k at worders_h[o * n_nodes + k]; a leaf's exact box comes from its vertices (tabc)
    const uint4* worders_h;
    // (the BVH variant stages the small tables (mats | lnodes | ltris) in LDS, the split's outside triangles
    //  (3 float4 per slot: a, e1, (e2, bits(triangle))) after them; rt_capi.cpp checks that they fit)
    // the triangles' vertices, 3 float4 per slot (FlatScene::tabc): the exact leaf boxes of the half-plane walk
    // (round 6: the vertex kernel's compact-BVH walk, RT_QBVH, is gone)
    const float4* tabc;
    float light_area; float light_emission[3]; int has_light;
    // Whitted shading (rt_whitted.hip): per-material (diffuse color, phong_diffuse), point lights, sky
    const float4* wmats; const float4* plights; uint32_t n_plights; float sky[3];
    // Whitted world (rt_whitted.hip, config C1): entities + their mesh triangles (rt_layout.h)
    const float4* went; const float4* wtris; uint32_t n_went; int32_t max_bounce_depth; float intersection_correction;
    // camera: position, inverse projection, inverse view (column-major glm mat4)
    float cam_pos[3]; float iproj[16]; float iview[16];
    // image and sampling
    uint32_t W, H;
    uint32_t first_frame, n_frames;
    uint64_t seed; float rr;
    // correctly rounded reciprocals of the uniform divisors (host IEEE divisions) for rt_device.h div_fast:
    // 1/PDF (PDF = 1/(2*PI), MC/WhittedMaterial.h:44-56), 1/rr, lpdf = 1/light_area and 1/lpdf, 1/W, 1/H
    float y_pdf, y_rr, lpdf, y_lpdf, y_w, y_h;
    uint32_t rr_fast;   // rr in [2^-20, 1): the fold's division by rr may take Markstein's path (rt_device.h div2_core)
    uint32_t lpdf_fast; // lpdf in [2^-20, 2^20): the direct term's division by the light PDF likewise
    uint32_t wh_fast;   // W and H below 2^20: the camera's divisions by W and H likewise
    // pixels of this device: row bands of `band` rows dealt round-robin over `nranks`
    uint32_t band, rank, nranks, n_local_rows;
    uint32_t tiles_x; uint32_t n_items;
    // (float)(1 / d) of the uniform divisors band, tiles_x, n_tiles (rt_device.h udiv24), and whether every
    // dividend of this launch is below 2^24 (else the generic division)
    float r_band, r_tiles_x, r_n_tiles; uint32_t div24;
    // frame chunks: a pixel's n_frames are split into n_chunks work items of chunk_frames frames so
    // that a frame-range tail does not serialize a launch with few pixels per lane (multi-GPU bands);
    // chunk 0 accumulates into accum, later chunks store their samples (3 planes of floats,
    // frame-major: [frame - chunk_frames][local]) for the in-order sum of finalize_chunks_kernel
    uint32_t n_chunks, chunk_frames, items_per_chunk;
    float* lbuf; size_t lbuf_stride;
    // camera-ray misses of the pre-pass (the night sky, MC/Renderer.cpp:145) as bits instead of parked samples: bit
    // (fidx % 32) of word [fidx / 32][local] (null: every sample is parked); finalize_chunks_kernel adds the sky's
    // radiance for a set bit and reads the parked slot only for the others
    uint32_t* sky_bits; uint32_t sky_words;
    uint32_t park_all;              // every frame is parked (the vertex kernel): finalize accumulates all of them
    uint32_t lbuf_pixel_major;      // park_all: a pixel's 4-frame blocks are contiguous ([pixel][block]) instead of
                                    // [block][pixel] (lbuf_stride pixels apart)
    // outputs (compact local pixel order: local_row * W + x)
    float4* accum; uint32_t* rgba;
    // scratch
    uint32_t* work_counter;
    // the vertex kernel's segment parts are handed out by n_work_queues counters (1 or 8), 32 words apart from
    // work_queues: block b draws from queue b mod n (the XCD it runs on), part k = j * n + queue for its j-th
    // draw, and moves to the next queue when its own is dry
    uint32_t* work_queues; uint32_t n_work_queues;
    float4* stack_ld; int32_t* stack_mat; uint32_t stack_depth; uint32_t total_threads;
    // vertex kernel, EXACT: a scene of at most 8 materials keeps a fold level's material in the sign bits
    // of its direct term (always +0 or positive; a zero's sign never reaches the accumulation: the sums
    // start at +0), so a level is one float4 (stack_mat unused)
    uint32_t ring_pack;
    uint32_t lds_levels;            // EXACT: the first lds_levels stack levels live in LDS (after the scene)
    uint32_t lds_pad;               // diagnostic: unused dynamic LDS bytes per workgroup (occupancy experiments)
    uint32_t lds_scene_quads;       // float4s of LDS taken by the staged scene (0 when the scene is in HBM)
    // the vertex kernel's camera pre-pass (camera_prepass_kernel, rt_coherent.hip): samples in segments of one
    // 8x8 tile x seg_frames (a power of two <= 64) frames, segment s = chunk * n_tiles + tile (chunk-major);
    // the surface hits of segment s are records [s << seg_shift, + its record count) of crec: (location.xyz, tag),
    // tag = triangle | pixel-in-tile << 19 | frame-in-chunk << 25 | flipped normal << 31; the non-empty
    // segments are listed in seg_list[0, *seg_list_n) (misses and light hits are parked by the pre-pass);
    // the path kernel takes each listed segment in 2^seg_part_shift parts (consecutive record ranges), so a
    // pass with few tiles keeps long pre-pass segments and still hands out fine-grained work; a list entry is
    // (segment, its record count), so a wave's work fetch is the counter's atomic and one 8-byte load
    float4* crec; uint2* seg_list; uint32_t* seg_list_n;
    unsigned long long* tile_boxes;   // per tile: the leaf boxes its camera rays' frustum meets (tile_boxes_kernel)
    // split scenes (the BVH variant's pre-pass): a camera ray that enters the walked subtree's box is recorded as a
    // camera ray (triangle field CREC_CAMERA, its direction in the location's place) and traced by the path kernel,
    // instead of walked here (0: the pre-pass walks it)
    uint32_t pre_defer_walk;
    uint32_t n_segments, n_tiles, seg_frames, seg_shift, seg_part_shift;
    // ... and the list's last seg_tail_n segments in 2^seg_tail_shift parts (>= seg_part_shift; finer work at the
    // launch's end)
    uint32_t seg_tail_n, seg_tail_shift;
    uint32_t thresh;                // serve finished lanes once at most `thresh` lanes of a wave still trace
    uint32_t steps;                 // box tests per lane per traversal round (a parked leaf ends a round early)
    uint32_t force_walk;            // diagnostic (RT_FORCE_WALK): the vertex kernel walks the BVH for every ray
    unsigned long long* counters;   // [node_tests, tri_tests, rays, this pass's ring overflows (listed), ...,
                                    //  [13] levels dropped (megakernel) or overflows the list could not hold,
                                    //  [14] ring overflows listed in all passes]
    // EXACT: samples whose path outgrew the vertex kernel's fold ring -- (local pixel, frame index,
    // global pixel, frame) -- rendered again by resample_kernel with a deep stack (rt_resample.hip)
    uint4* ovf_list; uint32_t ovf_cap;
    float4* rs_stack; int32_t* rs_mat;
    // the Denoiser's G-buffer frame (set => pt_megakernel<..., GB = true>); one sample per pixel
    float4* gb_color; float4* gb_pos; float4* gb_nrm; int32_t* gb_prim; uint32_t gb_clamp;
};

// LDS staging of the scene: bytes needed (the kernel's dynamic shared memory when lds == true)
size_t rt_scene_lds_bytes(const KParams& P);
// bytes of LDS per 256-lane workgroup for `levels` EXACT stack levels (float4 + u8 material per lane)
size_t rt_stack_lds_bytes(uint32_t levels);
size_t rt_lane_state_lds_bytes(bool exact);   // the megakernel's per-lane cold state (256 lanes)
hipError_t rt_launch_megakernel(const KParams& P, bool exact, bool count, bool lds, uint32_t grid, uint32_t block, hipStream_t stream);
int rt_megakernel_occupancy(bool exact, bool count, bool lds, int block, size_t lds_bytes);
// the vertex-synchronous kernel (rt_coherent.hip; no counters, no G-buffer): small scenes (n_lboxes > 0,
// scene in LDS: LDS = scene | lane state) or, bvh = true, any scene in HBM (LDS = lane state)
hipError_t rt_launch_coherent(const KParams& P, bool exact, bool bvh, bool prepass, uint32_t grid, uint32_t block, size_t lds, hipStream_t stream);
// its camera pre-pass: every sample's camera ray traced, misses / light hits parked, surface hits recorded
// (KParams::crec); lds = the small scene's staged triangles + materials, or a split scene's staged outside
// triangles (bvh: the BVH variant's pre-pass, for split scenes; prepass == true in rt_launch_coherent)
hipError_t rt_launch_camera_prepass(const KParams& P, bool bvh, size_t lds, hipStream_t stream);
int rt_coherent_occupancy(bool exact, bool bvh, bool prepass, int block, size_t lds_bytes);
size_t rt_coherent_lane_state_lds_bytes(bool exact, bool lit, bool bvh);
// Whitted-style C3 renderer: one thread per local pixel, 16x16 tiles (grid_out: workgroups launched)
hipError_t rt_launch_whitted(const KParams& P, bool count, hipStream_t stream, uint32_t* grid_out);
// Whitted Style Ray Tracer world (spheres + textured meshes, reflection/refraction recursion), config C1
hipError_t rt_launch_whitted_world(const KParams& P, bool count, hipStream_t stream, uint32_t* grid_out);
hipError_t rt_launch_world_trace(const KParams& P, uint32_t n, const float* org, const float* dir, int32_t* ent, int32_t* tri, float* tb,
                                 hipStream_t stream);
// exact re-render of the listed ring overflows into their parked slots (before finalize)
hipError_t rt_launch_resample(const KParams& P, uint32_t threads, hipStream_t stream);
// device checks of the two primitives with shortcuts (rt_coherent.hip): Moller-Trumbore with its float
// pre-screen on (a, b, c, o, d) cases (hit, t); the slab test on (lo, hi, o, d) cases in its three forms
// (general, finite-reciprocal, the vertex kernel's leaf-box form; -1 where a form does not apply)
hipError_t rt_launch_debug_primitives(uint32_t n_mt, const float* mt, int32_t* mt_hit, double* mt_t, uint32_t n_box, const float* box,
                                      int32_t* box_hit, hipStream_t stream);
hipError_t rt_launch_finalize_chunks(const KParams& P, uint32_t n_px, hipStream_t stream);
hipError_t rt_launch_trace(const KParams& P, uint32_t n, const float* org, const float* dir, int32_t* tri, double* t, hipStream_t stream);
#if RT_WALK_STUDY
hipError_t rt_launch_walk_study(const KParams& P, uint32_t n, uint32_t k, const float* org, const float* dir, int32_t* tri, double* t, hipStream_t stream);
#endif
// SamplingAreaLight on given draws (3 u32 per case): out = 10 floats per case (location, normal, emission, PDF)
hipError_t rt_launch_light_sample(const KParams& P, uint32_t n, const uint32_t* u, float* out, hipStream_t stream);
hipError_t rt_launch_math(uint32_t n, const float* x, float* out, hipStream_t stream);

// the Denoiser's filters (rt_denoise.hip, DN/Denoiser.h): full frames, one device
struct DenoiseParams {
    int W, H;
    const float4* color; const float4* pos; const float4* nrm; const int32_t* prim;   // this frame's G-buffer
    float4* spatial;                  // joint bilateral output (== color when the filter is off)
    const float4* prev_color; const int32_t* prev_prim;   // the previous frame (its temporal output)
    float4* temporal; uint32_t* rgba;
    int jbf_half; float sigma_position, sigma_color, sigma_normal, sigma_coplanarity; int immediate_clamp;
    int temporal_half; float tolerance, weighting; int have_prev;
    float prev_proj[16], prev_view[16];
    int ieee_div;   // diagnostic (RT_JBF_IEEE): the filter's divisions by the IEEE sequence, not Markstein's correction
};
hipError_t rt_launch_denoise(const DenoiseParams& D, hipStream_t stream);

// GPU BVH build (rt_lbvh.hip): a Karras LBVH in the traversal layout (rt_layout.h nodes / tris).
// verts: 9 floats per triangle (a, b, c); recs: the triangle records (4 float4 per triangle); n >= 2.
hipError_t lbvh_build_device(uint32_t n, const float* verts, const float4* recs, float4* nodes, float4* tris, hipStream_t s);
// the same tree built on the host, sequentially (tests): 8 floats per node (2n - 1), 16 per triangle
bool lbvh_build_host(uint32_t n, const float* verts, const float* recs, std::vector<float>& nodes, std::vector<float>& tris);

#endif
