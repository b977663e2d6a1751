// rt_coherent.hip -- vertex-synchronous path tracing for small scenes (gfx950 / CDNA4, wave64).
//
// The general megakernel (rt_kernels.hip) advances every lane by one ray per loop iteration, so the
// lanes of a wave sit in different phases of the reference's shading (camera hit, shadow-ray return,
// indirect hit, end of path) and every iteration executes the union of those branches.  For a scene
// of at most 64 triangles whose distinct leaf boxes decide the traversal (rt_scene.cpp), this kernel
// advances every lane by one path VERTEX per iteration instead:
//
//   * at vertex v the lane draws everything Renderer::shading draws there, in the reference's order
//     (light pick, light-triangle x/y, Russian roulette, hemisphere z/phi; MC/Renderer.cpp:163-209),
//     and sets up BOTH rays -- the shadow ray toward the light sample and, if the roulette continues,
//     the indirect ray; the two share the shading point as origin;
//   * one trace step tests both rays against every distinct leaf box (wave-uniform loop, box planes
//     in scalar registers through scalar loads, the (plane - origin) differences shared by the two
//     rays), then runs Moller-Trumbore on each ray's candidate triangles in DFS order: closest hit for
//     the indirect (or camera) ray, any blocking hit for the shadow ray;
//   * the next service resolves vertex v's direct term from the shadow verdict and processes the
//     indirect hit as vertex v+1.
// A path of k vertices takes k+1 iterations instead of 2k+1, and all lanes of a wave run the same
// vertex code.  The arithmetic, the draws and the EXACT inner-first fold are the megakernel's, so the
// accumulation is bit-identical to it and to the reference (tests/test_gpu_parity.py).
//
// Rays with a non-finite reciprocal direction (an exactly axis-aligned component) have no monotone
// slab test; such a ray walks the BVH on its own lane (the reference's traversal, rt_path.h).
//
// Scenes without decisive leaf boxes (C5: Cornell + a 79k-triangle mesh) use the BVH variant
// (template argument BVH): same vertex loop, drain, parked samples and work pool, the scene in HBM,
// and the lane's two rays walking the stackless BVH in the megakernel's postponed-leaf rounds.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rt_device.h"
#include "rt_kernels.h"
#include "rt_path.h"

using namespace rtd;

namespace {

// per-lane cold state in LDS, [field][lane] words
enum : uint32_t {
    VS_LOCAL = 0,                        // the work item's local pixel
    VS_PIX = 1, VS_FRAME = 2,            // the sample's stream counter: global pixel y * W + x, frame number
    VS_LD = 3,                           // the pending vertex's unoccluded direct term (3 words)
    VS_PCOS = 6, VS_MAT = 7,             // the pending vertex's indirect cosine, and its material | the path's vertex
                                         // count << VS_DEPTH_SHIFT (the count lives here, not in a register)
    VS_BASE = 8,                         // EXACT: ring position of the current path's level 0
    VS_DL = 9,                           // EXACT drain: the partial fold (3 words)
    VS_DPOS = 12,                        // EXACT drain: ring position of the next level to fold
    VS_DT0 = 13, VS_DT1 = 14,            // EXACT drain: the sample's local pixel and frame index
    VS_THR = 8, VS_LSUM = 11,            // FAST: throughput, radiance
    VS_PEND = 15,                        // EXACT, leaf-box variant: a finished path's fold waiting behind the draining
                                         // one -- ring position of its top level | its levels << 12 (PEND_NONE: none)
    VS_PLOC = 16,                        //   ... and its sample's local pixel (its L and frame index: the ring slot above its top)
    VS_WORDS_EXACT = 17, VS_WORDS_FAST = 14,
    VS_RNG = 17,                         // unlit scenes only: the Philox block of the current 4 draws
    VS_WORDS_UNLIT = 21
};

// VS_MAT = material (< 2^14, host) | light-skip code << 14 (the sampled light triangle + 1 when its shadow-candidate
// skip mask applies, 0 when not: read back by the trace of the same iteration) | the path's vertex count << 19
// a camera-hit record's triangle field when the record is a camera ray left to the path kernel (its direction in
// the location's place; the BVH variant's pre-pass, scenes of < 2^19 - 1 triangles)
constexpr uint32_t CREC_CAMERA = 0x7FFFFu;
constexpr uint32_t VS_SKIP_SHIFT = 14, VS_DEPTH_SHIFT = 19, VS_MAT_MASK = (1u << VS_SKIP_SHIFT) - 1u;

// The six draws of a vertex of a lit scene, taken in order by sample_light / the roulette /
// sample_hemisphere (straight-line code: the index folds to constants)
struct FixedDraws {
    float u[6];
    int i;
    __device__ __forceinline__ float next() { return u[i++]; }
};

// The lane's uniform draws (rt_path.h LaneRng) with only the draw index in a register: the counter
// (pixel, frame) and the current block of 4 Philox words live in the lane's LDS words.  Draws are
// consumed one by one from index 0, so a new block starts exactly when the index is a multiple of 4.
struct VertexRng {
    uint32_t* w;        // the lane's word 0 of the cold state (stride 256)
    uint32_t k0, k1;    // key (uniform)
    uint32_t dim;
    __device__ __forceinline__ float next()
    {
        if ((dim & 3u) == 0u) {
            uint32_t o[4];
            philox4x32_10(w[VS_PIX * 256u], w[VS_FRAME * 256u], dim >> 2, 0u, k0, k1, o);
            w[VS_RNG * 256u] = o[0]; w[(VS_RNG + 1) * 256u] = o[1]; w[(VS_RNG + 2) * 256u] = o[2]; w[(VS_RNG + 3) * 256u] = o[3];
        }
        const uint32_t u = w[(VS_RNG + (dim & 3u)) * 256u];
        ++dim;
        return (float)u / 4294967296.0f;   // Walnut::Random::Float, (float)UINT32_MAX == 2^32 exactly
    }
    // A vertex of a lit scene draws dims d .. d+5 with d = 2 + 6 * vertex (2 camera draws, then 3 light
    // + roulette + 2 hemisphere per vertex), so d % 4 is 0 or 2 and the six draws lie in the two
    // Philox blocks d/4 and d/4 + 1: every vertex lane evaluates exactly those two blocks, in lockstep,
    // instead of one block wherever its own draw index crosses a multiple of 4 (which, with lanes at
    // different vertices, made every draw site run Philox for some lane).
    __device__ __forceinline__ void vertex_draws(FixedDraws& fd)
    {
        const uint32_t b = dim >> 2;
        uint32_t o[8];
        philox4x32_10(w[VS_PIX * 256u], w[VS_FRAME * 256u], b, 0u, k0, k1, o);
        philox4x32_10(w[VS_PIX * 256u], w[VS_FRAME * 256u], b + 1u, 0u, k0, k1, o + 4);
        // words (o[0..5] or o[2..7]) picked by a mask, not by an index: a select the compiler turns
        // into a dynamic array offset puts o[] in scratch memory
        const uint32_t msk = (dim & 2u) ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (int i = 0; i < 6; ++i) fd.u[i] = (float)(o[i] ^ ((o[i] ^ o[i + 2]) & msk)) / 4294967296.0f;
        fd.i = 0;
        dim += 6u;
    }
    // the camera draws: dims 0 and 1 of block 0 (the block is kept in LDS only for unlit scenes, whose
    // vertices draw through next())
    __device__ __forceinline__ void camera_draws(uint32_t px, uint32_t fr, bool keep, float& ux, float& uy)
    {
        uint32_t o[4];
        philox4x32_10(px, fr, 0u, 0u, k0, k1, o);
        if (keep) { w[VS_RNG * 256u] = o[0]; w[(VS_RNG + 1) * 256u] = o[1]; w[(VS_RNG + 2) * 256u] = o[2]; w[(VS_RNG + 3) * 256u] = o[3]; }
        ux = (float)o[0] / 4294967296.0f;
        uy = (float)o[1] / 4294967296.0f;
        dim = 2;
    }
    // a new sample (pixel, frame) whose camera draws (dims 0 and 1, camera_prepass_kernel) are taken:
    // the vertices continue at dim 2; an unlit scene's vertices draw through next(), which finds dims 2
    // and 3 in the block kept in LDS
    __device__ __forceinline__ void start(uint32_t px, uint32_t fr, bool unlit)
    {
        if (unlit) {
            uint32_t o[4];
            philox4x32_10(px, fr, 0u, 0u, k0, k1, o);
            w[VS_RNG * 256u] = o[0]; w[(VS_RNG + 1) * 256u] = o[1]; w[(VS_RNG + 2) * 256u] = o[2]; w[(VS_RNG + 3) * 256u] = o[3];
        }
        dim = 2;
    }
};

// one fold level from the ring: (direct term, cosine) and material -- with ring_pack the material is
// the three sign bits of the direct term (one 16-byte load instead of two)
// (the load and the unpacking are separate steps, so that a drain step issues all its ring loads before it waits
// for the first: with the ring_pack branch inside one load-and-unpack call the compiler waited on each load
// before issuing the next)
__device__ __forceinline__ void ring_unpack(const CKParams& Q, size_t at, float4& e, int& m)
{
    if (Q.ring_pack) {
        const uint32_t x = __float_as_uint(e.x), y = __float_as_uint(e.y), z = __float_as_uint(e.z);
        m = (int)((x >> 31) | ((y >> 30) & 2u) | ((z >> 29) & 4u));
        // |x| as fabsf: the fold's adds take it as a free source modifier
        e = make_float4(__builtin_fabsf(e.x), __builtin_fabsf(e.y), __builtin_fabsf(e.z), e.w);
    } else {
        m = Q.stack_mat[at];
    }
}

// the distinct leaf boxes, read with scalar loads (constant address space: wave-uniform index)
typedef const __attribute__((address_space(4))) float cfloat;
typedef float box8 __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(4))) box8 cbox8;

// AABB_3D::intersects_with_ray (MC/BoundingVolume.h:173-215) for a ray with a finite reciprocal
// direction: per axis the near plane distance is min((lo - o) * rcp, (hi - o) * rcp) -- the
// correctly rounded subtraction and multiplication are monotone, so the min is exactly the value of
// the plane the reference selects by the direction's sign -- and no term can be NaN (rt_device.h
// slab_hit_finite).  sx = (lo.x - o.x, hi.x - o.x), ... in the halves of packed registers: one
// v_pk_mul_f32 per axis gives both plane distances, each rounded as the scalar product.
__device__ __forceinline__ bool box_hit_pk(const f2 sx, const f2 sy, const f2 sz, const V3& rc)
{
    const f2 ax = sx * f2{rc.x, rc.x}, ay = sy * f2{rc.y, rc.y}, az = sz * f2{rc.z, rc.z};
    const float tin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(ax.x, ax.y), __builtin_fminf(ay.x, ay.y)), __builtin_fminf(az.x, az.y));
    const float tout = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(ax.x, ax.y), __builtin_fmaxf(ay.x, ay.y)), __builtin_fmaxf(az.x, az.y));
    return (tout >= 0.0f) && (tin <= tout);
}
// the same, and the box is not entered beyond `bound`: a shadow ray's box entered beyond the light point
// holds no blocker (a blocker needs t <= slen - 0.01, MC/Renderer.cpp:184, and a triangle inside the box
// hits at t >= its entry; the bound keeps 1e-5 relative margin over the entry's 2e-7 rounding)
__device__ __forceinline__ bool box_hit_pk_within(const f2 sx, const f2 sy, const f2 sz, const V3& rc, float bound)
{
    const f2 ax = sx * f2{rc.x, rc.x}, ay = sy * f2{rc.y, rc.y}, az = sz * f2{rc.z, rc.z};
    const float tin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(ax.x, ax.y), __builtin_fminf(ay.x, ay.y)), __builtin_fminf(az.x, az.y));
    const float tout = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(ax.x, ax.y), __builtin_fmaxf(ay.x, ay.y)), __builtin_fmaxf(az.x, az.y));
    return (tout >= 0.0f) && (tin <= tout) && (tin <= bound);
}

// a finished sample's radiance into its parked slot (4-frame blocks: the 4 frames of a block of one pixel
// are 48 contiguous bytes); finalize_chunks_kernel accumulates every pixel's samples in frame order
template <class KP>
__device__ __forceinline__ void park_sample(KP& Q, V3 L, uint32_t local, uint32_t fidx)
{
    const size_t blk = Q.lbuf_pixel_major ? (size_t)local * ((Q.n_frames + 3u) >> 2) + (fidx >> 2) : (size_t)(fidx >> 2) * Q.lbuf_stride + local;
    const size_t at = (blk * 4u + (fidx & 3u)) * 3u;
    Q.lbuf[at] = L.x;
    Q.lbuf[at + 1] = L.y;
    Q.lbuf[at + 2] = L.z;
}

__device__ __forceinline__ V3 rcp3(V3 d) { return V3{rcp_f32(d.x), rcp_f32(d.y), rcp_f32(d.z)}; }
__device__ __forceinline__ bool finite3(V3 v) { return __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z); }

}  // namespace

// minimum waves per SIMD the register allocation must admit: 8 = at most 64 VGPRs (no VGPR spill; a
// few SGPRs spill to VGPR lanes) and 78 SGPRs, so 8 blocks of 256 lanes are resident per CU -- the
// hardware admits min(8, 800 / (ceil(sgpr / 16) * 16 + 16)) blocks (MI355X_MICROARCH.md, Residency),
// one fewer than the occupancy API at 82-96 SGPRs -- with 15 LDS words per lane (+1-2 % over 7; 7 / 6
// waves: C4 +0.2 % / -1.9 %, profiles/r02/ab/ab_waves_per_simd_*)
#ifndef RT_COH_MIN_WAVES
#define RT_COH_MIN_WAVES 8
#endif
// the BVH variant (scenes without decisive leaf boxes, e.g. C5): minimum waves per SIMD (without / with the
// camera pre-pass)
#ifndef RT_COH_BVH_MIN_WAVES
#define RT_COH_BVH_MIN_WAVES 8
#endif
#ifndef RT_BVH_DIV_FAST   // the BVH variant's divisions: IEEE sequences (0) or rt_device.h div_fast (1, A/B)
#define RT_BVH_DIV_FAST 0
#endif
#ifndef RT_COH_BVH_PRE_MIN_WAVES
#define RT_COH_BVH_PRE_MIN_WAVES 7
#endif
// section timing (diagnostic builds, tools/prof_one.py --sections / --hist; compiled by
// tests/test_build_variants.py): wave cycles spent in fold drain (top) / vertex / finish / work queue +
// service head / camera / box loop / Moller-Trumbore, summed into counters[16..23]
#ifndef RT_SECTIONS
#define RT_SECTIONS 0
#endif
// event counts of a sections build: [0] wave iterations, [1] lanes on a path, [2] vertex lanes,
// [3] finishing lanes, [4] camera lanes, [5] MT loop wave iterations, [6] MT lanes tested,
// [7] (lane, candidate) pairs, [8] 64-pair chunks, [9] finishing wave iterations with a fold still
// draining, [10] lanes finishing with a fold still draining, [11] lanes draining at the top,
// [12] MT lanes on ray A, [13] ray A pairs, [14] MT hits (fp64 part passed), [15] scratch, [16..18]
// distinct candidate triangles of the wave (ray A, ray B, either)
#define RT_SEC_COUNTS 20

// Tuned constants (A/B history: DESIGN.md 6.4, profiles/r02/ab/):
//  * leaf boxes per scalar-load group in the box loop (round 2: 4 boxes per wait +0.9 % over 1; after the
//    pre-pass and the tile cull, 1 box per wait +2.3 % over 4 at C4, profiles/r03/ab/ab_c4_box_unroll.json);
//  * fold levels drained per iteration at the top of the loop, their ring loads issued together (a fold
//    then rarely still drains when the next path ends): C4 1 level 5935, 2 6117, 3 6198, 4 6195 Msamples/s;
//  * ring levels loaded together when a fold is completed at once (drain_all).
#ifndef RT_BOX_UNROLL
#define RT_BOX_UNROLL 1
#endif
#ifndef RT_DRAIN_STEP
#define RT_DRAIN_STEP 3
#endif
#ifndef RT_DRAIN_BATCH
#define RT_DRAIN_BATCH 2
#endif

// pending fold (leaf-box variant, EXACT): a path that ends while the lane's previous fold still drains parks
// its own fold behind it (one ring slot holds its L and frame index) instead of completing the draining one
// at once -- that completion ran a whole fold loop for the one or two lanes that needed it in 83 % of the
// wave iterations (profiles/r03/c5_final/sections_c4_256spp.txt: fin_iters_with_drain)
#ifndef RT_PEND_FOLD
#define RT_PEND_FOLD 1
#endif
// the fold's two divisions (/PDF, /RR) by one wave-uniform range test and Markstein's correction for the three
// components (rt_device.h div2_core), instead of div_fast's per-component compare pairs and exec-mask branches
#ifndef RT_FOLD_DIV2
#define RT_FOLD_DIV2 1
#endif
// the same in the BVH variant's fold (whose other divisions keep the IEEE sequences, RT_BVH_DIV_FAST): C5
// 3840x2160x64 5842 -> 5973 Msamples/s, bitwise (the per-component div_fast had cost this variant registers)
#ifndef RT_BVH_FOLD_DIV2
#define RT_BVH_FOLD_DIV2 1
#endif
// (the same for the direct term's two divisions in the BVH variant: C5 +0.1 %, within the spread --
// profiles/r05/ab/ab_c5_nf_planes.json -- not kept)
// the BVH variant's rounds walk a lane's two rays TOGETHER when both are pending (round 6): ray B rides in a
// second walk slot of the near-first walk, its node load issued with ray A's, so a lane has two independent
// node loads in flight instead of one (the walk waits on dependent loads: SQ_WAIT_ANY 45 %, profiles/r05/c5)
#ifndef RT_BVH_PAIR
#define RT_BVH_PAIR 0
#endif
// the walk fallback (a non-finite reciprocal direction) and the pre-pass's walk without the sphere branch: these kernels
// never see a sphere (rt_capi.cpp: scenes with spheres render on the megakernel); 1 keeps it (4 spilled VGPRs in the
// leaf-box path kernel, 78 instead of 73 in the pre-pass: DESIGN.md 5.1)
#ifndef RT_COH_SPH
#define RT_COH_SPH 0
#endif
// the leaf-box variant's Moller-Trumbore on packed pairs (rt_device.h moller_trumbore_pk: the same IEEE operations, 12
// VALU fewer): C4 -3.3 %, bitwise (profiles/r06/ab/ab_c4_mt_packed.json) -- a v_pk_*_f32 of a wave64 occupies the
// SIMD twice as long as the scalar instruction on gfx950, so packing buys no issue cycles, and the build spills 2
// VGPRs; off (debug_primitives_kernel still checks the packed form against moller_trumbore_od bit for bit)
// the shadow ray's candidates tested from the last DFS triangle down (RT_B_TOP_FIRST=1; any order gives the verdict):
// C4 12,148 -> 11,803, C2 6762 -> 6564, bitwise (profiles/r06/ab/ab_c{4,2}_b_top_first.json) -- the DFS order already
// meets the Cornell blocks' faces first; off
// the leaf-box variant's candidate loop over two 32-bit masks (ray A's, then ray B's) instead of one 64-bit mask:
// 32-bit scans and clears, no 64-bit add; C4 +0.6 % / +0.5 % (both orders), C2 +0.7 %, bitwise
// (profiles/r06/ab/ab_c{4,2}_mt_loop32*.json)
// the BVH variant's split-phase candidate loop over two 32-bit masks (ray A's outside slots, then ray B's) instead of one
// 64-bit mask, as RT_MT_LOOP32 below: C5 3840x2160x32 path kernel 40.61 -> 40.35 ms and 40.52 -> 40.39 ms in the two A/B
// orders, bitwise (profiles/r06/ab/ab_c5_split_loop32*.json)
#ifndef RT_SPLIT_LOOP32
#define RT_SPLIT_LOOP32 1
#endif
#ifndef RT_MT_LOOP32
#define RT_MT_LOOP32 1
#endif
#ifndef RT_B_TOP_FIRST
#define RT_B_TOP_FIRST 0
#endif
#ifndef RT_MT_PK
#define RT_MT_PK 0
#endif
constexpr int BOX_UNROLL = RT_BOX_UNROLL;
constexpr uint32_t DRAIN_STEP = RT_DRAIN_STEP;
constexpr uint32_t DRAIN_BATCH = RT_DRAIN_BATCH;
// fold ring layout: lane-major ([thread][position]): a lane's consecutive levels share cache lines, so a
// drain read follows its push in L2
// (a 32-bit index: lanes x depth < 2^32, checked on the host; one register for the lane's base, no 64-bit product)
// (gtid < 2^20 and the ring < 2^12 positions: the 24-bit multiply is exact and full rate, rt_capi.cpp keeps the
// ring's total size below 2^32)
#define RING_AT(p) ((uint32_t)(__umul24(gtid, Q.stack_depth) + (p)))

struct FiniteSlab { static constexpr bool value = true; };
struct GeneralSlab { static constexpr bool value = false; };

// BVH = false: the scene in LDS, both rays against the distinct leaf boxes (one wave-uniform loop).
// BVH = true: the scene in HBM (read through L2/MALL); the two rays of a lane walk the stackless BVH
// one after the other (A, then B) in the megakernel's rounds of `steps` box tests with up to two
// postponed leaves, and a lane is served once both of its rays are done.
// NARROW (leaf-box variant, <= 32 triangles): ray A's and ray B's candidates in the two halves of one mask.
// PREPASS: paths start at their first surface vertex from the camera pre-pass's records (the leaf-box variant
// always; the BVH variant for split scenes, rt_capi.cpp), else the kernel traces the camera rays itself.
template <bool EXACT, bool BVH, bool NARROW, bool PREPASS>
__global__ void __launch_bounds__(256, BVH ? (PREPASS ? RT_COH_BVH_PRE_MIN_WAVES : RT_COH_BVH_MIN_WAVES) : RT_COH_MIN_WAVES) pt_coherent_kernel(KParams P)
{
    extern __shared__ __attribute__((aligned(16))) float4 lds_scene[];
    SceneView S;
    S.n_nodes = P.n_nodes;
    if (BVH) {
        S.nodes = P.nodes; S.tris = P.tris; S.mats = P.mats; S.lnodes = P.lnodes; S.ltris = P.ltris; S.lboxes = nullptr;
        uint32_t at = 0;
        {
            // the small tables in LDS (mats | lnodes | ltris; the host runs this variant only when they fit):
            // the service's material and the light sample wait on no HBM load, and every access to them is
            // an LDS read with a 32-bit address (a table that could be in LDS or HBM is a generic pointer:
            // flat loads and 64-bit addresses in VGPRs)
            const uint32_t mq = 2 * P.n_mats, lq = P.n_lnodes, ltq = 4 * P.n_ltris;
            float4* dm = lds_scene;
            float4* dl = dm + mq;
            float4* dlt = dl + lq;
            for (uint32_t i = threadIdx.x; i < mq; i += blockDim.x) dm[i] = P.mats[i];
            for (uint32_t i = threadIdx.x; i < lq; i += blockDim.x) dl[i] = P.lnodes[i];
            for (uint32_t i = threadIdx.x; i < ltq; i += blockDim.x) dlt[i] = P.ltris[i];
            S.mats = dm; S.lnodes = dl; S.ltris = dlt;
            at = mq + lq + ltq;
        }
        if (P.split_root != 0u) {
            // the split's outside triangles by slot (a, e1, (e2, bits(triangle))): a candidate's
            // Moller-Trumbore reads LDS instead of a slot -> triangle -> vertices chain of HBM loads
            float4* ds = lds_scene + at;
            for (uint32_t i = threadIdx.x; i < 3u * P.n_split_leaves; i += blockDim.x) {
                const uint32_t k = i / 3u, j = i - 3u * k;
                const int tri = P.stri[k];
                float4 v = P.tris[4 * tri + j];
                if (j == 2u) v.w = __int_as_float(tri);
                ds[i] = v;
            }
        }
        if (P.lds_scene_quads != 0u) __syncthreads();
    } else {
        // stage the scene into LDS once per workgroup: tris | mats | lnodes | ltris (the BVH nodes stay in
        // HBM -- only a ray with a non-finite reciprocal direction walks them -- and the leaf boxes are read
        // with scalar loads)
        const uint32_t tq = 4 * P.n_tris, mq = 2 * P.n_mats, lq = P.n_lnodes, ltq = 4 * P.n_ltris;
        float4* dt = lds_scene;
        float4* dm = dt + tq;
        float4* dl = dm + mq;
        float4* dlt = dl + lq;
        for (uint32_t i = threadIdx.x; i < tq; i += blockDim.x) dt[i] = P.tris[i];
        for (uint32_t i = threadIdx.x; i < mq; i += blockDim.x) dm[i] = P.mats[i];
        for (uint32_t i = threadIdx.x; i < lq; i += blockDim.x) dl[i] = P.lnodes[i];
        for (uint32_t i = threadIdx.x; i < ltq; i += blockDim.x) dlt[i] = P.ltris[i];
        __syncthreads();
        S.nodes = P.nodes; S.tris = dt; S.mats = dm; S.lnodes = dl; S.ltris = dlt; S.lboxes = nullptr;
    }

    const uint32_t lane = __lane_id();
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t tib = threadIdx.x;
    // the lane's cold state after the scene (the host gives this kernel no LDS fold levels)
    float* lstate = reinterpret_cast<float*>(lds_scene + P.lds_scene_quads);
    auto lsf = [&](uint32_t f) -> float& { return lstate[f * 256u + tib]; };
    auto lsu = [&](uint32_t f) -> uint32_t& { return reinterpret_cast<uint32_t*>(lstate)[f * 256u + tib]; };
    auto ls3 = [&](uint32_t f) { return V3{lsf(f), lsf(f + 1), lsf(f + 2)}; };
    auto st3 = [&](uint32_t f, V3 v) { lsf(f) = v.x; lsf(f + 1) = v.y; lsf(f + 2) = v.z; };
    const float PDF = 1.0f / (2.0f * PI_F);   // WhittedMaterial::PDF_at_the_sample, MC/WhittedMaterial.h:44-56
    // the leaf-box variant divides with rt_device.h div_fast (y = the divisor's correctly rounded
    // reciprocal; C4 +1.1 %); the BVH variant keeps the IEEE division sequence (its register budget: C5
    // -2.5 % with div_fast)
    constexpr bool IEEE_DIV = BVH && !RT_BVH_DIV_FAST;
    auto sdiv = [](float x, float d, float y) { return IEEE_DIV ? x / d : div_fast(x, d, y); };
    auto vdiv = [](V3 a, float d, float y) { return IEEE_DIV ? divs(a, d) : divs_fast(a, d, y); };
    // a finished sample is parked in the frame-major sample buffer (4-frame blocks: the 4 frames of a
    // block of one pixel are 48 contiguous bytes); finalize_chunks_kernel then accumulates every
    // pixel's samples in frame order (MC/Renderer.cpp:128-133).  The kernel issues no global load
    // after a store of the same iteration: on gfx950 a load waits for every older store of its wave
    // (vmcnt counts both), and a path-tracing iteration that read the accumulator after its parked
    // samples and fold-level stores waited for their write-back.
    auto complete = [&](V3 L, uint32_t local, uint32_t fidx) { park_sample(kargs4(), L, local, fidx); };
    // x mod R for x in [0, 2R): every ring-distance expression below is a position (< R) plus R minus a
    // position or a level count in [1, R), so one conditional subtract replaces the generic 32-bit remainder
    auto ring_wrap = [](uint32_t x, uint32_t R) { return x >= R ? x - R : x; };
    // up to N fold steps of the draining path, L = Ld_k + ((((L * brdf_k) * cos_k) / PDF) / RR)
    // (MC/Renderer.cpp:208,213), inner level first, from ring position `pos` down; the N ring loads are
    // issued together (levels past the fold re-read the first one, unused).  Returns the levels folded.
    auto fold_n = [&](auto NC, uint32_t& pos, uint32_t dleft, V3& L) -> uint32_t {
        constexpr uint32_t N = decltype(NC)::value;
        CKParams& Q = kargs4();
        const uint32_t R = Q.stack_depth;
        float4 e[N];
        int m[N];
        uint32_t at[N];
#pragma unroll
        for (uint32_t j = 0; j < N; ++j) {
            const uint32_t pj = pos >= j ? pos - j : pos + R - j;
            at[j] = RING_AT(j < dleft ? pj : pos);
            e[j] = Q.stack_ld[at[j]];
        }
#pragma unroll
        for (uint32_t j = 0; j < N; ++j) ring_unpack(Q, at[j], e[j], m[j]);
#pragma unroll
        for (uint32_t j = 0; j < N; ++j) {
            if (j < dleft) {
                const float4 mb2 = S.mats[2 * m[j]];
                const V3 f = (e[j].w >= 0.0f) ? V3{mb2.x, mb2.y, mb2.z} : V3{0.0f, 0.0f, 0.0f};
                const V3 x = muls(mul(L, f), e[j].w);
                V3 q;
                // both divisions on Markstein's exact path when every lane's numerator is in range (rt_device.h
                // div2_fast_range; the host sets rr_fast when RR lies in [2^-20, 1)): one wave-uniform test
                // instead of a compare pair and an exec-mask branch per component and division
                if ((!IEEE_DIV || RT_BVH_FOLD_DIV2) && RT_FOLD_DIV2 && Q.rr_fast && __all(div2_fast_range(x))) q = div2_core(x, PDF, Q.y_pdf, Q.rr, Q.y_rr);
                else q = vdiv(vdiv(x, PDF, Q.y_pdf), Q.rr, Q.y_rr);
                L = add(V3{e[j].x, e[j].y, e[j].z}, q);
            }
        }
        const uint32_t n = dleft < N ? dleft : N;
        pos = pos >= n ? pos - n : pos + R - n;
        return n;
    };
    // the pending fold (PEND): a finished path's fold waiting behind the draining one (lane flag hasPend; its
    // ring position | levels << 12 in VS_PEND, its local pixel in VS_PLOC, and (L, frame index) in the ring slot
    // above its top level)
    constexpr bool PEND = EXACT && !BVH && RT_PEND_FOLD != 0;
    bool hasPend = false;
    auto pend_meta_at = [&](uint32_t pd) -> size_t {
        CKParams& Q = kargs4();
        uint32_t mp = (pd & 0xFFFu) + 1u;
        if (mp >= Q.stack_depth) mp -= Q.stack_depth;
        return RING_AT(mp);
    };
    // the top of an iteration: DRAIN_STEP levels of the draining fold.  A lane whose fold completed in an
    // earlier iteration and which holds a pending one starts that here: its slot is loaded with the levels
    // (at the top of the iteration no store precedes the loads)
    auto drain_step = [&](uint32_t& dleft) {
        uint32_t pos, fid = 0;
        V3 L;
        bool act = false;
        if (PEND && dleft == 0u) {
            const uint32_t pd = lsu(VS_PEND);
            const float4 meta = kargs4().stack_ld[pend_meta_at(pd)];
            L = V3{meta.x, meta.y, meta.z};
            fid = __float_as_uint(meta.w);
            pos = pd & 0xFFFu;
            dleft = pd >> 12;
            act = true;
            hasPend = false;
        } else {
            pos = lsu(VS_DPOS);
            L = ls3(VS_DL);
        }
        dleft -= fold_n(std::integral_constant<uint32_t, DRAIN_STEP>{}, pos, dleft, L);
        if (PEND && act) {
            lsu(VS_DT0) = lsu(VS_PLOC);
            lsu(VS_DT1) = fid;
        }
        if (dleft == 0u) {
            complete(L, lsu(VS_DT0), lsu(VS_DT1));
        } else {
            st3(VS_DL, L);
            lsu(VS_DPOS) = pos;
        }
    };
    // the rest of a draining fold at once: the wave waits for one load latency per DRAIN_BATCH levels instead
    // of one per level; with PEND a pending fold is completed too
    auto drain_all = [&](uint32_t& dleft) {
        if (dleft != 0u) {
            uint32_t pos = lsu(VS_DPOS);
            V3 L = ls3(VS_DL);
            while (dleft != 0u) dleft -= fold_n(std::integral_constant<uint32_t, DRAIN_BATCH>{}, pos, dleft, L);
            complete(L, lsu(VS_DT0), lsu(VS_DT1));
        }
        if (PEND && hasPend) {
            const uint32_t pd = lsu(VS_PEND);
            const float4 meta = kargs4().stack_ld[pend_meta_at(pd)];
            V3 L = V3{meta.x, meta.y, meta.z};
            uint32_t pos = pd & 0xFFFu, left = pd >> 12;
            while (left != 0u) left -= fold_n(std::integral_constant<uint32_t, DRAIN_BATCH>{}, pos, left, L);
            complete(L, lsu(VS_PLOC), __float_as_uint(meta.w));
            hasPend = false;
        }
    };

    // PRE (the leaf-box variant): camera rays are traced by the pre-pass (camera_prepass_kernel) and a path
    // starts here at its first surface vertex; the BVH variant traces its camera rays itself (a pre-pass
    // cost it more than it saved, DESIGN.md 5.1: its time is in the secondary rays' BVH walks)
    constexpr bool PRE = PREPASS;
    bool alive = true, in_path = false;
    bool have_pixel = false;   // !PRE: the lane holds a work item (frame chunk, pixel)
    uint32_t k = 0;            // !PRE: frame of the current item (item of chunk c: frames c * chunk_frames + [0, kend))
    bool pend = false;         // !PRE: the last vertex waits for its shadow verdict (false: the camera ray's hit)
    uint32_t pool_base = 0, pool_count = 0;   // !PRE: the wave's batch of work items (wave-uniform)
    bool cont = false;    // the last vertex's roulette continued: ray A is its indirect ray
    VertexRng g;
    g.w = reinterpret_cast<uint32_t*>(lstate) + tib;
    g.k0 = (uint32_t)P.seed; g.k1 = (uint32_t)(P.seed >> 32);
    // the lane's rays: A = indirect (!PRE: or camera) ray (closest hit), B = shadow ray (any hit); shared origin
    V3 o{0.f, 0.f, 0.f}, dA{0.f, 0.f, 1.f}, rA{0.f, 0.f, 1.f}, dB{0.f, 0.f, 1.f}, rB{0.f, 0.f, 1.f};
    bool hasA = false, hasB = false;
    float slen = 0.0f;                        // length(q - p) of the shadow ray
    // closest t: the reference's IntersectionRecord default is DBL_MAX.  The BVH variant starts from +inf
    // instead, an inline constant (DBL_MAX is a 64-bit literal the register allocator spilled): every t the
    // intersection yields is +inf or at most FLT_MAX * 2^149 (a float over a float's double reciprocal), so
    // `t < tA` is the same test, and a tie at +inf is refused by the unsigned triangle compare (triA = -1)
    constexpr double TA_NONE = BVH ? __builtin_inf() : 1.7976931348623157e308;
    double tA = TA_NONE;
    V3 hloc{0.f, 0.f, 0.f};                   // !BVH: ray A's hit location (from the trace) ...
    bool hflip = false;                       // ... and whether its normal faces away from -dA
    int triA = -1;                            // closest triangle
    bool occB = false;                        // shadow ray blocked
    // EXACT: a finished path's levels are folded DRAIN_STEP per iteration ("drain"), not in a loop at the
    // end of the path: lanes end paths of different depths, and a fold loop runs as long as the deepest
    // one.  Levels live in a per-lane ring of stack_depth positions in HBM; the next path pushes above the
    // draining segment.  Every sample has its own parked slot, which finalize_chunks_kernel adds in frame
    // order.
    uint32_t dleft = 0;                       // levels of the draining fold still to apply
    if (EXACT) lsu(VS_BASE) = 0u;
    // BVH: next node of ray A / ray B (NN: no ray or done); the traversal spans iterations
    const uint32_t NN = S.n_nodes;
    uint32_t tiA = NN, tiB = NN;
    // the wave's current segment of camera-hit records (wave-uniform): records [seg_pos, seg_end) are not
    // yet taken; the non-empty segments are taken one per device atomic from the pre-pass's list
    uint32_t seg_pos = 0, seg_end = 0;
    uint32_t wq = blockIdx.x & (P.n_work_queues - 1u), wq_dry = 0;   // the wave's work queue; queues found dry in a row
    bool list_left = true;

#if RT_SECTIONS
    uint64_t sec_cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t sec_t = clock64();
    // the launch's timeline in the chip-wide 100 MHz clock (wall_clock64): the wave's entry, the moment its
    // work queue ran dry, its exit -> counters[440..447] (tools/prof_one.py --sections prints the tail)
    const uint64_t tl_entry = wall_clock64();
    uint64_t tl_empty = 0;
    int sec_cur = 7;
#define SEC_MARK(k) do { const uint64_t t_ = clock64(); sec_cyc[sec_cur] += t_ - sec_t; sec_t = t_; sec_cur = (k); } while (0)
    // wave-level event counts in the wave's LDS slot (RT_SEC_COUNTS words, written by the wave's first
    // active lane; tools/prof_one.py --sections names them)
    __shared__ uint32_t sec_cnt[4][RT_SEC_COUNTS];
    uint32_t* const sec_w = sec_cnt[threadIdx.x >> 6];
    if (lane < RT_SEC_COUNTS) sec_w[lane] = 0u;
    bool dbg_vertex = false, dbg_fin = false, dbg_cam = false;
    auto sec_first = [&]() { return lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1); };
#define SEC_COUNT(i, v) do { const uint32_t v_ = (v); if (sec_first()) sec_w[i] += v_; } while (0)
#define SEC_SUM(i, v) do { atomicAdd(&sec_w[i], (uint32_t)(v)); } while (0)
#else
#define SEC_COUNT(i, v) do { } while (0)
#define SEC_SUM(i, v) do { } while (0)
#define SEC_MARK(k) do { } while (0)
#endif
    // Lanes that need a sample take the wave's next records, in lane order (wave-collective); returns the
    // lane's record index or NO_REC.  Called at the top of the iteration, before any store: the record
    // loads (and the segment fetch's returning atomic) then wait for no store of the iteration.
    constexpr uint32_t NO_REC = 0xFFFFFFFFu;
    auto take_records = [&](const bool need) -> uint32_t {
        uint32_t rec = NO_REC;
        uint64_t mask = __ballot(need);
        while (mask != 0) {
            if (seg_pos == seg_end) {
                if (!list_left) break;
                CKParams& Q = kargs4();
                uint32_t k = 0;
                if (lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) k = atomicAdd(Q.work_queues + 32u * wq, 1u);
                k = __builtin_amdgcn_readfirstlane(k) * Q.n_work_queues + wq;
                // (the list length is read here, once per segment, not kept live across the loop)
                // list entry k: part (k mod 2^ps) of listed segment k >> ps, a consecutive range of its records;
                // the list's last seg_tail_n segments in 2^seg_tail_shift finer parts, so the waves run dry
                // within a short part of each other at the end of the launch (the launch's tail)
                const uint32_t nl = __builtin_amdgcn_readfirstlane(*Q.seg_list_n);
                const uint32_t ps = Q.seg_part_shift, pt = Q.seg_tail_shift;
                const uint32_t head = nl - (nl < Q.seg_tail_n ? nl : Q.seg_tail_n);
                uint32_t idx, part, sh;
                if (k < (head << ps)) {
                    idx = k >> ps; part = k & ((1u << ps) - 1u); sh = ps;
                } else {
                    const uint32_t k2 = k - (head << ps);
                    if (k2 >= ((nl - head) << pt)) {
                        // this queue is dry (for good: its draws only grow): the next one, until every queue
                        // has been found dry in a row
                        wq = (wq + 1u) & (Q.n_work_queues - 1u);
                        if (++wq_dry < Q.n_work_queues) continue;
                        list_left = false;
#if RT_SECTIONS
                        tl_empty = wall_clock64();
#endif
                        break;
                    }
                    idx = head + (k2 >> pt); part = k2 & ((1u << pt) - 1u); sh = pt;
                }
                wq_dry = 0;
                const uint2 ent = Q.seg_list[idx];   // (segment, record count)
                const uint32_t sg = __builtin_amdgcn_readfirstlane(ent.x);
                const uint32_t cnt = __builtin_amdgcn_readfirstlane(ent.y);
                seg_pos = (sg << Q.seg_shift) + ((part * cnt) >> sh);
                seg_end = (sg << Q.seg_shift) + (((part + 1u) * cnt) >> sh);
                continue;
            }
            const uint32_t avail = seg_end - seg_pos;
            const uint32_t j = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
            if (((mask >> lane) & 1ull) && j < avail) rec = seg_pos + j;
            const uint32_t n = (uint32_t)__popcll(mask);
            seg_pos += n < avail ? n : avail;
            mask = __ballot(need && rec == NO_REC);
        }
        if (need && rec == NO_REC) alive = false;
        return rec;
    };
    // Lanes without a work item take the next ones from the wave's pool, in lane order.  With `refill`
    // (the top of the iteration, before any store) an empty pool is refilled from the device counter;
    // without it (after the path-end block, so a lane whose item just ended starts the next one's camera
    // ray in the same iteration) only the pool's items are handed out -- no atomic, so nothing waits for
    // the iteration's stores.  (!PRE)
    auto take_items = [&](const bool refill) {
        const bool need = alive && !have_pixel;
        const uint64_t mask = __ballot(need);
        if (mask == 0) return;
        CKParams& Q = kargs4();
        uint32_t n = (uint32_t)__popcll(mask);
        if (!refill && n > pool_count) n = pool_count;
        if (n == 0) return;
        uint32_t fresh = 0;   // first item of a new batch (wave-uniform)
        if (n > pool_count) {
            uint32_t b = 0;
            if (lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) b = atomicAdd(Q.work_counter, 64u);
            fresh = __builtin_amdgcn_readfirstlane(b);
        }
        const uint32_t j = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
        if (need && j < n) {
            const uint32_t w = j < pool_count ? pool_base + j : fresh + (j - pool_count);
            if (w >= Q.n_items) {
                alive = false;
            } else {
                // item = (frame chunk, pixel), chunk-major; 8x8 tile swizzle in local (row, column) space
                const uint32_t c = w / Q.items_per_chunk, wp = w - c * Q.items_per_chunk;
                const uint32_t tile = wp >> 6, within = wp & 63u;
                const uint32_t trow = tile / Q.tiles_x, tcol = tile - trow * Q.tiles_x;
                const uint32_t lr = trow * 8u + (within >> 3), lx = tcol * 8u + (within & 7u);
                if (lr < Q.n_local_rows && lx < Q.W) {
                    // local row -> global row (row bands dealt round-robin over ranks)
                    const uint32_t band_k = lr / Q.band, in_band = lr - band_k * Q.band;
                    const uint32_t y = (Q.rank + band_k * Q.nranks) * Q.band + in_band;
                    const uint32_t local = lr * Q.W + lx;
                    lsu(VS_LOCAL) = local;
                    lsu(VS_PIX) = y * Q.W + lx;
                    lsu(VS_FRAME) = Q.first_frame + c * Q.chunk_frames;   // the frame of the item's first sample
                    have_pixel = true;
                    k = 0;
                }
            }
        }
        // (64 items per refill: a wave's pool never holds more than one item per lane, so the launch
        // tail stays one item long)
        if (n > pool_count) {
            pool_base = fresh + (n - pool_count);
            pool_count = 64u - (n - pool_count);
        } else {
            pool_base += n;
            pool_count -= n;
        }
    };
    for (;;) {
        SEC_MARK(0);
        // (the leaf-box variant's rays are set up and traced within an iteration: not loop-carried)
        if constexpr (!BVH) { o = V3{0.f, 0.f, 0.f}; dA = o; dB = o; }
        // ======================= the lanes whose path ends in this iteration's service =======================
        // decided from the trace results before any store: the roulette stopped, or the indirect ray missed or
        // hit the light (radiance_indirect = 0, MC/Renderer.cpp:193-209).  They and the idle lanes take their
        // next sample now, so a finishing lane shades its next path's first vertex in the same iteration.
        const bool served = in_path && (!BVH || (tiA >= NN && tiB >= NN));
        uint32_t depth = 0;   // vertices shaded so far on this path (from VS_MAT at the service; 0 for a new path)
        int mat = 0;
        bool emissive = false;
        if (served && hasA && triA >= 0) {
            mat = f2i(S.tris[4 * triA].w);
            emissive = S.mats[2 * mat].w != 0.0f;
        }
        // (a path ends at a vertex's service; a camera ray's service is its hit: !PRE, or the BVH variant's camera
        // rays the pre-pass left to it)
        const bool ends = served && ((PRE && !BVH) || pend) && (!cont || triA < 0 || emissive);
        // (as many fold levels as the wave's deepest drain needs instead of DRAIN_STEP, a wave-uniform choice
        // of 1 / 2 / 3: C4 -0.4 %, C5 +-0, profiles/r05/ab/ab_c{4,5}_drain_adapt.json)
        if (EXACT && __any(dleft != 0u || hasPend)) {
            if (dleft != 0u || hasPend) drain_step(dleft);
        }
        // (after the drain's ring loads are folded: the record's registers are then not live across them.
        // Issuing the record loads before the drain's, so that the two latencies overlap, measured -0.2 % at
        // C4 256 spp, profiles/r05/ab/ab_c4_rec_first.json)
        uint32_t rid = NO_REC;
        float4 rec = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (PRE) {
            rid = take_records(alive && (!in_path || ends));
            if (rid != NO_REC) rec = kargs4().crec[rid];
        }
        SEC_MARK(3);
        // !PRE: at the top of the iteration, before any store, a lane that finished its item takes the next
        // one (the returning atomic waits for no store of this iteration)
        if constexpr (!PRE) take_items(true);

        // ======================= service: the lanes whose rays are back =======================
        bool vertex = false;   // a surface vertex to shade: the indirect ray's hit, or a new path's camera hit
        if (served) {
            CKParams& Q = kargs4();
            bool finished = false;
            int fold_top = -1;   // EXACT: stack levels fold_top..0 are folded into L when the path ends
            bool relisted = false;   // EXACT: the sample went to the overflow list (no fold, no parked store)
            V3 L{0.f, 0.f, 0.f};
            if ((!PRE || BVH) && !pend) {
                // the camera ray's hit (cast_path, MC/Renderer.cpp:136-146)
                if (triA < 0) {   // miss: night sky (:145)
                    L = night_sky();
                    finished = true;
                } else if (emissive) {   // direct emission (:151-161)
                    const float4 em = S.mats[2 * mat + 1];
                    L = V3{em.x, em.y, em.z};
                    finished = true;
                } else {
                    vertex = true;
                }
            } else {
                // the last vertex's direct term (MC/Renderer.cpp:184-189): the shadow verdict
                const uint32_t vmat = lsu(VS_MAT);
                depth = vmat >> VS_DEPTH_SHIFT;
                V3 ld{0.f, 0.f, 0.f};
                if (hasB && !occB) ld = ls3(VS_LD);
                if (!EXACT) {
                    const V3 thr = ls3(VS_THR);
                    const V3 lsum = add(ls3(VS_LSUM), mul(thr, ld));
                    if (ends) {
                        L = lsum;
                        finished = true;
                    } else {
                        st3(VS_LSUM, lsum);
                        const float c = lsf(VS_PCOS);
                        const float4 mb = S.mats[2 * (vmat & VS_MAT_MASK)];
                        const V3 f = (c >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};
                        st3(VS_THR, muls(mul(thr, f), sdiv(sdiv(c, PDF, Q.y_pdf), Q.rr, Q.y_rr)));
                        vertex = true;
                    }
                } else if (ends) {
                    L = ld;
                    fold_top = (int)depth - 2;
                    finished = true;
                } else {
                    // the indirect ray hit a surface: vertex depth-1 becomes stack level depth-1
                    const uint32_t lvl = depth - 1;
                    const float4 e = make_float4(ld.x, ld.y, ld.z, lsf(VS_PCOS));
                    const uint32_t pm = vmat & VS_MAT_MASK;
                    const uint32_t R = Q.stack_depth;
                    uint32_t pos = lsu(VS_BASE) + lvl;
                    if (pos >= R) pos -= R;
                    // the ring holds this path's levels above the draining ones, which occupy the R positions
                    // [dpos - dleft + 1, dpos]: a level must fit in the ring and not land on an undrained one
                    // (with a pending fold behind the draining one, going up from here the draining levels come
                    // first; between a fold's completion and the pending one's start, the pending levels and
                    // their slot)
                    bool fits = lvl < R;
                    if (fits && dleft != 0u) {
                        const uint32_t lo = ring_wrap(lsu(VS_DPOS) + R + 1u - dleft, R);
                        fits = ring_wrap(pos + R - lo, R) >= dleft;
                    } else if (PEND && fits && hasPend) {
                        const uint32_t pd = lsu(VS_PEND), pm = pd >> 12;
                        const uint32_t lo = ring_wrap((pd & 0xFFFu) + R + 1u - pm, R);
                        fits = ring_wrap(pos + R - lo, R) >= pm + 1u;
                    }
                    if (fits) {
                        if (Q.ring_pack) {
                            // the material in the sign bits of the direct term (rt_kernels.h ring_pack)
                            const float4 pe = make_float4(__uint_as_float((__float_as_uint(e.x) & 0x7FFFFFFFu) | ((pm & 1u) << 31)),
                                                          __uint_as_float((__float_as_uint(e.y) & 0x7FFFFFFFu) | ((pm & 2u) << 30)),
                                                          __uint_as_float((__float_as_uint(e.z) & 0x7FFFFFFFu) | ((pm & 4u) << 29)), e.w);
                            Q.stack_ld[RING_AT(pos)] = pe;
                        } else {
                            Q.stack_ld[RING_AT(pos)] = e;
                            Q.stack_mat[RING_AT(pos)] = pm;
                        }
                        vertex = true;
                    } else {
                        // the path outgrew the ring: list the sample for the exact re-render
                        // (rt_resample.hip) and end it here; its parked slot is written there
                        const uint32_t slot = (uint32_t)atomicAdd((unsigned long long*)&Q.counters[3], 1ull);
                        const uint32_t frame = lsu(VS_FRAME);
                        if (slot < Q.ovf_cap) {
                            Q.ovf_list[slot] = make_uint4(lsu(VS_LOCAL), frame - Q.first_frame, lsu(VS_PIX), frame);
                            atomicAdd((unsigned long long*)&Q.counters[14], 1ull);
                        } else {
                            atomicAdd((unsigned long long*)&Q.counters[13], 1ull);   // lost: rt_render reports it
                        }
                        finished = true;
                        relisted = true;
                    }
                }
            }
            SEC_MARK(1);
#if RT_SECTIONS
            dbg_fin = finished;
#endif
            if (finished) {
                in_path = false;
                hasA = hasB = false;
                const uint32_t local = lsu(VS_LOCAL), frame = lsu(VS_FRAME);
                const uint32_t fidx = frame - Q.first_frame;   // the sample's frame index in this launch
                if (!PRE) {   // the item's next frame, or the end of the item
                    const uint32_t kbase = fidx - k;   // the item's first frame index
                    ++k;
                    lsu(VS_FRAME) = frame + 1u;
                    if (k == min(Q.chunk_frames, Q.n_frames - kbase)) have_pixel = false;
                }
                if (EXACT && relisted) {
                    // nothing to fold or park: resample_kernel writes this sample's slot
                } else if (EXACT) {
#if RT_SECTIONS
                    SEC_COUNT(9, __ballot(dleft != 0u) != 0 ? 1u : 0u);
                    SEC_COUNT(10, (uint32_t)__popcll(__ballot(dleft != 0u)));
#endif
                    const uint32_t m = (uint32_t)(fold_top + 1);
                    const uint32_t base = lsu(VS_BASE);
                    bool deferred = false;
                    if (PEND && m != 0u && dleft != 0u && !hasPend) {
                        // the previous fold still drains: this one waits behind it.  Its levels are ring positions
                        // base .. base + m - 1; the slot above them takes (L, frame index) unless it would land on
                        // the draining fold's undrained levels [lo, lo + dleft)
                        const uint32_t R = Q.stack_depth;
                        uint32_t top = base + m - 1u;
                        if (top >= R) top -= R;
                        uint32_t mp = top + 1u;
                        if (mp >= R) mp -= R;
                        const uint32_t lo = ring_wrap(lsu(VS_DPOS) + R + 1u - dleft, R);
                        if (m + 1u < R && ring_wrap(mp + R - lo, R) >= dleft) {
                            Q.stack_ld[RING_AT(mp)] = make_float4(L.x, L.y, L.z, __uint_as_float(fidx));
                            lsu(VS_PEND) = top | (m << 12);
                            lsu(VS_PLOC) = local;
                            hasPend = true;
                            uint32_t nb = mp + 1u;
                            if (nb >= R) nb -= R;
                            lsu(VS_BASE) = nb;   // the next path pushes above the pending fold
                            deferred = true;
                        }
                    }
                    // (a one-vertex path has no level: its sample is parked now, whatever still drains)
                    if (!deferred && !(PEND && m == 0u)) drain_all(dleft);   // the previous sample's fold completes first
                    if (deferred) {
                    } else if (m == 0u) {
                        complete(L, local, fidx);
                    } else {
                        // the fold drains from the innermost level, ring position base + m - 1
                        st3(VS_DL, L);
                        uint32_t top = base + m - 1u;
                        if (top >= Q.stack_depth) top -= Q.stack_depth;
                        lsu(VS_DPOS) = top;
                        lsu(VS_DT0) = local;
                        lsu(VS_DT1) = fidx;
                        dleft = m;
                        uint32_t nb = top + 1u;
                        if (nb >= Q.stack_depth) nb -= Q.stack_depth;
                        lsu(VS_BASE) = nb;   // the next path pushes above the draining levels
                    }
                } else {
                    complete(L, local, fidx);
                }
            }
        }
        if constexpr (!PRE) take_items(false);
        SEC_MARK(4);

        // ======================= the vertex to shade: (location, triangle, face-forward) =======================
        V3 loc;
        int tri;
        bool flip;
        if (PRE && rid != NO_REC) {
            // a new path from its camera-hit record: sample (pixel, frame) from the segment and the tag
            // (rt_kernels.h crec), the location and face-forwarded normal as the pre-pass computed them
            CKParams& Q = kargs4();
            const uint32_t tag = __float_as_uint(rec.w);
            const uint32_t sg = rid >> Q.seg_shift;
            // (with div24 every factor below is < 2^24 and every product < 2^32: 24-bit multiplies, full rate)
            const uint32_t c = udiv_u(sg, Q.n_tiles, Q.r_n_tiles, Q.div24), tile = sg - mul_u(c, Q.n_tiles, Q.div24);
            const uint32_t trow = udiv_u(tile, Q.tiles_x, Q.r_tiles_x, Q.div24), tcol = tile - mul_u(trow, Q.tiles_x, Q.div24);
            const uint32_t pit = (tag >> 19) & 63u;
            const uint32_t lr = trow * 8u + (pit >> 3), lx = tcol * 8u + (pit & 7u);
            // local row -> global row (row bands dealt round-robin over ranks)
            const uint32_t band_k = udiv_u(lr, Q.band, Q.r_band, Q.div24), in_band = lr - mul_u(band_k, Q.band, Q.div24);
            const uint32_t y = mul_u(Q.rank + mul_u(band_k, Q.nranks, Q.div24), Q.band, Q.div24) + in_band;
            const uint32_t pix = mul_u(y, Q.W, Q.div24) + lx;
            const uint32_t frame = Q.first_frame + mul_u(c, Q.seg_frames, Q.div24) + ((tag >> 25) & 63u);
            lsu(VS_LOCAL) = mul_u(lr, Q.W, Q.div24) + lx;
            lsu(VS_PIX) = pix;
            lsu(VS_FRAME) = frame;
            g.start(pix, frame, !Q.has_light);   // the vertex draws continue after the 2 camera draws
            depth = 0;
            in_path = true;
            if (!EXACT) { st3(VS_THR, V3{1.0f, 1.0f, 1.0f}); st3(VS_LSUM, V3{0, 0, 0}); }
            if (BVH && (tag & CREC_CAMERA) == CREC_CAMERA) {
                // a camera ray the pre-pass left to this kernel (it enters the walked subtree's box): traced here as a
                // fresh ray A -- the split phase, then the walk in the rounds -- whose hit the next service takes
                o = V3{Q.cam_pos[0], Q.cam_pos[1], Q.cam_pos[2]};
                dA = V3{rec.x, rec.y, rec.z};
                hasA = true; hasB = false;
                pend = false;
                tiA = 0u; tiB = NN;
                tA = TA_NONE; triA = -1; occB = false;
            } else {
                loc = V3{rec.x, rec.y, rec.z};
                tri = (int)(tag & 0x7FFFFu);
                flip = (tag >> 31) != 0u;
                mat = f2i(S.tris[4 * tri].w);
                vertex = true;
            }
#if RT_SECTIONS
            dbg_cam = true;
#endif
        } else {
            // the traced hit (the indirect ray's, or !PRE the camera ray's): Ray::operator() (MC/Ray.h:34-37) and
            // the face-forward against -dA
            tri = triA;
            if (BVH) {
                loc = add(o, smul((float)tA, dA));
                const float4 tn = S.tris[4 * (tri < 0 ? 0 : tri) + 3];
                flip = dot(V3{tn.x, tn.y, tn.z}, neg(dA)) < 0.0f;
            } else {
                loc = hloc;
                flip = hflip;
            }
        }
#if RT_SECTIONS
        dbg_vertex = vertex;
#endif
        if (vertex) {
            // ------------ vertex `depth`: Renderer::shading (MC/Renderer.cpp:163-209) up to its two rays
            CKParams& Q = kargs4();
            const float4 tq3 = S.tris[4 * tri + 3];
            const V3 N{tq3.x, tq3.y, tq3.z};
            const V3 n = flip ? neg(N) : N;
            const V3 p = add(loc, muls(n, INTERSECTION_CORRECTION));
            uint32_t skipc = 0;
            auto shade = [&](auto& G) {
                hasB = false;
                if (Q.has_light) {
                    V3 q, nl0;
                    int lt = 0;
                    sample_light(S, Q.light_area, G, q, nl0, nullptr, &lt);
                    const V3 p2q = sub(q, p);
                    const V3 wl = glm_normalize_wave(p2q);
                    const V3 nl = (dot(nl0, neg(wl)) < 0.0f) ? neg(nl0) : nl0;
                    const float sc1 = dot(wl, n), sc2 = dot(neg(wl), nl), sd2 = dot(p2q, p2q);
                    slen = sqrt_wave(dot(p2q, p2q));   // glm_length (the square root the normalize took)
                    // the unoccluded direct term; the shadow verdict selects it (BRDF: MC/WhittedMaterial.h:58-69)
                    const float4 mb = S.mats[2 * mat];
                    const V3 f = (sc1 >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};
                    const V3 X = muls(muls(mul(V3{Q.light_emission[0], Q.light_emission[1], Q.light_emission[2]}, f), sc1), sc2);
                    V3 ldu;
                    // (X / dist^2) / light PDF: both on Markstein's exact path when every lane's numerator lies in
                    // [2^-77, 2^77) (or is zero) and its dist^2 in [2^-20, 2^20) (the quotient then stays inside
                    // [2^-97, 2^97)), one wave-uniform test (rt_device.h div2_fast_range), as the fold's
                    if (!IEEE_DIV && RT_FOLD_DIV2 && Q.lpdf_fast && __all(div2_fast_range<0x19000000u, 0x66000000u>(X) && sd2 >= 0x1p-20f && sd2 < 0x1p20f))
                        ldu = div2_core(X, sd2, rcp_f32_mid(sd2), Q.lpdf, Q.y_lpdf);
                    else
                        ldu = vdiv(vdiv(X, sd2, IEEE_DIV ? 0.0f : rcp_f32(sd2)), Q.lpdf, Q.y_lpdf);   // Q.lpdf = 1.0f / light_area
                    st3(VS_LD, ldu);
                    dB = wl;
                    // a zero unoccluded term (the light behind the surface: f = 0) makes the verdict pick
                    // between +0 and +-0, which no accumulation can tell apart (sums start at +0): no
                    // shadow ray then (the direct term is taken as +0, as for an occluded light)
                    hasB = !(ldu.x == 0.0f && ldu.y == 0.0f && ldu.z == 0.0f);
                    // triangles (near-)coplanar with the sampled light triangle are hit, if at all, within
                    // 0.006 + 2e-5 * extent of q along a shadow ray meeting the light at |cos| >= 0.25,
                    // so `slen < t + 0.01f` holds for them: they cannot block (host: rt_scene.cpp)
                    // (the BVH variant's split phase: the same masks over its outside slots, rt_scene.cpp)
                    // (the sampled light triangle is kept as the skip code in VS_MAT: the trace reads its mask back)
                    if ((NARROW && !BVH) || BVH) skipc = (sc2 >= 0.25f && lt < 31) ? (uint32_t)lt + 1u : 0u;
                }
                // Russian roulette + indirect direction (the depth cap only bounds the loop: P = rr^4096)
                cont = G.next() < Q.rr && depth < 4096u;
                if (cont) {
                    const V3 wi = glm_normalize_big(sample_hemisphere(n, G));   // (a unit vector up to rounding, or NaN)
                    lsf(VS_PCOS) = dot(wi, n);
                    dA = wi;
                }
            };
            if (Q.has_light) {
                FixedDraws fd;
                g.vertex_draws(fd);
                shade(fd);
            } else {
                shade(g);
            }
            hasA = cont;
            o = p;
            pend = true;
            lsu(VS_MAT) = (uint32_t)mat | (skipc << VS_SKIP_SHIFT) | ((depth + 1u) << VS_DEPTH_SHIFT);
            if (BVH) {
                tiA = hasA ? 0u : NN; tiB = hasB ? 0u : NN;
                tA = TA_NONE; triA = -1; occB = false;
            }
        }

        // ======================= !PRE, a new sample: camera ray (MC/Camera.cpp:119-125 + MC/Renderer.cpp:128)
        if (!PRE && have_pixel && !in_path) {
            CKParams& Q = kargs4();
            const uint32_t pix = lsu(VS_PIX), y = pix / Q.W, x = pix - y * Q.W;
            float ux, uy;
            g.camera_draws(pix, lsu(VS_FRAME), !Q.has_light, ux, uy);
#if RT_SECTIONS
            dbg_cam = true;
#endif
            float cx = sdiv((float)x + ux, (float)Q.W, Q.y_w);
            float cy = sdiv((float)y + uy, (float)Q.H, Q.y_h);
            cx = cx * 2.0f - 1.0f;
            cy = cy * 2.0f - 1.0f;
            float tg[4];
            mat4_mul(Q.iproj, cx, cy, 1.0f, 1.0f, tg);
            const V3 dv = glm_normalize_wave(vdiv(V3{tg[0], tg[1], tg[2]}, tg[3], IEEE_DIV ? 0.0f : rcp_f32(tg[3])));
            float wd[4];
            mat4_mul(Q.iview, dv.x, dv.y, dv.z, 0.0f, wd);
            o = V3{Q.cam_pos[0], Q.cam_pos[1], Q.cam_pos[2]};
            dA = w_normalize_wave(V3{wd[0], wd[1], wd[2]});
            hasA = true; hasB = false;
            depth = 0;
            pend = false;
            in_path = true;
            if (BVH) {
                tiA = 0u; tiB = NN;
                tA = TA_NONE; triA = -1; occB = false;
            }
            if (!EXACT) { st3(VS_THR, V3{1.0f, 1.0f, 1.0f}); st3(VS_LSUM, V3{0, 0, 0}); }
        }

        if (!__any(in_path || alive || have_pixel)) {
            if (EXACT) drain_all(dleft);
            break;
        }

        SEC_MARK(5);
#if RT_SECTIONS
        SEC_COUNT(0, 1u);
        SEC_COUNT(1, (uint32_t)__popcll(__ballot(in_path)));
        SEC_COUNT(2, (uint32_t)__popcll(__ballot(dbg_vertex)));
        SEC_COUNT(3, (uint32_t)__popcll(__ballot(dbg_fin)));
        SEC_COUNT(4, (uint32_t)__popcll(__ballot(dbg_cam)));
        SEC_COUNT(11, (uint32_t)__popcll(__ballot(dleft != 0u)));
        dbg_vertex = dbg_fin = dbg_cam = false;
#endif
        // ======================= trace both rays of every lane =======================
        if (!BVH) {
        const bool trA = in_path && hasA, trB = in_path && hasB;
        tA = TA_NONE; triA = -1; occB = false;
        // the reciprocal directions are computed here, not when the rays are set up: they are then
        // temporaries of the box loop instead of 6 registers live across the iteration
        rA = rcp3(dA); rB = rcp3(dB);
        const bool fin = (!trA || finite3(rA)) && (!trB || finite3(rB)) && kargs4().force_walk == 0u;
        // candidate triangles (leaf-box masks): NARROW (<= 32 triangles) keeps ray A's in the low and
        // ray B's in the high half of one mask, so the Moller-Trumbore loop walks one mask in DFS order
        // (A first) without selecting between two
        uint64_t ca = 0, cb = 0;
        uint32_t ma = 0, mb = 0;
        {
            // a box is one 32-byte scalar load (s_load_dwordx8; a group of BOX_UNROLL boxes waits once)
            cbox8* bx = (cbox8*)kargs4().lboxes;
            const uint32_t nb = kargs4().n_lboxes;
            const float bndB = slen * 1.00001f + 1e-5f;   // ray B: no blocker in a box entered beyond the light point
            auto one_box = [&](const box8 q) {   // (lo.x, hi.x, lo.y, hi.y)(lo.z, hi.z, mask 0-31, mask 32-63), rt_layout.h
                // (lo - o, hi - o) per axis in the halves of packed registers, shared by the two rays
                const f2 sx = f2{q.s0, q.s1} - f2{o.x, o.x};
                const f2 sy = f2{q.s2, q.s3} - f2{o.y, o.y};
                const f2 sz = f2{q.s4, q.s5} - f2{o.z, o.z};
                const bool hA = box_hit_pk(sx, sy, sz, rA), hB = box_hit_pk_within(sx, sy, sz, rB, bndB);
                const uint32_t m0 = (uint32_t)f2i(q.s6);
                if (NARROW) {
                    ma |= hA ? m0 : 0u;
                    mb |= hB ? m0 : 0u;
                } else {
                    const uint64_t m = (uint64_t)m0 | ((uint64_t)(uint32_t)f2i(q.s7) << 32);
                    ca |= hA ? m : 0ull;
                    cb |= hB ? m : 0ull;
                }
            };
            uint32_t b = 0;
            for (; b + BOX_UNROLL <= nb; b += BOX_UNROLL) {
                box8 q[BOX_UNROLL];
#pragma unroll
                for (int u = 0; u < BOX_UNROLL; ++u) q[u] = bx[b + u];
#pragma unroll
                for (int u = 0; u < BOX_UNROLL; ++u) one_box(q[u]);
            }
            for (; b < nb; ++b) one_box(bx[b]);
        }
        if (NARROW) {
            // shadow-ray candidates that cannot block: the sampled light triangle's mask when the ray meets it at
            // |cos| >= 0.25 (the skip code the vertex left in VS_MAT, rt_scene.cpp)
            const uint32_t code = (lsu(VS_MAT) >> VS_SKIP_SHIFT) & 31u;
            const uint32_t bskip = code != 0u ? __float_as_uint(S.ltris[4 * (code - 1u)].w) : 0u;
            ca = ma; cb = mb & ~bskip;
        }
        if (!trA || !fin) ca = 0;
        if (!trB || !fin) cb = 0;
        if (!fin && (trA || trB)) {
            // a non-finite reciprocal direction: this lane walks the BVH (the reference's traversal)
            uint32_t nt = 0, tt = 0;
            if (trA) {
                const Ray r{o, dA, rA, dA.x < 0.0f, dA.y < 0.0f, dA.z < 0.0f};
                bool dummy = false;
                tA = 1.7976931348623157e308;
                traverse_impl<false, false, RT_COH_SPH>(S, r, false, 0.0, tA, triA, dummy, nt, tt);
            }
            if (trB) {
                const Ray r{o, dB, rB, dB.x < 0.0f, dB.y < 0.0f, dB.z < 0.0f};
                double db = 1.7976931348623157e308;
                int dt = -1;
                traverse_impl<false, false, RT_COH_SPH>(S, r, true, (double)slen, db, dt, occB, nt, tt);
            }
        }
        SEC_MARK(6);
#if RT_SECTIONS
        {   // (lane, candidate) pairs of this trace step: total, ray A's, and 64-lane chunks if compacted
            const uint32_t npair = (uint32_t)(__popcll(ca) + __popcll(cb));
            sec_w[15] = 0u;
            SEC_SUM(15, npair);
            SEC_SUM(7, npair);
            SEC_SUM(13, (uint32_t)__popcll(ca));
            const uint32_t tot = sec_w[15];
            SEC_COUNT(8, (tot + 63u) >> 6);
#if RT_SECTIONS >= 2
            // candidate overlap of the lane's two rays (its own build: timed with the MT section):
            // sum over lanes of |A & B|, and the wave's loop length per lane-candidate order --
            // max |A| + |B| (one test per ray and candidate) vs max |A | B| (one pass per triangle)
            uint32_t both = (uint32_t)__popcll(ca & cb), sep = (uint32_t)(__popcll(ca) + __popcll(cb)), uni = (uint32_t)__popcll(ca | cb);
            SEC_SUM(16, both);
            for (int off = 32; off >= 1; off >>= 1) {
                sep = max(sep, (uint32_t)__shfl_xor((int)sep, off));
                uni = max(uni, (uint32_t)__shfl_xor((int)uni, off));
            }
            SEC_COUNT(17, sep);
            SEC_COUNT(18, uni);
#endif
#if RT_SECTIONS >= 3
            {   // candidate histograms (global atomics; diagnostic builds only): [64 + n] lanes with n ray-A
                // candidates, [128 + n] with n ray-B candidates, [192 + n] trace steps whose busiest lane
                // has n, [256 + tri] / [288 + tri] ray A / ray B candidates by triangle
                unsigned long long* hc = (unsigned long long*)kargs4().counters;
                const uint32_t na = (uint32_t)__popcll(ca), nbb = (uint32_t)__popcll(cb);
                if (trA && fin) atomicAdd(&hc[64 + na], 1ull);
                if (trB && fin) atomicAdd(&hc[128 + nbb], 1ull);
                uint32_t mx = na + nbb;
                for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
                if (sec_first()) atomicAdd(&hc[192 + (mx < 63u ? mx : 63u)], 1ull);
                for (uint64_t m = ca; m != 0; m &= m - 1) atomicAdd(&hc[256 + (__builtin_ctzll(m) & 31)], 1ull);
                for (uint64_t m = cb; m != 0; m &= m - 1) atomicAdd(&hc[288 + (__builtin_ctzll(m) & 31)], 1ull);
                // the wave's union of candidate triangles: [400] ray A, [401] ray B, [402] either, [403] trace steps
                uint32_t oa = (uint32_t)ca, ob = (uint32_t)cb;
                for (int off = 32; off >= 1; off >>= 1) { oa |= (uint32_t)__shfl_xor((int)oa, off); ob |= (uint32_t)__shfl_xor((int)ob, off); }
                if (sec_first()) {
                    atomicAdd(&hc[400], (unsigned long long)__popc(oa)); atomicAdd(&hc[401], (unsigned long long)__popc(ob));
                    atomicAdd(&hc[402], (unsigned long long)__popc(oa | ob)); atomicAdd(&hc[403], 1ull);
                }
            }
#endif
        }
#endif
        // Moller-Trumbore on the candidates in DFS order: ray A first (closest hit, the later leaf wins
        // ties), then ray B (stops at the first blocking hit)
        auto test = [&](const bool useA, const int tri, uint64_t& rest) {
            const V3 d = useA ? dA : dB;
            const float4* T = S.tris + 4 * tri;
            const float4 t0 = T[0], t1 = T[1], t2 = T[2];
            double t;
#if RT_MT_PK
            const bool mh = moller_trumbore_pk(t0, t1, t2, o, d, t);
#else
            const bool mh = moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o, d, t);
#endif
#if RT_SECTIONS
            SEC_COUNT(5, 1u);
            SEC_COUNT(6, (uint32_t)__popcll(__ballot(1)));
            SEC_COUNT(12, (uint32_t)__popcll(__ballot(useA)));
            SEC_COUNT(14, (uint32_t)__popcll(__ballot(mh)));
#endif
            if (mh) {
                if (useA) {
                    if (t <= tA) { tA = t; triA = tri; }
                } else if (!((double)slen < t + (double)0.01f)) {   // MC/Renderer.cpp:184
                    occB = true;
                    rest = 0;   // B's candidates come last: nothing else to test
                }
            }
        };
        if (NARROW) {
            // (a cap on the tests per lane and iteration, the rest carried to the next iteration, measured
            // C4 -1 % at caps 6-10 and -10 % at 4: the carried state costs spills, profiles/r03/ab/)
#if RT_MT_LOOP32
            // two 32-bit masks instead of one 64-bit one: ray A's candidates in DFS order, then ray B's (the same order
            // as the 64-bit loop), with 32-bit bit scans and clears
            uint32_t am = (uint32_t)ca, bm = (uint32_t)cb;
            while ((am | bm) != 0u) {
                const bool useA = am != 0u;
                const uint32_t m = useA ? am : bm;
                const uint32_t bit = (uint32_t)__builtin_ctz(m);
                const uint32_t mn = m & (m - 1u);
                if (useA) am = mn;
                else bm = mn;
                uint64_t rest = 1;
                test(useA, (int)bit, rest);
                if (rest == 0) bm = 0u;   // ray B blocked: nothing else to test
            }
            if (false)
#endif
            {
            uint64_t cm = ca | (cb << 32);
            while (cm != 0) {
#if RT_B_TOP_FIRST
                // ray A's candidates in DFS order (its tie rule), then ray B's from the LAST triangle down: a shadow
                // verdict is any blocking hit, the same in any order, and a lane stops at its first blocker
                const uint32_t bit = ((uint32_t)cm != 0u) ? (uint32_t)__builtin_ctzll(cm) : 63u - (uint32_t)__builtin_clzll(cm);
                cm &= ~(1ull << bit);
#else
                const uint32_t bit = (uint32_t)__builtin_ctzll(cm);
                cm &= cm - 1;
#endif
                test(bit < 32u, (int)(bit & 31u), cm);
            }
            }
        } else {
            while ((ca | cb) != 0) {
                const bool useA = ca != 0;
                const uint64_t cur = useA ? ca : cb;
                const int tri = __builtin_ctzll(cur);
                if (useA) ca = cur & (cur - 1);
                else cb = cur & (cur - 1);
                test(useA, tri, cb);
            }
        }
        // the hit's location (Ray::operator(), MC/Ray.h:34-37) and the face-forward of its normal against
        // -dA (MC/Renderer.cpp:163-166), formed here: the next iteration's vertex needs only these, so the
        // rays (o, dA, dB) and the double t are not live across the iteration boundary
        if (trA && triA >= 0) {
            hloc = add(o, smul((float)tA, dA));
            const float4 tn = S.tris[4 * triA + 3];
            hflip = dot(V3{tn.x, tn.y, tn.z}, neg(dA)) < 0.0f;
        }
#if RT_SECTIONS >= 3
        {   // [320 + tri] ray A's closest hits by triangle, [352] blocked ray-B lanes (fin lanes)
            unsigned long long* hc = (unsigned long long*)kargs4().counters;
            if (trA && fin && triA >= 0) atomicAdd(&hc[320 + (triA & 31)], 1ull);
            if (trB && fin && occB) atomicAdd(&hc[352], 1ull);
        }
#endif
        } else {
            // BVH rounds (the megakernel's, rt_kernels.hip): `steps` box tests per round on the lane's
            // current ray (A until it is done, then B), up to two leaves postponed in DFS order and
            // intersected at the end of the round.  Rounds continue while more than `thresh` lanes
            // trace or nobody waits for service.
            CKParams& Q = kargs4();
            const uint32_t thresh = Q.thresh, steps = Q.steps;
            SEC_MARK(2);   // BVH: the split phase (section 2)
            if (Q.split_root != 0u) {
                // Split trace (rt_scene.cpp): a fresh ray (ti == 0) first tests the <= 32 leaves outside the
                // walked subtree by their own boxes -- one wave-uniform loop of scalar box loads, the
                // leaf-box variant's trace -- and the subtree's root box; it walks the subtree only when that
                // box is hit (entered within the bound).  Every ancestor box contains these boxes and the
                // finite slab test is monotone, so a box's own test decides whether the reference reaches it.
                // The closest hit is taken by (min t, max triangle) -- triangles are numbered in DFS order --
                // since the outside leaves are tested before the subtree's.
                // both fresh rays at once (the leaf-box variant's NARROW trace): one box loop shares each
                // box's plane - origin between ray A and ray B, and one candidate loop walks ray A's slots
                // (low half) then ray B's (high half) -- a wave loops over its busiest lane's A + B
                // candidates instead of the busiest A plus the busiest B (<= 32 outside leaves, rt_scene.cpp)
                const bool fA = in_path && tiA == 0u, fB = in_path && tiB == 0u && !occB;
                if (__any(fA || fB)) {
                    const V3 rA = rcp3(dA), rB = rcp3(dB);
                    const bool okA = fA && finite3(rA) && Q.force_walk == 0u, okB = fB && finite3(rB) && Q.force_walk == 0u;
                    const float bndB = slen * 1.00001f + 1e-5f;   // ray B: no blocker beyond the light point
                    uint32_t ma = 0, mb = 0;
                    {
                        cbox8* bx = (cbox8*)kargs4().sboxes;
                        const uint32_t nb = kargs4().n_sboxes;
                        for (uint32_t b = 0; b < nb; ++b) {
                            const box8 q = bx[b];
                            const f2 sx = f2{q.s0, q.s1} - f2{o.x, o.x};
                            const f2 sy = f2{q.s2, q.s3} - f2{o.y, o.y};
                            const f2 sz = f2{q.s4, q.s5} - f2{o.z, o.z};
                            const uint32_t m = (uint32_t)f2i(q.s6);
                            ma |= box_hit_pk(sx, sy, sz, rA) ? m : 0u;
                            mb |= box_hit_pk_within(sx, sy, sz, rB, bndB) ? m : 0u;
                        }
                    }
                    // the subtree's root box (ray A without a bound: the walk's first step tests the root
                    // again under the closest outside hit; ray B within the light distance)
                    uint32_t nA = NN, nB = NN;
                    {
                        const uint32_t root = kargs4().split_root;
                        const float4 n0 = S.nodes[2 * root], n1 = S.nodes[2 * root + 1];
                        const f2 sx = f2{n0.x, n0.w} - f2{o.x, o.x};
                        const f2 sy = f2{n0.y, n1.x} - f2{o.y, o.y};
                        const f2 sz = f2{n0.z, n1.y} - f2{o.z, o.z};
                        if (box_hit_pk(sx, sy, sz, rA)) nA = root;
                        if (box_hit_pk_within(sx, sy, sz, rB, bndB)) nB = root;
                    }
                    if (!okA) ma = 0u;
                    // outside slots near-coplanar with the sampled light triangle (its skip code in VS_MAT)
                    const uint32_t code = (lsu(VS_MAT) >> VS_SKIP_SHIFT) & 31u;
                    const uint32_t bskip = code != 0u ? __float_as_uint(S.ltris[4 * (code - 1u)].w) : 0u;
                    mb = okB ? mb & ~bskip : 0u;
#if RT_SPLIT_LOOP32
                    // two 32-bit masks (ray A's slots, then ray B's), as the leaf-box variant's candidate loop
                    uint32_t am = ma, bm = mb;
                    while ((am | bm) != 0u) {
                        const bool useA = am != 0u;
                        const uint32_t m = useA ? am : bm;
                        const uint32_t bit = (uint32_t)__builtin_ctz(m);
                        const uint32_t mn = m & (m - 1u);
                        if (useA) am = mn;
                        else bm = mn;
#else
                    uint64_t cm = (uint64_t)ma | ((uint64_t)mb << 32);
                    while (cm != 0) {
                        const uint32_t bit = (uint32_t)__builtin_ctzll(cm);
                        cm &= cm - 1;
                        const bool useA = bit < 32u;
#endif
                        // the slot's triangle, staged in LDS after the small tables (a, e1, (e2, bits(triangle)))
                        const float4* T = lds_scene + (2u * kargs4().n_mats + kargs4().n_lnodes + 4u * kargs4().n_ltris) + 3u * (bit & 31u);
                        const float4 t0 = T[0], t1 = T[1], t2 = T[2];
                        const int tri = f2i(t2.w);
                        double t;
                        if (moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o, useA ? dA : dB, t)) {
                            if (useA) {
                                if (t < tA || (t == tA && (uint32_t)tri > (uint32_t)triA)) { tA = t; triA = tri; }
                            } else if (!((double)slen < t + (double)0.01f)) {   // MC/Renderer.cpp:184
                                occB = true;
                                nB = NN;
#if RT_SPLIT_LOOP32
                                bm = 0u;   // nothing else to test
#else
                                cm = 0;   // ray B's candidates come last
#endif
                            }
                        }
                    }
                    if (okA) tiA = nA;
                    if (okB) tiB = nB;
                }
            }
            SEC_MARK(5);   // BVH: the rounds (walk; the postponed leaves' tests in section 6)
            for (;;) {
                const bool tracing = in_path && (tiA < NN || tiB < NN);
                const uint64_t act = __ballot(tracing);
                if (act == 0) break;
                const uint64_t srv = __ballot((in_path && !tracing) || (alive && !in_path));
                if ((uint32_t)__popcll(act) <= thresh && srv != 0) break;
                const bool curA = tiA < NN;
                const V3 d = curA ? dA : dB;
                // the current ray's reciprocal direction, recomputed per round (not 6 registers live
                // across the iteration)
                const Ray r{o, d, rcp3(d), d.x < 0.0f, d.y < 0.0f, d.z < 0.0f};
                const bool fin = __all(!tracing || finite3(r.rcp));
                // the walk skips a box entered beyond every t that could still matter (exact, DESIGN.md
                // 5.3): ray A's closest hit so far -- a triangle inside the box hits at t >= its entry, so
                // it would lose to the current hit (a tie needs entry <= t; the bound keeps 1e-5 relative
                // margin over the slab's 2e-7 rounding) -- and ray B's light distance (a triangle beyond
                // it cannot block: MC/Renderer.cpp:184 needs t <= slen - 0.01).  The reference visits every
                // hit box (MC/BVH.h:82-101); only boxes whose triangles cannot change the result are skipped.
                const float bound = curA ? ((tA < 1e30) ? (float)tA * 1.00001f + 1e-5f : __builtin_inff()) : slen * 1.00001f + 1e-5f;
#if RT_SECTIONS
                SEC_COUNT(5, 1u);                           // BVH: rounds
                SEC_COUNT(6, (uint32_t)__popcll(act));     // BVH: lanes tracing per round
#endif
                if (tracing) {
                    uint32_t ti = curA ? tiA : tiB;
                    // a split scene's finite ray walks only the subtree [split_root, split_end) (its walk started at the
                    // root; the nodes after the subtree hold outside leaves the split phase already tested): the DFS and
                    // compact walks end at the subtree's end, as the near-first orderings do (their exit reads NN)
                    const uint32_t tend = (kargs4().split_root != 0u && kargs4().force_walk == 0u && finite3(r.rcp)) ? kargs4().split_end : NN;
                    int parked0 = -1, parked1 = -1;
#if RT_BVH_PAIR
                    // ray B walks in a second slot when the lane's ray A is still walking too (the baked walk only)
                    const bool pair = curA && tiB < NN && !occB && finite3(rcp3(dB));
                    uint32_t ti2 = pair ? tiB : NN;
                    int park2 = -1;
#endif
                    auto walk = [&](auto kind, auto baked) {
                        // a split scene's ray with a finite reciprocal direction walks the subtree from its root:
                        // in the near-first ordering of its direction's octant when the scene has them, whose
                        // boxes are stored as that octant's (near, far) planes (BAKED)
                        constexpr bool BAKED = decltype(baked)::value;
                        const float4* wn = BAKED ? Q.wcopies + ((uint32_t)r.nx | ((uint32_t)r.ny << 1) | ((uint32_t)r.nz << 2)) * Q.wcopy_stride : S.nodes;
                        auto test_node = [&](const float4 q0, const float4 q1) -> bool {   // true: go on to ti + 1
                            const bool hit = BAKED                    ? slab_nf_within(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, bound)
                                             : decltype(kind)::value ? slab_hit_finite_within(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, bound)
                                                                     : slab_hit(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
                            const int tri = f2i(q1.w);
                            ti = (hit && tri < 0) ? ti + 1 : (uint32_t)f2i(q1.z);
                            if (hit && tri >= 0) {
                                if (parked0 < 0) parked0 = tri;
                                else { parked1 = tri; return false; }
                            }
                            return true;
                        };
                        // (two nodes per dependent load -- node ti and its pre-order successor, visited next when ti is
                        // entered or a leaf -- measured C5 -8 % at 7 waves (18 VGPRs spill) and -5 % at 6:
                        // profiles/r05/ab/ab_c5_walk_pair.json)
#if RT_BVH_PAIR
                        if (BAKED && pair) {
                            // ray B in the second slot: both slots' node loads before either test; slot 2 parks one
                            // leaf and stops stepping for the round
                            const float4* wn2 = Q.wcopies + ((uint32_t)(dB.x < 0.0f) | ((uint32_t)(dB.y < 0.0f) << 1) | ((uint32_t)(dB.z < 0.0f) << 2)) * Q.wcopy_stride;
                            const V3 rc2 = rcp3(dB);
                            const float bound2 = slen * 1.00001f + 1e-5f;
                            bool go1 = true;
                            for (uint32_t s = 0; s < steps; ++s) {
                                const bool g1 = go1 && ti < tend, g2 = ti2 < tend && park2 < 0;
                                if (!(g1 || g2)) break;
                                const uint32_t k1 = 2u * (g1 ? ti : 0u), k2 = 2u * (g2 ? ti2 : 0u);
                                const float4 q0 = wn[k1], q1 = wn[k1 + 1], u0 = wn2[k2], u1 = wn2[k2 + 1];
                                if (g1 && !test_node(q0, q1)) go1 = false;
                                if (g2) {
                                    const Ray r2{o, dB, rc2, dB.x < 0.0f, dB.y < 0.0f, dB.z < 0.0f};
                                    const bool hit = slab_nf_within(r2, u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, bound2);
                                    const int tri = f2i(u1.w);
                                    ti2 = (hit && tri < 0) ? ti2 + 1 : (uint32_t)f2i(u1.z);
                                    if (hit && tri >= 0) park2 = tri;
                                }
                            }
                            return;
                        }
#endif
                        for (uint32_t s = 0; s < steps && ti < tend; ++s) {
                            const float4 q0 = wn[2 * ti];
                            const float4 q1 = wn[2 * ti + 1];
                            if (!test_node(q0, q1)) break;
                        }
                    };
                    // (in a wave with a non-finite reciprocal the finite lanes still walk their ordering: a walk's
                    // position spans rounds, and it indexes the ordering; the others walk the DFS array with the
                    // general slab)
                    // (round 6: the compact 16-bit BVH walk, RT_QBVH, is gone from this kernel -- slower in every
                    // measurement, and its code cost the variant 2 spilled VGPRs: C5 +2.1 % without it,
                    // profiles/r06/ab/ab_c5_no_qbvh.json)
                    if (fin && Q.wcopies != nullptr) walk(FiniteSlab{}, std::true_type{});
                    else if (fin) walk(FiniteSlab{}, std::false_type{});
                    else if (Q.wcopies != nullptr && finite3(r.rcp)) walk(FiniteSlab{}, std::true_type{});
                    else walk(GeneralSlab{}, std::false_type{});
                    SEC_MARK(6);   // BVH: the postponed leaves' tests in the MT section
#if RT_SECTIONS
                    SEC_SUM(12, (uint32_t)(parked0 >= 0) + (uint32_t)(parked1 >= 0));   // BVH: leaves tested
#endif
                    for (int slot = 0; slot < 2; ++slot) {
                        const int pk = slot == 0 ? parked0 : parked1;
                        if (pk < 0 || (!curA && occB)) continue;
                        const float4 t0 = S.tris[4 * pk], t1 = S.tris[4 * pk + 1], t2 = S.tris[4 * pk + 2];
                        const V3 va{t0.x, t0.y, t0.z}, e1{t1.x, t1.y, t1.z}, e2{t2.x, t2.y, t2.z};
                        double t;
                        if (moller_trumbore_od(va, e1, e2, o, d, t)) {
                            if (curA) {
                                // the later leaf wins ties (MC/BVH.h:97-100): triangles are numbered in DFS order,
                                // and the split trace's outside leaves are tested first
                                if (t < tA || (t == tA && (uint32_t)pk > (uint32_t)triA)) { tA = t; triA = pk; }
                            } else if (!((double)slen < t + (double)0.01f)) {   // MC/Renderer.cpp:184
                                occB = true;
                                ti = NN;
                            }
                        }
                    }
                    if (ti >= tend) ti = NN;
                    if (curA) tiA = ti;
                    else tiB = ti;
#if RT_BVH_PAIR
                    if (pair) {
                        // ray B's parked leaf: the shadow verdict (MC/Renderer.cpp:184)
                        if (park2 >= 0) {
                            const float4 t0 = S.tris[4 * park2], t1 = S.tris[4 * park2 + 1], t2 = S.tris[4 * park2 + 2];
                            double t;
                            if (moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o, dB, t) &&
                                !((double)slen < t + (double)0.01f)) {
                                occB = true;
                                ti2 = NN;
                            }
                        }
                        tiB = ti2 >= tend ? NN : ti2;
                    }
#endif
                    SEC_MARK(5);
                }
            }
        }
        SEC_MARK(7);
    }
#if RT_SECTIONS
    // wave cycles per section -> counters[16 + section] (one atomic per wave and section)
    if (__lane_id() == 0)
        for (int i = 0; i < 8; ++i) atomicAdd((unsigned long long*)&P.counters[16 + i], (unsigned long long)sec_cyc[i]);
    // the wave's event counts -> counters[24 + i]
    if (lane < RT_SEC_COUNTS) atomicAdd((unsigned long long*)&P.counters[24 + lane], (unsigned long long)sec_w[lane]);
    if (__lane_id() == 0) {
        // [440] ~first entry, [441] last entry, [442] ~first dry queue, [443] last dry queue, [444] last exit,
        // [445] sum over waves of exit - dry queue, [446] waves, [447] sum of dry queue - entry (100 MHz ticks)
        const uint64_t tl_exit = wall_clock64();
        const uint64_t em = tl_empty != 0 ? tl_empty : tl_exit;
        unsigned long long* tc = (unsigned long long*)P.counters;
        atomicMax(&tc[440], (unsigned long long)~tl_entry); atomicMax(&tc[441], (unsigned long long)tl_entry);
        atomicMax(&tc[442], (unsigned long long)~em); atomicMax(&tc[443], (unsigned long long)em);
        atomicMax(&tc[444], (unsigned long long)tl_exit);
        atomicAdd(&tc[445], (unsigned long long)(tl_exit - em)); atomicAdd(&tc[446], 1ull); atomicAdd(&tc[447], (unsigned long long)(em - tl_entry));
        // [466 + b] waves by their time from the dry queue to their exit, 0.1 ms bins (the last one open)
        atomicAdd(&tc[466 + min((uint32_t)((tl_exit - em) / 10000u), 21u)], 1ull);
    }
#endif
}

template __global__ void pt_coherent_kernel<true, false, true, true>(KParams);
template __global__ void pt_coherent_kernel<false, false, true, true>(KParams);
template __global__ void pt_coherent_kernel<true, false, false, true>(KParams);
template __global__ void pt_coherent_kernel<false, false, false, true>(KParams);
template __global__ void pt_coherent_kernel<true, true, false, false>(KParams);
template __global__ void pt_coherent_kernel<false, true, false, false>(KParams);
template __global__ void pt_coherent_kernel<true, true, false, true>(KParams);
template __global__ void pt_coherent_kernel<false, true, false, true>(KParams);

// ---------------------------------------------------------------------------------------------
// The vertex kernel's camera pre-pass.  One wave per segment (an 8x8 tile of local pixels x the segment's
// frames, rt_kernels.h), one lane per pixel, the frames in order.  Each sample's camera ray
// (Camera::RecomputeRayDirections, MC/Camera.cpp:114-132, and RayGen_Shader's normalize,
// MC/Renderer.cpp:128) is traced to its closest hit (cast_path, MC/Renderer.cpp:136-146).  A miss (night
// sky, :145) or a hit on the light (direct emission, :151-161) is the sample's radiance: it is parked at
// once.  A surface hit becomes a record -- the hit location (Ray::operator(), MC/Ray.h:34-37) and the
// face-forward of the triangle's normal against -dir (MC/Renderer.cpp:163-166) -- from which the vertex
// kernel starts the path at its first vertex.  The camera rays of a tile are coherent, so the candidate
// loop here runs nearly converged, and the vertex kernel spends no iteration on camera rays or on sky
// samples.
//
// The leaf boxes a tile's camera rays can hit: the wave's segment is an 8x8 tile whose rays leave the
// camera through pixel positions x in [x0, x0 + 8], y in [y0, y1 + 1] (jitter in [0, 1]).  A box that lies
// wholly outside the frustum through the camera spanned by that pixel rectangle widened by one pixel on
// every side is hit by none of them: the float ray (RayGen's jitter, NDC, inverse projection, normalize,
// inverse view) is within ~1e-6 rad of the exact direction and the float slab test within ~1e-7 of the
// exact entry, while the margin is a pixel (~3e-4 rad at C4), so the box's own slab test -- which alone
// decides whether the reference tests its triangles (leaf-box monotonicity, rt_scene.cpp) -- fails for
// every ray of the tile.  Lane b tests box b in double; anything not finite keeps every box.
__device__ __forceinline__ uint64_t tile_box_mask(const KParams& P, uint32_t lane, double px0, double px1, double py0, double py1)
{
    // the leaf-box table of a small scene, or a split scene's outside boxes (rt_scene.cpp sboxes) with the walked
    // subtree's root box as one more entry (bit n_sboxes)
    const bool split = P.split_root != 0u;
    const uint32_t nb = split ? P.n_sboxes + 1u : P.n_lboxes;
    // the rectangle's directions form a convex cone when the homogeneous w keeps one sign over it (a
    // perspective inverse: w does not depend on the pixel at all); otherwise nothing is culled
    int wsign = 0;
    auto dirv = [&](double px, double py, double out[3]) -> bool {
        const double cx = (px / (double)P.W) * 2.0 - 1.0, cy = (py / (double)P.H) * 2.0 - 1.0;
        double v[4];
        for (int i = 0; i < 4; ++i) v[i] = (double)P.iproj[i] * cx + (double)P.iproj[4 + i] * cy + (double)P.iproj[8 + i] + (double)P.iproj[12 + i];
        if (!(v[3] != 0.0)) return false;
        const int sg = v[3] > 0.0 ? 1 : -1;
        if (wsign != 0 && sg != wsign) return false;
        wsign = sg;
        const double a = v[0] / v[3], b = v[1] / v[3], c = v[2] / v[3];
        for (int i = 0; i < 3; ++i) out[i] = (double)P.iview[i] * a + (double)P.iview[4 + i] * b + (double)P.iview[8 + i] * c;
        return __builtin_isfinite(out[0]) && __builtin_isfinite(out[1]) && __builtin_isfinite(out[2]);
    };
    double c[4][3], m[3];
    bool ok = dirv(px0 - 1.0, py0 - 1.0, c[0]) && dirv(px1 + 1.0, py0 - 1.0, c[1]) && dirv(px1 + 1.0, py1 + 1.0, c[2]) &&
              dirv(px0 - 1.0, py1 + 1.0, c[3]) && dirv(0.5 * (px0 + px1), 0.5 * (py0 + py1), m);
    bool keep = true;
    if (ok && lane < nb) {
        float q[6];
        if (split && lane == P.n_sboxes) {   // the subtree root's node: (lo.xyz, hi.x)(hi.y, hi.z, skip, tri)
            const float4 n0 = P.nodes[2 * P.split_root], n1 = P.nodes[2 * P.split_root + 1];
            q[0] = n0.x; q[1] = n0.w; q[2] = n0.y; q[3] = n1.x; q[4] = n0.z; q[5] = n1.y;
        } else {   // (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z, masks)
            const float* b = reinterpret_cast<const float*>(split ? P.sboxes : P.lboxes) + 8 * (size_t)lane;
            for (int k = 0; k < 6; ++k) q[k] = b[k];
        }
        const double lo[3] = {(double)q[0] - (double)P.cam_pos[0], (double)q[2] - (double)P.cam_pos[1], (double)q[4] - (double)P.cam_pos[2]};
        const double hi[3] = {(double)q[1] - (double)P.cam_pos[0], (double)q[3] - (double)P.cam_pos[1], (double)q[5] - (double)P.cam_pos[2]};
        for (int e = 0; e < 4 && keep; ++e) {
            const double* u = c[e];
            const double* w = c[(e + 1) & 3];
            double n[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
            if (n[0] * m[0] + n[1] * m[1] + n[2] * m[2] < 0.0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
            // the box corner furthest along n: outside when even it is behind the plane
            const double far = n[0] * (n[0] > 0.0 ? hi[0] : lo[0]) + n[1] * (n[1] > 0.0 ? hi[1] : lo[1]) + n[2] * (n[2] > 0.0 ? hi[2] : lo[2]);
            if (far < 0.0) keep = false;
        }
    }
    const uint64_t culled = __ballot(ok && lane < nb && !keep);
    return ~culled;
}

// one wave per tile: KParams::tile_boxes[tile] for the pre-pass
__global__ void __launch_bounds__(256) tile_boxes_kernel(KParams P)
{
    const uint32_t lane = __lane_id();
    const uint32_t tile = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (tile >= P.n_tiles) return;   // whole waves
    const uint32_t trow = tile / P.tiles_x, tcol = tile - trow * P.tiles_x;
    const uint32_t lr = trow * 8u + (lane >> 3), lx = tcol * 8u + (lane & 7u);
    const bool valid = lr < P.n_local_rows && lx < P.W;
    const uint32_t band_k = lr / P.band, in_band = lr - band_k * P.band;
    const uint32_t y = (P.rank + band_k * P.nranks) * P.band + in_band;
    // the tile's pixel rectangle: x in [x0, x0 + 8], y over its lanes' global rows (row bands)
    double ylo = valid ? (double)y : 1e30, yhi = valid ? (double)y : -1e30;
    for (int off = 32; off >= 1; off >>= 1) {
        ylo = fmin(ylo, __shfl_xor(ylo, off));
        yhi = fmax(yhi, __shfl_xor(yhi, off));
    }
    uint64_t m = ~0ull;
    if (ylo <= yhi) m = tile_box_mask(P, lane, (double)(tcol * 8u), (double)(tcol * 8u + 8u), ylo, yhi + 1.0);
    if (lane == 0) P.tile_boxes[tile] = m;
}

// The closest hit of a split scene's camera ray below the outside leaves' result (best, best_tri): the walk of
// the subtree [root, end) in DFS pre-order with skip pointers (the reference's traversal restricted to the
// subtree, whose root box lies inside every ancestor's, rt_scene.cpp), hit leaves postponed to one test per
// round, boxes entered beyond the best hit skipped (exact: a triangle inside a box hits at t >= its entry,
// the bound keeps 1e-5 relative margin), and the (min t, max DFS triangle) rule across both parts
// (BVH::traverse_BVH_from_node's later-leaf-wins, MC/BVH.h:97-100).
__device__ __forceinline__ void walk_subtree(const SceneView& S, const Ray& r, uint32_t root, uint32_t end, double& best, int& best_tri)
{
    uint32_t i = root;
    while (i < end) {
        const float bound = (best < 1e30) ? (float)best * 1.00001f + 1e-5f : __builtin_inff();
        int parked = -1;
        while (i < end) {
            const float4 q0 = S.nodes[2 * i];
            const float4 q1 = S.nodes[2 * i + 1];
            const bool hit = slab_hit_finite_within(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, bound);
            const int tri = f2i(q1.w);
            i = (hit && tri < 0) ? i + 1 : (uint32_t)f2i(q1.z);
            if (hit && tri >= 0) { parked = tri; break; }
        }
        if (parked >= 0) {
            const float4 t0 = S.tris[4 * parked], t1 = S.tris[4 * parked + 1], t2 = S.tris[4 * parked + 2];
            double t;
            if (moller_trumbore(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, r, t) &&
                (t < best || (t == best && parked > best_tri))) {
                best = t; best_tri = parked;
            }
        }
    }
}

// waves per SIMD the leaf-box pre-pass's registers are sized for (0: the compiler's choice, 7 at 67 VGPRs; 8 -- 64 VGPRs,
// 2 spilled, 42 SGPRs spilled -- pre-pass 15.25 -> 16.06 ms at C4, profiles/r06/ab/ab_c4_prepass_8waves.json)
#ifndef RT_COH_PRE_WAVES
#define RT_COH_PRE_WAVES 0
#endif
template <bool BVH>
__global__ void __launch_bounds__(256, (!BVH && RT_COH_PRE_WAVES) ? RT_COH_PRE_WAVES : 1) camera_prepass_kernel(KParams P)
{
    extern __shared__ __attribute__((aligned(16))) float4 lds_scene[];
    SceneView S;
    S.n_nodes = P.n_nodes; S.nodes = P.nodes; S.tris = P.tris; S.mats = P.mats; S.lnodes = P.lnodes; S.ltris = P.ltris; S.lboxes = nullptr;
    if (!BVH) {   // the small scene's triangles and materials in LDS (the leaf boxes come with scalar loads)
        const uint32_t tq = 4 * P.n_tris, mq = 2 * P.n_mats;
        float4* dt = lds_scene;
        float4* dm = dt + tq;
        for (uint32_t i = threadIdx.x; i < tq; i += blockDim.x) dt[i] = P.tris[i];
        for (uint32_t i = threadIdx.x; i < mq; i += blockDim.x) dm[i] = P.mats[i];
        __syncthreads();
        S.tris = dt; S.mats = dm;
    } else if (P.split_root != 0u) {
        // a split scene: its <= 32 outside triangles by slot, as the path kernel stages them (a, e1, (e2, bits(triangle)))
        for (uint32_t i = threadIdx.x; i < 3u * P.n_split_leaves; i += blockDim.x) {
            const uint32_t k = i / 3u, j = i - 3u * k;
            const int tri = P.stri[k];
            float4 v = P.tris[4 * tri + j];
            if (j == 2u) v.w = __int_as_float(tri);
            lds_scene[i] = v;
        }
        __syncthreads();
    }
    const uint32_t lane = __lane_id();
    const uint32_t sg = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (sg >= P.n_segments) return;   // whole waves
    const uint32_t c = sg / P.n_tiles, tile = sg - c * P.n_tiles;
    const uint32_t trow = tile / P.tiles_x, tcol = tile - trow * P.tiles_x;
    const uint32_t lr = trow * 8u + (lane >> 3), lx = tcol * 8u + (lane & 7u);
    const bool valid = lr < P.n_local_rows && lx < P.W;
    // local row -> global row (row bands dealt round-robin over ranks)
    const uint32_t band_k = lr / P.band, in_band = lr - band_k * P.band;
    const uint32_t y = (P.rank + band_k * P.nranks) * P.band + in_band;
    const uint32_t pix = y * P.W + lx, local = lr * P.W + lx;
    const uint32_t f0 = c * P.seg_frames;
    const uint32_t nf = min(P.seg_frames, P.n_frames - f0);
    const V3 o{P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]};
    float4* const out = P.crec + ((size_t)sg << P.seg_shift);
    // the leaf boxes (split scene: outside boxes + the subtree root) the tile's frustum meets (tile_boxes_kernel;
    // wave-uniform)
    const bool split = BVH && P.split_root != 0u;
    const uint64_t boxes = (BVH && !split) ? ~0ull : P.tile_boxes[tile];
    uint32_t cnt = 0;
    uint64_t skym = 0;   // the segment's camera-ray misses (P.sky_bits): bit j = frame f0 + j
    for (uint32_t j = 0; j < nf; ++j) {
        const uint32_t fidx = f0 + j, frame = P.first_frame + fidx;
        // the camera ray: the two camera draws (dims 0, 1 of the sample's stream), jitter, NDC,
        // inverse projection, normalize(xyz / w), inverse view, then Whitted::normalize
        uint32_t ow[4];
        philox4x32_10(pix, frame, 0u, 0u, (uint32_t)P.seed, (uint32_t)(P.seed >> 32), ow);
        const float ux = (float)ow[0] / 4294967296.0f, uy = (float)ow[1] / 4294967296.0f;
        // the divisions by Markstein's correction: (x + u) / W and (y + u) / H have numerators 0 or in [2^-32, 2^21)
        // (wh_fast: W and H below 2^20, a host flag), xyz / w when a wave-uniform test finds every operand in range
        float cx, cy;
        if (RT_FOLD_DIV2 && P.wh_fast) {
            cx = div1_core((float)lx + ux, (float)P.W, P.y_w);
            cy = div1_core((float)y + uy, (float)P.H, P.y_h);
        } else {
            cx = div_fast((float)lx + ux, (float)P.W, P.y_w);
            cy = div_fast((float)y + uy, (float)P.H, P.y_h);
        }
        cx = cx * 2.0f - 1.0f;
        cy = cy * 2.0f - 1.0f;
        float tg[4];
        mat4_mul(P.iproj, cx, cy, 1.0f, 1.0f, tg);
        const V3 txyz{tg[0], tg[1], tg[2]};
        V3 dq;
        const float aw = __builtin_fabsf(tg[3]);
        if (RT_FOLD_DIV2 && __all(div2_fast_range<kBits2m100, kBits2p100>(txyz) && aw >= 0x1p-20f && aw < 0x1p20f))
            dq = div1_core(txyz, tg[3], rcp_f32_mid(tg[3]));
        else
            dq = divs_fast(txyz, tg[3], rcp_f32(tg[3]));
        const V3 dv = glm_normalize_wave(dq);
        float wd[4];
        mat4_mul(P.iview, dv.x, dv.y, dv.z, 0.0f, wd);
        const V3 d = w_normalize_wave(V3{wd[0], wd[1], wd[2]});
        const Ray r = make_ray(o, d);
        // closest hit, the later leaf winning ties (MC/BVH.h:97-100)
        double t = 1.7976931348623157e308;
        int tri = -1;
        bool deferred = false;   // (split scenes) the ray is left to the path kernel
        bool fin = rcp_finite(r) && P.force_walk == 0u;
        if (!BVH) {
            // the distinct leaf boxes decide the candidates (rt_scene.cpp); Moller-Trumbore in DFS order
            uint64_t cm = 0;
            cbox8* bx = (cbox8*)P.lboxes;
            const uint64_t bset = P.n_lboxes >= 64u ? boxes : boxes & ((1ull << P.n_lboxes) - 1ull);
            for (uint64_t bm = bset; bm != 0; bm &= bm - 1) {
                const uint32_t b = (uint32_t)__builtin_ctzll(bm);
                const box8 q = bx[b];
                const f2 sx = f2{q.s0, q.s1} - f2{o.x, o.x};
                const f2 sy = f2{q.s2, q.s3} - f2{o.y, o.y};
                const f2 sz = f2{q.s4, q.s5} - f2{o.z, o.z};
                const uint64_t m = (uint64_t)(uint32_t)f2i(q.s6) | ((uint64_t)(uint32_t)f2i(q.s7) << 32);
                cm |= box_hit_pk(sx, sy, sz, r.rcp) ? m : 0ull;
            }
            if (!valid || !fin) cm = 0;
            while (cm != 0) {
                const int k = __builtin_ctzll(cm);
                cm &= cm - 1;
                const float4* T = S.tris + 4 * k;
                const float4 t0 = T[0], t1 = T[1], t2 = T[2];
                double tk;
                if (moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o, d, tk) && tk <= t) { t = tk; tri = k; }
            }
            fin = fin || !valid;
        } else if (split) {
            // the path kernel's split trace (rt_scene.cpp): the outside leaves by their own boxes, the subtree walked
            // when its root box is hit; a box's own test decides whether the reference reaches it (leaf-box
            // monotonicity), and the closest hit is taken by (min t, max DFS triangle)
            uint32_t cm = 0;
            const uint32_t ns = P.n_sboxes;
            cbox8* bx = (cbox8*)P.sboxes;
            const uint64_t bset = boxes & ((1ull << ns) - 1ull);
            for (uint64_t bm = bset; bm != 0; bm &= bm - 1) {
                const uint32_t b = (uint32_t)__builtin_ctzll(bm);
                const box8 q = bx[b];
                const f2 sx = f2{q.s0, q.s1} - f2{o.x, o.x};
                const f2 sy = f2{q.s2, q.s3} - f2{o.y, o.y};
                const f2 sz = f2{q.s4, q.s5} - f2{o.z, o.z};
                cm |= box_hit_pk(sx, sy, sz, r.rcp) ? (uint32_t)f2i(q.s6) : 0u;
            }
            bool walk = false;
            if ((boxes >> ns) & 1ull) {
                const float4 n0 = S.nodes[2 * P.split_root], n1 = S.nodes[2 * P.split_root + 1];
                const f2 sx = f2{n0.x, n0.w} - f2{o.x, o.x};
                const f2 sy = f2{n0.y, n1.x} - f2{o.y, o.y};
                const f2 sz = f2{n0.z, n1.y} - f2{o.z, o.z};
                walk = box_hit_pk(sx, sy, sz, r.rcp);
            }
            if (!valid || !fin) { cm = 0; walk = false; }
            if (walk && P.pre_defer_walk) { deferred = true; cm = 0; walk = false; }   // the path kernel traces it
            while (cm != 0) {
                const uint32_t k = (uint32_t)__builtin_ctz(cm);
                cm &= cm - 1;
                const float4* T = lds_scene + 3u * k;
                const float4 t0 = T[0], t1 = T[1], t2 = T[2];
                const int kt = f2i(t2.w);
                double tk;
                if (moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o, d, tk) &&
                    (tk < t || (tk == t && kt > tri))) { t = tk; tri = kt; }
            }
            if (walk) walk_subtree(S, r, P.split_root, P.split_end, t, tri);
            fin = fin || !valid;
        } else {
            fin = __all(!valid || fin);
        }
        if (valid && ((BVH && !split) || !fin)) {
            // the BVH variant's scene, or a ray with a non-finite reciprocal direction: the stackless walk
            // (the reference's traversal, rt_path.h)
            bool occ = false;
            uint32_t nt = 0, tt = 0;
            if (fin) traverse_impl<false, true, RT_COH_SPH>(S, r, false, 0.0, t, tri, occ, nt, tt);
            else traverse_impl<false, false, RT_COH_SPH>(S, r, false, 0.0, t, tri, occ, nt, tt);
        }
        bool surface = false;
        float4 rec = make_float4(0.f, 0.f, 0.f, 0.f);
        if (deferred) {
            // a camera ray entering the walked subtree's box: a record of its direction, traced by the path kernel
            surface = true;
            rec = make_float4(d.x, d.y, d.z, __uint_as_float(CREC_CAMERA | (lane << 19) | (j << 25)));
        } else if (valid) {
            V3 L = night_sky();   // cast_path miss: night sky (MC/Renderer.cpp:145)
            if (tri >= 0) {
                const int mat = f2i(S.tris[4 * tri].w);
                if (S.mats[2 * mat].w != 0.0f) {   // direct emission (MC/Renderer.cpp:151-161)
                    const float4 em = S.mats[2 * mat + 1];
                    L = V3{em.x, em.y, em.z};
                } else {
                    surface = true;
                    const V3 loc = add(o, smul((float)t, d));   // Ray::operator(), MC/Ray.h:34-37
                    const float4 tn = S.tris[4 * tri + 3];
                    const bool flip = dot(V3{tn.x, tn.y, tn.z}, neg(d)) < 0.0f;
                    rec = make_float4(loc.x, loc.y, loc.z, __uint_as_float((uint32_t)tri | (lane << 19) | (j << 25) | (flip ? 0x80000000u : 0u)));
                }
            }
            if (!surface) {
                if (P.sky_bits != nullptr && tri < 0) skym |= 1ull << j;   // the night sky: a bit, not a parked sample
                else park_sample(P, L, local, fidx);
            }
        }
        const uint64_t hits = __ballot(surface);
        if (surface) out[cnt + (uint32_t)__popcll(hits & ((1ull << lane) - 1ull))] = rec;
        cnt += (uint32_t)__popcll(hits);
    }
    if (P.sky_bits != nullptr && valid) {
        // the segment's whole 32-frame words (segments of >= 32 frames start on a word: rt_capi.cpp), word-major
        const size_t px = (size_t)P.n_local_rows * P.W;
        const uint32_t w0 = f0 >> 5;
        P.sky_bits[(size_t)w0 * px + local] = (uint32_t)skym;
        if (nf > 32u) P.sky_bits[(size_t)(w0 + 1u) * px + local] = (uint32_t)(skym >> 32);
    }
    if (lane == 0) {
        if (cnt != 0u) P.seg_list[atomicAdd(P.seg_list_n, 1u)] = make_uint2(sg, cnt);
#if RT_SECTIONS
        // (diagnostic) segments by record count, 256-record bins -> counters[448 + bin] (tools/prof_one.py)
        atomicAdd((unsigned long long*)&P.counters[448 + min(cnt >> 8, 16u)], 1ull);
#endif
    }
}

hipError_t rt_launch_camera_prepass(const KParams& P, bool bvh, size_t lds, hipStream_t stream)
{
    if (P.n_segments == 0) return hipSuccess;
    const uint32_t blocks = (P.n_segments + 3u) / 4u;
    if (bvh) {
        if (P.split_root != 0u) hipLaunchKernelGGL(tile_boxes_kernel, dim3((P.n_tiles + 3u) / 4u), dim3(256), 0, stream, P);
        hipLaunchKernelGGL(camera_prepass_kernel<true>, dim3(blocks), dim3(256), lds, stream, P);
    } else {
        hipLaunchKernelGGL(tile_boxes_kernel, dim3((P.n_tiles + 3u) / 4u), dim3(256), 0, stream, P);
        hipLaunchKernelGGL(camera_prepass_kernel<false>, dim3(blocks), dim3(256), lds, stream, P);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// device checks of the primitives the kernels shortcut (C-ABI rt_debug_primitives): the reference's
// fixtures (zero-area triangles, zero / axis-aligned directions, parallel rays, NaN slabs) through
//   * moller_trumbore_od with its float sign pre-test and |b2n| + |b3n| > |den| screen (rt_device.h)
//     -- Whitted::RayTriangleIntersection, MC/TriangleMesh.h:19-45 -- on (a, b, c, o, d): E1 = b - a,
//     E2 = c - a as the scene builder stores them;
//   * AABB_3D::intersects_with_ray (MC/BoundingVolume.h:173-215) in the three forms the kernels use:
//     slab_hit (std::max/min NaN rules), slab_hit_finite (IEEE max3/min3) and this file's box_hit_pk
//     (leaf boxes of the vertex kernel, packed products); the last two only for a finite reciprocal
//     direction, where the kernels use them (-1 otherwise).
__global__ void __launch_bounds__(256) debug_primitives_kernel(uint32_t n_mt, const float* __restrict__ mt, int32_t* __restrict__ mt_hit,
                                                               double* __restrict__ mt_t, uint32_t n_box, const float* __restrict__ box,
                                                               int32_t* __restrict__ box_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_mt) {
        const float* q = mt + 15 * (size_t)i;
        const V3 a{q[0], q[1], q[2]}, b{q[3], q[4], q[5]}, c{q[6], q[7], q[8]}, o{q[9], q[10], q[11]}, d{q[12], q[13], q[14]};
        double t = 0.0, tp = 0.0;
        const V3 e1 = sub(b, a), e2 = sub(c, a);
        const bool h = moller_trumbore_od(a, e1, e2, o, d, t);
        // the packed form (moller_trumbore_pk, the leaf-box variant's) must agree bit for bit: 2 flags a difference
        const bool hp = moller_trumbore_pk(make_float4(a.x, a.y, a.z, 0.0f), make_float4(e1.x, e1.y, e1.z, 0.0f),
                                           make_float4(e2.x, e2.y, e2.z, 0.0f), o, d, tp);
        const bool same = h == hp && (!h || __double_as_longlong(t) == __double_as_longlong(tp));
        mt_hit[i] = same ? (h ? 1 : 0) : 2;
        mt_t[i] = h ? t : 0.0;
    }
    if (i < n_box) {
        const float* q = box + 12 * (size_t)i;
        const Ray r = make_ray(V3{q[6], q[7], q[8]}, V3{q[9], q[10], q[11]});
        box_out[3 * i] = slab_hit(r, q[0], q[1], q[2], q[3], q[4], q[5]) ? 1 : 0;
        const bool fin = finite3(r.rcp);
        const f2 sx = f2{q[0], q[3]} - f2{r.o.x, r.o.x}, sy = f2{q[1], q[4]} - f2{r.o.y, r.o.y}, sz = f2{q[2], q[5]} - f2{r.o.z, r.o.z};
        box_out[3 * i + 1] = fin ? (slab_hit_finite(r, q[0], q[1], q[2], q[3], q[4], q[5]) ? 1 : 0) : -1;
        box_out[3 * i + 2] = fin ? (box_hit_pk(sx, sy, sz, r.rcp) ? 1 : 0) : -1;
    }
}

hipError_t rt_launch_debug_primitives(uint32_t n_mt, const float* mt, int32_t* mt_hit, double* mt_t, uint32_t n_box, const float* box,
                                      int32_t* box_hit, hipStream_t stream)
{
    const uint32_t n = n_mt > n_box ? n_mt : n_box;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(debug_primitives_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n_mt, mt, mt_hit, mt_t, n_box, box, box_hit);
    return hipGetLastError();
}

size_t rt_coherent_lane_state_lds_bytes(bool exact, bool lit, bool bvh)
{
    // (the BVH variant keeps no pending fold: its two words stay unallocated unless the unlit RNG block follows)
    const uint32_t exact_words = (bvh || RT_PEND_FOLD == 0) ? (uint32_t)VS_PEND : (uint32_t)VS_WORDS_EXACT;
    return (size_t)(lit ? (exact ? exact_words : VS_WORDS_FAST) : VS_WORDS_UNLIT) * 256 * sizeof(float);
}

hipError_t rt_launch_coherent(const KParams& P, bool exact, bool bvh, bool prepass, uint32_t grid, uint32_t block, size_t lds, hipStream_t stream)
{
    const bool narrow = !bvh && P.n_tris <= 32;
    if (bvh && prepass) {
        if (exact) hipLaunchKernelGGL((pt_coherent_kernel<true, true, false, true>), dim3(grid), dim3(block), lds, stream, P);
        else hipLaunchKernelGGL((pt_coherent_kernel<false, true, false, true>), dim3(grid), dim3(block), lds, stream, P);
    } else if (bvh) {
        if (exact) hipLaunchKernelGGL((pt_coherent_kernel<true, true, false, false>), dim3(grid), dim3(block), lds, stream, P);
        else hipLaunchKernelGGL((pt_coherent_kernel<false, true, false, false>), dim3(grid), dim3(block), lds, stream, P);
    } else if (narrow) {
        if (exact) hipLaunchKernelGGL((pt_coherent_kernel<true, false, true, true>), dim3(grid), dim3(block), lds, stream, P);
        else hipLaunchKernelGGL((pt_coherent_kernel<false, false, true, true>), dim3(grid), dim3(block), lds, stream, P);
    } else {
        if (exact) hipLaunchKernelGGL((pt_coherent_kernel<true, false, false, true>), dim3(grid), dim3(block), lds, stream, P);
        else hipLaunchKernelGGL((pt_coherent_kernel<false, false, false, true>), dim3(grid), dim3(block), lds, stream, P);
    }
    return hipGetLastError();
}

int rt_coherent_occupancy(bool exact, bool bvh, bool prepass, int block, size_t lds_bytes)
{
    int n = 0;
    hipError_t e;
    if (bvh && prepass) e = exact ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<true, true, false, true>, block, lds_bytes)
                                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<false, true, false, true>, block, lds_bytes);
    else if (bvh) e = exact ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<true, true, false, false>, block, lds_bytes)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<false, true, false, false>, block, lds_bytes);
    else e = exact ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<true, false, false, true>, block, lds_bytes)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<false, false, false, true>, block, lds_bytes);
    return e == hipSuccess ? n : 0;
}
