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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernels.h"
#include "rt_path.h"

using namespace rtd;

namespace {

// per-lane cold state in LDS, [field][lane] words
enum : uint32_t {
    VS_LOCAL = 0, VS_XY = 1, VS_C = 2,   // the work item: local pixel, (x, y) global, frame chunk
    VS_RNG = 3,                          // the Philox block of the current 4 draws (4 words)
    VS_LD = 7,                           // the pending vertex's unoccluded direct term (3 words)
    VS_PCOS = 10, VS_MAT = 11,           // the pending vertex's indirect cosine and material
    VS_PIX = 12, VS_FRAME = 13,          // the sample's stream counter (pixel, frame)
    VS_THR = 14, VS_LSUM = 17,           // FAST: throughput, radiance
    VS_WORDS_EXACT = 14, VS_WORDS_FAST = 20
};

// The lane's uniform draws (rt_path.h LaneRng) with only the draw index in a register: the counter
// (pixel, frame) and the current block of 4 Philox words live in the lane's LDS words.  Draws are
// consumed one by one from index 0, so a new block starts exactly when the index is a multiple of 4.
struct VertexRng {
    uint32_t* w;        // the lane's word 0 of the cold state (stride 256)
    uint32_t k0, k1;    // key (uniform)
    uint32_t dim;
    __device__ __forceinline__ void start(uint32_t px, uint32_t fr) { w[VS_PIX * 256u] = px; w[VS_FRAME * 256u] = fr; dim = 0; }
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
};

// the distinct leaf boxes, read with scalar loads (constant address space: wave-uniform index)
typedef const __attribute__((address_space(4))) float cfloat;

// AABB_3D::intersects_with_ray (MC/BoundingVolume.h:173-215) for a ray with a finite reciprocal
// direction: per axis the near plane distance is min((lo - o) * rcp, (hi - o) * rcp) -- the
// correctly rounded subtraction and multiplication are monotone, so the min is exactly the value of
// the plane the reference selects by the direction's sign -- and no term can be NaN (rt_device.h
// slab_hit_finite).  s0 = lo - o, s1 = hi - o.
__device__ __forceinline__ bool box_hit(const V3& s0, const V3& s1, const V3& rc)
{
    const float ax = s0.x * rc.x, bx = s1.x * rc.x;
    const float ay = s0.y * rc.y, by = s1.y * rc.y;
    const float az = s0.z * rc.z, bz = s1.z * rc.z;
    const float tin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(ax, bx), __builtin_fminf(ay, by)), __builtin_fminf(az, bz));
    const float tout = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(ax, bx), __builtin_fmaxf(ay, by)), __builtin_fmaxf(az, bz));
    return (tout >= 0.0f) && (tin <= tout);
}

__device__ __forceinline__ V3 rcp3(V3 d) { return V3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z}; }
__device__ __forceinline__ bool finite3(V3 v) { return __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z); }

}  // namespace

#ifndef RT_MIN_WAVES
#define RT_MIN_WAVES 1
#endif

template <bool EXACT>
__global__ void __launch_bounds__(256, RT_MIN_WAVES) pt_coherent_kernel(KParams P)
{
    extern __shared__ __attribute__((aligned(16))) float4 lds_scene[];
    SceneView S;
    S.n_nodes = P.n_nodes;
    {
        // stage the scene into LDS once per workgroup (nodes | tris | mats | lnodes | ltris | lboxes)
        const uint32_t nq = 2 * P.n_nodes, tq = 4 * P.n_tris, mq = 2 * P.n_mats, lq = P.n_lnodes, ltq = 4 * P.n_ltris;
        float4* dn = lds_scene;
        float4* dt = dn + nq;
        float4* dm = dt + tq;
        float4* dl = dm + mq;
        float4* dlt = dl + lq;
        for (uint32_t i = threadIdx.x; i < nq; i += blockDim.x) dn[i] = P.nodes[i];
        for (uint32_t i = threadIdx.x; i < tq; i += blockDim.x) dt[i] = P.tris[i];
        for (uint32_t i = threadIdx.x; i < mq; i += blockDim.x) dm[i] = P.mats[i];
        for (uint32_t i = threadIdx.x; i < lq; i += blockDim.x) dl[i] = P.lnodes[i];
        for (uint32_t i = threadIdx.x; i < ltq; i += blockDim.x) dlt[i] = P.ltris[i];
        __syncthreads();
        S.nodes = dn; S.tris = dt; S.mats = dm; S.lnodes = dl; S.ltris = dlt; S.lboxes = nullptr;
    }

    const uint32_t lane = __lane_id();
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t tib = threadIdx.x;
    // EXACT fold stack: levels [0, lds_levels) in LDS ([level][lane] float4 + u8 material), deeper in HBM
    float4* lstack = lds_scene + P.lds_scene_quads;
    uint8_t* lmat = reinterpret_cast<uint8_t*>(lstack + (size_t)P.lds_levels * 256);
    float* lstate = reinterpret_cast<float*>(lmat + (size_t)P.lds_levels * 256u);
    auto lsf = [&](uint32_t f) -> float& { return lstate[f * 256u + tib]; };
    auto lsu = [&](uint32_t f) -> uint32_t& { return reinterpret_cast<uint32_t*>(lstate)[f * 256u + tib]; };
    auto ls3 = [&](uint32_t f) { return V3{lsf(f), lsf(f + 1), lsf(f + 2)}; };
    auto st3 = [&](uint32_t f, V3 v) { lsf(f) = v.x; lsf(f + 1) = v.y; lsf(f + 2) = v.z; };
    const float PDF = 1.0f / (2.0f * PI_F);   // WhittedMaterial::PDF_at_the_sample, MC/WhittedMaterial.h:44-56

    bool alive = true, have_pixel = false, in_path = false;
    uint32_t k = 0;       // frame of the current item (item of chunk c: frames c * chunk_frames + [0, kend))
    uint32_t depth = 0;   // vertices shaded so far on this path
    bool pend = false;    // vertex depth-1 waits for its shadow verdict (and its indirect hit when cont)
    bool cont = false;    // vertex depth-1's roulette continued: ray A is its indirect ray
    VertexRng g;
    g.w = reinterpret_cast<uint32_t*>(lstate) + tib;
    g.k0 = (uint32_t)P.seed; g.k1 = (uint32_t)(P.seed >> 32);
    // the lane's rays: A = camera or indirect ray (closest hit), B = shadow ray (any hit); shared origin
    V3 o{0.f, 0.f, 0.f}, dA{0.f, 0.f, 1.f}, rA{0.f, 0.f, 1.f}, dB{0.f, 0.f, 1.f}, rB{0.f, 0.f, 1.f};
    bool hasA = false, hasB = false;
    float slen = 0.0f;                        // length(q - p) of the shadow ray
    double tA = 1.7976931348623157e308;       // closest t (DBL_MAX = IntersectionRecord default)
    int triA = -1;                            // closest triangle
    bool occB = false;                        // shadow ray blocked

    for (;;) {
        // ======================= service: every lane on a path has its rays back =======================
        if (in_path) {
            CKParams& Q = kargs4();
            bool finished = false;
            int fold_top = -1;   // EXACT: stack levels fold_top..0 are folded into L when the path ends
            V3 L{0.f, 0.f, 0.f};
            int mat = 0;
            bool emissive = false;
            if (hasA && triA >= 0) {
                mat = f2i(S.tris[4 * triA].w);
                emissive = S.mats[2 * mat].w != 0.0f;
            }
            bool vertex = false;
            if (pend) {
                // vertex depth-1's direct term (MC/Renderer.cpp:184-189): the shadow verdict
                V3 ld{0.f, 0.f, 0.f};
                if (hasB && !occB) ld = ls3(VS_LD);
                if (!EXACT) {
                    const V3 thr = ls3(VS_THR);
                    if (!cont) {
                        L = add(ls3(VS_LSUM), mul(thr, ld));
                        finished = true;
                    } else {
                        const V3 lsum = add(ls3(VS_LSUM), mul(thr, ld));
                        st3(VS_LSUM, lsum);
                        const float c = lsf(VS_PCOS);
                        const float4 mb = S.mats[2 * lsu(VS_MAT)];
                        const V3 f = (c >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};
                        st3(VS_THR, muls(mul(thr, f), c / PDF / Q.rr));
                        if (triA < 0 || emissive) { L = lsum; finished = true; }
                        else vertex = true;
                    }
                } else if (!cont || triA < 0 || emissive) {
                    // the roulette stopped, or the indirect ray missed / hit the light
                    // (radiance_indirect = 0, MC/Renderer.cpp:202): vertex depth-1 ends the path
                    L = ld;
                    fold_top = (int)depth - 2;
                    finished = true;
                } else {
                    // the indirect ray hit a surface: vertex depth-1 becomes stack level depth-1
                    const uint32_t lvl = depth - 1;
                    const float4 e = make_float4(ld.x, ld.y, ld.z, lsf(VS_PCOS));
                    const uint32_t pm = lsu(VS_MAT);
                    if (lvl < Q.lds_levels) {
                        lstack[lvl * 256u + tib] = e;
                        lmat[lvl * 256u + tib] = (uint8_t)pm;
                    } else if (lvl < Q.stack_depth) {
                        Q.stack_ld[(size_t)lvl * Q.total_threads + gtid] = e;
                        Q.stack_mat[(size_t)lvl * Q.total_threads + gtid] = pm;
                    } else {
                        atomicAdd((unsigned long long*)&Q.counters[3], 1ull);   // reported as stack overflow
                    }
                    vertex = true;
                }
            } else if (triA < 0) {   // cast_path miss: night sky (MC/Renderer.cpp:145)
                L = V3{12 / 255.0f, 20 / 255.0f, 69 / 255.0f};
                finished = true;
            } else if (emissive) {   // direct emission (MC/Renderer.cpp:151-161)
                const float4 em = S.mats[2 * mat + 1];
                L = V3{em.x, em.y, em.z};
                finished = true;
            } else {
                vertex = true;
            }

            if (vertex) {
                // ------------ vertex `depth`: Renderer::shading (MC/Renderer.cpp:163-209) up to its two rays
                const float4 tq3 = S.tris[4 * triA + 3];
                const V3 wo = neg(dA);
                const V3 loc = add(o, smul((float)tA, dA));   // Ray::operator(), MC/Ray.h:34-37
                const V3 N{tq3.x, tq3.y, tq3.z};
                const V3 n = (dot(N, wo) < 0.0f) ? neg(N) : N;
                const V3 p = add(loc, muls(n, INTERSECTION_CORRECTION));
                hasB = false;
                if (Q.has_light) {
                    V3 q, nl0;
                    sample_light(S, Q.light_area, g, q, nl0);
                    const V3 p2q = sub(q, p);
                    const V3 wl = glm_normalize(p2q);
                    const V3 nl = (dot(nl0, neg(wl)) < 0.0f) ? neg(nl0) : nl0;
                    const float sc1 = dot(wl, n), sc2 = dot(neg(wl), nl), sd2 = dot(p2q, p2q);
                    slen = glm_length(p2q);
                    // the unoccluded direct term; the shadow verdict selects it (BRDF: MC/WhittedMaterial.h:58-69)
                    const float4 mb = S.mats[2 * mat];
                    const V3 f = (sc1 >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};
                    st3(VS_LD, divs(divs(muls(muls(mul(V3{Q.light_emission[0], Q.light_emission[1], Q.light_emission[2]}, f), sc1), sc2), sd2),
                                    (1.0f / Q.light_area)));
                    dB = wl; rB = rcp3(wl);
                    hasB = true;
                }
                // Russian roulette + indirect direction (the depth cap only bounds the loop: P = rr^4096)
                cont = g.next() < Q.rr && depth < 4096u;
                if (cont) {
                    const V3 wi = glm_normalize(sample_hemisphere(n, g));
                    lsf(VS_PCOS) = dot(wi, n);
                    lsu(VS_MAT) = (uint32_t)mat;
                    dA = wi; rA = rcp3(wi);
                }
                hasA = cont;
                o = p;
                pend = true;
                depth = depth + 1;
            }

            if (finished) {
                if (EXACT) {
                    // fold inner-first: L = Ld_k + ((((L * brdf_k) * cos_k) / PDF) / RR)   (MC/Renderer.cpp:208,213)
                    for (int lvl = fold_top; lvl >= 0; --lvl) {
                        float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
                        int m = 0;
                        if ((uint32_t)lvl < Q.lds_levels) {
                            e = lstack[(uint32_t)lvl * 256u + tib];
                            m = lmat[(uint32_t)lvl * 256u + tib];
                        } else if ((uint32_t)lvl < Q.stack_depth) {
                            e = Q.stack_ld[(size_t)lvl * Q.total_threads + gtid];
                            m = Q.stack_mat[(size_t)lvl * Q.total_threads + gtid];
                        }
                        const float4 mb2 = S.mats[2 * m];
                        const V3 f = (e.w >= 0.0f) ? V3{mb2.x, mb2.y, mb2.z} : V3{0.0f, 0.0f, 0.0f};
                        L = add(V3{e.x, e.y, e.z}, divs(divs(muls(mul(L, f), e.w), PDF), Q.rr));
                    }
                }
                in_path = false;
                hasA = hasB = false;
                const uint32_t local = lsu(VS_LOCAL), kbase = lsu(VS_C) * Q.chunk_frames;
                float4 acc;
                if (kbase == 0) {
                    // chunk 0: temporal accumulation + clamp + pack (MC/Renderer.cpp:128-133), in place
                    acc = Q.accum[local];
                    acc.x = acc.x + L.x; acc.y = acc.y + L.y; acc.z = acc.z + L.z; acc.w = acc.w + 1.0f;
                    Q.accum[local] = acc;
                } else {
                    // a later chunk: the sample waits in 4-frame blocks for finalize_chunks_kernel
                    const uint32_t fp = kbase + k - Q.chunk_frames;
                    const size_t at = (((size_t)(fp >> 2) * Q.lbuf_stride + local) * 4u + (fp & 3u)) * 3u;
                    Q.lbuf[at] = L.x;
                    Q.lbuf[at + 1] = L.y;
                    Q.lbuf[at + 2] = L.z;
                }
                ++k;
                if (k == min(Q.chunk_frames, Q.n_frames - kbase)) {
                    if (kbase == 0 && Q.n_chunks == 1) {
                        const float fr = (float)(Q.first_frame + k - 1u);
                        const float rx = smin(smax(acc.x / fr, 0.0f), 1.0f), gy = smin(smax(acc.y / fr, 0.0f), 1.0f);
                        const float bz = smin(smax(acc.z / fr, 0.0f), 1.0f), aw = smin(smax(acc.w / fr, 0.0f), 1.0f);
                        Q.rgba[local] = (to_u8(aw) << 24) | (to_u8(bz) << 16) | (to_u8(gy) << 8) | to_u8(rx);
                    }
                    have_pixel = false;
                }
            }
        }

        // ======================= lane-level work queue (wave-collective) =======================
        const bool need = alive && !have_pixel;
        const uint64_t mask = __ballot(need);
        if (mask != 0) {
            CKParams& Q = kargs4();
            uint32_t base = 0;
            const int leader = __ffsll((unsigned long long)mask) - 1;
            if ((int)lane == leader) base = atomicAdd(Q.work_counter, (uint32_t)__popcll(mask));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t w = base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
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
                        lsu(VS_XY) = lx | (y << 16);
                        lsu(VS_C) = c;
                        have_pixel = true;
                        k = 0;
                        if (c == 0 && Q.first_frame == 1u) Q.accum[local] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            }
        }

        // ======================= new sample: camera ray (MC/Camera.cpp:119-125 + MC/Renderer.cpp:128)
        if (have_pixel && !in_path) {
            CKParams& Q = kargs4();
            const uint32_t xy = lsu(VS_XY), x = xy & 0xFFFFu, y = xy >> 16;
            g.start(y * Q.W + x, Q.first_frame + lsu(VS_C) * Q.chunk_frames + k);
            const float ux = g.next();
            const float uy = g.next();
            float cx = ((float)x + ux) / (float)Q.W;
            float cy = ((float)y + uy) / (float)Q.H;
            cx = cx * 2.0f - 1.0f;
            cy = cy * 2.0f - 1.0f;
            float tg[4];
            mat4_mul(Q.iproj, cx, cy, 1.0f, 1.0f, tg);
            const V3 dv = glm_normalize(divs(V3{tg[0], tg[1], tg[2]}, tg[3]));
            float wd[4];
            mat4_mul(Q.iview, dv.x, dv.y, dv.z, 0.0f, wd);
            o = V3{Q.cam_pos[0], Q.cam_pos[1], Q.cam_pos[2]};
            dA = w_normalize(V3{wd[0], wd[1], wd[2]});
            rA = rcp3(dA);
            hasA = true; hasB = false;
            depth = 0;
            pend = false;
            in_path = true;
            if (!EXACT) { st3(VS_THR, V3{1.0f, 1.0f, 1.0f}); st3(VS_LSUM, V3{0, 0, 0}); }
        }

        if (!__any(have_pixel || alive)) break;

        // ======================= trace both rays of every lane =======================
        const bool trA = in_path && hasA, trB = in_path && hasB;
        tA = 1.7976931348623157e308; triA = -1; occB = false;
        const bool fin = (!trA || finite3(rA)) && (!trB || finite3(rB)) && kargs4().force_walk == 0u;
        uint64_t ca = 0, cb = 0;
        {
            cfloat* bx = (cfloat*)kargs4().lboxes;
            const uint32_t nb = kargs4().n_lboxes;
            for (uint32_t b = 0; b < nb; ++b) {
                cfloat* q = bx + 8 * b;   // (lo.xyz, mask 0-31)(hi.xyz, mask 32-63), rt_layout.h
                const V3 s0{q[0] - o.x, q[1] - o.y, q[2] - o.z}, s1{q[4] - o.x, q[5] - o.y, q[6] - o.z};
                const uint64_t m = (uint64_t)(uint32_t)f2i(q[3]) | ((uint64_t)(uint32_t)f2i(q[7]) << 32);
                if (box_hit(s0, s1, rA)) ca |= m;
                if (box_hit(s0, s1, rB)) cb |= m;
            }
        }
        if (!trA || !fin) ca = 0;
        if (!trB || !fin) cb = 0;
        if (!fin && (trA || trB)) {
            // a non-finite reciprocal direction: this lane walks the BVH (the reference's traversal)
            uint32_t nt = 0, tt = 0;
            if (trA) {
                const Ray r{o, dA, rA, dA.x < 0.0f, dA.y < 0.0f, dA.z < 0.0f};
                bool dummy = false;
                traverse_impl<false, false>(S, r, false, 0.0, tA, triA, dummy, nt, tt);
            }
            if (trB) {
                const Ray r{o, dB, rB, dB.x < 0.0f, dB.y < 0.0f, dB.z < 0.0f};
                double db = 1.7976931348623157e308;
                int dt = -1;
                traverse_impl<false, false>(S, r, true, (double)slen, db, dt, occB, nt, tt);
            }
        }
        // Moller-Trumbore on the candidates in DFS order: ray A first (closest hit, the later leaf wins
        // ties), then ray B (stops at the first blocking hit)
        while ((ca | cb) != 0) {
            const bool useA = ca != 0;
            const uint64_t cur = useA ? ca : cb;
            const int tri = __builtin_ctzll(cur);
            if (useA) ca = cur & (cur - 1);
            else cb = cur & (cur - 1);
            const V3 d = useA ? dA : dB;
            const float4 t0 = S.tris[4 * tri], t1 = S.tris[4 * tri + 1], t2 = S.tris[4 * tri + 2];
            double t;
            if (moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o, d, t)) {
                if (useA) {
                    if (t <= tA) { tA = t; triA = tri; }
                } else if (!((double)slen < t + (double)0.01f)) {   // MC/Renderer.cpp:184
                    occB = true;
                    cb = 0;
                }
            }
        }
    }
}

template __global__ void pt_coherent_kernel<true>(KParams);
template __global__ void pt_coherent_kernel<false>(KParams);

size_t rt_coherent_lane_state_lds_bytes(bool exact) { return (size_t)(exact ? VS_WORDS_EXACT : VS_WORDS_FAST) * 256 * sizeof(float); }

hipError_t rt_launch_coherent(const KParams& P, bool exact, uint32_t grid, uint32_t block, size_t lds, hipStream_t stream)
{
    if (exact) hipLaunchKernelGGL(pt_coherent_kernel<true>, dim3(grid), dim3(block), lds, stream, P);
    else hipLaunchKernelGGL(pt_coherent_kernel<false>, dim3(grid), dim3(block), lds, stream, P);
    return hipGetLastError();
}

int rt_coherent_occupancy(bool exact, int block, size_t lds_bytes)
{
    int n = 0;
    const hipError_t e = exact ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<true>, block, lds_bytes)
                               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_coherent_kernel<false>, block, lds_bytes);
    return e == hipSuccess ? n : 0;
}
