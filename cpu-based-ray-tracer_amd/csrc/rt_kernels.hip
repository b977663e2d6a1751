// rt_kernels.hip -- the MI355X path-tracing megakernel (gfx950 / CDNA4, wave64).
//
// One persistent launch renders `n_frames` samples of every pixel assigned to this device:
//   * lane-level work queue: a lane that finishes its work item takes the next one from its wave's
//     pool (__ballot + popcount compaction), which refills 64 items per device atomic, so the wave
//     stays full until the queue drains; pixel order is 8x8-tile swizzled for ray coherence;
//   * per-pixel frames run in order inside the lane (accum += L per frame exactly like
//     Renderer::RayGen_Shader, MC/Renderer.cpp:124-134), so the float accumulation is the
//     reference's, bit for bit;
//   * path regeneration + one traversal per loop iteration: every lane advances by exactly one ray
//     (a camera/indirect closest-hit ray, or a shadow ray); shading is split at the shadow ray, so
//     all lanes of a wave run the same traversal loop each iteration whatever phase their path is in;
//   * the recursion of Renderer::shading (MC/Renderer.cpp:148-214) is made iterative: each bounce's
//     (direct radiance, cosine, material) is pushed to a per-lane stack and folded back in the
//     reference's inner-first order when the path ends (EXACT mode), or accumulated forward
//     (FAST mode: one rounding difference per bounce);
//   * BVH traversal is stackless: nodes are in DFS pre-order with skip links (rt_layout.h), so a
//     closest-hit walk tests exactly the boxes/triangles the reference's recursion tests
//     (BVH::traverse_BVH_from_node, MC/BVH.h:82-101, ties to the later leaf); shadow rays are
//     any-hit with early exit, which is exact because the reference's visibility predicate
//     `length(q-p) < t_closest + 0.01f` (MC/Renderer.cpp:184) is monotone in t;
//   * small scenes (the Cornell box: 4.4 KB) are staged into LDS once per workgroup and traversed
//     from LDS; large scenes are read through L1/L2/MALL from HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_glibc_math.h"
#include "rt_kernels.h"
#include "rt_path.h"

using namespace rtd;

namespace {

// per-lane cold state in LDS: word offsets of the fields, [field][lane] (pt_megakernel)
enum : uint32_t {
    LS_SN = 0,                  // shading normal across the shadow ray
    LS_SC1 = 3, LS_SC2 = 4, LS_SD2 = 5,
    LS_MATS = 6,                // shading material (bits 0-7), pending level's material (bits 8-15)
    LS_LOCAL = 7, LS_XY = 8, LS_C = 9,   // the work item: local pixel, (x, y) global, frame chunk
    LS_RNG = 10,                // the Philox block of the current 4 draws (4 words)
    LS_PEND = 14, LS_PCOS = 17, // EXACT: pending level (Ld, cos)
    LS_THR = 14, LS_LSUM = 17,  // FAST: throughput, radiance
    LS_WORDS_EXACT = 18, LS_WORDS_FAST = 20
};

}  // namespace

#ifndef WQ_BATCH
#define WQ_BATCH 64u     // work items per refill of a wave's pool (<= 64: at most one per lane)
#endif
#ifndef RT_MIN_WAVES
#define RT_MIN_WAVES 1   // minimum waves per SIMD the register allocation must admit (A/B knob)
#endif
// GB: the Denoiser project's frame (DN/Renderer.cpp:101-311): one sample per pixel through the
// pixel centre (no camera draws, DN/Camera.cpp:133), the camera hit's G-buffer (primitive id, world
// position, normalized face-forwarded normal) and the path color, clamped when immediate clamping is
// on, instead of the temporal accumulation.
template <bool EXACT, bool COUNT, bool LDS, bool GB = false>
__global__ void __launch_bounds__(256, RT_MIN_WAVES) pt_megakernel(KParams P)
{
    extern __shared__ __attribute__((aligned(16))) float4 lds_scene[];
    SceneView S;
    S.n_nodes = P.n_nodes;
    if (LDS) {
        // stage the whole scene into LDS once per workgroup (nodes | tris | mats | lnodes | ltris | lboxes)
        const uint32_t nq = 2 * P.n_nodes, tq = 4 * P.n_tris, mq = 2 * P.n_mats, lq = P.n_lnodes, ltq = 4 * P.n_ltris;
        const uint32_t bq = 2 * P.n_lboxes;
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
        float4* dbx = dlt + ltq;
        for (uint32_t i = threadIdx.x; i < bq; i += blockDim.x) dbx[i] = P.lboxes[i];
        __syncthreads();
        S.nodes = dn; S.tris = dt; S.mats = dm; S.lnodes = dl; S.ltris = dlt; S.lboxes = dbx;
    } else {
        S.nodes = P.nodes; S.tris = P.tris; S.mats = P.mats; S.lnodes = P.lnodes; S.ltris = P.ltris; S.lboxes = P.lboxes;
    }

    const uint32_t lane = __lane_id();
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    // EXACT fold stack: levels [0, lds_levels) in LDS ([level][lane] float4 + u8 material), deeper
    // levels in HBM ([level][thread])
    float4* lstack = lds_scene + P.lds_scene_quads;
    uint8_t* lmat = reinterpret_cast<uint8_t*>(lstack + (size_t)P.lds_levels * 256);
    const uint32_t tib = threadIdx.x;
    // the lane's cold state -- read and written only by the service code, never inside traversal --
    // lives in LDS ([field][lane] words after the fold stack), so the registers carry what the
    // traversal loops need and the kernel fits 5 waves per SIMD
    float* lstate = reinterpret_cast<float*>(lmat + (size_t)P.lds_levels * 256u);
    auto lsf = [&](uint32_t f) -> float& { return lstate[f * 256u + tib]; };
    auto lsu = [&](uint32_t f) -> uint32_t& { return reinterpret_cast<uint32_t*>(lstate)[f * 256u + tib]; };
    auto ls3 = [&](uint32_t f) { return V3{lsf(f), lsf(f + 1), lsf(f + 2)}; };
    auto st3 = [&](uint32_t f, V3 v) { lsf(f) = v.x; lsf(f + 1) = v.y; lsf(f + 2) = v.z; };
    const float PDF = 1.0f / (2.0f * PI_F);   // WhittedMaterial::PDF_at_the_sample, MC/WhittedMaterial.h:44-56

    uint32_t node_tests = 0, tri_tests = 0, rays = 0;
    // COUNT diagnostics: wave-level executions (counted by the first active lane)
    uint32_t w_rounds = 0, w_steps = 0, w_mt = 0, w_service = 0, w_fold = 0;
    bool alive = true, have_pixel = false, in_path = false;
    uint32_t k = 0;   // frame of the current item (item of chunk c: frames c * chunk_frames + [0, kend))
    LaneRng g;
    g.buf = reinterpret_cast<uint32_t*>(lstate) + LS_RNG * 256u + tib;
    g.k0 = (uint32_t)P.seed; g.k1 = (uint32_t)(P.seed >> 32);
    Ray ray;
    uint32_t depth = 0;
    bool shadow = false;            // the lane's current ray is a shadow ray
    double slen = 0.0;              // length(q - p) of the shadow ray
    // in LDS: the shading context carried across the shadow ray (face-forwarded normal LS_SN, material
    // in LS_MATS bits 0-7, the occlusion-independent factors LS_SC1/SC2/SD2 of the direct term); EXACT:
    // the level waiting to learn whether its indirect ray continues the path (LS_PEND, LS_PCOS, material
    // in LS_MATS bits 8-15); FAST: forward throughput LS_THR and radiance LS_LSUM
    // traversal state of the lane's current ray (persists across service rounds)
    const uint32_t NN = S.n_nodes;
    uint32_t ti = NN;                        // next node (NN: no ray / finished)
    double tbest = 1.7976931348623157e308;   // closest t so far (DBL_MAX = IntersectionRecord default)
    int ttri = -1;                           // closest triangle so far
    bool toccl = false;                      // shadow ray blocked
    bool tdone = true;

    uint64_t c_service = 0, c_queue = 0, c_trace = 0, s_lanes = 0;   // COUNT: wave-uniform cycle sums
    uint32_t pool_base = 0, pool_count = 0;   // the wave's batch of work items (wave-uniform)
    for (;;) {
        // ======================= service round: lanes whose ray has been traced =======================
        uint64_t tc0 = 0;
        if (COUNT) {
            tc0 = clock64();
            if (lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) ++w_service;
            s_lanes += (uint64_t)__popcll(__ballot(in_path && tdone));
        }
        if (in_path && tdone) {
            const KParams& Q = kargs();
            bool finished = false;
            int fold_top = -1;   // EXACT: stack levels fold_top..0 are folded into L when the path ends
            V3 L{0, 0, 0};
            bool part2 = false;  // run the post-shadow half of shading now
            bool new_ray = false;
            V3 ld{0.0f, 0.0f, 0.0f};
            if (!shadow) {
                int mat = 0;
                bool emissive = false;
                if (ttri >= 0) {
                    mat = f2i(S.tris[4 * ttri].w);
                    emissive = S.mats[2 * mat].w != 0.0f;
                }
                if (GB && depth == 0) {
                    // Renderer::cast_path's G-buffer writes, DN/Renderer.cpp:290-308
                    if (ttri >= 0) {
                        const float4 tq1 = S.tris[4 * ttri + 1], tq3 = S.tris[4 * ttri + 3];
                        const V3 loc = add(ray.o, smul((float)tbest, ray.d));
                        const V3 N{tq3.x, tq3.y, tq3.z};
                        const V3 nf = glm_normalize((dot(N, neg(ray.d)) < 0.0f) ? neg(N) : N);
                        const uint32_t local = lsu(LS_LOCAL);
                        Q.gb_prim[local] = f2i(tq1.w);
                        Q.gb_pos[local] = make_float4(loc.x, loc.y, loc.z, 0.0f);
                        Q.gb_nrm[local] = make_float4(nf.x, nf.y, nf.z, 0.0f);
                    } else {
                        Q.gb_prim[lsu(LS_LOCAL)] = -1;
                    }
                }
                if (depth == 0) {
                    if (ttri < 0) {   // cast_path miss: night sky (MC/Renderer.cpp:145)
                        L = night_sky();
                        finished = true;
                    } else if (emissive) {   // direct emission (MC/Renderer.cpp:151-161)
                        const float4 em = S.mats[2 * mat + 1];
                        L = V3{em.x, em.y, em.z};
                        finished = true;
                    }
                } else if (ttri < 0 || emissive) {
                    // the indirect ray missed or hit the light: radiance_indirect = 0 (MC/Renderer.cpp:202)
                    L = ls3(EXACT ? LS_PEND : LS_LSUM);
                    fold_top = (int)depth - 2;
                    finished = true;
                } else if (EXACT) {
                    // the pending level recurses into this hit: push it as stack level depth-1
                    const uint32_t lvl = depth - 1;
                    const float4 e = make_float4(lsf(LS_PEND), lsf(LS_PEND + 1), lsf(LS_PEND + 2), lsf(LS_PCOS));
                    const uint32_t pend_mat = lsu(LS_MATS) >> 8;
                    if (lvl < Q.lds_levels) {
                        lstack[lvl * 256u + tib] = e;
                        lmat[lvl * 256u + tib] = (uint8_t)pend_mat;
                    } else if (lvl < Q.stack_depth) {
                        Q.stack_ld[(size_t)lvl * Q.total_threads + gtid] = e;
                        Q.stack_mat[(size_t)lvl * Q.total_threads + gtid] = pend_mat;
                    } else {
                        // a level the stack cannot hold (sized from rr, rt_capi.cpp): counted, and rt_render
                        // reports the render as failed (RT_ERR_OVERFLOW) instead of returning a wrong sample
                        atomicAdd((unsigned long long*)&Q.counters[13], 1ull);
                    }
                }
                if (!finished) {
                    // ------------ shading, first half (MC/Renderer.cpp:163-186): shading point, light
                    // sample, shadow ray set-up
                    const V3 wo = neg(ray.d);
                    const V3 loc = add(ray.o, smul((float)tbest, ray.d));   // Ray::operator(), MC/Ray.h:34-37
                    const V3 N = leaf_normal(S, ttri, loc);
                    const V3 n = (dot(N, wo) < 0.0f) ? neg(N) : N;
                    const V3 p = add(loc, muls(n, INTERSECTION_CORRECTION));
                    st3(LS_SN, n);
                    lsu(LS_MATS) = (lsu(LS_MATS) & 0xFF00u) | (uint32_t)mat;
                    if (Q.has_light) {
                        V3 q, nl0;
                        sample_light(S, Q.light_area, g, q, nl0);
                        const V3 p2q = sub(q, p);
                        const V3 wl = glm_normalize(p2q);
                        const V3 nl = (dot(nl0, neg(wl)) < 0.0f) ? neg(nl0) : nl0;
                        lsf(LS_SC1) = dot(wl, n);
                        lsf(LS_SC2) = dot(neg(wl), nl);
                        lsf(LS_SD2) = dot(p2q, p2q);
                        slen = (double)glm_length(p2q);
                        ray = make_ray(p, wl);
                        shadow = true;
                        new_ray = true;
                    } else {
                        ray.o = p;   // no emitter: direct term 0, continue with roulette
                        part2 = true;
                    }
                }
            } else {
                // ------------ the shadow ray came back: direct term (MC/Renderer.cpp:187-189)
                if (!toccl) {
                    const float sc1 = lsf(LS_SC1);
                    const float4 mb = S.mats[2 * (lsu(LS_MATS) & 0xFFu)];
                    const V3 f = (sc1 >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};   // BRDF, MC/WhittedMaterial.h:58-69
                    ld = divs(divs(muls(muls(mul(V3{Q.light_emission[0], Q.light_emission[1], Q.light_emission[2]}, f), sc1), lsf(LS_SC2)), lsf(LS_SD2)), (1.0f / Q.light_area));
                }
                shadow = false;
                part2 = true;
            }

            if (part2) {
                // ------------ shading, second half: Russian roulette + indirect direction
                // (MC/Renderer.cpp:193-209; the depth cap only bounds the loop: P(depth > 4096) = rr^4096)
                if (g.next() < Q.rr && depth < 4096u) {
                    const V3 sn = ls3(LS_SN);
                    const uint32_t smat = lsu(LS_MATS) & 0xFFu;
                    const V3 wi = glm_normalize(sample_hemisphere(sn, g));
                    const float c = dot(wi, sn);
                    if (EXACT) {
                        st3(LS_PEND, ld); lsf(LS_PCOS) = c; lsu(LS_MATS) = smat | (smat << 8);
                    } else {
                        const V3 thr = ls3(LS_THR);
                        st3(LS_LSUM, add(ls3(LS_LSUM), mul(thr, ld)));
                        const float4 mb = S.mats[2 * smat];
                        const V3 f = (c >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};
                        st3(LS_THR, muls(mul(thr, f), c / PDF / Q.rr));
                    }
                    ray = make_ray(ray.o, wi);
                    depth = depth + 1;
                    new_ray = true;
                } else {
                    if (EXACT) L = ld;
                    else L = add(ls3(LS_LSUM), mul(ls3(LS_THR), ld));
                    fold_top = (int)depth - 1;
                    finished = true;
                }
            }

            if (finished) {
                if (EXACT) {
                    // fold inner-first: L = Ld_k + ((((L * brdf_k) * cos_k) / PDF) / RR)   (MC/Renderer.cpp:208,213)
                    for (int lvl = fold_top; lvl >= 0; --lvl) {
                        if (COUNT && lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) ++w_fold;
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
                if (GB) {
                    // RayGen_Shader, DN/Renderer.cpp:264-275: (clamped) color into the G-buffer
                    if (Q.gb_clamp) L = V3{smin(smax(L.x, 0.0f), 1.0f), smin(smax(L.y, 0.0f), 1.0f), smin(smax(L.z, 0.0f), 1.0f)};
                    Q.gb_color[lsu(LS_LOCAL)] = make_float4(L.x, L.y, L.z, 0.0f);
                    have_pixel = false;
                } else {
                const uint32_t local = lsu(LS_LOCAL), kbase = lsu(LS_C) * Q.chunk_frames;
                float4 acc;
                if (kbase == 0) {
                    // chunk 0: temporal accumulation + clamp + pack (MC/Renderer.cpp:128-133), the
                    // accumulator read-modified-written in place (L2-resident: the lane's own pixel)
                    acc = Q.accum[local];
                    acc.x = acc.x + L.x; acc.y = acc.y + L.y; acc.z = acc.z + L.z; acc.w = acc.w + 1.0f;
                    Q.accum[local] = acc;
                } else {
                    // a later chunk of the pixel's frames: the sample waits in the frame-major
                    // buffer for the in-order sum of rt_finalize_chunks
                    const uint32_t fp = kbase + k - Q.chunk_frames;
                    // 4-frame blocks: the 4 frames of a block of one pixel are 48 contiguous bytes, so a
                    // lane's consecutive samples merge into the same L2 lines (12 B scattered per plane
                    // became 32-B partial-line writes in HBM)
                    const size_t at = (((size_t)(fp >> 2) * Q.lbuf_stride + local) * 4u + (fp & 3u)) * 3u;
                    Q.lbuf[at] = L.x;
                    Q.lbuf[at + 1] = L.y;
                    Q.lbuf[at + 2] = L.z;
                }
                ++k;
                if (k == min(Q.chunk_frames, Q.n_frames - kbase)) {
                    if (kbase == 0) {
                        if (Q.n_chunks == 1) {
                            const float fr = (float)(Q.first_frame + k - 1u);
                            const float rx = smin(smax(acc.x / fr, 0.0f), 1.0f), gy = smin(smax(acc.y / fr, 0.0f), 1.0f);
                            const float bz = smin(smax(acc.z / fr, 0.0f), 1.0f), aw = smin(smax(acc.w / fr, 0.0f), 1.0f);
                            Q.rgba[local] = (to_u8(aw) << 24) | (to_u8(bz) << 16) | (to_u8(gy) << 8) | to_u8(rx);
                        }
                    }
                    have_pixel = false;
                }
                }
            }
            if (new_ray) {
                if (COUNT) ++rays;
                ti = 0; tbest = 1.7976931348623157e308; ttri = -1; toccl = false; tdone = false;
            }
        }

        uint64_t tc1 = 0;
        if (COUNT) { tc1 = clock64(); c_service += tc1 - tc0; }
        // ======================= lane-level work queue (wave-collective) =======================
        // items come from a wave-private pool refilled WQ_BATCH at a time from the device counter
        // (one returning atomic per refill saturates a single counter word: rt_coherent.hip)
        const bool need = alive && !have_pixel;
        const uint64_t mask = __ballot(need);
        if (mask != 0) {
            const KParams& Q = kargs();
            const uint32_t n = (uint32_t)__popcll(mask);
            uint32_t fresh = 0;
            if (n > pool_count) {
                uint32_t b = 0;
                if (lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) b = atomicAdd(Q.work_counter, WQ_BATCH);
                fresh = __builtin_amdgcn_readfirstlane(b);
            }
            const uint32_t pb = pool_base, pc = pool_count;
            if (n > pc) { pool_base = fresh + (n - pc); pool_count = WQ_BATCH - (n - pc); }
            else { pool_base = pb + n; pool_count = pc - n; }
            if (need) {
                const uint32_t j = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
                const uint32_t w = j < pc ? pb + j : fresh + (j - pc);
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
                        lsu(LS_LOCAL) = local;
                        lsu(LS_XY) = lx | (y << 16);
                        lsu(LS_C) = c;
                        have_pixel = true;
                        k = 0;
                        if (!GB && c == 0 && Q.first_frame == 1u) Q.accum[local] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            }
        }

        // ======================= new sample: camera ray (MC/Camera.cpp:119-125 + MC/Renderer.cpp:128)
        if (have_pixel && !in_path) {
            const KParams& Q = kargs();
            const uint32_t xy = lsu(LS_XY), x = xy & 0xFFFFu, y = xy >> 16;
            g.start(y * Q.W + x, Q.first_frame + lsu(LS_C) * Q.chunk_frames + k);
            float cx, cy;
            if (GB) {   // centre of the pixel, DN/Camera.cpp:133
                cx = ((float)x + 0.5f) / (float)Q.W;
                cy = ((float)y + 0.5f) / (float)Q.H;
            } else {
                const float ux = g.next();
                const float uy = g.next();
                cx = ((float)x + ux) / (float)Q.W;
                cy = ((float)y + uy) / (float)Q.H;
            }
            cx = cx * 2.0f - 1.0f;
            cy = cy * 2.0f - 1.0f;
            float tg[4];
            mat4_mul(Q.iproj, cx, cy, 1.0f, 1.0f, tg);
            const V3 dv = glm_normalize(divs(V3{tg[0], tg[1], tg[2]}, tg[3]));
            float wd[4];
            mat4_mul(Q.iview, dv.x, dv.y, dv.z, 0.0f, wd);
            ray = make_ray(V3{Q.cam_pos[0], Q.cam_pos[1], Q.cam_pos[2]}, w_normalize(V3{wd[0], wd[1], wd[2]}));
            depth = 0;
            shadow = false;
            in_path = true;
            if (!EXACT) { st3(LS_THR, V3{1.0f, 1.0f, 1.0f}); st3(LS_LSUM, V3{0, 0, 0}); }
            if (COUNT) ++rays;
            ti = 0; tbest = 1.7976931348623157e308; ttri = -1; toccl = false; tdone = false;
        }

        uint64_t tc2 = 0;
        if (COUNT) { tc2 = clock64(); c_queue += tc2 - tc1; }
        if (!__any(have_pixel || alive)) break;

        // ======================= small scenes: coherent trace =======================
        // Every tracing lane tests every distinct leaf box -- the whole wave reads the same box, one
        // uniform loop, no divergence -- then Moller-Trumbore on its candidate triangles in DFS order:
        // exactly the triangles the reference's traversal tests (the leaf's slab test decides, see
        // rt_scene.cpp), so the closest hit (ties: the later leaf) and the shadow verdict are the
        // reference's.  A ray with a non-finite reciprocal direction (no monotone slab test) sends its
        // wave through the BVH rounds below, run to completion.
        bool coherent = false;
        if (!COUNT && P.n_lboxes > 0) {
            const bool tracing = in_path && !tdone;
            coherent = __all(!tracing || rcp_finite(ray));
            if (coherent && tracing) {
                uint64_t cand = 0;
                for (uint32_t b = 0; b < P.n_lboxes; ++b) {
                    const float4 q0 = S.lboxes[2 * b], q1 = S.lboxes[2 * b + 1];   // (lo.x, hi.x, lo.y, hi.y)(lo.z, hi.z, masks)
                    if (slab_hit_finite(ray, q0.x, q0.z, q1.x, q0.y, q0.w, q1.y))
                        cand |= (uint64_t)(uint32_t)f2i(q1.z) | ((uint64_t)(uint32_t)f2i(q1.w) << 32);
                }
                while (cand != 0) {
                    const int tri = __builtin_ctzll(cand);
                    cand &= cand - 1;
                    const float4 t0 = S.tris[4 * tri], t1 = S.tris[4 * tri + 1], t2 = S.tris[4 * tri + 2];
                    double t;
                    if (moller_trumbore(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, ray, t)) {
                        if (shadow) {
                            if (!(slen < t + (double)0.01f)) { toccl = true; break; }   // MC/Renderer.cpp:184
                        } else if (t <= tbest) {
                            tbest = t; ttri = tri;   // the later leaf wins ties
                        }
                    }
                }
                ti = NN;
                tdone = true;
            }
        }

        // ======================= traversal rounds =======================
        // Rounds continue while more than `thresh` lanes are still tracing, or while nobody waits for
        // service; then the finished lanes are served while the stragglers keep their traversal state.
        // (Small scenes come here only for a non-finite ray: then every ray of the wave runs to the end.)
        const uint32_t thresh = (!COUNT && P.n_lboxes > 0) ? 0u : P.thresh;
        for (;;) {
            if (coherent) break;
            const bool tracing = in_path && !tdone;
            const uint64_t act = __ballot(tracing);
            if (act == 0) break;
            const uint64_t srv = __ballot((in_path && tdone) || (alive && !have_pixel));
            if ((uint32_t)__popcll(act) <= thresh && srv != 0) break;
            const bool fin = __all(!tracing || rcp_finite(ray));
            if (COUNT && lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) ++w_rounds;
            if (tracing) {
                // box steps; up to two leaves are parked (in DFS order) before the lane stops
                int parked0 = -1, parked1 = -1;
                if (fin) {
                    for (uint32_t s = 0; s < P.steps && ti < NN; ++s) {
                        const float4 q0 = S.nodes[2 * ti];
                        const float4 q1 = S.nodes[2 * ti + 1];
                        if (COUNT) { ++node_tests; if (lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) ++w_steps; }
                        const bool hit = slab_hit_finite(ray, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
                        const int tri = f2i(q1.w);
                        ti = (hit && tri < 0) ? ti + 1 : (uint32_t)f2i(q1.z);
                        if (hit && tri >= 0) {
                            if (parked0 < 0) parked0 = tri;
                            else { parked1 = tri; break; }
                        }
                    }
                } else {
                    for (uint32_t s = 0; s < P.steps && ti < NN; ++s) {
                        const float4 q0 = S.nodes[2 * ti];
                        const float4 q1 = S.nodes[2 * ti + 1];
                        if (COUNT) { ++node_tests; if (lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) ++w_steps; }
                        const bool hit = slab_hit(ray, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
                        const int tri = f2i(q1.w);
                        ti = (hit && tri < 0) ? ti + 1 : (uint32_t)f2i(q1.z);
                        if (hit && tri >= 0) {
                            if (parked0 < 0) parked0 = tri;
                            else { parked1 = tri; break; }
                        }
                    }
                }
                // intersect the parked triangles in order
                for (int slot = 0; slot < 2; ++slot) {
                    const int parked = slot == 0 ? parked0 : parked1;
                    if (parked < 0 || toccl) continue;
                    if (COUNT) { ++tri_tests; if (lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1)) ++w_mt; }
                    double t;
                    if (leaf_hit(S, parked, ray, t)) {
                        if (shadow) {
                            // not occluded iff length(q-p) < t + 0.01f for every hit (MC/Renderer.cpp:184)
                            if (!(slen < t + (double)0.01f)) { toccl = true; ti = NN; }
                        } else if (t <= tbest) {
                            // (left.t < right.t) ? left : right  ==> the later leaf wins ties
                            tbest = t; ttri = parked;
                        }
                    }
                }
                if (ti >= NN) tdone = true;
            }
        }
        if (COUNT) c_trace += clock64() - tc2;
    }

    if (COUNT) {
        // wave-reduce, one atomic per wave
        uint64_t a = node_tests, b = tri_tests, c = rays;
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_down(a, off); b += __shfl_down(b, off); c += __shfl_down(c, off);
        }
        // wave-level counts live in exactly one lane: the sum is the wave's count
        uint64_t wr = w_rounds, ws = w_steps, wm = w_mt, wv = w_service, wf = w_fold;
        for (int off = 32; off > 0; off >>= 1) {
            wr += __shfl_down(wr, off); ws += __shfl_down(ws, off); wm += __shfl_down(wm, off);
            wv += __shfl_down(wv, off); wf += __shfl_down(wf, off);
        }
        if (lane == 0) {
            atomicAdd((unsigned long long*)&P.counters[9], (unsigned long long)c_service);
            atomicAdd((unsigned long long*)&P.counters[10], (unsigned long long)c_queue);
            atomicAdd((unsigned long long*)&P.counters[11], (unsigned long long)c_trace);
            atomicAdd((unsigned long long*)&P.counters[12], (unsigned long long)s_lanes);
            atomicAdd((unsigned long long*)&P.counters[0], (unsigned long long)a);
            atomicAdd((unsigned long long*)&P.counters[1], (unsigned long long)b);
            atomicAdd((unsigned long long*)&P.counters[2], (unsigned long long)c);
            atomicAdd((unsigned long long*)&P.counters[4], (unsigned long long)wr);
            atomicAdd((unsigned long long*)&P.counters[5], (unsigned long long)ws);
            atomicAdd((unsigned long long*)&P.counters[6], (unsigned long long)wm);
            atomicAdd((unsigned long long*)&P.counters[7], (unsigned long long)wv);
            atomicAdd((unsigned long long*)&P.counters[8], (unsigned long long)wf);
        }
    }
}

#define RT_INST(E, C, L) template __global__ void pt_megakernel<E, C, L, false>(KParams);
template __global__ void pt_megakernel<true, false, true, true>(KParams);
template __global__ void pt_megakernel<true, false, false, true>(KParams);
RT_INST(true, false, true) RT_INST(true, true, true) RT_INST(false, false, true) RT_INST(false, true, true)
RT_INST(true, false, false) RT_INST(true, true, false) RT_INST(false, false, false) RT_INST(false, true, false)

namespace {
template <bool E, bool C, bool L>
hipError_t launch_one(const KParams& P, uint32_t grid, uint32_t block, size_t lds, hipStream_t s)
{
    hipLaunchKernelGGL((pt_megakernel<E, C, L>), dim3(grid), dim3(block), lds, s, P);
    return hipGetLastError();
}
template <bool E, bool C, bool L>
int occ_one(int block, size_t lds)
{
    int n = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_megakernel<E, C, L>, block, lds) == hipSuccess ? n : 0;
}
}  // namespace

size_t rt_stack_lds_bytes(uint32_t levels) { return (size_t)levels * 256 * (sizeof(float4) + 1); }

size_t rt_lane_state_lds_bytes(bool exact) { return (size_t)(exact ? LS_WORDS_EXACT : LS_WORDS_FAST) * 256 * sizeof(float); }

size_t rt_scene_lds_bytes(const KParams& P)
{
    return (size_t)(2 * P.n_nodes + 4 * P.n_tris + 2 * P.n_mats + P.n_lnodes + 4 * P.n_ltris + 2 * P.n_lboxes) * sizeof(float4);
}

hipError_t rt_launch_megakernel(const KParams& P, bool exact, bool count, bool lds, uint32_t grid, uint32_t block, hipStream_t stream)
{
    const size_t sh = (lds ? rt_scene_lds_bytes(P) : 0) + (exact ? rt_stack_lds_bytes(P.lds_levels) : 0) + rt_lane_state_lds_bytes(exact || P.gb_color) + P.lds_pad;
    if (P.gb_color) {   // the Denoiser's G-buffer frame (EXACT, no counters)
        if (lds) hipLaunchKernelGGL((pt_megakernel<true, false, true, true>), dim3(grid), dim3(block), sh, stream, P);
        else hipLaunchKernelGGL((pt_megakernel<true, false, false, true>), dim3(grid), dim3(block), sh, stream, P);
        return hipGetLastError();
    }
    const int sel = (exact ? 4 : 0) | (count ? 2 : 0) | (lds ? 1 : 0);
    switch (sel) {
        case 7: return launch_one<true, true, true>(P, grid, block, sh, stream);
        case 6: return launch_one<true, true, false>(P, grid, block, sh, stream);
        case 5: return launch_one<true, false, true>(P, grid, block, sh, stream);
        case 4: return launch_one<true, false, false>(P, grid, block, sh, stream);
        case 3: return launch_one<false, true, true>(P, grid, block, sh, stream);
        case 2: return launch_one<false, true, false>(P, grid, block, sh, stream);
        case 1: return launch_one<false, false, true>(P, grid, block, sh, stream);
        default: return launch_one<false, false, false>(P, grid, block, sh, stream);
    }
}

int rt_megakernel_occupancy(bool exact, bool count, bool lds, int block, size_t lds_bytes)
{
    const int sel = (exact ? 4 : 0) | (count ? 2 : 0) | (lds ? 1 : 0);
    switch (sel) {
        case 7: return occ_one<true, true, true>(block, lds_bytes);
        case 6: return occ_one<true, true, false>(block, lds_bytes);
        case 5: return occ_one<true, false, true>(block, lds_bytes);
        case 4: return occ_one<true, false, false>(block, lds_bytes);
        case 3: return occ_one<false, true, true>(block, lds_bytes);
        case 2: return occ_one<false, true, false>(block, lds_bytes);
        case 1: return occ_one<false, false, true>(block, lds_bytes);
        default: return occ_one<false, false, false>(block, lds_bytes);
    }
}

// ---------------------------------------------------------------------------------------------
// in-order completion of chunked pixels: accum (after chunk 0) += every later frame's sample in frame
// order, then clamp + pack (MC/Renderer.cpp:128-133).  One thread per local pixel; a 4-frame block is
// three float4 loads, adjacent pixels' blocks adjacent (coalesced across the wave).
__global__ void __launch_bounds__(256) finalize_chunks_kernel(KParams P, uint32_t n_px)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_px) return;
    // park_all: every frame of the launch is parked, the accumulation starts from 0 at frame 1 and from
    // the accumulator otherwise; else chunk 0 has accumulated in place and the later chunks are parked
    float4 acc = (P.park_all && P.first_frame == 1u) ? make_float4(0.f, 0.f, 0.f, 0.f) : P.accum[i];
    const uint32_t nfp = P.park_all ? P.n_frames : P.n_frames - P.chunk_frames;
    // the pre-pass's sky bits (KParams::sky_bits): a camera-ray miss adds the night sky's radiance, which the pre-pass
    // would have parked (cast_path, MC/Renderer.cpp:145); a 4-frame block of misses is not read at all
    const float SKY_R = kNightSkyR, SKY_G = kNightSkyG, SKY_B = kNightSkyB;
    uint32_t skyw = 0;
    for (uint32_t b = 0; b * 4u < nfp; ++b) {
        if (P.sky_bits != nullptr && (b & 7u) == 0u) skyw = P.sky_bits[(size_t)(b >> 3) * P.lbuf_stride + i];
        const uint32_t sky4 = P.sky_bits != nullptr ? (skyw >> (4u * (b & 7u))) & 0xFu : 0u;
        const uint32_t n = min(4u, nfp - b * 4u);
        float v[12];
        if (sky4 != ((1u << n) - 1u)) {
            const size_t bi = (P.park_all && P.lbuf_pixel_major) ? (size_t)i * ((nfp + 3u) >> 2) + b : (size_t)b * P.lbuf_stride + i;
            const float4* blk = reinterpret_cast<const float4*>(P.lbuf + bi * 12u);
            const float4 q0 = blk[0], q1 = blk[1], q2 = blk[2];
            v[0] = q0.x; v[1] = q0.y; v[2] = q0.z; v[3] = q0.w; v[4] = q1.x; v[5] = q1.y;
            v[6] = q1.z; v[7] = q1.w; v[8] = q2.x; v[9] = q2.y; v[10] = q2.z; v[11] = q2.w;
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            if (j < n) {
                const bool sky = (sky4 >> j) & 1u;
                acc.x = acc.x + (sky ? SKY_R : v[3 * j]); acc.y = acc.y + (sky ? SKY_G : v[3 * j + 1]); acc.z = acc.z + (sky ? SKY_B : v[3 * j + 2]);
                acc.w = acc.w + 1.0f;
            }
        }
    }
    const float fr = (float)(P.first_frame + P.n_frames - 1u);
    const float rx = smin(smax(acc.x / fr, 0.0f), 1.0f), gy = smin(smax(acc.y / fr, 0.0f), 1.0f);
    const float bz = smin(smax(acc.z / fr, 0.0f), 1.0f), aw = smin(smax(acc.w / fr, 0.0f), 1.0f);
    P.accum[i] = acc;
    P.rgba[i] = (to_u8(aw) << 24) | (to_u8(bz) << 16) | (to_u8(gy) << 8) | to_u8(rx);
}

hipError_t rt_launch_finalize_chunks(const KParams& P, uint32_t n_px, hipStream_t stream)
{
    if (n_px == 0 || (P.n_chunks <= 1 && !P.park_all)) return hipSuccess;
    hipLaunchKernelGGL(finalize_chunks_kernel, dim3((n_px + 255) / 256), dim3(256), 0, stream, P, n_px);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// closest-hit query kernel (unit-test entry point of the C-ABI: rt_trace)
__global__ void __launch_bounds__(256) trace_kernel(KParams P, uint32_t n, const float* __restrict__ org, const float* __restrict__ dir,
                                                    int32_t* __restrict__ tri_out, double* __restrict__ t_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SceneView S{P.nodes, P.tris, P.mats, P.lnodes, P.ltris, P.n_nodes, P.lboxes};
    const Ray r = make_ray(V3{org[3 * i], org[3 * i + 1], org[3 * i + 2]}, V3{dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]});
    uint32_t a = 0, b = 0;
    double best = 1.7976931348623157e308;
    int best_tri = -1;
    bool occl = false;
    traverse_impl<false, false>(S, r, false, 0.0, best, best_tri, occl, a, b);
    tri_out[i] = best_tri;
    t_out[i] = best_tri >= 0 ? best : 1.7976931348623157e308;
}

hipError_t rt_launch_trace(const KParams& P, uint32_t n, const float* org, const float* dir, int32_t* tri, double* t, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(trace_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, P, n, org, dir, tri, t);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// light-sampling query kernel (C-ABI rt_sample_light: Renderer::SamplingAreaLight of the drop-in,
// MC/Renderer.h:163-180): the path kernels' sample_light on three given u32 draws per case
struct GivenDraws {
    const uint32_t* u;
    uint32_t k;
    __device__ __forceinline__ float next() { return (float)u[k++] / 4294967296.0f; }   // Walnut::Random::Float (WN/Random.h:27-30)
};

__global__ void __launch_bounds__(256) light_sample_kernel(KParams P, uint32_t n, const uint32_t* __restrict__ u, float* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SceneView S{P.nodes, P.tris, P.mats, P.lnodes, P.ltris, P.n_nodes, P.lboxes};
    GivenDraws g{u + 3 * (size_t)i, 0u};
    V3 q, nl;
    sample_light(S, P.light_area, g, q, nl);
    float* o = out + 10 * (size_t)i;
    o[0] = q.x; o[1] = q.y; o[2] = q.z;
    o[3] = nl.x; o[4] = nl.y; o[5] = nl.z;
    o[6] = P.light_emission[0]; o[7] = P.light_emission[1]; o[8] = P.light_emission[2];
    o[9] = P.lpdf;   // the PDF Sampling_from_root overwrites with 1 / (the light's total area), MC/BVH.h:105-106
}

hipError_t rt_launch_light_sample(const KParams& P, uint32_t n, const uint32_t* u, float* out, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(light_sample_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, P, n, u, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// math self-test kernel: device f32 sqrt/div, f64 reciprocal, cos/sin as the megakernel evaluates them,
// and the denoiser's expf/acosf (rt_glibc_math.h)
__global__ void math_kernel(uint32_t n, const float* __restrict__ x, float* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    out[9 * i + 0] = __builtin_sqrtf(v);
    out[9 * i + 1] = rcp_f32(v);   // the kernels' reciprocal (rt_device.h); == 1.0f / v correctly rounded
    float cv, sv;
    sincos_f(v, cv, sv);   // what sample_hemisphere evaluates (rt_path.h)
    out[9 * i + 2] = cv;
    out[9 * i + 3] = sv;
    const double r = rcp_f64_of_f32(v);   // Moller-Trumbore's 1 / (double)den (rt_device.h)
    out[9 * i + 4] = __int_as_float((int)(uint32_t)(__double_as_longlong(r) & 0xFFFFFFFFull));
    out[9 * i + 5] = __int_as_float((int)(uint32_t)((unsigned long long)__double_as_longlong(r) >> 32));
    out[9 * i + 6] = pow_lobe(v, 25.0f);   // the C1 specular lobe, powf(x, specular_size_factor = 25)
    out[9 * i + 7] = glibc_math::expf<true>(v);   // the joint bilateral weight's exp (DN/Denoiser.h:203)
    out[9 * i + 8] = glibc_math::acosf(v);        // its normal-angle acos (DN/Denoiser.h:195)
}

hipError_t rt_launch_math(uint32_t n, const float* x, float* out, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(math_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n, x, out);
    return hipGetLastError();
}

#if RT_WALK_STUDY
// ---------------------------------------------------------------------------------------------
// Walk study (a variant build only: make KFLAGS=-DRT_WALK_STUDY=1, tools/walk_study.py; the product library has
// none of it).  The C5 path kernel's BVH rounds (rt_coherent.hip, the split scene's near-first walk of the subtree
// [split_root, split_end)) lifted into a kernel of their own whose lane carries K independent rays: per step every
// active ray's node load is issued before any is tested, so a lane keeps K dependent loads in flight instead of one.
// A round is `steps` node tests per ray, a ray parks up to two leaves and stops stepping for the round at the second,
// and the parked leaves are intersected at the round's end (the path kernel's round shape).  Closest hit within the
// subtree by (min t, max triangle) from t = +inf (MC/BVH.h:82-101 restricted to the subtree; equal to rt_trace's
// result whenever that lies in the subtree).  Ray k of wave w's lane l is ray (w * K + k) * 64 + l: each of a
// lane's slots is a run of 64 consecutive rays.
template <int K, bool COUNT = false>
__global__ void __launch_bounds__(256, K <= 2 ? 8 : 1) walk_study_kernel(KParams P, uint32_t n, const float* __restrict__ org, const float* __restrict__ dir,
                                                         int32_t* __restrict__ tri_out, double* __restrict__ t_out)
{
    const uint32_t lane = threadIdx.x & 63u, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t NN = P.n_nodes, root = P.split_root, tend = P.split_end, steps = P.steps;
    V3 o[K], d[K], rc[K];
    uint32_t ti[K], oct[K];
    double tA[K];
    int triA[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t i = (wave * (uint32_t)K + (uint32_t)k) * 64u + lane;
        const bool ok = i < n;
        const uint32_t j = ok ? i : 0u;
        o[k] = V3{org[3 * j], org[3 * j + 1], org[3 * j + 2]};
        d[k] = V3{dir[3 * j], dir[3 * j + 1], dir[3 * j + 2]};
        rc[k] = V3{rcp_f32(d[k].x), rcp_f32(d[k].y), rcp_f32(d[k].z)};
        const bool fin = __builtin_isfinite(rc[k].x) && __builtin_isfinite(rc[k].y) && __builtin_isfinite(rc[k].z);
        ti[k] = (ok && fin) ? root : NN;
        oct[k] = ((uint32_t)(d[k].x < 0.0f) | ((uint32_t)(d[k].y < 0.0f) << 1) | ((uint32_t)(d[k].z < 0.0f) << 2)) * P.wcopy_stride;
        tA[k] = 1.7976931348623157e308;
        triA[k] = (ok && !fin) ? -2 : -1;   // -2: a non-finite reciprocal direction (not walked here)
    }
    uint32_t rounds = 0;   // COUNT: the lane's (ray, round) pairs
    for (;;) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            any |= ti[k] < tend;
            if (COUNT) rounds += ti[k] < tend ? 1u : 0u;
        }
        if (!any) break;
        int p0[K], p1[K];
        float bnd[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            p0[k] = -1; p1[k] = -1;
            bnd[k] = (tA[k] < 1e30) ? (float)tA[k] * 1.00001f + 1e-5f : __builtin_inff();
        }
        for (uint32_t s = 0; s < steps; ++s) {
            bool go[K], anyg = false;
            float4 q0[K], q1[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                go[k] = ti[k] < tend && p1[k] < 0;
                anyg |= go[k];
            }
            if (!anyg) break;
#pragma unroll
            for (int k = 0; k < K; ++k) {   // every slot's load first (an idle slot reads the subtree root)
                const float4* wn = P.wcopies + oct[k];
                const uint32_t at = 2u * (go[k] ? ti[k] : root);
                q0[k] = wn[at];
                q1[k] = wn[at + 1];
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!go[k]) continue;
                const Ray r{o[k], d[k], rc[k], false, false, false};
                const bool hit = slab_nf_within(r, q0[k].x, q0[k].y, q0[k].z, q0[k].w, q1[k].x, q1[k].y, bnd[k]);
                const int tri = f2i(q1[k].w);
                ti[k] = (hit && tri < 0) ? ti[k] + 1u : (uint32_t)f2i(q1[k].z);
                if (hit && tri >= 0) {
                    if (p0[k] < 0) p0[k] = tri;
                    else p1[k] = tri;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            for (int slot = 0; slot < 2; ++slot) {
                const int pk = slot == 0 ? p0[k] : p1[k];
                if (pk < 0) continue;
                const float4 t0 = P.tris[4 * pk], t1 = P.tris[4 * pk + 1], t2 = P.tris[4 * pk + 2];
                double t;
                if (moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o[k], d[k], t))
                    if (t < tA[k] || (t == tA[k] && (uint32_t)pk > (uint32_t)triA[k])) { tA[k] = t; triA[k] = pk; }
            }
            if (ti[k] >= tend) ti[k] = NN;
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t i = (wave * (uint32_t)K + (uint32_t)k) * 64u + lane;
        if (i < n) {
            tri_out[i] = triA[k];
            t_out[i] = triA[k] >= 0 ? tA[k] : 1.7976931348623157e308;
        }
    }
    if (COUNT) {
        for (int off = 32; off >= 1; off >>= 1) rounds += (uint32_t)__shfl_xor((int)rounds, off);
        if (lane == 0) atomicAdd(&P.counters[8u * (blockIdx.x & 7u)], (unsigned long long)rounds);   // (64 B apart)
    }
}

// the same walk with refill: a persistent grid whose lanes take a new ray into a slot as soon as the slot's ray is done
// (one atomic per wave and slot: the wave's free slots counted by ballot, their rays numbered by mbcnt), so a lane's K
// slots do not wait for the longest of their rays
template <int K>
__global__ void __launch_bounds__(256, K <= 1 ? 8 : 1) walk_study_refill_kernel(KParams P, uint32_t n, const float* __restrict__ org, const float* __restrict__ dir,
                                                                int32_t* __restrict__ tri_out, double* __restrict__ t_out, uint32_t* __restrict__ next_ray)
{
    const uint32_t NN = P.n_nodes, root = P.split_root, tend = P.split_end, steps = P.steps;
    V3 o[K], d[K], rc[K];
    uint32_t ti[K], oct[K], id[K];
    double tA[K];
    int triA[K];
#pragma unroll
    for (int k = 0; k < K; ++k) { id[k] = 0xFFFFFFFFu; ti[k] = NN; }
    // the rays in 8 contiguous parts, one counter each (64 B apart), a block's part its blockIdx mod 8; a wave takes
    // CHUNK rays per atomic into a wave-uniform local range [qb, qe) and refills its free slots from it
    constexpr uint32_t CHUNK = 256;
    const uint32_t part = blockIdx.x & 7u;
    const uint32_t lo = (uint32_t)((uint64_t)n * part / 8u), hi = (uint32_t)((uint64_t)n * (part + 1u) / 8u);
    uint32_t* ctr = next_ray + 16u * part;
    uint32_t qb = 0, qe = 0;
    bool more = true;
    for (;;) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (more) {
                const bool need = id[k] == 0xFFFFFFFFu;
                const uint64_t m = __ballot(need);
                if (m != 0) {
                    if (qb == qe) {
                        uint32_t b = 0;
                        if (__lane_id() == (uint32_t)__builtin_ctzll(m)) b = atomicAdd(ctr, CHUNK);
                        b = lo + (uint32_t)__shfl((int)b, (int)__builtin_ctzll(m));
                        if (b >= hi) more = false;
                        else { qb = b; qe = min(b + CHUNK, hi); }
                    }
                    const uint32_t rank = (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull)), avail = qe - qb;
                    const uint32_t my = qb + rank;
                    qb += min(avail, (uint32_t)__popcll(m));
                    if (need && rank < avail) {
                        id[k] = my;
                        o[k] = V3{org[3 * my], org[3 * my + 1], org[3 * my + 2]};
                        d[k] = V3{dir[3 * my], dir[3 * my + 1], dir[3 * my + 2]};
                        rc[k] = V3{rcp_f32(d[k].x), rcp_f32(d[k].y), rcp_f32(d[k].z)};
                        const bool fin = __builtin_isfinite(rc[k].x) && __builtin_isfinite(rc[k].y) && __builtin_isfinite(rc[k].z);
                        ti[k] = fin ? root : NN;
                        oct[k] = ((uint32_t)(d[k].x < 0.0f) | ((uint32_t)(d[k].y < 0.0f) << 1) | ((uint32_t)(d[k].z < 0.0f) << 2)) * P.wcopy_stride;
                        tA[k] = 1.7976931348623157e308;
                        triA[k] = fin ? -1 : -2;
                    }
                }
            }
        }
        bool busy = false;
#pragma unroll
        for (int k = 0; k < K; ++k) busy |= id[k] != 0xFFFFFFFFu;
        if (!__any(busy)) break;
        int p0[K], p1[K];
        float bnd[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            p0[k] = -1; p1[k] = -1;
            bnd[k] = (tA[k] < 1e30) ? (float)tA[k] * 1.00001f + 1e-5f : __builtin_inff();
        }
        for (uint32_t s = 0; s < steps; ++s) {
            bool go[K], anyg = false;
            float4 q0[K], q1[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                go[k] = ti[k] < tend && p1[k] < 0;
                anyg |= go[k];
            }
            if (!anyg) break;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float4* wn = P.wcopies + oct[k];
                const uint32_t at = 2u * (go[k] ? ti[k] : root);
                q0[k] = wn[at];
                q1[k] = wn[at + 1];
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!go[k]) continue;
                const Ray r{o[k], d[k], rc[k], false, false, false};
                const bool hit = slab_nf_within(r, q0[k].x, q0[k].y, q0[k].z, q0[k].w, q1[k].x, q1[k].y, bnd[k]);
                const int tri = f2i(q1[k].w);
                ti[k] = (hit && tri < 0) ? ti[k] + 1u : (uint32_t)f2i(q1[k].z);
                if (hit && tri >= 0) {
                    if (p0[k] < 0) p0[k] = tri;
                    else p1[k] = tri;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            for (int slot = 0; slot < 2; ++slot) {
                const int pk = slot == 0 ? p0[k] : p1[k];
                if (pk < 0) continue;
                const float4 t0 = P.tris[4 * pk], t1 = P.tris[4 * pk + 1], t2 = P.tris[4 * pk + 2];
                double t;
                if (moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, o[k], d[k], t))
                    if (t < tA[k] || (t == tA[k] && (uint32_t)pk > (uint32_t)triA[k])) { tA[k] = t; triA[k] = pk; }
            }
            if (id[k] != 0xFFFFFFFFu && ti[k] >= tend) {   // done: its result out, the slot free
                tri_out[id[k]] = triA[k];
                t_out[id[k]] = triA[k] >= 0 ? tA[k] : 1.7976931348623157e308;
                id[k] = 0xFFFFFFFFu;
                ti[k] = NN;
            }
        }
    }
}

hipError_t rt_launch_walk_study(const KParams& P, uint32_t n, uint32_t k, const float* org, const float* dir, int32_t* tri, double* t, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    const uint32_t kk = k & 0xFFu, waves = (n + 64u * kk - 1u) / (64u * kk), grid = (waves + 3u) / 4u;
    if (k & 0x100u) {   // refill: a persistent grid of 8 waves per SIMD (256 CUs x 4 SIMDs x 8 / 4 waves per block)
        uint32_t* ctr = reinterpret_cast<uint32_t*>(P.counters);   // 8 counters, 64 B apart (zeroed by the caller)
        const uint32_t g = 256u * 8u;
        switch (k & 0xFFu) {
        case 1: hipLaunchKernelGGL(walk_study_refill_kernel<1>, dim3(g), dim3(256), 0, stream, P, n, org, dir, tri, t, ctr); break;
        case 2: hipLaunchKernelGGL(walk_study_refill_kernel<2>, dim3(g), dim3(256), 0, stream, P, n, org, dir, tri, t, ctr); break;
        case 3: hipLaunchKernelGGL(walk_study_refill_kernel<3>, dim3(g), dim3(256), 0, stream, P, n, org, dir, tri, t, ctr); break;
        case 4: hipLaunchKernelGGL(walk_study_refill_kernel<4>, dim3(g), dim3(256), 0, stream, P, n, org, dir, tri, t, ctr); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (k == 0x201u) {   // the round count (K = 1, lockstep; a ray's rounds do not depend on the kernel's mode)
        hipLaunchKernelGGL((walk_study_kernel<1, true>), dim3(grid * 1u), dim3(256), 0, stream, P, n, org, dir, tri, t);
        return hipGetLastError();
    }
    switch (k) {
    case 1: hipLaunchKernelGGL(walk_study_kernel<1>, dim3(grid), dim3(256), 0, stream, P, n, org, dir, tri, t); break;
    case 2: hipLaunchKernelGGL(walk_study_kernel<2>, dim3(grid), dim3(256), 0, stream, P, n, org, dir, tri, t); break;
    case 3: hipLaunchKernelGGL(walk_study_kernel<3>, dim3(grid), dim3(256), 0, stream, P, n, org, dir, tri, t); break;
    case 4: hipLaunchKernelGGL(walk_study_kernel<4>, dim3(grid), dim3(256), 0, stream, P, n, org, dir, tri, t); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
#endif
