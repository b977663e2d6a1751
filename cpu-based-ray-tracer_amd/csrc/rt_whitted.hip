// rt_whitted.hip -- Whitted-style ray tracing of the reference's "BVH Ray Tracer" (config C3:
// Stanford bunny + Utah teapot, two point lights; BV/ = "BVH Ray Tracer/8599RayTracerGUI/src/").
//
// Per pixel and frame, as Renderer::RayGen_Shader -> cast_Whitted_ray (BV/Renderer.cpp:109-233) with
// every triangle Diffuse_Glossy (BV/TriangleMesh.h:138-141):
//   * corner-of-pixel camera ray (BV/Camera.cpp:114-132; no jitter, the scene is deterministic);
//   * closest hit through the same flattened two-level BVH as the path tracer (rt_layout.h), ties to
//     the later leaf (BV/BVH.h:82-101);
//   * miss -> sky color; hit -> for each point light in order: light direction from the hit
//     location, shadow ray from the offset shading point, occluded iff the closest hit has
//     t*t < |L - x|^2 (evaluated any-hit: the predicate is monotone in t), diffuse term
//     radiance * |dot(l, n)|; color = (sum * diffuse_color) * phong_diffuse.  The specular term is
//     total_specular * phong_specular with phong_specular == 0 for every mesh of the scene
//     (BV/TriangleMesh.h:139); it adds +0 to a non-negative color and is not evaluated;
//   * accumulation, average, clamp and ABGR8 pack as RayGen_Shader.
// The scene (1.4 MB for C3) is read from HBM through L2; a block per 8x8 tile of local pixels, one wave per
// group of frames (whitted_kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rt_device.h"
#include "rt_kernels.h"
#include "rt_layout.h"

using namespace rtd;

namespace {

// box tests per round of the C3 walk; a round's hit leaves (two at most) are postponed to its end, so a
// wave runs Moller-Trumbore once per round (8: 6044 Msamples/s; 4: 5681, 16: 5729;
// profiles/r03/ab/ab_c3_whitted.json)
#ifndef RT_WH_STEPS
#define RT_WH_STEPS 8
#endif
#ifndef RT_WH_HALF
#define RT_WH_HALF 0   // 1: walk the 16-byte half-plane orderings when the scene has them (P.worders_h; measured -3 %: DESIGN.md 5.3)
#endif


struct FiniteSlab { static constexpr bool value = true; };
struct GeneralSlab { static constexpr bool value = false; };

// scalar loads of wave-uniform data (constant address space)
typedef float box8 __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(4))) box8 cbox8;
typedef float vec4f __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) vec4f cf4;

// the packet walk (round 6): a wave whose rays all have finite reciprocals and one direction octant walks the
// octant's near-first ordering TOGETHER -- one wave-uniform node index, each node one scalar load for the whole
// wave (s_load: the vector memory pipeline, which the per-lane walk's 64 gathers per step occupy, is not used),
// every lane testing it against its own ray and bound; the wave descends when any lane enters the box, and a
// leaf's triangle (scalar loads too) is intersected by the lanes whose own test entered the leaf's box.  Exact:
// a lane's tests are its own slab tests on the reference's planes, and a box inside one the lane missed (or
// entered beyond its bound) is missed too (the finite slab test is monotone, the entry only grows), so each
// lane intersects exactly the leaves its own walk would, and the closest hit is taken by (min t, max triangle)
// whatever the order.  Measured (bitwise, the C3 tests green): 14,835 -> 11,004 Msamples/s (profiles/r06/ab/
// ab_c3_packet_walk.json) -- a scalar load that misses the small scalar cache waits on L2 every step, longer than the
// per-lane gathers' vL1D hits, and the wave walks the union of its lanes' paths; off.
#ifndef RT_WH_PACKET
#define RT_WH_PACKET 0
#endif

// closest hit (shadow == false) or "any hit with t*t < d2" (shadow == true) over the global scene
template <bool COUNT>
__device__ __forceinline__ void whitted_traverse(const KParams& P, const Ray& r, bool shadow, double d2, double& best, int& best_tri, bool& occluded,
                                                 uint32_t& node_tests, uint32_t& tri_tests)
{
    // A box entered beyond every t that can still change the result is skipped (the C5 walk's rule,
    // rt_coherent.hip): a triangle inside the box hits at t >= the box's exact entry, and the float entry
    // is that value up to 3 roundings (2e-7 relative), so with 1e-5 relative margin only boxes whose
    // triangles lose are skipped -- to the closest hit so far (a tie needs t == best: entry <= best), or,
    // for a shadow ray, to the light (occluded needs t * t < d2, BV/Renderer.cpp:195, so t < sqrt(d2)).
    // The reference visits every hit box (BV/BVH.h:82-101).  Rays with a non-finite reciprocal keep the
    // std::max/min slab test and visit every hit box.
    const float4* __restrict__ nodes = P.nodes;
    const float4* __restrict__ tris = P.tris;
    const uint32_t n = P.n_nodes;
    const float sbound = shadow ? __builtin_sqrtf((float)d2) * 1.00001f + 1e-5f : 0.0f;
    auto tri_test_v = [&](int tri, const V3& va, const V3& e1, const V3& e2) -> bool {   // true: the shadow ray is occluded
        if (COUNT) ++tri_tests;
        double t;
        if (moller_trumbore(va, e1, e2, r, t)) {
            if (shadow) {
                // (shadow_record.has_intersection) && (t * t < light_distance_squared), BV/Renderer.cpp:195
                if (t * t < d2) { occluded = true; return true; }
            } else if (t < best || (t == best && tri > best_tri)) {
                // (left.t < right.t) ? left : right: the later DFS leaf wins ties -- triangles are numbered in
                // DFS order, so in any walk order the winner is (min t, max triangle)
                best = t; best_tri = tri;
            }
        }
        return false;
    };
    auto tri_test = [&](int tri) -> bool {
        const float4 t0 = tris[4 * tri], t1 = tris[4 * tri + 1], t2 = tris[4 * tri + 2];
        return tri_test_v(tri, V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z});
    };
    // the 16-byte orderings (P.worders_h, rt_scene.cpp compact_orderings): one 16-byte load per step instead of two,
    // half planes rounded outward -- a decoded box contains the exact one, so for a finite ray the walk visits every
    // box the exact walk visits (and maybe more), and a box entered beyond the bound is still beyond it -- and a
    // leaf the half box passes is tested against its EXACT box, its triangle's vertex box (Triangle::Get3DAABB,
    // BV/TriangleMesh.h; the same floats as the tree's leaf box, checked on the host), before Moller-Trumbore: the
    // candidates are exactly the float walk's.  (C3's walk is bound by the vL1D's gather rate -- 1.35 node loads
    // per CU-clock of the calibrated 1.54 in round 5 -- so the node bytes per step are the lever, not the latency.)
    auto walk_half = [&]() {
        const uint4* __restrict__ wh = P.worders_h + n * ((uint32_t)r.nx | ((uint32_t)r.ny << 1) | ((uint32_t)r.nz << 2));
        const float4* __restrict__ tabc = P.tabc;
        auto h2f = [](uint32_t b) { return (float)__builtin_bit_cast(_Float16, (unsigned short)b); };
        uint32_t i = 0;
        while (i < n) {
            const float bound = shadow ? sbound : ((best < 1e30) ? (float)best * 1.00001f + 1e-5f : __builtin_inff());
            int p0 = -1, p1 = -1;
            for (uint32_t s = 0; s < RT_WH_STEPS && i < n; ++s) {
                if (COUNT) ++node_tests;
                const uint4 q = wh[i];
                const bool hit = slab_nf_within(r, h2f(q.x & 0xFFFFu), h2f(q.y & 0xFFFFu), h2f(q.z & 0xFFFFu), h2f(q.x >> 16), h2f(q.y >> 16),
                                                h2f(q.z >> 16), bound);
                const bool leaf = (q.w & 0x80000000u) != 0u;
                i = (hit || leaf) ? i + 1 : q.w;
                if (hit && leaf) {
                    const int tri = (int)(q.w & 0x7FFFFFFFu);
                    if (p0 < 0) p0 = tri;
                    else { p1 = tri; break; }
                }
            }
            for (int k = 0; k < 2; ++k) {
                const int tri = k == 0 ? p0 : p1;
                if (tri < 0) continue;
                const float4 a = tabc[3 * tri], b = tabc[3 * tri + 1], c = tabc[3 * tri + 2];
                if (!slab_hit_finite_within(r, __builtin_fminf(__builtin_fminf(a.x, b.x), c.x), __builtin_fminf(__builtin_fminf(a.y, b.y), c.y),
                                            __builtin_fminf(__builtin_fminf(a.z, b.z), c.z), __builtin_fmaxf(__builtin_fmaxf(a.x, b.x), c.x),
                                            __builtin_fmaxf(__builtin_fmaxf(a.y, b.y), c.y), __builtin_fmaxf(__builtin_fmaxf(a.z, b.z), c.z), bound))
                    continue;
                const V3 va{a.x, a.y, a.z};
                if (tri_test_v(tri, va, sub(V3{b.x, b.y, b.z}, va), sub(V3{c.x, c.y, c.z}, va))) return;
            }
        }
    };
    auto walk = [&](auto kind, auto baked) {
        constexpr bool FIN = decltype(kind)::value;
        // a finite ray walks the near-first ordering of its direction's octant when the scene has them
        // (rt_scene.cpp near_first: the same leaf boxes, the closest hit found early, farther boxes skipped),
        // whose boxes are stored as the octant's (near, far) planes (BAKED, rt_device.h slab_nf_within)
        constexpr bool BAKED = decltype(baked)::value;
        const float4* __restrict__ wn = BAKED ? P.worders + 2u * n * ((uint32_t)r.nx | ((uint32_t)r.ny << 1) | ((uint32_t)r.nz << 2)) : nodes;
        uint32_t i = 0;
        while (i < n) {
            const float bound = shadow ? sbound : ((best < 1e30) ? (float)best * 1.00001f + 1e-5f : __builtin_inff());
            int p0 = -1, p1 = -1;
            auto test_node = [&](const float4 q0, const float4 q1) -> bool {   // false: two leaves postponed
                if (COUNT) ++node_tests;
                const bool hit = BAKED ? slab_nf_within(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, bound)
                                 : FIN ? slab_hit_finite_within(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, bound) : slab_hit(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
                const int tri = f2i(q1.w);
                i = (hit && tri < 0) ? i + 1 : (uint32_t)f2i(q1.z);
                if (hit && tri >= 0) {
                    if (p0 < 0) p0 = tri;
                    else { p1 = tri; return false; }
                }
                return true;
            };
            // (two nodes per dependent load, as rt_coherent.hip measured: C3 -12 %, profiles/r05/ab/ab_c3_orders.json)
            for (uint32_t s = 0; s < RT_WH_STEPS && i < n; ++s) {
                const float4 q0 = wn[2 * i];
                const float4 q1 = wn[2 * i + 1];
                if (!test_node(q0, q1)) break;
            }
            // the postponed leaves (closest hit: (min t, max triangle), whatever the order)
            if (p0 >= 0 && tri_test(p0)) return;
            if (p1 >= 0 && tri_test(p1)) return;
        }
    };
#if RT_WH_PACKET
    if (P.worders != nullptr) {
        const uint32_t oct = (uint32_t)r.nx | ((uint32_t)r.ny << 1) | ((uint32_t)r.nz << 2);
        const uint32_t oct0 = __builtin_amdgcn_readfirstlane(oct);
        if (__all(rcp_finite(r) && oct == oct0)) {
            cbox8* wn = (cbox8*)(P.worders + 2u * n * oct0);
            cf4* ctris = (cf4*)tris;
            bool live = true;   // a shadow ray stops at its first blocker
            uint32_t i = 0;
            while (i < n) {
                const box8 q = wn[i];
                const int tri = f2i(q.s7);
                const uint32_t skip = (uint32_t)f2i(q.s6);
                const float bound = shadow ? sbound : ((best < 1e30) ? (float)best * 1.00001f + 1e-5f : __builtin_inff());
                if (COUNT && live) ++node_tests;
                const bool hit = live && slab_nf_within(r, q.s0, q.s1, q.s2, q.s3, q.s4, q.s5, bound);
                if (tri >= 0) {
                    if (hit) {
                        const vec4f t0 = ctris[4 * tri], t1 = ctris[4 * tri + 1], t2 = ctris[4 * tri + 2];
                        if (tri_test_v(tri, V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z})) live = false;
                    }
                    i = skip;
                } else {
                    i = __any(hit) ? i + 1 : skip;
                }
                if (shadow && !__any(live)) break;
            }
            return;
        }
    }
#endif
    if (!rcp_finite(r)) walk(GeneralSlab{}, std::false_type{});
    else if (RT_WH_HALF && P.worders_h != nullptr) walk_half();
    else if (P.worders != nullptr) walk(FiniteSlab{}, std::true_type{});
    else walk(FiniteSlab{}, std::false_type{});
}

// The two lights' shadow rays of one hit walked TOGETHER (round 6): both start at the shading point, so the
// lane carries two small walk states -- node index, reciprocal direction, bound, ordering base -- and every
// step issues both rays' node loads before either test: two independent loads in flight per lane where the
// sequential walks had one (the walk waits on L2 latency, not on issue: VALU issue 27 %, SQ_WAIT_ANY 61 %,
// profiles/r05/c3).  A ray that meets a leaf parks it and stops stepping for the round; the round ends with
// each ray's parked leaf tested.  The verdict is any hit with t * t < d2 (BV/Renderer.cpp:195): an existence
// test, so the order of the walks does not matter, and boxes entered beyond the light are skipped with the same
// margin as whitted_traverse.  Rays with a finite reciprocal direction and a scene with near-first orderings
// only (the caller decides per wave).
#ifndef RT_WH_PAIR
#define RT_WH_PAIR 0
#endif
#ifndef RT_WH_PAIR_STEPS
#define RT_WH_PAIR_STEPS 8
#endif
template <bool COUNT>
__device__ __forceinline__ void whitted_shadow_pair(const KParams& P, const V3& x, const V3& sp, bool& occA, bool& occB, uint32_t& node_tests,
                                                    uint32_t& tri_tests)
{
    const uint32_t n = P.n_nodes;
    const float4* __restrict__ wo = P.worders;
    const float4* __restrict__ tris = P.tris;
    // light l's direction from x, normalized, and its squared distance: recomputed where needed (the same
    // operations give the same bits), so the walk keeps no direction live -- only the reciprocals
    auto light_dir = [&](uint32_t l, float& d2) {
        const float4 lp = P.plights[2 * l];
        const V3 ld = sub(V3{lp.x, lp.y, lp.z}, x);
        d2 = dot(ld, ld);
        return w_normalize(ld);
    };
    float d2a, d2b;
    const V3 la = light_dir(0, d2a), lb = light_dir(1, d2b);
    const V3 ra = V3{rcp_f32(la.x), rcp_f32(la.y), rcp_f32(la.z)}, rb = V3{rcp_f32(lb.x), rcp_f32(lb.y), rcp_f32(lb.z)};
    const uint32_t oct = ((uint32_t)(la.x < 0.0f) | ((uint32_t)(la.y < 0.0f) << 1) | ((uint32_t)(la.z < 0.0f) << 2)) |
                         (((uint32_t)(lb.x < 0.0f) | ((uint32_t)(lb.y < 0.0f) << 1) | ((uint32_t)(lb.z < 0.0f) << 2)) << 3);
    const float bA = __builtin_sqrtf(d2a) * 1.00001f + 1e-5f, bB = __builtin_sqrtf(d2b) * 1.00001f + 1e-5f;
    uint32_t ia = 0, ib = 0;
    occA = occB = false;
    auto shadow_test = [&](uint32_t l, int tri) -> bool {
        if (COUNT) ++tri_tests;
        float d2;
        const V3 d = light_dir(l, d2);
        const float4 t0 = tris[4 * tri], t1 = tris[4 * tri + 1], t2 = tris[4 * tri + 2];
        double t;
        return moller_trumbore_od(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, sp, d, t) && t * t < (double)d2;
    };
    auto slab = [&](const V3& rc, const float4& q0, const float4& q1, float bound) {   // slab_nf_within from sp
        const float tix = (q0.x - sp.x) * rc.x, tiy = (q0.y - sp.y) * rc.y, tiz = (q0.z - sp.z) * rc.z;
        const float tox = (q0.w - sp.x) * rc.x, toy = (q1.x - sp.y) * rc.y, toz = (q1.y - sp.z) * rc.z;
        const float tin = __builtin_fmaxf(tix, __builtin_fmaxf(tiy, tiz));
        const float tout = __builtin_fminf(tox, __builtin_fminf(toy, toz));
        return (tout >= 0.0f) && (tin <= tout) && (tin <= bound);
    };
    while (ia < n || ib < n) {
        int pa = -1, pb = -1;
        for (uint32_t s = 0; s < RT_WH_PAIR_STEPS; ++s) {
            const bool ga = ia < n && pa < 0, gb = ib < n && pb < 0;
            if (!(ga || gb)) break;
            // both node loads first (a finished ray reads node 0 of its ordering, discarded)
            const uint32_t ka = 2u * n * (oct & 7u) + 2u * (ga ? ia : 0u), kb = 2u * n * (oct >> 3) + 2u * (gb ? ib : 0u);
            const float4 a0 = wo[ka], a1 = wo[ka + 1], b0 = wo[kb], b1 = wo[kb + 1];
            if (ga) {
                if (COUNT) ++node_tests;
                const bool hit = slab(ra, a0, a1, bA);
                const int tri = f2i(a1.w);
                ia = (hit && tri < 0) ? ia + 1 : (uint32_t)f2i(a1.z);
                if (hit && tri >= 0) pa = tri;
            }
            if (gb) {
                if (COUNT) ++node_tests;
                const bool hit = slab(rb, b0, b1, bB);
                const int tri = f2i(b1.w);
                ib = (hit && tri < 0) ? ib + 1 : (uint32_t)f2i(b1.z);
                if (hit && tri >= 0) pb = tri;
            }
        }
        if (pa >= 0 && shadow_test(0, pa)) { occA = true; ia = n; }
        if (pb >= 0 && shadow_test(1, pb)) { occB = true; ib = n; }
    }
}

}  // namespace

// frame groups per block: an 8x8 tile per block, wave g rendering the frames k = g (mod 4) of it; the
// colors meet in LDS and wave 0 accumulates them in frame order (the reference's additions in its
// order).  Against one thread per pixel rendering every frame (16x16 tiles), the blocks are 4x as many
// at a quarter of the duration, so the last round of blocks leaves little of the chip idle, and a wave's
// rays come from an 8x8 tile instead of a 16x4 strip: C3 6151 -> 9759 Msamples/s, bitwise
// (profiles/r03/ab/ab_c3_whitted.json)
constexpr uint32_t WH_FG = 4;

// one frame of one pixel: Renderer::RayGen_Shader -> cast_Whitted_ray (BV/Renderer.cpp:109-233)
template <bool COUNT>
__device__ __forceinline__ V3 whitted_sample(const KParams& P, uint32_t lx, uint32_t y, float cam_x, uint32_t& node_tests, uint32_t& tri_tests, uint32_t& rays)
{
    // Camera::RecomputeRayDirections, BV/Camera.cpp:119-129: bottom-left corner of the pixel
    float cx = (float)lx / (float)P.W;
    float cy = (float)y / (float)P.H;
    cx = cx * 2.0f - 1.0f;
    cy = cy * 2.0f - 1.0f;
    float tg[4];
    mat4_mul(P.iproj, cx, cy, 1.0f, 1.0f, tg);
    const V3 dv = glm_normalize(divs(V3{tg[0], tg[1], tg[2]}, tg[3]));
    float wd[4];
    mat4_mul(P.iview, dv.x, dv.y, dv.z, 0.0f, wd);
    const V3 cam{cam_x, P.cam_pos[1], P.cam_pos[2]};
    const Ray ray = make_ray(cam, w_normalize(V3{wd[0], wd[1], wd[2]}));   // RayGen_Shader, BV/Renderer.cpp:113
    V3 color{P.sky[0], P.sky[1], P.sky[2]};
    double best = 1.7976931348623157e308;
    int best_tri = -1;
    bool occl = false;
    if (ray.d.x == 0.0f && ray.d.y == 0.0f && ray.d.z == 0.0f) {
        color = V3{0.0f, 0.0f, 0.0f};   // zero direction: no energy (BV/Renderer.cpp:123-126)
    } else {
        if (COUNT) ++rays;
        whitted_traverse<COUNT>(P, ray, false, 0.0, best, best_tri, occl, node_tests, tri_tests);
    }
    if (best_tri >= 0) {
        const float4 ta = P.tris[4 * best_tri], tn = P.tris[4 * best_tri + 3];
        const int mat = f2i(ta.w);
        const V3 x = add(ray.o, smul((float)best, ray.d));   // Ray::operator(), BV/Ray.h:34-37
        const V3 n{tn.x, tn.y, tn.z};
        const V3 off = muls(n, INTERSECTION_CORRECTION);
        const V3 sp = (dot(ray.d, n) < 0.0f) ? add(x, off) : sub(x, off);
        V3 diffuse{0.0f, 0.0f, 0.0f};
        uint32_t l = 0;
        if (RT_WH_PAIR && P.n_plights >= 2 && P.worders != nullptr) {
            // lights 0 and 1: their shadow rays walked together when every lane's pair has finite reciprocals
            // (wave-uniform: whitted_shadow_pair walks the near-first orderings only)
            auto ldir = [&](uint32_t k) {
                const float4 lp = P.plights[2 * k];
                return w_normalize(sub(V3{lp.x, lp.y, lp.z}, x));
            };
            const V3 l0 = ldir(0), l1 = ldir(1);
            const bool fin = rcp_finite(make_ray(sp, l0)) && rcp_finite(make_ray(sp, l1));
            if (__all(fin)) {
                // |dot(l, n)| of both lights now: the normal is not live across the walk
                const float c0 = __builtin_fabsf(dot(l0, n)), c1 = __builtin_fabsf(dot(l1, n));
                if (COUNT) rays += 2;
                bool o0, o1;
                whitted_shadow_pair<COUNT>(P, x, sp, o0, o1, node_tests, tri_tests);
                // the diffuse sum in light order (BV/Renderer.cpp:186-199)
                if (!o0) {
                    const float4 lr4 = P.plights[1];
                    diffuse = add(diffuse, V3{lr4.x * c0, lr4.y * c0, lr4.z * c0});
                }
                if (!o1) {
                    const float4 lr4 = P.plights[3];
                    diffuse = add(diffuse, V3{lr4.x * c1, lr4.y * c1, lr4.z * c1});
                }
                l = 2;
            }
        }
        for (; l < P.n_plights; ++l) {
            const float4 lp = P.plights[2 * l], lr4 = P.plights[2 * l + 1];
            V3 ld = sub(V3{lp.x, lp.y, lp.z}, x);
            const float d2 = dot(ld, ld);
            ld = w_normalize(ld);
            const Ray sray = make_ray(sp, ld);
            if (COUNT) ++rays;
            double sbest = 1.7976931348623157e308;
            int stri = -1;
            bool blocked = false;
            whitted_traverse<COUNT>(P, sray, true, (double)d2, sbest, stri, blocked, node_tests, tri_tests);
            if (blocked) continue;
            const float c = __builtin_fabsf(dot(ld, n));
            diffuse = add(diffuse, V3{lr4.x * c, lr4.y * c, lr4.z * c});
        }
        const float4 wm = P.wmats[mat];
        color = muls(mul(diffuse, V3{wm.x, wm.y, wm.z}), wm.w);
    }
    return color;
}

__device__ __forceinline__ void whitted_store(const KParams& P, uint32_t local, const float4 acc)
{
    const float fr = (float)(P.first_frame + P.n_frames - 1u);
    const float rx = smin(smax(acc.x / fr, 0.0f), 1.0f), gy = smin(smax(acc.y / fr, 0.0f), 1.0f);
    const float bz = smin(smax(acc.z / fr, 0.0f), 1.0f), aw = smin(smax(acc.w / fr, 0.0f), 1.0f);
    P.accum[local] = acc;
    P.rgba[local] = (to_u8(aw) << 24) | (to_u8(bz) << 16) | (to_u8(gy) << 8) | to_u8(rx);
}

#ifndef RT_WH_WAVES
#define RT_WH_WAVES 8   // waves per SIMD the register budget is sized for
#endif
template <bool COUNT>
__global__ void __launch_bounds__(256, RT_WH_WAVES) whitted_kernel(KParams P)
{
    uint32_t node_tests = 0, tri_tests = 0, rays = 0;
    constexpr uint32_t FG = WH_FG;
    static_assert(FG * 64 == 256, "one wave per frame group");
    __shared__ float4 col[2][FG][64];   // the step's colors, double-buffered (one barrier per step)
    const uint32_t tiles_x = (P.W + 7) / 8;
    const uint32_t tile = blockIdx.x;
    const uint32_t p = threadIdx.x & 63u, g = threadIdx.x >> 6;
    const uint32_t lr = (tile / tiles_x) * 8 + (p >> 3);
    const uint32_t lx = (tile % tiles_x) * 8 + (p & 7u);
    const bool valid = lr < P.n_local_rows && lx < P.W;
    const uint32_t band_k = lr / P.band, in_band = lr - band_k * P.band;
    const uint32_t y = (P.rank + band_k * P.nranks) * P.band + in_band;
    const uint32_t local = lr * P.W + lx;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g == 0 && valid && P.first_frame != 1u) acc = P.accum[local];
    float cam_x = P.cam_pos[0];
    const uint32_t nsteps = (P.n_frames + FG - 1u) / FG;
    for (uint32_t j = 0; j < nsteps; ++j) {
        // the reference evaluates every frame; keep the compiler from hoisting the frame's work
        asm volatile("" : "+v"(cam_x));
        const uint32_t k = j * FG + g;
        if (valid && k < P.n_frames) {
            const V3 c = whitted_sample<COUNT>(P, lx, y, cam_x, node_tests, tri_tests, rays);
            col[j & 1u][g][p] = make_float4(c.x, c.y, c.z, 0.0f);
        }
        __syncthreads();
        if (g == 0 && valid) {
            // frames j*FG .. j*FG+FG-1 in order (RayGen_Shader's accumulation)
            for (uint32_t u = 0; u < FG && j * FG + u < P.n_frames; ++u) {
                const float4 c = col[j & 1u][u][p];
                acc.x = acc.x + c.x; acc.y = acc.y + c.y; acc.z = acc.z + c.z; acc.w = acc.w + 1.0f;
            }
        }
        // buffer j & 1 is written again at step j + 2, after the barrier of step j + 1, which wave 0
        // reaches only when this chain is done
    }
    if (g == 0 && valid && P.n_frames > 0) whitted_store(P, local, acc);
    if (COUNT) {
        uint64_t a = node_tests, b = tri_tests, c = rays;
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_down(a, off); b += __shfl_down(b, off); c += __shfl_down(c, off);
        }
        if (__lane_id() == 0) {
            atomicAdd((unsigned long long*)&P.counters[0], (unsigned long long)a);
            atomicAdd((unsigned long long*)&P.counters[1], (unsigned long long)b);
            atomicAdd((unsigned long long*)&P.counters[2], (unsigned long long)c);
        }
    }
}

hipError_t rt_launch_whitted(const KParams& P, bool count, hipStream_t stream, uint32_t* grid_out)
{
    const uint32_t tiles = ((P.W + 7) / 8) * ((P.n_local_rows + 7) / 8);
    if (grid_out) *grid_out = tiles;
    if (tiles == 0) return hipSuccess;
    if (count) hipLaunchKernelGGL(whitted_kernel<true>, dim3(tiles), dim3(256), 0, stream, P);
    else hipLaunchKernelGGL(whitted_kernel<false>, dim3(tiles), dim3(256), 0, stream, P);
    return hipGetLastError();
}

// =============================================================================================
// The Whitted Style Ray Tracer's world (config C1; WH/ = "Whitted Style Ray Tracer/8599RayTracerGUI/src/"):
// spheres and textured triangle meshes intersected brute force in insertion order
// (get_intersection_payload, WH/Renderer.h:109-140), shaded by cast_Whitted_ray (WH/Renderer.h:184-310):
// Diffuse_Glossy ends the ray with two shadowed point lights (diffuse + Phong specular), Reflective and
// Reflective_Refractive recurse with Fresnel weights to depth 5.  The recursion is a per-lane explicit
// stack evaluated in the reference's post-order (reflected child, then refracted child, then the
// weighted sum), so every float operation happens in the reference's order.  One thread per pixel.
// =============================================================================================
namespace {

struct WHit { int ent; int tri; float t; float b2, b3; };

// QuadraticFormula, WH/WhittedUtilities.h:38-60 (the -0.5 literals are double)
__device__ __forceinline__ bool quadratic(float A, float B, float C, float& xs, float& xl)
{
    const float disc = B * B - 4.0f * A * C;
    if (disc < 0.0f) return false;
    if (disc == 0.0f) {
        xs = xl = (float)((-0.5 * (double)B) / (double)A);
    } else {
        const float sq = __builtin_sqrtf(disc);
        const float q = (float)((B > 0.0f) ? (-0.5 * (double)(B + sq)) : (-0.5 * (double)(B - sq)));
        xs = q / A;
        xl = C / q;
    }
    if (xs > xl) { const float t = xs; xs = xl; xl = t; }
    return true;
}

// Sphere::Intersect, WH/Sphere.h:26-59
__device__ __forceinline__ bool sphere_hit(const float4& c, float r2, const V3& o, const V3& d, float& t)
{
    const V3 oc = sub(o, V3{c.x, c.y, c.z});
    float ts, tl;
    if (!quadratic(dot(d, d), 2.0f * dot(d, oc), dot(oc, oc) - r2, ts, tl)) return false;
    if (ts < 0.0f) ts = tl;
    if (ts < 0.0f) return false;
    t = ts;
    return true;
}

// Whitted::RayTriangleIntersection (all float), WH/TriangleMesh.h:16-45
__device__ __forceinline__ bool tri_hit_f32(const V3& v1, const V3& v2, const V3& v3, const V3& o, const V3& d, float& t, float& b2, float& b3)
{
    const V3 E1 = sub(v2, v1), E2 = sub(v3, v1), S = sub(o, v1);
    const V3 S1 = cross(d, E2), S2 = cross(S, E1);
    const float den = dot(S1, E1);
    t = dot(S2, E2) / den;
    b2 = dot(S1, S) / den;
    b3 = dot(S2, d) / den;
    return (t > 0.0f) && (b2 > 0.0f) && (b3 > 0.0f) && (((1.0f - b2) - b3) > 0.0f);
}

// get_intersection_payload, WH/Renderer.h:109-140: entities in order, strict '<' (the first of equal
// t wins; inside a mesh, TriangleMesh::Intersect, WH/TriangleMesh.h:86-112, likewise)
__device__ __forceinline__ bool world_hit(const KParams& P, const V3& o, const V3& d, WHit& h)
{
    const float FMAX = 3.40282347e+38f;   // Whitted::positive_infinity
    float t_closest = FMAX;
    bool any = false;
    for (uint32_t e = 0; e < P.n_went; ++e) {
        const float4 q0 = P.went[4 * e], q1 = P.went[4 * e + 1], q2 = P.went[4 * e + 2];
        float t_local = FMAX;
        int tri = -1;
        float b2 = 0.0f, b3 = 0.0f;
        bool hit = false;
        if (f2i(q0.x) == RT_WORLD_SPHERE) {
            hit = sphere_hit(q1, q2.x, o, d, t_local);
        } else {
            const int first = f2i(q0.z), nt = f2i(q0.w);
            for (int k = 0; k < nt; ++k) {
                const float4 a = P.wtris[4 * (first + k)], b = P.wtris[4 * (first + k) + 1], c = P.wtris[4 * (first + k) + 2];
                float t, u, v;
                if (tri_hit_f32(V3{a.x, a.y, a.z}, V3{b.x, b.y, b.z}, V3{c.x, c.y, c.z}, o, d, t, u, v) && t < t_local) {
                    t_local = t; b2 = u; b3 = v; tri = first + k; hit = true;
                }
            }
        }
        if (hit && t_local < t_closest) {
            t_closest = t_local;
            h = WHit{(int)e, tri, t_local, b2, b3};
            any = true;
        }
    }
    return any;
}

// mirror_reflection_direction, WH/Renderer.h:41-45
__device__ __forceinline__ V3 mirror_dir(const V3& I, const V3& N) { return sub(I, smul(2.0f * dot(I, N), N)); }

__device__ __forceinline__ float clamp_float(float v, float lo, float hi) { return smax(smin(v, hi), lo); }   // WH/WhittedUtilities.h:33-36

// snell_refraction_direction, WH/Renderer.h:47-76
__device__ __forceinline__ V3 snell_dir(const V3& I, const V3& N, float eta)
{
    float eta_in = 1.0f, eta_out = eta;
    V3 normal = N;
    float ci = clamp_float(dot(I, N), -1.0f, 1.0f);
    if (ci < 0.0f) ci = -ci;
    else { const float t = eta_in; eta_in = eta_out; eta_out = t; normal = neg(normal); }
    const float er = eta_in / eta_out;
    const float k = 1.0f - er * er * (1.0f - ci * ci);
    return (k < 0.0f) ? V3{0.0f, 0.0f, 0.0f} : add(smul(er, I), smul(er * ci - __builtin_sqrtf(k), normal));
}

// accurate_fresnel_reflectance, WH/Renderer.h:78-107
__device__ __forceinline__ float fresnel(const V3& I, const V3& N, float eta)
{
    float eta_in = 1.0f, eta_out = eta;
    float ci = clamp_float(dot(I, N), -1.0f, 1.0f);
    if (ci < 0.0f) ci = -ci;
    else { const float t = eta_in; eta_in = eta_out; eta_out = t; }
    const float st = eta_in / eta_out * __builtin_sqrtf(smax(0.0f, 1.0f - ci * ci));
    if (st > 1.0f) return 1.0f;
    const float ct = __builtin_sqrtf(smax(0.0f, 1.0f - st * st));
    const float rs = (eta_in * ci - eta_out * ct) / (eta_in * ci + eta_out * ct);
    const float rp = (eta_in * ct - eta_out * ci) / (eta_in * ct + eta_out * ci);
    return (rs * rs + rp * rp) / 2.0f;
}

// TriangleMesh::GetDiffuseColor (the chessboard texture), WH/TriangleMesh.h:79-84; fmodf(v, 1) of a
// finite v is v - trunc(v), exactly
__device__ __forceinline__ V3 checker(float u, float v)
{
    const float a = u * 5.0f, b = v * 5.0f;
    const float fa = a - __builtin_truncf(a), fb = b - __builtin_truncf(b);
    const float pattern = ((fa > 0.5f) != (fb > 0.5f)) ? 1.0f : 0.0f;
    const V3 c0{(float)0.815, (float)0.235, (float)0.031}, c1{(float)0.937, (float)0.937, (float)0.231};
    return add(muls(c0, 1.0f - pattern), muls(c1, pattern));   // Whitted::lerp, WH/VectorFloat.h:16-19
}

struct WFrame {
    V3 o, d;
    int depth, stage;   // stage 0: trace; 1: reflected child done; 2: refracted child done; 3: mirror child done
    float R;
    V3 acc, to, td;
};
constexpr int kWorldFrames = 8;

template <bool COUNT>
__device__ V3 cast_whitted_world(const KParams& P, const V3& o0, const V3& d0, uint32_t& rays)
{
    WFrame st[kWorldFrames];
    int sp = 0;
    st[0].o = o0; st[0].d = d0; st[0].depth = 0; st[0].stage = 0;
    sp = 1;
    V3 ret{0.0f, 0.0f, 0.0f};
    const float eps = P.intersection_correction;
    while (sp > 0) {
        WFrame& F = st[sp - 1];
        if (F.stage == 0) {
            if (F.depth > P.max_bounce_depth || (F.d.x == 0.0f && F.d.y == 0.0f && F.d.z == 0.0f)) {
                ret = V3{0.0f, 0.0f, 0.0f};   // no energy received
                --sp;
                continue;
            }
            if (COUNT) ++rays;
            WHit h;
            if (!world_hit(P, F.o, F.d, h)) {
                ret = V3{P.sky[0], P.sky[1], P.sky[2]};
                --sp;
                continue;
            }
            const float4 e0 = P.went[4 * h.ent], e1 = P.went[4 * h.ent + 1], e2 = P.went[4 * h.ent + 2], e3 = P.went[4 * h.ent + 3];
            const V3 x = add(F.o, muls(F.d, h.t));
            V3 n;
            float tu = 0.0f, tv = 0.0f;
            if (f2i(e0.x) == RT_WORLD_SPHERE) {
                n = w_normalize(sub(x, V3{e1.x, e1.y, e1.z}));   // Sphere::GetHitInfo, WH/Sphere.h:61-72
            } else {
                // TriangleMesh::GetHitInfo, WH/TriangleMesh.h:114-136
                const float4 a = P.wtris[4 * h.tri], b = P.wtris[4 * h.tri + 1], c = P.wtris[4 * h.tri + 2], u = P.wtris[4 * h.tri + 3];
                const V3 v1{a.x, a.y, a.z}, v2{b.x, b.y, b.z}, v3{c.x, c.y, c.z};
                n = w_normalize(cross(w_normalize(sub(v2, v1)), w_normalize(sub(v3, v2))));
                const float s = (1.0f - h.b2) - h.b3;
                tu = (s * a.w + h.b2 * c.w) + h.b3 * u.y;
                tv = (s * b.w + h.b2 * u.x) + h.b3 * u.z;
            }
            const int nature = f2i(e0.y);
            const float eta = e2.y;
            if (nature == 0 || nature == 1) {
                const V3 rd = w_normalize(mirror_dir(F.d, n));
                const V3 ro = (dot(rd, n) < 0.0f) ? sub(x, muls(n, eps)) : add(x, muls(n, eps));
                if (nature == 0) {
                    F.R = fresnel(neg(rd), n, eta);
                    F.stage = 3;
                } else {
                    F.td = w_normalize(snell_dir(F.d, n, eta));
                    F.to = (dot(F.td, n) < 0.0f) ? sub(x, muls(n, eps)) : add(x, muls(n, eps));
                    F.R = fresnel(F.d, n, eta);
                    F.stage = 1;
                }
                WFrame& C = st[sp];
                C.o = ro; C.d = rd; C.depth = F.depth + 1; C.stage = 0;
                ++sp;
                continue;
            }
            // Diffuse_Glossy (WH/Renderer.h:261-305)
            V3 diff{0.0f, 0.0f, 0.0f}, spec{0.0f, 0.0f, 0.0f};
            const V3 spt = (dot(F.d, n) < 0.0f) ? add(x, muls(n, eps)) : sub(x, muls(n, eps));
            for (uint32_t l = 0; l < P.n_plights; ++l) {
                const float4 lp = P.plights[2 * l], lr4 = P.plights[2 * l + 1];
                V3 ld = sub(V3{lp.x, lp.y, lp.z}, x);
                const float d2 = dot(ld, ld);
                ld = w_normalize(ld);
                if (COUNT) ++rays;
                WHit oh;
                if (world_hit(P, spt, ld, oh) && (oh.t * oh.t < d2)) continue;
                const V3 rad{lr4.x, lr4.y, lr4.z};
                diff = add(diff, muls(rad, __builtin_fabsf(dot(ld, n))));
                const float lobe = pow_lobe(smax(0.0f, -dot(mirror_dir(neg(ld), n), F.d)), e3.w);
                spec = add(spec, smul(lobe, rad));
            }
            const V3 dc = (f2i(e0.x) == RT_WORLD_SPHERE) ? V3{e3.x, e3.y, e3.z} : checker(tu, tv);
            ret = add(muls(mul(diff, dc), e2.z), muls(spec, e2.w));
            --sp;
        } else if (F.stage == 1) {
            // the reflected color is in; trace the refracted ray
            F.acc = ret;
            F.stage = 2;
            WFrame& C = st[sp];
            C.o = F.to; C.d = F.td; C.depth = F.depth + 1; C.stage = 0;
            ++sp;
        } else if (F.stage == 2) {
            ret = add(smul(F.R, F.acc), smul(1.0f - F.R, ret));   // reflectance * reflected + (1 - reflectance) * refracted
            --sp;
        } else {
            ret = muls(ret, F.R);   // cast_Whitted_ray(reflected) * fresnel
            --sp;
        }
    }
    return ret;
}

}  // namespace

template <bool COUNT>
__global__ void __launch_bounds__(256) whitted_world_kernel(KParams P)
{
    const uint32_t tiles_x = (P.W + 15) / 16;
    const uint32_t tile = blockIdx.x;
    const uint32_t lr = (tile / tiles_x) * 16 + (threadIdx.x >> 4);
    const uint32_t lx = (tile % tiles_x) * 16 + (threadIdx.x & 15);
    uint32_t rays = 0;
    if (lr < P.n_local_rows && lx < P.W) {
        const uint32_t band_k = lr / P.band, in_band = lr - band_k * P.band;
        const uint32_t y = (P.rank + band_k * P.nranks) * P.band + in_band;
        const uint32_t local = lr * P.W + lx;
        float4 acc = (P.first_frame == 1u) ? make_float4(0.f, 0.f, 0.f, 0.f) : P.accum[local];
        float cam_x = P.cam_pos[0];
        for (uint32_t k = 0; k < P.n_frames; ++k) {
            asm volatile("" : "+v"(cam_x));   // every frame is evaluated, as the reference does
            // Camera::RecomputeRayDirections, WH/Camera.cpp:114-132: bottom-left corner of the pixel
            float cx = (float)lx / (float)P.W;
            float cy = (float)y / (float)P.H;
            cx = cx * 2.0f - 1.0f;
            cy = cy * 2.0f - 1.0f;
            float tg[4];
            mat4_mul(P.iproj, cx, cy, 1.0f, 1.0f, tg);
            const V3 dv = glm_normalize(divs(V3{tg[0], tg[1], tg[2]}, tg[3]));
            float wd[4];
            mat4_mul(P.iview, dv.x, dv.y, dv.z, 0.0f, wd);
            const V3 cam{cam_x, P.cam_pos[1], P.cam_pos[2]};
            // RayGen_Shader, WH/Renderer.cpp:116-125
            const V3 color = cast_whitted_world<COUNT>(P, cam, w_normalize(V3{wd[0], wd[1], wd[2]}), rays);
            acc.x = acc.x + color.x; acc.y = acc.y + color.y; acc.z = acc.z + color.z; acc.w = acc.w + 1.0f;
        }
        if (P.n_frames > 0) {
            const float fr = (float)(P.first_frame + P.n_frames - 1u);
            const float rx = smin(smax(acc.x / fr, 0.0f), 1.0f), gy = smin(smax(acc.y / fr, 0.0f), 1.0f);
            const float bz = smin(smax(acc.z / fr, 0.0f), 1.0f), aw = smin(smax(acc.w / fr, 0.0f), 1.0f);
            P.accum[local] = acc;
            P.rgba[local] = (to_u8(aw) << 24) | (to_u8(bz) << 16) | (to_u8(gy) << 8) | to_u8(rx);
        }
    }
    if (COUNT) {
        uint64_t c = rays;
        for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off);
        if (__lane_id() == 0) atomicAdd((unsigned long long*)&P.counters[2], (unsigned long long)c);
    }
}

hipError_t rt_launch_whitted_world(const KParams& P, bool count, hipStream_t stream, uint32_t* grid_out)
{
    // one block per 16x16 tile, whitted_world_kernel's blockIdx -> tile mapping
    const uint32_t tiles = ((P.W + 15) / 16) * ((P.n_local_rows + 15) / 16);
    if (grid_out) *grid_out = tiles;
    if (tiles == 0) return hipSuccess;
    if (P.max_bounce_depth + 2 > kWorldFrames) return hipErrorInvalidValue;   // the explicit stack bounds the recursion
    if (count) hipLaunchKernelGGL(whitted_world_kernel<true>, dim3(tiles), dim3(256), 0, stream, P);
    else hipLaunchKernelGGL(whitted_world_kernel<false>, dim3(tiles), dim3(256), 0, stream, P);
    return hipGetLastError();
}

// closest hit of n rays against the world (unit-test entry point: rt_world_trace)
__global__ void __launch_bounds__(256) world_trace_kernel(KParams P, uint32_t n, const float* __restrict__ org, const float* __restrict__ dir,
                                                          int32_t* __restrict__ ent, int32_t* __restrict__ tri, float* __restrict__ tb)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    WHit h;
    const bool hit = world_hit(P, V3{org[3 * i], org[3 * i + 1], org[3 * i + 2]}, V3{dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]}, h);
    ent[i] = hit ? h.ent : -1;
    tri[i] = hit ? h.tri : -1;
    tb[3 * i] = hit ? h.t : 0.0f;
    tb[3 * i + 1] = hit && h.tri >= 0 ? h.b2 : 0.0f;
    tb[3 * i + 2] = hit && h.tri >= 0 ? h.b3 : 0.0f;
}

hipError_t rt_launch_world_trace(const KParams& P, uint32_t n, const float* org, const float* dir, int32_t* ent, int32_t* tri, float* tb,
                                 hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(world_trace_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, P, n, org, dir, ent, tri, tb);
    return hipGetLastError();
}
