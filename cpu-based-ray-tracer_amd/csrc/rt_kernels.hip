// rt_kernels.hip -- the MI355X path-tracing megakernel (gfx950 / CDNA4, wave64).
//
// One persistent launch renders `n_frames` samples of every pixel assigned to this device:
//   * lane-level work queue: a lane that finishes all frames of its pixel fetches the next pixel
//     from a device atomic (one atomic per wave per refill: __ballot + mbcnt compaction), so the
//     wave stays full until the queue drains; pixel order is 8x8-tile swizzled for ray coherence;
//   * per-pixel frames run in order inside the lane (accum += L per frame exactly like
//     Renderer::RayGen_Shader, MC/Renderer.cpp:124-134), so the float accumulation is the
//     reference's, bit for bit;
//   * path regeneration: each loop iteration advances every lane by one ray segment (camera ray,
//     or one bounce = closest hit + light sample + shadow ray + Russian roulette); a lane whose path
//     ended starts its next frame immediately;
//   * the recursion of Renderer::shading (MC/Renderer.cpp:148-214) is made iterative: each bounce's
//     (direct radiance, cosine, material) is pushed to a per-lane stack in HBM and folded back in
//     the reference's inner-first order when the path ends (EXACT mode), or accumulated forward
//     (FAST mode: one rounding difference per bounce);
//   * BVH traversal is stackless: nodes are in DFS pre-order with skip links (rt_layout.h), so a
//     closest-hit walk tests exactly the boxes/triangles the reference's recursion tests
//     (BVH::traverse_BVH_from_node, MC/BVH.h:82-101, ties to the later leaf); shadow rays are
//     any-hit with early exit, which is exact because the reference's visibility predicate
//     `length(q-p) < t_closest + 0.01f` (MC/Renderer.cpp:184) is monotone in t.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernels.h"

using namespace rtd;

namespace {


struct Hit {
    double t;
    int tri;
};

template <bool COUNT>
__device__ __forceinline__ Hit closest_hit(const KParams& P, const Ray& r, uint32_t& node_tests, uint32_t& tri_tests)
{
    double best = 1.7976931348623157e308;   // DBL_MAX (IntersectionRecord default, MC/IntersectionRecord.h:20-28)
    int best_tri = -1;
    const float4* __restrict__ nodes = P.nodes;
    const float4* __restrict__ tris = P.tris;
    uint32_t i = 0;
    const uint32_t n = P.n_nodes;
    while (i < n) {
        const float4 q0 = nodes[2 * i];
        const float4 q1 = nodes[2 * i + 1];
        if (COUNT) ++node_tests;
        const uint32_t skip = (uint32_t)f2i(q1.z);
        if (slab_hit(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y)) {
            const int tri = f2i(q1.w);
            if (tri >= 0) {
                if (COUNT) ++tri_tests;
                const float4 t0 = tris[4 * tri], t1 = tris[4 * tri + 1], t2 = tris[4 * tri + 2];
                double t;
                // (left.t < right.t) ? left : right  ==> the later leaf wins ties (t <= best)
                if (moller_trumbore(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, r, t) && t <= best) {
                    best = t; best_tri = tri;
                }
                i = skip;
            } else {
                i = i + 1;
            }
        } else {
            i = skip;
        }
    }
    return Hit{best, best_tri};
}

// occluded iff some hit t_i has !(len < t_i + 0.01f)  (MC/Renderer.cpp:184, evaluated in double)
template <bool COUNT>
__device__ __forceinline__ bool occluded(const KParams& P, const Ray& r, double len, uint32_t& node_tests, uint32_t& tri_tests)
{
    const float4* __restrict__ nodes = P.nodes;
    const float4* __restrict__ tris = P.tris;
    uint32_t i = 0;
    const uint32_t n = P.n_nodes;
    while (i < n) {
        const float4 q0 = nodes[2 * i];
        const float4 q1 = nodes[2 * i + 1];
        if (COUNT) ++node_tests;
        const uint32_t skip = (uint32_t)f2i(q1.z);
        if (slab_hit(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y)) {
            const int tri = f2i(q1.w);
            if (tri >= 0) {
                if (COUNT) ++tri_tests;
                const float4 t0 = tris[4 * tri], t1 = tris[4 * tri + 1], t2 = tris[4 * tri + 2];
                double t;
                if (moller_trumbore(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, r, t)) {
                    if (!(len < t + (double)0.01f)) return true;
                }
                i = skip;
            } else {
                i = i + 1;
            }
        } else {
            i = skip;
        }
    }
    return false;
}

// SamplingAreaLight -> TriangleMesh::Sampling -> BVH::Sampling_from_root/_node -> TrianglePrimitive::Sampling
// (MC/Renderer.h:163-180, MC/TriangleMesh.h:193-197, MC/BVH.h:103-129, MC/TriangleMesh.h:69-89)
__device__ __forceinline__ void sample_light(const KParams& P, Rng& g, V3& q, V3& nl)
{
    const float u0 = g.next();
    float p = u0 * P.light_area;
    int node = 0;
    for (;;) {
        const float4 ln = P.lnodes[node];
        const int left = f2i(ln.y);
        if (left < 0) break;
        const float la = P.lnodes[left].x;
        if (p < la) node = left;
        else { p = p - la; node = f2i(ln.z); }
    }
    const int lt = f2i(P.lnodes[node].w);
    const float4 A = P.ltris[4 * lt], B = P.ltris[4 * lt + 1], C = P.ltris[4 * lt + 2], N = P.ltris[4 * lt + 3];
    const float x = 1.0f - __builtin_sqrtf(g.next());
    const float y = g.next();
    const V3 a{A.x, A.y, A.z}, b{B.x, B.y, B.z}, c{C.x, C.y, C.z};
    q = add(add(smul(x, a), smul((1.0f - x) * y, b)), smul((1.0f - x) * (1.0f - y), c));
    nl = V3{N.x, N.y, N.z};
}

// WhittedMaterial::Sampling, MC/WhittedMaterial.h:71-117
__device__ __forceinline__ V3 sample_hemisphere(V3 n, Rng& g)
{
    const float z = g.next();
    const float rxy = __builtin_sqrtf(1.0f - z * z);
    const float phi = 2.0f * PI_F * g.next();
    const float x = rxy * cos_f(phi);
    const float y = rxy * sin_f(phi);
    V3 Y;
    if (__builtin_fabsf(n.x) > __builtin_fabsf(n.y)) Y = glm_normalize(V3{n.z, 0.0f, -(n.x)});
    else Y = glm_normalize(V3{0.0f, n.z, -(n.y)});
    const V3 X = cross(Y, n);
    return add(add(smul(x, X), smul(y, Y)), smul(z, n));
}

__device__ __forceinline__ uint32_t to_u8(float v)
{   // (uint8_t)(c * 255.0f), MC/Renderer.cpp:17-20 (v in [0,1] after clamp; NaN -> 0 like x86 cvttss2si)
    const float f = v * 255.0f;
    if (!(f == f)) return 0u;
    return ((uint32_t)(int32_t)f) & 0xFFu;
}

__device__ __forceinline__ uint32_t wave_lane() { return __lane_id(); }

}  // namespace

template <bool EXACT, bool COUNT>
__global__ void __launch_bounds__(256) pt_megakernel(KParams P)
{
    const uint32_t lane = wave_lane();
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const float PDF = 1.0f / (2.0f * PI_F);   // WhittedMaterial::PDF_at_the_sample, MC/WhittedMaterial.h:44-56
    const float rr = P.rr;
    const V3 cam{P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]};

    uint32_t node_tests = 0, tri_tests = 0, rays = 0;
    bool alive = true, have_pixel = false, in_path = false;
    uint32_t local = 0, px = 0, x = 0, y = 0, k = 0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    Rng g;
    Ray ray;
    uint32_t depth = 0;
    // pending level (direct radiance of the current bounce, waiting to know whether the indirect ray
    // continues the path)
    V3 pend_ld{0, 0, 0}; float pend_cos = 0.0f; int pend_mat = 0;
    V3 thr{1.0f, 1.0f, 1.0f}, Lsum{0, 0, 0};   // FAST mode

    for (;;) {
        // ---------------- lane-level work queue (wave-collective)
        const bool need = alive && !have_pixel;
        const uint64_t mask = __ballot(need);
        if (mask == 0 && !__any(alive)) break;
        if (mask != 0) {
            uint32_t base = 0;
            const int leader = __ffsll((unsigned long long)mask) - 1;
            if ((int)lane == leader) base = atomicAdd(P.work_counter, (uint32_t)__popcll(mask));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t rank_in = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
                const uint32_t w = base + rank_in;
                if (w >= P.n_items) {
                    alive = false;
                } else {
                    // 8x8 tile swizzle in local (row, column) space
                    const uint32_t tile = w >> 6, within = w & 63u;
                    const uint32_t trow = tile / P.tiles_x, tcol = tile - trow * P.tiles_x;
                    const uint32_t lr = trow * 8u + (within >> 3), lx = tcol * 8u + (within & 7u);
                    if (lr < P.n_local_rows && lx < P.W) {
                        // local row -> global row (row bands dealt round-robin over ranks)
                        const uint32_t band_k = lr / P.band, in_band = lr - band_k * P.band;
                        y = (P.rank + band_k * P.nranks) * P.band + in_band;
                        x = lx;
                        local = lr * P.W + lx;
                        px = y * P.W + x;
                        have_pixel = true;
                        k = 0;
                        acc = (P.first_frame == 1u) ? make_float4(0.f, 0.f, 0.f, 0.f) : P.accum[local];
                    }
                }
            }
        }
        if (!have_pixel) continue;

        // ---------------- start a new sample: camera ray (MC/Camera.cpp:119-125 + MC/Renderer.cpp:128)
        if (!in_path) {
            const uint32_t frame = P.first_frame + k;
            g.start(P.seed, px, frame);
            const float ux = g.next();
            const float uy = g.next();
            float cx = ((float)x + ux) / (float)P.W;
            float cy = ((float)y + uy) / (float)P.H;
            cx = cx * 2.0f - 1.0f;
            cy = cy * 2.0f - 1.0f;
            float tg[4];
            mat4_mul(P.iproj, cx, cy, 1.0f, 1.0f, tg);
            const V3 dv = glm_normalize(divs(V3{tg[0], tg[1], tg[2]}, tg[3]));
            float wd[4];
            mat4_mul(P.iview, dv.x, dv.y, dv.z, 0.0f, wd);
            ray = make_ray(cam, w_normalize(V3{wd[0], wd[1], wd[2]}));
            depth = 0;
            in_path = true;
            if (!EXACT) { thr = V3{1.0f, 1.0f, 1.0f}; Lsum = V3{0, 0, 0}; }
        }

        // ---------------- one ray segment
        if (COUNT) ++rays;
        const Hit h = closest_hit<COUNT>(P, ray, node_tests, tri_tests);
        bool finished = false;
        int fold_top = -1;   // EXACT: stack levels fold_top..0 are folded into L when the path ends
        V3 L{0, 0, 0};
        int mat = 0;
        float4 tq3 = make_float4(0.f, 0.f, 0.f, 0.f);
        bool emissive = false;
        if (h.tri >= 0) {
            mat = f2i(P.tris[4 * h.tri].w);
            tq3 = P.tris[4 * h.tri + 3];
            emissive = P.mats[2 * mat].w != 0.0f;
        }
        if (depth == 0) {
            if (h.tri < 0) {   // cast_path miss: night sky (MC/Renderer.cpp:145)
                L = V3{12 / 255.0f, 20 / 255.0f, 69 / 255.0f};
                finished = true;
            } else if (emissive) {   // shading: direct emission (MC/Renderer.cpp:151-161)
                const float4 em = P.mats[2 * mat + 1];
                L = V3{em.x, em.y, em.z};
                finished = true;
            }
        } else if (h.tri < 0 || emissive) {
            // the indirect ray missed or hit the light: radiance_indirect = 0 (MC/Renderer.cpp:202);
            // the pending level's radiance is its direct term
            L = EXACT ? pend_ld : Lsum;
            fold_top = (int)depth - 2;
            finished = true;
        } else if (EXACT) {
            // the pending level recurses into this hit: push it as stack level depth-1
            const uint32_t lvl = depth - 1;
            if (lvl < P.stack_depth) {
                P.stack_ld[(size_t)lvl * P.total_threads + gtid] = make_float4(pend_ld.x, pend_ld.y, pend_ld.z, pend_cos);
                P.stack_mat[(size_t)lvl * P.total_threads + gtid] = pend_mat;
            } else {
                atomicAdd((unsigned long long*)&P.counters[3], 1ull);   // reported as stack overflow
            }
        }

        if (!finished) {
            // ------------ shading at the hit (MC/Renderer.cpp:163-214)
            const V3 wo = neg(ray.d);
            const V3 loc = add(ray.o, smul((float)h.t, ray.d));   // Ray::operator(), MC/Ray.h:34-37
            const V3 N{tq3.x, tq3.y, tq3.z};
            const V3 n = (dot(N, wo) < 0.0f) ? neg(N) : N;
            const V3 p = add(loc, muls(n, INTERSECTION_CORRECTION));
            const float4 mb = P.mats[2 * mat];
            const V3 brdf_m{mb.x, mb.y, mb.z};
            V3 ld{0.0f, 0.0f, 0.0f};
            if (P.has_light) {
                V3 q, nl0;
                sample_light(P, g, q, nl0);
                const V3 p2q = sub(q, p);
                const V3 wl = glm_normalize(p2q);
                const V3 nl = (dot(nl0, neg(wl)) < 0.0f) ? neg(nl0) : nl0;
                if (COUNT) ++rays;
                const Ray sr = make_ray(p, wl);
                if (!occluded<COUNT>(P, sr, (double)glm_length(p2q), node_tests, tri_tests)) {
                    const float c1 = dot(wl, n);
                    const V3 f = (c1 >= 0.0f) ? brdf_m : V3{0.0f, 0.0f, 0.0f};   // WhittedMaterial::BRDF :58-69
                    const V3 E{P.light_emission[0], P.light_emission[1], P.light_emission[2]};
                    const float lpdf = 1.0f / P.light_area;                       // BVH::Sampling_from_root :106
                    ld = divs(divs(muls(muls(mul(E, f), c1), dot(neg(wl), nl)), dot(p2q, p2q)), lpdf);
                }
            }
            // Russian roulette (MC/Renderer.cpp:193); the depth cap only bounds the loop
            // (P(depth > 4096) = rr^4096, i.e. 0 for rr <= 0.99)
            if (g.next() < rr && depth < 4096u) {
                const V3 wi = glm_normalize(sample_hemisphere(n, g));
                const float c = dot(wi, n);
                if (EXACT) {
                    pend_ld = ld; pend_cos = c; pend_mat = mat;
                } else {
                    Lsum = add(Lsum, mul(thr, ld));
                    const V3 f = (c >= 0.0f) ? brdf_m : V3{0.0f, 0.0f, 0.0f};
                    thr = muls(mul(thr, f), c / PDF / rr);
                }
                ray = make_ray(p, wi);
                depth = depth + 1;
            } else {
                if (EXACT) L = ld;
                else { Lsum = add(Lsum, mul(thr, ld)); L = Lsum; }
                fold_top = (int)depth - 1;
                finished = true;
            }
        }

        if (finished) {
            if (EXACT) {
                // fold inner-first: L = Ld_k + ((((L * brdf_k) * cos_k) / PDF) / RR)   (MC/Renderer.cpp:208,213)
                for (int lvl = fold_top; lvl >= 0; --lvl) {
                    float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
                    int m = 0;
                    if ((uint32_t)lvl < P.stack_depth) {
                        e = P.stack_ld[(size_t)lvl * P.total_threads + gtid];
                        m = P.stack_mat[(size_t)lvl * P.total_threads + gtid];
                    }
                    const float4 mb2 = P.mats[2 * m];
                    const V3 f = (e.w >= 0.0f) ? V3{mb2.x, mb2.y, mb2.z} : V3{0.0f, 0.0f, 0.0f};
                    L = add(V3{e.x, e.y, e.z}, divs(divs(muls(mul(L, f), e.w), PDF), rr));
                }
            }
            // temporal accumulation + clamp + pack (MC/Renderer.cpp:128-133)
            acc.x = acc.x + L.x; acc.y = acc.y + L.y; acc.z = acc.z + L.z; acc.w = acc.w + 1.0f;
            in_path = false;
            ++k;
            if (k == P.n_frames) {
                const float fr = (float)(P.first_frame + k - 1u);
                const float rx = smin(smax(acc.x / fr, 0.0f), 1.0f), gy = smin(smax(acc.y / fr, 0.0f), 1.0f);
                const float bz = smin(smax(acc.z / fr, 0.0f), 1.0f), aw = smin(smax(acc.w / fr, 0.0f), 1.0f);
                P.accum[local] = acc;
                P.rgba[local] = (to_u8(aw) << 24) | (to_u8(bz) << 16) | (to_u8(gy) << 8) | to_u8(rx);
                have_pixel = false;
            }
        }
    }

    if (COUNT) {
        // wave-reduce, one atomic per wave
        uint64_t a = node_tests, b = tri_tests, c = rays;
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_down(a, off); b += __shfl_down(b, off); c += __shfl_down(c, off);
        }
        if (lane == 0) {
            atomicAdd((unsigned long long*)&P.counters[0], (unsigned long long)a);
            atomicAdd((unsigned long long*)&P.counters[1], (unsigned long long)b);
            atomicAdd((unsigned long long*)&P.counters[2], (unsigned long long)c);
        }
    }
}

// explicit instantiations + launchers (C linkage inside rt_capi.cpp)
template __global__ void pt_megakernel<true, false>(KParams);
template __global__ void pt_megakernel<true, true>(KParams);
template __global__ void pt_megakernel<false, false>(KParams);
template __global__ void pt_megakernel<false, true>(KParams);

hipError_t rt_launch_megakernel(const KParams& P, bool exact, bool count, uint32_t grid, uint32_t block, hipStream_t stream)
{
    if (exact && count) hipLaunchKernelGGL((pt_megakernel<true, true>), dim3(grid), dim3(block), 0, stream, P);
    else if (exact) hipLaunchKernelGGL((pt_megakernel<true, false>), dim3(grid), dim3(block), 0, stream, P);
    else if (count) hipLaunchKernelGGL((pt_megakernel<false, true>), dim3(grid), dim3(block), 0, stream, P);
    else hipLaunchKernelGGL((pt_megakernel<false, false>), dim3(grid), dim3(block), 0, stream, P);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// closest-hit query kernel (unit-test entry point of the C-ABI: rt_trace)
__global__ void __launch_bounds__(256) trace_kernel(KParams P, uint32_t n, const float* __restrict__ org, const float* __restrict__ dir,
                                                    int32_t* __restrict__ tri_out, double* __restrict__ t_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Ray r = make_ray(V3{org[3 * i], org[3 * i + 1], org[3 * i + 2]}, V3{dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]});
    uint32_t a = 0, b = 0;
    const Hit h = closest_hit<false>(P, r, a, b);
    tri_out[i] = h.tri;
    t_out[i] = h.tri >= 0 ? h.t : 1.7976931348623157e308;
}

hipError_t rt_launch_trace(const KParams& P, uint32_t n, const float* org, const float* dir, int32_t* tri, double* t, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(trace_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, P, n, org, dir, tri, t);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// math self-test kernel: device f32 sqrt/div, f64 reciprocal, cos/sin as the megakernel evaluates them
__global__ void math_kernel(uint32_t n, const float* __restrict__ x, float* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    out[6 * i + 0] = __builtin_sqrtf(v);
    out[6 * i + 1] = 1.0f / v;
    out[6 * i + 2] = cos_f(v);
    out[6 * i + 3] = sin_f(v);
    const double r = 1.0 / (double)v;
    out[6 * i + 4] = __int_as_float((int)(uint32_t)(__double_as_longlong(r) & 0xFFFFFFFFull));
    out[6 * i + 5] = __int_as_float((int)(uint32_t)((unsigned long long)__double_as_longlong(r) >> 32));
}

hipError_t rt_launch_math(uint32_t n, const float* x, float* out, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(math_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n, x, out);
    return hipGetLastError();
}

int rt_megakernel_occupancy(bool exact, bool count, int block)
{
    int n = 0;
    hipError_t e;
    if (exact && count) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_megakernel<true, true>, block, 0);
    else if (exact) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_megakernel<true, false>, block, 0);
    else if (count) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_megakernel<false, true>, block, 0);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pt_megakernel<false, false>, block, 0);
    return e == hipSuccess ? n : 0;
}
