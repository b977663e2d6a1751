// rt_path.h -- device helpers shared by the path-tracing kernels (rt_kernels.hip: the general
// megakernel; rt_coherent.hip: the vertex-synchronous kernel for small scenes): the lane's random
// stream, kernel-parameter access, the stackless BVH walk, light and hemisphere sampling.
#ifndef RT_PATH_H
#define RT_PATH_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernels.h"

namespace rtd {

// Uniform draws of the lane's current sample: Walnut::Random::Float's formula (WN/Random.h:27-30) on
// the Philox stream of (pixel, frame) (rt_device.h), the block of 4 draws buffered in LDS
struct LaneRng {
    uint32_t* buf;              // the lane's LS_RNG words (stride 256)
    uint32_t k0, k1;            // key (uniform)
    uint32_t pixel, frame, dim, blk;
    __device__ __forceinline__ void start(uint32_t px, uint32_t fr) { pixel = px; frame = fr; dim = 0; blk = 0xFFFFFFFFu; }
    __device__ __forceinline__ float next()
    {
        const uint32_t want = dim >> 2;
        if (want != blk) {
            uint32_t o[4];
            philox4x32_10(pixel, frame, want, 0u, k0, k1, o);
            buf[0] = o[0]; buf[256] = o[1]; buf[512] = o[2]; buf[768] = o[3];
            blk = want;
        }
        const uint32_t u = buf[(dim & 3u) * 256u];
        ++dim;
        return (float)u / 4294967296.0f;   // (float)UINT32_MAX == 2^32 exactly
    }
};

// The kernel's parameters re-read from the kernarg segment where a section uses them: the empty asm
// keeps the compiler from hoisting the scalar loads to the kernel entry, where ~100 long-lived uniforms
// overflow the SGPRs into VGPR lanes and cost the kernel a wave per SIMD.
__device__ __forceinline__ const KParams& kargs()
{
    const KParams* kp = (const KParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *kp;
}
// The same, keeping the constant address space: members are read with scalar loads into SGPRs
// (the generic-pointer form above reads them with flat loads into VGPRs).
typedef const __attribute__((address_space(4))) KParams CKParams;
__device__ __forceinline__ CKParams& kargs4()
{
    CKParams* kp = (CKParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *kp;
}

struct SceneView {
    const float4* nodes;
    const float4* tris;
    const float4* mats;
    const float4* lnodes;
    const float4* ltris;
    uint32_t n_nodes;
    const float4* lboxes;   // small scenes: distinct leaf boxes (rt_layout.h), else unused
};

// A leaf's primitive: Moller-Trumbore on a triangle slot, the sphere quadratic on a sphere slot (the flag in
// q2.w, rt_layout.h; scenes with spheres render on the megakernel).  SPH = false for the kernels that never see a
// sphere (the vertex-synchronous kernel and its pre-pass): the sphere branch cost their walk fallback 4 spilled VGPRs
template <bool SPH = true>
__device__ __forceinline__ bool leaf_hit(const SceneView& S, int slot, const Ray& r, double& t)
{
    const float4 t0 = S.tris[4 * slot], t1 = S.tris[4 * slot + 1], t2 = S.tris[4 * slot + 2];
    if (SPH && __float_as_uint(t2.w) != 0u) return sphere_hit(V3{t0.x, t0.y, t0.z}, t1.x, r, t);
    return moller_trumbore(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, r, t);
}
// the surface normal of a hit at `loc`: a triangle's face normal (q3), a sphere's Whitted::normalize(loc - center)
// (MC/Sphere.h:94)
__device__ __forceinline__ V3 leaf_normal(const SceneView& S, int slot, const V3& loc)
{
    const float4 t2 = S.tris[4 * slot + 2];
    if (__float_as_uint(t2.w) != 0u) {
        const float4 t0 = S.tris[4 * slot];
        return w_normalize(sub(loc, V3{t0.x, t0.y, t0.z}));
    }
    const float4 t3 = S.tris[4 * slot + 3];
    return V3{t3.x, t3.y, t3.z};
}

// One traversal: closest hit (shadow == false) or any blocking hit (shadow == true).
// Leaf triangles are postponed: a lane that reaches a leaf whose box it hits parks the triangle and
// the wave keeps walking boxes until every lane has a parked triangle or has finished; then all
// parked triangles are intersected together (Aila & Laine's while-while), so the Moller-Trumbore
// body runs once per "leaf round" instead of once per box step.  Each lane still tests its
// triangles in DFS order, so the tie rule (later leaf wins) and the any-hit exit are unchanged.
template <bool COUNT, bool FINITE, bool SPH = true>
__device__ __forceinline__ void traverse_impl(const SceneView& S, const Ray& r, bool shadow, double slen, double& best, int& best_tri,
                                              bool& occluded, uint32_t& node_tests, uint32_t& tri_tests)
{
    uint32_t i = 0;
    const uint32_t n = S.n_nodes;
    for (;;) {
        int parked = -1;
        while (i < n) {
            const float4 q0 = S.nodes[2 * i];
            const float4 q1 = S.nodes[2 * i + 1];
            if (COUNT) ++node_tests;
            const bool hit = FINITE ? slab_hit_finite(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y)
                                    : slab_hit(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
            const int tri = f2i(q1.w);
            const uint32_t skip = (uint32_t)f2i(q1.z);
            i = (hit && tri < 0) ? i + 1 : skip;
            if (hit && tri >= 0) { parked = tri; break; }
        }
        if (parked >= 0) {
            if (COUNT) ++tri_tests;
            double t;
            if (leaf_hit<SPH>(S, parked, r, t)) {
                if (shadow) {
                    // not occluded iff length(q-p) < t + 0.01f for every hit (MC/Renderer.cpp:184)
                    if (!(slen < t + (double)0.01f)) { occluded = true; i = n; }
                } else if (t <= best) {
                    // (left.t < right.t) ? left : right  ==> the later leaf wins ties
                    best = t; best_tri = parked;
                }
            }
        }
        if (i >= n) break;
    }
}

template <bool COUNT>
__device__ __forceinline__ void traverse(const SceneView& S, const Ray& r, bool shadow, double slen, double& best, int& best_tri,
                                         bool& occluded, uint32_t& node_tests, uint32_t& tri_tests)
{
    // wave-uniform choice: IEEE min/max when no lane can produce a NaN slab distance
    if (__all(rcp_finite(r))) traverse_impl<COUNT, true>(S, r, shadow, slen, best, best_tri, occluded, node_tests, tri_tests);
    else traverse_impl<COUNT, false>(S, r, shadow, slen, best, best_tri, occluded, node_tests, tri_tests);
}

// SamplingAreaLight -> TriangleMesh::Sampling -> BVH::Sampling_from_root/_node -> TrianglePrimitive::Sampling
// (MC/Renderer.h:163-180, MC/TriangleMesh.h:193-197, MC/BVH.h:103-129, MC/TriangleMesh.h:69-89)
template <class G>
__device__ __forceinline__ void sample_light(const SceneView& S, float light_area, G& g, V3& q, V3& nl, uint32_t* aw = nullptr, int* lt_out = nullptr)
{
    const float u0 = g.next();
    float p = u0 * light_area;
    int node = 0;
    for (;;) {
        const float4 ln = S.lnodes[node];
        const int left = f2i(ln.y);
        if (left < 0) break;
        const float la = S.lnodes[left].x;
        if (p < la) node = left;
        else { p = p - la; node = f2i(ln.z); }
    }
    const int lt = f2i(S.lnodes[node].w);
    const float4 A = S.ltris[4 * lt], B = S.ltris[4 * lt + 1], C = S.ltris[4 * lt + 2], N = S.ltris[4 * lt + 3];
    const float x = 1.0f - sqrt_big(g.next());   // (a draw is 0 or in [2^-32, 1]: sqrt_big's range)
    const float y = g.next();
    const V3 a{A.x, A.y, A.z}, b{B.x, B.y, B.z}, c{C.x, C.y, C.z};
    q = add(add(smul(x, a), smul((1.0f - x) * y, b)), smul((1.0f - x) * (1.0f - y), c));
    nl = V3{N.x, N.y, N.z};
    if (aw) *aw = __float_as_uint(A.w);   // the light triangle's shadow-candidate skip mask (rt_layout.h ltris)
    if (lt_out) *lt_out = lt;
}

// WhittedMaterial::Sampling, MC/WhittedMaterial.h:71-117
template <class G>
__device__ __forceinline__ V3 sample_hemisphere(V3 n, G& g)
{
    const float z = g.next();
    const float rxy = sqrt_big(1.0f - z * z);   // (z a draw in [0, 1]: 1 - z * z is 0 or >= 2^-23)
    const float phi = 2.0f * PI_F * g.next();
    float cphi, sphi;
    sincos_f(phi, cphi, sphi);
    const float x = rxy * cphi;
    const float y = rxy * sphi;
    V3 Y;
    // (n a unit normal, NaN or infinite for a degenerate triangle: the squared length is >= 1/2 up to
    // rounding, NaN or +inf, inside sqrt_big's range)
    if (__builtin_fabsf(n.x) > __builtin_fabsf(n.y)) Y = glm_normalize_big(V3{n.z, 0.0f, -(n.x)});
    else Y = glm_normalize_big(V3{0.0f, n.z, -(n.y)});
    const V3 X = cross(Y, n);
    return add(add(smul(x, X), smul(y, Y)), smul(z, n));
}

}  // namespace rtd
#endif
