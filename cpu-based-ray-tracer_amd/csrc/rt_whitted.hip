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
// The scene (1.4 MB for C3) is read from HBM through L2; one thread per local pixel in 16x16 tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernels.h"

using namespace rtd;

namespace {

// closest hit (shadow == false) or "any hit with t*t < d2" (shadow == true) over the global scene
template <bool COUNT>
__device__ __forceinline__ void whitted_traverse(const KParams& P, const Ray& r, bool shadow, double d2, double& best, int& best_tri, bool& occluded,
                                                 uint32_t& node_tests, uint32_t& tri_tests)
{
    const float4* __restrict__ nodes = P.nodes;
    const float4* __restrict__ tris = P.tris;
    const uint32_t n = P.n_nodes;
    uint32_t i = 0;
    while (i < n) {
        const float4 q0 = nodes[2 * i];
        const float4 q1 = nodes[2 * i + 1];
        if (COUNT) ++node_tests;
        const bool hit = slab_hit(r, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y);
        const int tri = f2i(q1.w);
        const uint32_t skip = (uint32_t)f2i(q1.z);
        if (hit && tri >= 0) {
            if (COUNT) ++tri_tests;
            const float4 t0 = tris[4 * tri], t1 = tris[4 * tri + 1], t2 = tris[4 * tri + 2];
            double t;
            if (moller_trumbore(V3{t0.x, t0.y, t0.z}, V3{t1.x, t1.y, t1.z}, V3{t2.x, t2.y, t2.z}, r, t)) {
                if (shadow) {
                    // (shadow_record.has_intersection) && (t * t < light_distance_squared), BV/Renderer.cpp:195
                    if (t * t < d2) { occluded = true; return; }
                } else if (t <= best) {
                    best = t; best_tri = tri;   // (left.t < right.t) ? left : right: the later leaf wins ties
                }
            }
        }
        i = (hit && tri < 0) ? i + 1 : skip;
    }
}

}  // namespace

template <bool COUNT>
__global__ void __launch_bounds__(256) whitted_kernel(KParams P)
{
    const uint32_t tiles_x = (P.W + 15) / 16;
    const uint32_t tile = blockIdx.x;
    const uint32_t lr = (tile / tiles_x) * 16 + (threadIdx.x >> 4);
    const uint32_t lx = (tile % tiles_x) * 16 + (threadIdx.x & 15);
    uint32_t node_tests = 0, tri_tests = 0, rays = 0;
    if (lr < P.n_local_rows && lx < P.W) {
        const uint32_t band_k = lr / P.band, in_band = lr - band_k * P.band;
        const uint32_t y = (P.rank + band_k * P.nranks) * P.band + in_band;
        const uint32_t local = lr * P.W + lx;
        float4 acc = (P.first_frame == 1u) ? make_float4(0.f, 0.f, 0.f, 0.f) : P.accum[local];
        float cam_x = P.cam_pos[0];
        for (uint32_t k = 0; k < P.n_frames; ++k) {
            // the reference evaluates every frame; keep the compiler from hoisting the frame's work
            asm volatile("" : "+v"(cam_x));
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
                for (uint32_t l = 0; l < P.n_plights; ++l) {
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
    const uint32_t tiles = ((P.W + 15) / 16) * ((P.n_local_rows + 15) / 16);
    if (grid_out) *grid_out = tiles;
    if (tiles == 0) return hipSuccess;
    if (count) hipLaunchKernelGGL(whitted_kernel<true>, dim3(tiles), dim3(256), 0, stream, P);
    else hipLaunchKernelGGL(whitted_kernel<false>, dim3(tiles), dim3(256), 0, stream, P);
    return hipGetLastError();
}
