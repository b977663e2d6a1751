// rt_resample.hip -- exact re-render of the samples whose path outgrew the vertex kernel's fold ring.
//
// The vertex kernel (rt_coherent.hip) keeps a path's EXACT levels in a per-lane HBM ring of
// `stack_depth` positions shared with the fold still draining.  A push that does not fit ends that
// sample at once: the lane appends (local pixel, frame index, global pixel, frame) to the overflow list
// and renders on.  This kernel then renders every listed sample again from its counter-based stream
// -- the same draws, traversal and arithmetic, so the same bits -- keeping the levels in a deep
// per-thread stack in HBM, folds them inner-first (MC/Renderer.cpp:208,213) and parks the result in the
// sample's slot of the parked-sample buffer, before finalize_chunks_kernel accumulates the frames in
// order.  A path is cut at 4096 vertices like in the vertex kernel (P = rr^4096; the reference has no
// cap).  The grid is persistent and exits at once when the list is empty (the common case), so the host
// launches it unconditionally, without a synchronisation.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernels.h"
#include "rt_path.h"

using namespace rtd;

__global__ void __launch_bounds__(256) resample_kernel(KParams P)
{
    const unsigned long long listed = *reinterpret_cast<const volatile unsigned long long*>(&P.counters[3]);
    const uint32_t n = listed < (unsigned long long)P.ovf_cap ? (uint32_t)listed : P.ovf_cap;
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= n) return;
    SceneView S{P.nodes, P.tris, P.mats, P.lnodes, P.ltris, P.n_nodes, nullptr};
    const float PDF = 1.0f / (2.0f * PI_F);   // WhittedMaterial::PDF_at_the_sample, MC/WhittedMaterial.h:44-56
    float4* stk = P.rs_stack;
    int32_t* smat = P.rs_mat;
    auto at = [&](uint32_t lvl) { return (size_t)lvl * nthreads + tid; };
    for (uint32_t i = tid; i < n; i += nthreads) {
        const uint4 e = P.ovf_list[i];   // (local pixel, frame index in the launch, global pixel, frame)
        const uint32_t local = e.x, fidx = e.y, pix = e.z, frame = e.w;
        const uint32_t y = pix / P.W, x = pix - y * P.W;
        Rng g;
        g.key(P.seed);
        g.start(pix, frame);
        // RayGen_Shader's camera ray (MC/Camera.cpp:119-125, MC/Renderer.cpp:128), as rt_coherent.hip
        const float ux = g.next(), uy = g.next();
        float cx = ((float)x + ux) / (float)P.W;
        float cy = ((float)y + uy) / (float)P.H;
        cx = cx * 2.0f - 1.0f;
        cy = cy * 2.0f - 1.0f;
        float tg[4];
        mat4_mul(P.iproj, cx, cy, 1.0f, 1.0f, tg);
        const V3 dv = glm_normalize(divs(V3{tg[0], tg[1], tg[2]}, tg[3]));
        float wd[4];
        mat4_mul(P.iview, dv.x, dv.y, dv.z, 0.0f, wd);
        V3 o{P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]};
        V3 d = w_normalize(V3{wd[0], wd[1], wd[2]});
        uint32_t nt = 0, tt = 0;
        double t = 1.7976931348623157e308;
        int tri = -1;
        bool occ = false;
        traverse<false>(S, make_ray(o, d), false, 0.0, t, tri, occ, nt, tt);
        V3 L{0.f, 0.f, 0.f};
        int top = -1;   // levels top..0 are folded into L
        if (tri < 0) {
            L = night_sky();   // cast_path miss, MC/Renderer.cpp:145
        } else if (S.mats[2 * f2i(S.tris[4 * tri].w)].w != 0.0f) {
            const float4 em = S.mats[2 * f2i(S.tris[4 * tri].w) + 1];   // direct emission, MC/Renderer.cpp:151-161
            L = V3{em.x, em.y, em.z};
        } else {
            for (uint32_t depth = 0;; ++depth) {
                // Renderer::shading at the hit (MC/Renderer.cpp:163-209), in the vertex kernel's order
                const int mat = f2i(S.tris[4 * tri].w);
                const float4 tq3 = S.tris[4 * tri + 3];
                const V3 wo = neg(d);
                const V3 loc = add(o, smul((float)t, d));   // Ray::operator(), MC/Ray.h:34-37
                const V3 N{tq3.x, tq3.y, tq3.z};
                const V3 nn = (dot(N, wo) < 0.0f) ? neg(N) : N;
                const V3 p = add(loc, muls(nn, INTERSECTION_CORRECTION));
                V3 ld{0.f, 0.f, 0.f};
                if (P.has_light) {
                    V3 q, nl0;
                    sample_light(S, P.light_area, g, q, nl0);
                    const V3 p2q = sub(q, p);
                    const V3 wl = glm_normalize(p2q);
                    const V3 nl = (dot(nl0, neg(wl)) < 0.0f) ? neg(nl0) : nl0;
                    const float sc1 = dot(wl, nn), sc2 = dot(neg(wl), nl), sd2 = dot(p2q, p2q);
                    const float slen = glm_length(p2q);
                    double ts = 1.7976931348623157e308;
                    int tris = -1;
                    bool blocked = false;
                    traverse<false>(S, make_ray(p, wl), true, (double)slen, ts, tris, blocked, nt, tt);
                    if (!blocked) {
                        const float4 mb = S.mats[2 * mat];
                        const V3 f = (sc1 >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};
                        ld = divs(divs(muls(muls(mul(V3{P.light_emission[0], P.light_emission[1], P.light_emission[2]}, f), sc1), sc2), sd2),
                                  (1.0f / P.light_area));
                    }
                }
                const bool cont = g.next() < P.rr && depth < 4096u;
                if (!cont) { L = ld; top = (int)depth - 1; break; }
                const V3 wi = glm_normalize(sample_hemisphere(nn, g));
                const float c = dot(wi, nn);
                o = p; d = wi;
                t = 1.7976931348623157e308; tri = -1; occ = false;
                traverse<false>(S, make_ray(o, d), false, 0.0, t, tri, occ, nt, tt);
                if (tri < 0 || S.mats[2 * f2i(S.tris[4 * tri].w)].w != 0.0f) {   // radiance_indirect = 0, MC/Renderer.cpp:202
                    L = ld; top = (int)depth - 1; break;
                }
                stk[at(depth)] = make_float4(ld.x, ld.y, ld.z, c);   // level `depth` recurses into the new hit
                smat[at(depth)] = mat;
            }
        }
        for (int lvl = top; lvl >= 0; --lvl) {   // inner-first: L = Ld_k + ((((L * brdf_k) * cos_k) / PDF) / RR)
            const float4 q = stk[at((uint32_t)lvl)];
            const float4 mb = S.mats[2 * smat[at((uint32_t)lvl)]];
            const V3 f = (q.w >= 0.0f) ? V3{mb.x, mb.y, mb.z} : V3{0.0f, 0.0f, 0.0f};
            L = add(V3{q.x, q.y, q.z}, divs(divs(muls(mul(L, f), q.w), PDF), P.rr));
        }
        // the sample's parked slot (rt_coherent.hip: complete)
        const size_t blk = P.lbuf_pixel_major ? (size_t)local * ((P.n_frames + 3u) >> 2) + (fidx >> 2) : (size_t)(fidx >> 2) * P.lbuf_stride + local;
        const size_t a = (blk * 4u + (fidx & 3u)) * 3u;
        P.lbuf[a] = L.x;
        P.lbuf[a + 1] = L.y;
        P.lbuf[a + 2] = L.z;
    }
}

hipError_t rt_launch_resample(const KParams& P, uint32_t threads, hipStream_t stream)
{
    if (!P.ovf_list || threads == 0) return hipSuccess;
    hipLaunchKernelGGL(resample_kernel, dim3((threads + 255) / 256), dim3(256), 0, stream, P);
    return hipGetLastError();
}
