// rt_denoise.hip -- the reference's Denoiser (DN/ = "Denoiser/8599RayTracerGUI/src/", DN/Denoiser.h) as
// image-space HIP kernels over the G-buffer the megakernel writes in its GB mode:
//   * joint bilateral filter (Denoiser::JointBilateralFiltering, DN/Denoiser.h:133-228): per pixel a
//     (2h+1)^2 window, weights exp(-(position + color + normal-angle + coplanarity distances)),
//     columns outer / rows inner as the reference sums them;
//   * temporal filter (Denoiser::TemporalFiltering, DN/Denoiser.h:235-328): reprojection of the
//     world position with the previous frame's projection * view, primitive-id test, clamp of the
//     history to mean +- tolerance * deviation of the current (2t+1)^2 neighbourhood, blend; fused
//     with the final clamp + RGBA8 pack (DN/Renderer.cpp:265-280).
// Every float operation is the reference's; exp and acos (glibc expf / acosf in the reference) are
// evaluated in double and rounded once, so a weight can differ from glibc's in the last place.
// One thread per pixel in 16x16 tiles; the G-buffer (5 x 16 B per pixel) is read through L1/L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernels.h"

using namespace rtd;

namespace {

__device__ __forceinline__ V3 v3(const float4& q) { return V3{q.x, q.y, q.z}; }

__device__ __forceinline__ void tile_xy(const DenoiseParams& D, int& x, int& y)
{
    const int tiles_x = (D.W + 15) / 16;
    x = (int)(blockIdx.x % tiles_x) * 16 + (int)(threadIdx.x & 15);
    y = (int)(blockIdx.x / tiles_x) * 16 + (int)(threadIdx.x >> 4);
}

}  // namespace

__global__ void __launch_bounds__(256) jbf_kernel(DenoiseParams D)
{
    int x, y;
    tile_xy(D, x, y);
    if (x >= D.W || y >= D.H) return;
    const int i = y * D.W + x;
    const float4 c0 = D.color[i];
    if (D.prim[i] == -1) {   // not a contributor: copied, unclamped
        D.spatial[i] = c0;
        return;
    }
    const int h = D.jbf_half;
    const int kl = max(0, x - h), kr = min(D.W - 1, x + h);
    const int kb = max(0, y - h), kt = min(D.H - 1, y + h);
    const V3 cc = v3(c0), cp = v3(D.pos[i]), cn = v3(D.nrm[i]);
    const float dsp = 2.0f * D.sigma_position * D.sigma_position, dsc = 2.0f * D.sigma_color * D.sigma_color;
    const float dsn = 2.0f * D.sigma_normal * D.sigma_normal, dsk = 2.0f * D.sigma_coplanarity * D.sigma_coplanarity;
    V3 acc{0.0f, 0.0f, 0.0f};
    float wsum = 0.0f;
    for (int kc = kl; kc <= kr; ++kc) {
        for (int krow = kb; krow <= kt; ++krow) {
            const int j = krow * D.W + kc;
            if (D.prim[j] == -1) continue;
            const V3 kcol = v3(D.color[j]);
            if (kc == x && krow == y) {
                wsum = wsum + 1.0f;   // every distance is zero
                acc = add(acc, cc);
                continue;
            }
            const V3 dp = sub(v3(D.pos[j]), cp);
            const float wpd = dot(dp, dp) / dsp;
            const V3 dc = sub(kcol, cc);
            const float cd = dot(dc, dc) / dsc;
            float snd = (float)acos((double)smin(smax(0.0f, dot(v3(D.nrm[j]), cn)), 1.0f));
            snd = snd * snd;
            snd = snd / dsn;
            float cop = dot(cn, glm_normalize(dp));
            cop = cop * cop;
            cop = cop / dsk;
            const float w = (float)exp((double)(-(((wpd + cd) + snd) + cop)));
            wsum = wsum + w;
            acc = add(acc, smul(w, kcol));
        }
    }
    V3 f = divs(acc, wsum);
    if (D.immediate_clamp) f = V3{smin(smax(f.x, 0.0f), 1.0f), smin(smax(f.y, 0.0f), 1.0f), smin(smax(f.z, 0.0f), 1.0f)};
    D.spatial[i] = make_float4(f.x, f.y, f.z, 0.0f);
}

__global__ void __launch_bounds__(256) temporal_kernel(DenoiseParams D)
{
    int x, y;
    tile_xy(D, x, y);
    if (x >= D.W || y >= D.H) return;
    const int i = y * D.W + x;
    const V3 cur = v3(D.spatial[i]);
    V3 prev{0.0f, 0.0f, 0.0f};
    float wgt = 1.0f;   // all from the current frame
    const int id = D.prim[i];
    if (D.have_prev && id != -1) {
        const float4 wp = D.pos[i];
        float vq[4], c4[4];
        mat4_mul(D.prev_view, wp.x, wp.y, wp.z, 1.0f, vq);         // view * world_position
        mat4_mul(D.prev_proj, vq[0], vq[1], vq[2], vq[3], c4);    // projection * (...)
        const float cx = c4[0] / c4[3], cy = c4[1] / c4[3];
        const float sx = (cx + 1.0f) / 2.0f, sy = (cy + 1.0f) / 2.0f;
        const float px = sx * (float)D.W, py = sy * (float)D.H;
        if (px > 0.0f && px < (float)D.W && py > 0.0f && py < (float)D.H) {
            const int j = (int)py * D.W + (int)px;
            if (id == D.prev_prim[j]) {
                prev = v3(D.prev_color[j]);
                wgt = D.weighting;
                const int t = D.temporal_half;
                const int kl = max(0, x - t), kr = min(D.W - 1, x + t);
                const int kb = max(0, y - t), kt = min(D.H - 1, y + t);
                V3 mean{0.0f, 0.0f, 0.0f}, var{0.0f, 0.0f, 0.0f};
                int n = 0;
                for (int a = kl; a <= kr; ++a) {
                    for (int b = kb; b <= kt; ++b) {
                        ++n;
                        const V3 q = v3(D.spatial[b * D.W + a]);
                        mean = add(mean, q);
                        const V3 diff = sub(cur, q);
                        var = add(var, mul(diff, diff));
                    }
                }
                mean = divs(mean, (float)n);
                var.x = __builtin_sqrtf(smax(var.x / (float)n, 0.0f));
                var.y = __builtin_sqrtf(smax(var.y / (float)n, 0.0f));
                var.z = __builtin_sqrtf(smax(var.z / (float)n, 0.0f));
                const V3 lo = sub(mean, smul(D.tolerance, var)), hi = add(mean, smul(D.tolerance, var));
                prev = V3{smin(smax(prev.x, lo.x), hi.x), smin(smax(prev.y, lo.y), hi.y), smin(smax(prev.z, lo.z), hi.z)};
            }
        }
    }
    const V3 out = add(smul(1.0f - wgt, prev), smul(wgt, cur));
    D.temporal[i] = make_float4(out.x, out.y, out.z, 0.0f);
    // final clamp + pack (DN/Renderer.cpp:265-280)
    const float r = smin(smax(out.x, 0.0f), 1.0f), g = smin(smax(out.y, 0.0f), 1.0f), b = smin(smax(out.z, 0.0f), 1.0f);
    D.rgba[i] = (to_u8(1.0f) << 24) | (to_u8(b) << 16) | (to_u8(g) << 8) | to_u8(r);
}

hipError_t rt_launch_denoise(const DenoiseParams& D, hipStream_t stream)
{
    const uint32_t tiles = (uint32_t)(((D.W + 15) / 16) * ((D.H + 15) / 16));
    if (tiles == 0) return hipSuccess;
    if (D.jbf_half > 0) {
        hipLaunchKernelGGL(jbf_kernel, dim3(tiles), dim3(256), 0, stream, D);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(temporal_kernel, dim3(tiles), dim3(256), 0, stream, D);
    return hipGetLastError();
}
