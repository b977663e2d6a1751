// rt_denoise.hip -- the reference's Denoiser (DN/ = "Denoiser/8599RayTracerGUI/src/", DN/Denoiser.h) as
// image-space HIP kernels over the G-buffer the megakernel writes in its GB mode:
//   * joint bilateral filter (Denoiser::JointBilateralFiltering, DN/Denoiser.h:133-228): per pixel a
//     (2h+1)^2 window, weights exp(-(position + color + normal-angle + coplanarity distances)),
//     columns outer / rows inner as the reference sums them;
//   * temporal filter (Denoiser::TemporalFiltering, DN/Denoiser.h:235-328): reprojection of the
//     world position with the previous frame's projection * view, primitive-id test, clamp of the
//     history to mean +- tolerance * deviation of the current (2t+1)^2 neighbourhood, blend; fused
//     with the final clamp + RGBA8 pack (DN/Renderer.cpp:265-280).
// Every float operation is the reference's; exp and acos are glibc's expf / acosf restated
// (rt_glibc_math.h), so the weights -- and the filtered frames -- are the reference's bit for bit.
// The joint bilateral filter stages the window's columns through LDS (jbf_lds_kernel); the temporal
// filter runs one thread per pixel in 16x16 tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "rt_device.h"
#include "rt_glibc_math.h"
#include "rt_kernels.h"
#include "rt_knobs.h"

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

// One tap of the window (DN/Denoiser.h:178-205) for a contributing neighbour: its weight and weighted
// color added in the reference's order.  Bit-identical to the reference, with three economies:
//   * the divisions are by the launch's constants 2 sigma^2: from y = RN(1/d), Markstein's correction
//     q + (x - q d) y (rt_device.h div_fast_core) is the IEEE quotient for every x in [2^-100, 2^100)
//     and 0 (tools/verify_glibc_math.cpp checks the default divisors exhaustively); a wave with any x
//     outside falls back to the division;
//   * the normal term depends on the neighbour's normal alone (the centre's is fixed): a lane keeps the
//     last normal's term and recomputes it only when the normal changes (flat-shaded surfaces: rarely);
//   * expf / acosf in their branch-free forms for the filter's domains (rt_glibc_math.h).
struct JbfConsts {
    float dsp, dsc, dsn, dsk;   // 2 sigma^2 of position, color, normal, coplanarity
    float ysp, ysc, ysn, ysk;   // their reciprocals (used when `fast`)
    bool fast;
};

struct JbfMemo {
    uint32_t nx = 0x7fc00000u, ny = 0u, nz = 0u;   // the normal the term belongs to (NaN: none yet)
    float snd = 0.0f;
};

__device__ __forceinline__ bool div_range(float x)
{   // x in [2^-100, 2^100) or +0 (x >= +0 or NaN here: squares and a vector's dot with itself)
    const uint32_t u = __float_as_uint(x);
    return (u - 0x0d800000u) < 0x64000000u || u == 0u;
}

__device__ __forceinline__ void jbf_tap(const JbfConsts& K, const V3& cc, const V3& cp, const V3& cn, const V3& kcol, const V3& kpos,
                                        const V3& knrm, JbfMemo& memo, V3& acc, float& wsum)
{
    if (__float_as_uint(knrm.x) != memo.nx || __float_as_uint(knrm.y) != memo.ny || __float_as_uint(knrm.z) != memo.nz) {
        float snd = glibc_math::acosf_unit(smin(smax(0.0f, dot(knrm, cn)), 1.0f));
        snd = snd * snd;
        memo.snd = (K.fast && div_range(snd)) ? div_fast_core(snd, K.dsn, K.ysn) : snd / K.dsn;
        memo.nx = __float_as_uint(knrm.x); memo.ny = __float_as_uint(knrm.y); memo.nz = __float_as_uint(knrm.z);
    }
    const V3 dp = sub(kpos, cp);
    const float xp = dot(dp, dp);
    const V3 dc = sub(kcol, cc);
    const float xc = dot(dc, dc);
    float cop = dot(cn, glm_normalize(dp));   // (the short square root here measured neutral: profiles/r05/ab/dn_sqrt_ab.jsonl)
    cop = cop * cop;
    float wpd, cd, cq;
    if (K.fast && __all(div_range(xp) && div_range(xc) && div_range(cop))) {
        wpd = div_fast_core(xp, K.dsp, K.ysp);
        cd = div_fast_core(xc, K.dsc, K.ysc);
        cq = div_fast_core(cop, K.dsk, K.ysk);
    } else {
        wpd = xp / K.dsp;
        cd = xc / K.dsc;
        cq = cop / K.dsk;
    }
    const float w = glibc_math::expf_nonpos<true>(-(((wpd + cd) + memo.snd) + cq));
    wsum = wsum + w;
    acc = add(acc, smul(w, kcol));
}

__device__ __forceinline__ JbfConsts jbf_consts(const DenoiseParams& D)
{
    JbfConsts K;
    K.dsp = 2.0f * D.sigma_position * D.sigma_position;
    K.dsc = 2.0f * D.sigma_color * D.sigma_color;
    K.dsn = 2.0f * D.sigma_normal * D.sigma_normal;
    K.dsk = 2.0f * D.sigma_coplanarity * D.sigma_coplanarity;
    K.ysp = rcp_f32(K.dsp); K.ysc = rcp_f32(K.dsc); K.ysn = rcp_f32(K.dsn); K.ysk = rcp_f32(K.dsk);
    auto ok = [](float d) { return d >= 0x1p-20f && d < 0x1p20f; };   // div_fast's verified divisor range
    K.fast = ok(K.dsp) && ok(K.dsc) && ok(K.dsn) && ok(K.dsk) && D.ieee_div == 0;
    return K;
}

__device__ __forceinline__ void jbf_store(const DenoiseParams& D, int i, V3 acc, float wsum)
{
    V3 f = divs(acc, wsum);
    if (D.immediate_clamp) f = V3{smin(smax(f.x, 0.0f), 1.0f), smin(smax(f.y, 0.0f), 1.0f), smin(smax(f.z, 0.0f), 1.0f)};
    D.spatial[i] = make_float4(f.x, f.y, f.z, 0.0f);
}

// The joint bilateral filter through LDS.  A workgroup filters an 8 x 32 block of pixels (a wave: 8
// columns x 8 rows).  The reference sums each window column by column (outer), rows inner; every lane of
// the block is at the same column offset dk at the same time, so the block needs the 8 columns
// x0 + dk .. x0 + dk + 7 of rows y0 - h .. y0 + 31 + h.  They sit in a ring of 9 LDS columns: at step dk
// the workgroup loads column x0 + dk + 8 into the slot column x0 + dk - 1 left, filters, and meets at
// one barrier.  Each G-buffer pixel is read from HBM/L2 once per block instead of once per tap.  A slot
// holds 9 planes (color, position, normal; a pixel outside the image or not a contributor carries a NaN
// normal x and is skipped, as the reference's window bounds and contributor test skip it).  Plane pitch
// CHP = 4 (mod 32) keeps a ds_read_b32 lane group (4 rows x 8 slots) on distinct banks.
constexpr int JBW = 8, JSLOTS = JBW + 1, JB_MAX_HALF = 80;

__host__ __device__ inline int jbf_pitch(int jbh, int h) { const int ch = jbh + 2 * h; return ch + ((4 - ch % 32) + 32) % 32; }

template <int JBH>
__global__ void __launch_bounds__(8 * JBH) jbf_lds_kernel(DenoiseParams D)
{
    extern __shared__ float lds[];
    const int h = D.jbf_half, CH = JBH + 2 * h, CHP = jbf_pitch(JBH, h);
    const int tiles_x = (D.W + JBW - 1) / JBW;
    const int x0 = (int)(blockIdx.x % (uint32_t)tiles_x) * JBW, y0 = (int)(blockIdx.x / (uint32_t)tiles_x) * JBH;
    const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
    const int lx = lane & 7, ly = (lane >> 3) + 8 * wv;
    const int x = x0 + lx, y = y0 + ly;
    const bool in = x < D.W && y < D.H;
    const int i = in ? y * D.W + x : 0;
    const float4 c0 = D.color[i];
    const bool active = in && D.prim[i] != -1;
    if (in && !active) D.spatial[i] = c0;   // not a contributor: copied, unclamped
    const V3 cc = v3(c0), cp = v3(D.pos[i]), cn = v3(D.nrm[i]);
    const JbfConsts K = jbf_consts(D);
    auto plane = [&](int f, int slot) { return lds + (f * JSLOTS + slot) * CHP; };
    // column k (absolute x = x0 - h + k): thread t < CH fetches row y0 - h + t (CH <= 192); the planes
    // are written separately so a step's fetch is in flight while the step filters
    const int t_ld = (int)threadIdx.x;
    auto fetch_col = [&](int k, float v[9]) {
        const int gx = x0 - h + k, gy = y0 - h + t_ld;
        bool ok = t_ld < CH && gx >= 0 && gx < D.W && gy >= 0 && gy < D.H;
        const int j = ok ? gy * D.W + gx : 0;
        ok = ok && D.prim[j] != -1;
        if (ok) {
            const float4 a = D.color[j], b = D.pos[j], n = D.nrm[j];
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = b.x; v[4] = b.y; v[5] = b.z; v[6] = n.x; v[7] = n.y; v[8] = n.z;
        } else {
#pragma unroll
            for (int f = 0; f < 9; ++f) v[f] = 0.0f;
            v[6] = __builtin_nanf("");
        }
    };
    auto store_col = [&](int k, const float v[9]) {
        if (t_ld < CH) {
            const int slot = k % JSLOTS;
#pragma unroll
            for (int f = 0; f < 9; ++f) plane(f, slot)[t_ld] = v[f];
        }
    };
    float v[9];
    for (int k = 0; k < JBW; ++k) {
        fetch_col(k, v);
        store_col(k, v);
    }
    __syncthreads();
    V3 acc{0.0f, 0.0f, 0.0f};
    float wsum = 0.0f;
    JbfMemo memo;
    const int steps = 2 * h + 1;
    for (int s = 0; s < steps; ++s) {
        // column s + 8 (first read at step s + 1) goes to the slot column s - 1 left; none after the last step
        const bool more = s + 1 < steps;
        if (more) fetch_col(s + JBW, v);
        if (active) {
            const int slot = (s + lx) % JSLOTS;
            const float* p0 = plane(0, slot);
            const int stride = JSLOTS * CHP;   // plane f of this slot: p0 + f * stride
            const bool centre_col = s == h;
            for (int dr = 0; dr <= 2 * h; ++dr) {
                const int t = ly + dr;
                const float nx = p0[6 * stride + t];
                if (nx != nx) continue;   // outside the image or not a contributor
                const V3 kcol{p0[t], p0[stride + t], p0[2 * stride + t]};
                if (centre_col && dr == h) {
                    wsum = wsum + 1.0f;   // every distance is zero
                    acc = add(acc, cc);
                    continue;
                }
                const V3 kpos{p0[3 * stride + t], p0[4 * stride + t], p0[5 * stride + t]};
                const V3 knrm{nx, p0[7 * stride + t], p0[8 * stride + t]};
                jbf_tap(K, cc, cp, cn, kcol, kpos, knrm, memo, acc, wsum);
            }
        }
        if (more) store_col(s + JBW, v);
        __syncthreads();
    }
    if (active) jbf_store(D, i, acc, wsum);
}

// The same filter straight from the G-buffer (one thread per pixel in 16 x 16 tiles): windows wider than
// the LDS ring holds (jbf_half > JB_MAX_HALF).
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
    const JbfConsts K = jbf_consts(D);
    V3 acc{0.0f, 0.0f, 0.0f};
    float wsum = 0.0f;
    JbfMemo memo;
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
            jbf_tap(K, cc, cp, cn, kcol, v3(D.pos[j]), v3(D.nrm[j]), memo, acc, wsum);
        }
    }
    jbf_store(D, i, acc, wsum);
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
        DenoiseParams Dl = D;
        Dl.ieee_div = rt_knob("RT_JBF_IEEE") ? 1 : 0;   // diagnostic: every division by the IEEE sequence (tests)
        if (D.jbf_half <= JB_MAX_HALF && !rt_knob("RT_JBF_GLOBAL")) {
            // 8 x 64 blocks (8 waves) for wide windows: the ring's halo rows are shared by twice the pixels
            // and 6 waves per SIMD fit instead of 4 (DN65 13.8 -> 12.6 ms); 8 x 32 below a half width of 24
            // (DN33 3.41 ms against 3.66); the 8 x 64 ring must fit 64 KiB of LDS: half widths up to 64.
            // RT_JBF_TALL=32/64 forces one (A/B, tests)
            const int want = rt_knob("RT_JBF_TALL") ? atoi(rt_knob("RT_JBF_TALL")) : (D.jbf_half >= 24 ? 64 : 32);
            const int jbh = (want == 64 && D.jbf_half <= 64) ? 64 : 32;
            const uint32_t blocks = (uint32_t)(((D.W + JBW - 1) / JBW) * ((D.H + jbh - 1) / jbh));
            const size_t lds = (size_t)9 * JSLOTS * jbf_pitch(jbh, D.jbf_half) * sizeof(float);
            if (jbh == 64) hipLaunchKernelGGL(jbf_lds_kernel<64>, dim3(blocks), dim3(512), lds, stream, Dl);
            else hipLaunchKernelGGL(jbf_lds_kernel<32>, dim3(blocks), dim3(256), lds, stream, Dl);
        } else {
            hipLaunchKernelGGL(jbf_kernel, dim3(tiles), dim3(256), 0, stream, Dl);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(temporal_kernel, dim3(tiles), dim3(256), 0, stream, D);
    return hipGetLastError();
}
