// rt_glibc_math.h -- glibc 2.35's expf and acosf restated for the device (and the host checker).
//
// The reference's denoiser calls std::exp / std::acos on floats (DN/Denoiser.h:195,203), which on its
// Linux build are glibc's expf / acosf.  Neither is correctly rounded, so a device exp/acos (or a
// double evaluation rounded once) differs from them in the last place now and then; these
// restatements follow glibc's algorithms operation for operation so the joint bilateral filter's
// weights are the reference's bit for bit:
//   * expf: sysdeps/ieee754/flt-32/e_expf.c + e_exp2f_data.c (ARM optimized-routines): x*32/ln2 =
//     k + r in double, 2^(k/32) from a 32-entry table, a cubic in r, one rounding to float.  x86-64
//     glibc runs its FMA build (sysdeps/x86_64/fpu/multiarch/e_expf-fma.c, the same C compiled with
//     -mfma -mavx2: GCC contracts every multiply whose uses are all additions); `Fma` selects it.
//   * acosf: sysdeps/ieee754/flt-32/e_acosf.c (fdlibm): float arithmetic, a rational minimax of
//     asin on [0, 0.5] and the half-angle identity above 0.5 with a split sqrt.
// Checked against the host's libm for every float of the filter's domains -- expf on [-inf, 0],
// acosf on [0, 1] -- by tools/verify_glibc_math.cpp (tests/test_glibc_math.py runs a strided sweep).
#ifndef RT_GLIBC_MATH_H
#define RT_GLIBC_MATH_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtd {
namespace glibc_math {

__host__ __device__ inline uint32_t fbits(float x) { return __builtin_bit_cast(uint32_t, x); }
__host__ __device__ inline float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }
__host__ __device__ inline uint64_t dbits(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ inline double bitsd(uint64_t u) { return __builtin_bit_cast(double, u); }

// 2^(i/32) as uint64 bits minus i << 47 (e_exp2f_data.c `tab`)
#define RT_EXP2F_TAB                                                                                    \
    {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,        \
     0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,        \
     0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,        \
     0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,        \
     0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,        \
     0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,        \
     0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,        \
     0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}

__device__ __constant__ static const uint64_t exp2f_tab_dev[32] = RT_EXP2F_TAB;
static const uint64_t exp2f_tab_host[32] = RT_EXP2F_TAB;

__host__ __device__ inline uint64_t exp2f_tab(uint32_t i)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return exp2f_tab_dev[i];
#else
    return exp2f_tab_host[i];
#endif
}

constexpr double EXPF_INVLN2N = 0x1.71547652b82fep+0 * 32;
constexpr double EXPF_SHIFT = 0x1.8p+52;
constexpr double EXPF_C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, EXPF_C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                 EXPF_C2 = 0x1.62e42ff0c52d6p-1 / 32;

__host__ __device__ inline uint32_t top12(float x) { return fbits(x) >> 20; }

// the main path (|x| < 104: the table index and the scale's exponent stay in range)
template <bool Fma>
__host__ __device__ inline float expf_core(float x)
{
    const double xd = (double)x;
    double kd, r;
    uint64_t ki;
    if (Fma) {   // z = InvLn2N * xd has only additive uses: fused into both
        kd = __builtin_fma(EXPF_INVLN2N, xd, EXPF_SHIFT);
        ki = dbits(kd);
        kd -= EXPF_SHIFT;
        r = __builtin_fma(EXPF_INVLN2N, xd, -kd);
    } else {
        const double z = EXPF_INVLN2N * xd;
        kd = z + EXPF_SHIFT;
        ki = dbits(kd);
        kd -= EXPF_SHIFT;
        r = z - kd;
    }
    uint64_t t = exp2f_tab((uint32_t)(ki % 32));
    t += ki << (52 - 5);
    const double s = bitsd(t);
    double y;
    if (Fma) {
        const double z = __builtin_fma(EXPF_C0, r, EXPF_C1);
        const double r2 = r * r;
        y = __builtin_fma(EXPF_C2, r, 1.0);
        y = __builtin_fma(z, r2, y);
    } else {
        const double z = EXPF_C0 * r + EXPF_C1;
        const double r2 = r * r;
        y = EXPF_C2 * r + 1.0;
        y = z * r2 + y;
    }
    y = y * s;
    return (float)y;
}

template <bool Fma>
__host__ __device__ inline float expf(float x)
{
    const uint32_t abstop = top12(x) & 0x7ffu;
    if (abstop >= top12(88.0f)) {   // |x| >= 88 or NaN
        if (fbits(x) == fbits(-__builtin_inff())) return 0.0f;
        if (abstop >= top12(__builtin_inff())) return x + x;
        if (x > 0x1.62e42ep6f) return __builtin_inff();   // __math_oflowf
        if (x < -0x1.9fe368p6f) return 0.0f;              // __math_uflowf
    }
    return expf_core<Fma>(x);
}

// expf on its non-positive domain (and NaN) without branches: the main path on an input clamped to
// [-104, 0] (table index and scale stay in range), then glibc's special returns selected -- 0 below
// log(2^-150) (-inf included; __math_uflowf), x + x for a NaN.  The joint bilateral weight
// exp(-(distances)) only ever takes this domain.
template <bool Fma>
__host__ __device__ inline float expf_nonpos(float x)
{
    const float xc = (x < -104.0f) ? -104.0f : x;
    float y = expf_core<Fma>(xc);
    y = (x < -0x1.9fe368p6f) ? 0.0f : y;
    return (x != x) ? x + x : y;
}

constexpr float ACOS_PI = 3.1415925026e+00f, ACOS_PIO2_HI = 1.5707962513e+00f, ACOS_PIO2_LO = 7.5497894159e-08f;
constexpr float ACOS_PS0 = 1.6666667163e-01f, ACOS_PS1 = -3.2556581497e-01f, ACOS_PS2 = 2.0121252537e-01f,
                ACOS_PS3 = -4.0055535734e-02f, ACOS_PS4 = 7.9153501429e-04f, ACOS_PS5 = 3.4793309169e-05f;
constexpr float ACOS_QS1 = -2.4033949375e+00f, ACOS_QS2 = 2.0209457874e+00f, ACOS_QS3 = -6.8828397989e-01f,
                ACOS_QS4 = 7.7038154006e-02f;

__host__ __device__ inline float acos_p(float z)
{
    return z * (ACOS_PS0 + z * (ACOS_PS1 + z * (ACOS_PS2 + z * (ACOS_PS3 + z * (ACOS_PS4 + z * ACOS_PS5)))));
}
__host__ __device__ inline float acos_q(float z) { return 1.0f + z * (ACOS_QS1 + z * (ACOS_QS2 + z * (ACOS_QS3 + z * ACOS_QS4))); }

__host__ __device__ inline float acosf(float x)
{
    const int32_t hx = (int32_t)fbits(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return (hx > 0) ? 0.0f : ACOS_PI + 2.0f * ACOS_PIO2_LO;   // |x| == 1
    if (ix > 0x3f800000) return (x - x) / (x - x);                                   // |x| > 1, NaN
    if (ix < 0x3f000000) {                                                           // |x| < 0.5
        if (ix <= 0x32800000) return ACOS_PIO2_HI + ACOS_PIO2_LO;
        const float z = x * x;
        const float r = acos_p(z) / acos_q(z);
        return ACOS_PIO2_HI - (x - (ACOS_PIO2_LO - x * r));
    }
    if (hx < 0) {   // x < -0.5
        const float z = (1.0f + x) * 0.5f;
        const float s = __builtin_sqrtf(z);
        const float r = acos_p(z) / acos_q(z);
        const float w = r * s - ACOS_PIO2_LO;
        return ACOS_PI - 2.0f * (s + w);
    }
    // x > 0.5
    const float z = (1.0f - x) * 0.5f;
    const float s = __builtin_sqrtf(z);
    const float df = bitsf(fbits(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float r = acos_p(z) / acos_q(z);
    const float w = r * s + c;
    return 2.0f * (df + w);
}

// acosf on [+0, 1] without branches (the filter's clamped cosine): both of glibc's paths on the selected
// reduced argument, one rational evaluation, the special returns selected.
__host__ __device__ inline float acosf_unit(float x)
{
    const uint32_t ix = fbits(x);
    const bool small = ix < 0x3f000000u;   // x < 0.5
    const float z = small ? x * x : (1.0f - x) * 0.5f;
    const float r = acos_p(z) / acos_q(z);
    const float r_small = ACOS_PIO2_HI - (x - (ACOS_PIO2_LO - x * r));
    const float s = __builtin_sqrtf(z);
    const float df = bitsf(fbits(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float w = r * s + c;
    const float r_large = 2.0f * (df + w);
    float res = small ? r_small : r_large;
    res = (ix <= 0x32800000u) ? ACOS_PIO2_HI + ACOS_PIO2_LO : res;
    return (ix == 0x3f800000u) ? 0.0f : res;
}

}  // namespace glibc_math
}  // namespace rtd
#endif
