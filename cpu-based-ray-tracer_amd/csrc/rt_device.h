// rt_device.h -- device arithmetic of the path tracer, in the reference's operation order.
//
// Every expression mirrors the reference (MC/ = "Monte Carlo Path Tracer/8599RayTracerGUI/src/")
// and glm 0.9.9.9 (GLM/ = ".../Walnut/vendor/glm/glm/") term by term.  The file is compiled with
// -ffp-contract=off, without fast-math, and with correctly rounded f32 division/sqrt, so each
// operation is the same IEEE operation the CPU reference performs.  cos/sin of the hemisphere
// angle restate glibc's cosf/sinf (what the reference calls on Linux) bit for bit on [0, 2*PI].
#ifndef RT_DEVICE_H
#define RT_DEVICE_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtd {

struct V3 { float x, y, z; };
// cast_path's miss radiance, the night sky (12, 20, 69) / 255 (MC/Renderer.cpp:145): one definition for every
// kernel that adds it (the path kernels, the camera pre-pass, the finalize of the pre-pass's sky bits, the resample)
constexpr float kNightSkyR = 12 / 255.0f, kNightSkyG = 20 / 255.0f, kNightSkyB = 69 / 255.0f;
__device__ __forceinline__ V3 night_sky() { return V3{kNightSkyR, kNightSkyG, kNightSkyB}; }

__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V3 muls(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ V3 smul(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ V3 divs(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ V3 neg(V3 a) { return V3{-a.x, -a.y, -a.z}; }
// glm::dot, GLM/detail/func_geometric.inl:48-55
__device__ __forceinline__ float dot(V3 a, V3 b) { float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z; return (tx + ty) + tz; }
// glm::cross, GLM/detail/func_geometric.inl:68-80
__device__ __forceinline__ V3 cross(V3 x, V3 y) { return V3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
// ------------------------------------------------------------------------------ short reciprocals
// 1 / (double)x for a finite nonzero float x, bit-identical to the IEEE double division: v_rcp_f64 and
// two Newton steps.  The result depends only on x's 24-bit significand and exponent; every finite
// nonzero float was checked exhaustively on gfx950 (tools/verify_rcp.hip).
__device__ __forceinline__ double rcp_f64_of_f32(float x)
{
    const double b = (double)x;
    double y = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-b, y, 1.0);
    return __builtin_fma(y, e, y);
}
// 1.0f / x, bit-identical to the correctly rounded division for every float x: v_rcp_f32 and one
// Newton step where operand and result are normal (|x| in [2^-126, 2^126)), the division elsewhere
// (exhaustive check as above)
__device__ __forceinline__ float rcp_f32(float x)
{
    const float ax = __builtin_fabsf(x);
    if (ax >= 0x1p-126f && ax < 0x1p126f) {
        const float r = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    }
    return 1.0f / x;
}

#ifndef RT_DIV_ZERO_FAST
#define RT_DIV_ZERO_FAST 1
#endif
// x / d correctly rounded, from y = RN(1/d): q = RN(x * y), the exact residual r = x - q * d (one fma),
// then RN(q + r * y) -- Markstein's correction.  Checked bit for bit against the IEEE division for every
// x with 2^-100 <= |x| < 2^100 and a list of divisors (tools/verify_div.hip); div_fast takes the IEEE
// division outside that range and for divisors outside [2^-20, 2^20).
__device__ __forceinline__ float div_fast_core(float x, float d, float y)
{
    const float q = x * y;
    const float r = __builtin_fmaf(-q, d, x);
    return __builtin_fmaf(r, y, q);
}
__device__ __forceinline__ float div_fast(float x, float d, float y)
{
    const float ax = __builtin_fabsf(x), ad = __builtin_fabsf(d);
    if (ad >= 0x1p-20f && ad < 0x1p20f) {
        if (ax >= 0x1p-100f && ax < 0x1p100f) return div_fast_core(x, d, y);
#if RT_DIV_ZERO_FAST
        // a zero numerator (an occluded or back-facing direct term, a black path's fold) is common: +-0 / d is
        // +-0 with the sign of x times the sign of d, which x * y gives exactly (y = RN(1 / d) has d's sign);
        // without this a wave with one zero lane ran the IEEE division sequence too
        if (x == 0.0f) return x * y;
#endif
    }
    return x / d;
}

__device__ __forceinline__ V3 divs_fast(V3 a, float d, float y) { return V3{div_fast(a.x, d, y), div_fast(a.y, d, y), div_fast(a.z, d, y)}; }

// Every component of a in [2^-97, 2^97) or zero: (a / d1) / d2 then takes div_fast's exact path in both divisions
// for divisors d1, d2 in [2^-20, 1] (|a / d1| <= |a| * 2^20 and >= |a| stay inside [2^-100, 2^100) when
// 2^-97 <= |a| < 2^77; the fold's divisors are PDF = 1/(2 pi) and the roulette probability, so the bound used
// below is the tighter [2^-97, 2^77)).  One test per vector instead of two compares and an exec-mask branch per
// component and division.  Zero: the unsigned (bits - 1) of |a| wraps to the top.
// (LO, HI: the bit patterns of the bounds; the defaults are bits(2^-97) = 0x0F000000 and bits(2^77) = 0x66000000)
template <uint32_t LO = 0x0F000000u, uint32_t HI = 0x66000000u>
__device__ __forceinline__ bool div2_fast_range(V3 a)
{
    const uint32_t bx = __float_as_uint(a.x) & 0x7FFFFFFFu, by = __float_as_uint(a.y) & 0x7FFFFFFFu, bz = __float_as_uint(a.z) & 0x7FFFFFFFu;
    const uint32_t lo = __builtin_elementwise_min(__builtin_elementwise_min(bx - 1u, by - 1u), bz - 1u);
    const uint32_t hi = __builtin_elementwise_max(__builtin_elementwise_max(bx, by), bz);
    return lo >= LO - 1u && hi < HI;
}
// the correctly rounded 1 / d for d in [2^-20, 2^20) (rcp_f32's Newton step without its range branch)
__device__ __forceinline__ float rcp_f32_mid(float d)
{
    const float r = __builtin_amdgcn_rcpf(d);
    return __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
}
// (a / d1) / d2 by Markstein's correction in both divisions, for a inside div2_fast_range and d1, d2 in [2^-20, 1]
// (y1 = RN(1/d1), y2 = RN(1/d2)); a zero component keeps its signed-zero quotient x * y, as div_fast does
__device__ __forceinline__ float div2_core1(float x, float d1, float y1, float d2, float y2)
{
    const float q1 = x * y1;
    const float a1 = x == 0.0f ? q1 : __builtin_fmaf(__builtin_fmaf(-q1, d1, x), y1, q1);
    const float q2 = a1 * y2;
    return a1 == 0.0f ? q2 : __builtin_fmaf(__builtin_fmaf(-q2, d2, a1), y2, q2);
}
__device__ __forceinline__ V3 div2_core(V3 a, float d1, float y1, float d2, float y2)
{
    return V3{div2_core1(a.x, d1, y1, d2, y2), div2_core1(a.y, d1, y1, d2, y2), div2_core1(a.z, d1, y1, d2, y2)};
}
// one division x / d on Markstein's path, for x == 0 or 2^-100 <= |x| < 2^100 and d in [2^-20, 2^20)
// (the caller tests the ranges once, for a wave: div2_fast_range<bits(2^-100), bits(2^100)> for a vector)
__device__ __forceinline__ float div1_core(float x, float d, float y)
{
    const float q = x * y;
    return x == 0.0f ? q : __builtin_fmaf(__builtin_fmaf(-q, d, x), y, q);
}
__device__ __forceinline__ V3 div1_core(V3 a, float d, float y) { return V3{div1_core(a.x, d, y), div1_core(a.y, d, y), div1_core(a.z, d, y)}; }
constexpr uint32_t kBits2m100 = 0x0D800000u, kBits2p100 = 0x71800000u;   // bits(2^-100), bits(2^100)

// sqrt for x = +-0 or x >= 2^-96 (and +inf, NaN): the compiler's correctly rounded sequence under
// -fhip-fp32-correctly-rounded-divide-sqrt -- v_sqrt_f32, then one ulp down or up by the sign of the fma
// residual -- without its input scaling, which only inputs below 2^-96 take, and its final class test,
// which returns x for +-0 and +inf, values the sequence already gives.  Every such float gives the bits of
// __builtin_sqrtf (tools/verify_sqrt.hip checks them all); 8 instructions fewer per square root.
#ifndef RT_FAST_SQRT
#define RT_FAST_SQRT 1   // 0: __builtin_sqrtf everywhere (A/B)
#endif
__device__ __forceinline__ float sqrt_big(float x)
{
    if (!RT_FAST_SQRT) return __builtin_sqrtf(x);
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __int_as_float(__float_as_int(s) - 1);
    const float s1 = (__builtin_fmaf(-sdn, s, x) <= 0.0f) ? sdn : s;
    const float sup = __int_as_float(__float_as_int(s) + 1);
    return (__builtin_fmaf(-sup, s, x) > 0.0f) ? sup : s1;
}
// the argument range of sqrt_big
__device__ __forceinline__ bool sqrt_big_ok(float x) { return x >= 0x1p-96f || x == 0.0f; }
// sqrt(x) by sqrt_big when every active lane's x lies in its range (one wave-uniform test), else __builtin_sqrtf
__device__ __forceinline__ float sqrt_wave(float x) { return (RT_FAST_SQRT && __all(sqrt_big_ok(x))) ? sqrt_big(x) : __builtin_sqrtf(x); }

// glm::normalize = v * (1 / sqrt(dot(v,v))), GLM/detail/func_geometric.inl:82-90, func_exponential.inl:136-139
__device__ __forceinline__ V3 glm_normalize(V3 v) { float is = rcp_f32(__builtin_sqrtf(dot(v, v))); return muls(v, is); }
__device__ __forceinline__ float glm_length(V3 v) { return __builtin_sqrtf(dot(v, v)); }
// the same with sqrt_big, for vectors whose squared length is provably 0, NaN, +inf or >= 2^-96 (unit
// directions, unit normals' components), and with sqrt_wave for any vector
__device__ __forceinline__ V3 glm_normalize_big(V3 v) { float is = rcp_f32(sqrt_big(dot(v, v))); return muls(v, is); }
__device__ __forceinline__ V3 glm_normalize_wave(V3 v) { float is = rcp_f32(sqrt_wave(dot(v, v))); return muls(v, is); }
// Whitted::normalize (zero-safe), MC/VectorFloat.h:22-31
__device__ __forceinline__ V3 w_normalize(V3 v)
{
    float l2 = ((v.x * v.x) + (v.y * v.y)) + (v.z * v.z);
    if (l2 > 0.0f) { float inv = rcp_f32(__builtin_sqrtf(l2)); return V3{v.x * inv, v.y * inv, v.z * inv}; }
    return v;
}
__device__ __forceinline__ V3 w_normalize_wave(V3 v)
{
    float l2 = ((v.x * v.x) + (v.y * v.y)) + (v.z * v.z);
    if (l2 > 0.0f) { float inv = rcp_f32(sqrt_wave(l2)); return V3{v.x * inv, v.y * inv, v.z * inv}; }
    return v;
}
// std::max / std::min / glm::max / glm::min: compare-select, the first operand survives a NaN
// (MC/BoundingVolume.h:207-208); never lowered to v_max_f32 (no nnan flag without fast-math)
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }

__device__ __forceinline__ int f2i(float f) { return __float_as_int(f); }

// x / d for x < 2^24 and 1 <= d < 2^24, from rd = (float)(1 / d): (float)x is exact and the float quotient is
// within one of x / d (relative error <= 2^-23, exact for d a power of two), so one correction either way
// makes it exact -- full-rate instructions, where the generic 32-bit division is ~22 with five at quarter rate
__device__ __forceinline__ uint32_t udiv24(uint32_t x, uint32_t d, float rd)
{
    uint32_t q = (uint32_t)((float)x * rd);
    const int32_t r = (int32_t)(x - __umul24(q, d));
    if (r < 0) --q;
    else if (r >= (int32_t)d) ++q;
    return q;
}
// a * b, as a 24-bit multiply when the launch's factors are below 2^24 and its products below 2^32 (fast)
__device__ __forceinline__ uint32_t mul_u(uint32_t a, uint32_t b, uint32_t fast)
{
    return fast ? __umul24(a, b) : a * b;
}
// the launch's uniform choice: udiv24 when every dividend is below 2^24 (KParams::div24), else x / d
__device__ __forceinline__ uint32_t udiv_u(uint32_t x, uint32_t d, float rd, uint32_t fast)
{
    return fast ? udiv24(x, d, rd) : x / d;
}

constexpr float PI_F = 3.141592653589793f;            // MC/WhittedUtilities.h:20
constexpr float INTERSECTION_CORRECTION = 0.00001f;   // MC/WhittedUtilities.h:18

// ------------------------------------------------------------------------------ RNG
// Frozen stream (oracle/philox.h restates it independently): Philox4x32-10, key = seed,
// counter = (pixel, frame, dim >> 2, 0), u32 = out[dim & 3], Float = (float)u / (float)UINT32_MAX
// (Walnut::Random::Float, WN/Random.h:27-30).
#ifndef RT_PHILOX_KEY_BARRIER
#define RT_PHILOX_KEY_BARRIER 1
#endif
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t out[4])
{
    // each 32 x 32 -> 64-bit product as ONE v_mad_u64_u32 (the split __umulhi + low multiply is two
    // quarter-rate instructions)
#if RT_PHILOX_KEY_BARRIER
    // the key (uniform) through an opaque scalar move: the ten round keys are then formed here with scalar adds
    // instead of being hoisted out of the kernel's loop as loop invariants, where the path kernels kept them
    // in spilled SGPRs and read every one back with a v_readlane (a VALU slot and a hazard nop per round key)
    asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct Rng {
    uint32_t k0, k1, pixel, frame, dim;
    uint32_t blk;
    uint32_t b0, b1, b2, b3;
    // the key is set once per kernel (uniform: it stays in scalar registers), the counter per sample
    __device__ __forceinline__ void key(uint64_t seed) { k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32); }
    __device__ __forceinline__ void start(uint32_t px, uint32_t fr)
    {
        pixel = px; frame = fr; dim = 0; blk = 0xFFFFFFFFu;
    }
    __device__ __forceinline__ float next()
    {
        const uint32_t want = dim >> 2;
        if (want != blk) {
            uint32_t o[4];
            philox4x32_10(pixel, frame, want, 0u, k0, k1, o);
            b0 = o[0]; b1 = o[1]; b2 = o[2]; b3 = o[3];
            blk = want;
        }
        const uint32_t s = dim & 3u;
        const uint32_t u = s == 0 ? b0 : (s == 1 ? b1 : (s == 2 ? b2 : b3));
        ++dim;
        return (float)u / 4294967296.0f;   // (float)UINT32_MAX == 2^32 exactly
    }
};

// ------------------------------------------------------------------------------ ray / slab / MT
struct Ray {   // AccelerationStructure::Ray, MC/Ray.h:23-44
    V3 o, d, rcp;
    bool nx, ny, nz;
};
__device__ __forceinline__ Ray make_ray(V3 o, V3 d)
{
    Ray r;
    r.o = o; r.d = d;
    r.rcp = V3{rcp_f32(d.x), rcp_f32(d.y), rcp_f32(d.z)};
    r.nx = d.x < 0.0f; r.ny = d.y < 0.0f; r.nz = d.z < 0.0f;
    return r;
}

// AABB_3D::intersects_with_ray, MC/BoundingVolume.h:173-215.  Selecting the far slab for a
// negative direction before the subtraction yields exactly the swapped values.
__device__ __forceinline__ bool slab_hit(const Ray& r, float lx, float ly, float lz, float hx, float hy, float hz)
{
    const float ax = r.nx ? hx : lx, bx = r.nx ? lx : hx;
    const float ay = r.ny ? hy : ly, by = r.ny ? ly : hy;
    const float az = r.nz ? hz : lz, bz = r.nz ? lz : hz;
    const float tix = (ax - r.o.x) * r.rcp.x, tiy = (ay - r.o.y) * r.rcp.y, tiz = (az - r.o.z) * r.rcp.z;
    const float tox = (bx - r.o.x) * r.rcp.x, toy = (by - r.o.y) * r.rcp.y, toz = (bz - r.o.z) * r.rcp.z;
    const float tin = smax(tix, smax(tiy, tiz));
    const float tout = smin(tox, smin(toy, toz));
    return (tout >= 0.0f) && (tin <= tout);
}

// The same test without NaN semantics, for rays whose reciprocal direction is finite in every
// component: then no (slab - o) * rcp is NaN (0 * inf needs an infinite reciprocal), and IEEE
// max/min agree with std::max/std::min up to the sign of a zero, which the two comparisons below do
// not see.  Lowers to v_max3_f32 / v_min3_f32.
__device__ __forceinline__ bool slab_hit_finite(const Ray& r, float lx, float ly, float lz, float hx, float hy, float hz)
{
    const float ax = r.nx ? hx : lx, bx = r.nx ? lx : hx;
    const float ay = r.ny ? hy : ly, by = r.ny ? ly : hy;
    const float az = r.nz ? hz : lz, bz = r.nz ? lz : hz;
    const float tix = (ax - r.o.x) * r.rcp.x, tiy = (ay - r.o.y) * r.rcp.y, tiz = (az - r.o.z) * r.rcp.z;
    const float tox = (bx - r.o.x) * r.rcp.x, toy = (by - r.o.y) * r.rcp.y, toz = (bz - r.o.z) * r.rcp.z;
    const float tin = __builtin_fmaxf(tix, __builtin_fmaxf(tiy, tiz));
    const float tout = __builtin_fminf(tox, __builtin_fminf(toy, toz));
    return (tout >= 0.0f) && (tin <= tout);
}
// slab_hit_finite, and the box is not entered beyond `bound`: a hit whose entry t exceeds the bound
// reports a miss.  The entry t is the box's exact entry t up to 3 roundings (relative 2e-7): a caller
// passes a bound with margin above every t it must keep.
__device__ __forceinline__ bool slab_hit_finite_within(const Ray& r, float lx, float ly, float lz, float hx, float hy, float hz, float bound)
{
    const float ax = r.nx ? hx : lx, bx = r.nx ? lx : hx;
    const float ay = r.ny ? hy : ly, by = r.ny ? ly : hy;
    const float az = r.nz ? hz : lz, bz = r.nz ? lz : hz;
    const float tix = (ax - r.o.x) * r.rcp.x, tiy = (ay - r.o.y) * r.rcp.y, tiz = (az - r.o.z) * r.rcp.z;
    const float tox = (bx - r.o.x) * r.rcp.x, toy = (by - r.o.y) * r.rcp.y, toz = (bz - r.o.z) * r.rcp.z;
    const float tin = __builtin_fmaxf(tix, __builtin_fmaxf(tiy, tiz));
    const float tout = __builtin_fminf(tox, __builtin_fminf(toy, toz));
    return (tout >= 0.0f) && (tin <= tout) && (tin <= bound);
}
// slab_hit_finite_within on a box stored as its near and far planes for the ray's direction octant (the
// near-first orderings, rt_scene.cpp near_first: x planes (hi, lo) when d.x < 0, else (lo, hi), ...): the
// planes slab_hit_finite_within selects by the direction's signs, so the same subtractions, products,
// max3/min3 and compares without the six selects
__device__ __forceinline__ bool slab_nf_within(const Ray& r, float nx, float ny, float nz, float fx, float fy, float fz, float bound)
{
    const float tix = (nx - r.o.x) * r.rcp.x, tiy = (ny - r.o.y) * r.rcp.y, tiz = (nz - r.o.z) * r.rcp.z;
    const float tox = (fx - r.o.x) * r.rcp.x, toy = (fy - r.o.y) * r.rcp.y, toz = (fz - r.o.z) * r.rcp.z;
    const float tin = __builtin_fmaxf(tix, __builtin_fmaxf(tiy, tiz));
    const float tout = __builtin_fminf(tox, __builtin_fminf(toy, toz));
    return (tout >= 0.0f) && (tin <= tout) && (tin <= bound);
}
__device__ __forceinline__ bool rcp_finite(const Ray& r)
{
    return __builtin_isfinite(r.rcp.x) && __builtin_isfinite(r.rcp.y) && __builtin_isfinite(r.rcp.z);
}

// Whitted::RayTriangleIntersection, MC/TriangleMesh.h:19-45 (float cross/dot, double reciprocal
// and barycentrics, strict inequalities).  A float sign pre-test rejects exactly the cases whose
// double products cannot all be positive; a conservative |b2+b3| > |den| screen rejects cases the
// double test would reject too; survivors run the reference's double arithmetic unchanged.
__device__ __forceinline__ bool moller_trumbore_od(const V3& a, const V3& e1, const V3& e2, const V3& o, const V3& d, double& t_out)
{
    const V3 S = sub(o, a);
    const V3 S1 = cross(d, e2), S2 = cross(S, e1);
    const float den = dot(S1, e1);
    const float tn = dot(S2, e2), b2n = dot(S1, S), b3n = dot(S2, d);
    // tn, b2n, b3n share one strict sign (v_min3 / v_max3 instead of six compares and their mask logic).  A NaN
    // among them is dropped by min/max, where the compares failed at once -- the outcome is the same: a NaN
    // tn, b2n or den reaches the double stage as a NaN t or b2 and `t > 0.0` / `(1 - b2) - b3 > 0.0` fail
    const float lo3 = __builtin_fminf(__builtin_fminf(tn, b2n), b3n), hi3 = __builtin_fmaxf(__builtin_fmaxf(tn, b2n), b3n);
    if (!(lo3 > 0.0f || hi3 < 0.0f)) return false;
    const float sb = __builtin_fabsf(b2n) + __builtin_fabsf(b3n), aden = __builtin_fabsf(den);
    if (sb > aden * 1.00001f) return false;
    const double inv = rcp_f64_of_f32(den);   // == 1.0 / (double)den
    const double t = (double)tn * inv;
    t_out = t;
    // b2 > 0 and b3 > 0 follow from t > 0: tn, b2n, b3n share one strict sign (above), inv is finite
    // and nonzero or NaN (den = +-inf: NaN, t > 0 fails as the reference's t = +-0 does), and no product
    // of a nonzero float with inv underflows or overflows in double
    // ((1 - b2) - b3 > 0 decided in float away from the third edge, the double products only for a wave with a
    // lane in the band |b2 + b3 - 1| < 2^-20: C4 -1.4 %, C5 -0.4 %, C3 -0.9 % -- the ballot and branch cost
    // more than the fp64 products; tests/test_mt_edges.py keeps the edge cases; profiles/r05/ab/ab_*_mt_sure.json)
    const double b2 = (double)b2n * inv;
    const double b3 = (double)b3n * inv;
    return (t > 0.0) && (((1.0 - b2) - b3) > 0.0);
}
__device__ __forceinline__ bool moller_trumbore(const V3& a, const V3& e1, const V3& e2, const Ray& r, double& t_out)
{
    return moller_trumbore_od(a, e1, e2, r.o, r.d, t_out);
}

// Whitted::Sphere::GetIntersectionRecord (MC/Sphere.h:62-97) by Whitted::QuadraticFormula (MC/WhittedUtilities.h:36-60):
// A = dot(d, d), B = 2 dot(d, o - c), C = dot(o - c, o - c) - r^2 and the discriminant B*B - (4*A)*C in float; a
// double root -0.5*B/A and q = -0.5*(B +- sqrt(disc)) in double (the reference's double literal), each rounded to
// float as the reference assigns it; x_small = q/A, x_large = C/q in float, ordered; the nearer root unless it is
// negative, then the farther; no hit when both are.  A NaN root (only from non-finite operands) is no hit: the
// reference would return a record with t = NaN, which its t comparisons then order inconsistently.
__device__ __forceinline__ bool sphere_hit(const V3& c, float r2, const Ray& r, double& t_out)
{
    const V3 co = sub(r.o, c);
    const float A = dot(r.d, r.d);
    const float B = 2.0f * dot(r.d, co);
    const float C = dot(co, co) - r2;
    const float disc = B * B - (4.0f * A) * C;
    if (disc < 0.0f) return false;
    float xs, xl;
    if (disc == 0.0f) {
        xl = (float)((-0.5 * (double)B) / (double)A);
        xs = xl;
    } else {
        const float sq = __builtin_sqrtf(disc);
        const float q = (B > 0.0f) ? (float)(-0.5 * (double)(B + sq)) : (float)(-0.5 * (double)(B - sq));
        xs = q / A;
        xl = C / q;
    }
    if (xs > xl) { const float tmp = xs; xs = xl; xl = tmp; }
    if (xs < 0.0f) xs = xl;
    if (xs < 0.0f || xs != xs) return false;
    t_out = (double)xs;
    return true;
}

// ------------------------------------------------------------------------------ packed f32
// two floats in the halves of a register pair: v_pk_mul_f32 / v_pk_add_f32 round each half exactly like
// the scalar instruction, at half the issue cost
typedef float f2 __attribute__((ext_vector_type(2)));

// Moller-Trumbore on packed pairs (round 6, RT_MT_PK, measured slower and off: rt_coherent.hip): moller_trumbore_od's
// IEEE operations, every product and difference rounded on its own, two of them per v_pk_mul_f32 / v_pk_add_f32
// (41 -> 29 VALU for the float part).
// glm::cross(u, v) (GLM/detail/func_geometric.inl:68-80) = (u.y*v.z - v.y*u.z, u.z*v.x - v.z*u.x, u.x*v.y - v.x*u.y):
//   Q1 = u.z * (v.x, v.y) = (cy's first, cx's second product), Q2 = v.z * (u.y, u.x) = (cx's first, cy's second),
//   (cx, cy) = (Q2.lo - Q1.hi, Q1.lo - Q2.hi): one v_pk_add_f32 whose op_sel picks the halves and whose
//   neg_lo / neg_hi negate the subtrahends (RN(a + (-b)) = RN(a - b));  R = (u.x*v.y, u.y*v.x), cz = R.lo - R.hi.
// glm::dot(a, b) = (a.x*b.x + a.y*b.y) + a.z*b.z, the first two products in one v_pk_mul_f32.  The op_sel forms are
// inline asm: the compiler materialises broadcasts and swaps with moves instead.
__device__ __forceinline__ f2 pk_mul_bcast(f2 s, f2 v)        // (s.lo * v.lo, s.lo * v.hi)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(s), "v"(v));
    return r;
}
__device__ __forceinline__ f2 pk_mul_bcast_swap(f2 s, f2 v)   // (s.lo * v.hi, s.lo * v.lo)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,0]" : "=v"(r) : "v"(s), "v"(v));
    return r;
}
__device__ __forceinline__ f2 pk_mul_swap(f2 u, f2 v)         // (u.lo * v.hi, u.hi * v.lo)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(u), "v"(v));
    return r;
}
__device__ __forceinline__ f2 pk_cross_xy(f2 q2, f2 q1)       // (q2.lo - q1.hi, q1.lo - q2.hi)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[1,0]" : "=v"(r) : "v"(q2), "v"(q1));
    return r;
}
// glm::cross(u, v) for u = (uxy, uz), v = (vxy, vz.lo): (x, y) packed, z alone; vz and uz_b carry their z in .lo
__device__ __forceinline__ void pk_cross(f2 uxy, f2 uz_b, f2 vxy, f2 vz_b, f2& cxy, float& cz)
{
    cxy = pk_cross_xy(pk_mul_bcast_swap(vz_b, uxy), pk_mul_bcast(uz_b, vxy));
    const f2 r = pk_mul_swap(uxy, vxy);
    cz = r.x - r.y;
}
__device__ __forceinline__ float pk_dot(f2 axy, float az, f2 bxy, float bz)
{
    const f2 p = axy * bxy;
    return (p.x + p.y) + az * bz;
}
// moller_trumbore_od with a = t0.xyz, e1 = t1.xyz, e2 = t2.xyz (the .w words only ride in the pairs)
__device__ __forceinline__ bool moller_trumbore_pk(const float4 t0, const float4 t1, const float4 t2, const V3& o, const V3& d, double& t_out)
{
    const f2 dxy{d.x, d.y}, e1xy{t1.x, t1.y}, e2xy{t2.x, t2.y};
    const f2 e1zw{t1.z, t1.w}, e2zw{t2.z, t2.w};
    const f2 Sxy = f2{o.x, o.y} - f2{t0.x, t0.y};
    const float Sz = o.z - t0.z;
    f2 S1xy, S2xy;
    float S1z, S2z;
    pk_cross(dxy, f2{d.z, d.z}, e2xy, e2zw, S1xy, S1z);   // S1 = cross(d, e2)
    pk_cross(Sxy, f2{Sz, Sz}, e1xy, e1zw, S2xy, S2z);     // S2 = cross(S, e1)
    const float den = pk_dot(S1xy, S1z, e1xy, t1.z);
    const float tn = pk_dot(S2xy, S2z, e2xy, t2.z), b2n = pk_dot(S1xy, S1z, Sxy, Sz), b3n = pk_dot(S2xy, S2z, dxy, d.z);
    const float lo3 = __builtin_fminf(__builtin_fminf(tn, b2n), b3n), hi3 = __builtin_fmaxf(__builtin_fmaxf(tn, b2n), b3n);
    if (!(lo3 > 0.0f || hi3 < 0.0f)) return false;
    const float sb = __builtin_fabsf(b2n) + __builtin_fabsf(b3n), aden = __builtin_fabsf(den);
    if (sb > aden * 1.00001f) return false;
    const double inv = rcp_f64_of_f32(den);
    const double t = (double)tn * inv;
    t_out = t;
    const double b2 = (double)b2n * inv;
    const double b3 = (double)b3n * inv;
    return (t > 0.0) && (((1.0 - b2) - b3) > 0.0);
}

// cos/sin of the hemisphere angle phi = 2*PI*U in [0, 2*PI] (MC/WhittedMaterial.h:80-81 calls
// std::cos/std::sin(float) -> glibc cosf/sinf).  Restatement of glibc 2.35's single-precision
// algorithm (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h; ARM optimized-routines):
// double-precision Cody-Waite style reduction by pi/2 (`reduce_fast`, 0 <= x < 120) and two
// polynomials, one rounding to float.  Verified bit-identical to glibc's sinf/cosf for every float
// in [0, 2*PI] (both its FMA and non-FMA builds), see tests/test_device_trig.py.
namespace glibc_trig {
constexpr double S1 = -0x1.555545995a603p-3, S2 = 0x1.1107605230bc4p-7, S3 = -0x1.994eb3774cf24p-13;
constexpr double C0 = 0x1p0, C1 = -0x1.ffffffd0c621cp-2, C2 = 0x1.55553e1068f19p-5, C3 = -0x1.6c087e89a359dp-10,
                 C4 = 0x1.99343027bf8c3p-16;
constexpr double HPI_INV = 0x1.45F306DC9C883p+23, HPI = 0x1.921FB54442D18p0;
__device__ __forceinline__ uint32_t top12(float x) { return ((uint32_t)__float_as_int(x) >> 20) & 0x7ffu; }
// sinf_poly: odd n -> cosine polynomial, even n -> sine polynomial
__device__ __forceinline__ double poly(double x, double x2, int n)
{
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = S2 + x2 * S3;
        const double x7 = x3 * x2;
        const double s = x + x3 * S1;
        return s + x7 * s1;
    }
    const double x4 = x2 * x2;
    const double c2 = C3 + x2 * C4;
    const double c1 = C0 + x2 * C1;
    const double x6 = x4 * x2;
    const double c = c1 + x4 * C2;
    return c + x6 * c2;
}
// x in [0, 120): quadrant n and reduced argument (reduce_fast)
__device__ __forceinline__ double reduce(double x, int& n)
{
    const double r = x * HPI_INV;
    n = ((int32_t)r + 0x800000) >> 24;
    return x - (double)n * HPI;
}
}  // namespace glibc_trig

__device__ __forceinline__ float cos_f(float y)
{
    using namespace glibc_trig;
    double x = y;
    if (top12(y) < top12(0x1.921FB6p-1f)) {   // |y| < pi/4
        if (top12(y) < top12(0x1p-12f)) return 1.0f;
        return (float)poly(x, x * x, 1);
    }
    int n;
    x = reduce(x, n);
    const double s = (n & 2) ? ((n & 1) ? 1.0 : -1.0) : ((n & 1) ? -1.0 : 1.0);   // sign[n & 3] = {1,-1,-1,1}
    double r = poly(x * s, x * x, n ^ 1);
    if (((n ^ 1) & 1) && (n & 2)) r = -r;   // second table: negated cosine coefficients
    return (float)r;
}

__device__ __forceinline__ float sin_f(float y)
{
    using namespace glibc_trig;
    double x = y;
    if (top12(y) < top12(0x1.921FB6p-1f)) {
        if (top12(y) < top12(0x1p-12f)) return y;
        return (float)poly(x, x * x, 0);
    }
    int n;
    x = reduce(x, n);
    const double s = (n & 2) ? ((n & 1) ? 1.0 : -1.0) : ((n & 1) ? -1.0 : 1.0);
    double r = poly(x * s, x * x, n);
    if ((n & 1) && (n & 2)) r = -r;
    return (float)r;
}

// cos_f(y) and sin_f(y) together, branch-free: one reduction, each polynomial once (cos_f and sin_f
// evaluate the same two polynomials of the same reduced argument and pick / negate by the quadrant).
__device__ __forceinline__ void sincos_f(float y, float& c, float& s)
{
    using namespace glibc_trig;
    const double x = y;
    const bool small = top12(y) < top12(0x1.921FB6p-1f);   // |y| < pi/4: no reduction, n = 0
    int nr;
    const double xr0 = reduce(x, nr);
    const int n = small ? 0 : nr;
    const double xr = small ? x : xr0;
    const double sg = (n & 2) ? ((n & 1) ? 1.0 : -1.0) : ((n & 1) ? -1.0 : 1.0);   // sign[n & 3]
    const double x2 = xr * xr;
    const double ps = poly(xr * sg, x2, 0), pc = poly(xr * sg, x2, 1);
    const double npc = (n & 2) ? -pc : pc;
    double rc = (n & 1) ? ps : npc;
    double rs = (n & 1) ? npc : ps;
    float fc = (float)rc, fs = (float)rs;
    if (top12(y) < top12(0x1p-12f)) { fc = 1.0f; fs = y; }   // the tiny-argument returns
    c = fc;
    s = fs;
}

// powf of the specular lobe (WH/Renderer.h:287-292: std::powf -> glibc powf).  Evaluated as
// exp(y * log(x)) in double and rounded once to float: correctly rounded except within ~1e-15 of a
// rounding boundary, as glibc's powf (double-precision log2/exp2 core) is; x >= 0 here.
__device__ __forceinline__ float pow_lobe(float x, float y)
{
    if (x == 0.0f) return (y > 0.0f) ? 0.0f : ((y == 0.0f) ? 1.0f : __builtin_inff());
    if (x == 1.0f || y == 0.0f) return 1.0f;
    return (float)exp((double)y * log((double)x));
}

__device__ __forceinline__ uint32_t to_u8(float v)
{   // (uint8_t)(c * 255.0f), MC/Renderer.cpp:17-20 (v in [0,1] after clamp; NaN -> 0 like x86 cvttss2si)
    const float f = v * 255.0f;
    if (!(f == f)) return 0u;
    return ((uint32_t)(int32_t)f) & 0xFFu;
}

// glm mat4 * vec4, GLM/detail/type_mat4x4.inl:561-572: (m0*v0 + m1*v1) + (m2*v2 + m3*v3); m column-major
template <class PF>
__device__ __forceinline__ void mat4_mul(PF m, float v0, float v1, float v2, float v3, float out[4])
{
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float mul0 = m[0 + i] * v0, mul1 = m[4 + i] * v1, mul2 = m[8 + i] * v2, mul3 = m[12 + i] * v3;
        const float add0 = mul0 + mul1, add1 = mul2 + mul3;
        out[i] = add0 + add1;
    }
}

}  // namespace rtd
#endif
