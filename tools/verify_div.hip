// tools/verify_div.hip -- exhaustive check of the short correctly rounded f32 division (rt_device.h
// div_fast: y = RN(1/d) by rcp_f32, q = RN(x*y), r = fma(-q, d, x), RN(q + r*y) -- Markstein's
// correction) against the IEEE division the kernels compiled with -fhip-fp32-correctly-rounded-divide-sqrt
// use.  For each divisor d of a list (the path tracer's constant PDF = 1/(2*PI), Russian-roulette
// probabilities, random floats), EVERY float x with 2^-100 <= |x| < 2^100 (the range where div_fast is
// used; outside it the kernels take the IEEE division) is checked bit for bit.  Build + run (GPU):
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -fno-gpu-flush-denormals-to-zero tools/verify_div.hip -o /tmp/verify_div && /tmp/verify_div [N_RANDOM_DIVISORS] [PAIR_CHUNKS]
// A second pass checks div_fast with a per-lane divisor (y = rcp_f32(d)) on PAIR_CHUNKS x 2^28 random
// (x, d) pairs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../cpu-based-ray-tracer_amd/csrc/rt_device.h"

__global__ void check(float d, uint64_t base, unsigned long long* bad, unsigned long long* first)
{
    // x enumerates the biased exponents [27, 227) x all mantissas x both signs
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t sign = (uint32_t)(i & 1u), rest = (uint32_t)(i >> 1);
    const uint32_t mant = rest & 0x7FFFFFu, e = 27u + (rest >> 23);
    if (e >= 227u) return;
    const float x = __uint_as_float((sign << 31) | (e << 23) | mant);
    const float ref = x / d;
    const float got = rtd::div_fast_core(x, d, rtd::rcp_f32(d));
    const bool miss = __float_as_uint(ref) != __float_as_uint(got);
    const unsigned long long m = __ballot(miss);
    if (__lane_id() == 0 && m) atomicAdd(bad, (unsigned long long)__popcll(m));
    if (miss) atomicCAS(first, 0ull, ((unsigned long long)__float_as_uint(x) << 32) | __float_as_uint(d));
}

// per-lane divisors: random (x, d) pairs, d in [2^-20, 2^20), x in the fast range (a Philox-style hash of
// the index picks both)
__global__ void check_pairs(uint64_t base, unsigned long long* bad)
{
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t o[4];
    rtd::philox4x32_10((uint32_t)i, (uint32_t)(i >> 32), 77u, 0u, 0x1234u, 0x5678u, o);
    const uint32_t ed = 107u + o[0] % 40u, ex = 27u + o[1] % 200u;
    const float d = __uint_as_float(((o[2] & 1u) << 31) | (ed << 23) | (o[2] >> 9));
    const float x = __uint_as_float(((o[3] & 1u) << 31) | (ex << 23) | (o[3] >> 9));
    const bool miss = __float_as_uint(x / d) != __float_as_uint(rtd::div_fast(x, d, rtd::rcp_f32(d)));
    const unsigned long long m = __ballot(miss);
    if (__lane_id() == 0 && m) atomicAdd(bad, (unsigned long long)__popcll(m));
}

int main(int argc, char** argv)
{
    const int n_random = argc > 1 ? atoi(argv[1]) : 64;
    float ds[1024];
    int nd = 0;
    ds[nd++] = 1.0f / (2.0f * 3.141592653589793f);   // WhittedMaterial::PDF_at_the_sample
    const float rr[] = {0.8f, 0.9f, 0.5f, 0.99f, 0.95f, 0.7f, 0.6f, 0.3f, 0.1f, 0.999f, 0.25f, 1.0f / 3.0f, 0.875f, 0.75f};
    for (float v : rr) ds[nd++] = v;
    uint32_t s = 12345u;
    for (int k = 0; k < n_random && nd < 1024; ++k) {   // random significands, exponents in [2^-20, 2^20]
        s = s * 1664525u + 1013904223u;
        const uint32_t mant = s >> 9;
        s = s * 1664525u + 1013904223u;
        const uint32_t e = 107u + (s >> 24) % 40u;
        ds[nd++] = __builtin_bit_cast(float, (e << 23) | mant);
    }
    ds[nd++] = __builtin_bit_cast(float, 0x3F7FFFFFu);   // significand all ones
    ds[nd++] = __builtin_bit_cast(float, 0x3F800001u);
    unsigned long long *bad, *first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 2;
    unsigned long long total = 0;
    const uint64_t count = 200ull << 24;   // exponents x mantissas x signs
    const uint64_t chunk = 1ull << 28;
    for (int k = 0; k < nd; ++k) {
        (void)hipMemset(bad, 0, 8);
        (void)hipMemset(first, 0, 8);
        for (uint64_t base = 0; base < count; base += chunk)
            hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, ds[k], base, bad, first);
        unsigned long long h = 0, f = 0;
        if (hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(&f, first, 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
        total += h;
        if (h) printf("divisor %a (%08x): %llu mismatches, first x bits %08llx\n", (double)ds[k], __builtin_bit_cast(uint32_t, ds[k]), h, f >> 32);
    }
    const int pair_chunks = argc > 2 ? atoi(argv[2]) : 64;   // x 2^28 random pairs
    (void)hipMemset(bad, 0, 8);
    for (int k = 0; k < pair_chunks; ++k)
        hipLaunchKernelGGL(check_pairs, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, (uint64_t)k * chunk, bad);
    unsigned long long hp = 0;
    if (hipMemcpy(&hp, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("{\"divisors\": %d, \"inputs_per_divisor\": %llu, \"mismatches\": %llu, \"random_pairs\": %llu, \"pair_mismatches\": %llu}\n", nd,
           (unsigned long long)count, total, (unsigned long long)pair_chunks * chunk, hp);
    return (total == 0 && hp == 0) ? 0 : 1;
}
