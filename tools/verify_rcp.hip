// tools/verify_rcp.hip -- exhaustive check of short reciprocal sequences against the correctly rounded
// division the kernels use today (gfx950).  For every float x (all 2^32 bit patterns, finite and
// nonzero) it compares, bit for bit:
//   f64: 1.0 / (double)x            vs  v_rcp_f64 + Newton steps        (Moller-Trumbore's 1/den)
//   f32: 1.0f / x (correctly rounded) vs  v_rcp_f32 + one Newton step     (ray reciprocals, 1/sqrt)
// and reports the mismatch count per candidate.  Build + run (GPU):
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -fno-gpu-flush-denormals-to-zero tools/verify_rcp.hip -o /tmp/verify_rcp && /tmp/verify_rcp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../cpu-based-ray-tracer_amd/csrc/rt_device.h"

// one atomic per wave: count the lanes whose candidate differs
__device__ __forceinline__ void tally(bool miss, unsigned long long* slot)
{
    const unsigned long long m = __ballot(miss);
    if (__lane_id() == 0 && m) atomicAdd(slot, (unsigned long long)__popcll(m));
}

__global__ void check(uint64_t base, unsigned long long* bad)
{
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t u = (uint32_t)i;
    const float x = __uint_as_float(u);
    const bool valid = __builtin_isfinite(x) && x != 0.0f;
    // f64 reciprocal of a float
    const double b = (double)x;
    const double ref = 1.0 / b;
    double y = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    const double y1 = y;                 // one Newton step
    e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);          // two Newton steps
    const double y2 = y;
    tally(valid && (__double_as_longlong(y1) != __double_as_longlong(ref)), &bad[0]);
    tally(valid && (__double_as_longlong(y2) != __double_as_longlong(ref)), &bad[1]);
    tally(valid && (__double_as_longlong(rtd::rcp_f64_of_f32(x)) != __double_as_longlong(ref)), &bad[4]);
    // f32 reciprocal
    const float rf = 1.0f / x;
    float r = __builtin_amdgcn_rcpf(x);
    const float ef = __builtin_fmaf(-x, r, 1.0f);
    const float r1 = __builtin_fmaf(ef, r, r);
    tally(valid && (__float_as_uint(r1) != __float_as_uint(rf)), &bad[2]);
    tally(valid && (__float_as_uint((float)(1.0 / b)) != __float_as_uint(rf)), &bad[3]);   // sanity: double-rounded
    tally(valid && (__float_as_uint(rtd::rcp_f32(x)) != __float_as_uint(rf)), &bad[5]);
    // the raw one-step sequence restricted to |x| in [2^-126, 2^126) (normal operand and result)
    const float ax = __builtin_fabsf(x);
    const bool mid = ax >= 0x1p-126f && ax < 0x1p126f;
    tally(valid && mid && (__float_as_uint(r1) != __float_as_uint(rf)), &bad[6]);
    tally(valid && !mid, &bad[7]);
}

int main()
{
    unsigned long long* bad;
    if (hipMalloc(&bad, 8 * sizeof(unsigned long long)) != hipSuccess) return 2;
    if (hipMemset(bad, 0, 8 * sizeof(unsigned long long)) != hipSuccess) return 2;
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad);
    unsigned long long h[8];
    if (hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("{\"f64_rcp_1nr\": %llu, \"f64_rcp_2nr\": %llu, \"f32_rcp_1nr\": %llu, \"f32_via_f64_div\": %llu, "
           "\"rcp_f64_of_f32\": %llu, \"rcp_f32\": %llu, \"f32_rcp_1nr_normal_range\": %llu, \"outside_normal_range\": %llu, "
           "\"inputs\": 4278190078}\n",
           h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
    return (h[4] == 0 && h[5] == 0) ? 0 : 1;
}
