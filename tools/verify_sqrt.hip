// tools/verify_sqrt.hip -- exhaustive check of rt_device.h sqrt_big (the correctly rounded square root
// without the input scaling and class test) against __builtin_sqrtf as the kernels compile it
// (-fhip-fp32-correctly-rounded-divide-sqrt): EVERY float bit pattern in sqrt_big's range -- +-0 and all
// of [2^-96, +inf] with both NaN ranges, i.e. every pattern except the positive and negative values below
// 2^-96 other than zero -- must give identical bits.  Build + run (GPU):
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -fno-gpu-flush-denormals-to-zero -Icpu-based-ray-tracer_amd/csrc tools/verify_sqrt.hip -o /tmp/verify_sqrt && /tmp/verify_sqrt
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "rt_device.h"

__global__ void check(uint64_t base, unsigned long long* bad, unsigned long long* checked, unsigned long long* first)
{
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > 0xFFFFFFFFull) return;
    const float x = __uint_as_float((uint32_t)i);
    const bool in = rtd::sqrt_big_ok(x) || __builtin_isnan(x);
    const bool miss = in && __float_as_uint(rtd::sqrt_big(x)) != __float_as_uint(__builtin_sqrtf(x));
    const unsigned long long m = __ballot(miss), c = __ballot(in);
    if (__lane_id() == 0) {
        if (m) atomicAdd(bad, (unsigned long long)__popcll(m));
        atomicAdd(checked, (unsigned long long)__popcll(c));
    }
    if (miss) atomicCAS(first, 0ull, 0x100000000ull | (uint32_t)i);
}

int main()
{
    unsigned long long *bad, *checked, *first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&checked, 8) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(checked, 0, 8);
    (void)hipMemset(first, 0, 8);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad, checked, first);
    unsigned long long h = 0, c = 0, f = 0;
    if (hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(&c, checked, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&f, first, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return 3;
    printf("{\"patterns_checked\": %llu, \"mismatches\": %llu, \"first_mismatch_bits\": \"%08llx\"}\n", c, h, f & 0xFFFFFFFFull);
    return h == 0 ? 0 : 1;
}
