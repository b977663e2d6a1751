// tools/calib_gather.hip -- the vector-memory rate of the BVH walk's access shape: every lane of a wave
// loads its own 16-byte record (a BVH node half, a triangle quad) from a table the size of C5's scene,
// so no two lanes share a cache line.  Measures lane-loads per second (and per CU-clock) for
//   * independent loads (each lane K loads whose addresses do not depend on each other): the issue /
//     tag-lookup ceiling of the L1 (TA/TCP) and the L2 behind it;
//   * dependent chains (the next address from the loaded value, as a walk's next node): latency-bound;
//   * 32-byte records read as two 16-byte loads (the walk's AoS node) against one 16-byte load;
// at table sizes inside L1 (16 KiB), inside one XCD's L2 (2 MiB), C5's scene (10 MiB) and beyond the L2s
// (64 MiB), with 8 waves per SIMD like the vertex kernel.  One JSON line per case.
//   hipcc -O3 --offload-arch=gfx950 tools/calib_gather.hip -o tools/_calib_gather && tools/_calib_gather
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// independent: K loads per lane at hashed addresses (mask + 1 = records, a power of two)
template <int REC>
__global__ void __launch_bounds__(256) k_indep(const float4* __restrict__ t, uint32_t mask, uint32_t K, float* __restrict__ out)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.0f;
    for (uint32_t k = 0; k < K; k += 4) {
        float4 v[4][REC];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = mix(g * 0x9E3779B9u + (k + u)) & mask;
#pragma unroll
            for (int r = 0; r < REC; ++r) v[u][r] = t[(size_t)i * REC + r];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int r = 0; r < REC; ++r) acc += v[u][r].x;
    }
    if (acc == -1.0f) out[g] = acc;   // never: keeps the loads
}

// dependent: the next record's index comes from the loaded one (a pointer chase per lane)
template <int REC>
__global__ void __launch_bounds__(256) k_chase(const float4* __restrict__ t, uint32_t mask, uint32_t K, float* __restrict__ out)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t i = mix(g) & mask;
    float acc = 0.0f;
    for (uint32_t k = 0; k < K; ++k) {
        float4 v[REC];
#pragma unroll
        for (int r = 0; r < REC; ++r) v[r] = t[(size_t)i * REC + r];
        i = (__float_as_uint(v[0].w) + k) & mask;
#pragma unroll
        for (int r = 0; r < REC; ++r) acc += v[r].x;
    }
    if (acc == -1.0f) out[g] = acc;
}

__global__ void k_fill(float4* t, uint32_t n, uint32_t mask)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        t[i] = make_float4(1.0f, 2.0f, 3.0f, __uint_as_float(mix(i * 2654435761u) & mask));
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } } while (0)

int main()
{
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const double clk_hz = prop.clockRate * 1e3;
    const size_t max_bytes = 64ull << 20;
    float4* t;
    float* out;
    CK(hipMalloc(&t, max_bytes));
    CK(hipMalloc(&out, 4));
    const dim3 block(256), grid(cus * 8);   // 8 blocks of 4 waves per CU = 8 waves per SIMD
    const uint32_t lanes = grid.x * block.x;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const size_t sizes[] = {16ull << 10, 2ull << 20, 10ull << 20, 64ull << 20};
    for (size_t bytes : sizes) {
        for (int rec = 1; rec <= 2; ++rec) {
            const uint32_t records = (uint32_t)(bytes / (16 * rec));
            uint32_t p2 = 1;
            while (p2 * 2 <= records) p2 *= 2;
            const uint32_t mask = p2 - 1;
            hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, t, (uint32_t)(bytes / 16), mask);
            CK(hipDeviceSynchronize());
            for (int dep = 0; dep < 2; ++dep) {
                const uint32_t K = dep ? 64 : 256;
                float ms = 0.0f;
                for (int rep = 0; rep < 3; ++rep) {
                    CK(hipEventRecord(a, 0));
                    if (dep) {
                        if (rec == 1) hipLaunchKernelGGL(k_chase<1>, grid, block, 0, 0, t, mask, K, out);
                        else hipLaunchKernelGGL(k_chase<2>, grid, block, 0, 0, t, mask, K, out);
                    } else {
                        if (rec == 1) hipLaunchKernelGGL(k_indep<1>, grid, block, 0, 0, t, mask, K, out);
                        else hipLaunchKernelGGL(k_indep<2>, grid, block, 0, 0, t, mask, K, out);
                    }
                    CK(hipEventRecord(b, 0));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));   // the last of 3 (warm)
                }
                const double lane_loads = (double)lanes * K * rec;
                const double per_s = lane_loads / (ms * 1e-3);
                printf("{\"table_bytes\": %zu, \"record_bytes\": %d, \"pattern\": \"%s\", \"ms\": %.3f, \"lane_loads_per_ns\": %.1f, "
                       "\"lane_loads_per_cu_clk\": %.3f, \"records_per_cu_clk\": %.3f, \"clock_ghz\": %.2f}\n",
                       bytes, 16 * rec, dep ? "dependent" : "independent", ms, per_s * 1e-9, per_s / (cus * clk_hz),
                       per_s / rec / (cus * clk_hz), clk_hz * 1e-9);
                fflush(stdout);
            }
        }
    }
    return 0;
}
