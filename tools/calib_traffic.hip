// tools/calib_traffic.hip -- known-byte kernels for the L2 -> fabric request counters (the rocprofv3
// FETCH_SIZE / WRITE_SIZE inputs and their per-size splits TCC_EA0_RDREQ_{32B,64B,128B},
// TCC_EA0_WRREQ_64B).  Each kernel moves a known number of bytes in one access shape of the vertex
// kernel's scratch traffic (csrc/rt_coherent.hip); profiles/run_rocprof.sh profiles this program with
// the same counter passes as the bench, and profiles/summarize_pmc.py prints counted / known bytes.
//   hipcc -O3 --offload-arch=gfx950 tools/calib_traffic.hip -o tools/_calib_traffic && tools/_calib_traffic
// Footprints exceed the 256 MiB Infinity Cache so that nothing is served from it twice.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// wide coalesced stream: 16 B per lane read and written
__global__ void k_stream_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// the parked-sample shape: one float3 (12 B) per pixel into 48-byte 4-frame blocks, frame f of the
// block per launch; `stagger` puts neighbouring lanes at different frames (as lanes of a wave are)
__global__ void k_park12(float* __restrict__ lbuf, size_t px, uint32_t f, uint32_t stagger)
{
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < px; p += (size_t)gridDim.x * blockDim.x) {
        const uint32_t fr = stagger ? (uint32_t)((f + p) & 3u) : f;
        float* d = lbuf + p * 12 + fr * 3;
        d[0] = 1.0f; d[1] = 2.0f; d[2] = 3.0f;
    }
}

// the parked-sample read of finalize_chunks_kernel: a pixel's 48-byte block read by its lane
__global__ void k_read48(const float4* __restrict__ lbuf, float* __restrict__ out, size_t px)
{
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < px; p += (size_t)gridDim.x * blockDim.x) {
        const float4 x = lbuf[3 * p], y = lbuf[3 * p + 1], z = lbuf[3 * p + 2];
        const float s = x.x + x.y + x.z + x.w + y.x + y.y + y.z + y.w + z.x + z.y + z.z + z.w;
        if (s == -1.0f) out[p] = s;   // never true: keeps the loads
    }
}

// the fold-ring shape ([thread][position], 16-byte levels): each lane reads one level and writes the next
__global__ void k_ring16(float4* __restrict__ ring, size_t lanes, uint32_t stride, uint32_t at)
{
    for (size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x; l < lanes; l += (size_t)gridDim.x * blockDim.x) {
        float4 v = ring[l * stride + at];
        v.x += 1.0f;
        ring[l * stride + at + 1] = v;
    }
}

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(x), __LINE__); return 2; } } while (0)

int main()
{
    const dim3 grid(4096), block(256);
    // 1 GiB stream
    const size_t n4 = (1ull << 30) / 16;
    float4 *a, *b;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, n4 * 16));
    CK(hipMemset(a, 0, n4 * 16));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_stream_copy, grid, block, 0, 0, a, b, n4);
    CK(hipDeviceSynchronize());
    CK(hipFree(a));
    CK(hipFree(b));
    // parked samples: 2^24 pixels x 48 B = 768 MiB, written in 4 launches of 12 B per pixel, aligned then staggered
    const size_t px = 1ull << 24;
    float* lbuf;
    float* out;
    CK(hipMalloc(&lbuf, px * 48));
    CK(hipMalloc(&out, px * 4));
    CK(hipDeviceSynchronize());
    for (uint32_t f = 0; f < 4; ++f) hipLaunchKernelGGL(k_park12, grid, block, 0, 0, lbuf, px, f, 0u);
    CK(hipDeviceSynchronize());
    for (uint32_t f = 0; f < 4; ++f) hipLaunchKernelGGL(k_park12, grid, block, 0, 0, lbuf, px, f, 1u);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_read48, grid, block, 0, 0, (const float4*)lbuf, out, px);
    CK(hipDeviceSynchronize());
    CK(hipFree(lbuf));
    CK(hipFree(out));
    // ring: 2^20 lanes x 192 positions x 16 B = 3 GiB, one 16-byte read + one 16-byte write per lane
    const size_t lanes = 1ull << 20;
    float4* ring;
    CK(hipMalloc(&ring, lanes * 192 * 16));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_ring16, grid, block, 0, 0, ring, lanes, 192u, 5u);
    CK(hipDeviceSynchronize());
    CK(hipFree(ring));
    printf("{\"k_stream_copy\": {\"read\": %zu, \"write\": %zu}, \"k_park12\": {\"write_per_launch\": %zu}, "
           "\"k_read48\": {\"read\": %zu}, \"k_ring16\": {\"read\": %zu, \"write\": %zu}}\n",
           n4 * 16, n4 * 16, px * 12, px * 48, lanes * 16, lanes * 16);
    return 0;
}
