// rt_kernels.h -- launch interface between the C-ABI layer (rt_capi.cpp) and the HIP kernels.
#ifndef RT_KERNELS_H
#define RT_KERNELS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

struct KParams {
    // scene (rt_layout.h)
    const float4* nodes; uint32_t n_nodes;
    const float4* tris;
    const float4* mats;
    const float4* lnodes;
    const float4* ltris;
    float light_area; float light_emission[3]; int has_light;
    // camera: position, inverse projection, inverse view (column-major glm mat4)
    float cam_pos[3]; float iproj[16]; float iview[16];
    // image and sampling
    uint32_t W, H;
    uint32_t first_frame, n_frames;
    uint64_t seed; float rr;
    // pixels of this device: row bands of `band` rows dealt round-robin over `nranks`
    uint32_t band, rank, nranks, n_local_rows;
    uint32_t tiles_x; uint32_t n_items;
    // outputs (compact local pixel order: local_row * W + x)
    float4* accum; uint32_t* rgba;
    // scratch
    uint32_t* work_counter;
    float4* stack_ld; int32_t* stack_mat; uint32_t stack_depth; uint32_t total_threads;
    unsigned long long* counters;   // [node_tests, tri_tests, rays, stack_overflow]
};

hipError_t rt_launch_megakernel(const KParams& P, bool exact, bool count, uint32_t grid, uint32_t block, hipStream_t stream);
hipError_t rt_launch_trace(const KParams& P, uint32_t n, const float* org, const float* dir, int32_t* tri, double* t, hipStream_t stream);
int rt_megakernel_occupancy(bool exact, bool count, int block);
hipError_t rt_launch_math(uint32_t n, const float* x, float* out, hipStream_t stream);

#endif
