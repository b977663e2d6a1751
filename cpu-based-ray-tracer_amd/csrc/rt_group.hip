// rt_group.hip -- several GPUs rendering one frame (include/rt_capi.h, "several GPUs, one frame").
//
// The reference renders a frame with a std::execution::par loop over rows (MC/Renderer.cpp:100-110).
// Here the rows are dealt to the group's members in bands (rt_resize's band / rank / nranks): each
// member renders its band set in one persistent launch on its own device and stream, then the RGBA8
// band sets travel to member 0 -- one ncclGather per member issued as one RCCL group when the devices
// are distinct (xGMI), device-to-device copies otherwise -- and a small kernel on member 0 puts every
// row back at its global position.  The gather moves 4 bytes per pixel (8.3 MB at 1920x1080): well
// under a millisecond over xGMI against a ~50 ms band render at 8 GPUs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rt_capi.h"
#include "rt_knobs.h"

struct rt_group {
    std::vector<int> dev;
    std::vector<rt_ctx*> m;
    std::vector<hipStream_t> st;     // one per member, owned (handed to rt_create)
    std::vector<ncclComm_t> comm;    // RCCL gather: one communicator per member
    bool rccl = false;
    std::string err;
    uint32_t W = 0, H = 0, band = 8, max_rows = 0;
    std::vector<uint32_t> rows;      // local rows per member
    std::vector<uint32_t*> send;     // RCCL: per member, max_rows x W (ncclGather sends equal counts)
    std::vector<hipEvent_t> ready;   // copy path: member i's band set is complete
    uint32_t* d_gath = nullptr;      // member 0: n x max_rows x W
    uint32_t* d_frame = nullptr;     // member 0: W x H
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool pending = false;
    float last_ms = 0.0f, max_kernel_ms = 0.0f;
};

namespace {

__global__ void __launch_bounds__(256) assemble_rows_kernel(const uint32_t* __restrict__ gath, uint32_t* __restrict__ frame, uint32_t W,
                                                            uint32_t H, uint32_t band, uint32_t n, uint32_t max_rows)
{
    // global row y belongs to member (y / band) mod n, at its local row ((y / band) / n) * band + y mod band
    const uint64_t total = (uint64_t)W * H;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t y = (uint32_t)(i / W), x = (uint32_t)(i - (uint64_t)y * W);
        const uint32_t b = y / band, k = b % n, lr = (b / n) * band + (y - b * band);
        frame[i] = gath[((uint64_t)k * max_rows + lr) * W + x];
    }
}

uint32_t local_rows(uint32_t H, uint32_t band, uint32_t rank, uint32_t n)
{
    uint32_t r = 0;
    for (uint32_t b = rank; (uint64_t)b * band < H; b += n) r += std::min(band, H - b * band);
    return r;
}

rt_status fail(rt_group* g, rt_status s, const std::string& what)
{
    g->err = what;
    return s;
}

#define GHIP(g, call)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) return fail(g, RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorName(e_)); \
    } while (0)
#define GNCCL(g, call)                                                                             \
    do {                                                                                           \
        ncclResult_t r_ = (call);                                                                  \
        if (r_ != ncclSuccess) return fail(g, RT_ERR_HIP, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)
#define GMEM(g, i, call)                                                                           \
    do {                                                                                           \
        rt_status s_ = (call);                                                                     \
        if (s_ != RT_OK) return fail(g, s_, "member " + std::to_string(i) + ": " + rt_last_error(g->m[i])); \
    } while (0)

void free_buffers(rt_group* g)
{
    for (size_t i = 0; i < g->send.size(); ++i)
        if (g->send[i]) { (void)hipSetDevice(g->dev[i]); (void)hipFree(g->send[i]); }
    g->send.assign(g->dev.size(), nullptr);
    (void)hipSetDevice(g->dev[0]);
    if (g->d_gath) (void)hipFree(g->d_gath);
    if (g->d_frame) (void)hipFree(g->d_frame);
    g->d_gath = nullptr; g->d_frame = nullptr;
}

}  // namespace

extern "C" {

rt_status rt_group_create(rt_group** out, const int32_t* devices, uint32_t n)
{
    if (!out || !devices || n == 0 || n > 64) return RT_ERR_INVALID;
    *out = nullptr;
    rt_group* g = new (std::nothrow) rt_group();
    if (!g) return RT_ERR_OOM;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= count) { delete g; return RT_ERR_INVALID; }
    g->dev.assign(devices, devices + n);
    g->m.assign(n, nullptr);
    g->st.assign(n, nullptr);
    g->ready.assign(n, nullptr);
    g->send.assign(n, nullptr);
    auto cleanup = [&](rt_status s) { rt_group_destroy(g); return s; };
    for (uint32_t i = 0; i < n; ++i) {
        if (hipSetDevice(g->dev[i]) != hipSuccess || hipStreamCreateWithFlags(&g->st[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&g->ready[i], hipEventDisableTiming) != hipSuccess)
            return cleanup(RT_ERR_HIP);
        rt_device_cfg cfg{g->dev[i], (void*)g->st[i], 0};
        if (rt_create(&g->m[i], &cfg) != RT_OK) return cleanup(RT_ERR_HIP);
    }
    if (hipSetDevice(g->dev[0]) != hipSuccess || hipEventCreate(&g->e0) != hipSuccess || hipEventCreate(&g->e1) != hipSuccess)
        return cleanup(RT_ERR_HIP);
    // RCCL takes one rank per GPU: the gather is a collective only when the devices are distinct
    std::vector<int> sorted(g->dev);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const char* mode = rt_knob("RT_GROUP_GATHER");
    g->rccl = distinct && !(mode && std::strcmp(mode, "copy") == 0);
    if (g->rccl) {
        g->comm.assign(n, nullptr);
        if (ncclCommInitAll(g->comm.data(), (int)n, g->dev.data()) != ncclSuccess) {
            g->comm.clear();
            g->rccl = false;   // no RCCL on this node: copies over xGMI instead
        }
    }
    *out = g;
    return RT_OK;
}

void rt_group_destroy(rt_group* g)
{
    if (!g) return;
    for (size_t i = 0; i < g->st.size(); ++i)
        if (g->st[i]) { (void)hipSetDevice(g->dev[i]); (void)hipStreamSynchronize(g->st[i]); }
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    free_buffers(g);
    for (size_t i = 0; i < g->m.size(); ++i) {
        if (g->m[i]) rt_destroy(g->m[i]);
        (void)hipSetDevice(g->dev[i]);
        if (g->ready[i]) (void)hipEventDestroy(g->ready[i]);
        if (g->st[i]) (void)hipStreamDestroy(g->st[i]);
    }
    if (!g->dev.empty()) (void)hipSetDevice(g->dev[0]);
    if (g->e0) (void)hipEventDestroy(g->e0);
    if (g->e1) (void)hipEventDestroy(g->e1);
    delete g;
}

const char* rt_group_last_error(const rt_group* g) { return g ? g->err.c_str() : "null group"; }
uint32_t rt_group_size(const rt_group* g) { return g ? (uint32_t)g->m.size() : 0; }
rt_ctx* rt_group_member(rt_group* g, uint32_t i) { return g && i < g->m.size() ? g->m[i] : nullptr; }

rt_status rt_group_upload_scene(rt_group* g, const rt_scene* s)
{
    if (!g || !s) return RT_ERR_INVALID;
    for (size_t i = 0; i < g->m.size(); ++i) GMEM(g, i, rt_upload_scene(g->m[i], s));
    return RT_OK;
}

rt_status rt_group_resize(rt_group* g, uint32_t W, uint32_t H, uint32_t band)
{
    if (!g || W == 0 || H == 0 || band == 0) return RT_ERR_INVALID;
    const uint32_t n = (uint32_t)g->m.size();
    const rt_status sy = rt_group_synchronize(g);
    if (sy != RT_OK) return sy;
    for (uint32_t i = 0; i < n; ++i) GMEM(g, i, rt_resize(g->m[i], W, H, band, i, n));
    free_buffers(g);
    g->W = W; g->H = H; g->band = band;
    g->rows.assign(n, 0);
    g->max_rows = 0;
    for (uint32_t i = 0; i < n; ++i) {
        g->rows[i] = rt_local_rows(g->m[i]);
        if (g->rows[i] != local_rows(H, band, i, n)) return fail(g, RT_ERR_STATE, "member band bookkeeping disagrees");
        g->max_rows = std::max(g->max_rows, g->rows[i]);
    }
    const size_t slab = (size_t)std::max<uint32_t>(g->max_rows, 1) * W;
    if (g->rccl)
        for (uint32_t i = 0; i < n; ++i) {
            GHIP(g, hipSetDevice(g->dev[i]));
            GHIP(g, hipMalloc((void**)&g->send[i], slab * sizeof(uint32_t)));
        }
    GHIP(g, hipSetDevice(g->dev[0]));
    GHIP(g, hipMalloc((void**)&g->d_gath, (size_t)n * slab * sizeof(uint32_t)));
    GHIP(g, hipMalloc((void**)&g->d_frame, (size_t)W * H * sizeof(uint32_t)));
    GHIP(g, hipMemsetAsync(g->d_frame, 0, (size_t)W * H * sizeof(uint32_t), g->st[0]));
    return RT_OK;
}

rt_status rt_group_render(rt_group* g, const rt_camera* cam, const rt_render_params* p, uint32_t* out_rgba)
{
    if (!g || !cam || !p) return RT_ERR_INVALID;
    if (!g->d_frame) return fail(g, RT_ERR_STATE, "no viewport (rt_group_resize)");
    const uint32_t n = (uint32_t)g->m.size();
    GHIP(g, hipSetDevice(g->dev[0]));
    GHIP(g, hipEventRecord(g->e0, g->st[0]));
    // every member's band set, concurrently on its own device and stream
    for (uint32_t i = 0; i < n; ++i) GMEM(g, i, rt_render(g->m[i], cam, p, nullptr, nullptr));
    const size_t slab = (size_t)g->max_rows * g->W;
    if (g->rccl) {
        for (uint32_t i = 0; i < n; ++i) {
            void* d_rgba = nullptr;
            GMEM(g, i, rt_device_buffers(g->m[i], nullptr, &d_rgba));
            GHIP(g, hipSetDevice(g->dev[i]));
            GHIP(g, hipMemcpyAsync(g->send[i], d_rgba, (size_t)g->rows[i] * g->W * sizeof(uint32_t), hipMemcpyDeviceToDevice, g->st[i]));
        }
        GNCCL(g, ncclGroupStart());
        for (uint32_t i = 0; i < n; ++i)
            GNCCL(g, ncclGather(g->send[i], i == 0 ? g->d_gath : nullptr, slab, ncclUint32, 0, g->comm[i], g->st[i]));
        GNCCL(g, ncclGroupEnd());
    } else {
        for (uint32_t i = 0; i < n; ++i) {
            void* d_rgba = nullptr;
            GMEM(g, i, rt_device_buffers(g->m[i], nullptr, &d_rgba));
            GHIP(g, hipSetDevice(g->dev[i]));
            GHIP(g, hipEventRecord(g->ready[i], g->st[i]));
            GHIP(g, hipSetDevice(g->dev[0]));
            GHIP(g, hipStreamWaitEvent(g->st[0], g->ready[i], 0));
            const size_t bytes = (size_t)g->rows[i] * g->W * sizeof(uint32_t);
            if (g->dev[i] == g->dev[0]) GHIP(g, hipMemcpyAsync(g->d_gath + i * slab, d_rgba, bytes, hipMemcpyDeviceToDevice, g->st[0]));
            else GHIP(g, hipMemcpyPeerAsync(g->d_gath + i * slab, g->dev[0], d_rgba, g->dev[i], bytes, g->st[0]));
        }
    }
    GHIP(g, hipSetDevice(g->dev[0]));
    const uint64_t total = (uint64_t)g->W * g->H;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((total + 255) / 256, 65535);
    hipLaunchKernelGGL(assemble_rows_kernel, dim3(blocks), dim3(256), 0, g->st[0], g->d_gath, g->d_frame, g->W, g->H, g->band, n, g->max_rows);
    GHIP(g, hipGetLastError());
    GHIP(g, hipEventRecord(g->e1, g->st[0]));
    g->pending = true;
    if (out_rgba) {
        GHIP(g, hipMemcpyAsync(out_rgba, g->d_frame, total * sizeof(uint32_t), hipMemcpyDeviceToHost, g->st[0]));
        return rt_group_synchronize(g);
    }
    return RT_OK;
}

rt_status rt_group_synchronize(rt_group* g)
{
    if (!g) return RT_ERR_INVALID;
    for (size_t i = 0; i < g->m.size(); ++i) GMEM(g, i, rt_synchronize(g->m[i]));   // also reports overflows
    GHIP(g, hipSetDevice(g->dev[0]));
    GHIP(g, hipStreamSynchronize(g->st[0]));
    return RT_OK;
}

rt_status rt_group_frame_device(rt_group* g, void** d_rgba)
{
    if (!g || !d_rgba) return RT_ERR_INVALID;
    *d_rgba = g->d_frame;
    return g->d_frame ? RT_OK : RT_ERR_STATE;
}

rt_status rt_group_read_accumulation(rt_group* g, float* out_accum)
{
    if (!g || !out_accum) return RT_ERR_INVALID;
    if (!g->d_frame) return fail(g, RT_ERR_STATE, "no viewport (rt_group_resize)");
    const uint32_t n = (uint32_t)g->m.size(), W = g->W, band = g->band;
    std::vector<float> local;
    for (uint32_t i = 0; i < n; ++i) {
        local.resize((size_t)g->rows[i] * W * 4);
        if (local.empty()) continue;
        // the member's accumulation after a synchronisation (its stats stay those of its last render)
        GMEM(g, i, rt_read_accumulation(g->m[i], local.data()));
        for (uint32_t r = 0; r < g->rows[i]; ++r) {
            const uint32_t y = (i + (r / band) * n) * band + r % band;
            std::memcpy(out_accum + (size_t)y * W * 4, local.data() + (size_t)r * W * 4, (size_t)W * 4 * sizeof(float));
        }
    }
    return RT_OK;
}

rt_status rt_group_reset_accumulation(rt_group* g)
{
    if (!g) return RT_ERR_INVALID;
    for (size_t i = 0; i < g->m.size(); ++i) GMEM(g, i, rt_reset_accumulation(g->m[i]));
    return RT_OK;
}

rt_status rt_group_get_stats(rt_group* g, rt_group_stats* s)
{
    if (!g || !s) return RT_ERR_INVALID;
    if (g->pending) {
        GHIP(g, hipSetDevice(g->dev[0]));
        GHIP(g, hipEventSynchronize(g->e1));
        GHIP(g, hipEventElapsedTime(&g->last_ms, g->e0, g->e1));
        g->max_kernel_ms = 0.0f;
        for (size_t i = 0; i < g->m.size(); ++i) {
            rt_stats ms{};
            GMEM(g, i, rt_get_stats(g->m[i], &ms));
            g->max_kernel_ms = std::max(g->max_kernel_ms, ms.last_kernel_ms);
        }
        g->pending = false;
    }
    s->last_ms = g->last_ms;
    s->max_member_kernel_ms = g->max_kernel_ms;
    s->gather = g->rccl ? 1u : 0u;
    s->n = (uint32_t)g->m.size();
    return RT_OK;
}

}  // extern "C"
