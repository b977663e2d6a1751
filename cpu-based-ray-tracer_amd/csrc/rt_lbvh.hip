// rt_lbvh.hip -- the scene BVH built on the device: a non-parity fast path for large meshes
// ("later: GPU LBVH build"; the reference builds on the host, MC/BVH.h:131-214).
//
// Karras's linear BVH ("Maximizing parallelism in the construction of BVHs, octrees, and k-d trees",
// HPG 2012) over 30-bit Morton codes of the triangle-box centroids, one triangle per leaf, written
// straight into the traversal layout of rt_layout.h: nodes in DFS pre-order with skip pointers, the
// triangles in DFS leaf order (the sorted Morton order).  Every kernel is one thread per triangle or
// node:
//   1. leaf boxes (min/max of the vertices, as Triangle::Get3DAABB) and the centroid bounds;
//   2. Morton codes; 3. a stable radix sort of (code, triangle) (hipcub);
//   4. the internal nodes' children from the sorted codes (equal codes split by index);
//   5. boxes and subtree sizes bottom-up (the second child to arrive at a node computes it);
//   6. each node's DFS position from its ancestors' left-subtree sizes, then the node and triangle
//      records.
// lbvh_build_host runs the same per-node functions sequentially; the device tree equals it bit for
// bit (tests/test_lbvh.py).  Rays find the same closest t as with the reference's tree (the
// Moller-Trumbore operations do not depend on the tree), but a tie between two triangles at one t
// resolves by this tree's DFS order, and the traversal visits other boxes: images agree with the
// reference-tree render except at such ties.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "rt_kernels.h"

namespace {

constexpr int kMaxWalk = 256;   // ancestors of a node: 30-bit codes + index bits bound the depth far below

__host__ __device__ inline uint32_t clz32(uint32_t x)
{
#ifdef __HIP_DEVICE_COMPILE__
    return (uint32_t)__clz((int)x);
#else
    return (uint32_t)__builtin_clz(x);
#endif
}

// the 10 low bits of v spread to every third bit
__host__ __device__ inline uint32_t expand10(uint32_t v)
{
    v &= 1023u;
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// the leaf box of triangle i from its vertices (9 floats: a, b, c)
__host__ __device__ inline void leaf_box(const float* v, uint32_t i, float lo[3], float hi[3])
{
    const float* t = v + 9 * (size_t)i;
    for (int a = 0; a < 3; ++a) {
        lo[a] = fminf(fminf(t[a], t[3 + a]), t[6 + a]);
        hi[a] = fmaxf(fmaxf(t[a], t[3 + a]), t[6 + a]);
    }
}

// Morton code of a box centroid in the centroid bounds (smin, 1 / extent per axis; 0 for a flat axis)
__host__ __device__ inline uint32_t morton_of(const float lo[3], const float hi[3], const float smin[3], const float sinv[3])
{
    uint32_t q[3];
    for (int a = 0; a < 3; ++a) {
        float t = ((lo[a] + hi[a]) * 0.5f - smin[a]) * sinv[a];
        t = t > 0.0f ? t : 0.0f;
        t = t < 1.0f ? t : 1.0f;
        q[a] = (uint32_t)(t * 1023.0f);
    }
    return (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
}

// common prefix length of sorted keys i and j, the index breaking ties between equal codes (Karras)
__host__ __device__ inline int delta(const uint32_t* code, int n, int i, int j)
{
    if (j < 0 || j >= n) return -1;
    const uint32_t x = code[i] ^ code[j];
    return x ? (int)clz32(x) : 32 + (int)clz32((uint32_t)i ^ (uint32_t)j);
}

// internal node i (0 = root) of n >= 2 leaves: its children as node ids (internal 0..n-2, leaf k = n-1+k)
__host__ __device__ inline void karras_children(const uint32_t* code, int n, int i, int& left, int& right)
{
    const int d = delta(code, n, i, i + 1) - delta(code, n, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = delta(code, n, i, i - d);
    int lmax = 2;
    while (delta(code, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(code, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(code, n, i, j);
    int s = 0;
    for (int t = (l + 1) / 2;; t = (t + 1) / 2) {
        if (delta(code, n, i, i + (s + t) * d) > dnode) s += t;
        if (t == 1) break;
    }
    const int g = i + s * d + (d < 0 ? -1 : 0);
    left = (i < j ? i : j) == g ? n - 1 + g : g;
    right = (i > j ? i : j) == g + 1 ? n - 1 + g + 1 : g + 1;
}

// the node and triangle records (rt_layout.h): node = (lo.xyz, hi.x)(hi.y, hi.z, bits(skip), bits(tri))
__host__ __device__ inline void write_node(float* nodes, uint32_t pos, const float* box, uint32_t size, int tri)
{
    float* q = nodes + 8 * (size_t)pos;
    q[0] = box[0]; q[1] = box[1]; q[2] = box[2]; q[3] = box[3]; q[4] = box[4]; q[5] = box[5];
    const uint32_t skip = pos + size;
    std::memcpy(&q[6], &skip, 4);
    std::memcpy(&q[7], &tri, 4);
}

// ------------------------------------------------------------------ device pipeline
// float min / max on the ordered integer images: a float with the sign bit clear orders as a signed
// int, one with the sign bit set in reverse as an unsigned int.  The branch is on the sign BIT: -0.0
// (0x80000000) must take the unsigned path, where it orders above every negative float's image.
__device__ inline void atomic_min_f(float* a, float v)
{
    if (__float_as_int(v) >= 0) atomicMin((int*)a, __float_as_int(v));
    else atomicMax((unsigned int*)a, __float_as_uint(v));
}
__device__ inline void atomic_max_f(float* a, float v)
{
    if (__float_as_int(v) >= 0) atomicMax((int*)a, __float_as_int(v));
    else atomicMin((unsigned int*)a, __float_as_uint(v));
}
__device__ inline float load_c(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline uint32_t load_c(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// leaf boxes (6 floats per triangle) and the centroid bounds cb[0..2] (min) / cb[3..5] (max)
__global__ void __launch_bounds__(256) k_leaf_boxes(uint32_t n, const float* __restrict__ verts, float* __restrict__ lbox, float* cb)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    float c[3] = {INFINITY, INFINITY, INFINITY}, C[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (i < n) {
        float lo[3], hi[3];
        leaf_box(verts, i, lo, hi);
        for (int a = 0; a < 3; ++a) {
            lbox[6 * (size_t)i + a] = lo[a];
            lbox[6 * (size_t)i + 3 + a] = hi[a];
            c[a] = C[a] = (lo[a] + hi[a]) * 0.5f;
        }
    }
    // wave reduction, then one atomic per wave and bound
    for (int off = 32; off >= 1; off >>= 1)
        for (int a = 0; a < 3; ++a) {
            c[a] = fminf(c[a], __shfl_xor(c[a], off));
            C[a] = fmaxf(C[a], __shfl_xor(C[a], off));
        }
    if (__lane_id() == 0)
        for (int a = 0; a < 3; ++a) { atomic_min_f(&cb[a], c[a]); atomic_max_f(&cb[3 + a], C[a]); }
}

__global__ void __launch_bounds__(256) k_morton(uint32_t n, const float* __restrict__ lbox, const float* __restrict__ cb,
                                                uint32_t* __restrict__ code, uint32_t* __restrict__ idx)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float smin[3], sinv[3];
    for (int a = 0; a < 3; ++a) {
        smin[a] = cb[a];
        const float ext = cb[3 + a] - cb[a];
        sinv[a] = ext > 0.0f ? 1.0f / ext : 0.0f;
    }
    code[i] = morton_of(lbox + 6 * (size_t)i, lbox + 6 * (size_t)i + 3, smin, sinv);
    idx[i] = i;
}

__global__ void __launch_bounds__(256) k_karras(int n, const uint32_t* __restrict__ code, int* __restrict__ left, int* __restrict__ right,
                                                int* __restrict__ parent)
{
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n - 1) return;
    int l, r;
    karras_children(code, n, i, l, r);
    left[i] = l; right[i] = r;
    parent[l] = i; parent[r] = i;
}

// boxes (6 floats per node) and subtree sizes (nodes) bottom-up: one thread per leaf climbs while it is the
// second of a node's children to arrive
__global__ void __launch_bounds__(256) k_bottom_up(int n, const uint32_t* __restrict__ idx, const float* __restrict__ lbox,
                                                   const int* __restrict__ left, const int* __restrict__ right, const int* __restrict__ parent,
                                                   uint32_t* __restrict__ arrive, float* box, uint32_t* size)
{
    const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= n) return;
    int node = n - 1 + k;
    const float* lb = lbox + 6 * (size_t)idx[k];
    for (int a = 0; a < 6; ++a) box[6 * (size_t)node + a] = lb[a];
    size[node] = 1u;
    for (int step = 0; step < kMaxWalk && node != 0; ++step) {
        const int p = parent[node];
        __threadfence();
        if (atomicAdd(&arrive[p], 1u) == 0u) return;   // the sibling is not done yet: it continues
        __threadfence();
        const int l = left[p], r = right[p];
        float* bp = box + 6 * (size_t)p;
        for (int a = 0; a < 3; ++a) {
            bp[a] = fminf(load_c(box + 6 * (size_t)l + a), load_c(box + 6 * (size_t)r + a));
            bp[3 + a] = fmaxf(load_c(box + 6 * (size_t)l + 3 + a), load_c(box + 6 * (size_t)r + 3 + a));
        }
        size[p] = load_c(size + l) + load_c(size + r) + 1u;
        node = p;
    }
}

// a node's DFS position: every ancestor edge adds 1, a right child also its left sibling's subtree
__global__ void __launch_bounds__(256) k_write(int n, const uint32_t* __restrict__ idx, const int* __restrict__ left,
                                               const int* __restrict__ right, const int* __restrict__ parent, const float* __restrict__ box,
                                               const uint32_t* __restrict__ size, const float4* __restrict__ recs, float* __restrict__ nodes,
                                               float4* __restrict__ tris)
{
    const int x = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (x >= 2 * n - 1) return;
    uint32_t pos = 0;
    int y = x;
    for (int step = 0; step < kMaxWalk && y != 0; ++step) {
        const int p = parent[y];
        pos += 1u + (right[p] == y ? size[left[p]] : 0u);
        y = p;
    }
    const bool leaf = x >= n - 1;
    const int k = x - (n - 1);
    write_node(nodes, pos, box + 6 * (size_t)x, size[x], leaf ? k : -1);
    if (leaf) {
        const uint32_t t = idx[k];
        for (int q = 0; q < 4; ++q) tris[4 * (size_t)k + q] = recs[4 * (size_t)t + q];
    }
}

}  // namespace

// ------------------------------------------------------------------ host reference (same functions, in order)
bool lbvh_build_host(uint32_t n, const float* verts, const float* recs, std::vector<float>& nodes, std::vector<float>& tris)
{
    if (n < 2) return false;
    std::vector<float> lbox(6 * (size_t)n);
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < n; ++i) {
        leaf_box(verts, i, &lbox[6 * (size_t)i], &lbox[6 * (size_t)i + 3]);
        for (int a = 0; a < 3; ++a) {
            const float c = (lbox[6 * (size_t)i + a] + lbox[6 * (size_t)i + 3 + a]) * 0.5f;
            cmin[a] = fminf(cmin[a], c);
            cmax[a] = fmaxf(cmax[a], c);
        }
    }
    float sinv[3];
    for (int a = 0; a < 3; ++a) {
        const float ext = cmax[a] - cmin[a];
        sinv[a] = ext > 0.0f ? 1.0f / ext : 0.0f;
    }
    std::vector<uint32_t> code0(n), idx(n), code(n);
    for (uint32_t i = 0; i < n; ++i) { code0[i] = morton_of(&lbox[6 * (size_t)i], &lbox[6 * (size_t)i + 3], cmin, sinv); idx[i] = i; }
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return code0[a] < code0[b]; });
    for (uint32_t i = 0; i < n; ++i) code[i] = code0[idx[i]];
    const int N = (int)n, M = 2 * N - 1;
    std::vector<int> left(N - 1), right(N - 1), parent(M, -1);
    for (int i = 0; i < N - 1; ++i) {
        karras_children(code.data(), N, i, left[i], right[i]);
        parent[left[i]] = i; parent[right[i]] = i;
    }
    // boxes and sizes in post-order
    std::vector<float> box(6 * (size_t)M);
    std::vector<uint32_t> size(M);
    std::vector<std::pair<int, bool>> st{{0, false}};
    while (!st.empty()) {
        auto [x, done] = st.back();
        st.pop_back();
        if (x >= N - 1) {
            const float* lb = &lbox[6 * (size_t)idx[x - (N - 1)]];
            std::copy(lb, lb + 6, &box[6 * (size_t)x]);
            size[x] = 1;
        } else if (!done) {
            st.push_back({x, true});
            st.push_back({right[x], false});
            st.push_back({left[x], false});
        } else {
            for (int a = 0; a < 3; ++a) {
                box[6 * (size_t)x + a] = fminf(box[6 * (size_t)left[x] + a], box[6 * (size_t)right[x] + a]);
                box[6 * (size_t)x + 3 + a] = fmaxf(box[6 * (size_t)left[x] + 3 + a], box[6 * (size_t)right[x] + 3 + a]);
            }
            size[x] = size[left[x]] + size[right[x]] + 1;
        }
    }
    nodes.assign(8 * (size_t)M, 0.0f);
    tris.assign(16 * (size_t)N, 0.0f);
    // DFS positions in pre-order
    std::vector<int> pre{0};
    uint32_t pos = 0;
    while (!pre.empty()) {
        const int x = pre.back();
        pre.pop_back();
        const bool leaf = x >= N - 1;
        const int k = x - (N - 1);
        write_node(nodes.data(), pos++, &box[6 * (size_t)x], size[x], leaf ? k : -1);
        if (leaf) std::copy(recs + 16 * (size_t)idx[k], recs + 16 * (size_t)idx[k] + 16, &tris[16 * (size_t)k]);
        else { pre.push_back(right[x]); pre.push_back(left[x]); }
    }
    return true;
}

// ------------------------------------------------------------------ device build
// verts: 9 floats per triangle, recs: 4 float4 per triangle (rt_layout.h tris), both on the device;
// nodes (2 float4 x (2n - 1)) and tris (4 float4 x n) receive the tree.  n >= 2.
hipError_t lbvh_build_device(uint32_t n, const float* verts, const float4* recs, float4* nodes, float4* tris, hipStream_t s)
{
    const int N = (int)n, M = 2 * N - 1;
    char* buf = nullptr;
    // scratch: lbox 6n f, cb 6 f, code/idx x 2 (n u32 each), left/right (n-1 i32), parent M i32, arrive n-1 u32,
    // box 6M f, size M u32, sort temp
    size_t temp = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                                      (uint32_t*)nullptr, N, 0, 30, s);
    if (e != hipSuccess) return e;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_lbox = 0, o_cb = o_lbox + al(24 * (size_t)n), o_c0 = o_cb + al(24), o_i0 = o_c0 + al(4 * (size_t)n),
                 o_c1 = o_i0 + al(4 * (size_t)n), o_i1 = o_c1 + al(4 * (size_t)n), o_l = o_i1 + al(4 * (size_t)n),
                 o_r = o_l + al(4 * (size_t)n), o_p = o_r + al(4 * (size_t)n), o_a = o_p + al(4 * (size_t)M),
                 o_box = o_a + al(4 * (size_t)n), o_sz = o_box + al(24 * (size_t)M), o_tmp = o_sz + al(4 * (size_t)M), total = o_tmp + al(temp);
    if ((e = hipMalloc((void**)&buf, total)) != hipSuccess) return e;
    float* lbox = (float*)(buf + o_lbox);
    float* cb = (float*)(buf + o_cb);
    uint32_t *c0 = (uint32_t*)(buf + o_c0), *i0 = (uint32_t*)(buf + o_i0), *c1 = (uint32_t*)(buf + o_c1), *i1 = (uint32_t*)(buf + o_i1);
    int *left = (int*)(buf + o_l), *right = (int*)(buf + o_r), *parent = (int*)(buf + o_p);
    uint32_t* arrive = (uint32_t*)(buf + o_a);
    float* box = (float*)(buf + o_box);
    uint32_t* size = (uint32_t*)(buf + o_sz);
    const float cb0[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    const uint32_t g1 = (n + 255) / 256, gM = ((uint32_t)M + 255) / 256;
    do {
        if ((e = hipMemcpyAsync(cb, cb0, sizeof cb0, hipMemcpyHostToDevice, s)) != hipSuccess) break;
        if ((e = hipMemsetAsync(arrive, 0, 4 * (size_t)n, s)) != hipSuccess) break;
        if ((e = hipMemsetAsync(parent, 0xFF, 4 * (size_t)M, s)) != hipSuccess) break;
        hipLaunchKernelGGL(k_leaf_boxes, dim3(g1), dim3(256), 0, s, n, verts, lbox, cb);
        hipLaunchKernelGGL(k_morton, dim3(g1), dim3(256), 0, s, n, lbox, cb, c0, i0);
        if ((e = hipGetLastError()) != hipSuccess) break;
        if ((e = hipcub::DeviceRadixSort::SortPairs(buf + o_tmp, temp, c0, c1, i0, i1, N, 0, 30, s)) != hipSuccess) break;
        hipLaunchKernelGGL(k_karras, dim3(g1), dim3(256), 0, s, N, c1, left, right, parent);
        hipLaunchKernelGGL(k_bottom_up, dim3(g1), dim3(256), 0, s, N, i1, lbox, left, right, parent, arrive, box, size);
        hipLaunchKernelGGL(k_write, dim3(gM), dim3(256), 0, s, N, i1, left, right, parent, box, size, recs, (float*)nodes, tris);
        if ((e = hipGetLastError()) != hipSuccess) break;
        e = hipStreamSynchronize(s);
    } while (false);
    (void)hipStreamSynchronize(s);
    (void)hipFree(buf);
    return e;
}
