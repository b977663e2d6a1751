// oracle/rt_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see rt_oracle.h for the contract).
//
// A deliberately plain, recursive CPU restatement of the reference's path: it keeps the
// reference's structure (two-level BVH, un-pruned both-children recursion, by-value hit records,
// recursive shading) so that its work counters equal the reference's per-sample work, and every
// floating-point expression keeps glm 0.9.9.9's operation order.  Build: oracle/Makefile
// (g++ -O2 -ffp-contract=off, no fast-math).
#include "rt_oracle.h"
#include "philox.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <string>
#include <thread>
#include <vector>

namespace {

// ------------------------------------------------------------------ glm-order vector math
struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };
inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 muls(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }          // vec * scalar
inline V3 smul(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }          // scalar * vec
inline V3 divs(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }          // vec / scalar (true division)
inline V3 neg(V3 a) { return V3{-a.x, -a.y, -a.z}; }
// GLM/detail/func_geometric.inl:48-55: tmp = a*b; return tmp.x + tmp.y + tmp.z
inline float dot(V3 a, V3 b) { float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z; return tx + ty + tz; }
// GLM/detail/func_geometric.inl:68-80
inline V3 cross(V3 x, V3 y) { return V3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
// GLM normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt (func_geometric.inl:82-90, func_exponential.inl:136-139)
inline V3 glm_normalize(V3 v) { float is = 1.0f / sqrtf(dot(v, v)); return muls(v, is); }
inline float glm_length(V3 v) { return sqrtf(dot(v, v)); }
// Whitted::normalize, MC/VectorFloat.h:22-31 (zero-safe)
inline V3 w_normalize(V3 v)
{
    float l2 = v.x * v.x + v.y * v.y + v.z * v.z;
    if (l2 > 0) { float inv = 1 / sqrtf(l2); return V3{v.x * inv, v.y * inv, v.z * inv}; }
    return v;
}
// glm::min / glm::max, GLM/detail/func_common.inl:17-30 ; std::min/max have the same form
inline float gmin(float x, float y) { return (y < x) ? y : x; }
inline float gmax(float x, float y) { return (x < y) ? y : x; }

constexpr float PI_F = 3.141592653589793f;                 // MC/WhittedUtilities.h:20
constexpr float INTERSECTION_CORRECTION = 0.00001f;        // MC/WhittedUtilities.h:18

// ------------------------------------------------------------------ RNG (per-sample stream)
struct Rng {
    uint64_t seed; uint32_t pixel, frame, dim;
    uint32_t buf[4]; uint32_t buf_block;
    uint64_t* draws;
    const uint32_t* list = nullptr;   // explicit draws (unit-test entry points)
    float next()
    {   // Walnut::Random::Float replaced by the frozen Philox stream (oracle/philox.h)
        if (list) return oracle_u32_to_float(list[dim++]);
        uint32_t blk = dim >> 2;
        if (blk != buf_block) {
            uint32_t ctr[4] = {pixel, frame, blk, 0u};
            uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
            oracle_philox4x32_10(ctr, key, buf);
            buf_block = blk;
        }
        uint32_t u = buf[dim & 3u];
        ++dim;
        if (draws) ++*draws;
        return oracle_u32_to_float(u);
    }
};

// ------------------------------------------------------------------ geometry
struct AABB { V3 mn, mx; };
// AABB_3D() empty box, MC/BoundingVolume.h:32-39 (double max -> +inf in float)
inline AABB aabb_empty() { float inf = (float)std::numeric_limits<double>::max(); return AABB{V3{inf, inf, inf}, V3{-inf, -inf, -inf}}; }
inline AABB aabb_union(const AABB& a, const AABB& b) { return AABB{V3{gmin(a.mn.x, b.mn.x), gmin(a.mn.y, b.mn.y), gmin(a.mn.z, b.mn.z)}, V3{gmax(a.mx.x, b.mx.x), gmax(a.mx.y, b.mx.y), gmax(a.mx.z, b.mx.z)}}; }
inline AABB aabb_union_pt(const AABB& a, V3 p) { return AABB{V3{gmin(a.mn.x, p.x), gmin(a.mn.y, p.y), gmin(a.mn.z, p.z)}, V3{gmax(a.mx.x, p.x), gmax(a.mx.y, p.y), gmax(a.mx.z, p.z)}}; }
inline V3 aabb_center(const AABB& b) { return smul(0.5f, add(b.mx, b.mn)); }   // center_vector :116-119
inline int aabb_longest_axis(const AABB& b)                                       // longest_axis :132-148
{
    V3 d = sub(b.mx, b.mn);
    if ((d.x > d.y) && (d.x > d.z)) return 0;
    else if (d.y > d.z) return 1;
    return 2;
}

struct Ray {   // AccelerationStructure::Ray, MC/Ray.h:23-44
    V3 o, d, rcp; int neg[3];
    Ray(V3 org, V3 dir) : o(org), d(dir)
    {
        rcp = V3{1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z};
        neg[0] = dir.x < 0.0f; neg[1] = dir.y < 0.0f; neg[2] = dir.z < 0.0f;
    }
    V3 at(double t) const { return add(o, smul((float)t, d)); }
};

// AABB_3D::intersects_with_ray, MC/BoundingVolume.h:173-215 (std::max/min keep the first operand on NaN)
inline bool slab_hit(const AABB& b, const Ray& r)
{
    float tix = (b.mn.x - r.o.x) * r.rcp.x, tiy = (b.mn.y - r.o.y) * r.rcp.y, tiz = (b.mn.z - r.o.z) * r.rcp.z;
    float tox = (b.mx.x - r.o.x) * r.rcp.x, toy = (b.mx.y - r.o.y) * r.rcp.y, toz = (b.mx.z - r.o.z) * r.rcp.z;
    if (r.neg[0]) std::swap(tix, tox);
    if (r.neg[1]) std::swap(tiy, toy);
    if (r.neg[2]) std::swap(tiz, toz);
    float tin = std::max(tix, std::max(tiy, tiz));
    float tout = std::min(tox, std::min(toy, toz));
    return tout >= 0 && tin <= tout;
}

// Whitted::RayTriangleIntersection (Moller-Trumbore, mixed float/double), MC/TriangleMesh.h:19-45
inline bool moller_trumbore(V3 v1, V3 v2, V3 v3_, V3 o, V3 d, double& t)
{
    V3 E1 = sub(v2, v1), E2 = sub(v3_, v1), S = sub(o, v1);
    V3 S1 = cross(d, E2), S2 = cross(S, E1);
    double inv = 1.0 / dot(S1, E1);
    t = dot(S2, E2) * inv;
    double b2 = dot(S1, S) * inv;
    double b3 = dot(S2, d) * inv;
    return (t > 0.0) && (b2 > 0.0) && (b3 > 0.0) && ((1.0 - b2 - b3) > 0.0);
}

struct Material { V3 albedo, emission; bool emitting; V3 brdf; };
struct Tri { V3 a, b, c, n; float area; AABB box; int mesh; int id; };

struct Node {   // BVH_Node, MC/BVH.h:21-43 (index-linked)
    AABB box; float area; int left = -1, right = -1; int entity = -1;
};

struct Record {   // Whitted::IntersectionRecord, MC/IntersectionRecord.h:18-38
    bool hit = false; double t = std::numeric_limits<double>::max();
    V3 loc{0, 0, 0}, n{0, 0, 0}, emission{0, 0, 0}; int mat = -1; int tri = -1;
};

struct Mesh {
    std::vector<Tri> tris; std::vector<Node> nodes; int root = -1;
    float total_area = 0.0f; AABB box; int mat;
};

struct WorkCount { uint64_t rays = 0, node_tests = 0, tri_tests = 0, draws = 0, shading = 0, max_depth = 0; };

// BVH::build_BVH, MC/BVH.h:131-214 -- items are indices into an entity table with box/area
struct BuildItem { AABB box; float area; int entity; };
int build_bvh(std::vector<Node>& nodes, std::vector<BuildItem> items)
{
    int me = (int)nodes.size();
    nodes.push_back(Node{});
    if (items.size() == 1) {
        nodes[me].box = items[0].box; nodes[me].area = items[0].area; nodes[me].entity = items[0].entity;
        return me;
    } else if (items.size() == 2) {
        int l = build_bvh(nodes, {items[0]});
        int r = build_bvh(nodes, {items[1]});
        nodes[me].left = l; nodes[me].right = r;
        nodes[me].box = aabb_union(nodes[l].box, nodes[r].box);
        nodes[me].area = nodes[l].area + nodes[r].area;
        return me;
    }
    AABB cb = aabb_empty();
    for (auto& it : items) cb = aabb_union_pt(cb, aabb_center(it.box));
    switch (aabb_longest_axis(cb)) {
        case 0: std::sort(items.begin(), items.end(), [](const BuildItem& a, const BuildItem& b) { return aabb_center(a.box).x < aabb_center(b.box).x; }); break;
        case 1: std::sort(items.begin(), items.end(), [](const BuildItem& a, const BuildItem& b) { return aabb_center(a.box).y < aabb_center(b.box).y; }); break;
        default: std::sort(items.begin(), items.end(), [](const BuildItem& a, const BuildItem& b) { return aabb_center(a.box).z < aabb_center(b.box).z; }); break;
    }
    size_t mid = items.size() / 2;
    std::vector<BuildItem> lh(items.begin(), items.begin() + mid), rh(items.begin() + mid, items.end());
    int l = build_bvh(nodes, lh);
    int r = build_bvh(nodes, rh);
    nodes[me].left = l; nodes[me].right = r;
    nodes[me].box = aabb_union(nodes[l].box, nodes[r].box);
    nodes[me].area = nodes[l].area + nodes[r].area;
    return me;
}

}  // namespace

struct or_scene {
    std::vector<Mesh> meshes;
    std::vector<Material> mats;
    std::vector<Node> top; int top_root = -1;
    int light_mesh = -1;
    int ntris = 0;
    // flattened DFS leaf id of (mesh, local tri)
    std::vector<std::vector<int>> flat_id;
};

namespace {

Record trace_mesh(const or_scene* s, const Mesh& m, int node, const Ray& r, WorkCount& wc)
{   // BVH::traverse_BVH_from_node, MC/BVH.h:82-101, over triangles
    wc.node_tests++;
    const Node& nd = m.nodes[node];
    if (!slab_hit(nd.box, r)) return Record{};
    if (nd.left < 0 && nd.right < 0) {
        // TrianglePrimitive::GetIntersectionRecord, MC/TriangleMesh.h:118-134
        const Tri& t = m.tris[nd.entity];
        Record rec;
        wc.tri_tests++;
        if (moller_trumbore(t.a, t.b, t.c, r.o, r.d, rec.t)) {
            rec.hit = true; rec.mat = m.mat; rec.n = t.n; rec.loc = r.at(rec.t);
            rec.tri = s->flat_id[t.mesh][nd.entity];
        } else {
            rec.t = std::numeric_limits<double>::max();
        }
        return rec;
    }
    Record L = trace_mesh(s, m, nd.left, r, wc);
    Record R = trace_mesh(s, m, nd.right, r, wc);
    return (L.t < R.t) ? L : R;
}

Record trace_top(const or_scene* s, int node, const Ray& r, WorkCount& wc)
{
    wc.node_tests++;
    const Node& nd = s->top[node];
    if (!slab_hit(nd.box, r)) return Record{};
    if (nd.left < 0 && nd.right < 0) {
        // TriangleMesh::GetIntersectionRecord, MC/TriangleMesh.h:209-217
        const Mesh& m = s->meshes[nd.entity];
        if (m.root < 0) return Record{};
        return trace_mesh(s, m, m.root, r, wc);
    }
    Record L = trace_top(s, nd.left, r, wc);
    Record R = trace_top(s, nd.right, r, wc);
    return (L.t < R.t) ? L : R;
}

Record trace(const or_scene* s, const Ray& r, WorkCount& wc)
{   // BVH::traverse_BVH_from_root, MC/BVH.h:72-80
    wc.rays++;
    if (s->top_root < 0) return Record{};
    return trace_top(s, s->top_root, r, wc);
}

// TrianglePrimitive::Sampling, MC/TriangleMesh.h:69-89
void tri_sample(const Tri& t, Rng& g, Record& out, float& pdf)
{
    float x = 1 - sqrtf(g.next());
    float y = g.next();
    out.loc = add(add(smul(x, t.a), smul((1.0f - x) * y, t.b)), smul((1.0f - x) * (1.0f - y), t.c));
    out.n = t.n;
    pdf = 1.0f / t.area;
}

// BVH::Sampling_from_node, MC/BVH.h:114-129
void bvh_sample_node(const Mesh& m, int node, float p, Rng& g, Record& out, float& pdf)
{
    const Node& nd = m.nodes[node];
    if (nd.left < 0 && nd.right < 0) { tri_sample(m.tris[nd.entity], g, out, pdf); return; }
    if (p < m.nodes[nd.left].area) bvh_sample_node(m, nd.left, p, g, out, pdf);
    else bvh_sample_node(m, nd.right, p - m.nodes[nd.left].area, g, out, pdf);
}

// Renderer::SamplingAreaLight (MC/Renderer.h:163-180) -> TriangleMesh::Sampling (MC/TriangleMesh.h:193-197)
// -> BVH::Sampling_from_root (MC/BVH.h:103-107)
void sample_light(const or_scene* s, Rng& g, Record& out, float& pdf)
{
    if (s->light_mesh < 0) return;
    const Mesh& m = s->meshes[s->light_mesh];
    out.emission = s->mats[m.mat].emission;
    bvh_sample_node(m, m.root, g.next() * m.nodes[m.root].area, g, out, pdf);
    pdf = 1.0f / (m.nodes[m.root].area);
}

// WhittedMaterial::Sampling, MC/WhittedMaterial.h:71-117
V3 material_sample(V3 n, Rng& g)
{
    V3 l;
    l.z = g.next();
    float rxy = sqrtf(1.0f - l.z * l.z);
    float phi = 2.0f * PI_F * g.next();
    l.x = rxy * cosf(phi);
    l.y = rxy * sinf(phi);
    V3 Y;
    if (fabsf(n.x) > fabsf(n.y)) Y = glm_normalize(V3{n.z, 0.0f, -(n.x)});
    else Y = glm_normalize(V3{0.0f, n.z, -(n.y)});
    V3 X = cross(Y, n);
    return add(add(smul(l.x, X), smul(l.y, Y)), smul(l.z, n));
}

// WhittedMaterial::BRDF, MC/WhittedMaterial.h:58-69
inline V3 brdf(const Material& m, V3 wi, V3 n) { if (dot(wi, n) >= 0.0f) return m.brdf; return V3{0.0f, 0.0f, 0.0f}; }

struct Ctx { const or_scene* s; float rr; Rng* g; WorkCount* wc; };

// Renderer::shading, MC/Renderer.cpp:148-214
V3 shading(const Ctx& c, const Record& rec, V3 wo, uint64_t depth)
{
    c.wc->shading++;
    if (depth > c.wc->max_depth) c.wc->max_depth = depth;
    const Material& M = c.s->mats[rec.mat];
    if (M.emitting) return M.emission;
    V3 n = rec.n;
    if (dot(rec.n, wo) < 0.0f) n = neg(rec.n);
    V3 p = add(rec.loc, muls(n, INTERSECTION_CORRECTION));
    V3 Ld{0.0f, 0.0f, 0.0f};
    Record ls; float ls_pdf = 0.0f;
    sample_light(c.s, *c.g, ls, ls_pdf);
    V3 q = ls.loc;
    V3 p2q = sub(q, p);
    V3 wl = glm_normalize(p2q);
    V3 nl = ls.n;
    if (dot(ls.n, neg(wl)) < 0.0f) nl = neg(ls.n);
    Record occ = trace(c.s, Ray(p, wl), *c.wc);
    if (glm_length(p2q) < occ.t + 0.01f) {
        Ld = divs(divs(muls(muls(mul(ls.emission, brdf(M, wl, n)), dot(wl, n)), dot(neg(wl), nl)), dot(p2q, p2q)), ls_pdf);
    }
    V3 Li{0.0f, 0.0f, 0.0f};
    if (c.g->next() < c.rr) {
        V3 wi = glm_normalize(material_sample(n, *c.g));
        float pdf = 1.0f / (2.0f * PI_F);   // PDF_at_the_sample, MC/WhittedMaterial.h:44-56
        Record d = trace(c.s, Ray(p, wi), *c.wc);
        if (d.hit && !c.s->mats[d.mat].emitting) {
            V3 Lr = shading(c, d, neg(wi), depth + 1);
            Li = divs(divs(muls(mul(Lr, brdf(M, wi, n)), dot(wi, n)), pdf), c.rr);
        }
    }
    return add(Ld, Li);
}

// Renderer::cast_path, MC/Renderer.cpp:136-146
V3 cast_path(const Ctx& c, const Ray& r)
{
    Record rec = trace(c.s, r, *c.wc);
    if (rec.hit) return shading(c, rec, neg(r.d), 0);
    return V3{12 / 255.0f, 20 / 255.0f, 69 / 255.0f};
}

// ------------------------------------------------------------------ camera (restated glm)
struct M4 { float m[4][4]; };   // m[col][row], glm layout
inline V4 mulmv(const M4& M, V4 v)
{   // GLM/detail/type_mat4x4.inl:561-572: (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
    float r[4];
    for (int i = 0; i < 4; ++i) {
        float mul0 = M.m[0][i] * v.x, mul1 = M.m[1][i] * v.y, mul2 = M.m[2][i] * v.z, mul3 = M.m[3][i] * v.w;
        float add0 = mul0 + mul1, add1 = mul2 + mul3;
        r[i] = add0 + add1;
    }
    return V4{r[0], r[1], r[2], r[3]};
}
M4 perspective_fov(float fov, float width, float height, float zNear, float zFar)
{   // glm::perspectiveFovRH_NO, GLM/ext/matrix_clip_space.inl:372-389
    float rad = fov;
    float h = cosf(0.5f * rad) / sinf(0.5f * rad);
    float w = h * height / width;
    M4 R; std::memset(&R, 0, sizeof R);
    R.m[0][0] = w; R.m[1][1] = h;
    R.m[2][2] = -(zFar + zNear) / (zFar - zNear);
    R.m[2][3] = -1.0f;
    R.m[3][2] = -(2.0f * zFar * zNear) / (zFar - zNear);
    return R;
}
M4 look_at(V3 eye, V3 center, V3 up)
{   // glm::lookAtRH, GLM/ext/matrix_transform.inl:99-119
    V3 f = glm_normalize(sub(center, eye));
    V3 s = glm_normalize(cross(f, up));
    V3 u = cross(s, f);
    M4 R; std::memset(&R, 0, sizeof R);
    for (int i = 0; i < 4; ++i) R.m[i][i] = 1.0f;
    R.m[0][0] = s.x; R.m[1][0] = s.y; R.m[2][0] = s.z;
    R.m[0][1] = u.x; R.m[1][1] = u.y; R.m[2][1] = u.z;
    R.m[0][2] = -f.x; R.m[1][2] = -f.y; R.m[2][2] = -f.z;
    R.m[3][0] = -dot(s, eye); R.m[3][1] = -dot(u, eye); R.m[3][2] = dot(f, eye);
    return R;
}
M4 inverse4(const M4& M)
{   // glm compute_inverse<4,4>, GLM/detail/func_matrix.inl:347-405
    auto m = [&](int c, int r) { return M.m[c][r]; };
    float C00 = m(2,2) * m(3,3) - m(3,2) * m(2,3), C02 = m(1,2) * m(3,3) - m(3,2) * m(1,3), C03 = m(1,2) * m(2,3) - m(2,2) * m(1,3);
    float C04 = m(2,1) * m(3,3) - m(3,1) * m(2,3), C06 = m(1,1) * m(3,3) - m(3,1) * m(1,3), C07 = m(1,1) * m(2,3) - m(2,1) * m(1,3);
    float C08 = m(2,1) * m(3,2) - m(3,1) * m(2,2), C10 = m(1,1) * m(3,2) - m(3,1) * m(1,2), C11 = m(1,1) * m(2,2) - m(2,1) * m(1,2);
    float C12 = m(2,0) * m(3,3) - m(3,0) * m(2,3), C14 = m(1,0) * m(3,3) - m(3,0) * m(1,3), C15 = m(1,0) * m(2,3) - m(2,0) * m(1,3);
    float C16 = m(2,0) * m(3,2) - m(3,0) * m(2,2), C18 = m(1,0) * m(3,2) - m(3,0) * m(1,2), C19 = m(1,0) * m(2,2) - m(2,0) * m(1,2);
    float C20 = m(2,0) * m(3,1) - m(3,0) * m(2,1), C22 = m(1,0) * m(3,1) - m(3,0) * m(1,1), C23 = m(1,0) * m(2,1) - m(2,0) * m(1,1);
    float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
    float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
    float V0[4] = {m(1,0), m(0,0), m(0,0), m(0,0)}, V1[4] = {m(1,1), m(0,1), m(0,1), m(0,1)};
    float V2[4] = {m(1,2), m(0,2), m(0,2), m(0,2)}, V3_[4] = {m(1,3), m(0,3), m(0,3), m(0,3)};
    float I0[4], I1[4], I2[4], I3[4];
    for (int i = 0; i < 4; ++i) {
        I0[i] = (V1[i] * F0[i] - V2[i] * F1[i]) + V3_[i] * F2[i];
        I1[i] = (V0[i] * F0[i] - V2[i] * F3[i]) + V3_[i] * F4[i];
        I2[i] = (V0[i] * F1[i] - V1[i] * F3[i]) + V3_[i] * F5[i];
        I3[i] = (V0[i] * F2[i] - V1[i] * F4[i]) + V2[i] * F5[i];
    }
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    M4 Inv;
    for (int i = 0; i < 4; ++i) { Inv.m[0][i] = I0[i] * SA[i]; Inv.m[1][i] = I1[i] * SB[i]; Inv.m[2][i] = I2[i] * SA[i]; Inv.m[3][i] = I3[i] * SB[i]; }
    float Row0[4] = {Inv.m[0][0], Inv.m[1][0], Inv.m[2][0], Inv.m[3][0]};
    float D0[4]; for (int i = 0; i < 4; ++i) D0[i] = M.m[0][i] * Row0[i];
    float D1 = (D0[0] + D0[1]) + (D0[2] + D0[3]);
    float ood = 1.0f / D1;
    M4 R;
    for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) R.m[c][r] = Inv.m[c][r] * ood;
    return R;
}

struct Cam { V3 pos; M4 proj, iproj, view, iview; };
Cam make_camera(uint32_t W, uint32_t H)
{   // Camera defaults MC/Camera.h:19-37, Camera{35,0.1,100} MC/mainloop.cpp:22,
    // RecomputeProjectionMatrix/ViewMatrix MC/Camera.cpp:101-112
    Cam c;
    c.pos = V3{(float)2.81432, (float)4.20749, (float)-9.11751};
    V3 fwd{(float)0.00209191, (float)-0.148299, (float)0.988941};
    V3 up{0.0f, 1.0f, 0.0f};
    float fov = 35.0f * (float)0.01745329251994329576923690768489;   // glm::radians
    c.proj = perspective_fov(fov, (float)W, (float)H, 0.1f, 100.0f);
    c.iproj = inverse4(c.proj);
    c.view = look_at(c.pos, add(c.pos, fwd), up);
    c.iview = inverse4(c.view);
    return c;
}
// loop body of Camera::RecomputeRayDirections, MC/Camera.cpp:119-125
V3 camera_dir(const Cam& c, uint32_t x, uint32_t y, uint32_t W, uint32_t H, Rng& g)
{
    float ux = g.next();
    float uy = g.next();
    float cx = ((float)x + ux) / (float)W, cy = ((float)y + uy) / (float)H;
    cx = cx * 2.0f - 1.0f; cy = cy * 2.0f - 1.0f;
    V4 target = mulmv(c.iproj, V4{cx, cy, 1.0f, 1.0f});
    V3 d = glm_normalize(divs(V3{target.x, target.y, target.z}, target.w));
    V4 r = mulmv(c.iview, V4{d.x, d.y, d.z, 0.0f});
    return V3{r.x, r.y, r.z};
}

inline uint8_t to_u8(float v)
{   // (uint8_t)(c*255.0f), MC/Renderer.cpp:17-20; x86 cvttss2si semantics for NaN
    float f = v * 255.0f;
    if (f != f) return 0;
    return (uint8_t)(int32_t)f;
}

// ------------------------------------------------------------------ objl subset
std::string first_token(const std::string& in)
{   // objl::algorithm::firstToken, MC/OBJ_Loader.h:381-398
    if (!in.empty()) {
        size_t a = in.find_first_not_of(" \t"), b = in.find_first_of(" \t", a);
        if (a != std::string::npos && b != std::string::npos) return in.substr(a, b - a);
        else if (a != std::string::npos) return in.substr(a);
    }
    return "";
}
std::string tail(const std::string& in)
{   // objl::algorithm::tail, MC/OBJ_Loader.h:363-378
    size_t ts = in.find_first_not_of(" \t"), ss = in.find_first_of(" \t", ts), ta = in.find_first_not_of(" \t", ss), te = in.find_last_not_of(" \t");
    if (ta != std::string::npos && te != std::string::npos) return in.substr(ta, te - ta + 1);
    else if (ta != std::string::npos) return in.substr(ta);
    return "";
}
void split(const std::string& in, std::vector<std::string>& out, const std::string& tok)
{   // objl::algorithm::split, MC/OBJ_Loader.h:324-360
    out.clear();
    std::string temp;
    for (int i = 0; i < (int)in.size(); i++) {
        std::string test = in.substr(i, tok.size());
        if (test == tok) {
            if (!temp.empty()) { out.push_back(temp); temp.clear(); i += (int)tok.size() - 1; }
            else out.push_back("");
        } else if (i + tok.size() >= in.size()) {
            temp += in.substr(i, tok.size()); out.push_back(temp); break;
        } else temp += in[i];
    }
}

}  // namespace

// ============================================================================== C API
extern "C" {

int64_t or_obj_positions(const char* path, float* out, int64_t cap)
{   // objl::Loader::LoadFile (MC/OBJ_Loader.h:434-720), v/f records of a single-mesh file
    std::string p(path);
    if (p.size() < 4 || p.substr(p.size() - 4) != ".obj") return -1;
    std::ifstream f(p);
    if (!f.is_open()) return -1;
    std::vector<V3> pos;
    std::vector<float> verts;
    std::string line;
    std::vector<std::string> sp, sf, sv;
    while (std::getline(f, line)) {
        std::string ft = first_token(line);
        if (ft == "v") {
            split(tail(line), sp, " ");
            pos.push_back(V3{std::stof(sp[0]), std::stof(sp[1]), std::stof(sp[2])});
        } else if (ft == "f") {   // GenVerticesFromRawOBJ, MC/OBJ_Loader.h:734-842 (positions only)
            split(tail(line), sf, " ");
            for (auto& s : sf) {
                split(s, sv, "/");
                if (sv.empty() || sv.size() > 3) continue;
                int idx = std::stoi(sv[0]);
                idx = idx < 0 ? (int)pos.size() + idx : idx - 1;
                const V3& v = pos[idx];
                verts.push_back(v.x); verts.push_back(v.y); verts.push_back(v.z);
            }
        } else if (ft == "o" || ft == "g") {
            if (!verts.empty()) return -1;   // multi-mesh files are outside this oracle's scope
        }
    }
    if (out) {
        if ((int64_t)verts.size() > cap) return -1;
        std::memcpy(out, verts.data(), verts.size() * sizeof(float));
    }
    return (int64_t)verts.size();
}

or_scene* or_scene_new(void) { return new or_scene; }
void or_scene_free(or_scene* s) { delete s; }

int or_scene_add_mesh(or_scene* s, const float* raw, int64_t n_tris, const float albedo[3], const float emission[3])
{
    Material M;
    M.albedo = V3{albedo[0], albedo[1], albedo[2]};
    M.emission = V3{emission[0], emission[1], emission[2]};
    M.emitting = glm_length(M.emission) > 0.00001f;        // MC/WhittedMaterial.h:34-41
    M.brdf = divs(M.albedo, PI_F);                          // diffuse_coefficient / PI, :66
    int mi = (int)s->mats.size();
    s->mats.push_back(M);
    Mesh m;
    m.mat = mi;
    int mesh_id = (int)s->meshes.size();
    // TriangleMesh::TriangleMesh, MC/TriangleMesh.h:148-186
    const float scale = 0.01f;
    float inf = std::numeric_limits<float>::infinity();
    V3 rmin{inf, inf, inf}, rmax{-inf, -inf, -inf};
    for (int64_t i = 0; i < n_tris; ++i) {
        V3 v[3];
        for (int j = 0; j < 3; ++j) {
            const float* q = raw + 9 * i + 3 * j;
            v[j] = smul(scale, V3{q[0], q[1], q[2]});
            rmin = V3{std::min(rmin.x, v[j].x), std::min(rmin.y, v[j].y), std::min(rmin.z, v[j].z)};
            rmax = V3{std::max(rmax.x, v[j].x), std::max(rmax.y, v[j].y), std::max(rmax.z, v[j].z)};
        }
        Tri t;   // TrianglePrimitive ctor, :54-60
        t.a = v[0]; t.b = v[1]; t.c = v[2];
        V3 cp = cross(sub(t.b, t.a), sub(t.c, t.a));
        t.area = 0.5f * glm_length(cp);
        t.n = w_normalize(cp);
        AABB ab{V3{fminf(t.a.x, t.b.x), fminf(t.a.y, t.b.y), fminf(t.a.z, t.b.z)}, V3{fmaxf(t.a.x, t.b.x), fmaxf(t.a.y, t.b.y), fmaxf(t.a.z, t.b.z)}};
        t.box = aabb_union_pt(ab, t.c);     // Get3DAABB, :96-99
        t.mesh = mesh_id; t.id = (int)i;
        m.tris.push_back(t);
    }
    m.box = AABB{V3{fminf(rmin.x, rmax.x), fminf(rmin.y, rmax.y), fminf(rmin.z, rmax.z)}, V3{fmaxf(rmin.x, rmax.x), fmaxf(rmin.y, rmax.y), fmaxf(rmin.z, rmax.z)}};
    std::vector<BuildItem> items;
    for (auto& t : m.tris) { m.total_area += t.area; items.push_back(BuildItem{t.box, t.area, t.id}); }
    if (!items.empty()) m.root = build_bvh(m.nodes, items);
    s->meshes.push_back(std::move(m));
    return mesh_id;
}

static void flat_walk(or_scene* s, const Mesh& m, int node, int& counter)
{
    const Node& nd = m.nodes[node];
    if (nd.left < 0 && nd.right < 0) { s->flat_id[m.tris[nd.entity].mesh][nd.entity] = counter++; return; }
    flat_walk(s, m, nd.left, counter);
    flat_walk(s, m, nd.right, counter);
}
static void flat_walk_top(or_scene* s, int node, int& counter)
{
    const Node& nd = s->top[node];
    if (nd.left < 0 && nd.right < 0) { const Mesh& m = s->meshes[nd.entity]; if (m.root >= 0) flat_walk(s, m, m.root, counter); return; }
    flat_walk_top(s, nd.left, counter);
    flat_walk_top(s, nd.right, counter);
}

int or_scene_build(or_scene* s)
{   // Renderer::GenerateBVH, MC/Renderer.h:83-86 (entity AABB = mesh box, area = total_area)
    s->top.clear();
    std::vector<BuildItem> items;
    for (size_t i = 0; i < s->meshes.size(); ++i) items.push_back(BuildItem{s->meshes[i].box, s->meshes[i].total_area, (int)i});
    s->top_root = items.empty() ? -1 : build_bvh(s->top, items);
    s->light_mesh = -1;
    for (size_t i = 0; i < s->meshes.size(); ++i) if (s->mats[s->meshes[i].mat].emitting) { s->light_mesh = (int)i; break; }
    s->flat_id.assign(s->meshes.size(), {});
    s->ntris = 0;
    for (size_t i = 0; i < s->meshes.size(); ++i) { s->flat_id[i].assign(s->meshes[i].tris.size(), -1); s->ntris += (int)s->meshes[i].tris.size(); }
    int counter = 0;
    if (s->top_root >= 0) flat_walk_top(s, s->top_root, counter);
    return counter == s->ntris ? 0 : -1;
}

int or_scene_num_tris(const or_scene* s) { return s->ntris; }
int or_scene_num_nodes(const or_scene* s)
{
    int n = 0;
    for (auto& nd : s->top) if (!(nd.left < 0 && nd.right < 0)) ++n;
    for (auto& m : s->meshes) n += (int)m.nodes.size();
    return n;
}

static void dump_mesh(const or_scene* s, const Mesh& m, int node, int mesh, int& ni, float* nf, int32_t* nI, float* tf, int32_t* tI)
{
    const Node& nd = m.nodes[node];
    int me = ni++;
    float* f = nf + 7 * me; int32_t* I = nI + 5 * me;
    f[0] = nd.box.mn.x; f[1] = nd.box.mn.y; f[2] = nd.box.mn.z; f[3] = nd.box.mx.x; f[4] = nd.box.mx.y; f[5] = nd.box.mx.z; f[6] = nd.area;
    I[0] = -1; I[1] = -1; I[2] = -1; I[3] = mesh; I[4] = 0;
    if (nd.left < 0 && nd.right < 0) {
        const Tri& t = m.tris[nd.entity];
        int ti = s->flat_id[mesh][nd.entity];
        I[2] = ti;
        float* T = tf + 13 * ti;
        V3 vs[4] = {t.a, t.b, t.c, t.n};
        for (int k = 0; k < 4; ++k) { T[3 * k] = vs[k].x; T[3 * k + 1] = vs[k].y; T[3 * k + 2] = vs[k].z; }
        T[12] = t.area;
        tI[2 * ti] = mesh; tI[2 * ti + 1] = m.mat;
        return;
    }
    I[0] = ni; dump_mesh(s, m, nd.left, mesh, ni, nf, nI, tf, tI);
    I[1] = ni; dump_mesh(s, m, nd.right, mesh, ni, nf, nI, tf, tI);
}
static void dump_top(const or_scene* s, int node, int& ni, float* nf, int32_t* nI, float* tf, int32_t* tI)
{
    const Node& nd = s->top[node];
    if (nd.left < 0 && nd.right < 0) { const Mesh& m = s->meshes[nd.entity]; if (m.root >= 0) dump_mesh(s, m, m.root, nd.entity, ni, nf, nI, tf, tI); return; }
    int me = ni++;
    float* f = nf + 7 * me; int32_t* I = nI + 5 * me;
    f[0] = nd.box.mn.x; f[1] = nd.box.mn.y; f[2] = nd.box.mn.z; f[3] = nd.box.mx.x; f[4] = nd.box.mx.y; f[5] = nd.box.mx.z; f[6] = nd.area;
    I[2] = -1; I[3] = -1; I[4] = 1;
    I[0] = ni; dump_top(s, nd.left, ni, nf, nI, tf, tI);
    I[1] = ni; dump_top(s, nd.right, ni, nf, nI, tf, tI);
}

int or_scene_dump(const or_scene* s, float* nf, int32_t* nI, float* tf, int32_t* tI)
{
    int ni = 0;
    if (s->top_root >= 0) dump_top(s, s->top_root, ni, nf, nI, tf, tI);
    return ni;
}

void or_trace(const or_scene* s, int64_t n, const float* org, const float* dir, int32_t* hit, int32_t* tri, int32_t* mat, double* t, float* loc, float* nrm)
{
    WorkCount wc;
    for (int64_t i = 0; i < n; ++i) {
        Ray r(V3{org[3 * i], org[3 * i + 1], org[3 * i + 2]}, V3{dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]});
        Record rec = trace(s, r, wc);
        hit[i] = rec.hit; tri[i] = rec.hit ? rec.tri : -1; mat[i] = rec.hit ? rec.mat : -1; t[i] = rec.t;
        loc[3 * i] = rec.loc.x; loc[3 * i + 1] = rec.loc.y; loc[3 * i + 2] = rec.loc.z;
        nrm[3 * i] = rec.n.x; nrm[3 * i + 1] = rec.n.y; nrm[3 * i + 2] = rec.n.z;
    }
}

void or_mt(int64_t n, const float* c, int32_t* hit, double* t)
{
    for (int64_t i = 0; i < n; ++i) {
        const float* q = c + 15 * i;
        double tt = 0.0;
        hit[i] = moller_trumbore(V3{q[0], q[1], q[2]}, V3{q[3], q[4], q[5]}, V3{q[6], q[7], q[8]}, V3{q[9], q[10], q[11]}, V3{q[12], q[13], q[14]}, tt);
        t[i] = tt;
    }
}

void or_aabb(int64_t n, const float* c, int32_t* hit)
{
    for (int64_t i = 0; i < n; ++i) {
        const float* q = c + 12 * i;
        Ray r(V3{q[6], q[7], q[8]}, V3{q[9], q[10], q[11]});
        hit[i] = slab_hit(AABB{V3{q[0], q[1], q[2]}, V3{q[3], q[4], q[5]}}, r);
    }
}

void or_camera_matrices(uint32_t W, uint32_t H, float mats[64])
{
    Cam c = make_camera(W, H);
    const M4* ms[4] = {&c.proj, &c.iproj, &c.view, &c.iview};
    for (int k = 0; k < 4; ++k) for (int col = 0; col < 4; ++col) for (int r = 0; r < 4; ++r) mats[16 * k + 4 * col + r] = ms[k]->m[col][r];
}

void or_camera_dirs(uint32_t W, uint32_t H, uint32_t frame, uint64_t seed, float* dirs)
{
    Cam c = make_camera(W, H);
    for (uint32_t y = 0; y < H; ++y) for (uint32_t x = 0; x < W; ++x) {
        uint32_t px = y * W + x;
        Rng g{seed, px, frame, 0, {0, 0, 0, 0}, 0xFFFFFFFFu, nullptr};
        V3 d = camera_dir(c, x, y, W, H, g);
        dirs[3 * px] = d.x; dirs[3 * px + 1] = d.y; dirs[3 * px + 2] = d.z;
    }
}

int or_render(const or_scene* s, uint32_t W, uint32_t H, uint32_t first_frame, uint32_t n_frames, uint64_t seed, float rr, int threads,
              uint32_t row_begin, uint32_t row_end, float* accum, uint32_t* rgba, or_counters* counters)
{
    if (first_frame == 0 || W == 0 || H == 0) return -1;
    if (row_end == 0 || row_end > H) row_end = H;
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    Cam cam = make_camera(W, H);
    std::atomic<uint32_t> next{row_begin};
    std::vector<WorkCount> wcs(threads);
    auto worker = [&](int tid) {
        WorkCount& wc = wcs[tid];
        for (;;) {
            uint32_t y = next.fetch_add(1);
            if (y >= row_end) break;
            for (uint32_t x = 0; x < W; ++x) {
                uint32_t px = y * W + x;
                float* A = accum + 4 * (size_t)px;
                // Renderer::Render memsets the accumulation buffer on frame 1 (MC/Renderer.cpp:95-98)
                if (first_frame == 1) { A[0] = A[1] = A[2] = A[3] = 0.0f; }
                float fin[4] = {0, 0, 0, 0};
                for (uint32_t k = 0; k < n_frames; ++k) {
                    uint32_t frame = first_frame + k;
                    Rng g{seed, px, frame, 0, {0, 0, 0, 0}, 0xFFFFFFFFu, &wc.draws};
                    Ctx c{s, rr, &g, &wc};
                    // RayGen_Shader, MC/Renderer.cpp:124-134
                    V3 dir = camera_dir(cam, x, y, W, H, g);
                    V3 L = cast_path(c, Ray(cam.pos, w_normalize(dir)));
                    A[0] = A[0] + L.x; A[1] = A[1] + L.y; A[2] = A[2] + L.z; A[3] = A[3] + 1.0f;
                    for (int i = 0; i < 4; ++i) {
                        float v = A[i] / (float)frame;
                        v = gmin(gmax(v, 0.0f), 1.0f);   // glm::clamp, GLM/detail/func_common.inl:240-245
                        fin[i] = v;
                    }
                }
                if (n_frames > 0) {
                    uint8_t r = to_u8(fin[0]), gg = to_u8(fin[1]), b = to_u8(fin[2]), a = to_u8(fin[3]);
                    rgba[px] = ((uint32_t)a << 24) | ((uint32_t)b << 16) | ((uint32_t)gg << 8) | r;   // MC/Renderer.cpp:15-23
                }
            }
        }
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(worker, i);
    for (auto& t : ts) t.join();
    if (counters) {
        or_counters c{};
        for (auto& w : wcs) {
            c.rays += w.rays; c.node_tests += w.node_tests; c.tri_tests += w.tri_tests; c.draws += w.draws;
            c.shading_calls += w.shading; c.max_depth = std::max<uint64_t>(c.max_depth, w.max_depth);
        }
        c.samples = (uint64_t)W * (row_end - row_begin) * n_frames;
        *counters = c;
    }
    return 0;
}

void or_light_sample(const or_scene* s, int64_t n, const uint32_t* u, float* loc, float* nrm, float* emission, float* pdf)
{
    for (int64_t i = 0; i < n; ++i) {
        Rng g{0, 0, 0, 0, {0, 0, 0, 0}, 0xFFFFFFFFu, nullptr, u + 3 * i};
        Record r; float p = -1.0f;
        sample_light(s, g, r, p);
        loc[3 * i] = r.loc.x; loc[3 * i + 1] = r.loc.y; loc[3 * i + 2] = r.loc.z;
        nrm[3 * i] = r.n.x; nrm[3 * i + 1] = r.n.y; nrm[3 * i + 2] = r.n.z;
        emission[3 * i] = r.emission.x; emission[3 * i + 1] = r.emission.y; emission[3 * i + 2] = r.emission.z;
        pdf[i] = p;
    }
}

void or_material_sample(int64_t n, const float* nrm, const float* wi, const uint32_t* u, const float* albedo, float* raw, float* dir, float* brdf_out, float* pdf)
{
    for (int64_t i = 0; i < n; ++i) {
        Rng g{0, 0, 0, 0, {0, 0, 0, 0}, 0xFFFFFFFFu, nullptr, u + 2 * i};
        V3 N{nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]}, W{wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]};
        Material M; M.albedo = V3{albedo[3 * i], albedo[3 * i + 1], albedo[3 * i + 2]}; M.brdf = divs(M.albedo, PI_F);
        V3 r = material_sample(N, g);
        V3 d = glm_normalize(r);
        V3 b = brdf(M, W, N);
        raw[3 * i] = r.x; raw[3 * i + 1] = r.y; raw[3 * i + 2] = r.z;
        dir[3 * i] = d.x; dir[3 * i + 1] = d.y; dir[3 * i + 2] = d.z;
        brdf_out[3 * i] = b.x; brdf_out[3 * i + 1] = b.y; brdf_out[3 * i + 2] = b.z;
        pdf[i] = 1.0f / (2.0f * PI_F);
    }
}

void or_trig(int64_t n, const float* x, float* cos_out, float* sin_out)
{   // the libm the reference calls (std::cos/std::sin on float, MC/WhittedMaterial.h:80-81)
    for (int64_t i = 0; i < n; ++i) { cos_out[i] = cosf(x[i]); sin_out[i] = sinf(x[i]); }
}

void or_exp_acos(int64_t n, const float* x, float* exp_out, float* acos_out)
{   // the libm the reference's denoiser calls (std::exp / std::acos on float, DN/Denoiser.h:195,203)
    for (int64_t i = 0; i < n; ++i) { exp_out[i] = expf(x[i]); acos_out[i] = acosf(x[i]); }
}

uint32_t or_rng_u32(uint64_t seed, uint32_t pixel, uint32_t frame, uint32_t dim) { return oracle_rng_u32(seed, pixel, frame, dim); }
float or_rng_float(uint64_t seed, uint32_t pixel, uint32_t frame, uint32_t dim) { return oracle_u32_to_float(oracle_rng_u32(seed, pixel, frame, dim)); }

}  // extern "C"
