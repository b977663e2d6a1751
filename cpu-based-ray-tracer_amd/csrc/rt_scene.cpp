// rt_scene.cpp -- host scene path (see rt_scene.h).
//
// Reference anchors (MC/ = "Monte Carlo Path Tracer/8599RayTracerGUI/src/"):
//   OBJ records          objl::Loader::LoadFile / GenVerticesFromRawOBJ, MC/OBJ_Loader.h:434-842
//   mesh construction    Whitted::TriangleMesh::TriangleMesh, MC/TriangleMesh.h:148-186 (x0.01 scale)
//   triangle             Whitted::TrianglePrimitive ctor / Get3DAABB, MC/TriangleMesh.h:54-60,96-99
//   BVH build            AccelerationStructure::BVH::build_BVH, MC/BVH.h:131-214 (median split,
//                        std::sort on the centroid along the longest centroid axis)
//   boxes                AABB_3D, MC/BoundingVolume.h:32-45,116-171
// Every float expression keeps the reference's (glm 0.9.9.9's) operation order; the tree and the
// numbers are checked bit-exactly against tests/golden/cornell_scene.npz.
#include "rt_scene.h"
#include "rt_knobs.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <cmath>
#include <fstream>
#include <limits>
#include <sstream>

namespace rt {
namespace {

inline F3 sub(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 cross(F3 x, F3 y) { return F3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
inline float dot(F3 a, F3 b) { float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z; return tx + ty + tz; }
inline float gmin(float x, float y) { return (y < x) ? y : x; }   // glm::min / std::min
inline float gmax(float x, float y) { return (x < y) ? y : x; }   // glm::max / std::max
inline float bits_as_float(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }

struct Box { F3 lo, hi; };
inline Box box_union(const Box& a, const Box& b)
{
    return Box{F3{gmin(a.lo.x, b.lo.x), gmin(a.lo.y, b.lo.y), gmin(a.lo.z, b.lo.z)},
               F3{gmax(a.hi.x, b.hi.x), gmax(a.hi.y, b.hi.y), gmax(a.hi.z, b.hi.z)}};
}
inline F3 centre(const Box& b)
{   // center_vector: 0.5f * (max + min)
    return F3{0.5f * (b.hi.x + b.lo.x), 0.5f * (b.hi.y + b.lo.y), 0.5f * (b.hi.z + b.lo.z)};
}

struct Tri {
    F3 a, b, c, n;
    float area;
    Box box;
    int mesh;
    int id;   // primitive id: 1 + creation index over all meshes (DN/TriangleMesh.h:54-62, DN/Renderer.cpp:36-43)
    // a sphere entity's one slot (a = its center): radius and radius_squared (MC/Sphere.h:19-23)
    bool sphere = false;
    float radius = 0.0f, r2 = 0.0f;
};

// A built (unflattened) binary tree; leaves reference an item id.
struct BNode { Box box; float area; int left = -1, right = -1, item = -1; };

struct Item { Box box; float area; F3 c; int id; };

// Binned SAH tree over the walked subtree's leaves (the split trace's near-first orderings, below): one leaf per
// triangle -- the leaf boxes are the reference's own leaf boxes, so every internal box, the float union of its
// children's, contains them exactly and the leaf's own slab test still decides -- with the
// same node count as the reference's subtree.  The tree is free for finite rays: the kernel takes the closest
// hit by (min t, max reference DFS triangle) and skips boxes entered beyond the bound, so only the visit count
// changes (tools/sim_sah_c5.py: C5's bunny rays test 17 % fewer boxes than on the median-split tree).
struct SNode { Box box; int left = -1, right = -1, tri = -1, size = 1; };

inline float half_area(const Box& b)
{
    const float ex = std::max(0.0f, b.hi.x - b.lo.x), ey = std::max(0.0f, b.hi.y - b.lo.y), ez = std::max(0.0f, b.hi.z - b.lo.z);
    return ex * ey + ey * ez + ez * ex;
}

constexpr int kMaxSahBins = 1024;

int build_sah(std::vector<SNode>& nodes, std::vector<std::pair<Box, int>>& leaves, size_t lo, size_t hi, const int kBins)
{
    const int me = (int)nodes.size();
    nodes.emplace_back();
    Box b = leaves[lo].first;
    for (size_t i = lo + 1; i < hi; ++i) b = box_union(b, leaves[i].first);
    nodes[me].box = b;
    if (hi - lo == 1) { nodes[me].tri = leaves[lo].second; return me; }
    auto cen = [](const Box& x, int a) { return a == 0 ? 0.5f * (x.lo.x + x.hi.x) : a == 1 ? 0.5f * (x.lo.y + x.hi.y) : 0.5f * (x.lo.z + x.hi.z); };
    float cl[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity()};
    float ch[3] = {-cl[0], -cl[0], -cl[0]};
    for (size_t i = lo; i < hi; ++i)
        for (int a = 0; a < 3; ++a) { const float c = cen(leaves[i].first, a); cl[a] = std::min(cl[a], c); ch[a] = std::max(ch[a], c); }
    const size_t n = hi - lo;
    double best = std::numeric_limits<double>::infinity();
    int best_ax = -1;
    float best_split = 0.0f;
    size_t best_k = 0;   // exact sweep: the first best_k leaves (sorted on best_ax) go left
    for (int a = 0; a < 3; ++a) {
        if (!(ch[a] > cl[a])) continue;
        if (n <= 2 * kBins) {   // small nodes: every split of the sorted order
            std::sort(leaves.begin() + lo, leaves.begin() + hi, [&](const auto& x, const auto& y) {
                const float cx = cen(x.first, a), cy = cen(y.first, a);
                return cx < cy || (cx == cy && x.second < y.second);
            });
            std::vector<float> suf(n + 1, 0.0f);
            Box sb = leaves[hi - 1].first;
            for (size_t k = n - 1; k >= 1; --k) { sb = box_union(sb, leaves[lo + k].first); suf[k] = half_area(sb); }
            Box pb = leaves[lo].first;
            for (size_t k = 1; k < n; ++k) {
                if (k > 1) pb = box_union(pb, leaves[lo + k - 1].first);
                const double cost = (double)half_area(pb) * (double)k + (double)suf[k] * (double)(n - k);
                if (cost < best) { best = cost; best_ax = a; best_k = k; best_split = std::numeric_limits<float>::quiet_NaN(); }
            }
            continue;
        }
        Box bb[kMaxSahBins];
        size_t cnt[kMaxSahBins] = {};
        bool used[kMaxSahBins] = {};
        const float scale = (float)kBins / (ch[a] - cl[a]);
        for (size_t i = lo; i < hi; ++i) {
            int k = (int)((cen(leaves[i].first, a) - cl[a]) * scale);
            k = std::min(std::max(k, 0), kBins - 1);
            bb[k] = used[k] ? box_union(bb[k], leaves[i].first) : leaves[i].first;
            used[k] = true;
            ++cnt[k];
        }
        float rarea[kMaxSahBins];
        size_t rcnt[kMaxSahBins];
        { Box rb{}; bool any = false; size_t c = 0;
          for (int k = kBins - 1; k >= 1; --k) {
              if (used[k]) { rb = any ? box_union(rb, bb[k]) : bb[k]; any = true; }
              c += cnt[k];
              rarea[k] = any ? half_area(rb) : 0.0f; rcnt[k] = c;
          } }
        Box lb{}; bool lany = false; size_t lc = 0;
        for (int k = 1; k < kBins; ++k) {
            if (used[k - 1]) { lb = lany ? box_union(lb, bb[k - 1]) : bb[k - 1]; lany = true; }
            lc += cnt[k - 1];
            if (lc == 0 || rcnt[k] == 0) continue;
            const double cost = (double)half_area(lb) * (double)lc + (double)rarea[k] * (double)rcnt[k];
            if (cost < best) { best = cost; best_ax = a; best_split = cl[a] + (float)k / scale; best_k = 0; }
        }
    }
    size_t mid;
    if (best_ax < 0) {
        mid = lo + n / 2;   // every centroid equal
    } else if (best_k != 0) {
        std::sort(leaves.begin() + lo, leaves.begin() + hi, [&](const auto& x, const auto& y) {
            const float cx = cen(x.first, best_ax), cy = cen(y.first, best_ax);
            return cx < cy || (cx == cy && x.second < y.second);
        });
        mid = lo + best_k;
    } else {
        // the bin boundary as the binning computed it: leaf i goes left iff its bin index < k
        const float scale = (float)kBins / (ch[best_ax] - cl[best_ax]);
        const int kk = (int)std::lround((best_split - cl[best_ax]) * scale);
        auto it = std::partition(leaves.begin() + lo, leaves.begin() + hi, [&](const auto& x) {
            int k = (int)((cen(x.first, best_ax) - cl[best_ax]) * scale);
            k = std::min(std::max(k, 0), kBins - 1);
            return k < kk;
        });
        mid = (size_t)(it - leaves.begin());
        if (mid == lo || mid == hi) mid = lo + n / 2;
    }
    const int l = build_sah(nodes, leaves, lo, mid, kBins);
    const int r = build_sah(nodes, leaves, mid, hi, kBins);
    nodes[me].left = l; nodes[me].right = r;
    nodes[me].size = 1 + nodes[l].size + nodes[r].size;
    return me;
}

// IEEE half of a float rounded toward -inf (down) or +inf (up): the nearest half, stepped one half-ulp when it
// lies on the wrong side (+-65504 beyond the half range round to +-inf on the outward side)
uint16_t half_directed(float v, bool up)
{
    _Float16 h = (_Float16)v;
    uint16_t b;
    std::memcpy(&b, &h, 2);
    const float back = (float)h;
    if (up ? back >= v : back <= v) return b;
    // one step toward the requested side
    const bool neg = (b & 0x8000u) != 0u;
    const uint16_t mag = b & 0x7FFFu;
    if (up) {
        if (neg) return mag == 0u ? (uint16_t)0x0001u : (uint16_t)(b - 1u);   // -0 -> +min subnormal
        return (uint16_t)(b + 1u);
    }
    if (!neg) return mag == 0u ? (uint16_t)0x8001u : (uint16_t)(b - 1u);
    return (uint16_t)(b + 1u);
}

// 16-byte nodes of near-first orderings (FlatScene::worders_h): false when a leaf's successor is not the next
// node of its ordering or an index does not fit
bool compact_orderings(const std::vector<float>& src, uint32_t M, uint32_t first, std::vector<uint32_t>& dst)
{
    dst.assign((size_t)8 * M * 4, 0u);
    for (uint32_t oct = 0; oct < 8; ++oct) {
        const bool neg[3] = {(oct & 1u) != 0u, (oct & 2u) != 0u, (oct & 4u) != 0u};
        for (uint32_t k = 0; k < M; ++k) {
            const float* q = &src[((size_t)oct * M + k) * 8];
            uint32_t* w = &dst[((size_t)oct * M + k) * 4];
            for (int a = 0; a < 3; ++a) {
                // near = the low plane unless the direction is negative on this axis (rt_scene.cpp near_first);
                // a low plane rounds down, a high plane up
                const uint16_t nh = half_directed(q[a], neg[a]), fh = half_directed(q[3 + a], !neg[a]);
                w[a] = (uint32_t)nh | ((uint32_t)fh << 16);
            }
            int32_t skip, tri;
            std::memcpy(&skip, &q[6], 4);
            std::memcpy(&tri, &q[7], 4);
            if (tri >= 0) {
                if ((uint32_t)skip != first + k + 1u && !(k + 1u == M)) return false;
                w[3] = 0x80000000u | (uint32_t)tri;
            } else {
                if (skip < 0) return false;
                w[3] = (uint32_t)skip;
            }
        }
    }
    return true;
}

int build_bvh(std::vector<BNode>& nodes, std::vector<Item>& items, size_t lo, size_t hi)
{
    const size_t n = hi - lo;
    const int me = (int)nodes.size();
    nodes.emplace_back();
    if (n == 1) {
        nodes[me].box = items[lo].box; nodes[me].area = items[lo].area; nodes[me].item = items[lo].id;
        return me;
    }
    size_t mid;
    if (n == 2) {
        mid = lo + 1;   // two entities: no sort (MC/BVH.h:150-158)
    } else {
        // centroid bounds start from the empty box (double max -> +inf as float, MC/BoundingVolume.h:32-39)
        const float inf = (float)std::numeric_limits<double>::max();
        Box cb{F3{inf, inf, inf}, F3{-inf, -inf, -inf}};
        for (size_t i = lo; i < hi; ++i) {
            const F3 p = items[i].c;
            cb = Box{F3{gmin(cb.lo.x, p.x), gmin(cb.lo.y, p.y), gmin(cb.lo.z, p.z)}, F3{gmax(cb.hi.x, p.x), gmax(cb.hi.y, p.y), gmax(cb.hi.z, p.z)}};
        }
        const F3 d = sub(cb.hi, cb.lo);
        int axis = ((d.x > d.y) && (d.x > d.z)) ? 0 : (d.y > d.z ? 1 : 2);   // longest_axis
        auto first = items.begin() + (std::ptrdiff_t)lo, last = items.begin() + (std::ptrdiff_t)hi;
        // std::sort (introsort) with the reference's strict comparator; sorting the sub-range in place
        // performs the same comparisons as the reference's sort of its copied half.
        if (axis == 0) std::sort(first, last, [](const Item& a, const Item& b) { return a.c.x < b.c.x; });
        else if (axis == 1) std::sort(first, last, [](const Item& a, const Item& b) { return a.c.y < b.c.y; });
        else std::sort(first, last, [](const Item& a, const Item& b) { return a.c.z < b.c.z; });
        mid = lo + n / 2;
    }
    const int l = build_bvh(nodes, items, lo, mid);
    const int r = build_bvh(nodes, items, mid, hi);
    nodes[me].left = l; nodes[me].right = r;
    nodes[me].box = box_union(nodes[l].box, nodes[r].box);
    nodes[me].area = nodes[l].area + nodes[r].area;
    return me;
}

// objl helpers (MC/OBJ_Loader.h:324-398)
std::string first_token(const std::string& in)
{
    if (in.empty()) return "";
    size_t a = in.find_first_not_of(" \t");
    if (a == std::string::npos) return "";
    size_t b = in.find_first_of(" \t", a);
    return b == std::string::npos ? in.substr(a) : in.substr(a, b - a);
}
std::string tail(const std::string& in)
{
    size_t ts = in.find_first_not_of(" \t");
    size_t ss = in.find_first_of(" \t", ts);
    size_t ta = in.find_first_not_of(" \t", ss);
    size_t te = in.find_last_not_of(" \t");
    if (ta != std::string::npos && te != std::string::npos) return in.substr(ta, te - ta + 1);
    if (ta != std::string::npos) return in.substr(ta);
    return "";
}
std::vector<std::string> split_on(const std::string& in, char tok)
{   // objl::algorithm::split with a one-character token: empty fields are kept, trailing token dropped
    std::vector<std::string> out;
    std::string cur;
    for (size_t i = 0; i < in.size(); ++i) {
        if (in[i] == tok) {
            out.push_back(cur);
            cur.clear();
        } else {
            cur += in[i];
            if (i + 1 == in.size()) out.push_back(cur);
        }
    }
    return out;
}

}  // namespace

bool SceneBuilder::load_obj_positions(const std::string& path, std::vector<float>& raw, std::string& err)
{
    raw.clear();
    if (path.size() < 4 || path.substr(path.size() - 4) != ".obj") { err = "not an .obj file: " + path; return false; }
    std::ifstream f(path);
    if (!f.is_open()) { err = "cannot open " + path; return false; }
    std::vector<F3> pos;
    std::string line;
    int groups = 0;
    while (std::getline(f, line)) {
        const std::string ft = first_token(line);
        if (ft == "v") {
            auto sp = split_on(tail(line), ' ');
            if (sp.size() < 3) { err = "bad v record"; return false; }
            pos.push_back(F3{std::stof(sp[0]), std::stof(sp[1]), std::stof(sp[2])});
        } else if (ft == "f") {
            for (const auto& s : split_on(tail(line), ' ')) {
                auto sv = split_on(s, '/');
                if (sv.empty() || sv.size() > 3 || sv[0].empty()) continue;
                int idx = std::stoi(sv[0]);
                idx = idx < 0 ? (int)pos.size() + idx : idx - 1;   // objl::algorithm::getElement
                if (idx < 0 || idx >= (int)pos.size()) { err = "face index out of range"; return false; }
                raw.push_back(pos[idx].x); raw.push_back(pos[idx].y); raw.push_back(pos[idx].z);
            }
        } else if (ft == "o" || ft == "g") {
            // a second object would start objl's second mesh; TriangleMesh asserts a single mesh
            // (MC/TriangleMesh.h:158)
            if (!raw.empty() && ++groups > 0) { err = "multi-mesh OBJ files are not supported (TriangleMesh asserts one mesh)"; return false; }
        }
    }
    // TriangleMesh consumes Vertices three at a time (MC/TriangleMesh.h:165); a ragged tail is ignored
    raw.resize(raw.size() - raw.size() % 9);
    return true;
}

void SceneBuilder::add_cornell_box()
{
    for (auto& m : cornell_box_meshes()) add_mesh(std::move(m));
}

std::vector<MeshDesc> SceneBuilder::cornell_box_meshes()
{
    std::vector<MeshDesc> out;
    // Cornell box measurement data (http://www.graphics.cornell.edu/online/box/data.html), laid out
    // as the reference's cornellbox/*.obj: vertex lists + 1-based faces, millimetres.
    struct Raw { const char* name; std::vector<F3> v; std::vector<int> f; MaterialDesc m; };
    const MaterialDesc red{{0.63f, 0.065f, 0.05f}, {0, 0, 0}}, green{{0.1f, 0.5f, 0.1f}, {0, 0, 0}},
        white{{0.7f, 0.7f, 0.7f}, {0, 0, 0}}, light{{0.7f, 0.7f, 0.7f}, {47.8f, 38.6f, 31.1f}};   // MC/Renderer.cpp:28-35
    const std::vector<int> quad{1, 2, 3, 1, 3, 4};
    std::vector<int> box_faces;
    for (int k = 0; k < 5; ++k) for (int j : quad) box_faces.push_back(4 * k + j);
    const Raw meshes[6] = {
        {"floor", {{552.8f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 559.2f}, {549.6f, 0.0f, 559.2f},
                   {556.0f, 548.8f, 0.0f}, {556.0f, 548.8f, 559.2f}, {0.0f, 548.8f, 559.2f}, {0.0f, 548.8f, 0.0f},
                   {549.6f, 0.0f, 559.2f}, {0.0f, 0.0f, 559.2f}, {0.0f, 548.8f, 559.2f}, {556.0f, 548.8f, 559.2f}},
         {1, 2, 3, 3, 4, 1, 5, 6, 7, 7, 8, 5, 9, 10, 11, 11, 12, 9}, white},
        {"shortbox", {{130.0f, 165.0f, 65.0f}, {82.0f, 165.0f, 225.0f}, {240.0f, 165.0f, 272.0f}, {290.0f, 165.0f, 114.0f},
                      {290.0f, 0.0f, 114.0f}, {290.0f, 165.0f, 114.0f}, {240.0f, 165.0f, 272.0f}, {240.0f, 0.0f, 272.0f},
                      {130.0f, 0.0f, 65.0f}, {130.0f, 165.0f, 65.0f}, {290.0f, 165.0f, 114.0f}, {290.0f, 0.0f, 114.0f},
                      {82.0f, 0.0f, 225.0f}, {82.0f, 165.0f, 225.0f}, {130.0f, 165.0f, 65.0f}, {130.0f, 0.0f, 65.0f},
                      {240.0f, 0.0f, 272.0f}, {240.0f, 165.0f, 272.0f}, {82.0f, 165.0f, 225.0f}, {82.0f, 0.0f, 225.0f}},
         box_faces, white},
        {"tallbox", {{423.0f, 330.0f, 247.0f}, {265.0f, 330.0f, 296.0f}, {314.0f, 330.0f, 456.0f}, {472.0f, 330.0f, 406.0f},
                     {423.0f, 0.0f, 247.0f}, {423.0f, 330.0f, 247.0f}, {472.0f, 330.0f, 406.0f}, {472.0f, 0.0f, 406.0f},
                     {472.0f, 0.0f, 406.0f}, {472.0f, 330.0f, 406.0f}, {314.0f, 330.0f, 456.0f}, {314.0f, 0.0f, 456.0f},
                     {314.0f, 0.0f, 456.0f}, {314.0f, 330.0f, 456.0f}, {265.0f, 330.0f, 296.0f}, {265.0f, 0.0f, 296.0f},
                     {265.0f, 0.0f, 296.0f}, {265.0f, 330.0f, 296.0f}, {423.0f, 330.0f, 247.0f}, {423.0f, 0.0f, 247.0f}},
         box_faces, white},
        {"left", {{552.8f, 0.0f, 0.0f}, {549.6f, 0.0f, 559.2f}, {556.0f, 548.8f, 559.2f}, {556.0f, 548.8f, 0.0f}}, quad, red},
        {"right", {{0.0f, 0.0f, 559.2f}, {0.0f, 0.0f, 0.0f}, {0.0f, 548.8f, 0.0f}, {0.0f, 548.8f, 559.2f}}, quad, green},
        {"light", {{343.0f, 548.7f, 227.0f}, {343.0f, 548.7f, 332.0f}, {213.0f, 548.7f, 332.0f}, {213.0f, 548.7f, 227.0f}}, quad, light},
    };
    for (const auto& m : meshes) {
        MeshDesc d;
        d.name = m.name;
        d.material = m.m;
        for (int idx : m.f) { const F3& p = m.v[idx - 1]; d.raw.push_back(p.x); d.raw.push_back(p.y); d.raw.push_back(p.z); }
        out.push_back(std::move(d));
    }
    return out;
}

int SceneBuilder::add_sphere(const F3& center, float radius, const MaterialDesc& m)
{
    MeshDesc d;
    d.sphere = true;
    d.center = center;
    d.radius = radius;
    d.material = m;
    d.name = "sphere" + std::to_string(meshes_.size());
    return add_mesh(std::move(d));
}

int SceneBuilder::add_mesh(MeshDesc m)
{
    meshes_.push_back(std::move(m));
    return (int)meshes_.size() - 1;
}

void SceneBuilder::add_two_spheres_scene()
{
    // WH/Renderer.cpp:29-48: glm::vec3(-1, 0, -12) r 2 diffuse (0.6, 0.7, 0.8); glass (0.5, -0.5, -8) r 1.5,
    // refractive index 1.5; the 10x10 chessboard at y = -3 (indices 0 1 3 / 1 2 3, uv corners); two lights
    WorldEntity diffuse;
    diffuse.kind = 0; diffuse.center = F3{-1.0f, 0.0f, -12.0f}; diffuse.radius = 2.0f; diffuse.nature = 2;
    diffuse.diffuse_color = F3{(float)0.6, (float)0.7, (float)0.8};
    add_world_entity(diffuse);
    WorldEntity glass;
    glass.kind = 0; glass.center = F3{(float)0.5, (float)-0.5, -8.0f}; glass.radius = 1.5f; glass.nature = 1;
    glass.refractive_index = (float)1.5;
    add_world_entity(glass);
    WorldEntity board;
    board.kind = 1; board.nature = 2;
    board.vertices = {{-5, -3, -6}, {5, -3, -6}, {5, -3, -16}, {-5, -3, -16}};
    board.indices = {0, 1, 3, 1, 2, 3};
    board.uv = {0, 0, 1, 0, 1, 1, 0, 1};
    add_world_entity(board);
    add_point_light(PointLight{{-20.0f, 70.0f, 20.0f}, {0.5f, 0.5f, 0.5f}});
    add_point_light(PointLight{{30.0f, 50.0f, -12.0f}, {0.5f, 0.5f, 0.5f}});
}

// World entities -> went / wtris (rt_layout.h)
static void flatten_world(const std::vector<WorldEntity>& world, FlatScene& out)
{
    uint32_t ntri = 0;
    for (const auto& e : world) {
        out.went.resize(out.went.size() + 16);
        float* q = &out.went[out.went.size() - 16];
        const uint32_t nt = e.kind == 1 ? (uint32_t)(e.indices.size() / 3) : 0u;
        q[0] = bits_as_float(e.kind); q[1] = bits_as_float(e.nature); q[2] = bits_as_float((int)ntri); q[3] = bits_as_float((int)nt);
        q[4] = e.center.x; q[5] = e.center.y; q[6] = e.center.z; q[7] = e.radius;
        q[8] = e.radius * e.radius;   // Sphere::radius_squared, WH/Sphere.h:19-22
        q[9] = e.refractive_index; q[10] = e.phong_diffuse; q[11] = e.phong_specular;
        q[12] = e.diffuse_color.x; q[13] = e.diffuse_color.y; q[14] = e.diffuse_color.z; q[15] = e.specular_size_factor;
        for (uint32_t t = 0; t < nt; ++t) {
            const uint32_t i1 = e.indices[3 * t], i2 = e.indices[3 * t + 1], i3 = e.indices[3 * t + 2];
            const F3 a = e.vertices[i1], b = e.vertices[i2], c = e.vertices[i3];
            const float w[16] = {a.x, a.y, a.z, e.uv[2 * i1], b.x, b.y, b.z, e.uv[2 * i1 + 1],
                                 c.x, c.y, c.z, e.uv[2 * i2], e.uv[2 * i2 + 1], e.uv[2 * i3], e.uv[2 * i3 + 1], 0.0f};
            out.wtris.insert(out.wtris.end(), w, w + 16);
        }
        ntri += nt;
    }
    out.hdr.n_went = (uint32_t)world.size();
    out.hdr.n_wtris = ntri;
}

bool SceneBuilder::build(FlatScene& out, std::string& err) const
{
    out = FlatScene{};
    // the split trace's walked tree: 1 = a binned-SAH tree over the subtree's leaves (default), 0 = the reference's
    // subtree (A/B knob RT_WALK_TREE)
    bool walk_tree_sah = true;
    if (const char* e = rt_knob("RT_WALK_TREE")) walk_tree_sah = std::strtol(e, nullptr, 10) != 0;
    // bins per axis of the SAH build (A/B knob RT_SAH_BINS)
    int sah_bins = 16;
    if (const char* e = rt_knob("RT_SAH_BINS")) sah_bins = std::min(std::max((int)std::strtol(e, nullptr, 10), 2), kMaxSahBins);
    const size_t nm = meshes_.size();
    for (const auto& e : world_) {
        if (e.kind == 0 && !(e.radius > 0.0f)) { err = "world sphere with a non-positive radius"; return false; }
        if (e.kind == 1) {
            if (e.indices.empty() || e.indices.size() % 3 || e.uv.size() != 2 * e.vertices.size()) { err = "bad world mesh"; return false; }
            for (uint32_t i : e.indices) if (i >= e.vertices.size()) { err = "world mesh index out of range"; return false; }
        }
    }
    if (nm == 0 && !world_.empty()) {
        // a pure Whitted world (config C1): no BVH, brute-force entities
        flatten_world(world_, out);
        out.plights.resize(lights_.size() * 8);
        for (size_t k = 0; k < lights_.size(); ++k) {
            float* q = &out.plights[8 * k];
            q[0] = lights_[k].position.x; q[1] = lights_[k].position.y; q[2] = lights_[k].position.z; q[3] = 0.0f;
            q[4] = lights_[k].radiance.x; q[5] = lights_[k].radiance.y; q[6] = lights_[k].radiance.z; q[7] = 0.0f;
        }
        out.hdr.n_plights = (uint32_t)lights_.size();
        out.hdr.sky[0] = sky_.x; out.hdr.sky[1] = sky_.y; out.hdr.sky[2] = sky_.z;
        out.hdr.light_mesh = -1;
        out.hdr.max_bounce_depth = 5;               // WH/World.h:55
        out.hdr.intersection_correction = 0.00001f; // WH/World.h:56
        return true;
    }
    if (!world_.empty()) { err = "a scene holds either triangle meshes or a Whitted world, not both"; return false; }
    if (nm == 0) { err = "empty scene"; return false; }
    // ---- per mesh: triangles, mesh box, total area, mesh BVH (TriangleMesh ctor)
    std::vector<std::vector<Tri>> tris(nm);
    std::vector<std::vector<BNode>> mesh_nodes(nm);
    std::vector<int> mesh_root(nm, -1);
    std::vector<Box> mesh_box(nm);
    std::vector<float> mesh_area(nm, 0.0f);
    int id_count = 1;
    uint32_t n_spheres = 0;
    for (size_t mi = 0; mi < nm; ++mi) {
        if (meshes_[mi].sphere) {
            // Whitted::Sphere (MC/Sphere.h:19-23,45-48): radius_squared = r * r, surface_area = 4 * PI * r^2 (4 * PI
            // first, a float), Get3DAABB = AABB_3D{center + r, center - r} (componentwise std::fmin / std::fmax,
            // MC/BoundingVolume.h:47-51); a top-level leaf of the entity BVH with one sphere slot
            const MeshDesc& d = meshes_[mi];
            const float PI = 3.141592653589793f;   // MC/WhittedUtilities.h:20
            Tri tr{};
            tr.sphere = true;
            tr.a = d.center; tr.radius = d.radius; tr.r2 = d.radius * d.radius;
            tr.area = 4 * PI * tr.r2;
            const F3 p1{d.center.x + d.radius, d.center.y + d.radius, d.center.z + d.radius};
            const F3 p2{d.center.x - d.radius, d.center.y - d.radius, d.center.z - d.radius};
            tr.box = Box{F3{std::fmin(p1.x, p2.x), std::fmin(p1.y, p2.y), std::fmin(p1.z, p2.z)},
                         F3{std::fmax(p1.x, p2.x), std::fmax(p1.y, p2.y), std::fmax(p1.z, p2.z)}};
            tr.mesh = (int)mi; tr.id = id_count++;
            tris[mi].push_back(tr);
            mesh_box[mi] = tr.box;
            mesh_area[mi] = tr.area;
            mesh_nodes[mi].push_back(BNode{tr.box, tr.area, -1, -1, 0});
            mesh_root[mi] = 0;
            ++n_spheres;
            continue;
        }
        const auto& raw = meshes_[mi].raw;
        const size_t nt = raw.size() / 9;
        if (nt == 0) { err = "mesh without triangles: " + meshes_[mi].name; return false; }
        const float inf = std::numeric_limits<float>::infinity();
        F3 rmin{inf, inf, inf}, rmax{-inf, -inf, -inf};
        for (size_t t = 0; t < nt; ++t) {
            F3 v[3];
            for (int j = 0; j < 3; ++j) {
                const float* q = &raw[9 * t + 3 * j];
                const float sc = meshes_[mi].scale;
                v[j] = F3{sc * q[0], sc * q[1], sc * q[2]};   // mesh_scale * vec3
                if (meshes_[mi].has_offset) {                  // world_coordinates + mesh_scale * vec3
                    const F3& o = meshes_[mi].offset;
                    v[j] = F3{o.x + v[j].x, o.y + v[j].y, o.z + v[j].z};
                }
                rmin = F3{std::min(rmin.x, v[j].x), std::min(rmin.y, v[j].y), std::min(rmin.z, v[j].z)};
                rmax = F3{std::max(rmax.x, v[j].x), std::max(rmax.y, v[j].y), std::max(rmax.z, v[j].z)};
            }
            Tri tr;
            tr.a = v[0]; tr.b = v[1]; tr.c = v[2]; tr.mesh = (int)mi; tr.id = id_count++;
            const F3 cp = cross(sub(tr.b, tr.a), sub(tr.c, tr.a));
            tr.area = 0.5f * std::sqrt(dot(cp, cp));
            const float l2 = cp.x * cp.x + cp.y * cp.y + cp.z * cp.z;   // Whitted::normalize (zero-safe)
            if (l2 > 0) { const float inv = 1 / std::sqrt(l2); tr.n = F3{cp.x * inv, cp.y * inv, cp.z * inv}; }
            else tr.n = cp;
            const Box ab{F3{std::fmin(tr.a.x, tr.b.x), std::fmin(tr.a.y, tr.b.y), std::fmin(tr.a.z, tr.b.z)},
                         F3{std::fmax(tr.a.x, tr.b.x), std::fmax(tr.a.y, tr.b.y), std::fmax(tr.a.z, tr.b.z)}};
            tr.box = Box{F3{gmin(ab.lo.x, tr.c.x), gmin(ab.lo.y, tr.c.y), gmin(ab.lo.z, tr.c.z)},
                         F3{gmax(ab.hi.x, tr.c.x), gmax(ab.hi.y, tr.c.y), gmax(ab.hi.z, tr.c.z)}};
            tris[mi].push_back(tr);
        }
        mesh_box[mi] = Box{F3{std::fmin(rmin.x, rmax.x), std::fmin(rmin.y, rmax.y), std::fmin(rmin.z, rmax.z)},
                           F3{std::fmax(rmin.x, rmax.x), std::fmax(rmin.y, rmax.y), std::fmax(rmin.z, rmax.z)}};
        std::vector<Item> items;
        for (size_t t = 0; t < nt; ++t) {
            mesh_area[mi] += tris[mi][t].area;
            items.push_back(Item{tris[mi][t].box, tris[mi][t].area, centre(tris[mi][t].box), (int)t});
        }
        mesh_root[mi] = build_bvh(mesh_nodes[mi], items, 0, items.size());
    }
    // ---- top level: BVH over meshes (entity box = mesh box, area = total_area)
    std::vector<BNode> top;
    std::vector<Item> titems;
    for (size_t mi = 0; mi < nm; ++mi) titems.push_back(Item{mesh_box[mi], mesh_area[mi], centre(mesh_box[mi]), (int)mi});
    const int top_root = build_bvh(top, titems, 0, titems.size());

    // ---- flatten: DFS pre-order, top leaves replaced by mesh roots
    struct FN { Box box; float area; int tri; int mesh; int top; int skip; int left, right; };
    std::vector<FN> fn;
    std::vector<const Tri*> slot_tri;
    std::vector<std::pair<int, int>> slot_src;   // (mesh, local tri)
    std::function<int(int, int)> walk_mesh = [&](int mi, int ni) -> int {
        const BNode& b = mesh_nodes[mi][ni];
        const int me = (int)fn.size();
        fn.push_back(FN{b.box, b.area, -1, mi, 0, -1, -1, -1});
        if (b.left < 0) {
            fn[me].tri = (int)slot_tri.size();
            slot_tri.push_back(&tris[mi][b.item]);
            slot_src.emplace_back(mi, b.item);
        } else {
            const int l = walk_mesh(mi, b.left);
            const int r = walk_mesh(mi, b.right);
            fn[me].left = l; fn[me].right = r;
        }
        fn[me].skip = (int)fn.size();
        return me;
    };
    std::function<int(int)> walk_top = [&](int ni) -> int {
        const BNode& b = top[ni];
        if (b.left < 0) {
            const int mi = b.item;
            // a top-level leaf box is the mesh box; it must equal the mesh-root box for the flattening
            const Box& mb = mesh_nodes[mi][mesh_root[mi]].box;
            if (std::memcmp(&mb, &b.box, sizeof(Box)) != 0) { err = "mesh box != mesh root box"; return -1; }
            return walk_mesh(mi, mesh_root[mi]);
        }
        const int me = (int)fn.size();
        fn.push_back(FN{b.box, b.area, -1, -1, 1, -1, -1, -1});
        const int l = walk_top(b.left);
        const int r = walk_top(b.right);
        if (l < 0 || r < 0) return -1;
        fn[me].left = l; fn[me].right = r;
        fn[me].skip = (int)fn.size();
        return me;
    };
    if (walk_top(top_root) < 0) return false;

    const uint32_t NN = (uint32_t)fn.size(), NT = (uint32_t)slot_tri.size();
    out.nodes.resize((size_t)NN * 8);
    out.dbg_node_f.resize((size_t)NN * 7);
    out.dbg_node_i.resize((size_t)NN * 5);
    for (uint32_t i = 0; i < NN; ++i) {
        const FN& n = fn[i];
        float* q = &out.nodes[8 * (size_t)i];
        q[0] = n.box.lo.x; q[1] = n.box.lo.y; q[2] = n.box.lo.z; q[3] = n.box.hi.x;
        q[4] = n.box.hi.y; q[5] = n.box.hi.z; q[6] = bits_as_float(n.skip); q[7] = bits_as_float(n.tri);
        float* d = &out.dbg_node_f[7 * (size_t)i];
        d[0] = n.box.lo.x; d[1] = n.box.lo.y; d[2] = n.box.lo.z; d[3] = n.box.hi.x; d[4] = n.box.hi.y; d[5] = n.box.hi.z; d[6] = n.area;
        int32_t* e = &out.dbg_node_i[5 * (size_t)i];
        e[0] = n.left; e[1] = n.right; e[2] = n.tri; e[3] = n.mesh; e[4] = n.top;
    }
    // ---- distinct leaf boxes of a small scene (the megakernel's coherent trace, rt_kernels.hip).
    // The reference tests a triangle iff the slab test passes for its leaf box and every ancestor box
    // (BVH::traverse_BVH_from_node, MC/BVH.h:82-101).  An ancestor box contains the leaf box exactly
    // (checked here), and for a ray whose reciprocal direction is finite the slab test's correctly
    // rounded subtractions and multiplications are monotone in the box planes, so an ancestor's entry
    // distance is <= the leaf's and its exit distance >= the leaf's: the leaf's own test decides.
    // Triangles with identical leaf boxes (the two halves of a quad) share one test.
    out.lboxes.clear();
    out.hdr.n_lboxes = 0;
    // (scenes with spheres render on the megakernel's BVH walk: no leaf-box trace, split trace, near-first
    // orderings or light-plane masks, which are all built for triangle leaves)
    if (NT > 0 && NT <= 64 && n_spheres == 0) {
        bool contained = true;
        std::vector<std::pair<Box, uint64_t>> uniq;
        for (uint32_t i = 0; i < NN && contained; ++i) {
            if (fn[i].tri < 0) continue;
            const Box& lb = fn[i].box;
            for (uint32_t j = 0; j < i; ++j) {
                if (fn[j].tri >= 0 || fn[j].skip <= (int)i) continue;   // not an ancestor of leaf i
                const Box& ab = fn[j].box;
                if (!(ab.lo.x <= lb.lo.x && ab.lo.y <= lb.lo.y && ab.lo.z <= lb.lo.z && ab.hi.x >= lb.hi.x && ab.hi.y >= lb.hi.y &&
                      ab.hi.z >= lb.hi.z)) { contained = false; break; }
            }
            size_t k = 0;
            while (k < uniq.size() && std::memcmp(&uniq[k].first, &lb, sizeof(Box)) != 0) ++k;
            if (k == uniq.size()) uniq.emplace_back(lb, 0ull);
            uniq[k].second |= 1ull << fn[i].tri;
        }
        if (contained) {
            out.hdr.n_lboxes = (uint32_t)uniq.size();
            out.lboxes.resize(uniq.size() * 8);
            for (size_t k = 0; k < uniq.size(); ++k) {
                const Box& b = uniq[k].first;
                float* q = &out.lboxes[8 * k];
                q[0] = b.lo.x; q[1] = b.hi.x; q[2] = b.lo.y; q[3] = b.hi.y;   // rt_layout.h: planes of an axis adjacent
                q[4] = b.lo.z; q[5] = b.hi.z;
                q[6] = bits_as_float((int32_t)(uint32_t)uniq[k].second); q[7] = bits_as_float((int32_t)(uint32_t)(uniq[k].second >> 32));
            }
        }
    }
    // near-first orderings of the subtree [r, rend) (the whole tree: [0, NN)), one per direction octant (bit 0:
    // d.x < 0, bit 1: d.y, bit 2: d.z): the same leaves in the pre-order that visits, at every internal node,
    // first the child whose box centre lies nearer along the axis that separates the two centres most, node k
    // of ordering o at dst[(o * (rend - r) + k) * 8] in the nodes layout (indices r + position).  A walk stops
    // at the subtree's end (its skip pointers reach rend only when it is done: stored as NN).  Exact in any
    // order: the kernels keep the closest hit by (min t, max DFS triangle) and a box entered beyond it is
    // skipped, and a shadow ray's verdict is any blocking hit.  The tree the orderings lay
    // out: the reference's subtree as it is, or (walk_tree_sah, default) a binned-SAH tree over its leaves
    // (build_sah: the same leaf boxes and node count)
    auto near_first = [&](const uint32_t r, const uint32_t rend, std::vector<float>& dst) -> bool {
        const uint32_t M = rend - r;
        dst.assign((size_t)8 * M * 8, 0.0f);
        std::vector<SNode> tn;
        int troot = 0;
        if (walk_tree_sah) {
            std::vector<std::pair<Box, int>> leaves;
            for (uint32_t i = r; i < rend; ++i)
                if (fn[i].tri >= 0) leaves.emplace_back(fn[i].box, fn[i].tri);
            tn.reserve(2 * leaves.size());
            troot = build_sah(tn, leaves, 0, leaves.size(), sah_bins);
        } else {
            tn.resize(M);
            for (uint32_t i = r; i < rend; ++i) {
                SNode& t = tn[i - r];
                t.box = fn[i].box; t.tri = fn[i].tri; t.size = fn[i].skip - (int)i;
                if (fn[i].tri < 0) { t.left = (int)(i + 1 - r); t.right = fn[i + 1].skip - (int)r; }
            }
        }
        if (tn.size() != M) return err = "walk tree: node count differs from the subtree's", false;
        auto centre = [](const Box& b, int a) { return a == 0 ? b.lo.x + b.hi.x : a == 1 ? b.lo.y + b.hi.y : b.lo.z + b.hi.z; };
        std::vector<int> st;
        for (uint32_t oct = 0; oct < 8; ++oct) {
            float* base = &dst[(size_t)oct * M * 8];
            uint32_t pos = 0;
            st.assign(1, troot);
            while (!st.empty()) {
                const int i = st.back();
                st.pop_back();
                const SNode& n = tn[i];
                uint32_t sk = r + pos + (uint32_t)n.size;   // the subtree of i occupies [pos, pos + size) of the ordering
                if (sk >= rend) sk = NN;
                float* q = base + 8 * (size_t)pos++;
                // the box as (near planes, far planes) for the octant's direction signs: x is (hi, lo) when
                // d.x < 0 -- the planes the slab test selects for such a ray (rt_device.h slab_nf_within)
                const bool sx = (oct & 1u) != 0u, sy = (oct & 2u) != 0u, sz = (oct & 4u) != 0u;
                q[0] = sx ? n.box.hi.x : n.box.lo.x; q[1] = sy ? n.box.hi.y : n.box.lo.y; q[2] = sz ? n.box.hi.z : n.box.lo.z;
                q[3] = sx ? n.box.lo.x : n.box.hi.x; q[4] = sy ? n.box.lo.y : n.box.hi.y; q[5] = sz ? n.box.lo.z : n.box.hi.z;
                q[6] = bits_as_float((int32_t)sk); q[7] = bits_as_float(n.tri);
                if (n.tri >= 0) continue;
                const int a = n.left, b = n.right;
                int ax = 0;
                float best = -1.0f;
                for (int k = 0; k < 3; ++k) {
                    const float dk = std::fabs(centre(tn[a].box, k) - centre(tn[b].box, k));
                    if (dk > best) { best = dk; ax = k; }
                }
                const bool neg = ((oct >> ax) & 1u) != 0u;
                const bool a_first = (centre(tn[a].box, ax) <= centre(tn[b].box, ax)) != neg;
                st.push_back(a_first ? b : a);
                st.push_back(a_first ? a : b);
            }
        }
        return true;
    };
    // ---- split trace of a larger scene: the deepest internal node whose subtree leaves at most 32 leaves
    // outside it (the kernel keeps ray A's and ray B's outside candidates in the halves of one mask) (the subtrees with that property form the chain from the root down to it).  The outside
    // leaves are tested by their own boxes, exactly as the small scenes' leaf boxes above (every ancestor
    // box must contain the leaf box), and the subtree is walked from its root, whose box must likewise lie
    // inside every ancestor's: then the root's own slab test decides whether the reference enters it.
    out.sboxes.clear();
    out.wcopies.clear();
    out.stri.clear();
    out.split_root = out.split_end = 0;
    if (NT > 64 && n_spheres == 0) {
        std::vector<uint32_t> leaf_pre(NN + 1, 0);   // leaves among nodes [0, i)
        for (uint32_t i = 0; i < NN; ++i) leaf_pre[i + 1] = leaf_pre[i] + (fn[i].tri >= 0 ? 1u : 0u);
        const uint32_t n_leaves = leaf_pre[NN];
        uint32_t r = 0;
        for (uint32_t i = 1; i < NN; ++i) {
            if (fn[i].tri >= 0) continue;
            const uint32_t end = (uint32_t)fn[i].skip;
            const uint32_t outside = n_leaves - (leaf_pre[end] - leaf_pre[i]);
            if (outside <= 32 && (r == 0 || end - i < (uint32_t)fn[r].skip - r)) r = i;
        }
        auto inside_ancestors = [&](uint32_t i) {   // every ancestor box of node i contains its box
            const Box& lb = fn[i].box;
            for (uint32_t j = 0; j < i; ++j) {
                if (fn[j].tri >= 0 || fn[j].skip <= (int)i) continue;   // not an ancestor of node i
                const Box& ab = fn[j].box;
                if (!(ab.lo.x <= lb.lo.x && ab.lo.y <= lb.lo.y && ab.lo.z <= lb.lo.z && ab.hi.x >= lb.hi.x && ab.hi.y >= lb.hi.y &&
                      ab.hi.z >= lb.hi.z)) return false;
            }
            return true;
        };
        const uint32_t rend = r ? (uint32_t)fn[r].skip : 0u;
        bool ok = r != 0 && inside_ancestors(r);
        std::vector<std::pair<Box, uint64_t>> uniq;
        std::vector<int32_t> slots;
        for (uint32_t i = 0; i < NN && ok; ++i) {
            if (fn[i].tri < 0 || (i >= r && i < rend)) continue;
            if (!inside_ancestors(i)) { ok = false; break; }
            const Box& lb = fn[i].box;
            size_t k = 0;
            while (k < uniq.size() && std::memcmp(&uniq[k].first, &lb, sizeof(Box)) != 0) ++k;
            if (k == uniq.size()) uniq.emplace_back(lb, 0ull);
            uniq[k].second |= 1ull << slots.size();
            slots.push_back(fn[i].tri);
        }
        if (ok && !slots.empty()) {
            out.split_root = r;
            out.split_end = rend;
            out.stri = slots;
            if (!near_first(r, rend, out.wcopies)) return false;   // the walked subtree's near-first orderings
            out.sboxes.resize(uniq.size() * 8);
            for (size_t k = 0; k < uniq.size(); ++k) {
                const Box& b = uniq[k].first;
                float* q = &out.sboxes[8 * k];
                q[0] = b.lo.x; q[1] = b.hi.x; q[2] = b.lo.y; q[3] = b.hi.y;
                q[4] = b.lo.z; q[5] = b.hi.z;
                q[6] = bits_as_float((int32_t)(uint32_t)uniq[k].second); q[7] = bits_as_float((int32_t)(uint32_t)(uniq[k].second >> 32));
            }
        }
    }
    // ---- near-first orderings of the whole tree for the Whitted kernel (scenes with point lights, config C3):
    // every internal box contains its children's (checked; with the tree's nesting every ancestor then
    // contains a leaf box), so for a finite ray a leaf's own slab test decides whether the reference reaches
    // it and any pre-order of any tree over the same leaf boxes visits the same candidates
    out.worders.clear();
    if (!lights_.empty() && NT > 64 && n_spheres == 0) {
        bool nested = true;
        auto inside = [](const Box& a, const Box& b) {   // b inside a
            return a.lo.x <= b.lo.x && a.lo.y <= b.lo.y && a.lo.z <= b.lo.z && a.hi.x >= b.hi.x && a.hi.y >= b.hi.y && a.hi.z >= b.hi.z;
        };
        for (uint32_t i = 0; i < NN && nested; ++i)
            if (fn[i].tri < 0) nested = inside(fn[i].box, fn[fn[i].left].box) && inside(fn[i].box, fn[fn[i].right].box);
        if (nested && !near_first(0, NN, out.worders)) return false;
    }
    out.tris.resize((size_t)NT * 16);
    out.dbg_tri_f.resize((size_t)NT * 13);
    out.dbg_tri_i.resize((size_t)NT * 2);
    for (uint32_t s = 0; s < NT; ++s) {
        const Tri& t = *slot_tri[s];
        if (t.sphere) {   // rt_layout.h: (center, material)(r^2, r, 0, id)(0, 0, 0, bits(1))(0)
            float* q = &out.tris[16 * (size_t)s];
            q[0] = t.a.x; q[1] = t.a.y; q[2] = t.a.z; q[3] = bits_as_float(t.mesh);
            q[4] = t.r2; q[5] = t.radius; q[6] = 0.0f; q[7] = bits_as_float(t.id);
            q[8] = q[9] = q[10] = 0.0f; q[11] = bits_as_float(1);
            q[12] = q[13] = q[14] = q[15] = 0.0f;
            float* d = &out.dbg_tri_f[13 * (size_t)s];
            d[0] = t.a.x; d[1] = t.a.y; d[2] = t.a.z; d[3] = t.radius; d[4] = t.r2;
            for (int k = 5; k < 12; ++k) d[k] = 0.0f;
            d[12] = t.area;
            out.dbg_tri_i[2 * s] = t.mesh; out.dbg_tri_i[2 * s + 1] = -2;
            continue;
        }
        const F3 e1 = sub(t.b, t.a), e2 = sub(t.c, t.a);
        float* q = &out.tris[16 * (size_t)s];
        q[0] = t.a.x; q[1] = t.a.y; q[2] = t.a.z; q[3] = bits_as_float(t.mesh);   // material id == mesh id
        q[4] = e1.x; q[5] = e1.y; q[6] = e1.z; q[7] = bits_as_float(t.id);
        q[8] = e2.x; q[9] = e2.y; q[10] = e2.z; q[11] = 0.0f;
        q[12] = t.n.x; q[13] = t.n.y; q[14] = t.n.z; q[15] = 0.0f;
        float* d = &out.dbg_tri_f[13 * (size_t)s];
        const F3 vv[4] = {t.a, t.b, t.c, t.n};
        for (int k = 0; k < 4; ++k) { d[3 * k] = vv[k].x; d[3 * k + 1] = vv[k].y; d[3 * k + 2] = vv[k].z; }
        d[12] = t.area;
        out.dbg_tri_i[2 * s] = t.mesh; out.dbg_tri_i[2 * s + 1] = t.mesh;
    }
    // ---- the triangles' vertices by slot (`tabc`), where every leaf's box is its triangle's vertex box
    // (Triangle::Get3DAABB, MC/TriangleMesh.h:96-99): the Whitted half-plane walk (RT_WH_HALF) stores its boxes
    // rounded outward and recomputes a hit leaf's exact box from them.  (Round 6: the vertex kernel's 16-bit compact
    // BVH that also lived here, RT_QBVH, is gone -- slower in every measurement)
    out.tabc.clear();
    out.hdr.has_vboxes = 0;
    if (NN > 0 && NT > 0 && n_spheres == 0) {
        bool ok = true;
        for (uint32_t i = 0; i < NN && ok; ++i) {
            const FN& n = fn[i];
            if (n.tri < 0) continue;
            const Tri& t = *slot_tri[n.tri];
            auto mn3 = [](float x, float y, float z) { return std::min(std::min(x, y), z); };
            auto mx3 = [](float x, float y, float z) { return std::max(std::max(x, y), z); };
            ok = mn3(t.a.x, t.b.x, t.c.x) == n.box.lo.x && mn3(t.a.y, t.b.y, t.c.y) == n.box.lo.y && mn3(t.a.z, t.b.z, t.c.z) == n.box.lo.z &&
                 mx3(t.a.x, t.b.x, t.c.x) == n.box.hi.x && mx3(t.a.y, t.b.y, t.c.y) == n.box.hi.y && mx3(t.a.z, t.b.z, t.c.z) == n.box.hi.z &&
                 n.skip == (int)i + 1;
        }
        if (ok) {
            out.tabc.resize((size_t)NT * 12);
            for (uint32_t s2 = 0; s2 < NT; ++s2) {
                const Tri& t = *slot_tri[s2];
                float* q = &out.tabc[12 * (size_t)s2];
                q[0] = t.a.x; q[1] = t.a.y; q[2] = t.a.z; q[3] = bits_as_float(t.mesh);
                q[4] = t.b.x; q[5] = t.b.y; q[6] = t.b.z; q[7] = bits_as_float(t.id);
                q[8] = t.c.x; q[9] = t.c.y; q[10] = t.c.z; q[11] = 0.0f;
            }
            out.hdr.has_vboxes = 1;
        }
    }
    // ---- the Whitted orderings in 16 bytes per node, where the exact leaf test has the vertices (tabc)
    out.worders_h.clear();
    if (!out.worders.empty() && out.hdr.has_vboxes && !compact_orderings(out.worders, NN, 0u, out.worders_h)) out.worders_h.clear();
    // ---- materials (one per mesh): brdf = diffuse_coefficient / PI, emitting = length(emission) > 1e-5
    const float PI = 3.141592653589793f;   // MC/WhittedUtilities.h:20
    out.mats.resize(nm * 8);
    int light = -1;
    for (size_t mi = 0; mi < nm; ++mi) {
        const MaterialDesc& m = meshes_[mi].material;
        const bool emitting = std::sqrt(dot(m.emission, m.emission)) > 0.00001f;   // MC/WhittedMaterial.h:34
        if (emitting && light < 0) {
            if (meshes_[mi].sphere) {
                // SamplingAreaLight would call Sphere::Sampling, which sets nothing (a TODO, MC/Sphere.h:30-33)
                err = "the first emissive entity is a sphere: the reference's Sphere::Sampling is unimplemented";
                return false;
            }
            light = (int)mi;
        }
        float* q = &out.mats[8 * mi];
        q[0] = m.albedo.x / PI; q[1] = m.albedo.y / PI; q[2] = m.albedo.z / PI; q[3] = emitting ? 1.0f : 0.0f;
        q[4] = m.emission.x; q[5] = m.emission.y; q[6] = m.emission.z; q[7] = 0.0f;
    }
    // ---- Whitted shading data: (diffuse color, phong_diffuse) per material; point lights; sky
    out.wmats.resize(nm * 4);
    for (size_t mi = 0; mi < nm; ++mi) {
        const MaterialDesc& m = meshes_[mi].material;
        float* q = &out.wmats[4 * mi];
        q[0] = m.albedo.x; q[1] = m.albedo.y; q[2] = m.albedo.z; q[3] = m.phong_diffuse;
    }
    out.plights.resize(lights_.size() * 8);
    for (size_t k = 0; k < lights_.size(); ++k) {
        float* q = &out.plights[8 * k];
        q[0] = lights_[k].position.x; q[1] = lights_[k].position.y; q[2] = lights_[k].position.z; q[3] = 0.0f;
        q[4] = lights_[k].radiance.x; q[5] = lights_[k].radiance.y; q[6] = lights_[k].radiance.z; q[7] = 0.0f;
    }
    out.hdr.n_plights = (uint32_t)lights_.size();
    out.hdr.sky[0] = sky_.x; out.hdr.sky[1] = sky_.y; out.hdr.sky[2] = sky_.z;
    // ---- light sampling tree: the light mesh's own BVH (BVH::Sampling_from_root)
    out.hdr.light_mesh = light;
    if (light >= 0) {
        const auto& mn = mesh_nodes[light];
        std::vector<int> order;   // pre-order, root first
        std::function<int(int)> lw = [&](int ni) -> int {
            const int me = (int)order.size();
            order.push_back(ni);
            if (mn[ni].left >= 0) { lw(mn[ni].left); lw(mn[ni].right); }
            return me;
        };
        lw(mesh_root[light]);
        std::vector<int> pos(mn.size(), -1);
        for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (int)k;
        out.lnodes.resize(order.size() * 4);
        std::vector<int> ltri_of;
        for (size_t k = 0; k < order.size(); ++k) {
            const BNode& b = mn[order[k]];
            float* q = &out.lnodes[4 * k];
            q[0] = b.area;
            if (b.left >= 0) { q[1] = bits_as_float(pos[b.left]); q[2] = bits_as_float(pos[b.right]); q[3] = bits_as_float(-1); }
            else { q[1] = bits_as_float(-1); q[2] = bits_as_float(-1); q[3] = bits_as_float((int)ltri_of.size()); ltri_of.push_back(b.item); }
        }
        out.ltris.resize(ltri_of.size() * 16);
        for (size_t k = 0; k < ltri_of.size(); ++k) {
            const Tri& t = tris[light][ltri_of[k]];
            float* q = &out.ltris[16 * k];
            q[0] = t.a.x; q[1] = t.a.y; q[2] = t.a.z; q[3] = 0;
            q[4] = t.b.x; q[5] = t.b.y; q[6] = t.b.z; q[7] = 0;
            q[8] = t.c.x; q[9] = t.c.y; q[10] = t.c.z; q[11] = 0;
            q[12] = t.n.x; q[13] = t.n.y; q[14] = t.n.z; q[15] = t.area;
        }
        out.hdr.light_area = mn[mesh_root[light]].area;
        // Scenes of <= 32 triangles (the vertex kernel's narrow leaf-box build): per light triangle, the
        // triangles no shadow ray toward a point q of it can be blocked by.  A triangle T whose vertices
        // lie within eta of the light triangle's plane, with a normal parallel to it (|cos| >= 0.999) and
        // no sliver corner at its first vertex (sin >= 0.1), meets a ray p -> q only within eta / |cos|
        // of q; the kernel skips these candidates when |cos| >= 0.25 (rt_coherent.hip bskip), where the
        // reference's t (mixed-precision Moller-Trumbore, MC/TriangleMesh.h:19-45) is within
        // 5 * 2^-24 * (|o - a| + t) / (0.1 * 0.2) <= 3e-5 * extent of the true one.  So t > slen - 0.01 and
        // `slen < t + 0.01f` (MC/Renderer.cpp:184) holds: T never occludes.  eta / 0.25 + 6e-5 * extent
        // must stay below 0.008, else no mask is set.
        // A split scene (larger scenes, <= 32 leaves outside the walked subtree) gets the same masks over its
        // outside slots: the kernel's split phase tests those leaves like the narrow build's triangles.
        const bool split_masks = NT > 32 && !out.stri.empty();
        if ((NT <= 32 || split_masks) && n_spheres == 0) {
            double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
            auto vert = [&](uint32_t s, int k, double v[3]) {
                const float* q = &out.tris[16 * (size_t)s];
                for (int a = 0; a < 3; ++a) v[a] = (double)q[a] + (k == 1 ? (double)q[4 + a] : k == 2 ? (double)q[8 + a] : 0.0);
            };
            for (uint32_t s = 0; s < NT; ++s)
                for (int k = 0; k < 3; ++k) {
                    double v[3];
                    vert(s, k, v);
                    for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], v[a]); hi[a] = std::max(hi[a], v[a]); }
                }
            const double extent = std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) + (hi[1] - lo[1]) * (hi[1] - lo[1]) + (hi[2] - lo[2]) * (hi[2] - lo[2]));
            const double eta = 0.0015;
            if (eta / 0.25 + 6e-5 * extent <= 0.008) {
                for (size_t k = 0; k < ltri_of.size(); ++k) {
                    float* lq = &out.ltris[16 * k];
                    double n[3] = {lq[12], lq[13], lq[14]};
                    const double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
                    if (!(nn > 0.0)) continue;
                    for (int a = 0; a < 3; ++a) n[a] /= nn;
                    const double d0 = n[0] * lq[0] + n[1] * lq[1] + n[2] * lq[2];
                    uint32_t mask = 0;
                    const uint32_t n_cand = split_masks ? (uint32_t)out.stri.size() : NT;
                    for (uint32_t k = 0; k < n_cand; ++k) {
                        const uint32_t s = split_masks ? (uint32_t)out.stri[k] : k;   // mask bit k: triangle s
                        const float* q = &out.tris[16 * (size_t)s];
                        bool near = true;
                        for (int kk = 0; kk < 3 && near; ++kk) {
                            double v[3];
                            vert(s, kk, v);
                            near = std::fabs(n[0] * v[0] + n[1] * v[1] + n[2] * v[2] - d0) <= eta;
                        }
                        const double e1[3] = {q[4], q[5], q[6]}, e2[3] = {q[8], q[9], q[10]};
                        const double c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
                        const double l1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]), l2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
                        const double lc = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
                        if (!near || !(lc >= 0.1 * l1 * l2) || !(lc > 0.0)) continue;
                        if (std::fabs((c[0] * n[0] + c[1] * n[1] + c[2] * n[2]) / lc) < 0.999) continue;
                        mask |= 1u << k;
                    }
                    std::memcpy(&lq[3], &mask, 4);
                }
            }
        }
        const MaterialDesc& m = meshes_[light].material;
        out.hdr.light_emission[0] = m.emission.x; out.hdr.light_emission[1] = m.emission.y; out.hdr.light_emission[2] = m.emission.z;
    }
    uint32_t depth = 0;
    {
        std::vector<uint32_t> lv(NN, 0);
        for (uint32_t i = 0; i < NN; ++i) {
            if (fn[i].left >= 0) { lv[fn[i].left] = lv[i] + 1; lv[fn[i].right] = lv[i] + 1; }
            depth = std::max(depth, lv[i]);
        }
    }
    out.hdr.n_nodes = NN; out.hdr.n_tris = NT; out.hdr.n_mats = (uint32_t)nm;
    out.hdr.n_lnodes = (uint32_t)(out.lnodes.size() / 4); out.hdr.n_ltris = (uint32_t)(out.ltris.size() / 16);
    out.hdr.max_depth = depth;
    out.hdr.n_spheres = n_spheres;
    return true;
}

}  // namespace rt
