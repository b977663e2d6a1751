// oracle/ref/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (container-side golden-vector generator).
//
// Compiled by oracle/Makefile (target `ref`) together with the reference's own, unmodified
// sources where they lie under /root/reference:
//   MC/Camera.cpp, WN/Walnut/Random.cpp, and (through this TU) the header-only MC geometry core
//   MC/{TriangleMesh,BVH,BoundingVolume,WhittedMaterial,Ray,IntersectionRecord,Entity,
//   VectorFloat,WhittedUtilities,OBJ_Loader}.h plus the vendored glm 0.9.9.9.
// Output goes only to oracle/_ref/.  Nothing under /root/reference is copied or modified.
//
// What is NOT compiled: MC/Renderer.{h,cpp}.  Renderer.h includes Walnut/Image.h, which includes
// <vulkan/vulkan.h>; the image has no Vulkan SDK, so the integrator is unbuildable here (DESIGN.md
// "Oracle").  The ~60 lines of integrator glue (Render / RayGen_Shader / cast_path / shading,
// MC/Renderer.cpp:91-214) are therefore RESTATED below, on top of the reference's compiled BVH,
// triangle, material, light-sampling and camera code ("hybrid" image fixtures).
//
// RNG injection: Walnut::Random keeps a thread_local std::mt19937 and a
// uniform_int_distribution<mt19937::result_type> (WN/Random.h:27-30,47-48).  On glibc
// result_type is 64-bit, which makes Float() return values up to 4.3e9; MSVC (the reference's
// platform) has a 32-bit result_type.  The harness (a) re-assigns the distribution's range to
// [0, 2^32-1] at start-up (MSVC behaviour), and (b) before every sample writes the
// untempered form of the frozen Philox stream (oracle/philox.h) into the engine state with
// position 0, so the reference's own Float() returns exactly the counter-based uniforms.
#include <iostream>
#include <fstream>
#include <sstream>
#include <filesystem>
#include <vector>
#include <string>
#include <algorithm>
#include <random>
#include <array>
#include <limits>
#include <cmath>
#include <cassert>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <map>
#include <thread>
#include <atomic>
#include <optional>
#include <chrono>
#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#define private public
#include "TriangleMesh.h"
#include "Sphere.h"
#include "Camera.h"
#undef private
#include "../philox.h"

#include "mt_inject.h"

// raw injection of an explicit list of u32 draws (unit cases)
static void inject_list(const std::vector<uint32_t>& v)
{
    MTLayout l;
    size_t n = std::min<size_t>(v.size(), 624);
    for (size_t i = 0; i < n; ++i) l.x[i] = mt_untemper(v[i]);
    for (size_t i = n; i < 624; ++i) l.x[i] = 0;
    l.p = 0;
    std::memcpy((void*)&Walnut::Random::s_RandomEngine, &l, sizeof l);
}

// ---------------------------------------------------------------------------------------------
// binary I/O helpers
// ---------------------------------------------------------------------------------------------
template <class T> static std::vector<T> read_all(const char* path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(2); }
    std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<T> v(b.size() / sizeof(T));
    std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
    return v;
}
struct Out {
    FILE* f;
    explicit Out(const char* p) { f = fopen(p, "wb"); if (!f) { fprintf(stderr, "cannot write %s\n", p); exit(2); } }
    ~Out() { fclose(f); }
    template <class T> void put(const T& v) { fwrite(&v, sizeof(T), 1, f); }
    void putv(const glm::vec3& v) { put(v.x); put(v.y); put(v.z); }
};

// ---------------------------------------------------------------------------------------------
// scene: the Cornell box exactly as Renderer::Renderer() builds it (MC/Renderer.cpp:26-57),
// plus optional extra OBJ meshes appended via Add + GenerateBVH (MC/Renderer.h:78-86).
// ---------------------------------------------------------------------------------------------
struct Scene {
    std::vector<Whitted::WhittedMaterial*> materials;
    std::vector<Whitted::Entity*> entities;
    AccelerationStructure::BVH* bvh = nullptr;
    std::map<const Whitted::Entity*, int> tri_index;   // TrianglePrimitive* -> flattened DFS leaf index
    std::map<const Whitted::WhittedMaterial*, int> mat_index;
    std::vector<int> mesh_material;
    std::map<const Whitted::Entity*, std::array<float, 4>> sphere_def;   // Whitted::Sphere entities: center, radius
};

static Scene* build_cornell(const std::string& dir, const std::vector<std::string>& extra_objs)
{
    Scene* s = new Scene;
    Whitted::WhittedMaterial* red = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
    red->diffuse_coefficient = glm::vec3{0.63f, 0.065f, 0.05f};
    Whitted::WhittedMaterial* green = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
    green->diffuse_coefficient = glm::vec3{0.1f, 0.5f, 0.1f};
    Whitted::WhittedMaterial* white = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
    white->diffuse_coefficient = glm::vec3{0.7f, 0.7f, 0.7f};
    Whitted::WhittedMaterial* light_material = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3(47.8f, 38.6f, 31.1f));
    light_material->diffuse_coefficient = glm::vec3{0.7f, 0.7f, 0.7f};
    s->materials = {red, green, white, light_material};
    for (int i = 0; i < 4; ++i) s->mat_index[s->materials[i]] = i;
    const char* names[6] = {"floor.obj", "shortbox.obj", "tallbox.obj", "left.obj", "right.obj", "light.obj"};
    Whitted::WhittedMaterial* mats[6] = {white, white, white, red, green, light_material};
    for (int i = 0; i < 6; ++i) {
        s->entities.push_back(new Whitted::TriangleMesh(dir + "/" + names[i], mats[i]));
        s->mesh_material.push_back(s->mat_index[mats[i]]);
    }
    for (const auto& p : extra_objs) {
        if (p.rfind("sphere:", 0) == 0) {
            // "sphere:cx:cy:cz:r:m": new Whitted::Sphere(center, radius, material m of {red, green, white, light})
            // (MC/Sphere.h:19-23), added after the Cornell meshes like any entity (MC/Renderer.h:78-81)
            float v[4]; int m = 2;
            if (std::sscanf(p.c_str(), "sphere:%f:%f:%f:%f:%d", &v[0], &v[1], &v[2], &v[3], &m) != 5 || m < 0 || m > 3) {
                fprintf(stderr, "bad sphere spec %s\n", p.c_str()); exit(2);
            }
            auto* sp = new Whitted::Sphere(glm::vec3{v[0], v[1], v[2]}, v[3], s->materials[m]);
            s->entities.push_back(sp);
            s->mesh_material.push_back(m);
            s->sphere_def[sp] = {v[0], v[1], v[2], v[3]};
            continue;
        }
        s->entities.push_back(new Whitted::TriangleMesh(p, white));
        s->mesh_material.push_back(2);
    }
    s->bvh = new AccelerationStructure::BVH{s->entities};
    return s;
}

// DFS pre-order flattening of the two-level tree: a top-level leaf (a TriangleMesh) is replaced by
// its mesh BVH root.  Records written: see gen_golden.py (NODE_DT / TRI_DT).
struct FlatNode { glm::vec3 mn, mx; float area; int32_t left, right, tri, mesh, top; };
struct FlatTri { glm::vec3 a, b, c, n; float area; int32_t mesh, material; };

static void flatten_mesh(Scene* s, AccelerationStructure::BVH_Node* node, int mesh, std::vector<FlatNode>& nodes, std::vector<FlatTri>& tris)
{
    int me = (int)nodes.size();
    nodes.push_back(FlatNode{node->bounding_volume.min_slab_values, node->bounding_volume.max_slab_values, node->mesh_area, -1, -1, -1, mesh, 0});
    if (!node->left && !node->right) {
        auto* t = dynamic_cast<Whitted::TrianglePrimitive*>(node->entity);
        int ti = (int)tris.size();
        s->tri_index[t] = ti;
        tris.push_back(FlatTri{t->vertice_a, t->vertice_b, t->vertice_c, t->m_surface_normal, t->area, mesh, s->mat_index[t->material]});
        nodes[me].tri = ti;
        return;
    }
    int l = (int)nodes.size();
    flatten_mesh(s, node->left, mesh, nodes, tris);
    int r = (int)nodes.size();
    flatten_mesh(s, node->right, mesh, nodes, tris);
    nodes[me].left = l; nodes[me].right = r;
}

static void flatten_top(Scene* s, AccelerationStructure::BVH_Node* node, std::vector<FlatNode>& nodes, std::vector<FlatTri>& tris)
{
    if (!node->left && !node->right) {
        auto* m = dynamic_cast<Whitted::TriangleMesh*>(node->entity);
        int mesh = (int)(std::find(s->entities.begin(), s->entities.end(), node->entity) - s->entities.begin());
        if (!m) {   // a sphere: one leaf, one slot (a = center, b = (radius, radius^2, 0), as rt_scene_export writes it)
            const auto& d = s->sphere_def.at(node->entity);
            const int ti = (int)tris.size();
            s->tri_index[node->entity] = ti;
            tris.push_back(FlatTri{glm::vec3{d[0], d[1], d[2]}, glm::vec3{d[3], d[3] * d[3], 0.0f}, glm::vec3{0.0f}, glm::vec3{0.0f},
                                   node->entity->GetArea(), mesh, s->mesh_material[mesh]});
            nodes.push_back(FlatNode{node->bounding_volume.min_slab_values, node->bounding_volume.max_slab_values, node->mesh_area, -1, -1,
                                     ti, mesh, 0});
            return;
        }
        // the top-level leaf box must equal the mesh-root box for the flattening to be exact
        const auto& tb = node->bounding_volume; const auto& mb = m->bvh->root->bounding_volume;
        if (tb.min_slab_values != mb.min_slab_values || tb.max_slab_values != mb.max_slab_values) { fprintf(stderr, "mesh box mismatch\n"); exit(4); }
        flatten_mesh(s, m->bvh->root, mesh, nodes, tris);
        return;
    }
    int me = (int)nodes.size();
    nodes.push_back(FlatNode{node->bounding_volume.min_slab_values, node->bounding_volume.max_slab_values, node->mesh_area, -1, -1, -1, -1, 1});
    int l = (int)nodes.size();
    flatten_top(s, node->left, nodes, tris);
    int r = (int)nodes.size();
    flatten_top(s, node->right, nodes, tris);
    nodes[me].left = l; nodes[me].right = r;
}

// ---------------------------------------------------------------------------------------------
// integrator glue RESTATED from MC/Renderer.cpp (unbuildable here, see header)
// ---------------------------------------------------------------------------------------------
struct Counters { uint64_t rays = 0; uint64_t draws = 0; uint64_t samples = 0; uint64_t shading = 0; };
static thread_local Counters g_cnt;

struct Hybrid {
    Scene* s;
    float rr;
    Whitted::IntersectionRecord trace(const AccelerationStructure::Ray& ray) const
    {   // Renderer::ray_BVH_intersection_record, MC/Renderer.h:88-91
        g_cnt.rays++;
        return s->bvh->traverse_BVH_from_root(ray);
    }
    void sampling_area_light(Whitted::IntersectionRecord& sample, float& pdf) const
    {   // Renderer::SamplingAreaLight, MC/Renderer.h:163-180
        for (uint32_t n = 0; n < s->entities.size(); n++) {
            if (s->entities[n]->IsEmissive()) { s->entities[n]->Sampling(sample, pdf); break; }
        }
    }
    glm::vec3 shading(const Whitted::IntersectionRecord& record, const glm::vec3& W_out) const
    {   // Renderer::shading, MC/Renderer.cpp:148-214
        g_cnt.shading++;
        g_inj.refill_if_near(6);   // harness: keep the injected stream from twisting (mt_inject.h)
        if (record.hitted_entity_material->IsEmitting()) return record.hitted_entity_material->GetEmission();
        glm::vec3 n = record.surface_normal;
        if (glm::dot(record.surface_normal, W_out) < 0.0f) n = -(record.surface_normal);
        glm::vec3 p = record.location + n * INTERSECTION_CORRECTION;
        glm::vec3 radiance_direct = glm::vec3{0.0f, 0.0f, 0.0f};
        Whitted::IntersectionRecord ls;
        float ls_pdf;
        sampling_area_light(ls, ls_pdf);
        glm::vec3 q = ls.location;
        glm::vec3 p2q = q - p;
        glm::vec3 wl = glm::normalize(p2q);
        glm::vec3 nl = ls.surface_normal;
        if (glm::dot(ls.surface_normal, -wl) < 0.0f) nl = -(ls.surface_normal);
        Whitted::IntersectionRecord occ = trace(AccelerationStructure::Ray{p, wl});
        if (glm::length(p2q) < occ.t + 0.01f) {
            radiance_direct = ls.emission * record.hitted_entity_material->BRDF(W_out, wl, n) * glm::dot(wl, n) * glm::dot(-wl, nl) / (glm::dot(p2q, p2q)) / (ls_pdf);
        }
        glm::vec3 radiance_indirect = glm::vec3{0.0f, 0.0f, 0.0f};
        if (Whitted::get_random_float_0_1() < rr) {
            glm::vec3 W_in = glm::normalize(record.hitted_entity_material->Sampling(W_out, n));
            float PDF = record.hitted_entity_material->PDF_at_the_sample(W_out, W_in, n);
            Whitted::IntersectionRecord deeper = trace(AccelerationStructure::Ray{p, W_in});
            if (deeper.has_intersection && (!deeper.hitted_entity_material->IsEmitting())) {
                radiance_indirect = shading(deeper, -W_in) * record.hitted_entity_material->BRDF(W_out, W_in, n) * glm::dot(W_in, n) / PDF / rr;
            }
        }
        return radiance_direct + radiance_indirect;
    }
    glm::vec3 cast_path(const AccelerationStructure::Ray& ray) const
    {   // Renderer::cast_path, MC/Renderer.cpp:136-146
        Whitted::IntersectionRecord record = trace(ray);
        if (record.has_intersection) return shading(record, -(ray.m_direction));
        return glm::vec3{12 / 255.0f, 20 / 255.0f, 69 / 255.0f};
    }
};

static uint32_t vecRGBA_to_0xABGR(const glm::vec4& c)
{   // RTUtility::vecRGBA_to_0xABGR, MC/Renderer.cpp:15-23
    uint8_t r = (uint8_t)(c.r * 255.0f);
    uint8_t g = (uint8_t)(c.g * 255.0f);
    uint8_t b = (uint8_t)(c.b * 255.0f);
    uint8_t a = (uint8_t)(c.a * 255.0f);
    return ((a << 24) | (b << 16) | (g << 8) | r);
}

// camera direction of one pixel: the loop body of Camera::RecomputeRayDirections (MC/Camera.cpp:119-125),
// evaluated with the reference Camera's own matrices; the two Float() draws come from the injected engine.
static glm::vec3 camera_dir(const Camera& cam, uint32_t x, uint32_t y, uint32_t W, uint32_t H)
{
    glm::vec2 coordinate{((float)x + Walnut::Random::Float()) / W, ((float)y + Walnut::Random::Float()) / H};
    coordinate = coordinate * 2.0f - 1.0f;
    glm::vec4 target{cam.InverseProjectionMatrix() * glm::vec4{coordinate.x, coordinate.y, 1, 1}};
    glm::vec3 ray_direction{glm::vec3{cam.InverseViewMatrix() * glm::vec4{glm::normalize(glm::vec3{target} / target.w), 0}}};
    return ray_direction;
}

// ---------------------------------------------------------------------------------------------
// commands
// ---------------------------------------------------------------------------------------------
static std::vector<std::string> split_extra(const char* s)
{
    std::vector<std::string> v;
    if (!s || !*s) return v;
    std::string cur;
    for (const char* p = s; ; ++p) {
        if (*p == ',' || *p == 0) { if (!cur.empty()) v.push_back(cur); cur.clear(); if (!*p) break; }
        else cur += *p;
    }
    return v;
}

static int cmd_scene(const char* dir, const char* extra, const char* out_nodes, const char* out_tris, const char* out_meshes)
{
    Scene* s = build_cornell(dir, split_extra(extra));
    std::vector<FlatNode> nodes; std::vector<FlatTri> tris;
    flatten_top(s, s->bvh->root, nodes, tris);
    {
        Out o(out_nodes);
        for (auto& n : nodes) { o.putv(n.mn); o.putv(n.mx); o.put(n.area); o.put(n.left); o.put(n.right); o.put(n.tri); o.put(n.mesh); o.put(n.top); }
    }
    {
        Out o(out_tris);
        for (auto& t : tris) { o.putv(t.a); o.putv(t.b); o.putv(t.c); o.putv(t.n); o.put(t.area); o.put(t.mesh); o.put(t.material); }
    }
    {
        Out o(out_meshes);   // per mesh: raw objl positions are dumped by cmd_objraw; here area/box/material
        for (size_t i = 0; i < s->entities.size(); ++i) {
            Whitted::Entity* e = s->entities[i];
            const auto box = e->Get3DAABB();
            o.put(e->GetArea()); o.putv(box.min_slab_values); o.putv(box.max_slab_values);
            o.put((int32_t)s->mesh_material[i]); o.put((int32_t)(e->IsEmissive() ? 1 : 0));
        }
    }
    printf("nodes %zu tris %zu meshes %zu\n", nodes.size(), tris.size(), s->entities.size());
    return 0;
}

// raw objl positions (pre-scale, de-indexed) of one OBJ, as the reference loader produces them
static int cmd_objraw(const char* path, const char* out)
{
    objl::Loader L;
    if (!L.LoadFile(path)) { fprintf(stderr, "load failed\n"); return 1; }
    Out o(out);
    const auto& V = L.LoadedMeshes[0].Vertices;
    for (auto& v : V) { o.put(v.Position.X); o.put(v.Position.Y); o.put(v.Position.Z); }
    printf("meshes %zu verts %zu\n", L.LoadedMeshes.size(), V.size());
    return 0;
}

static int cmd_rays(const char* dir, const char* extra, const char* in_rays, const char* out)
{
    Scene* s = build_cornell(dir, split_extra(extra));
    std::vector<FlatNode> nodes; std::vector<FlatTri> tris;
    flatten_top(s, s->bvh->root, nodes, tris);
    auto r = read_all<float>(in_rays);
    size_t n = r.size() / 6;
    Out o(out);
    for (size_t i = 0; i < n; ++i) {
        glm::vec3 org{r[6 * i], r[6 * i + 1], r[6 * i + 2]}, d{r[6 * i + 3], r[6 * i + 4], r[6 * i + 5]};
        Whitted::IntersectionRecord rec = s->bvh->traverse_BVH_from_root(AccelerationStructure::Ray{org, d});
        int32_t hit = rec.has_intersection ? 1 : 0;
        int32_t ti = hit ? s->tri_index[rec.hitted_entity] : -1;
        int32_t mat = hit ? s->mat_index[rec.hitted_entity_material] : -1;
        o.put(hit); o.put(ti); o.put(mat); o.put(rec.t); o.putv(rec.location); o.putv(rec.surface_normal);
    }
    printf("rays %zu\n", n);
    return 0;
}

static int cmd_mt(const char* in, const char* out)
{
    auto v = read_all<float>(in);
    size_t n = v.size() / 15;
    Out o(out);
    for (size_t i = 0; i < n; ++i) {
        const float* c = &v[15 * i];
        double t = 0.0;
        bool h = Whitted::RayTriangleIntersection(glm::vec3{c[0], c[1], c[2]}, glm::vec3{c[3], c[4], c[5]}, glm::vec3{c[6], c[7], c[8]},
                                                   glm::vec3{c[9], c[10], c[11]}, glm::vec3{c[12], c[13], c[14]}, t);
        o.put((int32_t)h); o.put(t);
    }
    printf("mt %zu\n", n);
    return 0;
}

static int cmd_aabb(const char* in, const char* out)
{
    auto v = read_all<float>(in);
    size_t n = v.size() / 12;
    Out o(out);
    for (size_t i = 0; i < n; ++i) {
        const float* c = &v[12 * i];
        AccelerationStructure::AABB_3D box;
        box.min_slab_values = glm::vec3{c[0], c[1], c[2]};
        box.max_slab_values = glm::vec3{c[3], c[4], c[5]};
        AccelerationStructure::Ray ray{glm::vec3{c[6], c[7], c[8]}, glm::vec3{c[9], c[10], c[11]}};
        std::array<int, 3> neg{ray.m_direction.x < 0.0f, ray.m_direction.y < 0.0f, ray.m_direction.z < 0.0f};
        o.put((int32_t)box.intersects_with_ray(ray, ray.direction_reciprocal, neg));
    }
    printf("aabb %zu\n", n);
    return 0;
}

// light sampling: SamplingAreaLight with 3 injected draws per case (MC/Renderer.h:163-180, MC/BVH.h:103-129,
// MC/TriangleMesh.h:69-89,193-197)
static int cmd_light(const char* dir, const char* in_u32, const char* out)
{
    Scene* s = build_cornell(dir, {});
    Hybrid h{s, 0.8f};
    auto u = read_all<uint32_t>(in_u32);
    size_t n = u.size() / 3;
    Out o(out);
    for (size_t i = 0; i < n; ++i) {
        inject_list({u[3 * i], u[3 * i + 1], u[3 * i + 2]});
        Whitted::IntersectionRecord rec; float pdf = -1.0f;
        h.sampling_area_light(rec, pdf);
        o.putv(rec.location); o.putv(rec.surface_normal); o.putv(rec.emission); o.put(pdf);
    }
    printf("light %zu\n", n);
    return 0;
}

// material: Sampling (2 injected draws) + normalize (as the caller does, MC/Renderer.cpp:196), BRDF, PDF
static int cmd_material(const char* in, const char* out)
{
    auto v = read_all<uint32_t>(in);   // per case: n.xyz (f32 bits), wi.xyz (f32 bits), u_z, u_phi, albedo index
    size_t n = v.size() / 9;
    Whitted::WhittedMaterial m(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f});
    const glm::vec3 albedo[3] = {{0.63f, 0.065f, 0.05f}, {0.1f, 0.5f, 0.1f}, {0.7f, 0.7f, 0.7f}};
    Out o(out);
    for (size_t i = 0; i < n; ++i) {
        float f[6];
        std::memcpy(f, &v[9 * i], 24);
        glm::vec3 nn{f[0], f[1], f[2]}, wi{f[3], f[4], f[5]};
        m.diffuse_coefficient = albedo[v[9 * i + 8] % 3];
        inject_list({v[9 * i + 6], v[9 * i + 7]});
        glm::vec3 raw = m.Sampling(-wi, nn);
        glm::vec3 s = glm::normalize(raw);
        glm::vec3 brdf = m.BRDF(-wi, wi, nn);
        float pdf = m.PDF_at_the_sample(-wi, s, nn);
        o.putv(raw); o.putv(s); o.putv(brdf); o.put(pdf);
    }
    printf("material %zu\n", n);
    return 0;
}

static int cmd_camera(uint32_t W, uint32_t H, uint32_t frame, uint64_t seed, const char* out)
{
    Camera cam{35.0f, 0.1f, 100.0f};   // MC/mainloop.cpp:22
    bool inject = (uint64_t)W * H * 2 <= 624;
    if (inject) {
        std::vector<uint32_t> l;
        for (uint32_t p = 0; p < W * H; ++p) { l.push_back(oracle_rng_u32(seed, p, frame, 0)); l.push_back(oracle_rng_u32(seed, p, frame, 1)); }
        inject_list(l);
    }
    cam.ResizeViewport(W, H);
    Out o(out);
    auto putm = [&](const glm::mat4& m) { for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) o.put(m[c][r]); };
    putm(cam.ProjectionMatrix()); putm(cam.InverseProjectionMatrix()); putm(cam.ViewMatrix()); putm(cam.InverseViewMatrix());
    o.putv(cam.Position()); o.putv(cam.ForwardDirection());
    o.put((int32_t)inject);
    if (inject) for (auto& d : cam.RayDirections()) o.putv(d);
    printf("camera %ux%u inject=%d\n", W, H, (int)inject);
    return 0;
}

// (row_stride > 1: only the rows y % row_stride == row_offset are rendered -- a full-spp fixture of selected rows; the
// others stay zero)
static int cmd_image(const char* dir, const char* extra, uint32_t W, uint32_t H, uint32_t spp, uint64_t seed, float rr, int threads,
                     const char* out_accum, const char* out_rgba, const char* out_stats, uint32_t row_stride = 1, uint32_t row_offset = 0)
{
    Scene* s = build_cornell(dir, split_extra(extra));
    Camera cam{35.0f, 0.1f, 100.0f};
    cam.ResizeViewport(W, H);   // matrices only; its own jitter draws are irrelevant here
    Hybrid h{s, rr};
    std::vector<float> accum((size_t)W * H * 4, 0.0f);
    std::vector<uint32_t> rgba((size_t)W * H, 0);
    std::atomic<uint32_t> next_row{0};
    std::atomic<uint64_t> rays{0}, draws{0}, shading{0}, overflow{0};
    auto worker = [&]() {
        set_msvc_distribution();
        Counters local;
        for (;;) {
            uint32_t y = next_row.fetch_add(1) * row_stride + row_offset;
            if (y >= H) break;
            for (uint32_t x = 0; x < W; ++x) {
                uint32_t px = y * W + x;
                glm::vec4 acc{0.0f};
                for (uint32_t f = 1; f <= spp; ++f) {
                    // A first fill of 64 words covers nearly every path; a longer one is re-filled at
                    // the top of a shading call (mt_inject.h refill_if_near), so the engine never twists.
                    g_cnt = Counters{};
                    g_inj.start(seed, px, f, std::min<uint32_t>(64, g_fill_words));
                    // RayGen_Shader, MC/Renderer.cpp:124-134 (camera direction drawn first, as
                    // UpdateCamera -> RecomputeRayDirections precedes Render, MC/mainloop.cpp:32-41)
                    glm::vec3 dir = camera_dir(cam, x, y, W, H);
                    glm::vec3 L = h.cast_path(AccelerationStructure::Ray{cam.Position(), Whitted::normalize(dir)});
                    uint32_t used = g_inj.used();
                    if (used == 0xFFFFFFFFu) { overflow++; used = 0; }
                    local.rays += g_cnt.rays; local.shading += g_cnt.shading; local.draws += used;
                    glm::vec4 color_rgba{L, 1.0f};
                    acc += color_rgba;
                    glm::vec4 fin = acc / (float)f;
                    fin = glm::clamp(fin, glm::vec4(0.0f), glm::vec4(1.0f));
                    rgba[px] = vecRGBA_to_0xABGR(fin);
                }
                std::memcpy(&accum[4 * (size_t)px], &acc, 16);
            }
        }
        rays += local.rays; draws += local.draws; shading += local.shading;
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
    { Out o(out_accum); fwrite(accum.data(), 4, accum.size(), o.f); }
    { Out o(out_rgba); fwrite(rgba.data(), 4, rgba.size(), o.f); }
    { Out o(out_stats); o.put((uint64_t)rays); o.put((uint64_t)draws); o.put((uint64_t)shading); o.put((uint64_t)overflow); o.put((uint64_t)W * H * spp); }
    printf("image %ux%u spp %u rays/sample %.4f draws/sample %.4f overflow %llu\n", W, H, spp,
           (double)rays / ((double)W * H * spp), (double)draws / ((double)W * H * spp), (unsigned long long)overflow);
    return overflow ? 5 : 0;
}

// The SHIPPED random stream, serially (statistical gate): one persistent
// thread_local std::mt19937 default-seeded with 5489 (WN/Random.cpp:5), the MSVC 32-bit distribution,
// and the reference's draw order per frame: Camera::RecomputeRayDirections draws 2 uniforms per
// pixel y-major (MC/Camera.cpp:114-132, via UpdateCamera before Render, MC/mainloop.cpp:32-41), then
// Render's pixel loop runs y-major (serial under libstdc++ without TBB, MC/Renderer.cpp:100-110).
// No injection: this is the reference's own sequence, for the statistical comparison only.
static int cmd_image_mt(const char* dir, uint32_t W, uint32_t H, uint32_t spp, float rr, const char* out_accum)
{
    Scene* s = build_cornell(dir, {});
    Camera cam{35.0f, 0.1f, 100.0f};
    cam.ResizeViewport(W, H);
    Walnut::Random::s_RandomEngine.seed(5489u);
    set_msvc_distribution();
    read_fill_words();
    Hybrid h{s, rr};
    std::vector<glm::vec4> acc((size_t)W * H, glm::vec4(0.0f));
    std::vector<glm::vec3> dirs((size_t)W * H);
    for (uint32_t f = 1; f <= spp; ++f) {
        for (uint32_t y = 0; y < H; ++y)
            for (uint32_t x = 0; x < W; ++x) dirs[(size_t)y * W + x] = camera_dir(cam, x, y, W, H);
        for (uint32_t y = 0; y < H; ++y)
            for (uint32_t x = 0; x < W; ++x) {
                const size_t px = (size_t)y * W + x;
                acc[px] += glm::vec4{h.cast_path(AccelerationStructure::Ray{cam.Position(), Whitted::normalize(dirs[px])}), 1.0f};
            }
    }
    Out o(out_accum);
    fwrite(acc.data(), 16, acc.size(), o.f);
    printf("image_mt %ux%u spp %u\n", W, H, spp);
    return 0;
}

// CPU BASELINE timing (bench.py cpu_baseline, tools/cpu_reference_configs.py): the reference's work per
// frame with its SHIPPED random stream -- thread_local std::mt19937 default-seeded 5489 behind the MSVC
// 32-bit distribution (WN/Random.h:27-30,47-48, WN/Random.cpp:5-6), no injection -- on a persistent
// pool of `threads` std::threads (the std::execution::par row loop of Renderer::Render,
// MC/Renderer.cpp:100-110; a pool created once, so no thread re-seeds its engine per frame, SURVEY.md
// section 8(c) pitfall).  Per frame and pixel: the jittered camera direction (Camera::
// RecomputeRayDirections' loop body, MC/Camera.cpp:119-125 -- run row-parallel here; the reference runs
// it serially on the UI thread, which would only make the baseline slower), RayGen_Shader (cast_path,
// accum += color, accum / frame, clamp, ABGR pack: MC/Renderer.cpp:124-134).  Frames are separated by a
// barrier, as consecutive Render() calls are.  Prints one line: samples, seconds (scene build excluded).
static int cmd_bench_mt(const char* dir, const char* extra, uint32_t W, uint32_t H, uint32_t spp, float rr, int threads)
{
    Scene* s = build_cornell(dir, split_extra(extra));
    Camera cam{35.0f, 0.1f, 100.0f};
    cam.ResizeViewport(W, H);
    Hybrid h{s, rr};
    std::vector<glm::vec4> acc((size_t)W * H, glm::vec4(0.0f));
    std::vector<uint32_t> rgba((size_t)W * H, 0);
    std::vector<std::atomic<uint32_t>> next(spp + 1);
    for (auto& a : next) a.store(0);
    std::atomic<int> arrived{0};
    std::atomic<uint32_t> generation{0};
    auto barrier = [&]() {   // sense-reversing spin barrier between frames (Render() calls)
        const uint32_t g = generation.load();
        if (arrived.fetch_add(1) + 1 == threads) { arrived.store(0); generation.fetch_add(1); }
        else while (generation.load() == g) std::this_thread::yield();
    };
    auto worker = [&]() {
        set_msvc_distribution();   // the shipped engine of this thread: default-seeded (5489), never re-seeded
        std::vector<glm::vec3> row(W);
        for (uint32_t f = 1; f <= spp; ++f) {
            for (;;) {
                const uint32_t y = next[f].fetch_add(1);
                if (y >= H) break;
                for (uint32_t x = 0; x < W; ++x) row[x] = camera_dir(cam, x, y, W, H);
                for (uint32_t x = 0; x < W; ++x) {
                    const size_t px = (size_t)y * W + x;
                    acc[px] += glm::vec4{h.cast_path(AccelerationStructure::Ray{cam.Position(), Whitted::normalize(row[x])}), 1.0f};
                    glm::vec4 fin = acc[px] / (float)f;
                    fin = glm::clamp(fin, glm::vec4(0.0f), glm::vec4(1.0f));
                    rgba[px] = vecRGBA_to_0xABGR(fin);
                }
            }
            barrier();
        }
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t chk = 0;
    for (uint32_t v : rgba) chk += v;
    printf("bench_mt samples %llu seconds %.6f threads %d checksum %llu\n", (unsigned long long)((uint64_t)W * H * spp), sec, threads,
           (unsigned long long)chk);
    return 0;
}

int main(int argc, char** argv)
{
    check_layout_once();
    set_msvc_distribution();
    read_fill_words();
    if (argc < 2) { fprintf(stderr, "usage: ref_harness <cmd> ...\n"); return 1; }
    std::string c = argv[1];
    if (c == "scene" && argc == 7) return cmd_scene(argv[2], argv[3], argv[4], argv[5], argv[6]);
    if (c == "objraw" && argc == 4) return cmd_objraw(argv[2], argv[3]);
    if (c == "rays" && argc == 6) return cmd_rays(argv[2], argv[3], argv[4], argv[5]);
    if (c == "mt" && argc == 4) return cmd_mt(argv[2], argv[3]);
    if (c == "aabb" && argc == 4) return cmd_aabb(argv[2], argv[3]);
    if (c == "light" && argc == 5) return cmd_light(argv[2], argv[3], argv[4]);
    if (c == "material" && argc == 4) return cmd_material(argv[2], argv[3]);
    if (c == "camera" && argc == 7) return cmd_camera(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), strtoull(argv[5], 0, 10), argv[6]);
    if (c == "image_mt" && argc == 8)
        return cmd_image_mt(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), (float)atof(argv[6]), argv[7]);
    if (c == "bench_mt" && argc == 9)
        return cmd_bench_mt(argv[2], argv[3], atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), (float)atof(argv[7]), atoi(argv[8]));
    if (c == "image" && argc >= 13 && argc <= 15)
        return cmd_image(argv[2], argv[3], atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), strtoull(argv[7], 0, 10), (float)atof(argv[8]), atoi(argv[9]),
                         argv[10], argv[11], argv[12], argc >= 14 ? (uint32_t)std::max(1, atoi(argv[13])) : 1u,
                         argc >= 15 ? (uint32_t)std::max(0, atoi(argv[14])) : 0u);
    fprintf(stderr, "bad command\n");
    return 1;
}
