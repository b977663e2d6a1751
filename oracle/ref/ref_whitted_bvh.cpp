// oracle/ref/ref_whitted_bvh.cpp -- TEST INFRASTRUCTURE ONLY (container-side golden-vector generator)
// for the reference's "BVH Ray Tracer" (config C3: Whitted-style shading of the Stanford bunny and
// the Utah teapot).  BV/ = "BVH Ray Tracer/8599RayTracerGUI/src/".
//
// Compiled by oracle/Makefile (target `ref`) with the reference's own, unmodified sources where they
// lie under /root/reference: BV/Camera.cpp, the header-only geometry core BV/{TriangleMesh,BVH,
// BoundingVolume,Ray,IntersectionRecord,Entity,WhittedMaterial,LightSource,VectorFloat,
// WhittedUtilities,OBJ_Loader}.h, and the vendored glm.  Output goes only to oracle/_ref/.
//
// Not compiled: BV/Renderer.{h,cpp} (Renderer.h includes Walnut/Image.h -> <vulkan/vulkan.h>, absent
// from the image).  The shading glue of Renderer::Renderer / RayGen_Shader / cast_Whitted_ray
// (BV/Renderer.cpp:26-43,109-233) is therefore RESTATED below on top of the reference's compiled
// BVH, triangle-mesh and camera code.  The scene has only Diffuse_Glossy triangles
// (BV/TriangleMesh.h:138-141), so only that branch of the material switch is restated.
#include <iostream>
#include <sstream>
#include <filesystem>
#include <random>
#include <optional>
#include <algorithm>
#include <array>
#include <atomic>
#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>
#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#define private public
#include "TriangleMesh.h"
#include "LightSource.h"
#include "Camera.h"
#undef private

namespace {

struct Out {
    FILE* f;
    explicit Out(const char* p) { f = fopen(p, "wb"); if (!f) { fprintf(stderr, "cannot write %s\n", p); exit(2); } }
    ~Out() { fclose(f); }
    template <class T> void put(const T& v) { fwrite(&v, sizeof(T), 1, f); }
    void putv(const glm::vec3& v) { put(v.x); put(v.y); put(v.z); }
};

template <class T> std::vector<T> read_all(const char* path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(2); }
    std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<T> v(b.size() / sizeof(T));
    std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
    return v;
}

// Renderer::Renderer(), BV/Renderer.cpp:26-43
struct Scene {
    std::vector<Whitted::Entity*> entities;
    std::vector<std::unique_ptr<Whitted::PointLightSource>> lights;
    AccelerationStructure::BVH* bvh = nullptr;
    std::map<const Whitted::Entity*, int> tri_index;
};

Scene* build_scene(const char* bunny, const char* teapot)
{
    Scene* s = new Scene;
    s->entities.push_back(new Whitted::TriangleMesh(bunny, 2, glm::vec3{-1, 6.1, 0}));
    s->entities.push_back(new Whitted::TriangleMesh(teapot, 1, glm::vec3{-1, 3, 0}));
    s->lights.push_back(std::make_unique<Whitted::PointLightSource>(glm::vec3(-20.0f, 70.0f, 20.0f), glm::vec3(1.0f)));
    s->lights.push_back(std::make_unique<Whitted::PointLightSource>(glm::vec3(20.0f, 70.0f, 20.0f), glm::vec3(1.0f)));
    s->bvh = new AccelerationStructure::BVH{s->entities};
    return s;
}

// DFS pre-order flattening (top-level mesh leaves replaced by the mesh BVH roots), as for the MC harness
struct FlatNode { glm::vec3 mn, mx; float area; int32_t left, right, tri, mesh, top; };
struct FlatTri { glm::vec3 a, b, c, n; float area; int32_t mesh, material; };

void flatten_mesh(Scene* s, AccelerationStructure::BVH_Node* node, int mesh, std::vector<FlatNode>& nodes, std::vector<FlatTri>& tris)
{
    int me = (int)nodes.size();
    nodes.push_back(FlatNode{node->bounding_volume.min_slab_values, node->bounding_volume.max_slab_values, 0.0f, -1, -1, -1, mesh, 0});
    if (!node->left && !node->right) {
        auto* t = dynamic_cast<Whitted::TrianglePrimitive*>(node->entity);
        int ti = (int)tris.size();
        s->tri_index[t] = ti;
        tris.push_back(FlatTri{t->vertice_a, t->vertice_b, t->vertice_c, t->m_surface_normal, 0.0f, mesh, 0});
        nodes[me].tri = ti;
        return;
    }
    int l = (int)nodes.size();
    flatten_mesh(s, node->left, mesh, nodes, tris);
    int r = (int)nodes.size();
    flatten_mesh(s, node->right, mesh, nodes, tris);
    nodes[me].left = l; nodes[me].right = r;
}

void flatten_top(Scene* s, AccelerationStructure::BVH_Node* node, std::vector<FlatNode>& nodes, std::vector<FlatTri>& tris)
{
    if (!node->left && !node->right) {
        auto* m = dynamic_cast<Whitted::TriangleMesh*>(node->entity);
        int mesh = (int)(std::find(s->entities.begin(), s->entities.end(), node->entity) - s->entities.begin());
        const auto& tb = node->bounding_volume; const auto& mb = m->bvh->root->bounding_volume;
        if (tb.min_slab_values != mb.min_slab_values || tb.max_slab_values != mb.max_slab_values) { fprintf(stderr, "mesh box mismatch\n"); exit(4); }
        flatten_mesh(s, m->bvh->root, mesh, nodes, tris);
        return;
    }
    int me = (int)nodes.size();
    nodes.push_back(FlatNode{node->bounding_volume.min_slab_values, node->bounding_volume.max_slab_values, 0.0f, -1, -1, -1, -1, 1});
    int l = (int)nodes.size();
    flatten_top(s, node->left, nodes, tris);
    int r = (int)nodes.size();
    flatten_top(s, node->right, nodes, tris);
    nodes[me].left = l; nodes[me].right = r;
}

std::atomic<uint64_t> g_rays{0};

// Renderer::cast_Whitted_ray, BV/Renderer.cpp:121-233, Diffuse_Glossy branch (:172-229) -- RESTATED
glm::vec3 cast_whitted_ray(const Scene* s, const AccelerationStructure::Ray& ray, uint64_t& rays)
{
    const glm::vec3 sky_color{0.2f, 0.7f, 0.8f};   // BV/Renderer.h:189
    if (ray.m_direction == glm::vec3{0.0f, 0.0f, 0.0f}) return glm::vec3{0.0f, 0.0f, 0.0f};
    glm::vec3 ray_color = sky_color;
    rays++;
    Whitted::IntersectionRecord record = s->bvh->traverse_BVH_from_root(ray);
    if (record.has_intersection) {
        if (record.hitted_entity_material->GetMaterialNature() != Whitted::Diffuse_Glossy) { fprintf(stderr, "unexpected material\n"); exit(6); }
        glm::vec3 intersection = record.location;
        glm::vec3 normal_at_intersection = record.surface_normal;
        glm::vec3 total_radiance_diffuse{0.0f, 0.0f, 0.0f};
        glm::vec3 total_radiance_specular{0.0f, 0.0f, 0.0f};
        glm::vec3 shading_point = (glm::dot(ray.m_direction, normal_at_intersection) < 0.0f)
                                      ? (intersection + normal_at_intersection * INTERSECTION_CORRECTION)
                                      : (intersection - normal_at_intersection * INTERSECTION_CORRECTION);
        for (const auto& light_source : s->lights) {
            glm::vec3 light_source_direction = light_source->m_light_source_origin - intersection;
            float light_distance_squared = glm::dot(light_source_direction, light_source_direction);
            light_source_direction = Whitted::normalize(light_source_direction);
            rays++;
            Whitted::IntersectionRecord shadow_record = s->bvh->traverse_BVH_from_root(AccelerationStructure::Ray{shading_point, light_source_direction});
            if ((shadow_record.has_intersection) && (shadow_record.t * shadow_record.t < light_distance_squared)) continue;
            total_radiance_diffuse += light_source->m_radiance * std::fabs(glm::dot(light_source_direction, normal_at_intersection));
            glm::vec3 refl = (-light_source_direction) - 2 * glm::dot(-light_source_direction, normal_at_intersection) * normal_at_intersection;
            total_radiance_specular += std::pow(std::max(0.0f, -glm::dot(refl, ray.m_direction)), record.hitted_entity_material->refractive_index) *
                                       light_source->m_radiance;
        }
        ray_color = total_radiance_diffuse * record.hitted_entity->GetDiffuseColor() * record.hitted_entity_material->phong_diffuse +
                    total_radiance_specular * record.hitted_entity_material->phong_specular;
    }
    return ray_color;
}

uint32_t vecRGBA_to_0xABGR(const glm::vec4& c)
{   // RTUtility::vecRGBA_to_0xABGR, BV/Renderer.cpp:13-23
    uint8_t r = (uint8_t)(c.r * 255.0f);
    uint8_t g = (uint8_t)(c.g * 255.0f);
    uint8_t b = (uint8_t)(c.b * 255.0f);
    uint8_t a = (uint8_t)(c.a * 255.0f);
    return ((a << 24) | (b << 16) | (g << 8) | r);
}

int cmd_scene(const char* bunny, const char* teapot, const char* out_nodes, const char* out_tris)
{
    Scene* s = build_scene(bunny, teapot);
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
    printf("nodes %zu tris %zu\n", nodes.size(), tris.size());
    return 0;
}

int cmd_rays(const char* bunny, const char* teapot, const char* in_rays, const char* out)
{
    Scene* s = build_scene(bunny, teapot);
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
        int32_t mat = hit ? 0 : -1;
        o.put(hit); o.put(ti); o.put(mat); o.put(rec.t); o.putv(rec.location); o.putv(rec.surface_normal);
    }
    printf("rays %zu\n", n);
    return 0;
}

// Camera{35, 0.1, 100} (BV/mainloop.cpp:22) + ResizeViewport: matrices and the corner-of-pixel
// directions of BV/Camera.cpp:114-132
int cmd_camera(uint32_t W, uint32_t H, const char* out)
{
    Camera cam{35.0f, 0.1f, 100.0f};
    cam.ResizeViewport(W, H);
    Out o(out);
    auto putm = [&](const glm::mat4& m) { for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) o.put(m[c][r]); };
    putm(cam.ProjectionMatrix()); putm(cam.InverseProjectionMatrix()); putm(cam.ViewMatrix()); putm(cam.InverseViewMatrix());
    o.putv(cam.Position()); o.putv(cam.ForwardDirection());
    for (auto& d : cam.RayDirections()) o.putv(d);
    printf("camera %ux%u\n", W, H);
    return 0;
}

// Renderer::Render x spp frames (BV/Renderer.cpp:69-107) with RayGen_Shader (:109-119).  The scene
// and camera are deterministic, so every frame's color is the same; it is computed once per pixel
// and added `spp` times, the reference's accumulation sequence.
int cmd_image(const char* bunny, const char* teapot, uint32_t W, uint32_t H, uint32_t spp, int threads, const char* out_accum,
              const char* out_rgba, const char* out_stats)
{
    Scene* s = build_scene(bunny, teapot);
    Camera cam{35.0f, 0.1f, 100.0f};
    cam.ResizeViewport(W, H);
    const auto& dirs = cam.RayDirections();
    std::vector<float> accum((size_t)W * H * 4, 0.0f);
    std::vector<uint32_t> rgba((size_t)W * H, 0);
    std::atomic<uint32_t> next_row{0};
    auto worker = [&]() {
        uint64_t rays = 0;
        for (;;) {
            uint32_t y = next_row.fetch_add(1);
            if (y >= H) break;
            for (uint32_t x = 0; x < W; ++x) {
                const size_t px = (size_t)y * W + x;
                glm::vec4 color_rgba{cast_whitted_ray(s, AccelerationStructure::Ray{cam.Position(), Whitted::normalize(dirs[px])}, rays), 1.0f};
                glm::vec4 acc{0.0f};
                for (uint32_t f = 1; f <= spp; ++f) {
                    acc += color_rgba;
                    glm::vec4 fin = acc / (float)f;
                    fin = glm::clamp(fin, glm::vec4(0.0f), glm::vec4(1.0f));
                    rgba[px] = vecRGBA_to_0xABGR(fin);
                }
                std::memcpy(&accum[4 * px], &acc, 16);
            }
        }
        g_rays += rays;
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
    { Out o(out_accum); fwrite(accum.data(), 4, accum.size(), o.f); }
    { Out o(out_rgba); fwrite(rgba.data(), 4, rgba.size(), o.f); }
    { Out o(out_stats); o.put((uint64_t)g_rays); o.put((uint64_t)W * H); }
    printf("whitted %ux%u spp %u rays/pixel-frame %.4f\n", W, H, spp, (double)g_rays / ((double)W * H));
    return 0;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 2) { fprintf(stderr, "usage: ref_whitted_bvh <cmd> ...\n"); return 1; }
    std::string c = argv[1];
    if (c == "scene" && argc == 6) return cmd_scene(argv[2], argv[3], argv[4], argv[5]);
    if (c == "rays" && argc == 6) return cmd_rays(argv[2], argv[3], argv[4], argv[5]);
    if (c == "camera" && argc == 5) return cmd_camera(atoi(argv[2]), atoi(argv[3]), argv[4]);
    if (c == "image" && argc == 11)
        return cmd_image(argv[2], argv[3], atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), argv[8], argv[9], argv[10]);
    fprintf(stderr, "bad command\n");
    return 1;
}
