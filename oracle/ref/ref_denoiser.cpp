// oracle/ref/ref_denoiser.cpp -- TEST INFRASTRUCTURE ONLY (container-side golden-vector generator)
// for the reference's "Denoiser" project: a 1-spp Monte Carlo path tracer of the Cornell box that
// records a G-buffer per frame, followed by the joint bilateral filter and the temporal filter of
// DN/Denoiser.h.  DN/ = "Denoiser/8599RayTracerGUI/src/".
//
// Compiled by oracle/Makefile (target `ref`) with the reference's own, unmodified sources where they
// lie under /root/reference: DN/Denoiser.h (the filters themselves: Denoising::Denoiser,
// G_Buffer, FrameBuffer -- compiled as they are), DN/Camera.cpp, the header-only geometry core
// DN/{TriangleMesh,BVH,BoundingVolume,WhittedMaterial,Ray,IntersectionRecord,Entity,VectorFloat,
// WhittedUtilities,OBJ_Loader}.h (with DN's per-triangle primitive ids), and the vendored glm.
//
// Not compiled: DN/Renderer.{h,cpp} (Renderer.h includes Walnut/Image.h -> <vulkan/vulkan.h>).  The glue
// of Renderer::Renderer, Render, RayGen_Shader, cast_path, shading and SamplingAreaLight
// (DN/Renderer.cpp:26-58,101-379, DN/Renderer.h:185-202) is RESTATED below on top of the compiled code.
// The random stream is injected into the reference's Walnut::Random exactly as in ref_harness.cpp
// (oracle/ref/mt_inject.h): key (seed, pixel, frame, dim), dims from 0 (the DN camera does not jitter).
#include <iostream>
#include <fstream>
#include <sstream>
#include <filesystem>
#include <execution>
#include <random>
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>
#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#define private public
#include "TriangleMesh.h"
#include "Camera.h"
#include "Denoiser.h"
#undef private
#include "../philox.h"

#include "mt_inject.h"

namespace {

struct Out {
    FILE* f;
    explicit Out(const char* p) { f = fopen(p, "wb"); if (!f) { fprintf(stderr, "cannot write %s\n", p); exit(2); } }
    ~Out() { fclose(f); }
    template <class T> void put(const T& v) { fwrite(&v, sizeof(T), 1, f); }
    template <class T> void putn(const T* v, size_t n) { fwrite(v, sizeof(T), n, f); }
};

// Renderer::Renderer(), DN/Renderer.cpp:26-58 (primitive ids from 1 in mesh creation order)
struct Scene {
    std::vector<Whitted::Entity*> entities;
    AccelerationStructure::BVH* bvh = nullptr;
};

Scene* build_scene(const std::string& dir)
{
    Scene* s = new Scene;
    auto* red = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
    red->diffuse_coefficient = glm::vec3{0.63f, 0.065f, 0.05f};
    auto* green = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
    green->diffuse_coefficient = glm::vec3{0.1f, 0.5f, 0.1f};
    auto* white = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
    white->diffuse_coefficient = glm::vec3{0.7f, 0.7f, 0.7f};
    auto* light = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3(47.8f, 38.6f, 31.1f));
    light->diffuse_coefficient = glm::vec3{0.7f, 0.7f, 0.7f};
    int id_count = 1;
    const char* names[6] = {"floor.obj", "shortbox.obj", "tallbox.obj", "left.obj", "right.obj", "light.obj"};
    Whitted::WhittedMaterial* mats[6] = {white, white, white, red, green, light};
    for (int i = 0; i < 6; ++i) s->entities.push_back(new Whitted::TriangleMesh(id_count, dir + "/" + names[i], mats[i]));
    s->bvh = new AccelerationStructure::BVH{s->entities};
    return s;
}

// ---- RESTATED glue (DN/Renderer.cpp:285-379, DN/Renderer.h:185-202)
struct Glue {
    const Scene* s;
    float rr = 0.8f;   // RR_survival_probability, DN/Renderer.h:226
    Whitted::IntersectionRecord trace(const AccelerationStructure::Ray& r) const { return s->bvh->traverse_BVH_from_root(r); }
    void sampling_area_light(Whitted::IntersectionRecord& sample, float& pdf) const
    {
        for (uint32_t n = 0; n < s->entities.size(); n++)
            if (s->entities[n]->IsEmissive()) { s->entities[n]->Sampling(sample, pdf); break; }
    }
    glm::vec3 shading(const Whitted::IntersectionRecord& record, const glm::vec3& W_out) const
    {
        if (record.hitted_entity_material->IsEmitting()) return record.hitted_entity_material->GetEmission();
        glm::vec3 n = record.surface_normal;
        if (glm::dot(record.surface_normal, W_out) < 0.0f) n = -(record.surface_normal);
        glm::vec3 p = record.location + n * INTERSECTION_CORRECTION;
        glm::vec3 direct{0.0f, 0.0f, 0.0f};
        Whitted::IntersectionRecord ls;
        float ls_pdf;
        sampling_area_light(ls, ls_pdf);
        glm::vec3 p2q = ls.location - p;
        glm::vec3 wl = glm::normalize(p2q);
        glm::vec3 nl = ls.surface_normal;
        if (glm::dot(ls.surface_normal, -wl) < 0.0f) nl = -(ls.surface_normal);
        Whitted::IntersectionRecord occ = trace(AccelerationStructure::Ray{p, wl});
        if (glm::length(p2q) < occ.t + 0.01f)
            direct = ls.emission * record.hitted_entity_material->BRDF(W_out, wl, n) * glm::dot(wl, n) * glm::dot(-wl, nl) / (glm::dot(p2q, p2q)) / (ls_pdf);
        glm::vec3 indirect{0.0f, 0.0f, 0.0f};
        if (Whitted::get_random_float_0_1() < rr) {
            glm::vec3 W_in = glm::normalize(record.hitted_entity_material->Sampling(W_out, n));
            float PDF = record.hitted_entity_material->PDF_at_the_sample(W_out, W_in, n);
            Whitted::IntersectionRecord deeper = trace(AccelerationStructure::Ray{p, W_in});
            if (deeper.has_intersection && (!(deeper.hitted_entity_material->IsEmitting())))
                indirect = shading(deeper, -W_in) * record.hitted_entity_material->BRDF(W_out, W_in, n) * glm::dot(W_in, n) / PDF / rr;
        }
        return direct + indirect;
    }
    // Renderer::cast_path with the G-buffer writes, DN/Renderer.cpp:285-311
    glm::vec3 cast_path(const AccelerationStructure::Ray& ray, Denoising::G_Buffer& g, int column, int row) const
    {
        Whitted::IntersectionRecord record = trace(ray);
        if (record.has_intersection) {
            g.primitive_id(column, row) = record.primitive_id;
            g.contributor(column, row) = 1;
            g.pixel_world_position(column, row) = record.location;
            glm::vec3 n = record.surface_normal;
            if (glm::dot(record.surface_normal, -(ray.m_direction)) < 0.0f) n = -(record.surface_normal);
            g.pixel_world_surface_normal(column, row) = glm::normalize(n);
            return shading(record, -(ray.m_direction));
        }
        g.primitive_id(column, row) = -1;
        g.contributor(column, row) = 0;
        return glm::vec3{12 / 255.0f, 20 / 255.0f, 69 / 255.0f};
    }
};

// Camera keeps `position` as its first (implicitly private) member and has no setter; the class is
// standard-layout, so the object's address is the member's (the harness moves the camera between
// frames the way UpdateCamera's WASD keys would, DN/Camera.cpp:40-85)
static_assert(std::is_standard_layout_v<Camera>, "Camera layout");
glm::vec3& camera_position(Camera& c) { return *reinterpret_cast<glm::vec3*>(&c); }

uint32_t vecRGBA_to_0xABGR(const glm::vec4& c)
{   // RTUtility::vecRGBA_to_0xABGR, DN/Renderer.cpp:13-23
    uint8_t r = (uint8_t)(c.r * 255.0f);
    uint8_t g = (uint8_t)(c.g * 255.0f);
    uint8_t b = (uint8_t)(c.b * 255.0f);
    uint8_t a = (uint8_t)(c.a * 255.0f);
    return ((a << 24) | (b << 16) | (g << 8) | r);
}

// frames 1..n of the denoised renderer: per frame the camera position is `pos0 + k * step` (the
// forward direction is the default), Renderer::Render = G-buffer pass + JointBilateralFiltering +
// TemporalFiltering + clamp/pack (DN/Renderer.cpp:101-283).  Writes, per frame: the G-buffer
// (color after the immediate clamp, position, normal, contributor, primitive id), the camera
// matrices, the spatial and temporal outputs and the RGBA8 frame.
int cmd_frames(const char* dir, uint32_t W, uint32_t H, uint32_t n, uint64_t seed, float step_x, int jbf_half, int temporal_half,
               float tolerance, float weighting, int immediate_clamp, int threads, const char* out_path)
{
    Scene* s = build_scene(dir);
    Glue glue{s};
    Camera cam{35.0f, 0.1f, 100.0f};
    const glm::vec3 pos0 = cam.Position();
    cam.ResizeViewport(W, H);
    Denoising::G_Buffer g((int)W, (int)H);
    Denoising::FrameBuffer<glm::vec3> spatial((int)W, (int)H), temporal((int)W, (int)H);
    Denoising::Denoiser dn;
    dn.Resize(W, H);
    dn.using_JBF_filtering = jbf_half > 0;
    if (jbf_half > 0) dn.JBF_FilterKernelHalfSize = jbf_half;
    dn.using_temporal_filtering = temporal_half > 0;
    if (temporal_half > 0) dn.Temporal_FilterKernelHalfSize = temporal_half;
    dn.tolerance = tolerance;
    dn.current_frame_weighting = weighting;
    Out o(out_path);
    std::vector<uint32_t> rgba((size_t)W * H);
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t frame = k + 1;
        camera_position(cam) = pos0 + glm::vec3{step_x * (float)k, 0.0f, 0.0f};
        cam.RecomputeViewMatrix();
        cam.RecomputeRayDirections();
        const auto& dirs = cam.RayDirections();
        std::atomic<uint32_t> next{0};
        auto worker = [&]() {
            set_msvc_distribution();
            for (;;) {
                const uint32_t y = next.fetch_add(1);
                if (y >= H) break;
                for (uint32_t x = 0; x < W; ++x) {
                    const uint32_t px = y * W + x;
                    g_inj.start(seed, px, frame, 624);
                    // RayGen_Shader, DN/Renderer.cpp:264-275
                    glm::vec3 c = glue.cast_path(AccelerationStructure::Ray{cam.Position(), Whitted::normalize(dirs[px])}, g, (int)x, (int)y);
                    if (immediate_clamp) c = glm::clamp(c, glm::vec3(0.0f), glm::vec3(1.0f));
                    g.pixel_color((int)x, (int)y) = c;
                }
            }
        };
        std::vector<std::thread> ts;
        for (int i = 0; i < threads; ++i) ts.emplace_back(worker);
        for (auto& t : ts) t.join();
        // G-buffer as rendered (before the filters overwrite pixel_color)
        o.putn(&g.pixel_color.buffer[0].x, 3 * (size_t)W * H);
        o.putn(&g.pixel_world_position.buffer[0].x, 3 * (size_t)W * H);
        o.putn(&g.pixel_world_surface_normal.buffer[0].x, 3 * (size_t)W * H);
        o.putn(g.contributor.buffer.data(), (size_t)W * H);
        o.putn(g.primitive_id.buffer.data(), (size_t)W * H);
        // Renderer::Render, DN/Renderer.cpp:243-262
        dn.JointBilateralFiltering(g, spatial, immediate_clamp != 0);
        g.projection_matrix = cam.ProjectionMatrix();
        g.view_matrix = cam.ViewMatrix();
        dn.TemporalFiltering(g, temporal);
        for (uint32_t i = 0; i < W * H; ++i) {
            glm::vec4 c{temporal.buffer[i], 1.0f};
            rgba[i] = vecRGBA_to_0xABGR(glm::clamp(c, glm::vec4(0.0f), glm::vec4(1.0f)));
        }
        o.putn(&g.projection_matrix[0][0], 16);
        o.putn(&g.view_matrix[0][0], 16);
        o.putn(&cam.Position().x, 3);
        o.putn(&spatial.buffer[0].x, 3 * (size_t)W * H);
        o.putn(&temporal.buffer[0].x, 3 * (size_t)W * H);
        o.putn(rgba.data(), (size_t)W * H);
    }
    printf("denoiser %ux%u frames %u jbf %d temporal %d\n", W, H, n, jbf_half, temporal_half);
    return 0;
}

}  // namespace

int main(int argc, char** argv)
{
    check_layout_once();
    set_msvc_distribution();
    if (argc == 15 && std::string(argv[1]) == "frames")
        return cmd_frames(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), strtoull(argv[6], 0, 10), (float)atof(argv[7]), atoi(argv[8]),
                          atoi(argv[9]), (float)atof(argv[10]), (float)atof(argv[11]), atoi(argv[12]), atoi(argv[13]), argv[14]);
    fprintf(stderr, "usage: ref_denoiser frames DIR W H N SEED STEP_X JBF_HALF TEMPORAL_HALF TOL WEIGHT CLAMP THREADS OUT\n");
    return 1;
}
