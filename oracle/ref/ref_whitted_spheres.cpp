// oracle/ref/ref_whitted_spheres.cpp -- TEST INFRASTRUCTURE ONLY (container-side golden-vector generator)
// for the reference's "Whitted Style Ray Tracer" (config C1: two spheres -- diffuse and glass -- over a
// two-triangle chessboard, two point lights, reflection/refraction recursion to depth 5; SURVEY.md
// section 3.3).  WH/ = "Whitted Style Ray Tracer/8599RayTracerGUI/src/".
//
// Compiled by oracle/Makefile (target `ref`) with the reference's own, unmodified sources where they
// lie under /root/reference: WH/Camera.cpp, the header-only entity core WH/{Sphere,TriangleMesh,Entity,
// World,LightSource,VectorFloat,WhittedUtilities}.h (Sphere::Intersect + QuadraticFormula,
// RayTriangleIntersection, TriangleMesh::Intersect/GetHitInfo/GetDiffuseColor), and the vendored glm.
// Output goes only to oracle/_ref/.
//
// Not compiled: WH/Renderer.{h,cpp}.  Renderer.h includes Walnut/Image.h -> <vulkan/vulkan.h>, absent
// from the image, and it holds the whole shading recursion.  The glue of Renderer::Renderer /
// RayGen_Shader (WH/Renderer.cpp:27-49,116-125) and the Renderer.h helpers mirror_reflection_direction,
// snell_refraction_direction, accurate_fresnel_reflectance, get_intersection_payload and
// cast_Whitted_ray (WH/Renderer.h:41-140,184-310) are therefore RESTATED below, on top of the
// reference's compiled entities and camera.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <optional>
#include <string>
#include <thread>
#include <vector>
#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#define private public
#include "Sphere.h"
#include "TriangleMesh.h"
#include "World.h"
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

// Renderer::Renderer(), WH/Renderer.cpp:27-49 (the reference's own entity classes)
void build_world(Whitted::World& world)
{
    auto diffuse_sphere = std::make_unique<Whitted::Sphere>(glm::vec3(-1, 0, -12), 2.0f);
    diffuse_sphere->material_nature = Whitted::Diffuse_Glossy;
    diffuse_sphere->diffuse_color = glm::vec3(0.6, 0.7, 0.8);
    world.Add(std::move(diffuse_sphere));
    auto glass_sphere = std::make_unique<Whitted::Sphere>(glm::vec3(0.5, -0.5, -8), 1.5f);
    glass_sphere->material_nature = Whitted::Reflective_Refractive;
    glass_sphere->refractive_index = 1.5;
    world.Add(std::move(glass_sphere));
    glm::vec3 vertices[4] = {{-5, -3, -6}, {5, -3, -6}, {5, -3, -16}, {-5, -3, -16}};
    uint32_t indices[6] = {0, 1, 3, 1, 2, 3};
    glm::vec2 uv[4] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
    auto chessboard = std::make_unique<Whitted::TriangleMesh>(vertices, indices, 2, uv);
    chessboard->material_nature = Whitted::Diffuse_Glossy;
    world.Add(std::move(chessboard));
    world.Add(std::make_unique<Whitted::PointLightSource>(glm::vec3(-20.0f, 70.0f, 20.0f), glm::vec3(0.5f)));
    world.Add(std::make_unique<Whitted::PointLightSource>(glm::vec3(30.0f, 50.0f, -12.0f), glm::vec3(0.5f)));
}

// ---- RESTATED from WH/Renderer.h (unbuildable here, see header)
struct Payload { const Whitted::Entity* entity; int index; uint32_t triangle_index; glm::vec2 bary; float t; };

glm::vec3 mirror_reflection_direction(const glm::vec3& I, const glm::vec3& N)
{   // WH/Renderer.h:41-45
    return I - 2 * glm::dot(I, N) * N;
}

glm::vec3 snell_refraction_direction(const glm::vec3& I, const glm::vec3& N, const float& eta)
{   // WH/Renderer.h:47-76
    float eta_in = 1.0, eta_out = eta;
    glm::vec3 normal = N;
    float cos_incident = Whitted::clamp_float(glm::dot(I, N), -1, 1);
    if (cos_incident < 0) cos_incident = -cos_incident;
    else { std::swap(eta_in, eta_out); normal = -normal; }
    float eta_ratio = eta_in / eta_out;
    float k = 1 - eta_ratio * eta_ratio * (1 - cos_incident * cos_incident);
    return (k < 0) ? (glm::vec3{0.0f, 0.0f, 0.0f}) : (eta_ratio * I + (eta_ratio * cos_incident - std::sqrt(k)) * normal);
}

float accurate_fresnel_reflectance(const glm::vec3& I, const glm::vec3& N, const float& eta)
{   // WH/Renderer.h:78-107
    float eta_in = 1.0, eta_out = eta;
    float cos_incident = Whitted::clamp_float(glm::dot(I, N), -1, 1);
    if (cos_incident < 0) cos_incident = -cos_incident;
    else std::swap(eta_in, eta_out);
    float sin_refract = eta_in / eta_out * std::sqrt(std::max(0.0f, 1 - cos_incident * cos_incident));
    if (sin_refract > 1.0f) return 1.0f;
    float cos_refract = std::sqrt(std::max(0.0f, 1 - sin_refract * sin_refract));
    float rs = (eta_in * cos_incident - eta_out * cos_refract) / (eta_in * cos_incident + eta_out * cos_refract);
    float rp = (eta_in * cos_refract - eta_out * cos_incident) / (eta_in * cos_refract + eta_out * cos_incident);
    return (rs * rs + rp * rp) / 2;
}

std::optional<Payload> get_intersection_payload(const glm::vec3& o, const glm::vec3& d, const Whitted::World& world)
{   // WH/Renderer.h:109-140: closest over the entities in insertion order, strict '<'
    std::optional<Payload> payload{};
    float t_closest = Whitted::positive_infinity;
    int k = 0;
    for (const auto& entity : world.GetEntities()) {
        float t_local = Whitted::positive_infinity;
        uint32_t tri;
        glm::vec2 bary;
        if (entity->Intersect(o, d, t_local, tri, bary) && t_local < t_closest) {
            payload.emplace();
            t_closest = t_local;
            *payload = Payload{entity.get(), k, tri, bary, t_closest};
        }
        ++k;
    }
    return payload;
}

struct Counters { uint64_t rays = 0; };

glm::vec3 cast_Whitted_ray(const glm::vec3& o, const glm::vec3& d, const Whitted::World& world, int bounced, Counters& c)
{   // Renderer::cast_Whitted_ray, WH/Renderer.h:184-310
    if ((bounced > world.max_bounce_depth) || (d == glm::vec3{0.0f, 0.0f, 0.0f})) return glm::vec3{0.0f, 0.0f, 0.0f};
    glm::vec3 ray_color = world.sky_color;
    c.rays++;
    if (std::optional<Payload> payload = get_intersection_payload(o, d, world)) {
        glm::vec3 intersection = o + d * payload->t;
        glm::vec3 n;
        glm::vec2 uv;
        payload->entity->GetHitInfo(intersection, d, payload->triangle_index, payload->bary, n, uv);
        const float eps = world.intersection_correction;
        switch (payload->entity->material_nature) {
        case Whitted::Reflective: {
            glm::vec3 rd = Whitted::normalize(mirror_reflection_direction(d, n));
            glm::vec3 ro = (glm::dot(rd, n) < 0.0f) ? (intersection - n * eps) : (intersection + n * eps);
            ray_color = cast_Whitted_ray(ro, rd, world, bounced + 1, c) * accurate_fresnel_reflectance(-rd, n, payload->entity->refractive_index);
            break;
        }
        case Whitted::Reflective_Refractive: {
            glm::vec3 rd = Whitted::normalize(mirror_reflection_direction(d, n));
            glm::vec3 ro = (glm::dot(rd, n) < 0.0f) ? (intersection - n * eps) : (intersection + n * eps);
            glm::vec3 td = Whitted::normalize(snell_refraction_direction(d, n, payload->entity->refractive_index));
            glm::vec3 to = (glm::dot(td, n) < 0.0f) ? (intersection - n * eps) : (intersection + n * eps);
            glm::vec3 rc = cast_Whitted_ray(ro, rd, world, bounced + 1, c);
            glm::vec3 tc = cast_Whitted_ray(to, td, world, bounced + 1, c);
            float R = accurate_fresnel_reflectance(d, n, payload->entity->refractive_index);
            ray_color = R * rc + (1.0f - R) * tc;
            break;
        }
        default: {
            glm::vec3 diffuse{0.0f, 0.0f, 0.0f}, specular{0.0f, 0.0f, 0.0f};
            glm::vec3 sp = (glm::dot(d, n) < 0.0f) ? (intersection + n * eps) : (intersection - n * eps);
            for (const auto& light : world.GetLightSources()) {
                glm::vec3 ld = light->m_position - intersection;
                float d2 = glm::dot(ld, ld);
                ld = Whitted::normalize(ld);
                c.rays++;
                std::optional<Payload> occ = get_intersection_payload(sp, ld, world);
                if (occ && (occ->t * occ->t < d2)) continue;
                diffuse += light->m_radiance * std::fabs(glm::dot(ld, n));
                specular += std::pow(std::max(0.0f, -glm::dot(mirror_reflection_direction(-ld, n), d)), payload->entity->specular_size_factor) *
                            light->m_radiance;
            }
            ray_color = diffuse * payload->entity->GetDiffuseColor(uv) * payload->entity->phong_diffuse + specular * payload->entity->phong_specular;
            break;
        }
        }
    }
    return ray_color;
}

uint32_t vecRGBA_to_0xABGR(const glm::vec4& c)
{   // RTUtility::vecRGBA_to_0xABGR, WH/Renderer.cpp:15-24
    uint8_t r = (uint8_t)(c.r * 255.0f);
    uint8_t g = (uint8_t)(c.g * 255.0f);
    uint8_t b = (uint8_t)(c.b * 255.0f);
    uint8_t a = (uint8_t)(c.a * 255.0f);
    return ((a << 24) | (b << 16) | (g << 8) | r);
}

// Camera{35, 0.1, 100} (WH/mainloop.cpp:23) + ResizeViewport: matrices, position and the
// corner-of-pixel directions (WH/Camera.cpp:97-132)
int cmd_camera(uint32_t W, uint32_t H, const char* out)
{
    Camera cam{35.0f, 0.1f, 100.0f};
    cam.ResizeViewport(W, H);
    Out o(out);
    auto putm = [&](const glm::mat4& m) { for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) o.put(m[c][r]); };
    putm(cam.ProjectionMatrix()); putm(cam.InverseProjectionMatrix()); putm(cam.ViewMatrix()); putm(cam.InverseViewMatrix());
    o.putv(cam.Position()); o.putv(cam.ForwardDirection());
    if ((uint64_t)W * H <= 4096) for (auto& d : cam.RayDirections()) o.putv(d);
    printf("camera %ux%u\n", W, H);
    return 0;
}

// closest hit of given rays: entity index, triangle index, barycentrics, t (get_intersection_payload)
int cmd_rays(const char* in_rays, const char* out)
{
    Whitted::World world;
    build_world(world);
    auto r = read_all<float>(in_rays);
    size_t n = r.size() / 6;
    Out o(out);
    for (size_t i = 0; i < n; ++i) {
        glm::vec3 org{r[6 * i], r[6 * i + 1], r[6 * i + 2]}, d{r[6 * i + 3], r[6 * i + 4], r[6 * i + 5]};
        auto p = get_intersection_payload(org, d, world);
        int32_t ent = p ? p->index : -1;
        int32_t tri = p && ent == 2 ? (int32_t)p->triangle_index : -1;
        float bx = p && ent == 2 ? p->bary.x : 0.0f, by = p && ent == 2 ? p->bary.y : 0.0f;
        float t = p ? p->t : 0.0f;
        o.put(ent); o.put(tri); o.put(t); o.put(bx); o.put(by);
    }
    printf("rays %zu\n", n);
    return 0;
}

// Renderer::Render x spp frames (WH/Renderer.cpp:82-114) with RayGen_Shader (:116-125).  Deterministic:
// each pixel's color is computed once and accumulated `spp` times, the reference's sequence.
int cmd_image(uint32_t W, uint32_t H, uint32_t spp, int threads, const char* out_accum, const char* out_rgba, const char* out_stats)
{
    Whitted::World world;
    build_world(world);
    Camera cam{35.0f, 0.1f, 100.0f};
    cam.ResizeViewport(W, H);
    const auto& dirs = cam.RayDirections();
    std::vector<float> accum((size_t)W * H * 4, 0.0f);
    std::vector<uint32_t> rgba((size_t)W * H, 0);
    std::atomic<uint32_t> next_row{0};
    std::atomic<uint64_t> rays{0};
    auto worker = [&]() {
        Counters c;
        for (;;) {
            uint32_t y = next_row.fetch_add(1);
            if (y >= H) break;
            for (uint32_t x = 0; x < W; ++x) {
                const size_t px = (size_t)y * W + x;
                glm::vec4 color{cast_Whitted_ray(cam.Position(), Whitted::normalize(dirs[px]), world, 0, c), 1.0f};
                glm::vec4 acc{0.0f};
                for (uint32_t f = 1; f <= spp; ++f) {
                    acc += color;
                    glm::vec4 fin = glm::clamp(acc / (float)f, glm::vec4(0.0f), glm::vec4(1.0f));
                    rgba[px] = vecRGBA_to_0xABGR(fin);
                }
                std::memcpy(&accum[4 * px], &acc, 16);
            }
        }
        rays += c.rays;
    };
    std::vector<std::thread> ts;
    for (int i = 0; i < threads; ++i) ts.emplace_back(worker);
    for (auto& t : ts) t.join();
    { Out o(out_accum); fwrite(accum.data(), 4, accum.size(), o.f); }
    { Out o(out_rgba); fwrite(rgba.data(), 4, rgba.size(), o.f); }
    { Out o(out_stats); o.put((uint64_t)rays); o.put((uint64_t)W * H); }
    printf("spheres %ux%u spp %u rays/pixel %.4f\n", W, H, spp, (double)rays / ((double)W * H));
    return 0;
}

// glibc powf on the cases the shading evaluates (specular lobe, exponent 25): the one libm call
// whose device restatement is not bit-exact by construction
int cmd_pow(const char* in, const char* out)
{
    auto v = read_all<float>(in);
    Out o(out);
    for (size_t i = 0; i + 1 < v.size(); i += 2) o.put((float)std::pow(v[i], v[i + 1]));
    printf("pow %zu\n", v.size() / 2);
    return 0;
}

// the Renderer's optics helpers (WH/Renderer.h:41-107; MC/Renderer.h:93-161 is the same code as const members) on
// (incident xyz, normal xyz, eta) cases -> mirror xyz, snell xyz, fresnel: the drop-in Renderer's fixtures
int cmd_optics(const char* in, const char* out)
{
    auto v = read_all<float>(in);
    Out o(out);
    for (size_t i = 0; i + 6 < v.size(); i += 7) {
        const glm::vec3 I{v[i], v[i + 1], v[i + 2]}, N{v[i + 3], v[i + 4], v[i + 5]};
        const float eta = v[i + 6];
        const glm::vec3 m = mirror_reflection_direction(I, N), t = snell_refraction_direction(I, N, eta);
        o.put(m.x); o.put(m.y); o.put(m.z); o.put(t.x); o.put(t.y); o.put(t.z); o.put(accurate_fresnel_reflectance(I, N, eta));
    }
    printf("optics %zu\n", v.size() / 7);
    return 0;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 2) { fprintf(stderr, "usage: ref_whitted_spheres <cmd> ...\n"); return 1; }
    std::string c = argv[1];
    if (c == "camera" && argc == 5) return cmd_camera(atoi(argv[2]), atoi(argv[3]), argv[4]);
    if (c == "rays" && argc == 4) return cmd_rays(argv[2], argv[3]);
    if (c == "pow" && argc == 4) return cmd_pow(argv[2], argv[3]);
    if (c == "optics" && argc == 4) return cmd_optics(argv[2], argv[3]);
    if (c == "image" && argc == 9) return cmd_image(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), argv[6], argv[7], argv[8]);
    fprintf(stderr, "bad command\n");
    return 1;
}
