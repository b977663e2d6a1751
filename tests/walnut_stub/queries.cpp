// tests/walnut_stub/queries.cpp -- TEST PROGRAM for the drop-in Renderer's scene queries and helpers
// (tests/test_walnut_queries.py): ray_BVH_intersection_record, SamplingAreaLight, mirror_reflection_direction,
// snell_refraction_direction and accurate_fresnel_reflectance (MC/Renderer.h:88-180), called with the
// reference's signatures on the default (Cornell box) Renderer of include/rt/walnut/Renderer.h.
//     queries RAYS_IN RAYS_OUT LIGHT_IN LIGHT_OUT OPTICS_IN OPTICS_OUT RNG_OUT
// RAYS_IN: 6 floats per ray (origin, direction) -> 40 bytes per ray (i32 hit, i32 material 0..3 / -1, f64 t,
// location, normal).  LIGHT_IN: 3 u32 draws per case -> 10 floats (location, normal, emission, PDF).
// OPTICS_IN: 7 floats (incident, normal, eta) -> 7 floats (mirror, snell, fresnel).  RNG_OUT: SamplingAreaLight
// with this thread's engine seeded 12345, and with the engine's first three words given explicitly (20 floats).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "Camera.h"     // -> include/rt/walnut/Camera.h (tests/walnut_stub/dropin)
#include "Renderer.h"   // -> include/rt/walnut/Renderer.h

template <class T> static std::vector<T> read_all(const char* p)
{
    std::ifstream f(p, std::ios::binary);
    std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<T> v(b.size() / sizeof(T));
    std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
    return v;
}

int main(int argc, char** argv)
{
    if (argc < 8) { std::fprintf(stderr, "usage: %s RAYS_IN RAYS_OUT LIGHT_IN LIGHT_OUT OPTICS_IN OPTICS_OUT RNG_OUT\n", argv[0]); return 2; }
    Renderer renderer;
    {   // closest hits
        const auto r = read_all<float>(argv[1]);
        std::ofstream o(argv[2], std::ios::binary);
        for (size_t i = 0; i + 5 < r.size(); i += 6) {
            AccelerationStructure::Ray ray{glm::vec3{r[i], r[i + 1], r[i + 2]}, glm::vec3{r[i + 3], r[i + 4], r[i + 5]}};
            const Whitted::IntersectionRecord rec = renderer.ray_BVH_intersection_record(ray);
            int32_t hit = rec.has_intersection ? 1 : 0, mat = -1;
            if (rec.hitted_entity_material) {
                // albedo -> the reference's material index (red, green, white, light by emission)
                const glm::vec3 a = rec.hitted_entity_material->diffuse_coefficient;
                if (rec.hitted_entity_material->IsEmitting()) mat = 3;
                else if (a.x == 0.63f) mat = 0;
                else if (a.x == 0.1f) mat = 1;
                else mat = 2;
            }
            const float f[6] = {rec.location.x, rec.location.y, rec.location.z, rec.surface_normal.x, rec.surface_normal.y, rec.surface_normal.z};
            o.write((const char*)&hit, 4); o.write((const char*)&mat, 4); o.write((const char*)&rec.t, 8); o.write((const char*)f, 24);
        }
    }
    {   // light samples on given draws
        const auto u = read_all<uint32_t>(argv[3]);
        std::ofstream o(argv[4], std::ios::binary);
        for (size_t i = 0; i + 2 < u.size(); i += 3) {
            Whitted::IntersectionRecord s;
            float pdf = -1.0f;
            renderer.SamplingAreaLight(s, pdf, &u[i]);
            const float f[10] = {s.location.x, s.location.y, s.location.z, s.surface_normal.x, s.surface_normal.y, s.surface_normal.z,
                                 s.emission.x, s.emission.y, s.emission.z, pdf};
            o.write((const char*)f, sizeof f);
        }
    }
    {   // optics
        const auto v = read_all<float>(argv[5]);
        std::ofstream o(argv[6], std::ios::binary);
        for (size_t i = 0; i + 6 < v.size(); i += 7) {
            const glm::vec3 I{v[i], v[i + 1], v[i + 2]}, N{v[i + 3], v[i + 4], v[i + 5]};
            const float eta = v[i + 6];
            const glm::vec3 m = renderer.mirror_reflection_direction(I, N), t = renderer.snell_refraction_direction(I, N, eta);
            const float f[7] = {m.x, m.y, m.z, t.x, t.y, t.z, renderer.accurate_fresnel_reflectance(I, N, eta)};
            o.write((const char*)f, sizeof f);
        }
    }
    {   // the reference signature draws from this thread's Walnut::Random engine
        std::ofstream o(argv[7], std::ios::binary);
        Whitted::random_engine().seed(12345u);
        Whitted::IntersectionRecord a, b;
        float pa = -1.0f, pb = -1.0f;
        renderer.SamplingAreaLight(a, pa);
        std::mt19937 e(12345u);
        const uint32_t w[3] = {(uint32_t)e(), (uint32_t)e(), (uint32_t)e()};
        renderer.SamplingAreaLight(b, pb, w);
        for (const auto* s : {&a, &b}) {
            const float f[9] = {s->location.x, s->location.y, s->location.z, s->surface_normal.x, s->surface_normal.y, s->surface_normal.z,
                                s->emission.x, s->emission.y, s->emission.z};
            o.write((const char*)f, sizeof f);
        }
        o.write((const char*)&pa, 4); o.write((const char*)&pb, 4);
    }
    std::printf("queries done\n");
    return 0;
}
