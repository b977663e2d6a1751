// tests/walnut_stub/spheres.cpp -- TEST PROGRAM for the reference's Entity extension point through the drop-in
// (tests/test_walnut_spheres.py): Whitted::Sphere entities added the reference's way -- `renderer.Add(new
// Whitted::Sphere(center, radius, material))`, GenerateBVH (MC/Sphere.h:16-108, MC/Renderer.h:78-86) -- against
// include/rt/walnut/*.h, with the public `entities` / `bvh` members (MC/Renderer.h:200-201).
//
//   spheres entities SPHERES_IN RAYS_IN OUT      (no GPU) the Whitted::Entity interface of Whitted::Sphere and of
//       Whitted::TriangleMesh on their own: per sphere GetArea, Get3DAABB, IsEmissive, GetHitInfo, and each ray's
//       Sphere::GetIntersectionRecord against every sphere (the host restatement of MC/Sphere.h:62-97)
//   spheres render SPHERES_IN RAYS_IN OUT W H SPP   the Cornell Renderer + the spheres; renderer.bvh->
//       traverse_BVH_from_root for every ray, then SPP frames of W x H through Render (accumulation written)
// SPHERES_IN: 5 floats per sphere (center, radius, material index 0..3 of red / green / white / light).
// RAYS_IN: 6 floats per ray.  Records written: see tests/test_walnut_spheres.py.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
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

static Whitted::WhittedMaterial* material(int k)
{   // MC/Renderer.cpp:28-35: red, green, white, light
    static Whitted::WhittedMaterial* m[4] = {nullptr, nullptr, nullptr, nullptr};
    if (!m[0]) {
        const glm::vec3 albedo[4] = {{0.63f, 0.065f, 0.05f}, {0.1f, 0.5f, 0.1f}, {0.7f, 0.7f, 0.7f}, {0.7f, 0.7f, 0.7f}};
        for (int i = 0; i < 4; ++i) {
            m[i] = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, i == 3 ? glm::vec3{47.8f, 38.6f, 31.1f} : glm::vec3{0.0f, 0.0f, 0.0f});
            m[i]->diffuse_coefficient = albedo[i];
        }
    }
    return m[k];
}

static void put_record(std::ofstream& o, const Whitted::IntersectionRecord& rec, int32_t entity)
{
    const int32_t hit = rec.has_intersection ? 1 : 0;
    const float f[6] = {rec.location.x, rec.location.y, rec.location.z, rec.surface_normal.x, rec.surface_normal.y, rec.surface_normal.z};
    o.write((const char*)&hit, 4); o.write((const char*)&entity, 4); o.write((const char*)&rec.t, 8); o.write((const char*)f, 24);
}

int main(int argc, char** argv)
{
    if (argc < 5) { std::fprintf(stderr, "usage: %s entities|render SPHERES_IN RAYS_IN OUT [W H SPP]\n", argv[0]); return 2; }
    const std::string mode = argv[1];
    const auto sp = read_all<float>(argv[2]);
    const auto rays = read_all<float>(argv[3]);
    std::vector<Whitted::Sphere*> spheres;
    for (size_t i = 0; i + 4 < sp.size(); i += 5)
        spheres.push_back(new Whitted::Sphere(glm::vec3{sp[i], sp[i + 1], sp[i + 2]}, sp[i + 3], material((int)sp[i + 4])));
    std::ofstream o(argv[4], std::ios::binary);

    if (mode == "entities") {
        for (Whitted::Sphere* s : spheres) {
            Whitted::Entity* e = s;   // through the reference's virtual interface
            const AccelerationStructure::AABB_3D b = e->Get3DAABB();
            glm::vec3 n{0.0f, 0.0f, 0.0f};
            glm::vec2 uv{0.0f, 0.0f};
            e->GetHitInfo(b.max_slab_values, glm::vec3{0.0f, 0.0f, 0.0f}, 0, glm::vec2{0.0f, 0.0f}, n, uv);
            const float f[11] = {e->GetArea(), b.min_slab_values.x, b.min_slab_values.y, b.min_slab_values.z, b.max_slab_values.x,
                                 b.max_slab_values.y, b.max_slab_values.z, e->IsEmissive() ? 1.0f : 0.0f, n.x, n.y, n.z};
            o.write((const char*)f, sizeof f);
        }
        for (size_t i = 0; i + 5 < rays.size(); i += 6) {
            AccelerationStructure::Ray ray{glm::vec3{rays[i], rays[i + 1], rays[i + 2]}, glm::vec3{rays[i + 3], rays[i + 4], rays[i + 5]}};
            for (size_t k = 0; k < spheres.size(); ++k) put_record(o, spheres[k]->GetIntersectionRecord(ray), (int32_t)k);
        }
        std::printf("entities %zu rays %zu\n", spheres.size(), rays.size() / 6);
        return 0;
    }
    if (mode != "render" || argc < 8) return 2;
    const uint32_t W = (uint32_t)std::stoul(argv[5]), H = (uint32_t)std::stoul(argv[6]), spp = (uint32_t)std::stoul(argv[7]);
    Renderer renderer;
    for (Whitted::Sphere* s : spheres) renderer.Add(s);
    renderer.GenerateBVH();
    // the public members, as a reference caller reads them
    std::printf("entities %zu\n", renderer.entities.size());
    for (size_t i = 0; i + 5 < rays.size(); i += 6) {
        AccelerationStructure::Ray ray{glm::vec3{rays[i], rays[i + 1], rays[i + 2]}, glm::vec3{rays[i + 3], rays[i + 4], rays[i + 5]}};
        const Whitted::IntersectionRecord rec = renderer.bvh->traverse_BVH_from_root(ray);
        int32_t entity = -1;
        for (size_t k = 0; k < renderer.entities.size(); ++k)
            if (rec.hitted_entity == renderer.entities[k]) entity = (int32_t)k;
        put_record(o, rec, entity);
    }
    Camera camera(35.0f, 0.1f, 100.0f);   // MC/mainloop.cpp:22
    camera.ResizeViewport(W, H);
    renderer.ResizeViewport(W, H);
    for (uint32_t k = 0; k < spp; ++k) renderer.Render(camera);
    const std::vector<float>& acc = renderer.Core().GetAccumulation();
    std::ofstream a(std::string(argv[4]) + ".accum", std::ios::binary);
    a.write((const char*)acc.data(), (std::streamsize)acc.size() * 4);
    std::printf("%u spp\n", renderer.GetSPP());
    return 0;
}
