// include/rt/walnut/Renderer.h -- the reference's Renderer for a Walnut front-end: MC/Renderer.h:30-202 with
// GetFinalImage() returning the std::shared_ptr<Walnut::Image> the layer displays (ImGui::Image of its
// descriptor set, MC/mainloop.cpp:55-58), filled with Image::SetData after every Render as
// MC/Renderer.cpp:112 does.  The frame is rendered by the core rt::Renderer (include/rt/Renderer.h: the
// MI355X kernels behind the C-ABI).  A layer written against the reference compiles unchanged but for its
// include lines:   #include "Renderer.h"  ->  #include <rt/walnut/Renderer.h>
#ifndef RT_WALNUT_RENDERER_H
#define RT_WALNUT_RENDERER_H
#ifndef RT_NO_GLOBAL_NAMES
#define RT_NO_GLOBAL_NAMES
#endif
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <memory>
#include <utility>
#include <vector>

#include "Walnut/Image.h"
#include "Camera.h"
#include "Ray.h"       // AccelerationStructure::Ray, as MC/Renderer.h brings it
#include "Whitted.h"   // Whitted::TriangleMesh / Sphere / WhittedMaterial / Entity / IntersectionRecord, as MC/Renderer.h brings them
#include "BVH.h"       // AccelerationStructure::BVH (the public `bvh` member)
#include "../Renderer.h"

// Average indices of refraction, MC/Renderer.h:22-28
#ifndef eta_Vacuum
#define eta_Vacuum 1.0
#define eta_Air 1.00029
#define eta_20C_Water 1.333
#define eta_Glass1 1.5
#define eta_Glass2 1.6
#define eta_Diamond 2.42
#endif

class Renderer {
public:
    using Settings = rt::Renderer::Settings;   // Settings::accumulating, MC/Renderer.h:34-37

    // the Cornell box (MC/Renderer.cpp:26-57): six Whitted::TriangleMesh entities over the core's built-in
    // Cornell positions and the reference's four materials, then GenerateBVH
    Renderer()
    {
        auto mk = [](glm::vec3 emission, glm::vec3 albedo) {
            auto m = std::make_unique<Whitted::WhittedMaterial>(Whitted::MaterialNature::Diffuse, emission);
            m->diffuse_coefficient = albedo;
            return m;
        };
        builtin_materials_.push_back(mk(glm::vec3{0.0f, 0.0f, 0.0f}, glm::vec3{0.63f, 0.065f, 0.05f}));   // red
        builtin_materials_.push_back(mk(glm::vec3{0.0f, 0.0f, 0.0f}, glm::vec3{0.1f, 0.5f, 0.1f}));       // green
        builtin_materials_.push_back(mk(glm::vec3{0.0f, 0.0f, 0.0f}, glm::vec3{0.7f, 0.7f, 0.7f}));       // white
        builtin_materials_.push_back(mk(glm::vec3{47.8f, 38.6f, 31.1f}, glm::vec3{0.7f, 0.7f, 0.7f}));    // light
        // floor, shortbox, tallbox: white; left: red; right: green; light (MC/Renderer.cpp:36-41)
        const int which[6] = {2, 2, 2, 0, 1, 3};
        const std::vector<rt::Entity*> cornell = core_.GetEntities();
        for (size_t k = 0; k < cornell.size() && k < 6; ++k) {
            builtin_meshes_.push_back(std::make_unique<Whitted::TriangleMesh>(cornell[k]->RawPositions(), builtin_materials_[which[k]].get()));
            Add(builtin_meshes_.back().get());
        }
        GenerateBVH();
    }
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    // MC/Renderer.cpp:59-89: the Walnut image is created once and resized with the viewport
    void ResizeViewport(uint32_t width, uint32_t height)
    {
        core_.ResizeViewport(width, height);
        if (frame_image_final) {
            if (frame_image_final->GetWidth() == width && frame_image_final->GetHeight() == height) return;
            frame_image_final->Resize(width, height);
        } else {
            frame_image_final = std::make_shared<Walnut::Image>(width, height, Walnut::ImageFormat::RGBA);
        }
    }
    // +1 spp (MC/Renderer.cpp:91-122), then Image::SetData of the RGBA8 frame (:112)
    void Render(const Camera& camera)
    {
        core_.RR_survival_probability = RR_survival_probability;
        core_.Render(camera.Core());
        if (frame_image_final) frame_image_final->SetData(core_.GetFinalImage()->GetData());
    }
    std::shared_ptr<Walnut::Image> GetFinalImage() const { return frame_image_final; }
    void Reaccumulate() { core_.Reaccumulate(); }
    uint32_t GetSPP() { return core_.GetSPP(); }
    Settings& GetSettings() { return core_.GetSettings(); }
    // the scene-extension API, MC/Renderer.h:72-86: Add(new Whitted::TriangleMesh(path, material)) or
    // Add(new Whitted::Sphere(center, radius, material)), then GenerateBVH(), which builds the device scene from
    // `entities` (a user-defined Whitted::Entity has no device form: rt::Error)
    [[nodiscard]] const std::vector<Whitted::Entity*>& GetEntities() const { return entities; }
    void Add(Whitted::Entity* entity_pointer) { entities.push_back(entity_pointer); }
    void GenerateBVH()
    {
        core_.entities.assign(entities.begin(), entities.end());
        core_.GenerateBVH();
        bvh_.reset(new AccelerationStructure::BVH([this](const AccelerationStructure::Ray& r) { return ray_BVH_intersection_record(r); }));
        bvh = bvh_.get();
        // TriangleMesh::Sampling of the light -- the first emissive entity, the one SamplingAreaLight samples
        // (MC/Renderer.h:169-179) -- runs the device's light sampler
        for (Whitted::Entity* e : entities) {
            if (auto* t = dynamic_cast<Whitted::TriangleMesh*>(e)) t->light_sampler = nullptr;
        }
        for (Whitted::Entity* e : entities) {
            if (!e->IsEmissive()) continue;
            if (auto* t = dynamic_cast<Whitted::TriangleMesh*>(e))
                t->light_sampler = [this](Whitted::IntersectionRecord& rec, float& pdf) { SamplingAreaLight(rec, pdf); };
            break;
        }
    }

    // Renderer::ray_BVH_intersection_record (MC/Renderer.h:88-91): the closest hit of the ray in the scene of
    // the last GenerateBVH -- the device traversal (rt_trace), the reference's double t and tie rule -- filled
    // as TrianglePrimitive::GetIntersectionRecord fills it (MC/TriangleMesh.h:118-134): the face normal, the
    // location ray((float)t), the material; a miss is a default record (t = DBL_MAX)
    Whitted::IntersectionRecord ray_BVH_intersection_record(const AccelerationStructure::Ray& ray) const
    {
        Whitted::IntersectionRecord record;
        const rt::Renderer::Hit h = core_.Trace(rt::vec3{ray.m_origin.x, ray.m_origin.y, ray.m_origin.z},
                                                rt::vec3{ray.m_direction.x, ray.m_direction.y, ray.m_direction.z});
        if (!h.hit) return record;
        record.has_intersection = true;
        record.t = h.t;
        record.location = ray(h.t);
        record.surface_normal = glm::vec3{h.normal.x, h.normal.y, h.normal.z};
        record.hitted_entity = entity_of(h.mesh);
        record.hitted_entity_material = material_of(h.mesh);
        return record;
    }

    // MC/Renderer.h:93-97
    glm::vec3 mirror_reflection_direction(const glm::vec3& incident_ray_direction, const glm::vec3& surface_normal) const
    {
        const float k = 2 * dot(incident_ray_direction, surface_normal);
        return glm::vec3{incident_ray_direction.x - k * surface_normal.x, incident_ray_direction.y - k * surface_normal.y,
                         incident_ray_direction.z - k * surface_normal.z};
    }

    // MC/Renderer.h:99-129 (unit incident direction towards the surface, outward unit normal; (0,0,0) on total
    // internal reflection)
    glm::vec3 snell_refraction_direction(const glm::vec3& incident_ray_direction, const glm::vec3& surface_normal,
                                         const float& entity_refraction_index) const
    {
        float eta_in = eta_Vacuum;
        float eta_out = entity_refraction_index;
        glm::vec3 normal = surface_normal;
        float cos_incident = Whitted::clamp_float(dot(incident_ray_direction, surface_normal), -1, 1);
        if (cos_incident < 0) {
            cos_incident = -cos_incident;   // from the outside
        } else {
            std::swap(eta_in, eta_out);     // from the inside (cos_incident == 0 counts as inside)
            normal = glm::vec3{-normal.x, -normal.y, -normal.z};
        }
        const float eta_ratio = eta_in / eta_out;
        const float cos_refract_squared = 1 - eta_ratio * eta_ratio * (1 - cos_incident * cos_incident);
        if (cos_refract_squared < 0) return glm::vec3{0.0f, 0.0f, 0.0f};
        const float k = eta_ratio * cos_incident - std::sqrt(cos_refract_squared);
        return glm::vec3{eta_ratio * incident_ray_direction.x + k * normal.x, eta_ratio * incident_ray_direction.y + k * normal.y,
                         eta_ratio * incident_ray_direction.z + k * normal.z};
    }

    // MC/Renderer.h:131-161: the unpolarised Fresnel reflectance (not Schlick's approximation)
    float accurate_fresnel_reflectance(const glm::vec3& incident_ray_direction, const glm::vec3& surface_normal,
                                       const float& entity_refraction_index) const
    {
        float eta_in = eta_Vacuum;
        float eta_out = entity_refraction_index;
        float cos_incident = Whitted::clamp_float(dot(incident_ray_direction, surface_normal), -1, 1);
        if (cos_incident < 0) cos_incident = -cos_incident;
        else std::swap(eta_in, eta_out);
        const float sin_refract = eta_in / eta_out * std::sqrt(std::max(0.0f, 1 - cos_incident * cos_incident));
        if (sin_refract > 1.0f) return 1.0f;   // total internal reflection
        const float cos_refract = std::sqrt(std::max(0.0f, 1 - sin_refract * sin_refract));
        const float R_s_sqrt = (eta_in * cos_incident - eta_out * cos_refract) / (eta_in * cos_incident + eta_out * cos_refract);
        const float R_p_sqrt = (eta_in * cos_refract - eta_out * cos_incident) / (eta_in * cos_refract + eta_out * cos_incident);
        return (R_s_sqrt * R_s_sqrt + R_p_sqrt * R_p_sqrt) / 2;
    }

    // Renderer::SamplingAreaLight (MC/Renderer.h:163-180): the first emissive entity's Sampling -- emission, a point
    // of the light drawn area-uniformly (BVH::Sampling_from_root, MC/BVH.h:103-129; TrianglePrimitive::Sampling,
    // MC/TriangleMesh.h:69-89), its face normal and PDF = 1 / the light's total area -- with three draws of
    // Whitted::get_random_u32 (this thread's Walnut::Random engine); on the device (rt_sample_light).  No
    // emissive entity: the record and PDF are left as they are.
    void SamplingAreaLight(Whitted::IntersectionRecord& sample, float& PDF) const
    {
        if (!has_light()) return;
        uint32_t u[3];
        for (uint32_t& w : u) w = Whitted::get_random_u32();
        SamplingAreaLight(sample, PDF, u);
    }
    // the same on three given draws (the raw engine words)
    void SamplingAreaLight(Whitted::IntersectionRecord& sample, float& PDF, const uint32_t draws[3]) const
    {
        if (!has_light()) return;
        const rt::Renderer::LightSample ls = core_.SampleLight(draws);
        sample.emission = glm::vec3{ls.emission.x, ls.emission.y, ls.emission.z};
        sample.location = glm::vec3{ls.location.x, ls.location.y, ls.location.z};
        sample.surface_normal = glm::vec3{ls.normal.x, ls.normal.y, ls.normal.z};
        PDF = ls.pdf;
    }

    float RR_survival_probability = 0.8f;   // MC/Renderer.h:199 (read at every Render)
    AccelerationStructure::BVH* bvh = nullptr;   // MC/Renderer.h:200: the scene of the last GenerateBVH
    std::vector<Whitted::Entity*> entities;      // MC/Renderer.h:201: what GenerateBVH builds the scene from

    rt::Renderer& Core() { return core_; }

private:
    static float dot(const glm::vec3& a, const glm::vec3& b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }   // glm's order
    Whitted::Entity* entity_of(int32_t mesh) const
    {   // the entities of the last GenerateBVH, in Add order
        const auto& e = core_.GetEntities();
        return mesh >= 0 && (size_t)mesh < e.size() ? dynamic_cast<Whitted::Entity*>(e[mesh]) : nullptr;
    }
    Whitted::WhittedMaterial* material_of(int32_t mesh) const
    {
        Whitted::Entity* e = entity_of(mesh);
        if (auto* t = dynamic_cast<Whitted::TriangleMesh*>(e)) return t->UnifiedMaterial();
        if (auto* sp = dynamic_cast<Whitted::Sphere*>(e)) return sp->UnifiedMaterial();
        return nullptr;
    }
    bool has_light() const
    {   // IsEmissive of some entity of the scene (MC/Renderer.h:169-179)
        for (rt::Entity* e : core_.GetEntities())
            if (auto* w = dynamic_cast<Whitted::Entity*>(e); w && w->IsEmissive()) return true;
        return false;
    }

    rt::Renderer core_;
    std::shared_ptr<Walnut::Image> frame_image_final;
    std::vector<std::unique_ptr<Whitted::WhittedMaterial>> builtin_materials_;
    std::vector<std::unique_ptr<Whitted::TriangleMesh>> builtin_meshes_;
    std::unique_ptr<AccelerationStructure::BVH> bvh_;
};

#endif
