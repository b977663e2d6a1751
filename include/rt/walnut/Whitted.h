// include/rt/walnut/Whitted.h -- the reference's scene-extension types, spelled as the reference spells them:
//   Whitted::MaterialNature, Whitted::WhittedMaterial   MC/WhittedMaterial.h:15-153
//   Whitted::Entity                                    MC/Entity.h:17-55
//   Whitted::TriangleMesh(file_path, WhittedMaterial*) MC/TriangleMesh.h:144-267
// so that code which extends the scene the reference way compiles unchanged against the drop-in Renderer
// (include/rt/walnut/Renderer.h, which includes this header as MC/Renderer.h includes TriangleMesh.h):
//
//     Whitted::WhittedMaterial* white = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
//     white->diffuse_coefficient = glm::vec3{0.7f, 0.7f, 0.7f};
//     renderer.Add(new Whitted::TriangleMesh("bunny.obj", white));
//     renderer.GenerateBVH();
//
// What the path tracer reads of a material is what MC/Renderer.cpp reads: `diffuse_coefficient` (the albedo
// of WhittedMaterial::BRDF, MC/WhittedMaterial.h:58-69) and `m_emission` (MC/TriangleMesh.h:195).  A mesh
// keeps the material POINTER, as the reference's `unified_material` does: the values are taken when
// GenerateBVH builds the device scene.  The mesh is loaded as the reference loads it (objl positions,
// de-indexed, x 0.01: MC/TriangleMesh.h:150-172), by the library's OBJ reader (csrc/rt_scene.cpp).
// Needs the application's <glm/glm.hpp>, like include/rt/walnut/Camera.h.
#ifndef RT_WALNUT_WHITTED_H
#define RT_WALNUT_WHITTED_H
#ifndef RT_NO_GLOBAL_NAMES
#define RT_NO_GLOBAL_NAMES
#endif
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <random>
#include <string>
#include <vector>

#include <glm/glm.hpp>

#include "../Renderer.h"

namespace Whitted {

enum MaterialNature { Diffuse };   // MC/WhittedMaterial.h:17-20

class WhittedMaterial {   // MC/WhittedMaterial.h:22-42 (constructor), 119-153 (accessors, public members)
public:
    WhittedMaterial(MaterialNature material_nature = Whitted::MaterialNature::Diffuse, glm::vec3 emission = glm::vec3{0.0f, 0.0f, 0.0f},
                    glm::vec3 diffuse_color = glm::vec3{1.0f, 1.0f, 1.0f})
        : m_material_nature(material_nature), diffuse_coefficient(diffuse_color), m_diffuse_color(diffuse_color), m_emission(emission)
    {
        // glm::length(emission) > 0.00001f (MC/WhittedMaterial.h:34): sqrt of glm's dot, (x*x + y*y) + z*z
        emitting = std::sqrt((emission.x * emission.x + emission.y * emission.y) + emission.z * emission.z) > 0.00001f;
    }
    bool IsEmitting() { return emitting; }
    glm::vec3 GetEmission() { return m_emission; }
    MaterialNature GetMaterialNature() { return m_material_nature; }
    glm::vec3 GetDiffuseColor() { return m_diffuse_color; }

    MaterialNature m_material_nature;
    float refractive_index = 1.0f;
    // the albedo (i.e. what BRDF reads).  The reference leaves it uninitialised and every caller assigns it
    // after construction (MC/Renderer.cpp:28-35); here it starts as the constructor's diffuse_color.
    glm::vec3 diffuse_coefficient;
    glm::vec3 m_diffuse_color;
    float specular_size_factor = 0.0f;
    glm::vec3 m_emission;
    bool emitting;
};

// the path tracer's entities are triangle meshes (MC/Entity.h's interface is the renderer's business here)
using Entity = rt::Entity;

// Whitted::IntersectionRecord, MC/IntersectionRecord.h:18-38 (what ray_BVH_intersection_record and
// SamplingAreaLight of the drop-in Renderer return).  hitted_entity is the hit MESH (the flattened scene has
// no per-triangle entity objects; the reference points at its TrianglePrimitive), hitted_entity_material the
// mesh's material.
class IntersectionRecord {
public:
    bool has_intersection = false;
    double t = std::numeric_limits<double>::max();
    glm::vec3 location{0.0f, 0.0f, 0.0f};
    glm::vec3 surface_normal{0.0f, 0.0f, 0.0f};
    glm::vec3 emission{0.0f, 0.0f, 0.0f};
    Entity* hitted_entity = nullptr;
    WhittedMaterial* hitted_entity_material = nullptr;
};

// MC/WhittedUtilities.h:18-30
#ifndef INTERSECTION_CORRECTION
#define INTERSECTION_CORRECTION 0.00001f
#endif
inline float clamp_float(const float& value, const float& lower_bound, const float& upper_bound)
{
    return std::max(std::min(value, upper_bound), lower_bound);
}

// Walnut::Random as the reference's platform (MSVC) runs it (WN/Random.h:27-48, WN/Random.cpp:5-6): a
// thread_local std::mt19937 with its default seed, drawn through a 32-bit uniform distribution, so one draw is
// one engine word; Float() = (float)word / (float)UINT32_MAX.  get_random_float_0_1 is MC/WhittedUtilities.h:23-26.
inline std::mt19937& random_engine()
{
    static thread_local std::mt19937 engine;
    return engine;
}
inline uint32_t get_random_u32() { return (uint32_t)random_engine()(); }
inline float get_random_float_0_1() { return (float)get_random_u32() / (float)UINT32_MAX; }

class TriangleMesh : public rt::Entity {   // MC/TriangleMesh.h:144-267
public:
    TriangleMesh(const std::string& file_path, WhittedMaterial* m) : mesh_(file_path, rt::Material{}), unified_material(m) {}
    const std::vector<float>& RawPositions() const override { return mesh_.RawPositions(); }
    const rt::Material& GetMaterial() const override
    {   // the pointed-to material's values at this call (GenerateBVH)
        material_.diffuse_coefficient = rt::vec3{unified_material->diffuse_coefficient.x, unified_material->diffuse_coefficient.y,
                                                 unified_material->diffuse_coefficient.z};
        material_.emission = rt::vec3{unified_material->m_emission.x, unified_material->m_emission.y, unified_material->m_emission.z};
        return material_;
    }
    bool IsEmissive() { return unified_material->IsEmitting(); }   // MC/TriangleMesh.h:198-201
    WhittedMaterial* UnifiedMaterial() const { return unified_material; }   // (private in the reference)

private:
    rt::TriangleMesh mesh_;
    WhittedMaterial* unified_material = nullptr;
    mutable rt::Material material_;
};

}  // namespace Whitted

#endif
