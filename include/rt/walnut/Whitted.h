// include/rt/walnut/Whitted.h -- the reference's scene-extension types, spelled as the reference spells them:
//   Whitted::MaterialNature, Whitted::WhittedMaterial   MC/WhittedMaterial.h:15-153
//   Whitted::Entity (the whole virtual interface)      MC/Entity.h:17-55
//   Whitted::TriangleMesh(file_path, WhittedMaterial*) MC/TriangleMesh.h:144-267
//   Whitted::Sphere(center, radius, WhittedMaterial*)  MC/Sphere.h:16-108 (round 6: rendered on the GPU)
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
#include <functional>
#include <limits>
#include <random>
#include <string>
#include <vector>

#include <glm/glm.hpp>

#include "../Renderer.h"
#include "BoundingVolume.h"
#include "Ray.h"

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

class Entity;

// Whitted::IntersectionRecord, MC/IntersectionRecord.h:18-38 (what ray_BVH_intersection_record and
// SamplingAreaLight of the drop-in Renderer return).  hitted_entity is the hit ENTITY (a mesh or a sphere: the
// flattened scene has no per-triangle entity objects; the reference points at its TrianglePrimitive),
// hitted_entity_material the entity's material.
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

// MC/WhittedUtilities.h:18-60, MC/VectorFloat.h:17-31
#ifndef INTERSECTION_CORRECTION
#define INTERSECTION_CORRECTION 0.00001f
#endif
#ifndef PI
#define PI 3.141592653589793f
#endif
inline float clamp_float(const float& value, const float& lower_bound, const float& upper_bound)
{
    return std::max(std::min(value, upper_bound), lower_bound);
}
// zero-safe: v itself when its squared length is not positive
inline glm::vec3 normalize(const glm::vec3& v)
{
    const float l2 = v.x * v.x + v.y * v.y + v.z * v.z;
    if (l2 > 0) {
        const float inv = 1 / std::sqrt(l2);
        return glm::vec3{v.x * inv, v.y * inv, v.z * inv};
    }
    return v;
}
inline glm::vec3 lerp(const glm::vec3& a, const glm::vec3& b, const float& t)
{
    return glm::vec3{a.x * (1 - t) + b.x * t, a.y * (1 - t) + b.y * t, a.z * (1 - t) + b.z * t};
}
// the roots of A x^2 + B x + C in float, the reference's -0.5 literals in double (the device's sphere test,
// csrc/rt_device.h sphere_hit, is the same sequence)
inline bool QuadraticFormula(const float& A, const float& B, const float& C, float& x_small, float& x_large)
{
    const float discriminant = B * B - 4 * A * C;
    if (discriminant < 0) return false;
    if (discriminant == 0) {
        x_small = x_large = -0.5 * B / A;
    } else {
        const float q = (B > 0) ? (-0.5 * (B + std::sqrt(discriminant))) : (-0.5 * (B - std::sqrt(discriminant)));
        x_small = q / A;
        x_large = C / q;
    }
    if (x_small > x_large) std::swap(x_small, x_large);
    return true;
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

// Whitted::Entity, MC/Entity.h:19-55: the reference's virtual interface.  It is also an rt::Entity, the device's
// view GenerateBVH reads (include/rt/Renderer.h): TriangleMesh and Sphere below provide it; a user-defined
// subclass has no device form, and GenerateBVH throws rt::Error for it (its intersection code is host code).
class Entity : public rt::Entity {
public:
    Entity() {}
    virtual ~Entity() {}
    virtual float GetArea() = 0;
    virtual void Sampling(IntersectionRecord& sample, float& PDF) = 0;
    virtual bool IsEmissive() = 0;
    virtual AccelerationStructure::AABB_3D Get3DAABB() = 0;
    virtual glm::vec3 GetDiffuseColor(const glm::vec2& texture_coordinates = glm::vec2{0.0f, 0.0f}) const = 0;
    virtual IntersectionRecord GetIntersectionRecord(AccelerationStructure::Ray ray) = 0;
    virtual void GetHitInfo(const glm::vec3& intersection, const glm::vec3& light_direction, const uint32_t& triangle_index,
                            const glm::vec2& barycentric_coordinates, glm::vec3& surface_normal, glm::vec2& texture_coordinates) const = 0;
};

class TriangleMesh : public Entity {   // MC/TriangleMesh.h:144-267
public:
    TriangleMesh(const std::string& file_path, WhittedMaterial* m) : mesh_(file_path, rt::Material{}), unified_material(m) { summarize(); }
    // the same from objl positions already loaded (pre-scale, 9 floats per triangle; the drop-in Renderer's
    // Cornell meshes)
    TriangleMesh(std::vector<float> raw_positions, WhittedMaterial* m) : mesh_(std::move(raw_positions), rt::Material{}), unified_material(m)
    {
        summarize();
    }

    // rt::Entity: the positions and the pointed-to material's values at GenerateBVH
    const std::vector<float>& RawPositions() const override { return mesh_.RawPositions(); }
    const rt::Material& GetMaterial() const override
    {
        material_.diffuse_coefficient = rt::vec3{unified_material->diffuse_coefficient.x, unified_material->diffuse_coefficient.y,
                                                 unified_material->diffuse_coefficient.z};
        material_.emission = rt::vec3{unified_material->m_emission.x, unified_material->m_emission.y, unified_material->m_emission.z};
        return material_;
    }

    // Whitted::Entity
    float GetArea() override { return total_area; }
    // TriangleMesh::Sampling (MC/TriangleMesh.h:193-197) runs on the device for the scene's light (the mesh the
    // drop-in Renderer's SamplingAreaLight samples, rt_sample_light); the library keeps no host copy of other
    // meshes' sampling trees
    void Sampling(IntersectionRecord& sample, float& PDF) override
    {
        if (!light_sampler) throw rt::Error("Whitted::TriangleMesh::Sampling: only the scene's light mesh samples (on the device), via the Renderer it was added to");
        light_sampler(sample, PDF);
    }
    bool IsEmissive() override { return unified_material->IsEmitting(); }   // MC/TriangleMesh.h:198-201
    AccelerationStructure::AABB_3D Get3DAABB() override { return bounding_AABB; }
    glm::vec3 GetDiffuseColor(const glm::vec2& uv) const override
    {   // the procedural chessboard of MC/TriangleMesh.h:231-238
        const float frequency = 5;
        const float pattern = (std::fmod(uv.x * frequency, 1.0f) > 0.5f) ^ (std::fmod(uv.y * frequency, 1.0f) > 0.5f);
        return lerp(glm::vec3{0.815f, 0.235f, 0.031f}, glm::vec3{0.937f, 0.937f, 0.231f}, pattern);
    }
    // the mesh's own closest hit is the device traversal's business: the Renderer answers rays against the whole
    // scene (ray_BVH_intersection_record, bvh->traverse_BVH_from_root)
    IntersectionRecord GetIntersectionRecord(AccelerationStructure::Ray) override
    {
        throw rt::Error("Whitted::TriangleMesh::GetIntersectionRecord: rays are answered by the device scene "
                        "(Renderer::ray_BVH_intersection_record / renderer.bvh->traverse_BVH_from_root)");
    }
    // the reference reads vertex / index arrays that MC's TriangleMesh never fills (MC/TriangleMesh.h:241-262)
    void GetHitInfo(const glm::vec3&, const glm::vec3&, const uint32_t&, const glm::vec2&, glm::vec3&, glm::vec2&) const override
    {
        throw rt::Error("Whitted::TriangleMesh::GetHitInfo: no per-vertex data (the reference's MC mesh leaves it unset)");
    }

    WhittedMaterial* UnifiedMaterial() const { return unified_material; }   // (private in the reference)
    // set by the drop-in Renderer for its light mesh (include/rt/walnut/Renderer.h)
    std::function<void(IntersectionRecord&, float&)> light_sampler;

private:
    // total_area and bounding_AABB as the reference's constructor sums them (MC/TriangleMesh.h:150-186): scaled
    // vertices 0.01 * p, per triangle 0.5 * length(cross(b - a, c - a)) (glm's dot order), the std::min / max range
    void summarize()
    {
        const std::vector<float>& raw = mesh_.RawPositions();
        const float inf = std::numeric_limits<float>::infinity();
        glm::vec3 mn{inf, inf, inf}, mx{-inf, -inf, -inf};
        total_area = 0.0f;
        for (size_t t = 0; t + 9 <= raw.size(); t += 9) {
            glm::vec3 v[3];
            for (int j = 0; j < 3; ++j) {
                v[j] = glm::vec3{0.01f * raw[t + 3 * j], 0.01f * raw[t + 3 * j + 1], 0.01f * raw[t + 3 * j + 2]};
                mn = glm::vec3{std::min(mn.x, v[j].x), std::min(mn.y, v[j].y), std::min(mn.z, v[j].z)};
                mx = glm::vec3{std::max(mx.x, v[j].x), std::max(mx.y, v[j].y), std::max(mx.z, v[j].z)};
            }
            const float e1x = v[1].x - v[0].x, e1y = v[1].y - v[0].y, e1z = v[1].z - v[0].z;
            const float e2x = v[2].x - v[0].x, e2y = v[2].y - v[0].y, e2z = v[2].z - v[0].z;
            const float cx = e1y * e2z - e2y * e1z, cy = e1z * e2x - e2z * e1x, cz = e1x * e2y - e2x * e1y;
            const float pxx = cx * cx, pyy = cy * cy, pzz = cz * cz;
            total_area += 0.5f * std::sqrt((pxx + pyy) + pzz);
        }
        bounding_AABB = AccelerationStructure::AABB_3D{mn, mx};
    }

    rt::TriangleMesh mesh_;
    WhittedMaterial* unified_material = nullptr;
    mutable rt::Material material_;
    float total_area = 0.0f;
    AccelerationStructure::AABB_3D bounding_AABB;
};

class Sphere : public Entity {   // MC/Sphere.h:16-108
public:
    Sphere(const glm::vec3& center, const float& radius, WhittedMaterial* _material = new WhittedMaterial{})
        : material{_material}, m_center{center}, m_radius{radius}, radius_squared{radius * radius}
    {
        surface_area = 4 * PI * radius_squared;
    }

    // rt::Entity: rendered by the device's sphere test (csrc/rt_device.h sphere_hit, the same QuadraticFormula)
    bool SphereShape(rt::vec3& center, float& radius) const override
    {
        center = rt::vec3{m_center.x, m_center.y, m_center.z};
        radius = m_radius;
        return true;
    }
    const rt::Material& GetMaterial() const override
    {
        material_.diffuse_coefficient = rt::vec3{material->diffuse_coefficient.x, material->diffuse_coefficient.y, material->diffuse_coefficient.z};
        material_.emission = rt::vec3{material->m_emission.x, material->m_emission.y, material->m_emission.z};
        return material_;
    }

    // Whitted::Entity
    float GetArea() override { return surface_area; }
    void Sampling(IntersectionRecord&, float&) override {}   // a TODO in the reference (MC/Sphere.h:30-33)
    bool IsEmissive() override { return material->IsEmitting(); }
    glm::vec3 GetDiffuseColor(const glm::vec2&) const override { return material->GetDiffuseColor(); }
    AccelerationStructure::AABB_3D Get3DAABB() override
    {   // AABB_3D{center + radius, center - radius}
        return AccelerationStructure::AABB_3D{glm::vec3{m_center.x + m_radius, m_center.y + m_radius, m_center.z + m_radius},
                                              glm::vec3{m_center.x - m_radius, m_center.y - m_radius, m_center.z - m_radius}};
    }
    void GetHitInfo(const glm::vec3& intersection, const glm::vec3&, const uint32_t&, const glm::vec2&, glm::vec3& surface_normal,
                    glm::vec2&) const override
    {
        surface_normal = Whitted::normalize(glm::vec3{intersection.x - m_center.x, intersection.y - m_center.y, intersection.z - m_center.z});
    }
    // MC/Sphere.h:62-97: the nearer non-negative root of the ray's quadratic; location ray(t), outward normal
    IntersectionRecord GetIntersectionRecord(AccelerationStructure::Ray ray) override
    {
        IntersectionRecord record;
        const glm::vec3 co{ray.m_origin.x - m_center.x, ray.m_origin.y - m_center.y, ray.m_origin.z - m_center.z};
        const glm::vec3& d = ray.m_direction;
        float t_small, t_large;
        if (!QuadraticFormula((d.x * d.x + d.y * d.y) + d.z * d.z, 2 * ((d.x * co.x + d.y * co.y) + d.z * co.z),
                              ((co.x * co.x + co.y * co.y) + co.z * co.z) - radius_squared, t_small, t_large))
            return record;
        if (t_small < 0.0f) t_small = t_large;
        if (t_small < 0.0f) return record;
        record.has_intersection = true;
        record.t = t_small;
        record.hitted_entity = this;
        record.location = ray(t_small);
        record.hitted_entity_material = material;
        record.surface_normal = Whitted::normalize(glm::vec3{record.location.x - m_center.x, record.location.y - m_center.y,
                                                             record.location.z - m_center.z});
        return record;
    }

private:
    float surface_area;
    WhittedMaterial* material;
    glm::vec3 m_center;
    float m_radius;
    float radius_squared;
    mutable rt::Material material_;

public:
    WhittedMaterial* UnifiedMaterial() const { return material; }   // (private in the reference)
};

}  // namespace Whitted

#endif
