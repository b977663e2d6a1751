// include/rt/walnut/BoundingVolume.h -- AccelerationStructure::AABB_3D, the box type of the reference's Entity
// interface (Whitted::Entity::Get3DAABB, MC/Entity.h:38; MC/BoundingVolume.h:19-226), for code that extends the
// scene the reference's way.  The renderer never reads these boxes: GenerateBVH builds the device scene from the
// entities' shapes (rt::Entity), with the reference's own box arithmetic (csrc/rt_scene.cpp).  Needs the
// application's <glm/glm.hpp>; componentwise arithmetic only, as include/rt/walnut/Ray.h.
#ifndef RT_WALNUT_BOUNDING_VOLUME_H
#define RT_WALNUT_BOUNDING_VOLUME_H
#include <algorithm>
#include <array>
#include <cmath>
#include <limits>

#include <glm/glm.hpp>

#include "Ray.h"

namespace AccelerationStructure {

enum Axis { X_axis, Y_axis, Z_axis };   // MC/BoundingVolume.h:19-24

class AABB_3D {
public:
    // the box of nothing: double max / lowest narrowed to float, i.e. +inf / -inf (MC/BoundingVolume.h:32-39)
    AABB_3D()
    {
        const float inf = (float)std::numeric_limits<double>::max();
        min_slab_values = glm::vec3{inf, inf, inf};
        max_slab_values = glm::vec3{-inf, -inf, -inf};
    }
    explicit AABB_3D(const glm::vec3& point) : min_slab_values{point}, max_slab_values{point} {}
    // the box spanned by two corners, componentwise std::fmin / std::fmax (MC/BoundingVolume.h:47-51)
    AABB_3D(const glm::vec3& p1, const glm::vec3& p2)
    {
        min_slab_values = glm::vec3{std::fmin(p1.x, p2.x), std::fmin(p1.y, p2.y), std::fmin(p1.z, p2.z)};
        max_slab_values = glm::vec3{std::fmax(p1.x, p2.x), std::fmax(p1.y, p2.y), std::fmax(p1.z, p2.z)};
    }

    glm::vec3 center_vector() const
    {   // 0.5f * (max + min)
        return glm::vec3{0.5f * (max_slab_values.x + min_slab_values.x), 0.5f * (max_slab_values.y + min_slab_values.y),
                         0.5f * (max_slab_values.z + min_slab_values.z)};
    }
    glm::vec3 diagonal_vector() const
    {
        return glm::vec3{max_slab_values.x - min_slab_values.x, max_slab_values.y - min_slab_values.y, max_slab_values.z - min_slab_values.z};
    }
    int longest_axis() const
    {
        const glm::vec3 d = diagonal_vector();
        if (d.x > d.y && d.x > d.z) return X_axis;
        return d.y > d.z ? Y_axis : Z_axis;
    }
    // glm::min / glm::max: (b < a) ? b : a and (a < b) ? b : a per component
    AABB_3D Union_with_point(const glm::vec3& p) const
    {
        AABB_3D u;
        u.min_slab_values = glm::vec3{lo(min_slab_values.x, p.x), lo(min_slab_values.y, p.y), lo(min_slab_values.z, p.z)};
        u.max_slab_values = glm::vec3{hi(max_slab_values.x, p.x), hi(max_slab_values.y, p.y), hi(max_slab_values.z, p.z)};
        return u;
    }
    AABB_3D Union_with_3D_AABB(const AABB_3D& b) const
    {
        AABB_3D u;
        u.min_slab_values = glm::vec3{lo(min_slab_values.x, b.min_slab_values.x), lo(min_slab_values.y, b.min_slab_values.y),
                                      lo(min_slab_values.z, b.min_slab_values.z)};
        u.max_slab_values = glm::vec3{hi(max_slab_values.x, b.max_slab_values.x), hi(max_slab_values.y, b.max_slab_values.y),
                                      hi(max_slab_values.z, b.max_slab_values.z)};
        return u;
    }
    // the slab test of the reference's traversal (MC/BoundingVolume.h:173-215): entry and exit per axis swapped
    // for a negative direction, std::max / std::min of the three, a hit when exit >= 0 and entry <= exit
    bool intersects_with_ray(const Ray& ray, const glm::vec3& inv, const std::array<int, 3>& neg) const
    {
        float in[3] = {(min_slab_values.x - ray.m_origin.x) * inv.x, (min_slab_values.y - ray.m_origin.y) * inv.y,
                       (min_slab_values.z - ray.m_origin.z) * inv.z};
        float out[3] = {(max_slab_values.x - ray.m_origin.x) * inv.x, (max_slab_values.y - ray.m_origin.y) * inv.y,
                        (max_slab_values.z - ray.m_origin.z) * inv.z};
        for (int a = 0; a < 3; ++a)
            if (neg[a]) std::swap(in[a], out[a]);
        const float t_in = std::max(in[0], std::max(in[1], in[2]));
        const float t_out = std::min(out[0], std::min(out[1], out[2]));
        return t_out >= 0 && t_in <= t_out;
    }

    glm::vec3 min_slab_values;
    glm::vec3 max_slab_values;

private:
    static float lo(float a, float b) { return (b < a) ? b : a; }
    static float hi(float a, float b) { return (a < b) ? b : a; }
};

}  // namespace AccelerationStructure

#endif
