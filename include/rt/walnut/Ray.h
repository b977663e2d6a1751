// include/rt/walnut/Ray.h -- AccelerationStructure::Ray, MC/Ray.h:21-44, the argument of the drop-in
// Renderer's ray_BVH_intersection_record.  Needs the application's <glm/glm.hpp>.
#ifndef RT_WALNUT_RAY_H
#define RT_WALNUT_RAY_H
#include <limits>

#include <glm/glm.hpp>

namespace AccelerationStructure {

struct Ray {
    Ray(const glm::vec3& origin, const glm::vec3& direction) : m_origin(origin), m_direction(direction)
    {
        t_min = 0.0;
        t_max = std::numeric_limits<double>::max();
        direction_reciprocal = glm::vec3{1.0f / direction.x, 1.0f / direction.y, 1.0f / direction.z};
    }
    // origin + (float)t * direction (MC/Ray.h:34-37): the location of a hit record is computed with the float t
    glm::vec3 operator()(double t) const
    {
        const float tf = (float)t;
        return glm::vec3{m_origin.x + tf * m_direction.x, m_origin.y + tf * m_direction.y, m_origin.z + tf * m_direction.z};
    }

    glm::vec3 m_origin;
    glm::vec3 m_direction;
    glm::vec3 direction_reciprocal;
    double t_min;
    double t_max;
};

}  // namespace AccelerationStructure

#endif
