// include/rt/walnut/BVH.h -- AccelerationStructure::BVH as the drop-in Renderer exposes it (its public `bvh`
// member, MC/Renderer.h:200; MC/BVH.h:45-218).  The tree itself lives on the device (flattened, csrc/rt_scene.cpp,
// built from the Renderer's entities by GenerateBVH with the reference's own split rule); this object answers
// traverse_BVH_from_root with the device traversal (the Renderer's rt_trace query), so
// `renderer.bvh->traverse_BVH_from_root(ray)` reads as it does against the reference.  Needs <glm/glm.hpp>.
#ifndef RT_WALNUT_BVH_H
#define RT_WALNUT_BVH_H
#include <functional>
#include <utility>

#include "Ray.h"
#include "Whitted.h"

namespace AccelerationStructure {

class BVH {
public:
    explicit BVH(std::function<Whitted::IntersectionRecord(const Ray&)> trace) : trace_(std::move(trace)) {}
    // MC/BVH.h:72-80: the closest hit of the ray in the scene of the last GenerateBVH (a default record on a miss)
    Whitted::IntersectionRecord traverse_BVH_from_root(const Ray& ray) const { return trace_(ray); }
    // MC/BVH.h:103-107 draws an entity by area over the whole entity tree; the path tracer never calls it on the
    // scene's tree (SamplingAreaLight samples the light entity's own tree: Renderer::SamplingAreaLight)
    void Sampling_from_root(Whitted::IntersectionRecord&, float&)
    {
        throw rt::Error("AccelerationStructure::BVH::Sampling_from_root on the scene tree: use Renderer::SamplingAreaLight");
    }

private:
    std::function<Whitted::IntersectionRecord(const Ray&)> trace_;
};

}  // namespace AccelerationStructure

#endif
