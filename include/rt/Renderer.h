// include/rt/Renderer.h -- drop-in for the reference Renderer (Monte Carlo Path Tracer/8599RayTracerGUI/src/Renderer.h:30-202).
//
// Same public surface and semantics: Renderer() builds the Cornell box (MC/Renderer.cpp:26-57),
// ResizeViewport, Render(camera) = +1 spp with temporal accumulation / clamp / RGBA8 pack
// (MC/Renderer.cpp:91-134), Reaccumulate, GetSPP, GetSettings().accumulating, Add + GenerateBVH,
// RR_survival_probability.  The per-pixel work runs in the MI355X megakernel through the C-ABI
// (include/rt_capi.h); RenderFrames(camera, n) renders n spp in ONE launch (the GPU-native call).
// GetFinalImage() returns an rt::Image holding the RGBA8 frame (row 0 = bottom, ABGR u32) that a
// Walnut layer hands to Walnut::Image::SetData.
#ifndef RT_RENDERER_H
#define RT_RENDERER_H
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../rt_capi.h"
#include "Abi.h"
#include "Camera.h"

namespace rt {

struct Material {   // Whitted::WhittedMaterial (Diffuse only), MC/WhittedMaterial.h:17-153
    vec3 diffuse_coefficient{1.0f, 1.0f, 1.0f};
    vec3 emission{0.0f, 0.0f, 0.0f};
};

// The device's view of an entity (Whitted::Entity, MC/Entity.h:19-55), read by Renderer::GenerateBVH: a triangle
// mesh's objl positions (pre-scale), or a sphere's center and radius, and the material.  An entity that is
// neither (a user-defined shape: its intersection code runs on the host in the reference) has no device form, and
// GenerateBVH throws rt::Error for it.
class Entity {
public:
    virtual ~Entity() = default;
    virtual const std::vector<float>& RawPositions() const { static const std::vector<float> none; return none; }
    virtual bool SphereShape(vec3& center, float& radius) const { (void)center; (void)radius; return false; }
    virtual const Material& GetMaterial() const { static const Material none; return none; }
};

class Sphere : public Entity {   // Whitted::Sphere(center, radius, material), MC/Sphere.h:16-108
public:
    Sphere(const vec3& center, float radius, const Material& m) : center_(center), radius_(radius), material_(m) {}
    bool SphereShape(vec3& center, float& radius) const override { center = center_; radius = radius_; return true; }
    const Material& GetMaterial() const override { return material_; }
private:
    vec3 center_;
    float radius_;
    Material material_;
};

class TriangleMesh : public Entity {   // Whitted::TriangleMesh(file_path, material), MC/TriangleMesh.h:148-186
public:
    TriangleMesh(const std::string& file_path, const Material& m);
    TriangleMesh(std::vector<float> raw_positions, const Material& m);
    const std::vector<float>& RawPositions() const override { return raw_; }
    const Material& GetMaterial() const override { return material_; }
private:
    std::vector<float> raw_;
    Material material_;
};

class Image {   // the data side of Walnut::Image (WN/Image.h:16-52)
public:
    Image(uint32_t w, uint32_t h) : width_(w), height_(h), data_((size_t)w * h, 0u) {}
    uint32_t GetWidth() const { return width_; }
    uint32_t GetHeight() const { return height_; }
    const uint32_t* GetData() const { return data_.data(); }
    uint32_t* Data() { return data_.data(); }
    void Resize(uint32_t w, uint32_t h) { width_ = w; height_ = h; data_.assign((size_t)w * h, 0u); }
private:
    uint32_t width_, height_;
    std::vector<uint32_t> data_;
};

class Renderer {
    // first member: checked against the library's layout before any other member is written (rt/Abi.h)
    AbiGuard abi_;

public:
    struct Settings {
        bool accumulating = true;
        uint64_t seed = 0;          // RNG key (frames are keyed by frame index; Reaccumulate bumps the epoch)
        bool exact = true;          // inner-first fold of the path recursion (bit-faithful accumulation)
        int device = 0;
        // several GPUs for one frame (rt_group_*): row bands dealt over these devices, RGBA8 gathered to
        // the first (RCCL when the devices are distinct); empty or one entry: a single device
        std::vector<int> devices;
        uint32_t band = 8;          // rows per band of the multi-GPU split
    };

    Renderer() : Renderer(Settings{}, true) {}   // Cornell box, device 0
    explicit Renderer(const Settings& s, bool cornell_box = true)
        : Renderer(AbiTag{RT_CXX_ABI_VERSION, AbiClass::Renderer, sizeof(Renderer), sizeof(Settings)}, s, cornell_box)
    {
    }
    ~Renderer();
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    void ResizeViewport(uint32_t width, uint32_t height);
    void Render(const Camera& camera);                      // +1 spp
    void RenderFrames(const Camera& camera, uint32_t n);    // +n spp in one launch
    std::shared_ptr<rt::Image> GetFinalImage() const;
    const std::vector<float>& GetAccumulation();            // float4 per pixel (host copy)
    void Reaccumulate();
    uint32_t GetSPP();
    Settings& GetSettings();
    [[nodiscard]] const std::vector<rt::Entity*>& GetEntities() const { return entities; }
    void Add(rt::Entity* entity_pointer) { entities.push_back(entity_pointer); }
    void GenerateBVH();
    float LastKernelMilliseconds() const;
    // the flattened scene of the last GenerateBVH (host side: rt_scene_get_info / rt_scene_export), e.g. to
    // check a scene built through Add against the reference's BVH
    const rt_scene* Scene() const;

    // The reference Renderer's scene queries on the scene of the last GenerateBVH, answered by this library's
    // device kernels (rt_trace / rt_sample_light: the path kernels' own traversal and light sampling).  One ray
    // or one sample per call, a kernel launch and a synchronisation each; batch through the C-ABI for many.
    // ray_BVH_intersection_record (MC/Renderer.h:88-91 -> BVH::traverse_BVH_from_root, MC/BVH.h:72-101):
    // the closest hit's double t, its triangle (flattened slot), the entity it belongs to (index into
    // GetEntities()) and the surface normal at the hit (a triangle's face normal, MC/TriangleMesh.h:57-59,118-134;
    // a sphere's normalize(location - center), MC/Sphere.h:89-94)
    struct Hit { bool hit = false; double t = 1.7976931348623157e308; int32_t triangle = -1; int32_t mesh = -1; vec3 normal{}; };
    Hit Trace(const vec3& origin, const vec3& direction) const;
    // SamplingAreaLight (MC/Renderer.h:163-180) on three given Walnut::Random words (area pick, triangle x,
    // triangle y): the point, the light triangle's normal, the light's emission and PDF = 1 / total light area
    struct LightSample { vec3 location, normal, emission; float pdf = 0.0f; };
    LightSample SampleLight(const uint32_t draws[3]) const;

    float RR_survival_probability = 0.8f;        // MC/Renderer.h:199
    std::vector<rt::Entity*> entities;           // MC/Renderer.h:201

private:
    Renderer(const AbiTag& caller, const Settings& s, bool cornell_box);   // librt_hip.so
    // everything else lives behind one pointer, so that the library's state can grow without changing the
    // layout a caller allocates
    struct Impl;
    std::unique_ptr<Impl> impl_;
};

}  // namespace rt

// The reference's global name (MC/Renderer.h:30).  A Walnut front-end includes rt/walnut/Renderer.h
// instead, whose global Renderer hands Walnut::Image frames to the layer (it defines RT_NO_GLOBAL_NAMES).
#ifndef RT_NO_GLOBAL_NAMES
using Renderer = rt::Renderer;
#endif

#endif
