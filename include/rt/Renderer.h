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
#include "Camera.h"

namespace rt {

struct Material {   // Whitted::WhittedMaterial (Diffuse only), MC/WhittedMaterial.h:17-153
    vec3 diffuse_coefficient{1.0f, 1.0f, 1.0f};
    vec3 emission{0.0f, 0.0f, 0.0f};
};

class Entity {   // Whitted::Entity (MC/Entity.h:19-55): here only triangle meshes exist
public:
    virtual ~Entity() = default;
    virtual const std::vector<float>& RawPositions() const = 0;   // objl positions, pre-scale
    virtual const Material& GetMaterial() const = 0;
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

class Error : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

class Renderer {
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

    Renderer();                                  // Cornell box, device 0
    explicit Renderer(const Settings& s, bool cornell_box = true);
    ~Renderer();
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    void ResizeViewport(uint32_t width, uint32_t height);
    void Render(const Camera& camera);                      // +1 spp
    void RenderFrames(const Camera& camera, uint32_t n);    // +n spp in one launch
    std::shared_ptr<rt::Image> GetFinalImage() const { return frame_image_final; }
    const std::vector<float>& GetAccumulation();            // float4 per pixel (host copy)
    void Reaccumulate() { frame_accumulating = 1; ++epoch; }
    uint32_t GetSPP() { return frame_accumulating - 1; }
    Settings& GetSettings() { return settings; }
    [[nodiscard]] const std::vector<rt::Entity*>& GetEntities() const { return entities; }
    void Add(rt::Entity* entity_pointer) { entities.push_back(entity_pointer); }
    void GenerateBVH();
    float LastKernelMilliseconds() const;
    // the flattened scene of the last GenerateBVH (host side: rt_scene_get_info / rt_scene_export), e.g. to
    // check a scene built through Add against the reference's BVH
    const rt_scene* Scene() const { return scene_; }

    float RR_survival_probability = 0.8f;        // MC/Renderer.h:199
    std::vector<rt::Entity*> entities;

private:
    void check(rt_status s, const char* what) const;
    Settings settings;
    std::shared_ptr<rt::Image> frame_image_final;
    std::vector<float> accum_host;
    uint32_t frame_accumulating = 1;
    uint64_t epoch = 0;
    rt_ctx* ctx = nullptr;
    rt_group* group = nullptr;   // Settings::devices with more than one entry
    std::vector<std::unique_ptr<rt::Entity>> owned;   // the built-in Cornell meshes
    rt_scene* scene_ = nullptr;
    bool bvh_dirty = true;
};

}  // namespace rt

// The reference's global name (MC/Renderer.h:30).  A Walnut front-end includes rt/walnut/Renderer.h
// instead, whose global Renderer hands Walnut::Image frames to the layer (it defines RT_NO_GLOBAL_NAMES).
#ifndef RT_NO_GLOBAL_NAMES
using Renderer = rt::Renderer;
#endif

#endif
