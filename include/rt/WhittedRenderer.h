// include/rt/WhittedRenderer.h -- drop-in for the Renderer of the reference's two Whitted-style
// projects, on the MI355X Whitted kernels (csrc/rt_whitted.hip):
//   * "BVH Ray Tracer" (BV/Renderer.{h,cpp}): the Stanford bunny and the Utah teapot behind a BVH,
//     two point lights (BV/Renderer.cpp:26-43) -- WhittedRenderer::BVHRayTracer(bunny, teapot);
//   * "Whitted Style Ray Tracer" (WH/Renderer.{h,cpp}): a diffuse and a glass sphere over a textured
//     chessboard with Fresnel/Snell recursion to depth 5 (WH/Renderer.cpp:27-49) --
//     WhittedRenderer::TwoSpheres().
// Same public surface as those classes: ResizeViewport, Render(camera) = +1 frame with temporal
// accumulation / clamp / RGBA8 pack (BV/Renderer.cpp:69-119, WH/Renderer.cpp:82-125), GetFinalImage,
// Reaccumulate, GetSettings().accumulating.  In BV/mainloop.cpp or WH/mainloop.cpp the change is
// `Renderer renderer;` -> `auto renderer = rt::WhittedRenderer::BVHRayTracer(...)` / `::TwoSpheres()`
// (INTEGRATION.md).
#ifndef RT_WHITTED_RENDERER_H
#define RT_WHITTED_RENDERER_H
#include <cstdint>
#include <memory>
#include <string>

#include "../rt_capi.h"
#include "Camera.h"
#include "Renderer.h"

namespace rt {

struct WhittedSettings {
    bool accumulating = true;
    int device = 0;
};

class WhittedRenderer {
    // first member: checked against the library's layout before any other member is written (rt/Abi.h)
    AbiGuard abi_;

public:
    using Settings = WhittedSettings;
    // the two reference worlds
    static std::unique_ptr<WhittedRenderer> TwoSpheres(const Settings& s = Settings{});
    static std::unique_ptr<WhittedRenderer> BVHRayTracer(const std::string& bunny_obj, const std::string& teapot_obj,
                                                         const Settings& s = Settings{});
    // the cameras of those projects (Camera{35, 0.1, 100} with the project's member defaults)
    static Camera TwoSpheresCamera() { return Camera(35.0f, 0.1f, 100.0f, vec3{0.0f, 0.0f, 6.0f}, vec3{0.0f, 0.0f, -1.0f}); }
    static Camera BVHRayTracerCamera() { return Camera(35.0f, 0.1f, 100.0f, vec3{-1.0f, 5.0f, 10.0f}, vec3{0.0f, 0.0f, -1.0f}); }

    // any world built through the C-ABI scene builder (rt_scene_add_world_* or rt_scene_add_whitted_*)
    WhittedRenderer(rt_scene* built_scene, const Settings& s)
        : WhittedRenderer(AbiTag{RT_CXX_ABI_VERSION, AbiClass::WhittedRenderer, sizeof(WhittedRenderer), sizeof(Settings)}, built_scene, s)
    {
    }
    ~WhittedRenderer();
    WhittedRenderer(const WhittedRenderer&) = delete;
    WhittedRenderer& operator=(const WhittedRenderer&) = delete;

    void ResizeViewport(uint32_t width, uint32_t height);
    void Render(const Camera& camera);                      // +1 frame
    void RenderFrames(const Camera& camera, uint32_t n);    // +n frames in one launch
    std::shared_ptr<Image> GetFinalImage() const { return frame_image_final; }
    void Reaccumulate() { frame_accumulating = 1; }
    uint32_t GetSPP() const { return frame_accumulating - 1; }
    Settings& GetSettings() { return settings; }
    float LastKernelMilliseconds() const;

private:
    WhittedRenderer(const AbiTag& caller, rt_scene* built_scene, const Settings& s);   // librt_hip.so
    void check(rt_status s, const char* what) const;
    Settings settings;
    std::shared_ptr<Image> frame_image_final;
    uint32_t frame_accumulating = 1;
    rt_ctx* ctx = nullptr;
};

}  // namespace rt

#endif
