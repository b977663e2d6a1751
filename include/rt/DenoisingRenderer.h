// include/rt/DenoisingRenderer.h -- drop-in for the Renderer of the reference's "Denoiser" project
// (DN/Renderer.{h,cpp}): every Render(camera) is one 1-spp path-traced frame of the Cornell box
// through the pixel centres that records a G-buffer, the joint bilateral filter and the temporal
// filter of DN/Denoiser.h, and the RGBA8 pack (DN/Renderer.cpp:101-311) -- on the MI355X (the
// megakernel's G-buffer mode + csrc/rt_denoise.hip).
// Settings keeps the reference's UI flags (DN/Renderer.h:35-60) and Render() resolves them with the
// reference's precedence (DN/Renderer.cpp:108-241); RestartTemporal() drops the history.
// In DN/mainloop.cpp the change is `Renderer renderer;` -> `rt::DenoisingRenderer renderer;`
// (INTEGRATION.md).
#ifndef RT_DENOISING_RENDERER_H
#define RT_DENOISING_RENDERER_H
#include <cstdint>
#include <memory>

#include "../rt_capi.h"
#include "Camera.h"
#include "Renderer.h"

namespace rt {

class DenoisingRenderer {
    // first member: checked against the library's layout before any other member is written (rt/Abi.h)
    AbiGuard abi_;

public:
    struct Settings {   // DN/Renderer.h:35-60
        bool immediate_clamping = true;
        bool disable_JointBilateralFiltering = true;
        bool using_JointBilateralFiltering_15 = false;
        bool using_JointBilateralFiltering_33 = false;
        bool using_JointBilateralFiltering_65 = false;
        bool disable_TemporalFiltering = true;
        bool using_temporal_kernel_7 = false;
        bool using_temporal_kernel_15 = false;
        bool using_temporal_kernel_33 = false;
        bool using_temporal_variance_tolerance_1 = false;
        bool using_temporal_variance_tolerance_2 = false;
        bool using_temporal_variance_tolerance_3 = false;
        bool using_temporal_current_frame_weighting_10 = false;
        bool using_temporal_current_frame_weighting_5 = false;
        bool using_temporal_current_frame_weighting_20 = false;
        bool using_temporal_current_frame_weighting_50 = false;
        uint64_t seed = 0;   // RNG key (frame k of the stream is the k-th Render)
        int device = 0;
    };

    DenoisingRenderer() : DenoisingRenderer(Settings{}) {}   // the Cornell box (DN/Renderer.cpp:26-58), device 0
    explicit DenoisingRenderer(const Settings& s)
        : DenoisingRenderer(AbiTag{RT_CXX_ABI_VERSION, AbiClass::DenoisingRenderer, sizeof(DenoisingRenderer), sizeof(Settings)}, s)
    {
    }
    ~DenoisingRenderer();
    DenoisingRenderer(const DenoisingRenderer&) = delete;
    DenoisingRenderer& operator=(const DenoisingRenderer&) = delete;

    void ResizeViewport(uint32_t width, uint32_t height);   // also restarts the temporal history
    void Render(const Camera& camera);                       // one denoised frame
    std::shared_ptr<Image> GetFinalImage() const { return frame_image_final; }
    void RestartTemporal();                                  // DN/Renderer.h:74-77
    Settings& GetSettings() { return settings; }
    // the filter parameters Render() derived from the settings last time (DN/Renderer.cpp:108-241)
    rt_denoise_params Resolved() const { return params; }
    uint32_t FrameIndex() const { return frame; }
    float LastFrameMilliseconds() const;                     // G-buffer frame + filters

    const float RR_survival_probability = 0.8f;              // DN/Renderer.h:226

private:
    DenoisingRenderer(const AbiTag& caller, const Settings& s);   // librt_hip.so
    void check(rt_status s, const char* what) const;
    void resolve_settings();
    Settings settings;
    rt_denoise_params params{};
    // Denoising::Denoiser's switches as Render() leaves them (they persist between frames)
    bool jbf_on = true, temporal_on = true;
    int jbf_half = 7, temporal_half = 3;
    std::shared_ptr<Image> frame_image_final;
    uint32_t frame = 0;
    rt_ctx* ctx = nullptr;
};

}  // namespace rt

#endif
