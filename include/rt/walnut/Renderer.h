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
#include <cstdint>
#include <memory>
#include <vector>

#include "Walnut/Image.h"
#include "Camera.h"
#include "Whitted.h"   // Whitted::TriangleMesh / WhittedMaterial / Entity, as MC/Renderer.h brings them
#include "../Renderer.h"

class Renderer {
public:
    using Settings = rt::Renderer::Settings;   // Settings::accumulating, MC/Renderer.h:34-37

    Renderer() = default;   // the Cornell box (MC/Renderer.cpp:26-57)

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
    // the scene-extension API, MC/Renderer.h:72-86: Add(new Whitted::TriangleMesh(path, material)) then GenerateBVH()
    [[nodiscard]] const std::vector<Whitted::Entity*>& GetEntities() const { return core_.GetEntities(); }
    void Add(Whitted::Entity* entity_pointer) { core_.Add(entity_pointer); }
    void GenerateBVH() { core_.GenerateBVH(); }

    float RR_survival_probability = 0.8f;   // MC/Renderer.h:199 (read at every Render)

    rt::Renderer& Core() { return core_; }

private:
    rt::Renderer core_;
    std::shared_ptr<Walnut::Image> frame_image_final;
};

#endif
