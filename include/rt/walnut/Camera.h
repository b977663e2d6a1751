// include/rt/walnut/Camera.h -- the reference's Camera for a Walnut front-end: MC/Camera.h:15-95 with its glm
// types and its Walnut::Input fly camera (MC/Camera.cpp:24-85), on top of the core rt::Camera
// (include/rt/Camera.h).  A layer written against the reference (MC/mainloop.cpp) compiles unchanged but
// for its include lines:   #include "Camera.h"  ->  #include <rt/walnut/Camera.h>
// It needs the application's <glm/glm.hpp> and "Walnut/Input/Input.h" (the Walnut/ImGui/Vulkan app shell
// is not part of this library).
#ifndef RT_WALNUT_CAMERA_H
#define RT_WALNUT_CAMERA_H
#ifndef RT_NO_GLOBAL_NAMES
#define RT_NO_GLOBAL_NAMES
#endif
#include <cstdint>
#include <vector>

#include <glm/glm.hpp>

#include "Walnut/Input/Input.h"
#include "../Camera.h"

class Camera {
public:
    Camera(float verticalFOV, float NearClipPlaneDistance, float FarClipPlaneDistance)
        : core_(verticalFOV, NearClipPlaneDistance, FarClipPlaneDistance)
    {
        sync();
    }

    // MC/Camera.cpp:24-85: recompute the view; with the right mouse button held, WASD / Space / LeftShift
    // move and the mouse displacement turns the camera; returns whether it moved
    bool UpdateCamera(float dt)
    {
        const glm::vec2 at = Walnut::Input::GetMousePosition();
        const glm::vec2 displacement = at - mouse_was_at;
        mouse_was_at = at;
        if (!Walnut::Input::IsMouseButtonDown(Walnut::MouseButton::Right)) {
            Walnut::Input::SetCursorMode(Walnut::CursorMode::Normal);
            core_.UpdateCamera(dt);
            sync();
            return false;
        }
        Walnut::Input::SetCursorMode(Walnut::CursorMode::Locked);
        rt::CameraInput in;
        in.rotating = true;
        in.forward = Walnut::Input::IsKeyDown(Walnut::KeyCode::W);
        in.back = Walnut::Input::IsKeyDown(Walnut::KeyCode::S);
        in.right = Walnut::Input::IsKeyDown(Walnut::KeyCode::D);
        in.left = Walnut::Input::IsKeyDown(Walnut::KeyCode::A);
        in.up = Walnut::Input::IsKeyDown(Walnut::KeyCode::Space);
        in.down = Walnut::Input::IsKeyDown(Walnut::KeyCode::LeftShift);
        in.mouse_dx = displacement.x;
        in.mouse_dy = displacement.y;
        const bool moved = core_.UpdateCamera(dt, in);
        sync();
        return moved;
    }
    void ResizeViewport(uint32_t new_width, uint32_t new_height)
    {
        core_.ResizeViewport(new_width, new_height);
        sync();
    }

    float Sensitivity() const { return core_.Sensitivity(); }
    const glm::vec3& Position() const { return position_; }
    const glm::vec3& ForwardDirection() const { return forward_; }
    const glm::mat4& ProjectionMatrix() const { return projection_; }
    const glm::mat4& InverseProjectionMatrix() const { return inverse_projection_; }
    const glm::mat4& ViewMatrix() const { return view_; }
    const glm::mat4& InverseViewMatrix() const { return inverse_view_; }
    // this frame's jittered directions (the kernel generates the same ones on the device)
    const std::vector<glm::vec3>& RayDirections() const
    {
        const std::vector<rt::vec3>& d = core_.RayDirections();
        directions_.resize(d.size());
        for (size_t i = 0; i < d.size(); ++i) directions_[i] = glm::vec3(d[i].x, d[i].y, d[i].z);
        return directions_;
    }

    const rt::Camera& Core() const { return core_; }   // what the core Renderer renders with

private:
    static void to_glm(const rt::mat4& m, glm::mat4& g)
    {
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 4; ++r) g[c][r] = m(c, r);
    }
    void sync()
    {
        const rt::vec3 p = core_.Position(), f = core_.ForwardDirection();
        position_ = glm::vec3(p.x, p.y, p.z);
        forward_ = glm::vec3(f.x, f.y, f.z);
        to_glm(core_.ProjectionMatrix(), projection_);
        to_glm(core_.InverseProjectionMatrix(), inverse_projection_);
        to_glm(core_.ViewMatrix(), view_);
        to_glm(core_.InverseViewMatrix(), inverse_view_);
    }

    rt::Camera core_;
    glm::vec2 mouse_was_at{0.0f, 0.0f};
    glm::vec3 position_{0.0f, 0.0f, 0.0f}, forward_{0.0f, 0.0f, 1.0f};
    glm::mat4 projection_{1.0f}, inverse_projection_{1.0f}, view_{1.0f}, inverse_view_{1.0f};
    mutable std::vector<glm::vec3> directions_;
};

#endif
