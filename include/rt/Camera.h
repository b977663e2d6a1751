// include/rt/Camera.h -- drop-in for the reference Camera (Monte Carlo Path Tracer/8599RayTracerGUI/src/Camera.h:15-95).
//
// Same constructor, same defaults (position, forward, up, near/far), same ResizeViewport /
// UpdateCamera / getter surface.  Differences, by design (DESIGN.md "Boundary"):
//   * no glm dependency: vectors/matrices are rt::vec3 / rt::mat4 (column-major, glm layout;
//     glm::make_mat4(m.data()) converts);
//   * per-pixel jittered ray directions are generated on the GPU inside the render kernel from
//     (position, inverse projection, inverse view) and the frame's RNG stream, instead of the
//     serial host loop of RecomputeRayDirections (MC/Camera.cpp:114-132); RayDirections() still
//     returns them, computed on the host for the current frame when asked;
//   * UpdateCamera takes its movement from an rt::CameraInput instead of Walnut::Input.
#ifndef RT_CAMERA_H
#define RT_CAMERA_H
#include <array>
#include <cstdint>
#include <vector>

#include "../rt_capi.h"
#include "Abi.h"

namespace rt {

struct vec3 { float x = 0, y = 0, z = 0; };
struct mat4 {
    std::array<float, 16> m{};   // column-major
    const float* data() const { return m.data(); }
    float operator()(int col, int row) const { return m[4 * col + row]; }
};

struct CameraInput {   // what Walnut::Input provided (MC/Camera.cpp:32-80)
    bool forward = false, back = false, left = false, right = false, up = false, down = false;
    bool rotating = false;        // right mouse button held
    float mouse_dx = 0, mouse_dy = 0;
};

class Camera {
    // first member: checked against the library's layout before any other member is written (rt/Abi.h)
    AbiGuard abi_;

public:
    Camera(float verticalFOV, float NearClipPlaneDistance, float FarClipPlaneDistance)
        : Camera(AbiTag{RT_CXX_ABI_VERSION, AbiClass::Camera, sizeof(Camera), 0}, verticalFOV, NearClipPlaneDistance,
                 FarClipPlaneDistance)
    {
    }
    // the other projects' cameras differ only in their member defaults: the BVH Ray Tracer at
    // (-1, 5, 10) and the Whitted Style Ray Tracer at (0, 0, 6), both looking down -z
    // (BV/Camera.h:19-20, WH/Camera.h:17-19)
    Camera(float verticalFOV, float NearClipPlaneDistance, float FarClipPlaneDistance, rt::vec3 position, rt::vec3 forward)
        : Camera(AbiTag{RT_CXX_ABI_VERSION, AbiClass::Camera, sizeof(Camera), 0}, verticalFOV, NearClipPlaneDistance,
                 FarClipPlaneDistance, position, forward)
    {
    }
    // what a UpdateCamera key press does to the position (e.g. a scripted camera path); recomputes the view
    void SetPosition(rt::vec3 p);

    bool UpdateCamera(float dt);                                  // no input: recompute, never moves
    bool UpdateCamera(float dt, const rt::CameraInput& input);    // WASD/space/shift + mouse look
    void ResizeViewport(uint32_t new_width, uint32_t new_height);

    float Sensitivity() const { return 0.0006f; }
    const rt::vec3& Position() const { return position; }
    const rt::vec3& ForwardDirection() const { return forward_direction; }
    const rt::mat4& ProjectionMatrix() const { return projection_matrix; }
    const rt::mat4& InverseProjectionMatrix() const { return inverse_projection_matrix; }
    const rt::mat4& ViewMatrix() const { return view_matrix; }
    const rt::mat4& InverseViewMatrix() const { return inverse_view_matrix; }
    // host-side directions of frame `frame` under `seed` (the kernel computes the same values)
    const std::vector<rt::vec3>& RayDirections(uint32_t frame = 1, uint64_t seed = 0) const;

    uint32_t ViewportWidth() const { return viewport_width; }
    uint32_t ViewportHeight() const { return viewport_height; }
    // the C-ABI view of this camera
    rt_camera Native() const;

private:
    // librt_hip.so
    Camera(const AbiTag& caller, float verticalFOV, float NearClipPlaneDistance, float FarClipPlaneDistance);
    Camera(const AbiTag& caller, float verticalFOV, float NearClipPlaneDistance, float FarClipPlaneDistance, rt::vec3 position,
           rt::vec3 forward);
    void RecomputeProjectionMatrix();
    void RecomputeViewMatrix();

    rt::vec3 position{(float)2.81432, (float)4.20749, (float)-9.11751};   // MC/Camera.h:19-21
    rt::vec3 forward_direction{(float)0.00209191, (float)-0.148299, (float)0.988941};
    rt::vec3 up_direction{0.0f, 1.0f, 0.0f};
    uint32_t viewport_width = 0, viewport_height = 0;
    rt::mat4 projection_matrix, inverse_projection_matrix, view_matrix, inverse_view_matrix;
    float vertical_FOV = 45.0f;
    float near_clip_plane_distance = 0.1f;
    float far_clip_plane_distance = 100.0f;
    mutable std::vector<rt::vec3> ray_directions;
};

}  // namespace rt

// The reference's global name (MC/Camera.h:15).  A Walnut front-end includes rt/walnut/Camera.h instead,
// whose global Camera speaks glm and Walnut::Input (it defines RT_NO_GLOBAL_NAMES).
#ifndef RT_NO_GLOBAL_NAMES
using Camera = rt::Camera;
#endif

#endif
