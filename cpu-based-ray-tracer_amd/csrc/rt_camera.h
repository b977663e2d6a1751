// rt_camera.h -- host camera math shared by the C-ABI and the C++ Camera (rt_camera.cpp).
#ifndef RT_CAMERA_INTERNAL_H
#define RT_CAMERA_INTERNAL_H
namespace rt {
// glm::perspectiveFov(radians(vfov_deg), W, H, near, far) and glm::lookAt(pos, pos+fwd, +y) with
// their glm::inverse; all column-major, 16 floats each (any pointer may be null)
void camera_matrices(unsigned W, unsigned H, const float pos[3], const float fwd[3], float vfov_deg, float zn, float zf,
                     float* proj, float* iproj, float* view, float* iview);
}
#endif
