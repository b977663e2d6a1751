// rt_camera.cpp -- host camera math of the reference Camera (MC/Camera.cpp:87-112), restated on glm
// 0.9.9.9's operation order so the matrices are bit-identical to the reference's:
//   glm::perspectiveFovRH_NO  GLM/ext/matrix_clip_space.inl:372-389
//   glm::lookAtRH             GLM/ext/matrix_transform.inl:99-119
//   glm::inverse (mat4)       GLM/detail/func_matrix.inl:347-405
//   glm::radians              GLM/detail/func_trigonometric.inl:9-14
// Checked against tests/golden/camera.npz (matrices of the reference Camera at 8 viewport sizes).
#include <cmath>
#include <cstring>

#include "rt_camera.h"
#include "rt_capi.h"

namespace {

struct M4 { float m[4][4]; };   // m[column][row]
struct F3 { float x, y, z; };
inline F3 sub(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 add(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float dot(F3 a, F3 b) { float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z; return (tx + ty) + tz; }
inline F3 cross(F3 x, F3 y) { return F3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
inline F3 normalize(F3 v) { float s = 1.0f / std::sqrt(dot(v, v)); return F3{v.x * s, v.y * s, v.z * s}; }

M4 perspective_fov(float fov, float width, float height, float zn, float zf)
{
    const float h = std::cos(0.5f * fov) / std::sin(0.5f * fov);
    const float w = h * height / width;
    M4 R;
    std::memset(&R, 0, sizeof R);
    R.m[0][0] = w;
    R.m[1][1] = h;
    R.m[2][2] = -(zf + zn) / (zf - zn);
    R.m[2][3] = -1.0f;
    R.m[3][2] = -(2.0f * zf * zn) / (zf - zn);
    return R;
}

M4 look_at(F3 eye, F3 center, F3 up)
{
    const F3 f = normalize(sub(center, eye));
    const F3 s = normalize(cross(f, up));
    const F3 u = cross(s, f);
    M4 R;
    std::memset(&R, 0, sizeof R);
    R.m[0][0] = R.m[1][1] = R.m[2][2] = R.m[3][3] = 1.0f;
    R.m[0][0] = s.x; R.m[1][0] = s.y; R.m[2][0] = s.z;
    R.m[0][1] = u.x; R.m[1][1] = u.y; R.m[2][1] = u.z;
    R.m[0][2] = -f.x; R.m[1][2] = -f.y; R.m[2][2] = -f.z;
    R.m[3][0] = -dot(s, eye);
    R.m[3][1] = -dot(u, eye);
    R.m[3][2] = dot(f, eye);
    return R;
}

M4 inverse(const M4& M)
{
    auto m = [&](int c, int r) { return M.m[c][r]; };
    const float c00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3), c02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3), c03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3);
    const float c04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3), c06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3), c07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    const float c08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2), c10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2), c11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2);
    const float c12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3), c14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3), c15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    const float c16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2), c18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2), c19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2);
    const float c20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1), c22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1), c23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    const float fac[6][4] = {{c00, c00, c02, c03}, {c04, c04, c06, c07}, {c08, c08, c10, c11},
                             {c12, c12, c14, c15}, {c16, c16, c18, c19}, {c20, c20, c22, c23}};
    const float vec[4][4] = {{m(1, 0), m(0, 0), m(0, 0), m(0, 0)}, {m(1, 1), m(0, 1), m(0, 1), m(0, 1)},
                             {m(1, 2), m(0, 2), m(0, 2), m(0, 2)}, {m(1, 3), m(0, 3), m(0, 3), m(0, 3)}};
    const float sa[4] = {+1, -1, +1, -1}, sb[4] = {-1, +1, -1, +1};
    M4 inv;
    for (int i = 0; i < 4; ++i) {
        const float i0 = (vec[1][i] * fac[0][i] - vec[2][i] * fac[1][i]) + vec[3][i] * fac[2][i];
        const float i1 = (vec[0][i] * fac[0][i] - vec[2][i] * fac[3][i]) + vec[3][i] * fac[4][i];
        const float i2 = (vec[0][i] * fac[1][i] - vec[1][i] * fac[3][i]) + vec[3][i] * fac[5][i];
        const float i3 = (vec[0][i] * fac[2][i] - vec[1][i] * fac[4][i]) + vec[2][i] * fac[5][i];
        inv.m[0][i] = i0 * sa[i]; inv.m[1][i] = i1 * sb[i]; inv.m[2][i] = i2 * sa[i]; inv.m[3][i] = i3 * sb[i];
    }
    const float d0 = M.m[0][0] * inv.m[0][0], d1 = M.m[0][1] * inv.m[1][0], d2 = M.m[0][2] * inv.m[2][0], d3 = M.m[0][3] * inv.m[3][0];
    const float det = (d0 + d1) + (d2 + d3);
    const float ood = 1.0f / det;
    M4 R;
    for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) R.m[c][r] = inv.m[c][r] * ood;
    return R;
}

void store(const M4& M, float* out) { for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) out[4 * c + r] = M.m[c][r]; }

}  // namespace

namespace rt {
void camera_matrices(unsigned W, unsigned H, const float position[3], const float forward[3], float vfov_deg, float zn, float zf,
                     float* proj, float* iproj, float* view, float* iview)
{
    const F3 pos{position[0], position[1], position[2]}, fwd{forward[0], forward[1], forward[2]};
    const float fov = vfov_deg * (float)0.01745329251994329576923690768489;   // glm::radians
    const M4 P = perspective_fov(fov, (float)W, (float)H, zn, zf);
    const M4 V = look_at(pos, add(pos, fwd), F3{0.0f, 1.0f, 0.0f});
    if (proj) store(P, proj);
    if (iproj) store(inverse(P), iproj);
    if (view) store(V, view);
    if (iview) store(inverse(V), iview);
}
}  // namespace rt

extern "C" rt_status rt_camera_look(uint32_t W, uint32_t H, const float position[3], const float forward[3], float vfov_deg, float zn, float zf,
                                    rt_camera* out)
{
    if (!out || !position || !forward || W == 0 || H == 0) return RT_ERR_INVALID;
    const F3 pos{position[0], position[1], position[2]}, fwd{forward[0], forward[1], forward[2]};
    const float fov = vfov_deg * (float)0.01745329251994329576923690768489;   // glm::radians
    const M4 proj = perspective_fov(fov, (float)W, (float)H, zn, zf);
    const M4 view = look_at(pos, add(pos, fwd), F3{0.0f, 1.0f, 0.0f});
    std::memcpy(out->position, position, 3 * sizeof(float));
    store(inverse(proj), out->inv_projection);
    store(inverse(view), out->inv_view);
    return RT_OK;
}

extern "C" rt_status rt_camera_look_ex(uint32_t W, uint32_t H, const float position[3], const float forward[3], float vfov_deg, float zn,
                                       float zf, rt_camera* out, float* proj_out, float* view_out)
{
    rt_status s = rt_camera_look(W, H, position, forward, vfov_deg, zn, zf, out);
    if (s != RT_OK) return s;
    const F3 pos{position[0], position[1], position[2]}, fwd{forward[0], forward[1], forward[2]};
    if (proj_out) store(perspective_fov(vfov_deg * (float)0.01745329251994329576923690768489, (float)W, (float)H, zn, zf), proj_out);
    if (view_out) store(look_at(pos, add(pos, fwd), F3{0.0f, 1.0f, 0.0f}), view_out);
    return RT_OK;
}

extern "C" rt_status rt_camera_default(uint32_t W, uint32_t H, rt_camera* out, float* proj_out, float* view_out)
{
    // Camera member defaults, MC/Camera.h:19-21 (double literals narrowed to float), Camera{35, 0.1, 100}
    const float pos[3] = {(float)2.81432, (float)4.20749, (float)-9.11751};
    const float fwd[3] = {(float)0.00209191, (float)-0.148299, (float)0.988941};
    rt_status s = rt_camera_look(W, H, pos, fwd, 35.0f, 0.1f, 100.0f, out);
    if (s != RT_OK) return s;
    if (proj_out) store(perspective_fov(35.0f * (float)0.01745329251994329576923690768489, (float)W, (float)H, 0.1f, 100.0f), proj_out);
    if (view_out) {
        const F3 p{pos[0], pos[1], pos[2]}, f{fwd[0], fwd[1], fwd[2]};
        store(look_at(p, add(p, f), F3{0.0f, 1.0f, 0.0f}), view_out);
    }
    return RT_OK;
}
