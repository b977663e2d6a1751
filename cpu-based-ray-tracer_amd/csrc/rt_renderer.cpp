// rt_renderer.cpp -- the C++20 drop-in classes (include/rt/Renderer.h, include/rt/Camera.h) on top of
// the C-ABI.  Reference: MC/Renderer.{h,cpp}, MC/Camera.{h,cpp}.
#include <cmath>
#include <cstring>
#include <string>

#include "rt/Renderer.h"
#include "rt_camera.h"
#include "rt_scene.h"

namespace rt {

// ============================================================================ layout guard (rt/Abi.h)
namespace {
const char* abi_class_name(AbiClass c)
{
    switch (c) {
    case AbiClass::Renderer: return "rt::Renderer";
    case AbiClass::Camera: return "rt::Camera";
    case AbiClass::WhittedRenderer: return "rt::WhittedRenderer";
    case AbiClass::DenoisingRenderer: return "rt::DenoisingRenderer";
    }
    return "rt class";
}
}  // namespace

AbiGuard::AbiGuard(const AbiTag& caller, uint64_t lib_size, uint64_t lib_aux_size) : version_(RT_CXX_ABI_VERSION)
{
    // runs before any other member of the caller's object is written: nothing past this member is touched
    // when it throws
    if (caller.version != RT_CXX_ABI_VERSION || caller.size != lib_size || caller.aux_size != lib_aux_size)
        throw rt::Error(std::string(abi_class_name(caller.cls)) + ": the caller was compiled against a different include/rt " +
                        "header than librt_hip.so (C++ ABI " + std::to_string(caller.version) + " vs " +
                        std::to_string(RT_CXX_ABI_VERSION) + ", sizeof " + std::to_string(caller.size) + " vs " +
                        std::to_string(lib_size) + ", Settings " + std::to_string(caller.aux_size) + " vs " +
                        std::to_string(lib_aux_size) + "); rebuild the front-end against this library's headers");
    // the C structs too: the caller's RT_API_VERSION against the library's
    if (rt_api_version() != RT_API_VERSION)
        throw rt::Error("librt_hip.so C-ABI version " + std::to_string(rt_api_version()) + ", include/rt_capi.h " +
                        std::to_string(RT_API_VERSION));
}

// ============================================================================ Camera
Camera::Camera(const AbiTag& caller, float verticalFOV, float NearClipPlaneDistance, float FarClipPlaneDistance)
    : abi_(caller, sizeof(Camera), 0), vertical_FOV{verticalFOV}, near_clip_plane_distance{NearClipPlaneDistance},
      far_clip_plane_distance{FarClipPlaneDistance}
{
}

Camera::Camera(const AbiTag& caller, float verticalFOV, float NearClipPlaneDistance, float FarClipPlaneDistance, rt::vec3 p,
               rt::vec3 f)
    : abi_(caller, sizeof(Camera), 0), position{p}, forward_direction{f}, vertical_FOV{verticalFOV},
      near_clip_plane_distance{NearClipPlaneDistance}, far_clip_plane_distance{FarClipPlaneDistance}
{
}

void Camera::SetPosition(rt::vec3 p)
{
    position = p;
    RecomputeViewMatrix();
}

void Camera::RecomputeProjectionMatrix()
{   // MC/Camera.cpp:101-105
    const float p[3] = {position.x, position.y, position.z}, f[3] = {forward_direction.x, forward_direction.y, forward_direction.z};
    rt::camera_matrices(viewport_width, viewport_height, p, f, vertical_FOV, near_clip_plane_distance, far_clip_plane_distance,
                        projection_matrix.m.data(), inverse_projection_matrix.m.data(), nullptr, nullptr);
}

void Camera::RecomputeViewMatrix()
{   // MC/Camera.cpp:107-112
    const float p[3] = {position.x, position.y, position.z}, f[3] = {forward_direction.x, forward_direction.y, forward_direction.z};
    rt::camera_matrices(viewport_width ? viewport_width : 1, viewport_height ? viewport_height : 1, p, f, vertical_FOV,
                        near_clip_plane_distance, far_clip_plane_distance, nullptr, nullptr, view_matrix.m.data(), inverse_view_matrix.m.data());
    ray_directions.clear();
}

void Camera::ResizeViewport(uint32_t new_width, uint32_t new_height)
{   // MC/Camera.cpp:87-99
    if (viewport_width == new_width && viewport_height == new_height) return;
    viewport_width = new_width;
    viewport_height = new_height;
    RecomputeProjectionMatrix();
    RecomputeViewMatrix();
}

bool Camera::UpdateCamera(float dt)
{
    rt::CameraInput none;
    return UpdateCamera(dt, none);
}

bool Camera::UpdateCamera(float dt, const rt::CameraInput& in)
{   // MC/Camera.cpp:24-85 (input from the caller instead of Walnut::Input)
    RecomputeViewMatrix();
    if (!in.rotating) return false;
    bool moved = false;
    const float speed = 5.0f;
    auto cross = [](rt::vec3 a, rt::vec3 b) { return rt::vec3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; };
    const rt::vec3 right = cross(forward_direction, up_direction);
    auto step = [&](rt::vec3 d, float s) { position.x += s * d.x; position.y += s * d.y; position.z += s * d.z; moved = true; };
    if (in.forward) step(forward_direction, speed * dt);
    if (in.back) step(forward_direction, -speed * dt);
    if (in.right) step(right, speed * dt);
    if (in.left) step(right, -speed * dt);
    if (in.up) step(up_direction, speed * dt);
    if (in.down) step(up_direction, -speed * dt);
    if (in.mouse_dx != 0.0f || in.mouse_dy != 0.0f) {
        // q = normalize(angleAxis(-pitch, right) x angleAxis(-yaw, up)); forward = rotate(q, forward)
        const float pitch = in.mouse_dy * Sensitivity(), yaw = in.mouse_dx * Sensitivity();
        const float ha = -pitch * 0.5f, hb = -yaw * 0.5f;
        const float aw = std::cos(ha), as = std::sin(ha), bw = std::cos(hb), bs = std::sin(hb);
        const float ax = right.x * as, ay = right.y * as, az = right.z * as;
        const float bx = up_direction.x * bs, by = up_direction.y * bs, bz = up_direction.z * bs;
        float qw = aw * bw - (ax * bx + ay * by + az * bz);
        float qx = aw * bx + bw * ax + (ay * bz - az * by);
        float qy = aw * by + bw * ay + (az * bx - ax * bz);
        float qz = aw * bz + bw * az + (ax * by - ay * bx);
        const float n = std::sqrt(qw * qw + qx * qx + qy * qy + qz * qz);
        qw /= n; qx /= n; qy /= n; qz /= n;
        const rt::vec3 v = forward_direction;
        const rt::vec3 qv{qx, qy, qz};
        const rt::vec3 uv = cross(qv, v), uuv = cross(qv, uv);
        forward_direction = rt::vec3{v.x + 2.0f * (uv.x * qw + uuv.x), v.y + 2.0f * (uv.y * qw + uuv.y), v.z + 2.0f * (uv.z * qw + uuv.z)};
        moved = true;
    }
    if (moved) RecomputeViewMatrix();
    return moved;
}

rt_camera Camera::Native() const
{
    rt_camera c;
    c.position[0] = position.x; c.position[1] = position.y; c.position[2] = position.z;
    std::memcpy(c.inv_projection, inverse_projection_matrix.m.data(), 64);
    std::memcpy(c.inv_view, inverse_view_matrix.m.data(), 64);
    return c;
}

namespace {
// host copy of the frozen RNG stream (the kernel's rtd::Rng): Philox4x32-10
uint32_t rng_u32(uint64_t seed, uint32_t pixel, uint32_t frame, uint32_t dim)
{
    uint32_t c0 = pixel, c1 = frame, c2 = dim >> 2, c3 = 0, k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    const uint32_t o[4] = {c0, c1, c2, c3};
    return o[dim & 3u];
}
}  // namespace

const std::vector<rt::vec3>& Camera::RayDirections(uint32_t frame, uint64_t seed) const
{   // RecomputeRayDirections, MC/Camera.cpp:114-132, for one frame of the kernel's RNG stream
    const uint32_t W = viewport_width, H = viewport_height;
    ray_directions.resize((size_t)W * H);
    const float* ip = inverse_projection_matrix.m.data();
    const float* iv = inverse_view_matrix.m.data();
    auto mul = [](const float* m, float v0, float v1, float v2, float v3, float* o) {
        for (int i = 0; i < 4; ++i) { const float a = m[i] * v0, b = m[4 + i] * v1, c = m[8 + i] * v2, d = m[12 + i] * v3; o[i] = (a + b) + (c + d); }
    };
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            const uint32_t px = y * W + x;
            const float ux = (float)rng_u32(seed, px, frame, 0) / 4294967296.0f, uy = (float)rng_u32(seed, px, frame, 1) / 4294967296.0f;
            float cx = ((float)x + ux) / (float)W, cy = ((float)y + uy) / (float)H;
            cx = cx * 2.0f - 1.0f; cy = cy * 2.0f - 1.0f;
            float t[4], w[4];
            mul(ip, cx, cy, 1.0f, 1.0f, t);
            float d[3] = {t[0] / t[3], t[1] / t[3], t[2] / t[3]};
            const float dd = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
            const float s = 1.0f / std::sqrt(dd);
            mul(iv, d[0] * s, d[1] * s, d[2] * s, 0.0f, w);
            ray_directions[px] = rt::vec3{w[0], w[1], w[2]};
        }
    return ray_directions;
}

}  // namespace rt

// ============================================================================ entities
rt::TriangleMesh::TriangleMesh(const std::string& file_path, const Material& m) : material_(m)
{
    std::string err;
    if (!rt::SceneBuilder::load_obj_positions(file_path, raw_, err)) throw rt::Error("TriangleMesh: " + err);
}

rt::TriangleMesh::TriangleMesh(std::vector<float> raw_positions, const Material& m) : raw_(std::move(raw_positions)), material_(m) {}

// ============================================================================ Renderer
namespace rt {

// the library's state behind rt::Renderer's one pointer (the caller allocates only the public members, the
// guard and this pointer)
struct Renderer::Impl {
    Settings settings;
    std::shared_ptr<rt::Image> frame_image_final;
    std::vector<float> accum_host;
    uint32_t frame_accumulating = 1;
    uint64_t epoch = 0;
    rt_ctx* ctx = nullptr;
    rt_group* group = nullptr;   // Settings::devices with more than one entry
    std::vector<std::unique_ptr<rt::Entity>> owned;   // the built-in Cornell meshes
    rt_scene* scene = nullptr;
    bool bvh_dirty = true;
    // the queries' context: ctx, or (several devices) one on the first device holding the scene
    rt_ctx* qctx = nullptr;
    bool qctx_stale = true;
    std::vector<float> tri_normal;    // per flattened slot: a triangle's face normal, a sphere's center (rt_scene_export)
    std::vector<int32_t> tri_mesh;    // per flattened slot: entity index
    std::vector<uint8_t> tri_sphere;  // per flattened slot: a sphere

    void check(rt_status s, const std::string& what) const
    {
        if (s != RT_OK)
            throw rt::Error(what + " failed (" + std::to_string(s) + "): " + (group ? rt_group_last_error(group) : rt_last_error(ctx)));
    }
    rt_ctx* query_ctx()
    {
        if (ctx) return ctx;
        if (!qctx) {
            rt_device_cfg cfg{settings.devices.empty() ? settings.device : settings.devices[0], nullptr, 0};
            check(rt_create(&qctx, &cfg), "rt_create");
            qctx_stale = true;
        }
        if (qctx_stale) {
            const rt_status st = rt_upload_scene(qctx, scene);
            if (st != RT_OK) throw rt::Error(std::string("rt_upload_scene failed: ") + rt_last_error(qctx));
            qctx_stale = false;
        }
        return qctx;
    }
    ~Impl()
    {
        rt_group_destroy(group);
        rt_destroy(ctx);
        rt_destroy(qctx);
        rt_scene_destroy(scene);
    }
};

Renderer::Renderer(const AbiTag& caller, const Settings& s, bool cornell_box)
    : abi_(caller, sizeof(Renderer), sizeof(Settings)), impl_(std::make_unique<Impl>())
{
    Impl& I = *impl_;
    I.settings = s;
    if (I.settings.devices.size() > 1) {
        I.check(rt_group_create(&I.group, I.settings.devices.data(), (uint32_t)I.settings.devices.size()), "rt_group_create");
    } else {
        rt_device_cfg cfg{I.settings.devices.empty() ? I.settings.device : I.settings.devices[0], nullptr, 0};
        I.check(rt_create(&I.ctx, &cfg), "rt_create");
    }
    if (cornell_box) {
        // Renderer::Renderer(): materials + six meshes + GenerateBVH (MC/Renderer.cpp:26-57)
        for (auto& m : rt::SceneBuilder::cornell_box_meshes()) {
            rt::Material mat;
            mat.diffuse_coefficient = rt::vec3{m.material.albedo.x, m.material.albedo.y, m.material.albedo.z};
            mat.emission = rt::vec3{m.material.emission.x, m.material.emission.y, m.material.emission.z};
            I.owned.push_back(std::make_unique<rt::TriangleMesh>(std::move(m.raw), mat));
            Add(I.owned.back().get());
        }
        GenerateBVH();
    }
}

Renderer::~Renderer() = default;

std::shared_ptr<rt::Image> Renderer::GetFinalImage() const { return impl_->frame_image_final; }
void Renderer::Reaccumulate() { impl_->frame_accumulating = 1; ++impl_->epoch; }
uint32_t Renderer::GetSPP() { return impl_->frame_accumulating - 1; }
Renderer::Settings& Renderer::GetSettings() { return impl_->settings; }
const rt_scene* Renderer::Scene() const { return impl_->scene; }

void Renderer::GenerateBVH()
{
    Impl& I = *impl_;
    rt_scene* sc = nullptr;
    I.check(rt_scene_create(&sc), "rt_scene_create");
    for (size_t k = 0; k < entities.size(); ++k) {
        rt::Entity* e = entities[k];
        const rt::Material& m = e->GetMaterial();
        const float alb[3] = {m.diffuse_coefficient.x, m.diffuse_coefficient.y, m.diffuse_coefficient.z};
        const float em[3] = {m.emission.x, m.emission.y, m.emission.z};
        vec3 c{};
        float r = 0.0f;
        rt_status st;
        if (e->SphereShape(c, r)) {   // Whitted::Sphere (MC/Sphere.h:16-108)
            const float cc[3] = {c.x, c.y, c.z};
            st = rt_scene_add_sphere(sc, cc, r, alb, em, nullptr);
        } else {
            const auto& raw = e->RawPositions();
            if (raw.size() < 9) {
                rt_scene_destroy(sc);
                throw rt::Error("GenerateBVH: entity " + std::to_string(k) + " is neither a triangle mesh nor a sphere: a "
                                "user-defined shape has no device form (the path kernels intersect triangles and spheres)");
            }
            st = rt_scene_add_mesh(sc, raw.data(), raw.size() / 9, alb, em, nullptr);
        }
        if (st != RT_OK) { rt_scene_destroy(sc); I.check(st, "GenerateBVH (entity " + std::to_string(k) + ")"); }
    }
    rt_status st = rt_scene_build(sc);
    if (st == RT_OK) st = I.group ? rt_group_upload_scene(I.group, sc) : rt_upload_scene(I.ctx, sc);
    if (st != RT_OK) { rt_scene_destroy(sc); I.check(st, "GenerateBVH"); }
    rt_scene_destroy(I.scene);
    I.scene = sc;   // kept for Scene()
    I.bvh_dirty = false;
    I.qctx_stale = true;
    // the per-triangle records the queries return (face normal, mesh)
    rt_scene_info info{};
    I.check(rt_scene_get_info(sc, &info), "rt_scene_get_info");
    std::vector<float> nf((size_t)info.n_nodes * 7), tf((size_t)info.n_tris * 13);
    std::vector<int32_t> ni((size_t)info.n_nodes * 5), ti((size_t)info.n_tris * 2);
    I.check(rt_scene_export(sc, nf.data(), ni.data(), tf.data(), ti.data()), "rt_scene_export");
    I.tri_normal.resize((size_t)info.n_tris * 3);
    I.tri_mesh.resize(info.n_tris);
    I.tri_sphere.resize(info.n_tris);
    for (size_t i = 0; i < info.n_tris; ++i) {
        I.tri_sphere[i] = ti[2 * i + 1] == -2 ? 1 : 0;   // a sphere's slot: tri_f a = its center (rt_capi.h)
        for (int k = 0; k < 3; ++k) I.tri_normal[3 * i + k] = tf[13 * i + (I.tri_sphere[i] ? 0 : 9) + k];
        I.tri_mesh[i] = ti[2 * i];
    }
}

Renderer::Hit Renderer::Trace(const vec3& origin, const vec3& direction) const
{
    Impl& I = *impl_;
    if (I.bvh_dirty || !I.scene) throw rt::Error("ray_BVH_intersection_record before GenerateBVH");
    rt_ctx* q = I.query_ctx();
    const float o[3] = {origin.x, origin.y, origin.z}, d[3] = {direction.x, direction.y, direction.z};
    int32_t tri = -1;
    double t = 0.0;
    const rt_status st = rt_trace(q, 1, o, d, &tri, &t);
    if (st != RT_OK) throw rt::Error(std::string("rt_trace failed: ") + rt_last_error(q));
    Hit h;
    if (tri >= 0 && (size_t)tri < I.tri_mesh.size()) {
        h.hit = true; h.t = t; h.triangle = tri; h.mesh = I.tri_mesh[tri];
        const float* q = &I.tri_normal[3 * (size_t)tri];
        if (I.tri_sphere[tri]) {
            // Sphere::GetIntersectionRecord (MC/Sphere.h:92-94): location = ray((float)t), normal =
            // Whitted::normalize(location - center) (MC/VectorFloat.h:22-31), in float as the reference
            const float tf32 = (float)t;
            const float lx = origin.x + tf32 * direction.x, ly = origin.y + tf32 * direction.y, lz = origin.z + tf32 * direction.z;
            const float vx = lx - q[0], vy = ly - q[1], vz = lz - q[2];
            const float l2 = vx * vx + vy * vy + vz * vz;
            if (l2 > 0) { const float inv = 1 / std::sqrt(l2); h.normal = vec3{vx * inv, vy * inv, vz * inv}; }
            else h.normal = vec3{vx, vy, vz};
        } else {
            h.normal = vec3{q[0], q[1], q[2]};
        }
    }
    return h;
}

Renderer::LightSample Renderer::SampleLight(const uint32_t draws[3]) const
{
    Impl& I = *impl_;
    if (I.bvh_dirty || !I.scene) throw rt::Error("SamplingAreaLight before GenerateBVH");
    rt_ctx* q = I.query_ctx();
    float loc[3], n[3], em[3], pdf = 0.0f;
    const rt_status st = rt_sample_light(q, 1, draws, loc, n, em, &pdf);
    if (st != RT_OK) throw rt::Error(std::string("rt_sample_light failed: ") + rt_last_error(q));
    return LightSample{vec3{loc[0], loc[1], loc[2]}, vec3{n[0], n[1], n[2]}, vec3{em[0], em[1], em[2]}, pdf};
}

void Renderer::ResizeViewport(uint32_t width, uint32_t height)
{   // MC/Renderer.cpp:59-89
    Impl& I = *impl_;
    if (I.frame_image_final) {
        if (I.frame_image_final->GetWidth() == width && I.frame_image_final->GetHeight() == height) return;
        I.frame_image_final->Resize(width, height);
    } else {
        I.frame_image_final = std::make_shared<rt::Image>(width, height);
    }
    if (I.group) I.check(rt_group_resize(I.group, width, height, I.settings.band), "rt_group_resize");
    else I.check(rt_resize(I.ctx, width, height, 8, 0, 1), "rt_resize");
    I.frame_accumulating = 1;
}

void Renderer::Render(const Camera& camera) { RenderFrames(camera, 1); }

void Renderer::RenderFrames(const Camera& camera, uint32_t n)
{   // MC/Renderer.cpp:91-122, n frames per launch
    Impl& I = *impl_;
    if (!I.frame_image_final) throw rt::Error("Render before ResizeViewport");
    if (I.bvh_dirty) GenerateBVH();
    const rt_camera cam = camera.Native();
    if (!I.settings.accumulating) {
        // every frame restarts the average (frame_accumulating stays 1, MC/Renderer.cpp:95-98,114-121),
        // so only the last of n frames is visible: render that one, on a fresh RNG epoch so
        // successive frames carry fresh noise like the reference's free-running mt19937
        if (n == 0) return;
        ++I.epoch;
        n = 1;
    }
    rt_render_params p{I.frame_accumulating, n, I.settings.seed + I.epoch, RR_survival_probability, I.settings.exact ? RT_RENDER_EXACT : 0u};
    if (I.group) I.check(rt_group_render(I.group, &cam, &p, I.frame_image_final->Data()), "rt_group_render");
    else I.check(rt_render(I.ctx, &cam, &p, I.frame_image_final->Data(), nullptr), "rt_render");
    if (I.settings.accumulating) I.frame_accumulating += n;
    else I.frame_accumulating = 1;
}

const std::vector<float>& Renderer::GetAccumulation()
{
    Impl& I = *impl_;
    const size_t n = I.frame_image_final ? (size_t)I.frame_image_final->GetWidth() * I.frame_image_final->GetHeight() * 4 : 0;
    I.accum_host.resize(n);
    if (n) {
        if (I.group) I.check(rt_group_read_accumulation(I.group, I.accum_host.data()), "rt_group_read_accumulation");
        else I.check(rt_read_accumulation(I.ctx, I.accum_host.data()), "rt_read_accumulation");
    }
    return I.accum_host;
}

float Renderer::LastKernelMilliseconds() const
{
    const Impl& I = *impl_;
    if (I.group) {   // the slowest member's band render
        rt_group_stats gs{};
        if (rt_group_get_stats(I.group, &gs) != RT_OK) return -1.0f;
        return gs.max_member_kernel_ms;
    }
    rt_stats st{};
    if (rt_get_stats(I.ctx, &st) != RT_OK) return -1.0f;
    return st.last_kernel_ms;
}

}  // namespace rt

// ============================================================================ WhittedRenderer
#include "rt/WhittedRenderer.h"
#include "rt/DenoisingRenderer.h"

namespace rt {

void WhittedRenderer::check(rt_status s, const char* what) const
{
    if (s != RT_OK) throw Error(std::string(what) + " failed (" + std::to_string(s) + "): " + rt_last_error(ctx));
}

WhittedRenderer::WhittedRenderer(const AbiTag& caller, rt_scene* built_scene, const Settings& s)
    : abi_(caller, sizeof(WhittedRenderer), sizeof(Settings)), settings(s)
{
    rt_device_cfg cfg{settings.device, nullptr, 0};
    check(rt_create(&ctx, &cfg), "rt_create");
    check(rt_upload_scene(ctx, built_scene), "rt_upload_scene");
}

WhittedRenderer::~WhittedRenderer() { rt_destroy(ctx); }

namespace {
struct SceneGuard {
    rt_scene* s = nullptr;
    ~SceneGuard() { rt_scene_destroy(s); }
};
}  // namespace

std::unique_ptr<WhittedRenderer> WhittedRenderer::TwoSpheres(const Settings& s)
{   // Renderer::Renderer(), WH/Renderer.cpp:27-49
    SceneGuard g;
    if (rt_scene_create(&g.s) != RT_OK || rt_scene_add_two_spheres_scene(g.s) != RT_OK || rt_scene_build(g.s) != RT_OK)
        throw Error("TwoSpheres: scene build failed");
    return std::make_unique<WhittedRenderer>(g.s, s);
}

std::unique_ptr<WhittedRenderer> WhittedRenderer::BVHRayTracer(const std::string& bunny_obj, const std::string& teapot_obj, const Settings& s)
{   // Renderer::Renderer(), BV/Renderer.cpp:26-43
    SceneGuard g;
    if (rt_scene_create(&g.s) != RT_OK) throw Error("BVHRayTracer: rt_scene_create failed");
    if (rt_scene_add_bvh_tracer_scene(g.s, bunny_obj.c_str(), teapot_obj.c_str()) != RT_OK) throw Error("BVHRayTracer: cannot load the OBJ files");
    if (rt_scene_build(g.s) != RT_OK) throw Error("BVHRayTracer: scene build failed");
    return std::make_unique<WhittedRenderer>(g.s, s);
}

void WhittedRenderer::ResizeViewport(uint32_t width, uint32_t height)
{   // BV/Renderer.cpp:45-67, WH/Renderer.cpp:51-80
    if (frame_image_final) {
        if (frame_image_final->GetWidth() == width && frame_image_final->GetHeight() == height) return;
        frame_image_final->Resize(width, height);
    } else {
        frame_image_final = std::make_shared<Image>(width, height);
    }
    check(rt_resize(ctx, width, height, 8, 0, 1), "rt_resize");
    frame_accumulating = 1;
}

void WhittedRenderer::Render(const Camera& camera) { RenderFrames(camera, 1); }

void WhittedRenderer::RenderFrames(const Camera& camera, uint32_t n)
{   // Render + RayGen_Shader: every frame is the same deterministic image, accumulated in order
    if (!frame_image_final) throw Error("Render before ResizeViewport");
    if (!settings.accumulating && n > 1) n = 1;
    const rt_camera cam = camera.Native();
    rt_render_params p{frame_accumulating, n, 0, 0.0f, RT_RENDER_WHITTED};
    check(rt_render(ctx, &cam, &p, frame_image_final->Data(), nullptr), "rt_render");
    if (settings.accumulating) frame_accumulating += n;
    else frame_accumulating = 1;
}

float WhittedRenderer::LastKernelMilliseconds() const
{
    rt_stats st{};
    if (rt_get_stats(ctx, &st) != RT_OK) return -1.0f;
    return st.last_kernel_ms;
}

// ============================================================================ DenoisingRenderer
void DenoisingRenderer::check(rt_status s, const char* what) const
{
    if (s != RT_OK) throw Error(std::string(what) + " failed (" + std::to_string(s) + "): " + rt_last_error(ctx));
}

DenoisingRenderer::DenoisingRenderer(const AbiTag& caller, const Settings& s)
    : abi_(caller, sizeof(DenoisingRenderer), sizeof(Settings)), settings(s)
{
    rt_denoise_params_default(&params);   // Denoising::Denoiser's member defaults (DN/Denoiser.h:333-358)
    rt_device_cfg cfg{settings.device, nullptr, 0};
    check(rt_create(&ctx, &cfg), "rt_create");
    SceneGuard g;
    check(rt_scene_create(&g.s), "rt_scene_create");
    check(rt_scene_add_cornell_box(g.s), "rt_scene_add_cornell_box");   // DN/Renderer.cpp:26-58
    check(rt_scene_build(g.s), "rt_scene_build");
    check(rt_upload_scene(ctx, g.s), "rt_upload_scene");
}

DenoisingRenderer::~DenoisingRenderer() { rt_destroy(ctx); }

void DenoisingRenderer::ResizeViewport(uint32_t width, uint32_t height)
{   // DN/Renderer.cpp:60-99 (denoiser.Resize drops the history)
    if (frame_image_final) {
        if (frame_image_final->GetWidth() == width && frame_image_final->GetHeight() == height) return;
        frame_image_final->Resize(width, height);
    } else {
        frame_image_final = std::make_shared<Image>(width, height);
    }
    check(rt_resize(ctx, width, height, 8, 0, 1), "rt_resize");
    RestartTemporal();
}

void DenoisingRenderer::RestartTemporal() { check(rt_denoise_restart(ctx), "rt_denoise_restart"); }

void DenoisingRenderer::resolve_settings()
{   // Renderer::Render's settings -> denoiser members, DN/Renderer.cpp:108-241 (the members persist)
    Settings& s = settings;   // (the reference's `settings.disable_JointBilateralFiltering == false;` lines have no effect)
    if (s.disable_JointBilateralFiltering) {
        jbf_on = false;
        s.using_JointBilateralFiltering_15 = s.using_JointBilateralFiltering_33 = s.using_JointBilateralFiltering_65 = false;
    } else if (s.using_JointBilateralFiltering_15) {
        jbf_on = true; jbf_half = 3;
        s.using_JointBilateralFiltering_33 = s.using_JointBilateralFiltering_65 = false;
    } else if (s.using_JointBilateralFiltering_33) {
        jbf_on = true; jbf_half = 16;
        s.using_JointBilateralFiltering_15 = s.using_JointBilateralFiltering_65 = false;
    } else if (s.using_JointBilateralFiltering_65) {
        jbf_on = true; jbf_half = 32;
        s.using_JointBilateralFiltering_15 = s.using_JointBilateralFiltering_33 = false;
    }
    if (s.disable_TemporalFiltering) {
        temporal_on = false;
        s.using_temporal_kernel_7 = s.using_temporal_kernel_15 = s.using_temporal_kernel_33 = false;
        s.using_temporal_variance_tolerance_1 = s.using_temporal_variance_tolerance_2 = s.using_temporal_variance_tolerance_3 = false;
        s.using_temporal_current_frame_weighting_10 = s.using_temporal_current_frame_weighting_5 = false;
        s.using_temporal_current_frame_weighting_20 = false;
    } else {
        if (s.using_temporal_kernel_7) { temporal_on = true; temporal_half = 3; s.using_temporal_kernel_15 = s.using_temporal_kernel_33 = false; }
        else if (s.using_temporal_kernel_15) { temporal_on = true; temporal_half = 7; s.using_temporal_kernel_7 = s.using_temporal_kernel_33 = false; }
        else if (s.using_temporal_kernel_33) { temporal_on = true; temporal_half = 16; s.using_temporal_kernel_15 = s.using_temporal_kernel_7 = false; }
        if (s.using_temporal_variance_tolerance_1) { temporal_on = true; params.tolerance = 1.0f; s.using_temporal_variance_tolerance_2 = s.using_temporal_variance_tolerance_3 = false; }
        else if (s.using_temporal_variance_tolerance_2) { temporal_on = true; params.tolerance = 2.0f; s.using_temporal_variance_tolerance_1 = s.using_temporal_variance_tolerance_3 = false; }
        else if (s.using_temporal_variance_tolerance_3) { temporal_on = true; params.tolerance = 3.0f; s.using_temporal_variance_tolerance_2 = s.using_temporal_variance_tolerance_1 = false; }
        if (s.using_temporal_current_frame_weighting_5) {
            temporal_on = true; params.current_frame_weighting = 0.05f;
            s.using_temporal_current_frame_weighting_10 = s.using_temporal_current_frame_weighting_20 = s.using_temporal_current_frame_weighting_50 = false;
        } else if (s.using_temporal_current_frame_weighting_10) {
            temporal_on = true; params.current_frame_weighting = 0.1f;
            s.using_temporal_current_frame_weighting_5 = s.using_temporal_current_frame_weighting_20 = s.using_temporal_current_frame_weighting_50 = false;
        } else if (s.using_temporal_current_frame_weighting_20) {
            temporal_on = true; params.current_frame_weighting = 0.2f;
            s.using_temporal_current_frame_weighting_10 = s.using_temporal_current_frame_weighting_5 = s.using_temporal_current_frame_weighting_50 = false;
        } else if (s.using_temporal_current_frame_weighting_50) {
            temporal_on = true; params.current_frame_weighting = 0.5f;
            s.using_temporal_current_frame_weighting_10 = s.using_temporal_current_frame_weighting_20 = s.using_temporal_current_frame_weighting_5 = false;
        }
    }
    params.jbf_half_size = jbf_on ? jbf_half : 0;
    params.temporal_half_size = temporal_on ? temporal_half : 0;
    params.immediate_clamp = s.immediate_clamping ? 1 : 0;
}

void DenoisingRenderer::Render(const Camera& camera)
{   // Renderer::Render, DN/Renderer.cpp:101-283
    if (!frame_image_final) throw Error("Render before ResizeViewport");
    resolve_settings();
    ++frame;
    const rt_camera cam = camera.Native();
    check(rt_render_denoised(ctx, &cam, camera.ProjectionMatrix().data(), camera.ViewMatrix().data(), frame, settings.seed,
                             RR_survival_probability, &params, frame_image_final->Data(), nullptr),
          "rt_render_denoised");
}

float DenoisingRenderer::LastFrameMilliseconds() const
{
    rt_stats st{};
    if (rt_get_stats(ctx, &st) != RT_OK) return -1.0f;
    return st.last_kernel_ms + st.last_denoise_ms;
}

}  // namespace rt
