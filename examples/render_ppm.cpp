// examples/render_ppm.cpp -- headless front-end on the drop-in Renderer/Camera (include/rt/).
//
// What the Walnut layer does per frame (MC/mainloop.cpp:139-148: ResizeViewport x2 + Render),
// without a window: renders the reference Cornell box for `spp` frames and writes the image.
//   walnut mode (default): the RGBA8 frame (ABGR u32, row 0 = bottom, MC/Renderer.cpp:15-23,133)
//                          as a binary P6 PPM, rows flipped to top-down like ImGui::Image's uv flip
//                          (MC/mainloop.cpp:58-62)
//   --offline G:           the offline prototype's writer instead: P3 ASCII, per channel
//                          round_half_away(255 * clamp(pow(sum / spp, 1/G), 0, 1)) from the
//                          accumulation (offline prototype color.h:33-51)
//
//   rt_render_ppm W H SPP out.ppm [--seed S] [--rr P] [--fast] [--per-frame] [--offline G] [--obj FILE R G B]...
//                 [--devices 0,1,...] [--band ROWS]
//   --devices: one frame on several GPUs (Renderer::Settings::devices -> rt_group_*: row bands per
//              device, RGBA8 gathered to the first with RCCL); a device may repeat (bands on one GPU)
//
// The reference's other projects, through their drop-ins (include/rt/WhittedRenderer.h,
// include/rt/DenoisingRenderer.h); SPP = frames:
//   --project spheres                 Whitted Style Ray Tracer (two spheres, chessboard)
//   --project bvh BUNNY.obj TEAPOT.obj  BVH Ray Tracer (bunny + teapot)
//   --project denoiser [--jbf 15|33|65] [--temporal 7|15|33] [--tolerance 1|2|3] [--weighting 5|10|20|50]
//             [--no-clamp] [--move-x D]   Denoiser (per frame: 1 spp + G-buffer + filters); --move-x
//                                         moves the camera by D along x per frame (position = start + k*D)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt/DenoisingRenderer.h"
#include "rt/Renderer.h"
#include "rt/WhittedRenderer.h"

namespace {

int round_half_away(double r)
{   // round_real_to_int, offline prototype color.h:20-31
    if (r >= 0) return (r - (int)r >= 0.5) ? (int)r + 1 : (int)r;
    return ((int)r - r >= 0.5) ? (int)r - 1 : (int)r;
}

double clamp01(double v) { return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v); }

bool write_p6(const char* path, const rt::Image& img)
{
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    const uint32_t W = img.GetWidth(), H = img.GetHeight();
    std::fprintf(f, "P6\n%u %u\n255\n", W, H);
    std::vector<unsigned char> row(3 * (size_t)W);
    for (uint32_t r = 0; r < H; ++r) {
        const uint32_t* src = img.GetData() + (size_t)(H - 1 - r) * W;   // top-down
        for (uint32_t x = 0; x < W; ++x) {
            row[3 * x + 0] = (unsigned char)(src[x] & 0xFF);
            row[3 * x + 1] = (unsigned char)((src[x] >> 8) & 0xFF);
            row[3 * x + 2] = (unsigned char)((src[x] >> 16) & 0xFF);
        }
        std::fwrite(row.data(), 1, row.size(), f);
    }
    return std::fclose(f) == 0;
}

bool write_p3_offline(const char* path, const std::vector<float>& acc, uint32_t W, uint32_t H, uint32_t spp, double gamma)
{
    FILE* f = std::fopen(path, "w");
    if (!f) return false;
    std::fprintf(f, "P3\n%u %u\n255\n", W, H);
    for (uint32_t r = 0; r < H; ++r) {
        const size_t base = (size_t)(H - 1 - r) * W;
        for (uint32_t x = 0; x < W; ++x) {
            const float* p = &acc[4 * (base + x)];
            int c[3];
            for (int k = 0; k < 3; ++k) c[k] = round_half_away(255 * clamp01(std::pow((double)p[k] / spp, 1.0 / gamma)));
            std::fprintf(f, "%d %d %d\n", c[0], c[1], c[2]);
        }
    }
    return std::fclose(f) == 0;
}

// the BVH / Whitted / Denoiser projects (their mainloop.cpp's Render loop, headless)
int run_project(int argc, char** argv, int i, uint32_t W, uint32_t H, uint32_t frames, const char* out, uint64_t seed)
{
    const std::string proj = argv[i];
    try {
        if (proj == "spheres" || proj == "bvh") {
            std::unique_ptr<rt::WhittedRenderer> r;
            Camera camera = proj == "spheres" ? rt::WhittedRenderer::TwoSpheresCamera() : rt::WhittedRenderer::BVHRayTracerCamera();
            if (proj == "spheres") r = rt::WhittedRenderer::TwoSpheres();
            else {
                if (i + 2 >= argc) { std::fprintf(stderr, "--project bvh BUNNY.obj TEAPOT.obj\n"); return 2; }
                r = rt::WhittedRenderer::BVHRayTracer(argv[i + 1], argv[i + 2]);
            }
            r->ResizeViewport(W, H);
            camera.ResizeViewport(W, H);
            for (uint32_t f = 0; f < frames; ++f) r->Render(camera);
            if (!write_p6(out, *r->GetFinalImage())) { std::fprintf(stderr, "cannot write %s\n", out); return 1; }
            std::printf("{\"project\": \"%s\", \"width\": %u, \"height\": %u, \"frames\": %u, \"kernel_ms\": %.3f}\n", proj.c_str(), W, H,
                        r->GetSPP(), r->LastKernelMilliseconds());
            return 0;
        }
        if (proj == "denoiser") {
            rt::DenoisingRenderer::Settings st;
            st.seed = seed;
            float move_x = 0.0f;
            for (int k = i + 1; k < argc; ++k) {
                const std::string a = argv[k];
                const int v = (k + 1 < argc) ? std::atoi(argv[k + 1]) : 0;
                if (a == "--jbf") {
                    st.disable_JointBilateralFiltering = false;
                    st.using_JointBilateralFiltering_15 = v == 15; st.using_JointBilateralFiltering_33 = v == 33; st.using_JointBilateralFiltering_65 = v == 65;
                    ++k;
                } else if (a == "--temporal") {
                    st.disable_TemporalFiltering = false;
                    st.using_temporal_kernel_7 = v == 7; st.using_temporal_kernel_15 = v == 15; st.using_temporal_kernel_33 = v == 33;
                    ++k;
                } else if (a == "--tolerance") {
                    st.using_temporal_variance_tolerance_1 = v == 1; st.using_temporal_variance_tolerance_2 = v == 2; st.using_temporal_variance_tolerance_3 = v == 3;
                    ++k;
                } else if (a == "--weighting") {
                    st.using_temporal_current_frame_weighting_5 = v == 5; st.using_temporal_current_frame_weighting_10 = v == 10;
                    st.using_temporal_current_frame_weighting_20 = v == 20; st.using_temporal_current_frame_weighting_50 = v == 50;
                    ++k;
                } else if (a == "--no-clamp") {
                    st.immediate_clamping = false;
                } else if (a == "--move-x" && k + 1 < argc) {
                    move_x = std::strtof(argv[++k], nullptr);
                } else {
                    std::fprintf(stderr, "unknown denoiser argument %s\n", a.c_str());
                    return 2;
                }
            }
            rt::DenoisingRenderer r(st);
            Camera camera(35.0f, 0.1f, 100.0f);   // DN/mainloop.cpp:22
            const rt::vec3 p0 = camera.Position();
            r.ResizeViewport(W, H);
            camera.ResizeViewport(W, H);
            for (uint32_t f = 0; f < frames; ++f) {
                camera.SetPosition(rt::vec3{p0.x + move_x * (float)f, p0.y, p0.z});
                r.Render(camera);
            }
            if (!write_p6(out, *r.GetFinalImage())) { std::fprintf(stderr, "cannot write %s\n", out); return 1; }
            const rt_denoise_params dp = r.Resolved();
            std::printf("{\"project\": \"denoiser\", \"width\": %u, \"height\": %u, \"frames\": %u, \"jbf_half\": %d, \"temporal_half\": %d, "
                        "\"frame_ms\": %.3f}\n", W, H, frames, dp.jbf_half_size, dp.temporal_half_size, r.LastFrameMilliseconds());
            return 0;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    std::fprintf(stderr, "unknown project %s\n", proj.c_str());
    return 2;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s W H SPP out.ppm [--seed S] [--rr P] [--fast] [--per-frame] [--offline GAMMA] [--obj FILE R G B]...\n", argv[0]);
        return 2;
    }
    const uint32_t W = (uint32_t)std::atoi(argv[1]), H = (uint32_t)std::atoi(argv[2]), spp = (uint32_t)std::atoi(argv[3]);
    const char* out = argv[4];
    Renderer::Settings s;
    float rr = 0.8f;
    bool per_frame = false;
    double gamma = 0.0;
    struct Obj { std::string path; float r, g, b; };
    std::vector<Obj> objs;
    for (int i = 5; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--project" && i + 1 < argc) return run_project(argc, argv, i + 1, W, H, spp, out, s.seed);
        if (a == "--seed" && i + 1 < argc) s.seed = std::strtoull(argv[++i], nullptr, 10);
        else if (a == "--rr" && i + 1 < argc) rr = std::strtof(argv[++i], nullptr);
        else if (a == "--fast") s.exact = false;
        else if (a == "--per-frame") per_frame = true;
        else if (a == "--offline" && i + 1 < argc) gamma = std::strtod(argv[++i], nullptr);
        else if (a == "--band" && i + 1 < argc) s.band = (uint32_t)std::atoi(argv[++i]);
        else if (a == "--devices" && i + 1 < argc) {
            const std::string list = argv[++i];
            size_t at = 0;
            while (at <= list.size()) {
                const size_t comma = list.find(',', at);
                s.devices.push_back(std::atoi(list.substr(at, comma == std::string::npos ? std::string::npos : comma - at).c_str()));
                if (comma == std::string::npos) break;
                at = comma + 1;
            }
        } else if (a == "--obj" && i + 4 < argc) {
            objs.push_back({argv[i + 1], std::strtof(argv[i + 2], nullptr), std::strtof(argv[i + 3], nullptr), std::strtof(argv[i + 4], nullptr)});
            i += 4;
        } else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    try {
        Renderer renderer(s);
        std::vector<std::unique_ptr<rt::TriangleMesh>> extra;
        for (const Obj& o : objs) {   // Renderer::Add + GenerateBVH (MC/Renderer.h:78-86)
            rt::Material m;
            m.diffuse_coefficient = rt::vec3{o.r, o.g, o.b};
            extra.push_back(std::make_unique<rt::TriangleMesh>(o.path, m));
            renderer.Add(extra.back().get());
        }
        if (!objs.empty()) renderer.GenerateBVH();
        renderer.RR_survival_probability = rr;
        Camera camera(35.0f, 0.1f, 100.0f);   // MC/mainloop.cpp:22
        renderer.ResizeViewport(W, H);
        camera.ResizeViewport(W, H);
        if (per_frame) {
            for (uint32_t f = 0; f < spp; ++f) renderer.Render(camera);   // the GUI's one-spp-per-call loop
        } else {
            renderer.RenderFrames(camera, spp);
        }
        const bool ok = gamma > 0.0 ? write_p3_offline(out, renderer.GetAccumulation(), W, H, renderer.GetSPP(), gamma)
                                    : write_p6(out, *renderer.GetFinalImage());
        if (!ok) {
            std::fprintf(stderr, "cannot write %s\n", out);
            return 1;
        }
        std::printf("{\"width\": %u, \"height\": %u, \"spp\": %u, \"kernel_ms\": %.3f, \"devices\": %zu}\n", W, H, renderer.GetSPP(),
                    renderer.LastKernelMilliseconds(), s.devices.size() > 1 ? s.devices.size() : (size_t)1);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
