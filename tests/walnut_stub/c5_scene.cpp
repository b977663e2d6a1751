// tests/walnut_stub/c5_scene.cpp -- TEST PROGRAM for the scene-extension drop-in (tests/test_walnut_compat.py):
// configuration C5 built the way SURVEY.md 8(d) defines it, in the reference's own spelling -- the Renderer
// constructor's Cornell box (MC/Renderer.cpp:26-57), then a white material, one more Whitted::TriangleMesh
// from an OBJ file, Add and GenerateBVH (MC/Renderer.h:78-86, MC/TriangleMesh.h:148-186,
// MC/WhittedMaterial.h:24-42) -- against include/rt/walnut/*.h.  Then 16 frames of 96x54 through Render.
// Writes <out>_scene.bin (the flattened tree: rt_scene_export arrays) and <out>_accum.bin (float4 / pixel).
//     c5_scene BUNNY_OBJ OUT_PREFIX
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "Camera.h"     // -> include/rt/walnut/Camera.h (tests/walnut_stub/dropin)
#include "Renderer.h"   // -> include/rt/walnut/Renderer.h

int main(int argc, char** argv)
{
    if (argc < 3) { std::fprintf(stderr, "usage: %s OBJ OUT_PREFIX\n", argv[0]); return 2; }
    const std::string out = argv[2];

    Renderer renderer;
    Whitted::WhittedMaterial* white = new Whitted::WhittedMaterial(Whitted::MaterialNature::Diffuse, glm::vec3{0.0f, 0.0f, 0.0f});
    white->diffuse_coefficient = glm::vec3{0.7f, 0.7f, 0.7f};
    renderer.Add(new Whitted::TriangleMesh(argv[1], white));
    renderer.GenerateBVH();

    rt_scene_info info{};
    const rt_scene* sc = renderer.Core().Scene();
    if (!sc || rt_scene_get_info(sc, &info) != RT_OK) { std::fprintf(stderr, "no scene\n"); return 1; }
    std::vector<float> nf((size_t)info.n_nodes * 7), tf((size_t)info.n_tris * 13);
    std::vector<int32_t> ni((size_t)info.n_nodes * 5), ti((size_t)info.n_tris * 2);
    if (rt_scene_export(sc, nf.data(), ni.data(), tf.data(), ti.data()) != RT_OK) return 1;
    {
        std::ofstream f(out + "_scene.bin", std::ios::binary);
        const uint32_t n[2] = {info.n_nodes, info.n_tris};
        f.write((const char*)n, sizeof n);
        f.write((const char*)nf.data(), (std::streamsize)nf.size() * 4);
        f.write((const char*)ni.data(), (std::streamsize)ni.size() * 4);
        f.write((const char*)tf.data(), (std::streamsize)tf.size() * 4);
        f.write((const char*)ti.data(), (std::streamsize)ti.size() * 4);
    }
    std::printf("entities %zu nodes %u tris %u split_root %u\n", renderer.GetEntities().size(), info.n_nodes, info.n_tris, info.split_root);
    if (argc > 3 && std::string(argv[3]) == "--scene-only") return 0;

    Camera camera(35.0f, 0.1f, 100.0f);   // MC/mainloop.cpp:22
    camera.ResizeViewport(96, 54);
    renderer.ResizeViewport(96, 54);
    for (int k = 0; k < 16; ++k) renderer.Render(camera);
    const std::vector<float>& acc = renderer.Core().GetAccumulation();
    std::ofstream f(out + "_accum.bin", std::ios::binary);
    f.write((const char*)acc.data(), (std::streamsize)acc.size() * 4);
    std::printf("%u spp\n", renderer.GetSPP());
    return 0;
}
