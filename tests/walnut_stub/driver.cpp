// tests/walnut_stub/driver.cpp -- TEST DRIVER for the Walnut drop-in (tests/test_walnut_compat.py): runs the
// layer that Walnut::CreateApplication pushes (the reference's MC/mainloop.cpp, compiled unchanged against
// include/rt/walnut/*.h and the stubs beside this file) through scripted frames, and writes each displayed
// RGBA8 frame to <out>_<k>.bin.
//   frame 0: "Render Offline" (Reaccumulate + 1 spp)
//   frame 1: "Russian Roulette survival probability = 50%", then "Render Offline"
//   frame 2: "Render in Real-Time" (one more spp, accumulating)
//   frame 3: right mouse button + W held for one update (the camera moves: Reaccumulate), then a frame
#include <cstdio>
#include <fstream>
#include <string>

#include "Walnut/Application.h"
#include "Walnut/Image.h"
#include "Walnut/Input/Input.h"

static void dump(const std::string& path)
{
    const auto* img = static_cast<const Walnut::Image*>(stub::last_image);
    std::ofstream f(path, std::ios::binary);
    const uint32_t wh[2] = {img ? img->GetWidth() : 0u, img ? img->GetHeight() : 0u};
    f.write((const char*)wh, sizeof wh);
    if (img) f.write((const char*)img->pixels.data(), (std::streamsize)img->pixels.size() * 4);
}

int main(int argc, char** argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: %s OUT_PREFIX\n", argv[0]); return 2; }
    const std::string out = argv[1];
    Walnut::Application* app = Walnut::CreateApplication(argc, argv);
    Walnut::Layer& layer = *app->layers.at(0);
    stub::content = ImVec2(64, 48);
    auto frame = [&](float dt) {
        layer.OnUpdate(dt);
        layer.OnUIRender();   // the Image call shows the previous Render's frame; Render runs at the end
        layer.OnUIRender();   // ... so a second UI pass shows this frame's
    };
    stub::pressed.insert("Render Offline");
    frame(0.016f);
    dump(out + "_0.bin");
    stub::pressed.insert("Russian Roulette survival probability = 50%");
    stub::pressed.insert("Render Offline");
    frame(0.016f);
    dump(out + "_1.bin");
    stub::pressed.insert("Render in Real-Time");
    layer.OnUIRender();
    dump(out + "_2.bin");
    stub::right_button = true;
    stub::keys_down.insert((int)Walnut::KeyCode::W);
    layer.OnUpdate(0.05f);
    stub::right_button = false;
    stub::keys_down.clear();
    layer.OnUIRender();
    layer.OnUIRender();
    dump(out + "_3.bin");
    for (const std::string& t : stub::text) std::printf("%s\n", t.c_str());
    delete app;
    return 0;
}
