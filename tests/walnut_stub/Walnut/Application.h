// tests/walnut_stub/Walnut/Application.h -- TEST STUB of the Walnut application shell (no window, no Vulkan):
// it only holds the pushed layers for the driver to call.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "imgui.h"
#include "Walnut/Layer.h"
namespace Walnut {
struct ApplicationSpecification {
    std::string Name = "Walnut App";
    unsigned Width = 1600, Height = 900;
};
class Application {
public:
    explicit Application(const ApplicationSpecification& s = ApplicationSpecification()) : spec(s) {}
    template <typename T>
    void PushLayer() { layers.push_back(std::make_shared<T>()); }
    ApplicationSpecification spec;
    std::vector<std::shared_ptr<Layer>> layers;
};
Application* CreateApplication(int argc, char** argv);   // the layer file defines it
}  // namespace Walnut
