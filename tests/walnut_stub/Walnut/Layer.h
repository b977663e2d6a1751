// tests/walnut_stub/Walnut/Layer.h -- TEST STUB: the Walnut::Layer interface a layer overrides.
#pragma once
namespace Walnut {
class Layer {
public:
    virtual ~Layer() = default;
    virtual void OnAttach() {}
    virtual void OnDetach() {}
    virtual void OnUpdate(float) {}
    virtual void OnUIRender() {}
};
}  // namespace Walnut
