// tests/walnut_stub/Walnut/Image.h -- TEST STUB of Walnut::Image without Vulkan: SetData keeps a copy of the
// RGBA8 frame so the driver can compare it.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>
namespace Walnut {
enum class ImageFormat { None = 0, RGBA, RGBA32F };
class Image {
public:
    Image(uint32_t width, uint32_t height, ImageFormat format, const void* data = nullptr) : w_(width), h_(height), format_(format)
    {
        if (data) SetData(data);
    }
    void SetData(const void* data)
    {
        pixels.resize((size_t)w_ * h_);
        std::memcpy(pixels.data(), data, pixels.size() * 4);
        ++uploads;
    }
    void* GetDescriptorSet() const { return (void*)this; }
    void Resize(uint32_t width, uint32_t height) { w_ = width; h_ = height; pixels.clear(); }
    uint32_t GetWidth() const { return w_; }
    uint32_t GetHeight() const { return h_; }
    std::vector<uint32_t> pixels;   // test access: the last SetData
    int uploads = 0;
private:
    uint32_t w_, h_;
    ImageFormat format_;
};
}  // namespace Walnut
