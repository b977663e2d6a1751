// tests/walnut_stub/imgui.h -- TEST STUB of the Dear ImGui calls a Walnut layer makes (MC/mainloop.cpp); the
// driver scripts the window size and which buttons are "pressed", and reads what the layer printed.
#pragma once
#include <cstdarg>
#include <cstdio>
#include <set>
#include <string>
#include <vector>
struct ImVec2 {
    float x = 0, y = 0;
    ImVec2() = default;
    ImVec2(float a, float b) : x(a), y(b) {}
};
namespace stub {
inline ImVec2 content{64, 48};
inline std::set<std::string> pressed;        // buttons that report a click this frame (consumed)
inline std::vector<std::string> text;        // everything ImGui::Text printed
inline int images_shown = 0;
inline const void* last_image = nullptr;     // the descriptor set the layer displayed (stub: the Walnut::Image)
}  // namespace stub
namespace ImGui {
inline bool Begin(const char*) { return true; }
inline void End() {}
inline ImVec2 GetContentRegionAvail() { return stub::content; }
inline void Image(void* id, ImVec2, ImVec2 = ImVec2(0, 0), ImVec2 = ImVec2(1, 1))
{
    ++stub::images_shown;
    stub::last_image = id;
}
inline void Text(const char* fmt, ...)
{
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    stub::text.push_back(buf);
}
inline void Separator() {}
inline bool Button(const char* label) { return stub::pressed.erase(label) > 0; }
inline bool Checkbox(const char*, bool* v) { return v != nullptr; }
}  // namespace ImGui
