// tests/walnut_stub/Walnut/Input/Input.h -- TEST STUB of Walnut::Input: the driver sets the keys, buttons and
// mouse position the camera reads.
#pragma once
#include <set>

#include <glm/glm.hpp>

#include "KeyCodes.h"
namespace stub {
inline std::set<int> keys_down;
inline bool right_button = false;
inline glm::vec2 mouse{0.0f, 0.0f};
inline int cursor_mode = 0;
}  // namespace stub
namespace Walnut {
class Input {
public:
    static bool IsKeyDown(KeyCode k) { return stub::keys_down.count((int)k) > 0; }
    static bool IsMouseButtonDown(MouseButton b) { return b == MouseButton::Right && stub::right_button; }
    static glm::vec2 GetMousePosition() { return stub::mouse; }
    static void SetCursorMode(CursorMode m) { stub::cursor_mode = (int)m; }
};
}  // namespace Walnut
