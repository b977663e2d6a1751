// tests/walnut_stub/Walnut/Input/KeyCodes.h -- TEST STUB: the key / button / cursor enums a fly camera reads
// (values as GLFW's).
#pragma once
#include <cstdint>
namespace Walnut {
enum class KeyCode : uint16_t { Space = 32, A = 65, D = 68, S = 83, W = 87, LeftShift = 340 };
enum class MouseButton : uint16_t { Left = 0, Right = 1, Middle = 2 };
enum class CursorMode { Normal = 0, Hidden = 1, Locked = 2 };
}  // namespace Walnut
