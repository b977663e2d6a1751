// tests/walnut_stub/dropin/Renderer.h -- the caller's one edit, as an include path: "Renderer.h" -> the drop-in.
#pragma once
#include <rt/walnut/Renderer.h>
