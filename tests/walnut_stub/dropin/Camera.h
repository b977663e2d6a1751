// tests/walnut_stub/dropin/Camera.h -- the caller's one edit, as an include path: "Camera.h" -> the drop-in.
#pragma once
#include <rt/walnut/Camera.h>
