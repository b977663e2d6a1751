// rt_knobs.h -- the A/B and diagnostic knobs of the library.
//
// The knobs are read from the environment only when the caller opts in with RT_DEBUG_KNOBS=1: a stray
// RT_* variable in a product caller's environment never switches a kernel, a traversal schedule or a
// buffer layout.  Tests and the A/B tools (tests/conftest.py, tools/*) set the gate.
#pragma once
#include <cstdlib>
#include <cstring>

inline bool rt_debug_knobs_enabled()
{
    const char* g = std::getenv("RT_DEBUG_KNOBS");
    return g != nullptr && std::strcmp(g, "1") == 0;
}

// getenv(name) behind the gate: nullptr unless RT_DEBUG_KNOBS=1
inline const char* rt_knob(const char* name) { return rt_debug_knobs_enabled() ? std::getenv(name) : nullptr; }
