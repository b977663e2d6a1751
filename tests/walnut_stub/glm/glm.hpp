// tests/walnut_stub/glm/glm.hpp -- TEST STUB: the few glm types the Walnut layer and include/rt/walnut/*.h
// use (a Walnut application brings the real glm); not a restatement of glm's arithmetic.
#pragma once
namespace glm {
struct vec2 {
    float x = 0, y = 0;
    vec2() = default;
    vec2(float a, float b) : x(a), y(b) {}
    vec2 operator-(const vec2& o) const { return vec2(x - o.x, y - o.y); }
};
struct vec3 {
    float x = 0, y = 0, z = 0;
    vec3() = default;
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
};
struct vec4 {
    float v[4] = {0, 0, 0, 0};
    float& operator[](int i) { return v[i]; }
    float operator[](int i) const { return v[i]; }
};
struct mat4 {
    vec4 c[4];
    mat4() = default;
    explicit mat4(float d) { for (int i = 0; i < 4; ++i) c[i][i] = d; }
    vec4& operator[](int i) { return c[i]; }
    const vec4& operator[](int i) const { return c[i]; }
};
}  // namespace glm
