// tests/walnut_stub/Walnut/Timer.h -- TEST STUB: a millisecond wall-clock timer with Walnut::Timer's interface.
#pragma once
#include <chrono>
namespace Walnut {
class Timer {
public:
    Timer() { Reset(); }
    void Reset() { start_ = std::chrono::steady_clock::now(); }
    float Elapsed() { return std::chrono::duration<float>(std::chrono::steady_clock::now() - start_).count(); }
    float ElapsedMillis() { return Elapsed() * 1000.0f; }
private:
    std::chrono::steady_clock::time_point start_;
};
}  // namespace Walnut
