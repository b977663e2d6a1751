// oracle/ref/compat_cmath.h -- TEST INFRASTRUCTURE ONLY.
// Force-included (-include) when compiling the reference's sources for oracle/_ref.
// C++17 [cmath.syn] declares std::sqrtf / std::fmodf / std::fabsf / std::powf; libstdc++ 11 (the
// image's) does not (GCC bug 79700; added in GCC 14).  The reference (MSVC) uses these names at
// MC/VectorFloat.h:27 and MC/TriangleMesh.h:223.  These using-declarations name the very same libm
// functions; no reference header or behaviour is replaced.
#include <cmath>
namespace std { using ::sqrtf; using ::fmodf; using ::fabsf; using ::powf; }
