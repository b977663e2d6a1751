// include/rt/Abi.h -- the layout guard of the C++ drop-in classes (rt::Renderer, rt::Camera,
// rt::WhittedRenderer, rt::DenoisingRenderer).
//
// Their constructors live in librt_hip.so, but a caller allocates the object with the sizeof IT was compiled
// against.  A front-end built against an older header than the library's therefore hands the library an
// object that is too small, and the library's member initialisers write past it (the round-5 SIGSEGV of
// tests/test_walnut_compat.py: a tests/_bin/walnut_mainloop built before commit 8b334fb grew rt::Renderer
// from 200 to 264 bytes, run against the newer library).  RT_API_VERSION cannot catch
// that: it guards the C structs, and the old check compared the library's constant with itself.
//
// The guard: every public constructor is inline and delegates to a library constructor that takes an
// rt::AbiTag built in the CALLER (this header's RT_CXX_ABI_VERSION and the caller's sizeof of the class and
// of its Settings).  The library checks the tag while initialising the class's first member, before any
// other member is written, and throws rt::Error on a mismatch.  A caller built before this guard existed
// references constructor symbols the library no longer exports, so it fails at symbol lookup instead.
// Bump RT_CXX_ABI_VERSION whenever a class's layout or an exported virtual interface (rt::Entity) changes.
#ifndef RT_ABI_H
#define RT_ABI_H
#include <cstdint>
#include <stdexcept>

#define RT_CXX_ABI_VERSION 2   /* 2 (round 6): rt::Entity gained SphereShape, rt::Sphere */

namespace rt {

class Error : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

enum class AbiClass : uint32_t { Renderer = 1, Camera = 2, WhittedRenderer = 3, DenoisingRenderer = 4 };

// what the caller was compiled with
struct AbiTag {
    uint32_t version;      // RT_CXX_ABI_VERSION of the caller's header
    AbiClass cls;
    uint64_t size;         // caller's sizeof(class)
    uint64_t aux_size;     // caller's sizeof(class::Settings) (0: none)
};

// the first member of every guarded class: constructed from the tag by the library, which throws rt::Error
// unless the tag matches its own build
class AbiGuard {
public:
    explicit AbiGuard(const AbiTag& caller, uint64_t lib_size, uint64_t lib_aux_size);
    uint32_t version() const { return version_; }
private:
    uint32_t version_;
};

}  // namespace rt

#endif
