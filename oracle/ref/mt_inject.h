// oracle/ref/mt_inject.h -- TEST INFRASTRUCTURE ONLY: RNG injection into the reference's own
// Walnut::Random (WN/Random.h:27-48, WN/Random.cpp:5-6) for the container-side harnesses
// (ref_harness.cpp, ref_denoiser.cpp).  Include after Walnut/Random.h (through the reference headers)
// and ../philox.h.  Before each sample the untempered form of the frozen Philox stream is written into
// the engine state with position 0, so the reference's own Float() returns the counter-based uniforms;
// the distribution range is set to MSVC's 32-bit one.
#ifndef RT_MT_INJECT_H
#define RT_MT_INJECT_H
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

struct MTLayout { std::mt19937::result_type x[624]; size_t p; };
static_assert(sizeof(MTLayout) == sizeof(std::mt19937), "unexpected libstdc++ mt19937 layout");

static uint32_t mt_untemper(uint32_t y)
{
    // inverse of std::mt19937 tempering (u=11,d=0xffffffff,s=7,b=0x9d2c5680,t=15,c=0xefc60000,l=18)
    uint32_t x = y;
    x = y ^ (y >> 18);
    { uint32_t z = x; uint32_t r = z; for (int i = 0; i < 3; ++i) r = z ^ ((r << 15) & 0xefc60000u); x = r; }
    { uint32_t z = x; uint32_t r = z; for (int i = 0; i < 5; ++i) r = z ^ ((r << 7) & 0x9d2c5680u); x = r; }
    { uint32_t z = x; uint32_t r = z; for (int i = 0; i < 3; ++i) r = z ^ (r >> 11); x = r; }
    return x;
}

static void check_layout_once()
{
    std::mt19937 e;
    MTLayout l;
    for (int i = 0; i < 624; ++i) l.x[i] = mt_untemper(0x1000u + (uint32_t)i * 7919u);
    l.p = 0;
    std::memcpy((void*)&e, &l, sizeof l);
    for (int i = 0; i < 624; ++i) {
        uint32_t v = (uint32_t)e();
        if (v != 0x1000u + (uint32_t)i * 7919u) { fprintf(stderr, "mt19937 injection self-check failed at %d\n", i); exit(3); }
    }
}

struct Injector {
    uint64_t seed = 0;
    uint32_t pixel = 0, frame = 0;
    uint32_t filled = 0;
    uint32_t base = 0;   // stream index of engine word 0 (non-zero after a refill)
    std::mt19937::result_type x0 = 0;
    void start(uint64_t s, uint32_t px, uint32_t fr, uint32_t n) { seed = s; pixel = px; frame = fr; fill(0, n); }
    void fill(uint32_t from, uint32_t n)
    {
        MTLayout l;
        if (n > 624) n = 624;
        base = from;
        for (uint32_t i = 0; i < n; ++i) l.x[i] = mt_untemper(oracle_rng_u32(seed, pixel, frame, from + i));
        // past the filled prefix: all-ones draws (Float()==1.0f ends the path at the next RR test);
        // a path that still exhausts the engine triggers a twist, detected through x[0] in used()
        for (uint32_t i = n; i < 624; ++i) l.x[i] = mt_untemper(0xFFFFFFFFu);
        l.p = 0;
        filled = n;
        x0 = l.x[0];
        std::memcpy((void*)&Walnut::Random::s_RandomEngine, &l, sizeof l);
    }
    // number of draws consumed since start(); 0xFFFFFFFF if the engine twisted (more than the filled
    // words were drawn without a refill)
    uint32_t used() const
    {
        MTLayout l;
        std::memcpy(&l, (const void*)&Walnut::Random::s_RandomEngine, sizeof l);
        if (l.x[0] != x0) return 0xFFFFFFFFu;
        return base + (uint32_t)l.p;
    }
    // Called by the harness glue where the next `need` draws are about to be taken (the top of a
    // shading call, which draws at most 6).  If they would run past the filled words, the engine is
    // re-filled with the stream's next `g_fill_words` words (624 unless RT_HARNESS_FILL says fewer, a
    // self-check of this very mechanism) and its position reset, so a path of any length reads the
    // counter-based stream and the engine never twists.
    void refill_if_near(uint32_t need);
};
static thread_local Injector g_inj;
static uint32_t g_fill_words = 624;

inline void Injector::refill_if_near(uint32_t need)
{
    if (filled == 0) return;   // not injecting (the shipped-stream modes)
    MTLayout l;
    std::memcpy(&l, (const void*)&Walnut::Random::s_RandomEngine, sizeof l);
    if (l.x[0] != x0) return;   // already twisted: used() reports it
    if ((uint32_t)l.p + need <= filled) return;
    fill(base + (uint32_t)l.p, g_fill_words);
}

static void read_fill_words()
{
    if (const char* e = getenv("RT_HARNESS_FILL")) {
        long v = atol(e);
        if (v >= 8 && v <= 624) g_fill_words = (uint32_t)v;
    }
}

static void set_msvc_distribution()
{
    Walnut::Random::s_Distribution = std::uniform_int_distribution<std::mt19937::result_type>(0u, 0xFFFFFFFFu);
}

#endif
