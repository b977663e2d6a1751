/* oracle/philox.h -- TEST INFRASTRUCTURE ONLY (see oracle/README.md).
 *
 * Counter-based RNG that replaces the reference's per-thread std::mt19937
 * (Walnut::Random::Float, WN/Random.h:27-30,47-48; called through
 * Whitted::get_random_float_0_1, MC/WhittedUtilities.h:23-26).  The reference
 * RNG is not reproducible (thread_local engines, nondeterministic pixel->thread
 * mapping), so parity is defined on this frozen
 * stream, injected into the reference's own code by oracle/ref/ref_harness.cpp.
 *
 * Frozen spec (shared with the HIP kernel, restated independently there):
 *   Philox4x32-10 (Salmon et al., SC'11), key = (seed_lo, seed_hi),
 *   counter = (pixel, frame, dim >> 2, 0), u32 = out[dim & 3],
 *   Float = (float)u32 / (float)UINT32_MAX   (WN/Random.h:29, inclusive [0,1]).
 * pixel = y*W + x in frame_data order (MC/Renderer.cpp:124-134),
 * frame = the reference's 1-based frame_accumulating (MC/Renderer.h:195).
 */
#ifndef RT_ORACLE_PHILOX_H
#define RT_ORACLE_PHILOX_H
#include <stdint.h>

static inline void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* u32 draw number `dim` of sample (pixel, frame) under `seed`. */
static inline uint32_t oracle_rng_u32(uint64_t seed, uint32_t pixel, uint32_t frame, uint32_t dim)
{
    uint32_t ctr[4] = {pixel, frame, dim >> 2, 0u};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t out[4];
    oracle_philox4x32_10(ctr, key, out);
    return out[dim & 3u];
}

/* Walnut::Random::Float() formula, WN/Random.h:29: (float)u / (float)UINT32_MAX. */
static inline float oracle_u32_to_float(uint32_t u)
{
    return (float)u / (float)UINT32_MAX;
}

#endif
