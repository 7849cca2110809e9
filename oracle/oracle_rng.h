/*
 * oracle_rng.h -- TEST INFRASTRUCTURE ONLY (part of the parity oracle).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use anything under
 * oracle/.  This file is the oracle-side statement of how one camera sample's random stream
 * is keyed.  The product restates the same spec in
 * minimal_volumetric_path_tracer_amd/csrc/vpt_rng.h; tests check both agree bit for bit.
 *
 * Reference semantics being replaced: every random number in the reference comes from libc
 * erand48() on ONE global 48-bit state (include/Vector.h:38, include/Vector.cpp:8) that is
 * seeded from 3 bytes of getentropy (src/rt.cpp:746) and shared, racily, by all OpenMP
 * threads (src/rt.cpp:767).  That stream is neither reproducible nor shardable.
 *
 * Build semantics: the generator itself is unchanged -- POSIX erand48,
 *     X <- (0x5DEECE66D * X + 0xB) mod 2^48,   xi = X / 2^48  in [0,1)
 * -- but each camera sample (pixel idx, sample i) owns a private state whose start value is
 * derived from a 64-bit image seed by two splitmix64 rounds.  The oracle consumes this
 * stream through the real libc erand48() (libm mode) exactly as the reference does.
 */
#ifndef VPT_ORACLE_RNG_H
#define VPT_ORACLE_RNG_H

#include <stdint.h>

static inline uint64_t orc_splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* 48-bit erand48 start state of camera sample `sample` of pixel `idx` (file-order index
 * (h-y-1)*w+x, src/rt.cpp:773) for image seed `seed`. */
static inline uint64_t orc_stream_state(uint64_t seed, uint64_t idx, uint64_t sample)
{
    uint64_t k = orc_splitmix64(seed + 0x9E3779B97F4A7C15ull * (idx + 1ull));
    uint64_t s = orc_splitmix64(k ^ (sample * 0xD1B54A32D192ED03ull + 1ull));
    return s >> 16;
}

/* erand48 state <-> the xsubi[3] layout libc uses (xsubi[0] = low 16 bits). */
static inline void orc_state_to_xsubi(uint64_t X, unsigned short xs[3])
{
    xs[0] = (unsigned short)(X & 0xFFFFu);
    xs[1] = (unsigned short)((X >> 16) & 0xFFFFu);
    xs[2] = (unsigned short)((X >> 32) & 0xFFFFu);
}

static inline uint64_t orc_xsubi_to_state(const unsigned short xs[3])
{
    return (uint64_t)xs[0] | ((uint64_t)xs[1] << 16) | ((uint64_t)xs[2] << 32);
}

#endif
