/*
 * vpt_rng.h -- per-sample random streams (host + device).
 *
 * The reference draws every number with libc erand48(seed) on ONE global state
 * (include/Vector.h:38) shared by all OpenMP threads (src/rt.cpp:767) and seeded from 3 bytes of
 * getentropy (src/rt.cpp:746): not reproducible, not shardable.  Here the generator is the same
 * POSIX erand48 recurrence
 *     X <- (0x5DEECE66D * X + 0xB) mod 2^48,   xi = X / 2^48,
 * bit-identical to glibc's erand48 (which builds 1.m from X<<4 and subtracts 1.0), but every
 * camera sample (pixel idx, sample i) owns a private 48-bit state derived from the image seed by
 * two splitmix64 rounds.  Results therefore do not depend on thread, wave or GPU count.
 * oracle/oracle_rng.h states the same spec independently; tests compare the two.
 */
#ifndef VPT_RNG_H
#define VPT_RNG_H

#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define VPT_HD __host__ __device__ static inline __attribute__((always_inline))
#else
#define VPT_HD static inline
#endif

VPT_HD uint64_t vpt_splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* the pixel's key: file-order index `idx` (src/rt.cpp:773) under the image seed */
VPT_HD uint64_t vpt_stream_key(uint64_t seed, uint64_t idx)
{
    return vpt_splitmix64(seed + 0x9E3779B97F4A7C15ull * (idx + 1ull));
}

/* start state of sample `sample` of the pixel with key `key` */
VPT_HD uint64_t vpt_stream_start_key(uint64_t key, uint64_t sample)
{
    return vpt_splitmix64(key ^ (sample * 0xD1B54A32D192ED03ull + 1ull)) >> 16;
}

/* start state of sample `sample` of the pixel with file-order index `idx` */
VPT_HD uint64_t vpt_stream_start(uint64_t seed, uint64_t idx, uint64_t sample)
{
    return vpt_stream_start_key(vpt_stream_key(seed, idx), sample);
}

/* the value erand48 returns when its state has become x: x/2^48 exactly (glibc erand48_r
 * construction: the mantissa of 1.m from x<<4, minus 1.0) */
VPT_HD double vpt_erand48_value(uint64_t x)
{
    union {
        uint64_t u;
        double d;
    } b;
    b.u = 0x3FF0000000000000ull | (x << 4);
    return b.d - 1.0;
}

/* one erand48 draw: advances X, returns X/2^48 exactly */
VPT_HD double vpt_erand48(uint64_t* X)
{
    uint64_t x = (*X * 0x5DEECE66Dull + 0xBull) & 0xFFFFFFFFFFFFull;
    *X = x;
    return vpt_erand48_value(x);
}

/* the state three draws later, in one step: a^3 X + c (a^2 + a + 1) mod 2^48 */
VPT_HD uint64_t vpt_erand48_skip3(uint64_t X)
{
    return (X * 0xD498BD0AC4B5ull + 0xAA8544E593Dull) & 0xFFFFFFFFFFFFull;
}

/* the n-draw jump X -> A X + C mod 2^48 (the recurrence composed n times) */
VPT_HD void vpt_erand48_jump(int n, uint64_t* A, uint64_t* C)
{
    uint64_t a = 1, c = 0;
    for (int k = 0; k < n; ++k) {
        a = (a * 0x5DEECE66Dull) & 0xFFFFFFFFFFFFull;
        c = (c * 0x5DEECE66Dull + 0xBull) & 0xFFFFFFFFFFFFull;
    }
    *A = a;
    *C = c;
}

VPT_HD uint64_t vpt_erand48_skip(uint64_t X, uint64_t A, uint64_t C) { return (X * A + C) & 0xFFFFFFFFFFFFull; }

#endif
