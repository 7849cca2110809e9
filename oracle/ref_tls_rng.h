/*
 * ref_tls_rng.h -- TEST INFRASTRUCTURE ONLY (CPU baseline).  Force-included after ref_prelude.h
 * when oracle/Makefile builds _ref/rt_tls: the reference program unchanged except that every
 * erand48(seed) call (src/rt.cpp:787, include/vptShadeMethods.h, include/*SamplingFunctions.h)
 * draws from a state private to the calling thread instead of the global `seed`
 * (include/Vector.h:38) that all OpenMP threads share in the program as written (SURVEY H4:
 * a data race whose cache-line contention caps the reference at ~1.3 Msamples/s on any core
 * count).  This is BASELINE.md's "per-thread RNG" flavour: the reference's own arithmetic, with
 * its RNG made thread-safe, i.e. the fair upper bound of its CPU throughput.
 *
 * <stdlib.h> (which declares erand48) is included first, so the macro below rewrites only the
 * reference's calls.  Each thread's state is seeded from the program's global seed (getentropy at
 * src/rt.cpp:746, read on the thread's first draw) and a per-thread counter.
 */
#include <stdlib.h>

#include <atomic>

extern unsigned short seed[3];

static inline double vpt_ref_tls_erand48(unsigned short* /* the reference's shared state */)
{
    static std::atomic<unsigned> next_thread{0};
    thread_local unsigned short x[3];
    thread_local bool init = false;
    if (!init) {
        const unsigned t = next_thread.fetch_add(1) + 1;
        x[0] = (unsigned short)(seed[0] ^ (t * 0x9E37u));
        x[1] = (unsigned short)(seed[1] ^ (t * 0x79B9u));
        x[2] = (unsigned short)(seed[2] ^ t);
        init = true;
    }
    return erand48(x);
}
#define erand48(s) vpt_ref_tls_erand48(s)
