/*
 * vpt_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference hot path used as
 * the parity checker.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle*.so; the product never links it.
 *
 * Pinning: liboracle.so (libm transcendentals) is checked bit for bit against the reference's
 * own functions (oracle/_ref/libvpt_ref.so, fixtures in tests/golden/).  liboracle_vm.so is the
 * identical restatement evaluated with the build's portable FP64 math (csrc/vpt_math.h); the
 * HIP kernel must reproduce it bit for bit.
 */
#ifndef VPT_ORACLE_H
#define VPT_ORACLE_H
#include <stdint.h>

typedef struct {           /* byte layout of reference Sphere, include/Sphere.h:14-21 */
    double r;
    double p[3];
    double c[3];
    double radiance[3];
    int32_t material;
    int32_t pad_;
    double eta[3];
    double kappa[3];
    double alpha;
} orc_sphere;

typedef struct {
    double sigma_a, sigma_s;  /* src/rt.cpp:794 */
    double hg_g;              /* extension: 0 = reference isotropic phase */
    int32_t max_depth;        /* extension: 0 = unbounded (reference) */
    int32_t estimator;        /* include/vpt.h vpt_estimator: 0 iterativeVPTracerFree, 1 MISVPTTracerRecursive, ..., 5 iterativePathTracer, 6 rayMarching3, 7 rayMarching2, 8 rayMarchingGlobal, 9 rayMarching */
    double march_step;        /* rayMarching3 / rayMarching2: step; rayMarchingGlobal: segments; rayMarching: steps */
    int32_t march_light;      /* rayMarching3 / rayMarching2: idsource */
    int32_t reserved_;
} orc_medium;

typedef struct {           /* work counters (counting mode) */
    uint64_t tests;        /* ray-sphere tests, Sphere::intersect calls */
    uint64_t iterations;   /* estimator loop iterations */
    uint64_t surface;      /* surface events */
    uint64_t medium;       /* medium events */
} orc_counters;

#endif
