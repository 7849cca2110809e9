/*
 * vpt_device.h -- device side of the volumetric radiance loop (gfx950, FP64).
 *
 * Restates, for the GPU, the reference's per-sample estimators
 *   iterativeVPTracerFree   include/vptShadeMethods.h:1263-1340   (free-flight distance sampling)
 *   MISVPTTracerRecursive   include/vptShadeMethods.h:1345-1481   (equi-angular + surface MIS)
 * and everything they reach, with the reference's floating-point
 * evaluation order (the build compiles with -ffp-contract=off) and the build's portable libm
 * (vpt_math.h), so that one sample here is bit-identical to the oracle's portable-math build
 * (oracle/liboracle_vm.so).  Shortcuts taken here are exact (same bits, same random draws):
 *   - emitter list, MIS light list, material-3 presence: precomputed per scene (host);
 *   - visibility() from a sphere light (r > 1e-4) toward x: the shadow ray starts at the
 *     light's centre and hits the light's own surface at t = sqrt(fl(r*r)) = r, so the point is
 *     visible only when |light - x| < r; otherwise no ray is cast;
 *   - visibilityVPT() equals visibility() when the scene has no material-3 sphere.
 * Counting mode (COUNT = true) adds what the reference would have intersected.
 */
#ifndef VPT_DEVICE_H
#define VPT_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vpt_math.h"
#include "vpt_rng.h"
#include "vpt_scene.h"

#define VPT_DEV __device__ static inline __attribute__((always_inline))
#define VPT_PI 3.14159265358979323846
#define VPT_MAXFLOAT ((double)3.40282346638528859812e+38F) /* MAXFLOAT, vptShadeMethods.h:1287 */
#define VPT_DBL_MAX 1.7976931348623157e+308                 /* __DBL_MAX__, pathTracingUtilities.h:13 */
#ifndef VPT_ISECT_UNROLL
#define VPT_ISECT_UNROLL 5
#endif
/* MISv2's three rays from the surface point are intersected in one pass (scene_intersect_n<3>, for
 * diffuse surfaces): A/B rays fused off / 2 / 3: 5584 / 5569 / 5609 Ms/s (round 2) */
/* sphere loops taken G spheres at a time (scene_intersect_grouped): decide() and every other
 * site; A/B at 1024^2 x 256: off 4914, decide only G=5 4967 (G=10 4857), all sites G=5 5042, G=3 5009 */
#ifndef VPT_DECIDE_GROUP
#define VPT_DECIDE_GROUP 5
#endif
static_assert(VPT_DECIDE_GROUP >= 1, "spheres are taken G >= 1 at a time");

namespace vpt {

/* branches that are rare at the reference's scenes marked for the compiler (block layout and the
 * register allocator's spill placement favour the other side) */
#define VPT_UNLIKELY(c) __builtin_expect(!!(c), 0)
#define VPT_LIKELY(c) __builtin_expect(!!(c), 1)

#define ISECT_SQRT(x) vm_sqrt(x)
/* the sphere tests' root with a class test for its rare arguments (vm_sqrt_isect, vpt_math.h) */
#ifndef VPT_ISECT_CLASS
#define VPT_ISECT_CLASS 1
#endif

/* Debug section timers (builds with -DVPT_SECTIONS=1 only; scripts/sect_stats.py): the wave's
 * s_memtime cycles spent in each section, accumulated per
 * wave in LDS by its first active lane and flushed to g_vpt_sect[k] (entries: g_vpt_sect[SECT_N + k])
 * when the wave exits (sect_flush).  Wall cycles of one wave: the co-resident waves' issue shares
 * the SIMD, so these are shares of time, not instruction counts. */
#ifndef VPT_SECTIONS
#define VPT_SECTIONS 0
#endif
enum {
    SECT_SCHED = 0, SECT_LOAD, SECT_S_PLIGHT, SECT_S_MIS, SECT_S_MIS_ISECT, SECT_S_BDSF, SECT_M_SS, SECT_M_SS_DIR,
    SECT_M_SS_ISECT, SECT_M_SS_SHADOW, SECT_M_PHASE, SECT_CONT, SECT_A_PREP, SECT_A_DECIDE, SECT_A_ISECT, SECT_STORE,
    SECT_S_TOTAL, SECT_M_TOTAL, SECT_A_CAMERA, SECT_A_DECIDE_IN, SECT_M_SHADOW_IN, SECT_A_CAMERA_IN, SECT_M_EQA,
    SECT_M_TR, SECT_A_UNIT, SECT_A_R2, SECT_USED,
    SECT_N = 32
};
#if VPT_SECTIONS
/* one copy per translation unit (the EST = 1 pool kernel's unit reads its own: vpt_pool_mis.hip) */
static __device__ unsigned long long g_vpt_sect[3 * SECT_N];
__device__ static inline __attribute__((always_inline)) uint32_t* sect_lds()
{
    __shared__ uint32_t a[8][3 * SECT_USED];  /* per wave: cycles, entries, active lanes */
    return &a[(threadIdx.x >> 6) & 7][0];
}
#endif
__device__ static inline __attribute__((always_inline)) uint32_t sect_now()
{
#if VPT_SECTIONS
    return (uint32_t)__builtin_amdgcn_s_memtime();  /* (gfx950 reads HW_REG_SHADER_CYCLES as 0) */
#else
    return 0;
#endif
}
__device__ static inline __attribute__((always_inline)) void sect_add(int k, uint32_t t0)
{
#if VPT_SECTIONS
    const uint32_t dt = sect_now() - t0;
    const unsigned long long act = (unsigned long long)__ballot(1);
    const int first = __ffsll(act) - 1;
    if ((int)(threadIdx.x & 63) == first) {
        uint32_t* a = sect_lds();
        a[k] += dt;
        a[SECT_USED + k] += 1;
        a[2 * SECT_USED + k] += (uint32_t)__popcll(act);
    }
#else
    (void)k;
    (void)t0;
#endif
}
__device__ static inline __attribute__((always_inline)) void sect_init()
{
#if VPT_SECTIONS
    for (int l = threadIdx.x & 63; l < 3 * SECT_USED; l += 64) sect_lds()[l] = 0;
#endif
}
__device__ static inline __attribute__((always_inline)) void sect_flush()
{
#if VPT_SECTIONS
    for (int l = threadIdx.x & 63; l < 3 * SECT_USED; l += 64) {
        const uint32_t v = sect_lds()[l];
        atomicAdd(&g_vpt_sect[l < SECT_USED ? l : l < 2 * SECT_USED ? SECT_N + l - SECT_USED : 2 * SECT_N + l - 2 * SECT_USED],
                  (unsigned long long)v);
    }
#endif
}
#define SECT_BEGIN(name) const uint32_t _sect_##name = sect_now()
#define SECT_END(name, k) sect_add(k, _sect_##name)

/* Differential instruction counts (measurement builds only, scripts/dup_pmc.sh): with -DVPT_DUP=k,
 * section k (DUP_* below) runs twice -- the first time on opaque copies of its inputs, its results
 * sunk into an empty asm and discarded -- so the PMC counters of that build minus the release build's
 * are the section's dynamic instruction counts on the real workload (the same batches, lanes and
 * branches; the duplicate takes no draw from the task's stream). */
#ifndef VPT_DUP
#define VPT_DUP 0
#endif
#define DUP_DECIDE 1
#define DUP_DECIDE_ISECT 2
#define DUP_SURF 3
#define DUP_MIS 4
#define DUP_MIS_ISECT 5
#define DUP_MED 6
#define DUP_SS 7
#define DUP_EQA 8
#define DUP_PLIGHT 9
#define DUP_BDSF 10
#define DUP_PHASE 11
#define DUP_CAMERA 12
#define DUP_LDST 13
#define DUP_SS_ISECT 14
#define DUP_SS_DIR 15
#define DUP_MIS_DIRS 16
__device__ __forceinline__ void vpt_opaque(double& v) { __asm__ volatile("" : "+v"(v)); }
__device__ __forceinline__ void vpt_opaque(int& v) { __asm__ volatile("" : "+v"(v)); }
__device__ __forceinline__ void vpt_opaque(uint64_t& v) { __asm__ volatile("" : "+v"(v)); }
__device__ __forceinline__ void vpt_sink(double v) { __asm__ volatile("" ::"v"(v)); }
__device__ __forceinline__ void vpt_sink(int v) { __asm__ volatile("" ::"v"(v)); }
__device__ __forceinline__ void vpt_sink(uint64_t v) { __asm__ volatile("" ::"v"(v)); }

/* ------------------------------------------------------------------ vectors (Vector.h:10-36) */
struct dv3 {
    double x, y, z;
};
VPT_DEV dv3 mk(double x, double y, double z) { return dv3{x, y, z}; }
VPT_DEV dv3 ld3(const double* a) { return dv3{a[0], a[1], a[2]}; }
VPT_DEV dv3 add(dv3 a, dv3 b) { return dv3{a.x + b.x, a.y + b.y, a.z + b.z}; }
VPT_DEV dv3 sub(dv3 a, dv3 b) { return dv3{a.x - b.x, a.y - b.y, a.z - b.z}; }
VPT_DEV dv3 scl(dv3 a, double s) { return dv3{a.x * s, a.y * s, a.z * s}; }
VPT_DEV dv3 mul(dv3 a, dv3 b) { return dv3{a.x * b.x, a.y * b.y, a.z * b.z}; }
VPT_DEV double dot(dv3 a, dv3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
VPT_DEV void vpt_opaque(dv3& a)
{
    vpt_opaque(a.x);
    vpt_opaque(a.y);
    vpt_opaque(a.z);
}
VPT_DEV void vpt_sink(dv3 a)
{
    vpt_sink(a.x);
    vpt_sink(a.y);
    vpt_sink(a.z);
}
VPT_DEV dv3 cross(dv3 a, dv3 b) { return dv3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
/* the reference's normalize, 1.0 / sqrt(|a|^2) times a (inlined: out of line it was slower, round 5) */
VPT_DEV dv3 nrm(dv3 a) { return scl(a, vm_inv_sqrt(a.x * a.x + a.y * a.y + a.z * a.z)); }

struct Counters {
    uint64_t tests;
    uint64_t iterations;
    uint64_t draw_mismatch;  /* events whose draw count is not the pool's kill-prediction jump (trace_sample) */
};

/* Per-sample random stream + work counters.  HG g rides along (phase extension). */
template <bool COUNT>
struct Sampler {
    uint64_t X;
    double g;
    Counters cnt;
    __device__ __forceinline__ double next() { return vpt_erand48(&X); }
    __device__ __forceinline__ void tests(int n)
    {
        if (COUNT) cnt.tests += (uint64_t)n;
    }
};

/* One sphere test of Sphere::intersect (include/Sphere.h:27-37) from b = oc.d and det = b^2 - |oc|^2 + r^2:
 * the reference's
 *     tact = (t1 < 0 || |t1| < 0.0001) ? t2 : t1,   contact = tact > 0 && |tact| > 0.0001
 * with t1 = -b - sq, t2 = -b + sq, written with one comparison each: t1 < 0 || |t1| < 0.0001 is
 * t1 < 0.0001 and tact > 0 && |tact| > 0.0001 is tact > 0.0001, for every t1 / tact including NaN
 * (ordered comparisons: all false).  tact = 0 (no contact) when det < 0. */
VPT_DEV double sphere_tact(double b, double det)
{
    double tact = 0.0;
    if (det >= 0) {
        const double sq = ISECT_SQRT(det);
        const double t2 = -b + sq;
        const double t1 = -b - sq;
        tact = t1 < 0.0001 ? t2 : t1;
    }
    return tact;
}

/* the nearest-contact update of intersect() (include/pathTracingUtilities.h:17-30) as selects
 * (VPT_TAKE_SEL): two compares and three selects instead of two nested branches -- their exec-mask
 * bookkeeping is ~6 scalar instructions per sphere test, in the wave's one instruction stream.  Round 2
 * measured selects slower (56.8 vs 57.7 ms FF); on the round-6 kernel they are faster (A/B ab_r06b: FF
 * 40.39 -> 39.88 ms, MIS + HG 181.1 -> 177.9 ms). */
#ifndef VPT_TAKE_SEL
#define VPT_TAKE_SEL 1
#endif
/* (the contact flag as a bool is not cheaper: across the det >= 0 branch the compiler keeps it in a VGPR
 * and rebuilds the lane mask from it at every test -- 4 instructions instead of 1) */
typedef int contact_t;
VPT_DEV void sphere_take(double tact, int i, double& tmin, int& id, contact_t& contact)
{
    if (VPT_TAKE_SEL) {
        const bool c = tact > 0.0001;
        const bool take = c && tact < tmin;
        tmin = take ? tact : tmin;
        id = take ? i : id;
        contact = c ? (contact_t)1 : contact;
        return;
    }
    if (tact > 0.0001) {
        contact = 1;
        if (tact < tmin) {
            tmin = tact;
            id = i;
        }
    }
}

/* one sphere's contact and the nearest-contact update together (VPT_TAKE_IN): the update inside the
 * det >= 0 branch, so a wave whose every lane misses the sphere (det < 0: no contact, tact = 0 would
 * be taken by no lane) skips it as well as the root -- the same tmin, id and contact per lane */
#ifndef VPT_TAKE_IN
#define VPT_TAKE_IN 1
#endif
/* ZR: the ray leaves a light's centre (vm_sqrt_isect_z) */
#ifndef VPT_ISECT_ZERO
#define VPT_ISECT_ZERO 1
#endif
template <bool ZR = false>
VPT_DEV void sphere_test(double b, double det, int i, double& tmin, int& id, contact_t& contact)
{
    if (!VPT_TAKE_IN) {
        sphere_take(sphere_tact(b, det), i, tmin, id, contact);
        return;
    }
    if (det >= 0) {
        const double sq = (VPT_ISECT_ZERO && ZR) ? vm_sqrt_isect_z(det) : VPT_ISECT_CLASS ? vm_sqrt_isect(det) : ISECT_SQRT(det);
        const double t2 = -b + sq;
        const double t1 = -b - sq;
        sphere_take(t1 < 0.0001 ? t2 : t1, i, tmin, id, contact);
    }
}

/* ------------------------------------------------------------------ geometry */
/* Sphere::intersect (include/Sphere.h:27-37) folded into intersect()
 * (include/pathTracingUtilities.h:12-36).  The sphere index is wave-uniform, so the scene
 * record comes through scalar loads. */
template <bool COUNT, bool ZR = false>
VPT_DEV int scene_intersect(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d, double& t,
                            int& id, bool skip3)
{
    double tmin = VPT_DBL_MAX;
    contact_t contact = 0;
    const int n = S->n;
    /* unrolled so that consecutive sphere tests (independent dependency chains until the tmin
     * update, which stays in index order) overlap: +2% on the pool kernel (A/B, scripts/ab.sh) */
#pragma unroll VPT_ISECT_UNROLL
    for (int i = 0; i < n; ++i) {
        const GeoSphere g = S->geo[i];
        if (skip3 && g.mat3) continue;
        double ocx = o.x - g.px, ocy = o.y - g.py, ocz = o.z - g.pz;
        double b = ocx * d.x + ocy * d.y + ocz * d.z;
        double cc = ocx * ocx + ocy * ocy + ocz * ocz;
        double det = b * b - cc + g.r2;
        sphere_test<ZR>(b, det, i, tmin, id, contact);
    }
    smp.tests(skip3 ? S->n_non3 : n);
    if (contact) {
        t = tmin;
        return 1;
    }
    t = 0;
    return 0;
}

/* scene_intersect (skip3 = false) with the spheres taken G at a time: the G dependency chains
 * up to det are formed first (independent, so they overlap), then the G square-root blocks and
 * the tmin updates in index order -- the same operations per sphere, the same result. */
template <int G, bool COUNT, bool ZR = false>
VPT_DEV int scene_intersect_grouped(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d, double& t,
                                    int& id)
{
    static_assert(G >= 1, "spheres are taken G >= 1 at a time");
    double tmin = VPT_DBL_MAX;
    contact_t contact = 0;
    const int n = S->n;
    int i = 0;
    for (; i + G <= n; i += G) {
        double b[G], det[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const GeoSphere g = S->geo[i + k];
            const double ocx = o.x - g.px, ocy = o.y - g.py, ocz = o.z - g.pz;
            b[k] = ocx * d.x + ocy * d.y + ocz * d.z;
            const double cc = ocx * ocx + ocy * ocy + ocz * ocz;
            det[k] = b[k] * b[k] - cc + g.r2;
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
            sphere_test<ZR>(b[k], det[k], i + k, tmin, id, contact);
        }
    }
    for (; i < n; ++i) {
        const GeoSphere g = S->geo[i];
        const double ocx = o.x - g.px, ocy = o.y - g.py, ocz = o.z - g.pz;
        const double b = ocx * d.x + ocy * d.y + ocz * d.z;
        const double cc = ocx * ocx + ocy * ocy + ocz * ocz;
        const double det = b * b - cc + g.r2;
        sphere_test<ZR>(b, det, i, tmin, id, contact);
    }
    smp.tests(n);
    if (contact) {
        t = tmin;
        return 1;
    }
    t = 0;
    return 0;
}

/* scene_intersect_grouped for rays that all leave one point o, with oc = o - centre and
 * |oc|^2 of every sphere taken from oc[i][0..3] (formed once by the caller with the same operations,
 * march_origin_init): per sphere only b and det are formed -- the same values, the same result */
template <int G, bool COUNT, bool ZR = false>
VPT_DEV int scene_intersect_grouped_oc(const DevScene* __restrict__ S, Sampler<COUNT>& smp, const double (*oc)[4],
                                       dv3 d, double& t, int& id)
{
    static_assert(G >= 1, "spheres are taken G >= 1 at a time");
    double tmin = VPT_DBL_MAX;
    contact_t contact = 0;
    const int n = S->n;
    int i = 0;
    for (; i + G <= n; i += G) {
        double b[G], det[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const double ocx = oc[i + k][0], ocy = oc[i + k][1], ocz = oc[i + k][2], cc = oc[i + k][3];
            b[k] = ocx * d.x + ocy * d.y + ocz * d.z;
            det[k] = b[k] * b[k] - cc + S->geo[i + k].r2;
        }
#pragma unroll
        for (int k = 0; k < G; ++k) sphere_test<ZR>(b[k], det[k], i + k, tmin, id, contact);
    }
    for (; i < n; ++i) {
        const double ocx = oc[i][0], ocy = oc[i][1], ocz = oc[i][2], cc = oc[i][3];
        const double b = ocx * d.x + ocy * d.y + ocz * d.z;
        const double det = b * b - cc + S->geo[i].r2;
        sphere_test<ZR>(b, det, i, tmin, id, contact);
    }
    smp.tests(n);
    if (contact) {
        t = tmin;
        return 1;
    }
    t = 0;
    return 0;
}

/* oc[i] = (o - centre_i, |o - centre_i|^2) for every sphere, by the threads of a workgroup (the
 * operations of scene_intersect_grouped's first loop) */
__device__ static inline void march_origin_init(const DevScene* __restrict__ S, dv3 o, double (*oc)[4])
{
    for (int i = (int)threadIdx.x; i < S->n; i += (int)blockDim.x) {
        const GeoSphere g = S->geo[i];
        const double ocx = o.x - g.px, ocy = o.y - g.py, ocz = o.z - g.pz;
        oc[i][0] = ocx;
        oc[i][1] = ocy;
        oc[i][2] = ocz;
        oc[i][3] = ocx * ocx + ocy * ocy + ocz * ocz;
    }
}

/* every intersection site (not only decide) through the grouped loop, G spheres at a time */
#ifndef VPT_ISECT_GROUP_ALL
#define VPT_ISECT_GROUP_ALL 5
#endif
static_assert(VPT_ISECT_GROUP_ALL >= 1, "spheres are taken G >= 1 at a time");
template <bool COUNT, bool ZR = false>
VPT_DEV int scene_isect(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d, double& t, int& id,
                        bool skip3)
{
    if (!skip3) return scene_intersect_grouped<VPT_ISECT_GROUP_ALL, COUNT, ZR>(S, smp, o, d, t, id);
    return scene_intersect<COUNT, ZR>(S, smp, o, d, t, id, skip3);
}

/* visibility (include/pathTracingUtilities.h:39-53), skip3 = visibilityVPT
 * (include/volumetricBasicFunctions.h:92-106).  light_r: radius of the light sphere when the
 * light point is a sphere centre (exact shortcut, header comment), negative otherwise. */
/* ZR: sphere tests with vm_sqrt_isect_z (a point light's own sphere, det = 0, without the rare-argument
 * call): the one-lane-per-pixel ray-marching and punctual kernels (A/B ab_r06o: rayMarching3 99.1 -> 94.7 ms);
 * the pool kernel's point-light shadow rays were 0.5 % slower with it */
template <bool COUNT, bool ZR = false>
VPT_DEV int visibility(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 light, dv3 x, bool skip3,
                       double light_r, bool light_is3, const double (*light_oc)[4] = nullptr)
{
    dv3 lx = sub(light, x);
    double distance = vm_sqrt(dot(lx, lx));
    if (light_r > 0.0001 && !(skip3 && light_is3) && !(distance < light_r)) {
        smp.tests(skip3 ? S->n_non3 : S->n);
        return 0;
    }
    lx = nrm(lx);
    lx = scl(lx, -1);
    int id = 0;
    double t;
    if (light_oc != nullptr && !skip3) scene_intersect_grouped_oc<VPT_ISECT_GROUP_ALL, COUNT, ZR>(S, smp, light_oc, lx, t, id);
    else scene_isect<COUNT, ZR>(S, smp, light, lx, t, id, skip3);
    return (t > distance || t == 0);
}

/* visibility() given |light - x| and nrm(light - x), formed once by a caller that needs them as well
 * (p_light_nee): the same operations */
template <bool COUNT>
VPT_DEV int visibility_pre(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 light, double distance, dv3 wl,
                           bool skip3, double light_r, bool light_is3)
{
    if (light_r > 0.0001 && !(skip3 && light_is3) && !(distance < light_r)) {
        smp.tests(skip3 ? S->n_non3 : S->n);
        return 0;
    }
    const dv3 lx = scl(wl, -1);
    int id = 0;
    double t;
    scene_isect(S, smp, light, lx, t, id, skip3);
    return (t > distance || t == 0);
}

/* coordinateSystem, include/mathUtilities.h:10-19 */
VPT_DEV void coord_system(dv3 n, dv3& s, dv3& t)
{
#ifndef VPT_FRAME_SEL
#define VPT_FRAME_SEL 1
#endif
    if (VPT_FRAME_SEL) {
        /* the reference's two branches as one evaluation: with u = n.x or n.y by the branch condition, both
         * compute invLen = 1 / sqrt(u u + n.z n.z) and t from n.z invLen and -(u invLen) (negation is
         * exact) -- the same operations per lane, but a wave whose lanes take both branches (surface
         * normals of different walls, cone axes) pays one root and one division instead of two each */
        const bool bx = vm_fabs(n.x) > vm_fabs(n.y);
        const double u = bx ? n.x : n.y;
        const double invLen = 1.0 / vm_sqrt(u * u + n.z * n.z);
        const double a = n.z * invLen, c = -u * invLen;
        t = mk(bx ? a : 0.0, bx ? 0.0 : a, c);
    } else if (vm_fabs(n.x) > vm_fabs(n.y)) {
        double invLen = 1.0 / vm_sqrt(n.x * n.x + n.z * n.z);
        t = mk(n.z * invLen, 0.0, -n.x * invLen);
    } else {
        double invLen = 1.0 / vm_sqrt(n.y * n.y + n.z * n.z);
        t = mk(0.0, n.z * invLen, -n.y * invLen);
    }
    s = cross(t, n);
}

/* coordinateTraspose, include/mathUtilities.h:21-30 */
VPT_DEV dv3 to_local(dv3 n, dv3 w)
{
    dv3 s, t;
    coord_system(n, s, t);
    return mk(dot(s, w), dot(t, w), dot(n, w));
}

VPT_DEV dv3 from_local(dv3 n, double x1, double y1, double z1)
{
    dv3 s, t;
    coord_system(n, s, t);
    return add(add(scl(s, x1), scl(t, y1)), scl(n, z1));
}

/* The coordinateSystem frame of a normal formed once and shared by an event's to_local / from_local
 * calls (VPT_FRAME_CSE).  The compiler does not merge repeated coord_system(n) calls: the square root's
 * wave-uniform rare-argument branch makes each evaluation its own control flow, so every call was a
 * root, a division and a cross product again (a diffuse surface event formed the frame of its normal
 * six times).  Same operations, same bits. */
#ifndef VPT_FRAME_CSE
#define VPT_FRAME_CSE 1
#endif
struct Frame {
    dv3 s, t, n;
};
VPT_DEV Frame make_frame(dv3 n)
{
    Frame F;
    F.n = n;
    coord_system(n, F.s, F.t);
    return F;
}
VPT_DEV void vpt_opaque(Frame& F)
{
    vpt_opaque(F.s);
    vpt_opaque(F.t);
    vpt_opaque(F.n);
}
VPT_DEV dv3 to_local(const Frame& F, dv3 w) { return mk(dot(F.s, w), dot(F.t, w), dot(F.n, w)); }
VPT_DEV dv3 from_local(const Frame& F, double x1, double y1, double z1)
{
    return add(add(scl(F.s, x1), scl(F.t, y1)), scl(F.n, z1));
}

/* transmitance, include/volumetricBasicFunctions.h:14-21 */
VPT_DEV double transmitance(dv3 a, dv3 b, double sigma_t)
{
    dv3 aux = sub(b, a);
    double d = vm_sqrt(dot(aux, aux));
    return lm_exp(sigma_t * d * -1.0);
}

/* multipleT, include/volumetricBasicFunctions.h:26-57 (material-3 spheres only) */
template <bool COUNT>
VPT_DEV double multiple_t(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 x1, dv3 x2, double sigma_t)
{
    double T = 1;
    dv3 w = nrm(sub(x2, x1));
    for (int i = 0; i < S->n; ++i) {
        const GeoSphere g = S->geo[i];
        if (!g.mat3) continue;
        smp.tests(1);
        double ocx = x1.x - g.px, ocy = x1.y - g.py, ocz = x1.z - g.pz;
        double b = ocx * w.x + ocy * w.y + ocz * w.z;
        double det = b * b - (ocx * ocx + ocy * ocy + ocz * ocz) + g.r2;
        double ta = 0.0, tb = 0.0;
        if (!(det < 0)) {
            double sq = ISECT_SQRT(det);
            tb = -b + sq;
            ta = -b - sq;
        }
        if (tb < 0) T = T * lm_exp(-sigma_t * ta);
        if (tb - ta > 0) T = T * lm_exp(-sigma_t * (tb - ta));
    }
    return T;
}

/* ------------------------------------------------------------------ sampling */
/* direction at polar angle theta = acos(c) and azimuth phi around n: the reference computes
 * sin(acos c), cos(acos c), sin(phi), cos(phi) with libm (lm_dir_trig, bit for bit) */
template <class FL>
VPT_DEV dv3 dir_from_cos_fl(dv3 n, double c, double phi, FL fl)
{
    double st, ct, sp, cp;
    if (__ballot(c != 1.0) == 0) {
        /* c == 1 in every lane (the cone toward a point light: cmax = sqrt(1 - 0) = 1 and
         * (1 - e0) + e0 * 1 = 1 exactly): glibc's acos(1) = +0, sin(+0) = +0, cos(+0) = 1, so only
         * the azimuth's sin and cos are evaluated -- the same bits */
        st = 0.0;
        ct = 1.0;
        /* ... and when no component of n is zero, not even those: from_local(n, 0 cp, 0 sp, 1) =
         * (s (+-0) + t (+-0)) + n 1 = n exactly (the frame of a unit n is finite, so s and t scale
         * to signed zeros, which a nonzero n_k absorbs) -- the azimuth draw is taken by the caller */
        if (__ballot(n.x == 0 || n.y == 0 || n.z == 0 || !(n.x - n.x == 0 && n.y - n.y == 0 && n.z - n.z == 0)) == 0)
            return nrm(n);
        lm_sincos(phi, &sp, &cp);
    } else {
        lm_dir_trig(c, phi, &st, &ct, &sp, &cp);
    }
    return nrm(fl(st * cp, st * sp, ct));
}
VPT_DEV dv3 dir_from_cos(dv3 n, double c, double phi)
{
    return dir_from_cos_fl(n, c, phi, [&](double a, double b, double d) { return from_local(n, a, b, d); });
}
VPT_DEV dv3 dir_from_cos(const Frame& F, double c, double phi)
{
    return dir_from_cos_fl(F.n, c, phi, [&](double a, double b, double d) { return from_local(F, a, b, d); });
}

/* solidAngle(wc, costheta_max), include/samplingFunctions.h:65-82 */
template <bool COUNT>
VPT_DEV dv3 solid_angle_dir(Sampler<COUNT>& smp, dv3 wc, double cmax)
{
    double e0 = smp.next();
    double c = (1 - e0) + e0 * cmax;  /* theta = acos(c) */
    double phi = 2 * VPT_PI * smp.next();
    return dir_from_cos(wc, c, phi);
}

/* solidAngleProb, include/samplingFunctions.h:85-87 */
VPT_DEV double solid_angle_prob(double cmax) { return 1 / (2 * VPT_PI * (1 - cmax)); }

/* VPT_DIV_SHARE: divisions by one divisor share its reciprocal (vm_rcp, vpt_math.h) -- the same bits as
 * the compiler's division for operands it would not rescale, which a wave-uniform range test checks
 * (else the plain divisions run for the whole wave) */
#ifndef VPT_DIV_SHARE
#define VPT_DIV_SHARE 1
#endif
/* RN(1/pi), the reciprocal the compiler's division sequence forms for the divisor pi (v_rcp_f64 + two
 * Newton steps; equal on the device, tests/test_gpu_parity.py::test_device_shared_reciprocal_division) */
#define VPT_INV_PI_RCP 0x1.45f306dc9c883p-2
/* hemiCosineProb, include/samplingFunctions.h:92-94: c * 1 / pi, (c * 1) == c */
VPT_DEV double hemi_cosine_prob(double c)
{
    if (VPT_DIV_SHARE && __ballot(!vm_rcp_ok(c)) == 0) {
        const vm_rcp R = {VPT_PI, VPT_INV_PI_RCP};
        return vm_div_by(c, R);
    }
    return c * 1 / VPT_PI;
}
/* 1 / d and r / d -- r a sphere radius (>= 0; +0 for a point light gives +0 as the division does) --
 * with one reciprocal, when every lane's d and r are in range */
VPT_DEV void inv_and_ratio(double d, double r, double& inv, double& q)
{
    if (VPT_DIV_SHARE && __ballot(!(vm_rcp_ok(d) && (vm_as_u64(r) == 0 || vm_rcp_ok(r)))) == 0) {
        const vm_rcp R = vm_rcp_of(d);
        inv = vm_div_by(1.0, R);
        q = vm_div_by(r, R);
    } else {
        inv = 1 / d;
        q = r / d;
    }
}

/* cosineHemispheric, include/samplingFunctions.h:47-62 */
template <bool COUNT>
VPT_DEV dv3 cosine_hemispheric(Sampler<COUNT>& smp, dv3 n)
{
    double c = vm_sqrt(1 - smp.next());  /* theta = acos(c) */
    double phi = 2 * VPT_PI * smp.next();
    return dir_from_cos(n, c, phi);
}
template <bool COUNT>
VPT_DEV dv3 cosine_hemispheric(Sampler<COUNT>& smp, const Frame& F)
{
    double c = vm_sqrt(1 - smp.next());
    double phi = 2 * VPT_PI * smp.next();
    return dir_from_cos(F, c, phi);
}

/* isotropicPhaseSample, include/vptSamplingFunctions.h:34-47 (g == 0); Henyey-Greenstein
 * extension around the propagation direction din otherwise. */
template <bool COUNT>
VPT_DEV dv3 phase_sample(Sampler<COUNT>& smp, dv3 din)
{
    double xi1 = smp.next();
    double xi2 = smp.next();
    double g = smp.g;
    if (g == 0.0) {
        double phi = 2 * VPT_PI * xi2;
        double st, ct, sp, cp;
        lm_dir_trig(1 - 2 * xi1, phi, &st, &ct, &sp, &cp);  /* theta = acos(1 - 2 xi1) */
        return nrm(mk(st * cp, st * sp, ct));
    }
    double sq = (1.0 - g * g) / (1.0 - g + 2.0 * g * xi1);
    double ct = (1.0 + g * g - sq * sq) / (2.0 * g);
    double st2 = 1.0 - ct * ct;
    double st = st2 > 0.0 ? vm_sqrt(st2) : 0.0;
    double phi = 2 * VPT_PI * xi2;
    double sp, cp;
    lm_sincos(phi, &sp, &cp);
    return nrm(from_local(din, st * cp, st * sp, ct));
}

/* isotropicPhaseFunction (include/volumetricBasicFunctions.h:59-62) or HG value */
VPT_DEV double phase_value(double g, dv3 din, dv3 wl)
{
    if (g == 0.0) return 1 / (4 * VPT_PI);
    double mu = dot(din, wl);
    double den = 1.0 + g * g - 2.0 * g * mu;
    return (1.0 - g * g) / (4 * VPT_PI * (den * vm_sqrt(den)));
}

/* ------------------------------------------------------------------ microfacet (microFacetUtilities.h) */
/* fresnelSpectre, :11-18 */
VPT_DEV double fresnel_spectre(double cosine, double sine, double eta, double kappa)
{
    double a2b2 = vm_sqrt((eta * eta - kappa * kappa - sine * sine) * (eta * eta - kappa * kappa - sine * sine) +
                          4 * eta * eta * kappa * kappa);
    double a = vm_sqrt(0.5 * (a2b2 + eta * eta - kappa * kappa - sine * sine));
    double perpendicular = (a2b2 + cosine * cosine - 2 * a * cosine) / (a2b2 + cosine * cosine + 2 * a * cosine);
    double parallel = perpendicular *
                      (a2b2 * cosine * cosine + sine * sine * sine * sine - 2 * a * cosine * sine * sine) /
                      (a2b2 * cosine * cosine + sine * sine * sine * sine + 2 * a * cosine * sine * sine);
    return 0.5 * (parallel + perpendicular);
}

/* fresnel, :21-29 */
VPT_DEV dv3 fresnel(double cw, dv3 eta, dv3 kappa)
{
    double sw = vm_sqrt(1 - cw * cw);
    return mk(fresnel_spectre(cw, sw, eta.x, kappa.x), fresnel_spectre(cw, sw, eta.y, kappa.y),
              fresnel_spectre(cw, sw, eta.z, kappa.z));
}

/* NDF (Beckmann), :34-45 */
VPT_DEV double ndf(double cosine, double alpha)
{
    if (cosine >= 0) {
        double sine = vm_sqrt(1 - cosine * cosine);
        double fac1 = VPT_PI * alpha * alpha * cosine * cosine * cosine * cosine;
        double tang = sine / cosine;
        double fac2 = lm_exp((-1 * tang * tang) / (alpha * alpha));
        return (1 / fac1) * fac2;
    }
    return 0;
}

/* Gn, :47-61 */
VPT_DEV double g1(dv3 n, dv3 wv, dv3 wh, double alpha)
{
    double sn = vm_sqrt(1 - dot(n, wv) * dot(n, wv));
    double tn = sn / (dot(n, wv));
    double a = 1 / (alpha * tn);
    if (((dot(wv, wh)) / (dot(wv, n))) > 0) {
        if (a < 1.6) {
            double num = 3.535 * a + 2.181 * a * a;
            double den = 1 + 2.276 * a + 2.577 * a * a;
            return num / den;
        }
        return 1;
    }
    return 0;
}

/* vectorFacet, :71-84 */
template <bool COUNT>
VPT_DEV dv3 vector_facet(Sampler<COUNT>& smp, double alpha)
{
    double theta = lm_atan(vm_sqrt(-alpha * alpha * lm_log(1 - smp.next())));
    double phi = 2 * VPT_PI * smp.next();
    double st, ct, sp, cp;
    lm_sincos2(theta, phi, &st, &ct, &sp, &cp);
    return nrm(mk(st * cp, st * sp, ct));
}

/* microFacetProb, :86-92 */
VPT_DEV double microfacet_prob(dv3 wo, dv3 wh, double alpha, dv3 n)
{
    double num = dot(wh, n);
    double den = 4 * vm_fabs(dot(wo, wh));
    return ndf(dot(wh, n), alpha) * num / den;
}

/* frMicroFacet, :95-100 (G_smith :63-68).  Out of line: three Fresnel channels, two Smith terms and
 * the NDF are independent chains that the scheduler interleaves, and inlined at the five sites of a
 * metal surface event they set the kernel's register allocation (A/B round 3: 53.28 vs 53.50 ms FF) */
__device__ static __attribute__((noinline)) dv3 fr_microfacet(dv3 eta, dv3 kappa, dv3 wi, dv3 wh, dv3 wo, double alpha, dv3 n)
{
    double den = (4 * vm_fabs(dot(n, wi)) * vm_fabs(dot(n, wo)));
    double G = g1(n, wi, wh, alpha) * g1(n, wo, wh, alpha);
    return scl(scl(scl(fresnel(dot(wi, wh), eta, kappa), ndf(dot(n, wh), alpha)), G), (1 / den));
}

/* fresnelDie, :107-112 */
VPT_DEV double fresnel_die(double etai, double etat, double ct, double ci)
{
    double parallel = ((etat * ci - etai * ct) / (etat * ci + etai * ct)) * ((etat * ci - etai * ct) / (etat * ci + etai * ct));
    double perpendicular =
        ((etai * ci - etat * ct) / (etai * ci + etat * ct)) * ((etai * ci - etat * ct) / (etai * ci + etat * ct));
    return 0.5 * (parallel + perpendicular);
}

/* reflexDielectric, :117-120 */
VPT_DEV dv3 reflex_dielectric(dv3 wi, dv3 n) { return add(scl(wi, -1), scl(scl(n, dot(n, wi)), 2)); }

/* refraxDielectric, :123-141 */
VPT_DEV dv3 refrax_dielectric(double etai, double etat, dv3 wi, dv3 n)
{
    dv3 wil = to_local(n, wi);
    double ratio = etat / etai * -1;
    double cosinei = dot(wi, n);
    double invratio = etai / etat;
    double cosinet = vm_sqrt(1 - invratio * invratio * (1 - cosinei * cosinei)) - 1;
    return from_local(n, wil.x * ratio, wil.y * ratio, cosinet);
}

/* ------------------------------------------------------------------ shading records */
/* per-sphere flag of a per-lane sphere index: a shift of a wave-uniform mask (DevScene m_*) instead of
 * a per-lane load of the GeoSphere record (whose latency sat on decide()'s critical path) */
VPT_DEV int sph_flag(uint64_t m, int i) { return (int)((m >> (i & 63)) & 1ull); }

/* the emitter list's entry j (vptShadeMethods.h:1293-1303, idsource = arr[rand * count]): a per-lane
 * load (selects over scalar loads were slower: A/B round 3, 50.58 -> 51.20 ms FF) */
VPT_DEV int emit_pick(const DevScene* __restrict__ S, int /*count*/ j, int count)
{
    (void)count;
    return S->emit[j];
}

VPT_DEV dv3 sph_c(const DevScene* __restrict__ S, int i) { return ld3(S->sph[i].c); }
VPT_DEV dv3 sph_rad(const DevScene* __restrict__ S, int i) { return ld3(S->sph[i].radiance); }
VPT_DEV dv3 sph_p(const DevScene* __restrict__ S, int i) { return ld3(S->sph[i].p); }

/* material of sphere `obj`: MK >= 0 when the caller knows it at compile time (the pool kernel's
 * surface rings are keyed by material), which removes the other materials' code from that path */
template <int MK>
VPT_DEV int mat_of(const DevScene* __restrict__ S, int obj) { return MK >= 0 ? MK : S->sph[obj].material; }

/* rayTracer, include/pathTracingUtilities.h:56-64 */
template <bool COUNT>
VPT_DEV dv3 ray_tracer(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 x, dv3 wi, int& sourceid)
{
    double t;
    int id = 0;
    if (!scene_isect(S, smp, x, wi, t, id, false)) return mk(0, 0, 0);
    sourceid = id;
    return sph_rad(S, id);
}

/* cosinethetaMax, include/pathTracingUtilities.h:66-73 */
VPT_DEV double cos_theta_max(const DevScene* __restrict__ S, int sid, dv3 x)
{
    double radio = S->sph[sid].r;
    dv3 cx = sub(sph_p(S, sid), x);
    double normcx = vm_sqrt(dot(cx, cx));
    return vm_sqrt(1 - (radio / normcx) * (radio / normcx));
}

/* ------------------------------------------------------------------ light transport */
/* microfacet (BSDF-sampled light), include/samplingFunctions.h:97-118 */
template <bool COUNT>
VPT_DEV dv3 microfacet_light(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 x, dv3 wo, dv3 wh, dv3 n,
                             int obj, double alpha, int& idsource)
{
    const dv3 nl = mk(0, 0, 1);
    int sourceid = 0;
    wo = scl(wo, -1);
    wo = nrm(to_local(n, wo));
    dv3 wi = nrm(add(scl(wo, -1), scl(scl(wh, 2), dot(wh, wo))));
    dv3 wig = nrm(from_local(n, wi.x, wi.y, wi.z));
    dv3 Le = ray_tracer(S, smp, x, wig, sourceid);
    idsource = sourceid;
    dv3 fr = fr_microfacet(ld3(S->sph[obj].eta), ld3(S->sph[obj].kappa), wi, wh, wo, alpha, nl);
    return scl(scl(mul(Le, fr), dot(mk(0, 0, 1), wi)), (1 / microfacet_prob(wo, wh, alpha, nl)));
}

/* muestreoSA (include/samplingFunctions.h:238-247) + solidAngle 9-arg (:163-206) */
template <bool COUNT>
VPT_DEV dv3 light_sample_sa(const DevScene* __restrict__ S, Sampler<COUNT>& smp, int light, dv3 x, int obj, int omat,
                            dv3 n, dv3 wray, dv3& aux, double& cmax_out, double alpha)
{
    dv3 cx = sub(sph_p(S, light), x);
    double normcx = vm_sqrt(dot(cx, cx));
    double lr = S->sph[light].r;
    double inv, q;
    inv_and_ratio(normcx, lr, inv, q);  /* 1 / normcx, lr / normcx */
    cx = scl(cx, inv);
    double cmax = vm_sqrt(1 - q * q);
    cmax_out = cmax;
    dv3 wolocal = scl(wray, -1);
    dv3 wi = solid_angle_dir(smp, cx, cmax);
    aux = wi;
    dv3 wilocal = nrm(to_local(n, wi));
    wolocal = nrm(to_local(n, wolocal));
    dv3 wh = nrm(add(wilocal, wolocal));
    dv3 fr;
    if (omat == 0) fr = scl(sph_c(S, obj), (1 / VPT_PI));
    else if (omat == 2) fr = mk(0, 0, 0);
    else fr = fr_microfacet(ld3(S->sph[obj].eta), ld3(S->sph[obj].kappa), wilocal, wh, wolocal, alpha, mk(0, 0, 1));
    double t;
    int id = 0;
    scene_isect(S, smp, x, wi, t, id, false);
    dv3 Le = (light == id) ? sph_rad(S, id) : mk(0, 0, 0);
    return scl(scl(mul(Le, fr), dot(n, wi)), (1 / solid_angle_prob(cmax)));
}

/* softDielectric, include/samplingFunctions.h:209-235 */
template <bool COUNT>
VPT_DEV dv3 soft_dielectric(const DevScene* __restrict__ S, Sampler<COUNT>& smp, double etat, double etai, dv3 wi,
                            dv3 n, dv3 x, int& idsource)
{
    dv3 Ld;
    int sourceid = 0;
    dv3 wt = nrm(refrax_dielectric(etai, etat, wi, n));
    double F = fresnel_die(etai, etat, dot(n, wt), dot(n, wi));
    if (smp.next() < F) {
        dv3 wr = nrm(reflex_dielectric(wi, n));
        Ld = scl(ray_tracer(S, smp, x, wr, sourceid), (1 / vm_fabs(dot(n, wr))));
    } else {
        double ratio = etat / etai;
        Ld = scl(scl(scl(ray_tracer(S, smp, x, wt, sourceid), (1 / vm_fabs(dot(n, wt)))), ratio), ratio);
    }
    idsource = sourceid;
    return Ld;
}

/* powerHeuristics, include/misSamplingFunctions.h:12-16 */
VPT_DEV double power_heuristic(double f, double g)
{
    double f2 = f * f;
    double g2 = g * g;
    return f2 / (f2 + g2);
}

/* MISv2, include/misSamplingFunctions.h:96-170 (TR = true), and MIS, :19-91 (TR = false): the same
 * function without the transmitance factor on the light samples (:29 vs :106) */
template <bool COUNT, int MK = -1, bool TR = true>
VPT_DEV dv3 mis_v2(const DevScene* __restrict__ S, Sampler<COUNT>& smp, int obj, dv3 x, dv3 n, dv3 wray, double alpha,
                   double sigma_t)
{
    const int omat = mat_of<MK>(S, obj);
    dv3 mc = mk(0, 0, 0), g;
    dv3 wiLight = mk(0, 0, 0), wiBDRF = mk(0, 0, 0);
    double wg, fpdf = 0, gpdf = 0, cmax = 0;
    int sourceid = 0, sourceid2 = 0;
    dv3 wo = scl(wray, -1);
    for (int k = 0; k < S->n_mis; ++k) {  /* spheres with r > 0 && radiance.x > 0, in index order */
        const int light = S->mis_light[k];
        dv3 f = light_sample_sa(S, smp, light, x, obj, omat, n, wray, wiLight, cmax, alpha);
        if (TR) f = scl(f, transmitance(x, sph_p(S, light), sigma_t));
        fpdf = solid_angle_prob(cmax);
        if (omat == 0) {
            gpdf = hemi_cosine_prob(dot(n, wiLight));
        } else if (omat == 2) {
            dv3 wt = nrm(refrax_dielectric(1.0, 1.5, wo, n));
            gpdf = fresnel_die(1.0, 1.5, dot(n, wt), dot(n, wo));
            if (smp.next() > gpdf) gpdf = 1 - gpdf;
        } else {
            dv3 wh = nrm(add(wiLight, wo));
            gpdf = microfacet_prob(wo, wh, alpha, n);
        }
        double wf = power_heuristic(fpdf, gpdf);
        mc = add(mc, scl(f, wf));
    }
    if (omat == 0) {
        /* uniform(), include/samplingFunctions.h:250-261 */
        dv3 wi = nrm(cosine_hemispheric(smp, n));
        dv3 Le = ray_tracer(S, smp, x, wi, sourceid);
        g = add(mk(0, 0, 0), scl(scl(mul(Le, scl(sph_c(S, obj), (1 / VPT_PI))), dot(n, wi)), (1 / hemi_cosine_prob(dot(n, wi)))));
        wiBDRF = wi;
        gpdf = hemi_cosine_prob(dot(n, wiBDRF));
        if (g.x > 0 && g.y > 0 && g.z > 0) {
            cmax = cos_theta_max(S, sourceid, x);
            fpdf = solid_angle_prob(cmax);
            wg = power_heuristic(gpdf, fpdf);
        } else {
            wg = 0;
        }
    } else if (omat == 2) {
        g = soft_dielectric(S, smp, 1.5, 1.0, wo, n, x, sourceid);
        if (g.x > 0 && g.y > 0 && g.z > 0) {
            cmax = cos_theta_max(S, sourceid, x);
            fpdf = solid_angle_prob(cmax);
            wg = power_heuristic(gpdf, fpdf); /* gpdf: stale value from the light loop (reference) */
        } else {
            wg = 0;
        }
    } else {
        dv3 wh = vector_facet(smp, alpha);
        wo = nrm(to_local(n, wo));
        g = microfacet_light(S, smp, x, wray, wh, n, obj, alpha, sourceid2);
        gpdf = microfacet_prob(wo, wh, alpha, mk(0, 0, 1));
        if (g.x > 0) cmax = cos_theta_max(S, sourceid2, x);
        fpdf = solid_angle_prob(cmax);
        wg = power_heuristic(gpdf, fpdf);
    }
    return add(mc, scl(g, wg));
}

/* intersect() (include/pathTracingUtilities.h:12-36) of N rays from ONE origin in one pass over the
 * spheres: per ray exactly the operations of scene_intersect, in the same order (oc and |oc|^2 are
 * the same numbers for every ray, so they are formed once), and N independent dependency chains
 * per sphere instead of one.  id[k] must be initialised by the caller (left unchanged on a miss,
 * like scene_intersect). */
template <int N, bool COUNT>
VPT_DEV void scene_intersect_n(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, const dv3 (&d)[N],
                               double (&t)[N], int (&id)[N], bool (&hit)[N])
{
    double tmin[N];
    contact_t contact[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        tmin[k] = VPT_DBL_MAX;
        contact[k] = 0;
    }
    const int n = S->n;
    int i = 0;
#ifndef VPT_ISECT_N_GROUP
#define VPT_ISECT_N_GROUP 5
#endif
#ifndef VPT_ISECT_VIDX
#define VPT_ISECT_VIDX 1
#endif
    /* VPT_ISECT_N_GROUP spheres per loop iteration: their records come in one batch of scalar loads
     * (one wait instead of one per sphere) */
    for (; i + VPT_ISECT_N_GROUP <= n; i += VPT_ISECT_N_GROUP) {
#pragma unroll
        for (int j = 0; j < VPT_ISECT_N_GROUP; ++j) {
            const GeoSphere g = S->geo[i + j];
            const double ocx = o.x - g.px, ocy = o.y - g.py, ocz = o.z - g.pz;
            const double cc = ocx * ocx + ocy * ocy + ocz * ocz;
            /* the sphere index copied into a VGPR once for the N rays' id selects (VPT_ISECT_VIDX): a select
             * cannot take it from an SGPR beside its SGPR lane mask, so each test copied it again */
            int vi = i + j;
#if VPT_ISECT_VIDX && defined(__HIP_DEVICE_COMPILE__)
            if (N > 1) __asm__("v_mov_b32 %0, %1" : "=v"(vi) : "s"(i + j));
#endif
#pragma unroll
            for (int k = 0; k < N; ++k) {
                const double b = ocx * d[k].x + ocy * d[k].y + ocz * d[k].z;
                const double det = b * b - cc + g.r2;
                sphere_test(b, det, vi, tmin[k], id[k], contact[k]);
            }
        }
    }
    for (; i < n; ++i) {
        const GeoSphere g = S->geo[i];
        const double ocx = o.x - g.px, ocy = o.y - g.py, ocz = o.z - g.pz;
        const double cc = ocx * ocx + ocy * ocy + ocz * ocz;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const double b = ocx * d[k].x + ocy * d[k].y + ocz * d[k].z;
            const double det = b * b - cc + g.r2;
            sphere_test(b, det, i, tmin[k], id[k], contact[k]);
        }
    }
    smp.tests(N * n);
#pragma unroll
    for (int k = 0; k < N; ++k) {
        hit[k] = contact[k] != 0;
        t[k] = contact[k] ? tmin[k] : 0.0;
    }
}

/* MISv2 (include/misSamplingFunctions.h:96-170) for a scene with exactly two MIS lights, same bits
 * and draws as mis_v2: every draw of MISv2 precedes, and none depends on, the three ray casts
 * (the two light samples of muestreoSA, :163-206, and the BSDF sample of uniform / softDielectric
 * / microfacet), so the draws and directions are taken first in the reference's order, the three
 * rays from x are intersected in one pass (scene_intersect_n), and the arithmetic is then done in
 * the reference's order. */
/* Fn: the frame of n (make_frame), shared with the caller's pLight and bdsf (held through the three ray
 * casts: forming it again after them was slower, A/B ab_r06h 38.21 / 171.2 vs 37.91 / 171.0 ms).  VPT_MIS_REUSE: the
 * transmittance's distance is the light setup's |c - x| (transmitance() forms the same root of the same
 * dot product), the BSDF sample's hemiCosineProb is formed once for its two uses, and cosinethetaMax of
 * a light the BSDF ray hit is the setup's cone cosine of that light (the same operations on the same
 * operands) when every lane's hit is one of the two lights. */
#ifndef VPT_MIS_REUSE
#define VPT_MIS_REUSE 1
#endif
template <bool COUNT, int MK = -1>
VPT_DEV dv3 mis_v2_two_lights(const DevScene* __restrict__ S, Sampler<COUNT>& smp, int obj, dv3 x, dv3 n, dv3 wray,
                              double alpha, double sigma_t, const Frame& Fn)
{
    const int omat = mat_of<MK>(S, obj);
    const dv3 wo = scl(wray, -1);
    /* ---- draws and directions, in the reference's order */
    int lt[2];
    dv3 dirs[3];
    double cm[2], xtra[2] = {0, 0}, nd[2];
    dv3 cxk[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        lt[k] = S->mis_light[k];
        dv3 cx = sub(sph_p(S, lt[k]), x);
        const double normcx = vm_sqrt(dot(cx, cx));
        const double lr = S->sph[lt[k]].r;
        double inv, q;
        inv_and_ratio(normcx, lr, inv, q);  /* 1 / normcx, lr / normcx */
        cx = scl(cx, inv);
        cm[k] = vm_sqrt(1 - q * q);
        cxk[k] = cx;
        nd[k] = normcx;
    }
    if (omat != 2) {  /* both cone samples' draws (e0, phi per light, samplingFunctions.h:65-82), then their trig together */
        const double e00 = smp.next();
        const double c0 = (1 - e00) + e00 * cm[0];
        const double phi0 = 2 * VPT_PI * smp.next();
        const double e01 = smp.next();
        const double c1 = (1 - e01) + e01 * cm[1];
        const double phi1 = 2 * VPT_PI * smp.next();
        double st0, ct0, sp0, cp0, st1, ct1, sp1, cp1;
#if VPT_DUP == DUP_MIS_DIRS
        {
            double a0 = c0, a1 = phi0, a2 = c1, a3 = phi1;
            vpt_opaque(a0);
            vpt_opaque(a1);
            vpt_opaque(a2);
            vpt_opaque(a3);
            double q[8];
            lm_dir_trig2(a0, a1, a2, a3, &q[0], &q[1], &q[2], &q[3], &q[4], &q[5], &q[6], &q[7]);
            for (int k = 0; k < 8; ++k) vpt_sink(q[k]);
        }
#endif
        lm_dir_trig2(c0, phi0, c1, phi1, &st0, &ct0, &sp0, &cp0, &st1, &ct1, &sp1, &cp1);
        dirs[0] = nrm(from_local(cxk[0], st0 * cp0, st0 * sp0, ct0));
        dirs[1] = nrm(from_local(cxk[1], st1 * cp1, st1 * sp1, ct1));
    } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            dirs[k] = solid_angle_dir(smp, cxk[k], cm[k]);
            xtra[k] = smp.next();  /* the dielectric pdf coin of the light loop */
        }
    }
    dv3 wt_s = mk(0, 0, 0), wh_m = mk(0, 0, 0), wo_l = mk(0, 0, 0), wi_m = mk(0, 0, 0);
    bool refl = false;
    if (omat == 0) {
        /* uniform(), samplingFunctions.h:250-261 */
        dirs[2] = VPT_FRAME_CSE ? nrm(cosine_hemispheric(smp, Fn)) : nrm(cosine_hemispheric(smp, n));
    } else if (omat == 2) {  /* softDielectric, samplingFunctions.h:209-235 */
        wt_s = nrm(refrax_dielectric(1.0, 1.5, wo, n));
        const double F = fresnel_die(1.0, 1.5, dot(n, wt_s), dot(n, wo));
        refl = smp.next() < F;
        dirs[2] = refl ? nrm(reflex_dielectric(wo, n)) : wt_s;
    } else {  /* vectorFacet + microfacet, samplingFunctions.h:97-118 */
        wh_m = vector_facet(smp, alpha);
        wo_l = nrm(to_local(n, wo));
        wi_m = nrm(add(scl(wo_l, -1), scl(scl(wh_m, 2), dot(wh_m, wo_l))));
        dirs[2] = nrm(from_local(n, wi_m.x, wi_m.y, wi_m.z));
    }
    /* ---- the three ray casts from x */
    double tt[3];
    int ids[3] = {0, 0, 0};
    bool hits[3];
    SECT_BEGIN(mi);
    /* The BSDF-sampled ray (dirs[2]) is read only through the radiance of what it hits (rayTracer):
     * when its det (b^2 - |oc|^2 + r^2, the operations Sphere::intersect performs) is negative for every
     * sphere with a nonzero radiance, in every lane, no such sphere can be its nearest contact, the
     * radiance is (0, 0, 0) whatever it hits, and only the two light rays are intersected -- the same
     * values (A/B: FF 42.82 -> 42.27 ms, MIS + HG 193.6 -> 191.2 ms; testing contact itself, root and
     * tact > 0.0001, skips more batches but costs more: 42.31 / 191.8 ms) */
    bool skip2 = false;
    if (S->emit_all_radiance) {
        bool maybe = false;
        for (int j = 0; j < S->n_emit; ++j) {
            const GeoSphere g = S->geo[S->emit[j]];
            const double ocx = x.x - g.px, ocy = x.y - g.py, ocz = x.z - g.pz;
            const double cc = ocx * ocx + ocy * ocy + ocz * ocz;
            const double b = ocx * dirs[2].x + ocy * dirs[2].y + ocz * dirs[2].z;
            maybe = maybe || !(b * b - cc + g.r2 < 0);
        }
        skip2 = __ballot(maybe) == 0;
    }
#if VPT_DUP == DUP_MIS_ISECT
    {
        dv3 x2 = x;
        dv3 dd[3] = {dirs[0], dirs[1], dirs[2]};
        vpt_opaque(x2);
        for (int k = 0; k < 3; ++k) vpt_opaque(dd[k]);
        double tq[3];
        int iq[3] = {0, 0, 0};
        bool hq[3];
        if (skip2) {
            const dv3 d2[2] = {dd[0], dd[1]};
            double t2[2];
            int i2[2] = {0, 0};
            bool h2[2];
            scene_intersect_n<2>(S, smp, x2, d2, t2, i2, h2);
            tq[0] = t2[0], tq[1] = t2[1], iq[0] = i2[0], iq[1] = i2[1], hq[0] = h2[0], hq[1] = h2[1];
            tq[2] = 0, hq[2] = false;
        } else {
            scene_intersect_n<3>(S, smp, x2, dd, tq, iq, hq);
        }
        for (int k = 0; k < 3; ++k) {
            vpt_sink(tq[k]);
            vpt_sink(iq[k] + (hq[k] ? 256 : 0));
        }
    }
#endif
    if (skip2) {
        const dv3 d2[2] = {dirs[0], dirs[1]};
        double t2[2];
        int i2[2] = {0, 0};
        bool h2[2];
        scene_intersect_n<2>(S, smp, x, d2, t2, i2, h2);
        smp.tests(S->n);  /* (counting mode: the skipped ray's tests) */
        tt[0] = t2[0], tt[1] = t2[1], tt[2] = 0.0;
        ids[0] = i2[0], ids[1] = i2[1];
        hits[0] = h2[0], hits[1] = h2[1], hits[2] = false;
    } else {
        scene_intersect_n<3>(S, smp, x, dirs, tt, ids, hits);
    }
    SECT_END(mi, SECT_S_MIS_ISECT);
    /* ---- the reference's arithmetic */
    dv3 mc = mk(0, 0, 0);
    double fpdf = 0, gpdf = 0, cmax = 0, wg;
    const dv3 wolocal_f = VPT_FRAME_CSE ? nrm(to_local(Fn, wo)) : mk(0, 0, 0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const dv3 wi = dirs[k];
        const dv3 wilocal = VPT_FRAME_CSE ? nrm(to_local(Fn, wi)) : nrm(to_local(n, wi));
        const dv3 wolocal = VPT_FRAME_CSE ? wolocal_f : nrm(to_local(n, wo));
        const dv3 wh = nrm(add(wilocal, wolocal));
        dv3 fr;
        if (omat == 0) fr = scl(sph_c(S, obj), (1 / VPT_PI));
        else if (omat == 2) fr = mk(0, 0, 0);
        else fr = fr_microfacet(ld3(S->sph[obj].eta), ld3(S->sph[obj].kappa), wilocal, wh, wolocal, alpha, mk(0, 0, 1));
        const dv3 Le = (lt[k] == ids[k]) ? sph_rad(S, ids[k]) : mk(0, 0, 0);
        dv3 f = scl(scl(mul(Le, fr), dot(n, wi)), (1 / solid_angle_prob(cm[k])));
        f = scl(f, VPT_MIS_REUSE ? lm_exp(sigma_t * nd[k] * -1.0) : transmitance(x, sph_p(S, lt[k]), sigma_t));
        cmax = cm[k];
        fpdf = solid_angle_prob(cmax);
        if (omat == 0) {
            gpdf = hemi_cosine_prob(dot(n, wi));
        } else if (omat == 2) {
            const dv3 wt = nrm(refrax_dielectric(1.0, 1.5, wo, n));
            gpdf = fresnel_die(1.0, 1.5, dot(n, wt), dot(n, wo));
            if (xtra[k] > gpdf) gpdf = 1 - gpdf;
        } else {
            const dv3 whg = nrm(add(wi, wo));
            gpdf = microfacet_prob(wo, whg, alpha, n);
        }
        const double wf = power_heuristic(fpdf, gpdf);
        mc = add(mc, scl(f, wf));
    }
    dv3 g;
    const dv3 Lb = hits[2] ? sph_rad(S, ids[2]) : mk(0, 0, 0);  /* rayTracer */
    const int sourceid = hits[2] ? ids[2] : 0;
    if (omat == 0) {
        const dv3 wi = dirs[2];
        const double hc = hemi_cosine_prob(dot(n, wi));
        g = add(mk(0, 0, 0), scl(scl(mul(Lb, scl(sph_c(S, obj), (1 / VPT_PI))), dot(n, wi)),
                                 (1 / (VPT_MIS_REUSE ? hc : hemi_cosine_prob(dot(n, wi))))));
        gpdf = hc;
        if (g.x > 0 && g.y > 0 && g.z > 0) {
            if (VPT_MIS_REUSE && __ballot(sourceid != lt[0] && sourceid != lt[1]) == 0)
                cmax = sourceid == lt[0] ? cm[0] : cm[1];
            else
                cmax = cos_theta_max(S, sourceid, x);
            fpdf = solid_angle_prob(cmax);
            wg = power_heuristic(gpdf, fpdf);
        } else {
            wg = 0;
        }
    } else if (omat == 2) {
        if (refl) {
            g = scl(Lb, (1 / vm_fabs(dot(n, dirs[2]))));
        } else {
            const double ratio = 1.5 / 1.0;
            g = scl(scl(scl(Lb, (1 / vm_fabs(dot(n, wt_s)))), ratio), ratio);
        }
        if (g.x > 0 && g.y > 0 && g.z > 0) {
            cmax = cos_theta_max(S, sourceid, x);
            fpdf = solid_angle_prob(cmax);
            wg = power_heuristic(gpdf, fpdf); /* gpdf: stale value from the light loop (reference) */
        } else {
            wg = 0;
        }
    } else {
        const dv3 nl = mk(0, 0, 1);
        const dv3 fr = fr_microfacet(ld3(S->sph[obj].eta), ld3(S->sph[obj].kappa), wi_m, wh_m, wo_l, alpha, nl);
        g = scl(scl(mul(Lb, fr), dot(mk(0, 0, 1), wi_m)), (1 / microfacet_prob(wo_l, wh_m, alpha, nl)));
        gpdf = microfacet_prob(wo_l, wh_m, alpha, mk(0, 0, 1));
        if (g.x > 0) cmax = cos_theta_max(S, sourceid, x);
        fpdf = solid_angle_prob(cmax);
        wg = power_heuristic(gpdf, fpdf);
    }
    return add(mc, scl(g, wg));
}

/* bdsf (continuation sample), include/vptShadeMethods.h:16-59 */
template <bool COUNT, int MK = -1>
VPT_DEV dv3 bdsf(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3& aux, dv3 wray, dv3 n, double& prob, int id)
{
    const int mat = mat_of<MK>(S, id);
    dv3 wi, fs1 = mk(0, 0, 0);
    dv3 wo = scl(wray, -1);
    if (mat == 0) {
        wi = cosine_hemispheric(smp, n);
        fs1 = scl(sph_c(S, id), (1 / VPT_PI));
        prob = hemi_cosine_prob(dot(n, wi));
        aux = wi;
    } else if (mat == 2) {
        dv3 wt = nrm(refrax_dielectric(1.0, 1.5, wo, n));
        double F = fresnel_die(1.0, 1.5, dot(n, wt), dot(n, wo));
        if (smp.next() < F) {
            wi = nrm(reflex_dielectric(wo, n));
            fs1 = scl(scl(mk(1, 1, 1), (1 / dot(n, wi))), F);
            prob = F;
        } else {
            wi = wt;
            fs1 = scl(scl(scl(scl(mk(1, 1, 1), (1 / dot(n, wi))), (1 - F)), 1.5), 1.5);
            prob = 1 - F;
        }
        aux = wi;
    } else if (mat == 1) {
        double alpha = S->sph[id].alpha;
        dv3 whl = vector_facet(smp, alpha);
        dv3 wh = from_local(n, whl.x, whl.y, whl.z);
        wi = add(scl(wo, -1), scl(scl(wh, 2), dot(wh, wo)));
        fs1 = fr_microfacet(ld3(S->sph[id].eta), ld3(S->sph[id].kappa), wi, wh, wo, alpha, n);
        prob = microfacet_prob(wo, wh, alpha, n);
        aux = wi;
    }
    return fs1;
}

/* pLight (point-light NEE at a surface), include/vptShadeMethods.h:62-91.  PT: 1 when the caller
 * knows the light is a point (r == 0; the pool kernel's rings are keyed by it), -1 unknown. */
template <bool COUNT, int MK = -1, int PT = -1, bool ZR = false>  /* ZR: visibility's (iterativePathTracer: true) */
VPT_DEV dv3 p_light(const DevScene* __restrict__ S, Sampler<COUNT>& smp, int obj, dv3 x, dv3 n, dv3 wray, int src,
                    double alpha)
{
    const dv3 I = sph_rad(S, src);
    const dv3 light = sph_p(S, src);
    const double lr = PT == 1 ? 0.0 : S->sph[src].r;
    const bool l3 = sph_flag(S->m_mat3, src);
    dv3 Le;
    if (visibility<COUNT, ZR>(S, smp, light, x, false, lr, l3)) {
        Le = scl(I, (1 / (dot(sub(light, x), sub(light, x)))));
    } else if (VPT_LIKELY(S->n_mat3 == 0)) {
        smp.tests(S->n);  /* visibilityVPT == visibility (no material-3 sphere): same miss */
        Le = mk(0, 0, 0);
    } else if (visibility<COUNT, ZR>(S, smp, light, x, true, lr, l3)) {
        Le = scl(I, (1 / (dot(sub(light, x), sub(light, x)))));
        Le = scl(Le, multiple_t(S, smp, x, light, 0.05 + 0.009));
    } else {
        Le = mk(0, 0, 0);
    }
    dv3 wi = nrm(sub(light, x));
    dv3 wo = scl(wray, -1);
    wo = to_local(n, wo);
    wi = to_local(n, wi);
    wi = nrm(wi);
    wo = nrm(wo);
    dv3 wh = nrm(add(wi, wo));
    dv3 fr;
    if (mat_of<MK>(S, obj) == 1)
        fr = fr_microfacet(ld3(S->sph[obj].eta), ld3(S->sph[obj].kappa), wi, wh, wo, alpha, mk(0, 0, 1));
    else
        fr = scl(sph_c(S, obj), (1 / VPT_PI));
    return scl(mul(Le, fr), dot(n, nrm(sub(light, x))));
}

/* p_light for surface_event (VPT_PL_REUSE): the distance to the light, its square and the unit direction
 * formed once -- visibility(), Le's 1 / |light - x|^2, wi, the final cosine and the caller's
 * transmitance(x, light) all form them from the same light - x -- and the frame of n given (Fn).  Trs:
 * transmitance(x, light, sigma_t). */
#ifndef VPT_PL_REUSE
#define VPT_PL_REUSE 1
#endif
template <bool COUNT, int MK = -1, int PT = -1>
VPT_DEV dv3 p_light_nee(const DevScene* __restrict__ S, Sampler<COUNT>& smp, int obj, dv3 x, dv3 n, dv3 wray, int src,
                        double alpha, const Frame& Fn, double sigma_t, double& Trs)
{
    const dv3 I = sph_rad(S, src);
    const dv3 light = sph_p(S, src);
    const double lr = PT == 1 ? 0.0 : S->sph[src].r;
    const bool l3 = sph_flag(S->m_mat3, src);
    const dv3 lx = sub(light, x);
    const double dd = dot(lx, lx);
    const double distance = vm_sqrt(dd);
    const dv3 wl = nrm(lx);
    Trs = lm_exp(sigma_t * distance * -1.0);
    dv3 Le;
    if (visibility_pre(S, smp, light, distance, wl, false, lr, l3)) {
        Le = scl(I, (1 / dd));
    } else if (VPT_LIKELY(S->n_mat3 == 0)) {
        smp.tests(S->n);
        Le = mk(0, 0, 0);
    } else if (visibility_pre(S, smp, light, distance, wl, true, lr, l3)) {
        Le = scl(I, (1 / dd));
        Le = scl(Le, multiple_t(S, smp, x, light, 0.05 + 0.009));
    } else {
        Le = mk(0, 0, 0);
    }
    dv3 wo = scl(wray, -1);
    wo = to_local(Fn, wo);
    dv3 wi = to_local(Fn, wl);
    wi = nrm(wi);
    wo = nrm(wo);
    dv3 fr;
    if (mat_of<MK>(S, obj) == 1) {
        const dv3 wh = nrm(add(wi, wo));
        fr = fr_microfacet(ld3(S->sph[obj].eta), ld3(S->sph[obj].kappa), wi, wh, wo, alpha, mk(0, 0, 1));
    } else {
        fr = scl(sph_c(S, obj), (1 / VPT_PI));
    }
    return scl(mul(Le, fr), dot(n, wl));
}

/* freeSingleScattering (with_sigma = false), include/volumetricBasicFunctions.h:284-340, and
 * singleScattering (with_sigma = true), :225-281.  din: propagation direction (HG only).
 * For a point light the reference first casts the shadow ray (:295-304 / :236-245), then the cone
 * ray (:310-337), whose result REPLACES Ld whenever the cone ray's first hit is the light (SURVEY
 * H5: 80-87 % of point-light events).  The shadow ray draws nothing, so it is cast after the cone
 * ray here and only when its result survives: same draws, same bits, one ray cast fewer in most
 * point-light medium events (counting mode still adds its tests). */
/* the shadow ray toward a point light and its radiance, volumetricBasicFunctions.h:295-304 / :236-245
 * (single_scattering's point-light branch) */
/* mag: |lp - xt|, formed by the caller (VPT_PL_REUSE: visibility's distance and the transmittance's are
 * the same root of the same dot product) */
/* the radiance of a visible point light (wl = nrm(lp - xt) under VPT_PL_REUSE) */
template <bool COUNT>
VPT_DEV dv3 point_shadow_value(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 xt, dv3 din, int src,
                               double sigma_t, bool with_sigma, double sigma_s, double trxt, double probSource,
                               double mag, dv3 wl)
{
    const dv3 lp = sph_p(S, src);
    const dv3 rad = sph_rad(S, src);
    double distanceLight = dot(sub(lp, xt), sub(lp, xt));
    dv3 Le = scl(rad, (1 / distanceLight));
    double ph = smp.g == 0.0 ? 1 / (4 * VPT_PI) : phase_value(smp.g, din, VPT_PL_REUSE ? wl : nrm(sub(lp, xt)));
    dv3 Ls = scl(scl(Le, VPT_PL_REUSE ? lm_exp(sigma_t * mag * -1.0) : transmitance(xt, lp, sigma_t)), ph);
    if (with_sigma) return scl(scl(scl(Ls, trxt), sigma_s), (1 / probSource));
    return scl(Ls, (1 / probSource));
}
template <bool COUNT>
VPT_DEV dv3 point_shadow_ld(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 xt, dv3 din, int src,
                            double sigma_t, bool with_sigma, double sigma_s, double trxt, double probSource, double mag)
{
    const dv3 lp = sph_p(S, src);
    dv3 Ld = mk(0, 0, 0);
    const dv3 wl = VPT_PL_REUSE ? nrm(sub(lp, xt)) : mk(0, 0, 0);
    if (VPT_PL_REUSE ? visibility_pre(S, smp, lp, mag, wl, false, -1.0, false)
                     : visibility(S, smp, lp, xt, false, -1.0, false))
        Ld = point_shadow_value(S, smp, xt, din, src, sigma_t, with_sigma, sigma_s, trxt, probSource, mag, wl);
    return Ld;
}

/* Single scattering toward a point light (VPT_SS_FUSE): the light cone's ray can only score through
 * src == idHit, and its nearest contact is the light's r = 0 sphere only if that sphere's own test has
 * det >= 0.  A lane whose light sphere gives det < 0 (NaN included) on the cone ray -- formed here with
 * scene_isect's operations -- therefore ends in the shadow-ray branch whatever the other spheres give
 * (unless src == 0 and nothing is hit: idHit keeps its initial 0, so src == 0 lanes are left out), and
 * it casts its shadow ray in the cone ray's pass instead (its origin and direction per lane), with
 * visibility_pre's test on the result.  The shadow rays left for the divergent second pass are those of
 * lanes whose cone ray met another sphere first. */
#ifndef VPT_SS_FUSE
#define VPT_SS_FUSE 1
#endif

template <bool COUNT, int LT = -1>  /* LT: 1 point light, 0 not, -1 unknown (read r) */
VPT_DEV dv3 single_scattering(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 xt, dv3 din, int src,
                              double sigma_t, bool with_sigma, double sigma_s, double trxt, double probSource,
                              bool zero_ok = false)
{
    const double lr = LT == 1 ? 0.0 : S->sph[src].r;
    const dv3 lp = sph_p(S, src);
    const dv3 rad = sph_rad(S, src);
    const bool point = LT == 1 || (LT < 0 && lr == 0);
    dv3 Ld = mk(0, 0, 0);
    SECT_BEGIN(sd);
    dv3 wc = sub(lp, xt);
    double mag = vm_sqrt(dot(wc, wc));
    /* a point light (LT == 1, lr = 0): 0 / mag is +0 for mag > 0 (mag >= 0 or NaN), NaN otherwise,
     * so the cosine is 1 or NaN -- the same value without the division and the root */
    double cmax;
    if (LT == 1) {
        wc = scl(wc, (1 / mag));
        cmax = mag > 0 ? 1.0 : __builtin_nan("");
    } else {
        double inv, q;
        inv_and_ratio(mag, lr, inv, q);  /* 1 / mag, lr / mag */
        wc = scl(wc, inv);
        cmax = vm_sqrt(1 - q * q);
    }
#if VPT_DUP == DUP_SS_DIR
    {
        dv3 wc2 = wc;
        double cm2 = cmax;
        vpt_opaque(wc2);
        vpt_opaque(cm2);
        Sampler<COUNT> s2 = smp;
        vpt_opaque(s2.X);
        vpt_sink(solid_angle_dir(s2, wc2, cm2));
        vpt_sink(s2.X);
    }
#endif
    dv3 wl = solid_angle_dir(smp, wc, cmax);
    double prob_wl = solid_angle_prob(cmax);
    SECT_END(sd, SECT_M_SS_DIR);
    SECT_BEGIN(si);
    double tdist;
    int idHit = 0;
#if VPT_DUP == DUP_SS_ISECT
    {
        dv3 xt2 = xt, wl2 = wl;
        vpt_opaque(xt2);
        vpt_opaque(wl2);
        double td2 = 0;
        int id2 = 0;
        scene_isect(S, smp, xt2, wl2, td2, id2, false);
        vpt_sink(td2);
        vpt_sink(id2);
    }
#endif
    bool shl = false;  /* VPT_SS_FUSE: this lane's pass casts its shadow ray */
    dv3 wls = mk(0, 0, 0);
    if (VPT_SS_FUSE && VPT_PL_REUSE && point) {
        /* (geo[src] holds lp and r2 = r r = +0 for a point light: the same operands) */
        const double ocx = xt.x - lp.x, ocy = xt.y - lp.y, ocz = xt.z - lp.z;
        const double b = ocx * wl.x + ocy * wl.y + ocz * wl.z;
        const double cc = ocx * ocx + ocy * ocy + ocz * ocz;
        const double det = b * b - cc + 0.0;
        shl = src != 0 && !(det >= 0);
        if (shl) wls = nrm(sub(lp, xt));
    }
    if (VPT_SS_FUSE && VPT_PL_REUSE && point) scene_isect(S, smp, shl ? lp : xt, shl ? scl(wls, -1) : wl, tdist, idHit, false);
    else scene_isect(S, smp, xt, wl, tdist, idHit, false);
    SECT_END(si, SECT_M_SS_ISECT);
    SECT_BEGIN(sw);
    if (shl) {
        smp.tests(S->n);  /* the shadow ray (cast in the pass above) or the cone ray: each is counted */
        if (tdist > mag || tdist == 0)  /* visibility_pre */
            Ld = point_shadow_value(S, smp, xt, din, src, sigma_t, with_sigma, sigma_s, trxt, probSource, mag, wls);
    } else if (src == idHit) {
        if (point) smp.tests(S->n);  /* the shadow ray the reference casts first (result overwritten) */
        /* a point light's cone (cmax == 1: prob_wl = +inf) scores Ls * (1 / inf) = +-0 with Ls finite
         * (SURVEY H5); zero_ok: the caller's update absorbs a signed zero (finite throughput and
         * pdf), so +0 is the same result without the exponential and the phase value */
        if (!(point && zero_ok && cmax == 1.0)) {
            double it = lm_exp(sigma_t * tdist * -1.0);
            double ph = smp.g == 0.0 ? 1 / (4 * VPT_PI) : phase_value(smp.g, din, wl);
            dv3 Ls = scl(scl(rad, it), ph);
            if (with_sigma) Ld = scl(scl(scl(scl(Ls, trxt), sigma_s), (1 / prob_wl)), (1 / probSource));
            else Ld = scl(scl(Ls, (1 / prob_wl)), (1 / probSource));
        }
    } else if (point) {
        SECT_BEGIN(swi);
        Ld = point_shadow_ld(S, smp, xt, din, src, sigma_t, with_sigma, sigma_s, trxt, probSource, mag);
        SECT_END(swi, SECT_M_SHADOW_IN);
    }
    SECT_END(sw, SECT_M_SS_SHADOW);
    return Ld;
}

/* equiAngularParams2 (include/volumetricBasicFunctions.h:209-223) with its one draw x given: every
 * other operand is a function of the ray, the light and tMax, so the draw can be taken earlier in the
 * stream's order (it is the stream's next draw either way) and the arithmetic done later */
VPT_DEV double equiangular_setup(const DevScene* __restrict__ S, int src, double tMax, dv3 ro, dv3 rd, double x,
                                 double& D, double& ta, double& tb, double& sample_t)
{
    dv3 dv = sub(sph_p(S, src), ro);
    double dvn = vm_sqrt(dot(dv, dv));
    double proj = dot(dv, rd) / dot(rd, rd);
    D = vm_sqrt(dvn * dvn - proj * proj);
    ta = lm_atan2(0.0 - proj, D);
    tb = lm_atan2(tMax - proj, D);
    sample_t = D * lm_tan((1 - x) * ta + x * tb);
    return sample_t + proj;
}

template <bool COUNT>
VPT_DEV double equiangular_params2(const DevScene* __restrict__ S, Sampler<COUNT>& smp, int src, double tMax, dv3 ro,
                                   dv3 rd, double& D, double& ta, double& tb, double& sample_t)
{
    const double x = smp.next();
    return equiangular_setup(S, src, tMax, ro, rd, x, D, ta, tb, sample_t);
}

/* Equi-angular estimators (1, 4): decide() takes the distance draw and the surface coin, and the
 * equi-angular arithmetic (two atan2, a tan, the pdf) runs in the medium event only -- a surface
 * event (a third of them) never reads it.  The draw rides in Event::pdf, its sign bit marking a
 * ray that hit nothing (EST 4's psurf is 0 there). */

/* equiAngularProb, include/vptSamplingFunctions.h:60-62 */
VPT_DEV double equiangular_prob(double D, double ta, double tb, double s) { return D / vm_fabs(tb - ta) / (s * s + D * D); }

/* ------------------------------------------------------------------ estimators */
/* iterativeVPTracerFree (EST = 0), include/vptShadeMethods.h:1263-1340, and
 * MISVPTTracerRecursive (EST = 1), :1345-1481, split into the pieces a wave schedules
 * separately: decide() = one loop iteration up to the event choice (intersection, light pick,
 * distance sample), then surface_event() or medium_event().  The reference's FF stack holds at
 * most one frame and its MIS recursion is linear, so a path is (ray, throughput, radiance, depth)
 * carried forward. */
struct Medium {
    double sigma_a, sigma_s, g;
    int max_depth;
    double march_step;  /* ray-marching estimators 6-9: step (6, 7) or number of segments (8, 9) */
    int march_light;
};

struct Path {
    dv3 o, d;      /* current ray */
    dv3 beta;      /* throughput */
    dv3 L;         /* radiance gathered so far */
    int depth;     /* loop iteration (the reference's `profundidad`) */
};

struct Event {
    double t;      /* surface distance (MAXFLOAT when the ray escapes) */
    double dist;   /* FF: free-flight distance; MIS: equi-angular distance d_final */
    double pdf;    /* MIS: equi-angular pdf * (1 - psurf) */
    int id;        /* surface sphere */
    int src;       /* light picked for next-event estimation */
};

enum { EV_END = 0, EV_SURF = 1, EV_MED = 2 };

/* VPT_DUP measurement builds: opaque copies / sinks of a path and an event */
VPT_DEV void vpt_opaque(Path& p)
{
    vpt_opaque(p.o);
    vpt_opaque(p.d);
    vpt_opaque(p.beta);
    vpt_opaque(p.L);
    vpt_opaque(p.depth);
}
VPT_DEV void vpt_sink(const Path& p)
{
    vpt_sink(p.o);
    vpt_sink(p.d);
    vpt_sink(p.beta);
    vpt_sink(p.L);
    vpt_sink(p.depth);
}
VPT_DEV void vpt_opaque(Event& e)
{
    vpt_opaque(e.t);
    vpt_opaque(e.dist);
    vpt_opaque(e.pdf);
    vpt_opaque(e.id);
    vpt_opaque(e.src);
}
VPT_DEV void vpt_sink(const Event& e)
{
    vpt_sink(e.t);
    vpt_sink(e.dist);
    vpt_sink(e.pdf);
    vpt_sink(e.id);
    vpt_sink(e.src);
}

/* Russian roulette at the top of a loop iteration (vptShadeMethods.h:1282 / :1354) and the depth
 * cap extension; true = the path continues. */
template <bool COUNT>
VPT_DEV bool continue_path(Sampler<COUNT>& smp, const Path& p, const Medium& m)
{
    if (m.max_depth > 0 && p.depth >= m.max_depth) return false;
    if (COUNT) smp.cnt.iterations++;
    const double q = 1 - 0.6;
    return !(smp.next() < q);
}

/* Estimators (EST = include/vpt.h vpt_estimator):
 *   0 iterativeVPTracerFree          vptShadeMethods.h:1263   free flight, NEE, loop
 *   1 MISVPTTracerRecursive          vptShadeMethods.h:1345   equi-angular, NEE, surface test exp(-σt t)
 *   2 explicitVPTracerRecursiveFree  vptShadeMethods.h:1153   free flight, NEE, recursive sums
 *   3 implicitVPTracerRecursiveFree  vptShadeMethods.h:940    free flight, no NEE, lights at any depth
 *   4 explicitVPTracerRecursive      vptShadeMethods.h:1014   equi-angular, NEE, surface test Tr(x, xs)
 * The recursive ones (1-4) are R = A + B*R'; they are evaluated front to back with a running
 * throughput (same draws and branches; only the final sums are reassociated). */
template <int EST>
VPT_DEV constexpr bool est_free_flight() { return EST == 0 || EST == 2 || EST == 3; }

/* vptShadeMethods.h:1284-1307 (FF), :1357-1426 (MIS), :1166-1205 (explicit free), :950-977
 * (implicit free), :1031-1096 (explicit): what happens to the path this iteration. */
template <int EST, bool COUNT>
VPT_DEV int decide(const DevScene* __restrict__ S, Sampler<COUNT>& smp, Path& p, Event& e, const Medium& m)
{
    const double sigma_t = m.sigma_a + m.sigma_s;
    int id = 0;
    double t = 0.0;
    SECT_BEGIN(di);
#if VPT_DUP == DUP_DECIDE_ISECT
    {
        dv3 o2 = p.o, d2 = p.d;
        vpt_opaque(o2);
        vpt_opaque(d2);
        double t2 = 0;
        int id2 = 0;
        const int h2 = scene_intersect_grouped<VPT_DECIDE_GROUP>(S, smp, o2, d2, t2, id2);
        vpt_sink(t2);
        vpt_sink(id2);
        vpt_sink(h2);
    }
#endif
    const bool hit = scene_intersect_grouped<VPT_DECIDE_GROUP>(S, smp, p.o, p.d, t, id);
    SECT_END(di, SECT_A_ISECT);
    if constexpr (EST == 5) {  /* iterativePathTracer (shadeMethods.h:115-125): nearest hit or end */
        if (COUNT) smp.cnt.iterations++;
        e.t = t;
        e.id = id;
        e.src = 0;
        if (!hit) return EV_END;
        if (S->sph[id].radiance[0] > 0) {  /* a light: the camera ray returns its radiance, a later hit ends */
            if (p.depth < 1) p.L = sph_rad(S, id);
            return EV_END;
        }
        return EV_SURF;
    }
    if (!hit) t = VPT_MAXFLOAT;
    e.t = t;
    e.id = id;
    if (EST == 3) {  /* implicit: no light pick; success pdf freeFlightProb(d) * (1 - Tr(x, xs)) */
        const double TrActual = hit ? transmitance(p.o, add(p.o, scl(p.d, t)), sigma_t) : 0.0;
        e.src = 0;
        e.dist = -lm_log(1 - smp.next()) / sigma_t;
        e.pdf = (sigma_t * lm_exp(sigma_t * e.dist * -1.0)) * (1.0 - TrActual);  /* :977 */
        if (!(e.dist > t)) return EV_MED;
        if (sph_flag(S->m_emitter, id)) {  /* :978-980: a light returns its radiance at any depth */
            p.L = add(p.L, mul(p.beta, sph_rad(S, id)));
            return EV_END;
        }
        return EV_SURF;
    }
    const int count = S->n_emit;
    if (VPT_UNLIKELY(count == 0)) return EV_END;
    e.src = emit_pick(S, (int)(smp.next() * count), count);
    bool surf;
    if (est_free_flight<EST>()) {
        e.dist = -lm_log(1 - smp.next()) / sigma_t;  /* freeFlightSample, vptSamplingFunctions.h:11-14 */
        surf = e.dist > t;
    } else {
        /* MIS: psurf = exp(-σt t) (:1419); explicit: TrActual = Tr(x, xs), 0 on a miss (:1033-1041) */
        const double psurf = EST == 1 ? lm_exp(sigma_t * t * -1.0)
                                      : (hit ? transmitance(p.o, add(p.o, scl(p.d, t)), sigma_t) : 0.0);
        (void)smp.next();  /* equiAngularParams2's draw (volumetricBasicFunctions.h:219), read back by eqa_medium */
        e.pdf = psurf;     /* medium_event: eqa_medium */
        surf = EST == 1 ? smp.next() < psurf : smp.next() <= psurf;  /* :1423 / :1096 */
    }
    if (!surf) return EV_MED;
    if (sph_flag(S->m_emitter, id)) {  /* the path ends on a light; only a camera ray sees it */
        if (p.depth == 0) p.L = EST == 0 ? mul(sph_rad(S, id), p.beta) : sph_rad(S, id);
        return EV_END;
    }
    return EV_SURF;
}

/* surface event: point-light NEE (pLight), sphere-light MIS (MISv2), BSDF continuation (bdsf).
 * cont = false: the path ends at the next roulette draw (the pool's kill prediction), so only the
 * radiance is updated -- the continuation's draws, direction and throughput are never read. */
template <int EST, bool COUNT, int MK = -1, int PT = -1>  /* MK: material, PT: point light (1), if known */
VPT_DEV void surface_event(const DevScene* __restrict__ S, Sampler<COUNT>& smp, Path& p, const Event& e,
                           const Medium& m, bool cont = true, int lk = -1)
{
    /* the light kind: PT when the instantiation fixes it, else lk (wave-uniform: the pool's ring) */
    const int ptk = PT >= 0 ? PT : lk;
    const double sigma_t = m.sigma_a + m.sigma_s;
    const double continueprob = 0.6;
    const int id = e.id, src = e.src;
    const dv3 xs = add(p.o, scl(p.d, e.t));
    const dv3 nx = nrm(sub(xs, sph_p(S, id)));
    if (EST == 3) {  /* implicit: BSDF continuation only, vptShadeMethods.h:983-994 */
        dv3 wi = mk(0, 0, 0);
        double pdf = 0;
        dv3 fs = bdsf<COUNT, MK>(S, smp, wi, p.d, nx, pdf, id);
        wi = nrm(wi);
        const double cosine = dot(nx, wi);
        p.beta = scl(scl(scl(mul(p.beta, fs), (1 / continueprob)), cosine), (1 / pdf));
        p.o = xs;
        p.d = wi;
        p.depth++;
        return;
    }
    const double probSource = 1.0 / S->n_emit;
    const double alpha = S->sph[id].alpha;
    SECT_BEGIN(pl);
    dv3 Ldp = mk(0, 0, 0);
    /* pLight toward a sphere light (PT == 0: the pool's ring) is exactly zero unless x lies inside
     * the light (the shadow ray from the light's centre ends on the light's own surface):
     * Le = 0, and Le fr cos Trs / probSource is then +-0 whenever its other factors are finite --
     * which the distance and the normal decide.  Ld (MISv2) is never -0 (its sums start at +0), so
     * Ldp + Ld == Ld: when that holds in every lane of the wave, the frames, the normalisations and
     * the transmittance of pLight are skipped -- same bits, no draws involved. */
    bool plight_zero = false;
    if (ptk == 0 && S->n_mat3 == 0) {
        const dv3 lx = sub(sph_p(S, src), xs);
        const double dd = dot(lx, lx);
        const double distance = vm_sqrt(dd);  /* visibility()'s test, pathTracingUtilities.h:44-51 */
        const bool fin = dd > 0 && dd < VPT_DBL_MAX && nx.x - nx.x == 0 && nx.y - nx.y == 0 && nx.z - nx.z == 0;
        const bool zero = S->sph[src].r > 0.0001 && !(distance < S->sph[src].r) && fin;
        plight_zero = __ballot(!zero) == 0;
        if (plight_zero) smp.tests(2 * S->n);  /* what visibility + the visibilityVPT miss would count */
    }
    /* the normal's frame, formed once and shared by pLight, MISv2 and the diffuse bdsf below (VPT_FRAME_CSE;
     * A/B ab_r06i: formed here and held through pLight's shadow ray 37.89 / 169.5 ms, formed after pLight
     * with pLight forming its own 37.95 / 170.2, base 38.58 / 172.4) */
    Frame Fn = {};
    if (MK == 0 && VPT_FRAME_CSE) Fn = make_frame(nx);
#if VPT_DUP == DUP_PLIGHT
    if (!plight_zero) {
        dv3 xs2 = xs, nx2 = nx, d2 = p.d;
        int id2 = id, src2 = src;
        double a2 = alpha;
        Frame F2 = Fn;
        vpt_opaque(xs2);
        vpt_opaque(nx2);
        vpt_opaque(d2);
        vpt_opaque(id2);
        vpt_opaque(src2);
        vpt_opaque(a2);
        vpt_opaque(F2);
        Sampler<COUNT> s2 = smp;
        if (MK == 0 && VPT_PL_REUSE && VPT_FRAME_CSE) {
            double T2;
            const dv3 pl2 = p_light_nee<COUNT, MK, PT>(S, s2, id2, xs2, nx2, d2, src2, a2, F2, sigma_t, T2);
            vpt_sink(scl(scl(pl2, T2), (1 / probSource)));
        } else {
            double Trs2 = transmitance(xs2, sph_p(S, src2), sigma_t);
            vpt_sink(scl(scl(p_light<COUNT, MK, PT>(S, s2, id2, xs2, nx2, d2, src2, a2), Trs2), (1 / probSource)));
        }
    }
#endif
    if (!plight_zero) {
        if (MK == 0 && VPT_PL_REUSE && VPT_FRAME_CSE) {
            double Trs;
            const dv3 pl = p_light_nee<COUNT, MK, PT>(S, smp, id, xs, nx, p.d, src, alpha, Fn, sigma_t, Trs);
            Ldp = scl(scl(pl, Trs), (1 / probSource));
        } else {
            double Trs = transmitance(xs, sph_p(S, src), sigma_t);
            Ldp = scl(scl(p_light<COUNT, MK, PT>(S, smp, id, xs, nx, p.d, src, alpha), Trs), (1 / probSource));
        }
    }
    SECT_END(pl, SECT_S_PLIGHT);
    SECT_BEGIN(mis);
    /* the fused three-ray MISv2 for diffuse surfaces only: metal and dielectric take the sequential
     * one (round 3: scratch 448 -> 240 B/lane, FF 51.99 -> 51.53 ms) */
#if VPT_DUP == DUP_MIS
    if (MK == 0 && S->n_mis == 2) {
        dv3 xs2 = xs, nx2 = nx, d2 = p.d;
        int id2 = id;
        vpt_opaque(xs2);
        vpt_opaque(nx2);
        vpt_opaque(d2);
        vpt_opaque(id2);
        Sampler<COUNT> s2 = smp;
        vpt_opaque(s2.X);
        Frame F2 = Fn;
        vpt_opaque(F2);
        vpt_sink(mis_v2_two_lights<COUNT, MK>(S, s2, id2, xs2, nx2, d2, alpha, sigma_t, F2));
        vpt_sink(s2.X);
    }
#endif
    const dv3 Ld = MK == 0 && S->n_mis == 2 ? mis_v2_two_lights<COUNT, MK>(S, smp, id, xs, nx, p.d, alpha, sigma_t, Fn)
                                            : mis_v2<COUNT, MK>(S, smp, id, xs, nx, p.d, alpha, sigma_t);
    SECT_END(mis, SECT_S_MIS);
    SECT_BEGIN(bd);
    /* (the radiance update reads the throughput before bdsf's update, as in the reference) */
    if (EST == 0) p.L = add(p.L, scl(mul(add(Ldp, Ld), p.beta), (1 / continueprob)));
    else p.L = add(p.L, mul(p.beta, scl(add(Ldp, Ld), (1 / continueprob))));
#if VPT_DUP == DUP_BDSF
    if (cont) {
        dv3 wi2 = mk(0, 0, 0), d2 = p.d, nx2 = nx, b2 = p.beta;
        int id2 = id;
        vpt_opaque(d2);
        vpt_opaque(nx2);
        vpt_opaque(b2);
        vpt_opaque(id2);
        double pdf2 = 0;
        Sampler<COUNT> s2 = smp;
        vpt_opaque(s2.X);
        Frame F2 = Fn;
        vpt_opaque(F2);
        dv3 fs2;
        if (MK == 0 && VPT_FRAME_CSE) {
            wi2 = cosine_hemispheric(s2, F2);
            fs2 = scl(sph_c(S, id2), (1 / VPT_PI));
            pdf2 = hemi_cosine_prob(dot(nx2, wi2));
        } else {
            fs2 = bdsf<COUNT, MK>(S, s2, wi2, d2, nx2, pdf2, id2);
        }
        wi2 = nrm(wi2);
        vpt_sink(scl(scl(scl(mul(b2, fs2), (1 / continueprob)), dot(nx2, wi2)), (1 / pdf2)));
        vpt_sink(wi2);
        vpt_sink(s2.X);
    }
#endif
    if (cont) {
        dv3 wi = mk(0, 0, 0);
        double pdf = 0;
        dv3 fs;
        if (MK == 0 && VPT_FRAME_CSE) {  /* bdsf's diffuse branch (vptShadeMethods.h:16-59) on the shared frame */
            wi = cosine_hemispheric(smp, Fn);
            fs = scl(sph_c(S, id), (1 / VPT_PI));
            pdf = hemi_cosine_prob(dot(nx, wi));
        } else {
            fs = bdsf<COUNT, MK>(S, smp, wi, p.d, nx, pdf, id);
        }
        wi = nrm(wi);
        double cosine = dot(nx, wi);
        p.beta = scl(scl(scl(mul(p.beta, fs), (1 / continueprob)), cosine), (1 / pdf));
        p.o = xs;
        p.d = wi;
        p.depth++;
    }
    SECT_END(bd, SECT_S_BDSF);
}

/* medium event: single-scattering NEE toward the picked light, phase-function continuation.
 * LT: 1 point light, 0 not, -1 unknown (the pool kernel's medium rings are keyed by it) */
/* One bounce of iterativePathTracer (include/shadeMethods.h:126-160) at the surface hit of event e,
 * for the pool kernel: pLight for every r == 0 sphere in index order and MIS without transmittance
 * (Ld = term + Ld), the roulette draw (q = 0.4, after the NEE: a killed path drops this vertex's Ld),
 * then the BSDF continuation; Accum (p.L) += fs Ld factor, fs (p.beta) *= fs1, factor (carried in
 * the event's pdf slot) *= cos / (prob 0.6).  Same operations as trace_surface_pt.  Returns true when
 * the roulette ends the path.  MK: the hit sphere's material when the surface ring fixes it. */
template <bool COUNT, int MK = -1>
VPT_DEV bool surface_event_pt(const DevScene* __restrict__ S, Sampler<COUNT>& smp, Path& p, Event& e)
{
    const double q = 0.4;
    const double continueprob = 1.0 - q;
    const int id = e.id;
    const dv3 x = add(p.o, scl(p.d, e.t));
    const dv3 nx = nrm(sub(x, sph_p(S, id)));
    const double alpha = S->sph[id].alpha;
    dv3 Ld = mk(0, 0, 0);
    const int n = S->n;
    for (int l = 0; l < n; ++l)  /* wave-uniform: scalar loads of the scene */
        if (S->sph[l].r == 0) Ld = add(p_light<COUNT, MK, -1, true>(S, smp, id, x, nx, p.d, l, alpha), Ld);
    Ld = add(mis_v2<COUNT, MK, false>(S, smp, id, x, nx, p.d, alpha, 0.0), Ld);
    if (smp.next() < q) return true;
    double prob = 0;
    dv3 wi = mk(0, 0, 0);
    const dv3 fs1 = bdsf<COUNT, MK>(S, smp, wi, p.d, nx, prob, id);
    p.o = x;
    p.d = wi;
    const double cosine = dot(nx, wi);
    p.L = add(p.L, scl(mul(p.beta, Ld), e.pdf));
    p.beta = mul(p.beta, fs1);
    e.pdf = e.pdf * cosine * (1 / (prob * continueprob));
    p.depth++;
    return false;
}

/* the deferred equi-angular arithmetic of decide(): d_final and its pdf from the ray, the light,
 * tMax = e.t, decide()'s psurf (carried in e.pdf) and its equi-angular draw -- the value of the
 * stream state one draw before X, the state after decide()'s last draw (the surface coin): erand48
 * steps back by X -> a^-1 (X - c) mod 2^48 -- the operations decide() performed in round 2, in the
 * same order */
template <int EST>
VPT_DEV void eqa_medium(const DevScene* __restrict__ S, const Path& p, const Event& e, uint64_t X, double& dist,
                        double& pdf)
{
    const double t = e.t, psurf = e.pdf;
    const double x = vpt_erand48_value(((X - 0xBull) * 0xDFE05BCB1365ull) & 0xFFFFFFFFFFFFull);
    double D = 0, ta = 0, tb = 0, sd = 0;
    dist = equiangular_setup(S, e.src, t, p.o, p.d, x, D, ta, tb, sd);
    pdf = equiangular_prob(D, ta, tb, sd) * (1 - psurf);
}

/* the medium event after single scattering's Ld (vptShadeMethods.h:1318-1332 / :1461-1477): the
 * radiance update, then -- unless the path ends at the next roulette draw (cont = false) -- the phase
 * sample and the throughput.  T: transmittance to xt, pdf: the equi-angular pdf (estimators 1, 4). */
#if VPT_DUP == DUP_PHASE
#define VPT_DUP_PHASE()                      \
    {                                        \
        dv3 d2 = p.d;                        \
        vpt_opaque(d2);                      \
        Sampler<COUNT> s2 = smp;             \
        vpt_opaque(s2.X);                    \
        vpt_sink(phase_sample(s2, d2));      \
        vpt_sink(s2.X);                      \
    }
#else
#define VPT_DUP_PHASE() \
    do {                \
    } while (0)
#endif
template <int EST, bool COUNT>
VPT_DEV void medium_tail(Sampler<COUNT>& smp, Path& p, dv3 Ld, double T, double pdf, dv3 xt, const Medium& m, bool cont)
{
    const double sigma_a = m.sigma_a, sigma_s = m.sigma_s;
    const double sigma_t = sigma_a + sigma_s;
    const double continueprob = 0.6;
    if (EST == 0) {
        p.L = add(p.L, scl(scl(mul(Ld, p.beta), (sigma_s / sigma_t)), (1 / continueprob)));
        if (!cont) return;
        SECT_BEGIN(ph);
        VPT_DUP_PHASE();
        dv3 wi = phase_sample(smp, p.d);
        SECT_END(ph, SECT_M_PHASE);
        p.beta = scl(scl(p.beta, (sigma_s / sigma_t)), (1 / continueprob));
        p.d = wi;
    } else if (EST == 2) {  /* vptShadeMethods.h:1252-1258 */
        p.L = add(p.L, mul(p.beta, scl(scl(Ld, (sigma_s / sigma_t)), (1 / continueprob))));
        if (!cont) return;
        VPT_DUP_PHASE();
        dv3 wi = phase_sample(smp, p.d);
        p.beta = scl(scl(p.beta, (sigma_s / sigma_t)), (1 / continueprob));
        p.d = wi;
    } else {
        p.L = add(p.L, mul(p.beta, scl(scl(Ld, (1 / pdf)), (1 / continueprob))));
        if (!cont) return;
        SECT_BEGIN(ph);
        VPT_DUP_PHASE();
        dv3 wi = phase_sample(smp, p.d);
        SECT_END(ph, SECT_M_PHASE);
        p.beta = scl(scl(scl(scl(p.beta, sigma_s), T), (1 / continueprob)), (1 / pdf));
        p.d = wi;
    }
    p.o = xt;
    p.depth++;
}

/* medium event: single-scattering NEE toward the picked light, phase-function continuation.
 * LT: 1 point light, 0 not, -1 unknown (the pool kernel's medium rings are keyed by it).  cont = false:
 * radiance only (surface_event). */
template <int EST, bool COUNT, int LT = -1>
VPT_DEV void medium_event(const DevScene* __restrict__ S, Sampler<COUNT>& smp, Path& p, const Event& e0,
                          const Medium& m, bool cont = true)
{
    const double sigma_a = m.sigma_a, sigma_s = m.sigma_s;
    const double sigma_t = sigma_a + sigma_s;
    const double continueprob = 0.6;
    Event e = e0;
    SECT_BEGIN(eq);
#if VPT_DUP == DUP_EQA
    if (EST == 1 || EST == 4) {
        Path p2 = p;
        Event e2 = e0;
        uint64_t X2 = smp.X;
        vpt_opaque(p2);
        vpt_opaque(e2);
        vpt_opaque(X2);
        double dd = 0, pp = 0;
        eqa_medium<EST>(S, p2, e2, X2, dd, pp);
        vpt_sink(dd);
        vpt_sink(pp);
    }
#endif
    if (EST == 1 || EST == 4) eqa_medium<EST>(S, p, e0, smp.X, e.dist, e.pdf);
    SECT_END(eq, SECT_M_EQA);
    dv3 xt = add(p.o, scl(p.d, e.dist));
    if (EST == 3) {  /* implicit: vptShadeMethods.h:1000-1006 */
        const double T = transmitance(p.o, xt, sigma_t);
        VPT_DUP_PHASE();
        dv3 wi = phase_sample(smp, p.d);
        p.beta = scl(scl(scl(scl(p.beta, sigma_s), T), (1 / continueprob)), (1 / e.pdf));
        p.d = wi;
        p.o = xt;
        p.depth++;
        return;
    }
    const double probSource = 1.0 / S->n_emit;
    /* the updates below absorb a +-0 Ld exactly when the throughput (and, equi-angular, 1 / pdf) is
     * finite (p.L is never -0: it starts at +0 and only adds) -- single_scattering's H5 shortcut */
    const bool zero_ok = p.beta.x - p.beta.x == 0 && p.beta.y - p.beta.y == 0 && p.beta.z - p.beta.z == 0 &&
                         (!(EST == 1 || EST == 4) || (1 / e.pdf) - (1 / e.pdf) == 0);
    /* singleScattering (estimators 1, 4) weighs by the transmittance to xt; freeSingleScattering not */
    constexpr bool ws = EST == 1 || EST == 4;
    double T = 1.0;
    if (ws) {
        SECT_BEGIN(tr);
        T = transmitance(p.o, xt, sigma_t);
        SECT_END(tr, SECT_M_TR);
    }
    SECT_BEGIN(ss);
#if VPT_DUP == DUP_SS
    {
        dv3 xt2 = xt, d2 = p.d;
        int src2 = e.src;
        double T2 = T;
        vpt_opaque(xt2);
        vpt_opaque(d2);
        vpt_opaque(src2);
        vpt_opaque(T2);
        Sampler<COUNT> s2 = smp;
        vpt_opaque(s2.X);
        vpt_sink(single_scattering<COUNT, LT>(S, s2, xt2, d2, src2, sigma_t, ws, sigma_s, T2, probSource, zero_ok));
        vpt_sink(s2.X);
    }
#endif
    const dv3 Ld = single_scattering<COUNT, LT>(S, smp, xt, p.d, e.src, sigma_t, ws, sigma_s, T, probSource, zero_ok);
    SECT_END(ss, SECT_M_SS);
    medium_tail<EST, COUNT>(smp, p, Ld, T, e.pdf, xt, m, cont);
}

/* iterativePathTracer, include/shadeMethods.h:104-163 (estimator 5): surface-only path tracing.
 * Per iteration: nearest hit or end (:117-119); a light (radiance.x > 0) seen by the camera ray
 * returns its radiance, a later one ends the path (:122-125); pLight for every r == 0 sphere in
 * index order, then MIS (:133-141, Ld = term + Ld); the roulette draw, which drops this vertex's
 * Ld (:143-147); the BSDF continuation (:149, BDSF == bdsf), unnormalised (:151-153).  prob and wi
 * live across iterations as in the reference (a material-3 hit leaves them unchanged). */
template <bool COUNT>
__device__ static dv3 trace_surface_pt(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d)
{
    dv3 Accum = mk(0, 0, 0), fs = mk(1, 1, 1), Ld = mk(0, 0, 0), wi = mk(0, 0, 0);
    int bounces = 0;
    double factor = 1;
    const double q = 0.4;
    const double continueprob = 1.0 - q;
    double prob = 0;
    const int n = S->n;
    while (true) {
        if (COUNT) smp.cnt.iterations++;
        double t;
        int id = 0;
        if (!scene_intersect(S, smp, o, d, t, id, false)) break;
        if (S->sph[id].radiance[0] > 0) {
            if (bounces < 1) return sph_rad(S, id);
            break;
        }
        const dv3 x = add(o, scl(d, t));
        const dv3 nx = nrm(sub(x, sph_p(S, id)));
        const double alpha = S->sph[id].alpha;
        for (int l = 0; l < n; ++l)  /* wave-uniform: scalar loads of the scene */
            if (S->sph[l].r == 0) Ld = add(p_light<COUNT>(S, smp, id, x, nx, d, l, alpha), Ld);
        Ld = add(mis_v2<COUNT, -1, false>(S, smp, id, x, nx, d, alpha, 0.0), Ld);
        if (smp.next() < q) break;
        const dv3 fs1 = bdsf<COUNT>(S, smp, wi, d, nx, prob, id);
        o = x;
        d = wi;
        const double cosine = dot(nx, wi);
        Accum = add(Accum, scl(mul(fs, Ld), factor));
        fs = mul(fs, fs1);
        factor = factor * cosine * (1 / (prob * continueprob));
        bounces++;
        Ld = mk(0, 0, 0);
    }
    return Accum;
}

/* rayMarching3, include/rayMarchingMethods.h:330-384 (estimator 6): constant-step marching along the
 * camera ray up to its first hit (no hit: black), single scattering from light m.march_light at
 * every step i < t / step.  As written: step points measured from the ray origin (:351), their
 * transmittance from the hit point x (:353); no random draw.  The shadow rays go through
 * visibility() (a sphere light's own surface blocks them).  Steps per ray are capped at
 * VPT_MARCH_MAX_STEPS (the reference has no cap) so that every wave ends; a capped ray returns NaN. */
#ifndef VPT_MARCH_MAX_STEPS
#define VPT_MARCH_MAX_STEPS (1 << 22)
#ifndef VPT_MARCH_REUSE
#define VPT_MARCH_REUSE 1
#endif
#endif
template <bool COUNT>
__device__ static dv3 trace_ray_marching(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d,
                                         const Medium& m, const double (*light_oc)[4] = nullptr)
{
    const double sigma_a = m.sigma_a, sigma_s = m.sigma_s, step = m.march_step;
    const int src = m.march_light;
    double t;
    int id = 0;
    if (!scene_intersect(S, smp, o, d, t, id, false)) return mk(0, 0, 0);
    const dv3 x = add(o, scl(d, t));
    dv3 Li = mk(0, 0, 0);
    const dv3 lp = sph_p(S, src);
    const double lr = S->sph[src].r;
    const bool l3 = sph_flag(S->m_mat3, src);
    const double steps = t / step;
    if (!(steps < (double)VPT_MARCH_MAX_STEPS)) return mk(__builtin_nan(""), __builtin_nan(""), __builtin_nan(""));
    for (int i = 0; i < steps; i++) {
        if (COUNT) smp.cnt.iterations++;
        const dv3 xt = add(o, scl(scl(d, step), (double)i));
        const double T = transmitance(x, xt, sigma_a + sigma_s);
        const double phase = 1 / (4 * VPT_PI);  /* isotropicPhaseFunction, volumetricBasicFunctions.h:59-62 */
        const dv3 wc = sub(lp, xt);
        const double normwc = dot(wc, wc);
        /* VPT_MARCH_REUSE: visibility's distance and the light's transmittance are the same root of normwc,
         * its direction nrm(wc) -- formed once (visibility_pre) */
        double dist = 0.0;
        bool vis;
        if (VPT_MARCH_REUSE) {  /* visibility(S, smp, lp, xt, false, lr, l3, light_oc) with its distance kept */
            dist = vm_sqrt(normwc);
            if (lr > 0.0001 && !(dist < lr)) {
                smp.tests(S->n);
                vis = false;
            } else {
                const dv3 lx = scl(nrm(wc), -1);
                int idv = 0;
                double tv;
                if (light_oc != nullptr) scene_intersect_grouped_oc<VPT_ISECT_GROUP_ALL, COUNT, true>(S, smp, light_oc, lx, tv, idv);
                else scene_isect<COUNT, true>(S, smp, lp, lx, tv, idv, false);
                vis = tv > dist || tv == 0;
            }
        } else {
            vis = visibility<COUNT, true>(S, smp, lp, xt, false, lr, l3, light_oc);
        }
        if (vis) {
            const dv3 Le = scl(sph_rad(S, src), (1 / normwc));
            const double Tl = VPT_MARCH_REUSE ? lm_exp((sigma_a + sigma_s) * dist * -1.0) : transmitance(xt, lp, sigma_a + sigma_s);
            const dv3 Ls = scl(Le, (phase * Tl));
            Li = add(Li, scl(scl(scl(Ls, T), sigma_s), step));
        } else {
            Li = add(Li, mk(0, 0, 0));
        }
    }
    return Li;
}

/* The step loop of rayMarching (include/rayMarchingMethods.h:55-99), of rayMarchingGlobal's tail
 * (:208-254) and of rayMarching2 (:280-325): points xt = o + d*step*i for i < n_steps, their
 * transmittance from x, one solidAngle sample toward sphere `light`, its first hit; the sample
 * scores when the hit id (0 on a miss: the reference's initialiser) is the light.  Capped like
 * trace_ray_marching (NaN past VPT_MARCH_MAX_STEPS). */
template <bool COUNT>
VPT_DEV dv3 march_solid_angle(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d, dv3 x, double n_steps,
                              double step, int light, double sigma_t, double sigma_s)
{
    if (!(n_steps < (double)VPT_MARCH_MAX_STEPS)) return mk(__builtin_nan(""), __builtin_nan(""), __builtin_nan(""));
    dv3 Li = mk(0, 0, 0);
    const dv3 lp = sph_p(S, light);
    const double lr = S->sph[light].r;
    for (int i = 0; i < n_steps; i++) {
        if (COUNT) smp.cnt.iterations++;
        const dv3 xt = add(o, scl(scl(d, step), (double)i));
        const double T = transmitance(x, xt, sigma_t);
        const double phase = 1 / (4 * VPT_PI);  /* isotropicPhaseFunction */
        dv3 wc = sub(lp, xt);
        const double normcx = vm_sqrt(dot(wc, wc));
        wc = scl(wc, (1 / normcx));
        const double cmax = vm_sqrt(1 - (lr / normcx) * (lr / normcx));
        const dv3 wi = solid_angle_dir(smp, wc, cmax);
        double t2;
        int id2 = 0;
        scene_isect(S, smp, xt, wi, t2, id2, false);
        if (id2 == light) {
            const dv3 Ls = scl(sph_rad(S, light), (phase * transmitance(xt, lp, sigma_t)));
            const double prob = solid_angle_prob(cmax);
            Li = add(Li, scl(scl(scl(Ls, (T * 1 / prob)), sigma_s), step));
        } else {
            Li = add(Li, mk(0, 0, 0));
        }
    }
    return Li;
}

/* rayMarching, include/rayMarchingMethods.h:34-103: `steps` equal segments of the ray up to its first
 * hit, solid-angle samples toward the hard-coded sphere 5; a light hit scores nothing (:48-51).
 * x_new / idsource: the hit point and sphere (unchanged on a miss). */
template <bool COUNT>
VPT_DEV dv3 ray_marching_explicit(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d, double sigma_t,
                                  double sigma_s, double steps, dv3& x_new, int& idsource)
{
    double t;
    int id = 0;
    if (!scene_isect(S, smp, o, d, t, id, false)) return mk(0, 0, 0);
    idsource = id;
    const dv3 x = add(o, scl(d, t));
    x_new = x;
    if (S->sph[id].radiance[0] > 0) return mk(0, 0, 0);
    return march_solid_angle(S, smp, o, d, x, steps, t / steps, 5, sigma_t, sigma_s);
}

/* rayMarching2, include/rayMarchingMethods.h:262-327 (estimator 7): steps of m.march_step toward
 * sphere m.march_light by solid-angle sampling, plus the transmitted radiance of a light hit */
template <bool COUNT>
__device__ static dv3 trace_ray_marching2(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d,
                                          const Medium& m)
{
    const double step = m.march_step;
    double t;
    int id = 0;
    if (!scene_isect(S, smp, o, d, t, id, false)) return mk(0, 0, 0);
    const dv3 x = add(o, scl(d, t));
    dv3 Lo = mk(0, 0, 0);
    if (S->sph[id].radiance[0] > 0) Lo = scl(sph_rad(S, id), transmitance(o, x, m.sigma_a + m.sigma_s));
    const dv3 Li = march_solid_angle(S, smp, o, d, x, t / step, step, m.march_light, m.sigma_a + m.sigma_s, m.sigma_s);
    return add(Li, Lo);
}

/* rayMarchingGlobal, include/rayMarchingMethods.h:106-256 (estimator 8): up to 10 diffuse bounces,
 * each a solid-angle sample toward sphere 5 and a cosine-sampled ray marched by rayMarching in
 * m.march_step segments, then the camera ray marched from the last hit point.  As written: Ld keeps
 * its value when the light sample misses (:169); every bounce's transmittance runs from the camera
 * origin to the current x (:195). */
template <bool COUNT>
__device__ static dv3 trace_ray_marching_global(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d,
                                                const Medium& m)
{
    const double sigma_s = m.sigma_s, segmentos = m.march_step;
    const double sigma_t = m.sigma_a + m.sigma_s;
    double t;
    int id = 0;
    if (!scene_isect(S, smp, o, d, t, id, false)) return mk(0, 0, 0);
    dv3 x = add(o, scl(d, t));
    dv3 Lo = mk(0, 0, 0);
    if (S->sph[id].radiance[0] > 0) return scl(sph_rad(S, id), transmitance(o, x, sigma_t));
    dv3 fs = mk(1, 1, 1), Ld = mk(0, 0, 0);
    double factor = 1;
    const dv3 l5 = sph_p(S, 5);
    const double r5 = S->sph[5].r;
    for (int i = 0; i < 10; i++) {
        if (COUNT) smp.cnt.iterations++;
        const dv3 fr = scl(sph_c(S, id), (1 / VPT_PI));
        const dv3 n = nrm(sub(x, sph_p(S, id)));
        dv3 wc = sub(l5, x);
        const double normcx = vm_sqrt(dot(wc, wc));
        wc = scl(wc, (1 / normcx));
        const double cmax = vm_sqrt(1 - (r5 / normcx) * (r5 / normcx));
        const dv3 wi = solid_angle_dir(smp, wc, cmax);
        double t_aux;
        int id_aux = 0;
        scene_isect(S, smp, x, wi, t_aux, id_aux, false);
        if (id_aux == 5) {
            const dv3 Le = scl(sph_rad(S, 5), transmitance(x, l5, sigma_t));
            Ld = scl(scl(mul(Le, fr), (1 / solid_angle_prob(cmax))), dot(n, wi));
        }
        const dv3 wray = cosine_hemispheric(smp, n);
        const double prob = hemi_cosine_prob(dot(n, wray));
        dv3 x_new = mk(0, 0, 0);
        const dv3 Lm = ray_marching_explicit(S, smp, x, wray, sigma_t, sigma_s, segmentos, x_new, id);
        Ld = add(Ld, scl(scl(mul(Lm, fr), dot(n, wray)), (1 / prob)));
        Lo = add(Lo, scl(scl(mul(Ld, fs), transmitance(o, x, sigma_t)), factor));
        if (Lm.x == 0 && Lm.y == 0 && Lm.z == 0) return Lo;
        fs = mul(fs, fr);
        factor = factor * dot(n, wray) * (1 / (prob));
        x = x_new;
    }
    const dv3 Li = march_solid_angle(S, smp, o, d, x, segmentos, t / segmentos, 5, sigma_t, sigma_s);
    return add(Li, Lo);
}

/* punctualVolumetric, include/rayMarchingMethods.h:12-31: single scattering at x from the centre of
 * sphere idsource (visibilityVPT, multipleT); no draw */
template <bool COUNT>
VPT_DEV dv3 punctual_volumetric(const DevScene* __restrict__ S, Sampler<COUNT>& smp, int idsource, dv3 x, double phase,
                                double sigma_t, double sigma_s)
{
    const dv3 light = sph_p(S, idsource);
    if (visibility<COUNT, true>(S, smp, light, x, true, S->sph[idsource].r, S->geo[idsource].mat3)) {
        dv3 Le = sph_rad(S, idsource);
        const double distanceLight = dot(sub(light, x), sub(light, x));
        Le = scl(Le, (1 / distanceLight));
        const dv3 Ls = scl(scl(Le, phase), multiple_t(S, smp, x, light, sigma_t));
        return scl(Ls, sigma_s);
    }
    return mk(0, 0, 0);
}

/* One camera sample, sequentially (the reference's per-sample call; used by vpt_trace_batch). */
template <int EST, bool COUNT>
__device__ static dv3 trace_sample(const DevScene* __restrict__ S, Sampler<COUNT>& smp, dv3 o, dv3 d, const Medium& m,
                                  const double (*march_oc)[4] = nullptr)
{
    if constexpr (EST == 5) {
        return trace_surface_pt<COUNT>(S, smp, o, d);
    } else if constexpr (EST == 6) {
        return trace_ray_marching<COUNT>(S, smp, o, d, m, march_oc);
    } else if constexpr (EST == 7) {
        return trace_ray_marching2<COUNT>(S, smp, o, d, m);
    } else if constexpr (EST == 8) {
        return trace_ray_marching_global<COUNT>(S, smp, o, d, m);
    } else if constexpr (EST == 9) {  /* rayMarching: the Color it returns (sigma_t = sigma_a + sigma_s) */
        dv3 x_new = mk(0, 0, 0);
        int idsource = 0;
        return ray_marching_explicit<COUNT>(S, smp, o, d, m.sigma_a + m.sigma_s, m.sigma_s, m.march_step, x_new, idsource);
    } else {
        Path p;
        p.o = o;
        p.d = d;
        p.beta = mk(1, 1, 1);
        p.L = mk(0, 0, 0);
        p.depth = 0;
        Event e;
        e.pdf = 0;
        /* counting mode also checks the invariant the pool's kill-predicting rings rest on (vpt_pool.h
         * stage_a): from the state after decide(), a diffuse surface event (2 n_mis + 4 draws) or a
         * medium event (4 draws) and the next roulette draw end at the state the LCG jump predicts */
        constexpr bool CHECK = COUNT && (EST == 0 || EST == 1 || EST == 2 || EST == 4);
        uint64_t xd = 0, ja = 0, jc = 0;
        bool pend = false;
        while (continue_path(smp, p, m)) {
            if (CHECK && pend && smp.X != vpt_erand48_skip(xd, ja, jc)) smp.cnt.draw_mismatch++;
            pend = false;
            int ev = decide<EST>(S, smp, p, e, m);
            if (ev == EV_END) break;
            if (CHECK) {
                xd = smp.X;
                if (ev == EV_MED) {
                    vpt_erand48_jump(5, &ja, &jc);
                    pend = true;
                } else if ((sph_flag(S->m_skey1, e.id) | sph_flag(S->m_skey2, e.id)) == 0) {
                    ja = S->kp_sa;
                    jc = S->kp_sc;
                    pend = true;
                }
            }
            if (ev == EV_SURF) surface_event<EST>(S, smp, p, e, m);
            else medium_event<EST>(S, smp, p, e, m);
        }
        /* (a path the roulette ended drew it too; one the depth cap ended did not) */
        if (CHECK && pend && !(m.max_depth > 0 && p.depth >= m.max_depth) && smp.X != vpt_erand48_skip(xd, ja, jc))
            smp.cnt.draw_mismatch++;
        return p.L;
    }
}

}  // namespace vpt

#endif
