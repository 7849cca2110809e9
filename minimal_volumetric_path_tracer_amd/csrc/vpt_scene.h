/*
 * vpt_scene.h -- device-resident scene (host + device view).
 *
 * Replaces the reference's global std::vector<Sphere> spheres (include/Sphere.h:49,
 * include/Sphere.cpp:7-107) and the per-iteration emitter scan of the estimators
 * (include/vptShadeMethods.h:1293-1303, :1389-1407; include/misSamplingFunctions.h:106).
 * Two views of each sphere: a 48-byte GeoSphere read by the intersection loop with a
 * wave-uniform index (scalar loads), and the 144-byte reference record for shading lookups by a
 * per-lane id.  Derived lists are computed once per scene on the host.
 */
#ifndef VPT_SCENE_H
#define VPT_SCENE_H

#include <stdint.h>
#include "../../include/vpt.h"

struct GeoSphere {
    double px, py, pz;  /* centre */
    double r2;          /* fl(r*r), exactly the product Sphere::intersect forms (Sphere.h:30) */
    int32_t mat3;       /* material == 3 (skipped by intersectVPT) */
    int32_t emitter;    /* any radiance channel > 0 (vptShadeMethods.h:1296) */
    int32_t skey;       /* surface-stage ring of the pool kernel: 0 diffuse, 2 metal, 3 other */
    int32_t point;      /* r == 0: a point light (its NEE casts a shadow ray) */
};

struct DevScene {
    int32_t n;          /* number of spheres */
    int32_t n_emit;     /* emitters (idsource candidates) */
    int32_t n_mis;      /* spheres with r > 0 && radiance.x > 0 (MISv2 light loop) */
    int32_t n_mat3;     /* material-3 spheres */
    int32_t n_non3;     /* n - n_mat3 */
    int32_t emit_all_radiance; /* 1: every sphere with a nonzero radiance channel is in emit[] (MISv2's BSDF-ray skip) */
    int32_t pad_[2];
    /* per-sphere flags as bit masks (bit i = sphere i; VPT_MAX_SPHERES <= 64), read with a per-lane id
     * by shifts of wave-uniform words instead of per-lane loads of GeoSphere fields */
    uint64_t m_emitter, m_point, m_mat3, m_skey1, m_skey2;  /* skey = m_skey1 bit + 2 * m_skey2 bit */
    /* erand48 jump (A, C) from the state after decide() to the roulette draw that follows a diffuse
     * surface event: 2 n_mis + 4 draws of the event, then the roulette (the pool's kill prediction) */
    uint64_t kp_sa, kp_sc;
    uint64_t pad2_[1];
    int32_t emit[VPT_MAX_SPHERES];
    int32_t mis_light[VPT_MAX_SPHERES];
    GeoSphere geo[VPT_MAX_SPHERES];
    vpt_sphere sph[VPT_MAX_SPHERES];
};
static_assert(VPT_MAX_SPHERES <= 64, "DevScene's per-sphere bit masks (1ull << i) hold at most 64 spheres");

#endif
