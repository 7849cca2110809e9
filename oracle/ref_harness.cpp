/*
 * ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libvpt_ref.so).
 *
 * Drives the REFERENCE's own functions, compiled in place from /root/reference/include (never
 * copied), deterministically, so that golden vectors can be generated from the real reference
 * code.  Only tests/, tests/golden/make_golden.py, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * Determinism: the reference draws every random number with libc erand48(seed) on the global
 * `seed` (include/Vector.h:38).  The harness leaves that untouched and only SETS the global
 * state before each camera sample to the per-sample start state of oracle/oracle_rng.h, so the
 * reference consumes exactly the stream the build consumes.  Uninitialised locals in the
 * reference (e.g. idHitted, include/volumetricBasicFunctions.h:324; costhetaMax,
 * include/misSamplingFunctions.h:108) are defined as zero by -ftrivial-auto-var-init=zero.
 * The pixel loop mirrors main() (src/rt.cpp:752-805) with the jitter draws in clang's order,
 * x first.
 */
#include <cstdint>
#include <cstring>
#include <vector>

#include "Sphere.h"
#include "Vector.h"
#include "Ray.h"
#include "mathUtilities.h"
#include "pathTracingUtilities.h"
#include "samplingFunctions.h"
#include "microFacetUtilities.h"
#include "misSamplingFunctions.h"
#include "volumetricBasicFunctions.h"
#include "vptSamplingFunctions.h"
#include "vptShadeMethods.h"
#include "shadeMethods.h"
#include "rayMarchingMethods.h"

extern "C" {
#include "oracle_rng.h"
}

namespace {

struct PackedSphere {  // byte layout of reference Sphere (include/Sphere.h:14-21), 144 B
    double r;
    double p[3];
    double c[3];
    double radiance[3];
    int32_t material;
    int32_t pad_;
    double eta[3];
    double kappa[3];
    double alpha;
};
static_assert(sizeof(PackedSphere) == 144, "packed sphere must be 144 bytes");

std::vector<Sphere>& default_scene()
{
    static std::vector<Sphere> saved = spheres;  // first use happens before any ref_set_scene
    return saved;
}

inline Vector V(const double* a) { return Vector(a[0], a[1], a[2]); }
inline void put(const Vector& v, double* o) { o[0] = v.x; o[1] = v.y; o[2] = v.z; }
inline void set_state(uint64_t X) { orc_state_to_xsubi(X, seed); }
inline uint64_t get_state() { return orc_xsubi_to_state(seed); }

}  // namespace

extern "C" {

int ref_sizeof_sphere(void) { return (int)sizeof(Sphere); }

int ref_default_scene(void* out, int cap)
{
    std::vector<Sphere>& d = default_scene();
    int n = (int)d.size();
    if (out) {
        PackedSphere* o = (PackedSphere*)out;
        for (int i = 0; i < n && i < cap; ++i) {
            const Sphere& s = d[i];
            std::memset(&o[i], 0, sizeof(PackedSphere));
            o[i].r = s.r;
            put(s.p, o[i].p); put(s.c, o[i].c); put(s.radiance, o[i].radiance);
            o[i].material = s.material;
            put(s.eta, o[i].eta); put(s.kappa, o[i].kappa);
            o[i].alpha = s.alpha;
        }
    }
    return n;
}

void ref_set_scene(const void* in, int n)
{
    (void)default_scene();
    const PackedSphere* s = (const PackedSphere*)in;
    std::vector<Sphere> v;
    v.reserve(n);
    for (int i = 0; i < n; ++i)
        v.emplace_back(s[i].r, V(s[i].p), V(s[i].c), V(s[i].radiance), s[i].material,
                       V(s[i].eta), V(s[i].kappa), s[i].alpha);
    spheres = v;
}

/* The reference's estimators by the build's numbering (include/vpt.h vpt_estimator):
 *   0 iterativeVPTracerFree          vptShadeMethods.h:1263
 *   1 MISVPTTracerRecursive          vptShadeMethods.h:1345
 *   2 explicitVPTracerRecursiveFree  vptShadeMethods.h:1153
 *   3 implicitVPTracerRecursiveFree  vptShadeMethods.h:938
 *   4 explicitVPTracerRecursive      vptShadeMethods.h:1014
 *   5 iterativePathTracer            shadeMethods.h:104 (surface only: sa, ss unused)
 *   6 rayMarching3                   rayMarchingMethods.h:330 (step, idsource: ref_set_march)
 *   7 rayMarching2                   rayMarchingMethods.h:262 (step, idsource)
 *   8 rayMarchingGlobal              rayMarchingMethods.h:106 (segmentos = the march step parameter)
 *   9 rayMarching                    rayMarchingMethods.h:34  (sigma_t = sa + ss, steps = the march step
 *                                                              parameter; the Color it returns) */
static double g_march_step = 0.1;  /* src/rt.cpp:791 */
static int g_march_light = 7;
static Color run_estimator(int estimator, const Ray& r, double sa, double ss)
{
    switch (estimator) {
    case 0: return iterativeVPTracerFree(r, sa, ss);
    case 1: return MISVPTTracerRecursive(r, sa, ss, 0);
    case 2: return explicitVPTracerRecursiveFree(r, sa, ss, 0);
    case 3: return implicitVPTracerRecursiveFree(r, sa, ss);
    case 4: return explicitVPTracerRecursive(r, sa, ss, 0);
    case 5: return iterativePathTracer(r);
    case 7: return rayMarching2(r, sa, ss, g_march_step, g_march_light);
    case 8: return rayMarchingGlobal(r, sa, ss, g_march_step);
    case 9: {
        Point x_new;
        int idsource = 0;
        return rayMarching(r, sa + ss, ss, g_march_step, x_new, idsource);
    }
    default: return rayMarching3(r, sa, ss, g_march_step, g_march_light);
    }
}

/* One camera sample through an estimator.  `state` is the erand48 state before the call; the
 * state after the call is returned (tells how many draws were consumed). */
void ref_set_march(double step, int light)
{
    g_march_step = step;
    g_march_light = light;
}

uint64_t ref_trace(int estimator, const double ray[6], uint64_t state, double sa, double ss,
                   double out[3])
{
    set_state(state);
    Ray r(V(ray), V(ray + 3));
    Color c = run_estimator(estimator, r, sa, ss);
    put(c, out);
    return get_state();
}

/* main()'s pixel loop (src/rt.cpp:752-805) over camera rows [y0, y1), per-sample streams.
 * out_lin: w*h*3 doubles in file order (idx = (h-y-1)*w+x), the per-pixel average BEFORE the
 * clamp of src/rt.cpp:803 (callers clamp).  per_sample (optional): w*h*spp*3 doubles. */
void ref_render(int w, int h, int spp, int estimator, double sa, double ss, uint64_t img_seed,
                int y0, int y1, double* out_lin, double* per_sample)
{
    Ray camera(Point(0, 11.2, 214), Vector(0, -0.042612, -1).normalize());
    Vector cx = Vector(w * 0.5095 / h, 0., 0.);
    Vector cy = (cx % camera.d).normalize() * 0.5095;
    for (int y = y0; y < y1; ++y) {
        for (int x = 0; x < w; ++x) {
            int idx = (h - y - 1) * w + x;
            Color pixelValue = Color();
            for (int i = 0; i < spp; ++i) {
                set_state(orc_stream_state(img_seed, (uint64_t)idx, (uint64_t)i));
                double jx = erand48(seed);
                double jy = erand48(seed);
                Vector cameraRayDir = cx * ((static_cast<double>(x) + jx - 0.5) / w - .5) +
                                      cy * ((static_cast<double>(y) + jy - 0.5) / h - .5) + camera.d;
                Color L = run_estimator(estimator, Ray(camera.o, cameraRayDir.normalize()), sa, ss);
                if (per_sample) put(L, per_sample + ((size_t)idx * spp + i) * 3);
                pixelValue = L + pixelValue;
            }
            pixelValue = pixelValue * (1 / static_cast<double>(spp));
            put(pixelValue, out_lin + (size_t)idx * 3);
        }
    }
}

/* The camera ray of one sample (src/rt.cpp:755-759,787), x-then-y jitter. */
uint64_t ref_camera_ray(int w, int h, int x, int y, uint64_t state, double out_ray[6])
{
    set_state(state);
    Ray camera(Point(0, 11.2, 214), Vector(0, -0.042612, -1).normalize());
    Vector cx = Vector(w * 0.5095 / h, 0., 0.);
    Vector cy = (cx % camera.d).normalize() * 0.5095;
    double jx = erand48(seed);
    double jy = erand48(seed);
    Vector dir = cx * ((static_cast<double>(x) + jx - 0.5) / w - .5) +
                 cy * ((static_cast<double>(y) + jy - 0.5) / h - .5) + camera.d;
    dir.normalize();
    put(camera.o, out_ray);
    put(dir, out_ray + 3);
    return get_state();
}

int ref_to_display(double x) { return toDisplayValue(x); }

/* ---- primitives (function-level known-answer vectors) ---- */

double ref_sphere_intersect(int i, const double ray[6]) { return spheres[i].intersect(Ray(V(ray), V(ray + 3))); }

int ref_intersect(const double ray[6], double* t, int* id)
{
    return intersect(Ray(V(ray), V(ray + 3)), *t, *id) ? 1 : 0;
}

int ref_visibility(const double light[3], const double x[3]) { return visibility(V(light), V(x)) ? 1 : 0; }

double ref_transmitance(const double a[3], const double b[3], double st) { return transmitance(V(a), V(b), st); }

void ref_coordinate_system(const double n[3], double s[3], double t[3])
{
    Vector nn = V(n), ss, tt;
    coordinateSystem(nn, ss, tt);
    put(ss, s); put(tt, t);
}

uint64_t ref_solid_angle_dir(const double wc[3], double cmax, uint64_t state, double out[3])
{
    set_state(state);
    put(solidAngle(V(wc), cmax), out);
    return get_state();
}

uint64_t ref_cosine_hemispheric(const double n[3], uint64_t state, double out[3])
{
    set_state(state);
    put(cosineHemispheric(V(n)), out);
    return get_state();
}

uint64_t ref_isotropic_phase(uint64_t state, double out[3])
{
    set_state(state);
    put(isotropicPhaseSample(), out);
    return get_state();
}

uint64_t ref_vector_facet(double alpha, uint64_t state, double out[3])
{
    set_state(state);
    put(vectorFacet(alpha), out);
    return get_state();
}

void ref_fresnel(double c, const double eta[3], const double kappa[3], double out[3])
{
    put(fresnel(c, V(eta), V(kappa)), out);
}

void ref_fr_microfacet(const double eta[3], const double kappa[3], const double wi[3], const double wh[3],
                       const double wo[3], double alpha, const double n[3], double out[3])
{
    put(frMicroFacet(V(eta), V(kappa), V(wi), V(wh), V(wo), alpha, V(n)), out);
}

double ref_microfacet_prob(const double wo[3], const double wh[3], double alpha, const double n[3])
{
    return microFacetProb(V(wo), V(wh), alpha, V(n));
}

uint64_t ref_bdsf(const double wray[3], const double n[3], int id, uint64_t state, double fs[3],
                  double wi[3], double* prob)
{
    set_state(state);
    Vector aux;
    double p = 0;
    Color f = bdsf(aux, V(wray), V(n), p, id);
    put(f, fs); put(aux, wi); *prob = p;
    return get_state();
}

void ref_plight(int obj, const double x[3], const double n[3], const double wray[3], const double I[3],
                const double light[3], double alpha, double out[3])
{
    put(pLight(spheres[obj], V(x), V(n), V(wray), V(I), V(light), alpha), out);
}

uint64_t ref_misv2(int obj, const double x[3], const double n[3], const double wray[3], double alpha,
                   double st, uint64_t state, double out[3])
{
    set_state(state);
    put(MISv2(spheres[obj], V(x), V(n), V(wray), alpha, st), out);
    return get_state();
}

uint64_t ref_free_single_scattering(const double xt[3], int idsource, double st, double probSource,
                                    uint64_t state, double out[3])
{
    set_state(state);
    put(freeSingleScattering(V(xt), idsource, st, probSource), out);
    return get_state();
}

uint64_t ref_single_scattering(const double xt[3], int idsource, double st, double ss, double trxt,
                               double probSource, uint64_t state, double out[3])
{
    set_state(state);
    put(singleScattering(V(xt), idsource, st, ss, trxt, probSource), out);
    return get_state();
}

uint64_t ref_equiangular_params2(int idsource, double tmax, const double ray[6], double out[5], uint64_t state)
{
    set_state(state);
    double D = 0, ta = 0, tb = 0, s = 0;
    double d = equiAngularParams2(idsource, tmax, Ray(V(ray), V(ray + 3)), D, ta, tb, s);
    out[0] = d; out[1] = D; out[2] = ta; out[3] = tb; out[4] = s;
    return get_state();
}

double ref_equiangular_prob(double D, double ta, double tb, double s) { return equiAngularProb(D, ta, tb, s); }

/* punctualVolumetric, rayMarchingMethods.h:12 (draws nothing) */
void ref_punctual_volumetric(int idsource, const double x[3], double phase, double st, double ss, double out[3])
{
    put(punctualVolumetric(idsource, V(x), phase, st, ss), out);
}

/* rayMarching, rayMarchingMethods.h:34, with its two out-parameters: out[0..2] = Color,
 * out[3..5] = x_new (x_new_in when the ray hits nothing), *idsource (idsource_in on a miss) */
uint64_t ref_ray_marching_explicit(const double ray[6], double st, double ss, double steps, uint64_t state,
                                   const double x_new_in[3], int* idsource, double out[6])
{
    set_state(state);
    Point x_new = V(x_new_in);
    Color c = rayMarching(Ray(V(ray), V(ray + 3)), st, ss, steps, x_new, *idsource);
    put(c, out);
    put(x_new, out + 3);
    return get_state();
}

}  // extern "C"
