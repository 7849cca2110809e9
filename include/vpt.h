/*
 * vpt.h -- C ABI of the MI355X volumetric path tracer (libvpt.so).
 *
 * Drop-in boundary for the hot path of gabo99cas/minimal_volumetric_path_tracer.  The reference
 * has no FFI; its hot path is one C++ call per camera sample,
 *     Color iterativeVPTracerFree(const Ray&, double sigma_a, double sigma_s)   vptShadeMethods.h:1263
 *     Color MISVPTTracerRecursive(const Ray&, double, double, int depth)        vptShadeMethods.h:1345
 * made from main()'s OpenMP pixel loop (src/rt.cpp:767-805) with the scene in a global
 * std::vector<Sphere> (include/Sphere.h:49) and the RNG in a global erand48 state
 * (include/Vector.h:38).  A GPU cannot be fed one sample per call, so the boundary is lifted to
 * the pixel loop (vpt_render*), with the per-sample call kept as a batch entry
 * (vpt_trace_batch).  Implicit globals become explicit arguments; no global state remains.
 *
 * Plain C: fixed-width scalars and pointers only.  All functions return VPT_OK (0) or a
 * negative vpt_status; vpt_last_error() gives a thread-local message for the last failure.
 */
#ifndef VPT_H
#define VPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VPT_ABI_VERSION 3

typedef enum {
    VPT_OK = 0,
    VPT_E_INVALID = -1,        /* bad argument (null pointer, size, NaN parameter ...) */
    VPT_E_TOO_MANY = -2,       /* more spheres than VPT_MAX_SPHERES */
    VPT_E_NO_EMITTER = -3,     /* reserved */
    VPT_E_UNSUPPORTED = -4,    /* material id outside {0,1,2,3} */
    VPT_E_HIP = -5,            /* HIP runtime error (message in vpt_last_error) */
    VPT_E_IO = -6,             /* file could not be written */
    VPT_E_INTERNAL = -7        /* an internal invariant failed (message in vpt_last_error) */
} vpt_status;

#define VPT_MAX_SPHERES 64

/* Byte-identical to the reference's Sphere (include/Sphere.h:12-21; 144 B, offsets r 0, p 8,
 * c 32, radiance 56, material 80, eta 88, kappa 112, alpha 136), so spheres.data() of a
 * reference build can be passed as is.  material: 0 Lambert, 1 microfacet conductor, 2 smooth
 * dielectric (eta 1.5), 3 "volumetric" (only seen by the shadow-ray transmittance).  A sphere
 * is an emitter when any radiance channel is > 0; r == 0 makes it a point light. */
typedef struct vpt_sphere {
    double r;
    double p[3];
    double c[3];
    double radiance[3];
    int32_t material;
    int32_t reserved_;
    double eta[3];
    double kappa[3];
    double alpha;
} vpt_sphere;

/* Reference Ray (include/Ray.h:10-15): origin and direction (callers normalise). */
typedef struct vpt_ray {
    double o[3];
    double d[3];
} vpt_ray;

typedef enum {
    VPT_FREE_FLIGHT = 0,           /* iterativeVPTracerFree, vptShadeMethods.h:1263 (main's estimator) */
    VPT_MIS_EQUIANGULAR = 1,       /* MISVPTTracerRecursive, vptShadeMethods.h:1345 */
    VPT_EXPLICIT_FREE = 2,         /* explicitVPTracerRecursiveFree, vptShadeMethods.h:1153 */
    VPT_IMPLICIT_FREE = 3,         /* implicitVPTracerRecursiveFree, vptShadeMethods.h:940 */
    VPT_EXPLICIT_EQUIANGULAR = 4,  /* explicitVPTracerRecursive, vptShadeMethods.h:1014 */
    VPT_SURFACE_PT = 5,            /* iterativePathTracer, shadeMethods.h:104: surface-only path tracing (the
                                    * commented alternative at src/rt.cpp:793); sigma_a, sigma_s, hg_g and
                                    * max_depth are ignored; rendered by the task-pool kernel like 0-4
                                    * (chunk_spp applies) */
    VPT_RAY_MARCHING = 6,          /* rayMarching3, rayMarchingMethods.h:330: constant-step marching toward the
                                    * light march_light (the commented alternative at src/rt.cpp:791, which
                                    * passes sigma_a 0.001, sigma_s 0.0125, step 0.1, light 7); draws nothing
                                    * beyond the camera jitter; samples summed in the reference's order */
    VPT_RAY_MARCHING_SA = 7,       /* rayMarching2, rayMarchingMethods.h:262: steps of march_step toward sphere
                                    * march_light by solid-angle sampling, plus a hit light's radiance */
    VPT_RAY_MARCHING_GLOBAL = 8,   /* rayMarchingGlobal, rayMarchingMethods.h:106: 10 diffuse bounces, each
                                    * marched by rayMarching in march_step segments (a count), toward the
                                    * hard-coded sphere 5 (scenes need >= 6 spheres) */
    VPT_RAY_MARCHING_EXPLICIT = 9  /* rayMarching, rayMarchingMethods.h:34: the Color it returns for the camera
                                    * ray with sigma_t = sigma_a + sigma_s, steps = march_step (a count),
                                    * light = sphere 5; its out-parameters: vpt_ray_marching_batch */
} vpt_estimator;
#define VPT_NUM_ESTIMATORS 10

typedef enum {
    VPT_FB_F32 = 0,            /* framebuffer: 3 x float per pixel */
    VPT_FB_F64 = 1             /* framebuffer: 3 x double per pixel */
} vpt_fb_format;

/* Homogeneous medium + estimator (src/rt.cpp:794 passes sigma_a = 0.001, sigma_s = 0.009). */
typedef struct vpt_medium {
    double sigma_a;
    double sigma_s;
    double hg_g;               /* extension: Henyey-Greenstein g; 0 = the reference's isotropic phase */
    int32_t max_depth;         /* extension: max path vertices; 0 = unbounded (Russian roulette only) */
    int32_t estimator;         /* vpt_estimator */
    double march_step;         /* ray marching (6-9): step length (6, 7) or number of segments (8, 9); > 0,
                                * default 0.1 */
    int32_t march_light;       /* VPT_RAY_MARCHING, VPT_RAY_MARCHING_SA: index of the light sphere (default 7) */
    int32_t reserved_;
} vpt_medium;

/* One image (or one shard of an image): main() of src/rt.cpp:744-830 made explicit. */
typedef struct vpt_params {
    int32_t width, height;     /* src/rt.cpp:752 (1024 x 768) */
    int32_t spp;               /* src/rt.cpp:784 (argv[1]) */
    int32_t fb_format;         /* vpt_fb_format */
    vpt_medium medium;
    uint64_t seed;             /* image seed; every (pixel, sample) owns an erand48 stream */
    vpt_ray camera;            /* src/rt.cpp:755: o = (0, 11.2, 214), d = norm(0, -0.042612, -1) */
    double fov_scale;          /* src/rt.cpp:758-759: 0.5095 */
    /* Row sharding in FILE order (file row = h-1-y, src/rt.cpp:773).  File rows are cut into
     * bands of band_rows; this call renders bands band_offset, band_offset + band_stride, ...
     * and writes them compactly, in increasing file-row order.  Whole image: band_rows = height,
     * band_stride = 1, band_offset = 0 (vpt_default_params). */
    int32_t band_rows, band_stride, band_offset;
    /* Samples per partial sum (build extension).  A pixel's samples are summed sequentially inside
     * a chunk exactly as the reference sums a pixel (src/rt.cpp:794), and the chunk sums are then
     * added in chunk order; chunk_spp == 1 or >= spp is the reference's own sequential order.
     * Chunks are the GPU's unit of work.  chunk_spp > 0: uniform chunks of chunk_spp samples;
     * 0 = auto: chunks of min(spp, 32), the last 64 samples in shrinking chunks (22, 14, 10, ...,
     * 1; layout in csrc/vpt_chunks.h) so that a launch ends on short units.  spp <= 32 is one
     * chunk either way. */
    int32_t chunk_spp;
} vpt_params;

/* Fills the reference defaults: 1024x768, spp 16, free-flight, sigma 0.001/0.009, camera and
 * fov of src/rt.cpp:752-759, seed 0x5EED0001, float32 framebuffer, whole image. */
void vpt_default_params(vpt_params* p);

/* The reference scene (include/Sphere.cpp:11-22): writes min(cap, 10) spheres, returns 10. */
int vpt_default_scene(vpt_sphere* out, int cap);

/* Number of file rows a params' shard covers (output holds rows * width pixels). */
int vpt_shard_rows(const vpt_params* p);

/* ---- context: one device, one scene ---- */
typedef struct vpt_context vpt_context;

int vpt_context_create(int device, vpt_context** out);
void vpt_context_destroy(vpt_context* ctx);
/* Copies the scene to the device (replaces the reference's global `spheres`). */
int vpt_set_scene(vpt_context* ctx, const vpt_sphere* spheres, int n);

/* Renders into a DEVICE buffer on `stream` (a hipStream_t, NULL = default stream); returns
 * after enqueueing.  d_out: vpt_shard_rows(p) * width * 3 elements of fb_format, the
 * per-pixel average BEFORE the clamp of src/rt.cpp:803.  Renders on different streams of one
 * context may be in flight together: each stream gets its own work queue and partial-sum
 * buffer (stream-ordered, grown on demand); calls on one stream run in order.  The scene must
 * not change (vpt_set_scene) while a render that uses it is in flight. */
int vpt_render_device(vpt_context* ctx, const vpt_params* p, void* d_out, void* stream);

/* Same, synchronous, host output buffer. */
int vpt_render(vpt_context* ctx, const vpt_params* p, void* h_out);

/* ---- several GPUs of one process ----
 * One image rendered by devices 0 .. n_gpus-1 of this process (replaces the OpenMP pixel loop of
 * src/rt.cpp:767-805 on a multi-GPU node without a launcher).  Device g renders the file-row
 * bands g, g + n_gpus, ... (band_rows of `p` when it cuts the image, else 16 rows; p itself must
 * describe the whole image: band_stride 1, band_offset 0); the strips are gathered to device 0
 * over RCCL (one communicator per device, ncclCommInitAll; grouped ncclSend/ncclRecv) and
 * written to h_out in file order.  Bit-identical to vpt_render for any n_gpus.  Synchronous.
 * vpt_multi_* keep the contexts, streams, communicators and buffers between images. */
typedef struct vpt_multi vpt_multi;
int vpt_multi_create(int n_gpus, vpt_multi** out);
int vpt_multi_set_scene(vpt_multi* m, const vpt_sphere* spheres, int n);
int vpt_multi_render(vpt_multi* m, const vpt_params* p, void* h_out);
void vpt_multi_destroy(vpt_multi* m);
/* one-shot: create, set the scene, render, destroy */
int vpt_render_multi(const vpt_sphere* spheres, int n, const vpt_params* p, int n_gpus, void* h_out);

/* The per-sample call itself, batched: rays[i] with erand48 start state states[i] (low 48
 * bits) through the estimator of `m`; out_rgb[3i..3i+2] = the Color the reference returns,
 * out_states[i] (optional) = the erand48 state afterwards.  Host pointers; synchronous. */
int vpt_trace_batch(vpt_context* ctx, const vpt_medium* m, const vpt_ray* rays, const uint64_t* states, int n,
                    double* out_rgb, uint64_t* out_states);

/* punctualVolumetric(idsource, x, phase, sigma_t, sigma_s) (include/rayMarchingMethods.h:12-31; no
 * caller in the reference) at the n points x[3i..3i+2]: visibilityVPT from sphere idsource's centre,
 * radiance / distance^2 * phase * multipleT * sigma_s.  Host arrays; synchronous. */
int vpt_punctual_volumetric(vpt_context* ctx, int idsource, const double* x, int n, double phase, double sigma_t,
                            double sigma_s, double* out_rgb);

/* rayMarching(r, sigma_t, sigma_s, steps, x_new, idsource) (include/rayMarchingMethods.h:34-103) for
 * rays[i] with erand48 start state states[i]: out_rgb = the Color; x_new[3i..] and idsource[i] are
 * in/out like the reference's reference parameters (set to the first hit, unchanged on a miss);
 * out_states optional.  Needs >= 6 spheres (sphere 5 is hard-coded).  Host arrays; synchronous. */
int vpt_ray_marching_batch(vpt_context* ctx, double sigma_t, double sigma_s, double steps, const vpt_ray* rays,
                           const uint64_t* states, int n, double* out_rgb, double* x_new, int32_t* idsource,
                           uint64_t* out_states);

/* Counting mode: ray-sphere tests (Sphere::intersect calls, include/Sphere.h:27) the render
 * of `p` performs in the REFERENCE algorithm (shortcuts of this build count what they skip),
 * plus estimator loop iterations.  Synchronous. */
int vpt_count_work(vpt_context* ctx, const vpt_params* p, uint64_t* tests, uint64_t* iterations);

/* Start state of one sample's erand48 stream (host-side statement of the device spec). */
uint64_t vpt_stream_state(uint64_t seed, uint64_t pixel_idx, uint64_t sample);

/* Evaluates the device math library on the GPU: fn 0 sqrt, 1 exp, 2 log, 3 sin, 4 cos, 5 tan,
 * 6 atan, 7 acos, 8 atan2(x, y), 9 x / y, 10 / 11 sin / cos of acos(x), 12 1 / sqrt(x) (the
 * normalisation's reciprocal).  Host arrays, synchronous (parity tests). */
int vpt_math_probe(vpt_context* ctx, int fn, const double* x, const double* y, double* out, int n);

/* Henyey-Greenstein phase extension (the north-star's HG g; the reference has only the isotropic
 * phase, include/vptSamplingFunctions.h:34-47 and include/volumetricBasicFunctions.h:59-62, which
 * g == 0 reproduces bit for bit).  For each of the n erand48 states: the direction the medium event
 * samples around the propagation direction din (two draws), and the state after them; for each of
 * the nw directions wl: the phase value the NEE weights with (mu = din . wl).  Host arrays,
 * synchronous (property tests). */
int vpt_phase_probe(vpt_context* ctx, double g, const double din[3], const uint64_t* states, int n, double* dirs,
                    uint64_t* states_out, const double* wl, int nw, double* values);

/* PPM writer of main() (src/rt.cpp:812-820): clamp to [0,1] (src/rt.cpp:803), gamma 1/2.2,
 * int(v*255 + .5) (include/mathUtilities.h:43-45), "P3\n%d %d\n255\n" then "%d %d %d " per
 * pixel, byte-identical.  rgb: host framebuffer, w*h*3 of fb_format, file order. */
int vpt_write_ppm(const char* path, const void* rgb, int fb_format, int w, int h);
/* The same bytes into a caller buffer; returns the byte count (call with buf = NULL to size). */
int64_t vpt_encode_ppm(const void* rgb, int fb_format, int w, int h, char* buf, int64_t cap);

const char* vpt_last_error(void);
int vpt_abi_version(void);
/* Build provenance: 16 hex digits hashing the library's sources and compile flags
 * (scripts/build_id.py, baked in by csrc/Makefile). */
const char* vpt_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* VPT_H */
