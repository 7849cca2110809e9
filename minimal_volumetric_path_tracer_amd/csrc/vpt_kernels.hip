/*
 * vpt_kernels.hip -- HIP kernels (gfx950) and the device half of the C ABI (include/vpt.h).
 *
 * render_kernel replaces main()'s OpenMP pixel loop (src/rt.cpp:767-805): one lane owns one
 * pixel and runs its spp camera samples (src/rt.cpp:786-798) through the estimator, accumulating
 * in FP64 in the reference's order, then writes the average (src/rt.cpp:800) once.  A wave
 * covers an 8x8 pixel tile (neighbouring camera rays hit the same surfaces, which keeps the
 * sphere loop and the shading branches coherent); a 256-thread workgroup covers 16x16.
 */
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <vector>

#include "vpt_device.h"
#include "vpt_pool.h"
#include "vpt_internal.h"

/* the EST = 1 pool kernel comes from vpt_pool_mis.hip, compiled with flags of its own (VPT_MIS_TU;
 * -DVPT_MIS_TU=0 instantiates it here, as the syntax checks of tests/test_knobs.py do) */
#ifndef VPT_MIS_TU
#define VPT_MIS_TU 1
#endif
#if VPT_MIS_TU
namespace vpt {
extern template __global__ void pool_kernel<1, false>(PoolParams P0, Medium m0, const DevScene* __restrict__ S,
                                                      unsigned long long* counters, unsigned long long* stats);
}  // namespace vpt
#if VPT_SECTIONS
extern "C" int vpt_mis_sections_add(unsigned long long* out);
#endif
#endif

using namespace vpt;

namespace {

struct KParams {
    int32_t w, h, spp, fb;
    int32_t band_rows, band_stride, band_offset, shard_rows;
    double sigma_a, sigma_s, g;
    int32_t max_depth, est;
    double march_step;             /* rayMarching3 (estimator 6) */
    int32_t march_light;
    uint64_t seed;
    double o[3], d[3], cx[3], cy[3];
    void* out;
    unsigned long long* counters;  /* counting mode: [tests, iterations] */
    unsigned* queue;               /* pixel work queue head (zeroed before each launch) */
    int32_t tiles_x, tiles_y;      /* 8x8 pixel tiles covering the shard */
    int32_t cost_surf, cost_med;   /* event scheduler weights */
    int32_t chunk;                 /* samples per partial sum (pool kernel) */
    int32_t taper;                 /* tapered chunk layout (auto mode, vpt_chunks.h) */
};

#define HIP_OK(expr)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return vpt_fail(VPT_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));       \
    } while (0)

template <int EST, bool COUNT, int FB>
__global__ __launch_bounds__(256) void render_kernel_simple(KParams P, const DevScene* __restrict__ S)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int lr = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    /* rayMarching3: every shadow ray leaves the light's centre, so oc and |oc|^2 of each sphere are
     * formed once per workgroup (round 3: 26.7 -> 32.4 Msamples/s) */
    __shared__ double march_oc[EST == 6 ? VPT_MAX_SPHERES : 1][4];
    if (EST == 6) {
        march_origin_init(S, sph_p(S, P.march_light), march_oc);
        __syncthreads();
    }
    if (x >= P.w || lr >= P.shard_rows) return;
    const int k = lr / P.band_rows, r = lr - k * P.band_rows;
    const int fr = (P.band_offset + k * P.band_stride) * P.band_rows + r;  /* file row */
    const int y = P.h - 1 - fr;                                              /* camera row */
    const uint64_t idx = (uint64_t)fr * (uint64_t)P.w + (uint64_t)x;          /* src/rt.cpp:773 */
    const Medium m{P.sigma_a, P.sigma_s, P.g, P.max_depth, P.march_step, P.march_light};
    const dv3 o = mk(P.o[0], P.o[1], P.o[2]), cd = mk(P.d[0], P.d[1], P.d[2]);
    const dv3 cx = mk(P.cx[0], P.cx[1], P.cx[2]), cy = mk(P.cy[0], P.cy[1], P.cy[2]);
    dv3 acc = mk(0, 0, 0);
    uint64_t tests = 0, iters = 0, mism = 0;
    for (int i = 0; i < P.spp; ++i) {
        Sampler<COUNT> smp;
        smp.X = vpt_stream_start(P.seed, idx, (uint64_t)i);
        smp.g = P.g;
        smp.cnt.tests = 0;
        smp.cnt.iterations = 0;
        smp.cnt.draw_mismatch = 0;
        /* jittered camera ray, src/rt.cpp:787, x draw first */
        double jx = smp.next();
        double jy = smp.next();
        dv3 dir = add(add(scl(cx, (((double)x + jx - 0.5) / P.w - .5)), scl(cy, (((double)y + jy - 0.5) / P.h - .5))), cd);
        dir = nrm(dir);
        dv3 L = trace_sample<EST, COUNT>(S, smp, o, dir, m, EST == 6 ? march_oc : nullptr);
        acc = add(L, acc);
        if (COUNT) {
            tests += smp.cnt.tests;
            iters += smp.cnt.iterations;
            mism += smp.cnt.draw_mismatch;
        }
    }
    acc = scl(acc, (1 / (double)P.spp));
    const size_t oi = ((size_t)lr * (size_t)P.w + (size_t)x) * 3;
    if (FB == VPT_FB_F32) {
        float* out = (float*)P.out;
        out[oi] = (float)acc.x;
        out[oi + 1] = (float)acc.y;
        out[oi + 2] = (float)acc.z;
    } else {
        double* out = (double*)P.out;
        out[oi] = acc.x;
        out[oi + 1] = acc.y;
        out[oi + 2] = acc.z;
    }
    if (COUNT) {
        atomicAdd(&P.counters[0], (unsigned long long)tests);
        atomicAdd(&P.counters[1], (unsigned long long)iters);
        if (mism) atomicAdd(&P.counters[2], (unsigned long long)mism);
    }
}

/* camera ray of one sample, src/rt.cpp:787 (x draw first) */
template <bool COUNT>
__device__ __forceinline__ dv3 camera_dir(const KParams& P, Sampler<COUNT>& smp, int x, int y)
{
    const dv3 cd = mk(P.d[0], P.d[1], P.d[2]);
    const dv3 cx = mk(P.cx[0], P.cx[1], P.cx[2]), cy = mk(P.cy[0], P.cy[1], P.cy[2]);
    double jx = smp.next();
    double jy = smp.next();
    dv3 dir = add(add(scl(cx, (((double)x + jx - 0.5) / P.w - .5)), scl(cy, (((double)y + jy - 0.5) / P.h - .5))), cd);
    return nrm(dir);
}

template <int FB>
__device__ __forceinline__ void store_pixel(const KParams& P, int x, int lr, dv3 acc)
{
    acc = scl(acc, (1 / (double)P.spp));  /* src/rt.cpp:800 */
    const size_t oi = ((size_t)lr * (size_t)P.w + (size_t)x) * 3;
    if (FB == VPT_FB_F32) {
        float* out = (float*)P.out;
        out[oi] = (float)acc.x;
        out[oi + 1] = (float)acc.y;
        out[oi + 2] = (float)acc.z;
    } else {
        double* out = (double*)P.out;
        out[oi] = acc.x;
        out[oi + 1] = acc.y;
        out[oi + 2] = acc.z;
    }
}

/*
 * Persistent wavefront scheduler.  Every lane owns one pixel at a time and runs that pixel's
 * camera samples strictly in order (so the per-pixel FP64 sum is the reference's, bit for bit),
 * but the wave no longer waits for its longest path:
 *   - path regeneration: a lane whose path ends starts its next sample at once;
 *   - a lane that finishes its pixel takes the next one from a device-wide queue (one atomic per
 *     wave, 8x8-tile order for coherent camera rays), so waves drain together at the very end;
 *   - deferred events: after the common part of an iteration (roulette, intersection, light and
 *     distance sampling) a lane holds a pending SURFACE or MEDIUM event; each round the wave runs
 *     only ONE of the two shading blocks -- the one with more lanes per unit of cost -- and the
 *     other lanes keep their event for a later round (no data moves, no divergence between the
 *     two blocks).
 */
template <int EST, bool COUNT, int FB>
__global__ __launch_bounds__(256) void render_kernel(KParams P, const DevScene* __restrict__ S)
{
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1ull;
    const Medium m{P.sigma_a, P.sigma_s, P.g, P.max_depth, P.march_step, P.march_light};
    const dv3 o0 = mk(P.o[0], P.o[1], P.o[2]);
    const unsigned npix = (unsigned)P.tiles_x * (unsigned)P.tiles_y * 64u;

    int x = 0, y = 0, lr = 0;
    uint64_t idx = 0;
    int i = 0;                 /* next sample to start */
    bool done = false, need_pixel = true, in_path = false;
    int pending = EV_END;
    dv3 acc = mk(0, 0, 0);
    Path p;
    Event e;
    e.pdf = 0;
    Sampler<COUNT> smp;
    smp.X = 0;
    smp.g = P.g;
    smp.cnt.tests = 0;
    smp.cnt.iterations = 0;
    smp.cnt.draw_mismatch = 0;

    while (true) {
        /* (1) converged: lanes without a pixel take the next ones from the queue */
        const uint64_t needm = __ballot(need_pixel && !done);
        if (needm) {
            const int leader = __ffsll((unsigned long long)needm) - 1;
            unsigned base = 0;
            if (lane == leader) base = atomicAdd(P.queue, (unsigned)__popcll(needm));
            base = __shfl(base, leader);
            if (need_pixel && !done) {
                const unsigned q = base + (unsigned)__popcll(needm & below);
                if (q >= npix) {
                    done = true;
                } else {
                    const unsigned tile = q >> 6, within = q & 63u;
                    x = (int)(tile % (unsigned)P.tiles_x) * 8 + (int)(within & 7u);
                    lr = (int)(tile / (unsigned)P.tiles_x) * 8 + (int)(within >> 3);
                    if (x < P.w && lr < P.shard_rows) {
                        const int k = lr / P.band_rows, r = lr - k * P.band_rows;
                        const int fr = (P.band_offset + k * P.band_stride) * P.band_rows + r; /* file row */
                        y = P.h - 1 - fr;                                                       /* camera row */
                        idx = (uint64_t)fr * (uint64_t)P.w + (uint64_t)x;                       /* src/rt.cpp:773 */
                        i = 0;
                        acc = mk(0, 0, 0);
                        need_pixel = false;
                    }
                }
            }
        }
        if (__ballot(!done) == 0) break;

        /* (2) lanes without a pending event advance their path to the next event */
        if (!done && !need_pixel && pending == EV_END) {
            while (true) {
                if (!in_path) {
                    if (i == P.spp) {
                        store_pixel<FB>(P, x, lr, acc);
                        need_pixel = true;
                        break;
                    }
                    smp.X = vpt_stream_start(P.seed, idx, (uint64_t)i);
                    ++i;
                    p.o = o0;
                    p.d = camera_dir(P, smp, x, y);
                    p.beta = mk(1, 1, 1);
                    p.L = mk(0, 0, 0);
                    p.depth = 0;
                    in_path = true;
                }
                if (!continue_path(smp, p, m)) {
                    acc = add(p.L, acc);  /* src/rt.cpp:794 */
                    in_path = false;
                    continue;
                }
                const int ev = decide<EST>(S, smp, p, e, m);
                if (ev == EV_END) {
                    acc = add(p.L, acc);
                    in_path = false;
                    continue;
                }
                pending = ev;
                break;
            }
        }

        /* (3) run one shading block: the one with more pending lanes per unit of cost */
        const int ns = __popcll(__ballot(pending == EV_SURF));
        const int nm = __popcll(__ballot(pending == EV_MED));
        if (ns + nm == 0) continue;
        if (ns * P.cost_med >= nm * P.cost_surf) {
            if (pending == EV_SURF) {
                surface_event<EST>(S, smp, p, e, m);
                pending = EV_END;
            }
        } else {
            if (pending == EV_MED) {
                medium_event<EST>(S, smp, p, e, m);
                pending = EV_END;
            }
        }
    }
    if (COUNT) {
        atomicAdd(&P.counters[0], (unsigned long long)smp.cnt.tests);
        atomicAdd(&P.counters[1], (unsigned long long)smp.cnt.iterations);
    }
}

template <int EST>
__global__ __launch_bounds__(256) void trace_batch_kernel(const vpt_ray* __restrict__ rays,
                                                          const uint64_t* __restrict__ states, int n, Medium m,
                                                          double g, const DevScene* __restrict__ S, double* out,
                                                          uint64_t* out_states)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Sampler<false> smp;
    smp.X = states[i] & 0xFFFFFFFFFFFFull;
    smp.g = g;
    dv3 L = trace_sample<EST, false>(S, smp, ld3(rays[i].o), ld3(rays[i].d), m);
    out[3 * i] = L.x;
    out[3 * i + 1] = L.y;
    out[3 * i + 2] = L.z;
    out_states[i] = smp.X;
}

/* punctualVolumetric (include/rayMarchingMethods.h:12-31) at n points */
__global__ __launch_bounds__(256) void punctual_kernel(int idsource, const double* __restrict__ x, int n, double phase,
                                                       double sigma_t, double sigma_s, const DevScene* __restrict__ S,
                                                       double* out)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Sampler<false> smp;
    smp.X = 0;
    smp.g = 0;
    const dv3 L = punctual_volumetric(S, smp, idsource, ld3(x + 3 * i), phase, sigma_t, sigma_s);
    out[3 * i] = L.x;
    out[3 * i + 1] = L.y;
    out[3 * i + 2] = L.z;
}

/* rayMarching (include/rayMarchingMethods.h:34-103) with its out-parameters, one ray per lane */
__global__ __launch_bounds__(256) void ray_marching_kernel(const vpt_ray* __restrict__ rays,
                                                           const uint64_t* __restrict__ states, int n, double sigma_t,
                                                           double sigma_s, double steps, const DevScene* __restrict__ S,
                                                           double* out, double* x_new, int* idsource,
                                                           uint64_t* out_states)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Sampler<false> smp;
    smp.X = states[i] & 0xFFFFFFFFFFFFull;
    smp.g = 0;
    dv3 xn = ld3(x_new + 3 * i);
    int id = idsource[i];
    const dv3 L = ray_marching_explicit(S, smp, ld3(rays[i].o), ld3(rays[i].d), sigma_t, sigma_s, steps, xn, id);
    out[3 * i] = L.x;
    out[3 * i + 1] = L.y;
    out[3 * i + 2] = L.z;
    x_new[3 * i] = xn.x;
    x_new[3 * i + 1] = xn.y;
    x_new[3 * i + 2] = xn.z;
    idsource[i] = id;
    out_states[i] = smp.X;
}

__global__ void math_probe_kernel(int fn, const double* x, const double* y, double* out, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double a = x[i], b = y[i], r = 0;
    switch (fn) {
    case 0: r = vm_sqrt(a); break;
    case 1: r = lm_exp(a); break;
    case 2: r = lm_log(a); break;
    case 3: r = lm_sin(a); break;
    case 4: r = lm_cos(a); break;
    case 5: r = lm_tan(a); break;
    case 6: r = lm_atan(a); break;
    case 7: r = lm_acos(a); break;
    case 8: r = lm_atan2(a, b); break;
    case 12: r = vm_inv_sqrt(a); break;  /* 1.0 / sqrt(a) (nrm) */
    case 10:
    case 11: {
        double sv, cv;
        lm_sincos_acos(a, &sv, &cv);
        r = fn == 10 ? sv : cv;
        break;
    }
    case 14:
    case 15:
    case 16:
    case 17: {  /* lm_dir_trig(c = a, phi = b) as the direction samplers call it (cone path when every
                 * lane of the wave has c > 0.9925): sin(acos c), cos(acos c), sin(phi), cos(phi) */
        double q[4];
        lm_dir_trig(a, b, &q[0], &q[1], &q[2], &q[3]);
        r = q[fn - 14];
        break;
    }
    case 18: {  /* a / b through one shared reciprocal of b (VPT_DIV_SHARE), unconditionally */
        double bb = b;
        __asm__ volatile("" : "+v"(bb));
        r = vm_div_by(a, vm_rcp_of(bb));
        break;
    }
    case 19: r = hemi_cosine_prob(a); break;  /* a * 1 / pi */
    case 20: {                                /* 1 / a and b / a, their bits xor'ed (inv_and_ratio) */
        double inv, q;
        inv_and_ratio(a, b, inv, q);
        r = __longlong_as_double(__double_as_longlong(inv) ^ __double_as_longlong(q));
        break;
    }
    case 21: r = vm_sqrt_isect(a); break;    /* the sphere tests' root (VPT_ISECT_CLASS) */
    case 22: r = vm_sqrt_isect_z(a); break;  /* the shadow rays' (VPT_ISECT_ZERO) */
    default: r = a / b; break;
    }
    out[i] = r;
}

/* HG extension probe: phase_sample around din from each state (the two draws of the stream), and
 * phase_value toward each wl (vpt_phase_probe) */
__global__ void phase_probe_kernel(double g, double dx, double dy, double dz, const uint64_t* X, int n, double* dirs,
                                   uint64_t* Xout, const double* wl, int nw, double* vals)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const dv3 din = mk(dx, dy, dz);
    if (i < n) {
        Sampler<false> smp;
        smp.X = X[i];
        smp.g = g;
        smp.cnt.tests = smp.cnt.iterations = smp.cnt.draw_mismatch = 0;
        const dv3 w = phase_sample(smp, din);
        dirs[3 * i] = w.x;
        dirs[3 * i + 1] = w.y;
        dirs[3 * i + 2] = w.z;
        Xout[i] = smp.X;
    }
    if (i < nw) vals[i] = phase_value(g, din, mk(wl[3 * i], wl[3 * i + 1], wl[3 * i + 2]));
}

bool is_finite(double v) { return v == v && v - v == 0.0; }

unsigned long long* g_pool_stats = nullptr;  /* debug statistics buffer (VPT_POOL_STATS=1) */

}  // namespace

/* Per-stream launch state: a render enqueued on one stream must not share its work queue or its
 * chunk partials with a render in flight on another stream of the same context.  Each stream
 * that renders gets its own slot (queue head + partials, grown on demand, stream-ordered), so
 * vpt_render_device may be called on several streams of one context at once. */
struct StreamSlot {
    hipStream_t stream;
    unsigned* d_queue;
    double* d_partials;      /* chunk sums of the pool kernel */
    size_t partials_bytes;
    hipEvent_t done;         /* recorded after the slot's last launch */
    unsigned long long used; /* last use (context tick), for reuse by another stream */
};
/* at most this many slots (each holds a partials buffer): a further stream takes over the least
 * recently used slot whose work has finished, or waits for the least recently used one */
constexpr int MAX_STREAM_SLOTS = 8;
constexpr int LAUNCH_LOG2_MAX = 26;  /* samples per workgroup per pool launch <= 2^26 (launch_max_units) */

struct vpt_context {
    int device;
    DevScene* d_scene;
    DevScene h_scene;
    int has_scene;
    unsigned long long* d_counters;
    unsigned* d_guard;       /* pool_kernel's argument-layout guard flag (PoolParams::guard), sticky */
    unsigned guard_bias = 0; /* vpt_debug_karg_guard */
    std::mutex mu;           /* guards slots: held from taking a slot until its launches are enqueued */
    std::vector<std::unique_ptr<StreamSlot>> slots;  /* stable addresses */
    unsigned long long tick = 0;
    int launch_log2 = LAUNCH_LOG2_MAX;  /* samples per workgroup per launch <= 2^launch_log2 (vpt_debug_set_launch_bound) */
};

/* The stream's slot, created on first use (or taken over from an idle stream once MAX_STREAM_SLOTS
 * exist); partials grown to `pbytes` in stream order (the previous buffer is freed after the work
 * already queued on the stream).  The caller holds ctx->mu from here until its launches on the slot
 * are enqueued and slot_done() has recorded them, so no other thread can grow, free or hand over the
 * slot's buffers in between. */
static int stream_slot(vpt_context* ctx, hipStream_t stream, size_t pbytes, StreamSlot** out)
{
    StreamSlot* sl = nullptr;
    for (auto& x : ctx->slots)
        if (x->stream == stream) sl = x.get();
    if (!sl && (int)ctx->slots.size() < MAX_STREAM_SLOTS) {
        std::unique_ptr<StreamSlot> n(new StreamSlot{stream, nullptr, nullptr, 0, nullptr, 0});
        HIP_OK(hipMalloc((void**)&n->d_queue, sizeof(unsigned)));
        const hipError_t e = hipEventCreateWithFlags(&n->done, hipEventDisableTiming);
        if (e != hipSuccess) {
            (void)hipFree(n->d_queue);
            return vpt_fail(VPT_E_HIP, "hipEventCreateWithFlags: %s", hipGetErrorString(e));
        }
        ctx->slots.push_back(std::move(n));
        sl = ctx->slots.back().get();
    }
    if (!sl) {  /* every slot belongs to another stream: take an idle one, else wait for the oldest */
        StreamSlot* idle = nullptr;
        StreamSlot* oldest = nullptr;
        for (auto& x : ctx->slots) {
            if (!oldest || x->used < oldest->used) oldest = x.get();
            if (hipEventQuery(x->done) == hipSuccess && (!idle || x->used < idle->used)) idle = x.get();
        }
        sl = idle ? idle : oldest;
        if (!idle) HIP_OK(hipEventSynchronize(sl->done));
        sl->stream = stream;  /* its buffers are no longer read by the previous stream */
    }
    if (pbytes > sl->partials_bytes) {
        if (sl->d_partials) HIP_OK(hipFreeAsync(sl->d_partials, stream));
        sl->d_partials = nullptr;
        sl->partials_bytes = 0;
        HIP_OK(hipMallocAsync((void**)&sl->d_partials, pbytes, stream));
        sl->partials_bytes = pbytes;
    }
    sl->used = ++ctx->tick;
    *out = sl;
    return VPT_OK;
}

/* after the slot's launches: its event marks when the stream is done with its buffers */
static int slot_done(StreamSlot* sl, hipStream_t stream)
{
    HIP_OK(hipEventRecord(sl->done, stream));
    return VPT_OK;
}

static int check_medium(const vpt_medium* m)
{
    if (!m) return vpt_fail(VPT_E_INVALID, "medium is NULL");
    if (!is_finite(m->sigma_a) || !is_finite(m->sigma_s) || m->sigma_a < 0 || m->sigma_s < 0)
        return vpt_fail(VPT_E_INVALID, "sigma_a/sigma_s must be finite and >= 0");
    if (!is_finite(m->hg_g) || m->hg_g <= -1.0 || m->hg_g >= 1.0) return vpt_fail(VPT_E_INVALID, "hg_g must be in (-1, 1)");
    if (m->max_depth < 0) return vpt_fail(VPT_E_INVALID, "max_depth must be >= 0");
    if (m->estimator < 0 || m->estimator >= VPT_NUM_ESTIMATORS)
        return vpt_fail(VPT_E_INVALID, "unknown estimator %d", m->estimator);
    return VPT_OK;
}

/* the ray-marching estimators' parameters: march_step (the step of rayMarching3 / rayMarching2, the
 * segment count of rayMarchingGlobal / rayMarching) finite and > 0; march_light (6, 7) a sphere of
 * the scene; rayMarchingGlobal and rayMarching read the hard-coded sphere 5
 * (include/rayMarchingMethods.h:64,153), so the scene needs at least 6 spheres */
static int check_march(const vpt_context* ctx, const vpt_medium* m)
{
    if (m->estimator < VPT_RAY_MARCHING) return VPT_OK;
    if (!is_finite(m->march_step) || !(m->march_step > 0))
        return vpt_fail(VPT_E_INVALID, "march_step must be finite and > 0");
    if ((m->estimator == VPT_RAY_MARCHING || m->estimator == VPT_RAY_MARCHING_SA) &&
        (m->march_light < 0 || m->march_light >= ctx->h_scene.n))
        return vpt_fail(VPT_E_INVALID, "march_light %d is not a sphere of the scene (%d)", m->march_light, ctx->h_scene.n);
    if ((m->estimator == VPT_RAY_MARCHING_GLOBAL || m->estimator == VPT_RAY_MARCHING_EXPLICIT) && ctx->h_scene.n < 6)
        return vpt_fail(VPT_E_INVALID, "rayMarchingGlobal / rayMarching sample sphere 5: the scene has %d spheres",
                        ctx->h_scene.n);
    return VPT_OK;
}

static int build_kparams(const vpt_context* ctx, const vpt_params* p, void* d_out, KParams& K)
{
    if (!ctx || !p) return vpt_fail(VPT_E_INVALID, "NULL context or params");
    if (!ctx->has_scene) return vpt_fail(VPT_E_INVALID, "no scene set (vpt_set_scene)");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0) return vpt_fail(VPT_E_INVALID, "width/height/spp must be > 0");
    if ((int64_t)p->width * p->height > (int64_t)1 << 31) return vpt_fail(VPT_E_INVALID, "image too large");
    if (p->fb_format != VPT_FB_F32 && p->fb_format != VPT_FB_F64) return vpt_fail(VPT_E_INVALID, "bad fb_format");
    int rc = check_medium(&p->medium);
    if (!rc) rc = check_march(ctx, &p->medium);
    if (rc) return rc;
    if (p->band_rows <= 0 || p->band_stride <= 0 || p->band_offset < 0 || p->band_offset >= p->band_stride)
        return vpt_fail(VPT_E_INVALID, "bad band_rows/band_stride/band_offset");
    int rows = vpt_shard_rows(p);  /* 0: more shards than bands -- a legal no-op */
    const double* cd = p->camera.d;
    if (!is_finite(p->fov_scale) || !is_finite(cd[0]) || !is_finite(cd[1]) || !is_finite(cd[2]))
        return vpt_fail(VPT_E_INVALID, "bad camera");
    memset(&K, 0, sizeof K);
    K.w = p->width;
    K.h = p->height;
    K.spp = p->spp;
    K.fb = p->fb_format;
    K.band_rows = p->band_rows;
    K.band_stride = p->band_stride;
    K.band_offset = p->band_offset;
    K.shard_rows = rows;
    K.sigma_a = p->medium.sigma_a;
    K.sigma_s = p->medium.sigma_s;
    K.g = p->medium.hg_g;
    K.max_depth = p->medium.max_depth;
    K.est = p->medium.estimator;
    K.march_step = p->medium.march_step;
    K.march_light = p->medium.march_light;
    K.seed = p->seed;
    for (int i = 0; i < 3; ++i) {
        K.o[i] = p->camera.o[i];
        K.d[i] = cd[i];
    }
    /* Vector cx = Vector(w * 0.5095 / h, 0., 0.); cy = (cx % camera.d).normalize() * 0.5095
     * (src/rt.cpp:758-759), same operation order */
    K.cx[0] = p->width * p->fov_scale / p->height;
    K.cx[1] = 0.;
    K.cx[2] = 0.;
    double crx = K.cx[1] * cd[2] - K.cx[2] * cd[1];
    double cry = K.cx[2] * cd[0] - K.cx[0] * cd[2];
    double crz = K.cx[0] * cd[1] - K.cx[1] * cd[0];
    double inv = 1.0 / sqrt(crx * crx + cry * cry + crz * crz);
    K.cy[0] = crx * inv * p->fov_scale;
    K.cy[1] = cry * inv * p->fov_scale;
    K.cy[2] = crz * inv * p->fov_scale;
    K.out = d_out;
    if (p->chunk_spp < 0) return vpt_fail(VPT_E_INVALID, "chunk_spp must be >= 0");
    /* auto: 32 samples per work unit (A/B at 1024^2 x 256: chunk 4 / 8 / 16 / 32 / 64 -> 3816 / 3969 /
     * 4085 / 4153 / 4129 Ms/s), the last 32 of a pixel tapered (vpt_chunks.h); spp <= 32 is then one
     * chunk, i.e. the reference's sequential sum.  An explicit chunk_spp gives uniform chunks. */
    K.chunk = p->chunk_spp > 0 ? (p->chunk_spp < p->spp ? p->chunk_spp : p->spp) : vpt_auto_chunk(p->spp);
    K.taper = p->chunk_spp == 0;
    return VPT_OK;
}

/* the pool kernel's argument-layout guard (PoolParams::guard): after a synchronised render, a raised
 * flag means a launch read its parameters from the wrong place and rendered nothing */
static int check_guard(vpt_context* ctx, const char* who)
{
    unsigned g = 0;
    HIP_OK(hipMemcpy(&g, ctx->d_guard, sizeof g, hipMemcpyDeviceToHost));
    if (g) return vpt_fail(VPT_E_INTERNAL, "%s: pool_kernel's launch parameters are not at the start of its argument "
                           "segment (VPT_P_KARG guard); the image is NaN", who);
    return VPT_OK;
}

template <typename Kern>
static int persistent_grid(vpt_context* ctx, Kern kern, int* blocks, int threads = 256)
{
    int per_cu = 0, cus = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0));
    HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    if (per_cu < 1) per_cu = 1;
    *blocks = per_cu * cus;
    return VPT_OK;
}

/* A/B and debug switches read from the environment (VPT_SIMPLE_KERNEL, VPT_WAVE_KERNEL,
 * VPT_COST_SURF / VPT_COST_MED, VPT_POOL_STATS) exist only in builds made with -DVPT_DEBUG_ENV=1
 * (scripts/build_variant.sh); the production library ignores the environment, so a stray
 * variable cannot change the kernel or its timing. */
#ifndef VPT_DEBUG_ENV
#define VPT_DEBUG_ENV 0
#endif
static int env_int(const char* name, int dflt)
{
    if (!VPT_DEBUG_ENV) return dflt;
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

template <int EST, bool COUNT, int FB>
static int launch_wave(vpt_context* ctx, KParams K, hipStream_t stream);
template <int EST, int FB>
static int launch_pool(vpt_context* ctx, KParams K, hipStream_t stream);

/* The pool's ring positions are 32-bit counters that grow by ~3 per sample a workgroup runs, so a
 * render is split into launches of at most 2^LAUNCH_LOG2_MAX samples per workgroup: units in order
 * [unit0, unit0 + nunits), each unit one partial slot, so the split changes no value (the chunk
 * sums are per unit; reduce_kernel adds them after the last launch).  One launch holds up to
 * ~17 G samples on 256 CUs; BASELINE configs[4] (2^34 samples per GPU) takes two. */
static uint64_t launch_max_units(int blocks, int C, int log2_bound)
{
    const uint64_t m = (((uint64_t)1 << log2_bound) * (uint64_t)(blocks > 0 ? blocks : 1)) / (uint64_t)(C > 0 ? C : 1);
    return m < 1 ? 1 : m;
}

/* log2(v) when v is a power of two, else -1 (PoolParams shift fast paths) */
static int log2_exact(int64_t v)
{
    if (v <= 0 || (v & (v - 1)) != 0) return -1;
    int k = 0;
    while ((v >> k) != 1) ++k;
    return k;
}

template <int EST, bool COUNT, int FB>
static int launch_one(vpt_context* ctx, KParams K, hipStream_t stream)
{
    const DevScene* S = ctx->d_scene;
    /* counting (vpt_count_work) needs only the totals: the one-lane-per-pixel kernel, which is
     * also the A/B baseline (VPT_SIMPLE_KERNEL=1: samples in sequence per lane) */
    if (COUNT || env_int("VPT_SIMPLE_KERNEL", 0)) {
        dim3 grid((unsigned)((K.w + 15) / 16), (unsigned)((K.shard_rows + 15) / 16));
        render_kernel_simple<EST, COUNT, FB><<<grid, dim3(256), 0, stream>>>(K, S);
        HIP_OK(hipGetLastError());
        return VPT_OK;
    }
    if constexpr (!COUNT && EST <= 5) return launch_pool<EST, FB>(ctx, K, stream);
    if constexpr (EST >= 6) {  /* ray marching: one lane per pixel, samples summed in order */
        dim3 grid((unsigned)((K.w + 15) / 16), (unsigned)((K.shard_rows + 15) / 16));
        render_kernel_simple<EST, COUNT, FB><<<grid, dim3(256), 0, stream>>>(K, S);
        HIP_OK(hipGetLastError());
    }
    return VPT_OK;
}

template <int EST, int FB>
static int launch_pool(vpt_context* ctx, KParams K, hipStream_t stream)
{
    const DevScene* S = ctx->d_scene;
    constexpr bool COUNT = false;
    int blocks = 0;
    int rc;
    const bool wave = EST <= 1 && env_int("VPT_WAVE_KERNEL", 0);  /* A/B: the previous design, FF/MIS */
    if (!wave) {  /* default: workgroup task pool (vpt_pool.h) */
        if (K.w > 65535 || K.h > 65535) return vpt_fail(VPT_E_INVALID, "width and height must be < 65536");
        PoolParams Q;
        Q.w = K.w;
        Q.h = K.h;
        Q.spp = K.spp;
        Q.rows = K.shard_rows;
        Q.band_rows = K.band_rows;
        Q.band_stride = K.band_stride;
        Q.band_offset = K.band_offset;
        Q.tiles_x = K.tiles_x;
        Q.lay = vpt_chunks(K.spp, K.chunk, K.taper);
        Q.nch = Q.lay.n;
        Q.level_units = (unsigned)K.tiles_x * (unsigned)K.tiles_y * 64u;
        Q.sh_lu = log2_exact((int64_t)Q.level_units);
        Q.sh_tx = log2_exact(K.tiles_x);
        Q.sh_br = log2_exact(K.band_rows);
        Q.sh_bs = log2_exact(K.band_stride);
        Q.sh_c = log2_exact(Q.lay.C);
        Q.rw = log2_exact(K.w) >= 0 ? 1.0 / K.w : 0.0;
        Q.rh = log2_exact(K.h) >= 0 ? 1.0 / K.h : 0.0;
        const uint64_t units = (uint64_t)K.tiles_x * (uint64_t)K.tiles_y * 64u * (uint64_t)Q.nch;
        if (units >= 0xFFFFFFFFull) return vpt_fail(VPT_E_INVALID, "too many work units (%llu)", (unsigned long long)units);
        Q.seed = K.seed;
        for (int i = 0; i < 3; ++i) {
            Q.o[i] = K.o[i];
            Q.d[i] = K.d[i];
            Q.cx[i] = K.cx[i];
            Q.cy[i] = K.cy[i];
        }
        const size_t pbytes = (size_t)K.shard_rows * (size_t)K.w * (size_t)Q.nch * 3 * sizeof(double);
        std::lock_guard<std::mutex> lock(ctx->mu);  /* until the launches on the slot are enqueued */
        StreamSlot* sl = nullptr;
        rc = stream_slot(ctx, stream, pbytes, &sl);
        if (rc) return rc;
        Q.partials = sl->d_partials;
        Q.queue = sl->d_queue;
        Q.guard = ctx->d_guard;
        Q.guard_bias = ctx->guard_bias;
        const Medium m{K.sigma_a, K.sigma_s, K.g, K.max_depth, K.march_step, K.march_light};
        rc = persistent_grid(ctx, pool_kernel<EST, COUNT>, &blocks, VPT_POOL_THREADS);
        if (rc) return rc;
        const uint64_t need = (units + POOL - 1) / POOL;
        if ((uint64_t)blocks > need) blocks = (int)need;
        /* every workgroup adds UREFILL to the u32 queue once more after it runs dry */
        if (units + (uint64_t)blocks * (UREFILL + 1) >= 0xFFFFFFFFull)
            return vpt_fail(VPT_E_INVALID, "too many work units (%llu) for the u32 work queue", (unsigned long long)units);
        /* launches of at most 2^launch_log2 samples per workgroup (launch_max_units); samples per
         * unit: at most the layout's head chunk C, and a unit above 2^LAUNCH_LOG2_MAX is refused */
        if (Q.lay.C > (1 << LAUNCH_LOG2_MAX))
            return vpt_fail(VPT_E_INVALID, "chunk of %d samples > 2^26 (the per-workgroup launch bound)", Q.lay.C);
        const uint64_t max_units = launch_max_units(blocks, Q.lay.C, ctx->launch_log2);
        unsigned long long* stats = nullptr;
        if (env_int("VPT_POOL_STATS", 0)) {  /* debug: scheduler statistics, vpt_debug_pool_stats */
            if (!g_pool_stats) HIP_OK(hipMalloc((void**)&g_pool_stats, (TL0 + 3 * TL_MAXWG) * sizeof(unsigned long long)));
            HIP_OK(hipMemsetAsync(g_pool_stats, 0, TL0 * sizeof(unsigned long long), stream));
            HIP_OK(hipMemsetAsync(g_pool_stats + TL0, 0xFF, 3 * TL_MAXWG * sizeof(unsigned long long), stream));
            stats = g_pool_stats;
        }
        for (uint64_t u0 = 0; u0 < units; u0 += max_units) {
            Q.unit0 = (unsigned)u0;
            Q.nunits = (unsigned)(units - u0 < max_units ? units - u0 : max_units);
            HIP_OK(hipMemsetAsync(Q.queue, 0, sizeof(unsigned), stream));
            pool_kernel<EST, COUNT><<<dim3((unsigned)blocks), dim3(VPT_POOL_THREADS), 0, stream>>>(Q, m, S, K.counters, stats);
            HIP_OK(hipGetLastError());
        }
        const size_t npix = (size_t)K.shard_rows * (size_t)K.w;
        reduce_kernel<FB><<<dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, stream>>>(Q, K.out);
        HIP_OK(hipGetLastError());
        return slot_done(sl, stream);
    }
#if VPT_DEBUG_ENV
    /* the round-1 wave scheduler (render_kernel), an A/B path of debug builds only */
    if constexpr (EST <= 1) return launch_wave<EST, COUNT, FB>(ctx, K, stream);
#endif
    return VPT_OK;
}

template <int EST, bool COUNT, int FB>
static int launch_wave(vpt_context* ctx, KParams K, hipStream_t stream)
{
    const DevScene* S = ctx->d_scene;
    int blocks = 0;
    int rc = persistent_grid(ctx, render_kernel<EST, COUNT, FB>, &blocks);
    if (rc) return rc;
    const int tiles = K.tiles_x * K.tiles_y;
    const int need = (tiles + 3) / 4;  /* 4 waves per block, one tile per wave to start */
    if (blocks > need) blocks = need;
    if (blocks < 1) blocks = 1;
    std::lock_guard<std::mutex> lock(ctx->mu);
    StreamSlot* sl = nullptr;
    rc = stream_slot(ctx, stream, 0, &sl);
    if (rc) return rc;
    K.queue = sl->d_queue;
    HIP_OK(hipMemsetAsync(K.queue, 0, sizeof(unsigned), stream));
    render_kernel<EST, COUNT, FB><<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(K, S);
    HIP_OK(hipGetLastError());
    return slot_done(sl, stream);
}

template <bool COUNT>
static int launch_render(vpt_context* ctx, KParams K, hipStream_t stream)
{
    if (K.shard_rows == 0) return VPT_OK;
    K.tiles_x = (K.w + 7) / 8;
    K.tiles_y = (K.shard_rows + 7) / 8;
    K.cost_surf = env_int("VPT_COST_SURF", 1);
    K.cost_med = env_int("VPT_COST_MED", 1);
#define VPT_LAUNCH_EST(E)                                                              \
    case E:                                                                            \
        if (K.fb == VPT_FB_F32) return launch_one<E, COUNT, VPT_FB_F32>(ctx, K, stream); \
        return launch_one<E, COUNT, VPT_FB_F64>(ctx, K, stream);
    switch (K.est) {
        VPT_LAUNCH_EST(0)
        VPT_LAUNCH_EST(1)
        VPT_LAUNCH_EST(2)
        VPT_LAUNCH_EST(3)
        VPT_LAUNCH_EST(4)
        VPT_LAUNCH_EST(5)
        VPT_LAUNCH_EST(6)
        VPT_LAUNCH_EST(7)
        VPT_LAUNCH_EST(8)
        VPT_LAUNCH_EST(9)
    }
#undef VPT_LAUNCH_EST
    return vpt_fail(VPT_E_INVALID, "unknown estimator %d", K.est);
}

extern "C" {

int vpt_context_create(int device, vpt_context** out)
{
    vpt_clear_error();
    if (!out) return vpt_fail(VPT_E_INVALID, "vpt_context_create: out is NULL");
    *out = nullptr;
    int ndev = 0;
    HIP_OK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return vpt_fail(VPT_E_INVALID, "vpt_context_create: device %d of %d", device, ndev);
    HIP_OK(hipSetDevice(device));
    vpt_context* c = new vpt_context();
    memset(&c->h_scene, 0, sizeof c->h_scene);
    c->device = device;
    c->has_scene = 0;
    c->d_scene = nullptr;
    c->d_counters = nullptr;
    c->d_guard = nullptr;
    hipError_t e = hipMalloc((void**)&c->d_scene, sizeof(DevScene));
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_counters, 4 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_guard, sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(c->d_guard, 0, sizeof(unsigned));
    if (e != hipSuccess) {
        vpt_context_destroy(c);
        return vpt_fail(VPT_E_HIP, "vpt_context_create: hipMalloc: %s", hipGetErrorString(e));
    }
    *out = c;
    return VPT_OK;
}

void vpt_context_destroy(vpt_context* ctx)
{
    if (!ctx) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(ctx->device);
    if (ctx->d_scene) (void)hipFree(ctx->d_scene);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    if (ctx->d_guard) (void)hipFree(ctx->d_guard);
    for (auto& sl : ctx->slots) {
        if (sl->done) (void)hipEventSynchronize(sl->done);
        if (sl->d_partials) (void)hipFree(sl->d_partials);
        if (sl->d_queue) (void)hipFree(sl->d_queue);
        if (sl->done) (void)hipEventDestroy(sl->done);
    }
    (void)hipSetDevice(prev);
    delete ctx;
}

int vpt_set_scene(vpt_context* ctx, const vpt_sphere* s, int n)
{
    vpt_clear_error();
    if (!ctx || !s) return vpt_fail(VPT_E_INVALID, "vpt_set_scene: NULL argument");
    if (n < 1) return vpt_fail(VPT_E_INVALID, "vpt_set_scene: empty scene");
    if (n > VPT_MAX_SPHERES) return vpt_fail(VPT_E_TOO_MANY, "vpt_set_scene: %d spheres > %d", n, VPT_MAX_SPHERES);
    DevScene h;
    memset(&h, 0, sizeof h);
    h.n = n;
    for (int i = 0; i < n; ++i) {
        const vpt_sphere& q = s[i];
        if (q.material < 0 || q.material > 3)
            return vpt_fail(VPT_E_UNSUPPORTED, "vpt_set_scene: sphere %d material %d", i, q.material);
        const double* vals[6] = {q.p, q.c, q.radiance, q.eta, q.kappa, nullptr};
        bool ok = is_finite(q.r) && q.r >= 0 && is_finite(q.alpha);
        for (int a = 0; a < 5; ++a)
            for (int c = 0; c < 3; ++c) ok = ok && is_finite(vals[a][c]);
        if (!ok) return vpt_fail(VPT_E_INVALID, "vpt_set_scene: sphere %d has a non-finite or negative field", i);
        h.sph[i] = q;
        h.geo[i].px = q.p[0];
        h.geo[i].py = q.p[1];
        h.geo[i].pz = q.p[2];
        h.geo[i].r2 = q.r * q.r;
        h.geo[i].mat3 = q.material == 3;
        h.geo[i].emitter = (q.radiance[0] > 0 || q.radiance[1] > 0 || q.radiance[2] > 0);
        h.geo[i].skey = q.material == 0 ? 0 : q.material == 1 ? 2 : 3;
        h.geo[i].point = q.r == 0;
        if (h.geo[i].emitter) h.emit[h.n_emit++] = i;
        const uint64_t bit = 1ull << i;
        if (h.geo[i].emitter) h.m_emitter |= bit;
        if (h.geo[i].point) h.m_point |= bit;
        if (h.geo[i].mat3) h.m_mat3 |= bit;
        if (h.geo[i].skey & 1) h.m_skey1 |= bit;
        if (h.geo[i].skey & 2) h.m_skey2 |= bit;
        if (q.r > 0 && q.radiance[0] > 0) h.mis_light[h.n_mis++] = i;
        if (q.material == 3) h.n_mat3++;
    }
    h.n_non3 = n - h.n_mat3;
    vpt_erand48_jump(2 * h.n_mis + 5, &h.kp_sa, &h.kp_sc);
    h.emit_all_radiance = 1;
    for (int i = 0; i < n; ++i)
        if (!h.geo[i].emitter && (s[i].radiance[0] != 0 || s[i].radiance[1] != 0 || s[i].radiance[2] != 0))
            h.emit_all_radiance = 0;
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipMemcpy(ctx->d_scene, &h, sizeof h, hipMemcpyHostToDevice));
    ctx->h_scene = h;
    ctx->has_scene = 1;
    return VPT_OK;
}

int vpt_render_device(vpt_context* ctx, const vpt_params* p, void* d_out, void* stream)
{
    vpt_clear_error();
    if (!d_out) return vpt_fail(VPT_E_INVALID, "vpt_render_device: d_out is NULL");
    KParams K;
    int rc = build_kparams(ctx, p, d_out, K);
    if (rc) return rc;
    HIP_OK(hipSetDevice(ctx->device));
    return launch_render<false>(ctx, K, (hipStream_t)stream);
}

int vpt_render(vpt_context* ctx, const vpt_params* p, void* h_out)
{
    vpt_clear_error();
    if (!h_out) return vpt_fail(VPT_E_INVALID, "vpt_render: h_out is NULL");
    KParams K;
    int rc = build_kparams(ctx, p, (void*)1, K);
    if (rc) return rc;
    HIP_OK(hipSetDevice(ctx->device));
    size_t bytes = (size_t)K.shard_rows * (size_t)K.w * 3 * (K.fb == VPT_FB_F32 ? sizeof(float) : sizeof(double));
    if (bytes == 0) return VPT_OK;
    void* d = nullptr;
    HIP_OK(hipMalloc(&d, bytes));
    K.out = d;
    rc = launch_render<false>(ctx, K, nullptr);
    hipError_t e = rc ? hipSuccess : hipMemcpy(h_out, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return vpt_fail(VPT_E_HIP, "vpt_render: %s", hipGetErrorString(e));
    return check_guard(ctx, "vpt_render");
}

int vpt_count_work(vpt_context* ctx, const vpt_params* p, uint64_t* tests, uint64_t* iterations)
{
    vpt_clear_error();
    KParams K;
    int rc = build_kparams(ctx, p, (void*)1, K);
    if (rc) return rc;
    HIP_OK(hipSetDevice(ctx->device));
    size_t bytes = (size_t)K.shard_rows * (size_t)K.w * 3 * (K.fb == VPT_FB_F32 ? sizeof(float) : sizeof(double));
    if (bytes == 0) {
        if (tests) *tests = 0;
        if (iterations) *iterations = 0;
        return VPT_OK;
    }
    void* d = nullptr;
    HIP_OK(hipMalloc(&d, bytes));
    K.out = d;
    K.counters = ctx->d_counters;
    unsigned long long hc[3] = {0, 0, 0};
    hipError_t e = hipMemset(ctx->d_counters, 0, sizeof hc);
    if (e == hipSuccess) {
        rc = launch_render<true>(ctx, K, nullptr);
        if (!rc) e = hipMemcpy(hc, ctx->d_counters, sizeof hc, hipMemcpyDeviceToHost);
    }
    (void)hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return vpt_fail(VPT_E_HIP, "vpt_count_work: %s", hipGetErrorString(e));
    if (hc[2])  /* the kill-predicting rings would lose bit-exactness on this scene (vpt_pool.h) */
        return vpt_fail(VPT_E_INTERNAL, "vpt_count_work: %llu events drew a different number of samples than the "
                        "kill prediction assumes", (unsigned long long)hc[2]);
    if (tests) *tests = hc[0];
    if (iterations) *iterations = hc[1];
    return VPT_OK;
}

int vpt_trace_batch(vpt_context* ctx, const vpt_medium* m, const vpt_ray* rays, const uint64_t* states, int n,
                    double* out_rgb, uint64_t* out_states)
{
    vpt_clear_error();
    if (!ctx || !rays || !states || !out_rgb || n < 0) return vpt_fail(VPT_E_INVALID, "vpt_trace_batch: bad arguments");
    if (!ctx->has_scene) return vpt_fail(VPT_E_INVALID, "no scene set (vpt_set_scene)");
    int rc = check_medium(m);
    if (!rc) rc = check_march(ctx, m);
    if (rc) return rc;
    if (n == 0) return VPT_OK;
    HIP_OK(hipSetDevice(ctx->device));
    vpt_ray* dr = nullptr;
    uint64_t *ds = nullptr, *dso = nullptr;
    double* dout = nullptr;
    hipError_t e = hipMalloc((void**)&dr, sizeof(vpt_ray) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&ds, sizeof(uint64_t) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&dso, sizeof(uint64_t) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, sizeof(double) * 3 * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(dr, rays, sizeof(vpt_ray) * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(ds, states, sizeof(uint64_t) * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        Medium mm{m->sigma_a, m->sigma_s, m->hg_g, m->max_depth, m->march_step, m->march_light};
        dim3 grid((unsigned)((n + 255) / 256)), block(256);
        switch (m->estimator) {
        case 0: trace_batch_kernel<0><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 1: trace_batch_kernel<1><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 2: trace_batch_kernel<2><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 3: trace_batch_kernel<3><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 4: trace_batch_kernel<4><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 5: trace_batch_kernel<5><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 6: trace_batch_kernel<6><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 7: trace_batch_kernel<7><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        case 8: trace_batch_kernel<8><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        default: trace_batch_kernel<9><<<grid, block>>>(dr, ds, n, mm, m->hg_g, ctx->d_scene, dout, dso); break;
        }
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out_rgb, dout, sizeof(double) * 3 * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out_states) e = hipMemcpy(out_states, dso, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(dr);
    (void)hipFree(ds);
    (void)hipFree(dso);
    (void)hipFree(dout);
    if (e != hipSuccess) return vpt_fail(VPT_E_HIP, "vpt_trace_batch: %s", hipGetErrorString(e));
    return VPT_OK;
}

int vpt_punctual_volumetric(vpt_context* ctx, int idsource, const double* x, int n, double phase, double sigma_t,
                            double sigma_s, double* out_rgb)
{
    vpt_clear_error();
    if (!ctx || !x || !out_rgb || n < 0) return vpt_fail(VPT_E_INVALID, "vpt_punctual_volumetric: bad arguments");
    if (!ctx->has_scene) return vpt_fail(VPT_E_INVALID, "no scene set (vpt_set_scene)");
    if (idsource < 0 || idsource >= ctx->h_scene.n)
        return vpt_fail(VPT_E_INVALID, "idsource %d is not a sphere of the scene (%d)", idsource, ctx->h_scene.n);
    if (n == 0) return VPT_OK;
    HIP_OK(hipSetDevice(ctx->device));
    double *dx = nullptr, *dout = nullptr;
    const size_t b = sizeof(double) * 3 * (size_t)n;
    hipError_t e = hipMalloc((void**)&dx, b);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, b);
    if (e == hipSuccess) e = hipMemcpy(dx, x, b, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        punctual_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256)>>>(idsource, dx, n, phase, sigma_t, sigma_s,
                                                                           ctx->d_scene, dout);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out_rgb, dout, b, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    (void)hipFree(dout);
    if (e != hipSuccess) return vpt_fail(VPT_E_HIP, "vpt_punctual_volumetric: %s", hipGetErrorString(e));
    return VPT_OK;
}

int vpt_ray_marching_batch(vpt_context* ctx, double sigma_t, double sigma_s, double steps, const vpt_ray* rays,
                           const uint64_t* states, int n, double* out_rgb, double* x_new, int32_t* idsource,
                           uint64_t* out_states)
{
    vpt_clear_error();
    if (!ctx || !rays || !states || !out_rgb || !x_new || !idsource || n < 0)
        return vpt_fail(VPT_E_INVALID, "vpt_ray_marching_batch: bad arguments");
    if (!ctx->has_scene) return vpt_fail(VPT_E_INVALID, "no scene set (vpt_set_scene)");
    if (ctx->h_scene.n < 6) return vpt_fail(VPT_E_INVALID, "rayMarching samples sphere 5: the scene has %d spheres", ctx->h_scene.n);
    if (!is_finite(steps) || !(steps > 0)) return vpt_fail(VPT_E_INVALID, "steps must be finite and > 0");
    if (n == 0) return VPT_OK;
    HIP_OK(hipSetDevice(ctx->device));
    vpt_ray* dr = nullptr;
    uint64_t *ds = nullptr, *dso = nullptr;
    double *dout = nullptr, *dxn = nullptr;
    int* did = nullptr;
    hipError_t e = hipMalloc((void**)&dr, sizeof(vpt_ray) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&ds, sizeof(uint64_t) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&dso, sizeof(uint64_t) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, sizeof(double) * 3 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&dxn, sizeof(double) * 3 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc((void**)&did, sizeof(int) * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(dr, rays, sizeof(vpt_ray) * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(ds, states, sizeof(uint64_t) * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dxn, x_new, sizeof(double) * 3 * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(did, idsource, sizeof(int) * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        ray_marching_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256)>>>(dr, ds, n, sigma_t, sigma_s, steps,
                                                                               ctx->d_scene, dout, dxn, did, dso);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out_rgb, dout, sizeof(double) * 3 * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(x_new, dxn, sizeof(double) * 3 * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(idsource, did, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out_states) e = hipMemcpy(out_states, dso, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(dr);
    (void)hipFree(ds);
    (void)hipFree(dso);
    (void)hipFree(dout);
    (void)hipFree(dxn);
    (void)hipFree(did);
    if (e != hipSuccess) return vpt_fail(VPT_E_HIP, "vpt_ray_marching_batch: %s", hipGetErrorString(e));
    return VPT_OK;
}

int vpt_math_probe(vpt_context* ctx, int fn, const double* x, const double* y, double* out, int n)
{
    vpt_clear_error();
    if (!ctx || !x || !y || !out || n < 0) return vpt_fail(VPT_E_INVALID, "vpt_math_probe: bad arguments");
    if (n == 0) return VPT_OK;
    HIP_OK(hipSetDevice(ctx->device));
    double *dx = nullptr, *dy = nullptr, *dout = nullptr;
    size_t b = sizeof(double) * (size_t)n;
    hipError_t e = hipMalloc((void**)&dx, b);
    if (e == hipSuccess) e = hipMalloc((void**)&dy, b);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, b);
    if (e == hipSuccess) e = hipMemcpy(dx, x, b, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dy, y, b, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        math_probe_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256)>>>(fn, dx, dy, dout, n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, b, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    (void)hipFree(dy);
    (void)hipFree(dout);
    if (e != hipSuccess) return vpt_fail(VPT_E_HIP, "vpt_math_probe: %s", hipGetErrorString(e));
    return VPT_OK;
}

int vpt_phase_probe(vpt_context* ctx, double g, const double din[3], const uint64_t* states, int n, double* dirs,
                    uint64_t* states_out, const double* wl, int nw, double* values)
{
    vpt_clear_error();
    if (!ctx || !din || n < 0 || nw < 0 || (n > 0 && (!states || !dirs || !states_out)) || (nw > 0 && (!wl || !values)))
        return vpt_fail(VPT_E_INVALID, "vpt_phase_probe: bad arguments");
    if (!is_finite(g) || g <= -1.0 || g >= 1.0) return vpt_fail(VPT_E_INVALID, "vpt_phase_probe: g must be in (-1, 1)");
    const int m = n > nw ? n : nw;
    if (m == 0) return VPT_OK;
    HIP_OK(hipSetDevice(ctx->device));
    uint64_t *dX = nullptr, *dXo = nullptr;
    double *dd = nullptr, *dw = nullptr, *dv = nullptr;
    const size_t n1 = (size_t)(n > 0 ? n : 1), w1 = (size_t)(nw > 0 ? nw : 1);
    hipError_t e = hipMalloc((void**)&dX, n1 * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void**)&dXo, n1 * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void**)&dd, 3 * n1 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&dw, 3 * w1 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&dv, w1 * sizeof(double));
    if (e == hipSuccess && n > 0) e = hipMemcpy(dX, states, (size_t)n * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nw > 0) e = hipMemcpy(dw, wl, 3 * (size_t)nw * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        phase_probe_kernel<<<dim3((unsigned)((m + 255) / 256)), dim3(256)>>>(g, din[0], din[1], din[2], dX, n, dd, dXo, dw,
                                                                            nw, dv);
        e = hipGetLastError();
    }
    if (e == hipSuccess && n > 0) e = hipMemcpy(dirs, dd, 3 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess && n > 0) e = hipMemcpy(states_out, dXo, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && nw > 0) e = hipMemcpy(values, dv, (size_t)nw * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(dX);
    (void)hipFree(dXo);
    (void)hipFree(dd);
    (void)hipFree(dw);
    (void)hipFree(dv);
    if (e != hipSuccess) return vpt_fail(VPT_E_HIP, "vpt_phase_probe: %s", hipGetErrorString(e));
    return VPT_OK;
}

}  // extern "C"

/* Debug (not part of include/vpt.h): scheduler statistics of the last pool launch made with
 * VPT_POOL_STATS=1 -- NSTATS counters, layout in vpt_pool.h. */
extern "C" int vpt_debug_pool_stats(unsigned long long* out)
{
    if (!g_pool_stats || !out) return VPT_E_INVALID;
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, g_pool_stats, NSTATS * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return VPT_OK;
}

/* debug: the section timers of builds made with -DVPT_SECTIONS=1 (vpt_device.h), 3 x SECT_N
 * counters (cycles, entries, active lanes) accumulated since the last call; returns VPT_E_INVALID otherwise */
extern "C" int vpt_debug_sections(unsigned long long* out)
{
#if VPT_SECTIONS
    if (!out) return VPT_E_INVALID;
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpyFromSymbol(out, HIP_SYMBOL(vpt::g_vpt_sect), 3 * vpt::SECT_N * sizeof(unsigned long long)));
    static const unsigned long long zero[3 * vpt::SECT_N] = {};
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(vpt::g_vpt_sect), zero, sizeof(zero)));
#if VPT_MIS_TU
    if (vpt_mis_sections_add(out)) return vpt_fail(VPT_E_HIP, "section timers of the EST = 1 unit");
#endif
    return VPT_OK;
#else
    (void)out;
    return VPT_E_INVALID;
#endif
}

/* debug: the per-workgroup timeline of the last VPT_POOL_STATS launch (vpt_pool.h TL0), 3 x TL_MAXWG */
extern "C" int vpt_debug_pool_timeline(unsigned long long* out)
{
    if (!g_pool_stats || !out) return VPT_E_INVALID;
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, g_pool_stats + TL0, 3 * TL_MAXWG * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return VPT_OK;
}

/* debug: the per-launch bound of ctx's pool renders lowered to 2^log2 samples per workgroup (0..26; 26 =
 * the production bound), so that a small render takes the multi-launch path that BASELINE configs[4]
 * (2^34 samples per GPU) takes in production (tests/test_gpu_parity.py).  Returns VPT_E_INVALID
 * outside 0..26. */
extern "C" int vpt_debug_set_launch_bound(vpt_context* ctx, int log2)
{
    if (!ctx || log2 < 0 || log2 > LAUNCH_LOG2_MAX) return vpt_fail(VPT_E_INVALID, "launch bound 2^%d outside 2^0..2^26", log2);
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->launch_log2 = log2;
    return VPT_OK;
}

/* debug, host only (no GPU): the launches a pool render of p's shard makes on `blocks` workgroups with the
 * bound 2^log2 -- the same units (tiles of 8 x 8 pixels x chunks, vpt_chunks.h) and the same split as
 * launch_pool.  Writes up to cap (unit0, nunits) pairs; returns the number of launches, or < 0. */
/* debug: task slots per workgroup pool of this build (vpt_pool.h POOL) */
extern "C" int vpt_debug_pool_tasks(void) { return POOL; }


extern "C" int64_t vpt_debug_launch_plan(const vpt_params* p, int blocks, int log2, uint64_t* unit0, uint64_t* nunits,
                                         int64_t cap)
{
    if (!p || blocks < 1 || log2 < 0 || log2 > LAUNCH_LOG2_MAX || p->spp <= 0 || p->width <= 0 || p->chunk_spp < 0)
        return VPT_E_INVALID;
    const int rows = vpt_shard_rows(p);
    const int chunk = p->chunk_spp > 0 ? (p->chunk_spp < p->spp ? p->chunk_spp : p->spp) : vpt_auto_chunk(p->spp);
    const vpt_chunk_layout lay = vpt_chunks(p->spp, chunk, p->chunk_spp == 0);
    const uint64_t units = (uint64_t)((p->width + 7) / 8) * (uint64_t)((rows + 7) / 8) * 64u * (uint64_t)lay.n;
    /* launch_pool's clamp: no more workgroups than the units fill (one pool of POOL tasks each) */
    const uint64_t need = (units + POOL - 1) / POOL;
    if ((uint64_t)blocks > need) blocks = (int)need;
    const uint64_t max_units = launch_max_units(blocks, lay.C, log2);
    int64_t k = 0;
    for (uint64_t u0 = 0; u0 < units; u0 += max_units, ++k) {
        if (k < cap && unit0 && nunits) {
            unit0[k] = u0;
            nunits[k] = units - u0 < max_units ? units - u0 : max_units;
        }
    }
    return k;
}

/* Test hooks of two internal checks (tests/test_gpu_parity.py), each undone by passing 0:
 * vpt_debug_karg_guard: bias != 0 makes pool_kernel's argument-layout guard fail (and clears the sticky
 * flag when 0), so vpt_render must return VPT_E_INTERNAL;
 * vpt_debug_kill_jump: the kill prediction's surface jump (DevScene::kp_sa, kp_sc) set to `draws` draws
 * instead of 2 n_mis + 5, so vpt_count_work's draw-count check must fail (0: the scene's own). */
extern "C" int vpt_debug_karg_guard(vpt_context* ctx, unsigned bias)
{
    vpt_clear_error();
    if (!ctx) return vpt_fail(VPT_E_INVALID, "NULL context");
    HIP_OK(hipSetDevice(ctx->device));
    ctx->guard_bias = bias;
    if (bias == 0) HIP_OK(hipMemset(ctx->d_guard, 0, sizeof(unsigned)));
    return VPT_OK;
}
extern "C" int vpt_debug_kill_jump(vpt_context* ctx, int draws)
{
    vpt_clear_error();
    if (!ctx || !ctx->has_scene) return vpt_fail(VPT_E_INVALID, "NULL context or no scene");
    if (draws < 0) return vpt_fail(VPT_E_INVALID, "draws must be >= 0");
    DevScene& h = ctx->h_scene;
    vpt_erand48_jump(draws > 0 ? draws : 2 * h.n_mis + 5, &h.kp_sa, &h.kp_sc);
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipMemcpy(ctx->d_scene, &h, sizeof h, hipMemcpyHostToDevice));
    return VPT_OK;
}
