/*
 * vpt_host.cpp -- host-only part of libvpt: reference defaults, errors, PPM output.
 *
 * Default scene/camera/medium: include/Sphere.cpp:11-22, src/rt.cpp:752-759, src/rt.cpp:794.
 * PPM writer: src/rt.cpp:812-820 with the clamp of src/rt.cpp:803 and toDisplayValue of
 * include/mathUtilities.h:43-45; byte-identical output ("P3\n%d %d\n255\n", then "%d %d %d "
 * per pixel, no trailing newline).  The reference formats serially with fprintf; here the
 * pixels are converted and formatted in parallel (std::thread) and written with one fwrite
 * (a 4096^2 P3 file is ~150 MB).
 */
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include <thread>

#include "vpt_internal.h"
#include "vpt_rng.h"

static thread_local std::string g_err;

int vpt_fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

void vpt_clear_error(void) { g_err.clear(); }

extern "C" {

const char* vpt_last_error(void) { return g_err.c_str(); }
int vpt_abi_version(void) { return VPT_ABI_VERSION; }

uint64_t vpt_stream_state(uint64_t seed, uint64_t pixel_idx, uint64_t sample)
{
    return vpt_stream_start(seed, pixel_idx, sample);
}

void vpt_default_params(vpt_params* p)
{
    if (!p) return;
    memset(p, 0, sizeof *p);
    p->width = 1024;
    p->height = 768;
    p->spp = 16;
    p->fb_format = VPT_FB_F32;
    p->medium.sigma_a = 0.001;
    p->medium.sigma_s = 0.009;
    p->medium.hg_g = 0.0;
    p->medium.max_depth = 0;
    p->medium.estimator = VPT_FREE_FLIGHT;
    p->medium.march_step = 0.1;  /* rayMarching3's step and light at src/rt.cpp:791 */
    p->medium.march_light = 7;
    p->seed = 0x5EED0001ull;
    /* Ray camera(Point(0, 11.2, 214), Vector(0, -0.042612, -1).normalize()) */
    double dx = 0, dy = -0.042612, dz = -1;
    double inv = 1.0 / sqrt(dx * dx + dy * dy + dz * dz);
    p->camera.o[0] = 0; p->camera.o[1] = 11.2; p->camera.o[2] = 214;
    p->camera.d[0] = dx * inv; p->camera.d[1] = dy * inv; p->camera.d[2] = dz * inv;
    p->fov_scale = 0.5095;
    p->band_rows = p->height;
    p->band_stride = 1;
    p->band_offset = 0;
}

static void set_sphere(vpt_sphere* s, double r, double px, double py, double pz, double cr, double cg, double cb,
                       double lr, double lg, double lb, int mat, const double* eta, const double* kappa, double alpha)
{
    memset(s, 0, sizeof *s);
    s->r = r;
    s->p[0] = px; s->p[1] = py; s->p[2] = pz;
    s->c[0] = cr; s->c[1] = cg; s->c[2] = cb;
    s->radiance[0] = lr; s->radiance[1] = lg; s->radiance[2] = lb;
    s->material = mat;
    if (eta) memcpy(s->eta, eta, sizeof s->eta);
    if (kappa) memcpy(s->kappa, kappa, sizeof s->kappa);
    s->alpha = alpha;
}

int vpt_default_scene(vpt_sphere* out, int cap)
{
    vpt_sphere s[10];
    static const double al_eta[3] = {1.66058, 0.88143, 0.521467};   /* aluminium */
    static const double al_kappa[3] = {9.2282, 6.27077, 4.83803};
    set_sphere(&s[0], 1e5, -1e5 - 49, 0, 0, .5, .5, .5, 0, 0, 0, 0, 0, 0, 0);            /* left wall */
    set_sphere(&s[1], 1e5, 1e5 + 49, 0, 0, .0, .0, .5, 0, 0, 0, 0, 0, 0, 0);             /* right wall */
    set_sphere(&s[2], 1e5, 0, 0, -1e5 - 81.6, .5, .5, .5, 0, 0, 0, 0, 0, 0, 0);          /* back wall */
    set_sphere(&s[3], 1e5, 0, -1e5 - 40.8, 0, .5, .5, .5, 0, 0, 0, 0, 0, 0, 0);          /* floor */
    set_sphere(&s[4], 1e5, 0, 1e5 + 40.8, 0, .5, .5, .5, 0, 0, 0, 0, 0, 0, 0);           /* ceiling */
    set_sphere(&s[5], 16.5, -23, -24.3, -34.6, 0, 0, 0, 0, 0, 0, 1, al_eta, al_kappa, 0.09); /* metal */
    set_sphere(&s[6], 16.5, 23, -24.3, -3.6, .0, .0, .9, 0, 0, 0, 0, 0, 0, 0);           /* blue */
    set_sphere(&s[7], 2, 0, 24.3, -35, 0, 0, 0, 100, 100, 0, 0, 0, 0, 0);                /* light */
    set_sphere(&s[8], 0, -23, 24.3, 0, 0, 0, 0, 6000, 0, 0, 0, 0, 0, 0);                 /* point light */
    set_sphere(&s[9], 2, 23, 24.3, 35, 0, 0, 0, 75, 75, 60, 0, 0, 0, 0);                 /* light */
    if (out) {
        int n = cap < 10 ? cap : 10;
        if (n > 0) memcpy(out, s, sizeof(vpt_sphere) * (size_t)n);
    }
    return 10;
}

int vpt_shard_rows(const vpt_params* p)
{
    if (!p || p->height <= 0 || p->band_rows <= 0 || p->band_stride <= 0 || p->band_offset < 0 ||
        p->band_offset >= p->band_stride)
        return 0;
    int nb = (p->height + p->band_rows - 1) / p->band_rows;
    int rows = 0;
    for (int b = p->band_offset; b < nb; b += p->band_stride) {
        int r0 = b * p->band_rows;
        int r1 = r0 + p->band_rows;
        if (r1 > p->height) r1 = p->height;
        rows += r1 - r0;
    }
    return rows;
}

/* ---- PPM ---- */
static inline double clamp01(double x) { return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x); }
static inline int to_display(double x) { return (int)(pow(clamp01(x), 1.0 / 2.2) * 255 + .5); }

static inline char* put_int(char* p, int v)
{
    /* "%d" for the values toDisplayValue can produce (0..255; NaN inputs give INT_MIN) */
    if (v >= 0 && v < 1000) {
        if (v >= 100) *p++ = (char)('0' + v / 100);
        if (v >= 10) *p++ = (char)('0' + (v / 10) % 10);
        *p++ = (char)('0' + v % 10);
        return p;
    }
    return p + sprintf(p, "%d", v);
}

int64_t vpt_encode_ppm(const void* rgb, int fb_format, int w, int h, char* buf, int64_t cap)
{
    vpt_clear_error();
    if (!rgb || w <= 0 || h <= 0 || (fb_format != VPT_FB_F32 && fb_format != VPT_FB_F64))
        return vpt_fail(VPT_E_INVALID, "vpt_encode_ppm: bad arguments");
    const int64_t npix = (int64_t)w * h;
    char header[64];
    int hl = snprintf(header, sizeof header, "P3\n%d %d\n%d\n", w, h, 255);
    unsigned hc = std::thread::hardware_concurrency();
    int nthreads = (int)(hc == 0 ? 1 : (hc > 16 ? 16 : hc));
    if (npix < 65536) nthreads = 1;
    const int64_t chunk = (npix + nthreads - 1) / nthreads;
    std::vector<std::vector<char>> parts((size_t)nthreads);
    std::vector<int64_t> lens((size_t)nthreads, 0);
    auto work = [&](int t) {
        int64_t p0 = t * chunk, p1 = p0 + chunk < npix ? p0 + chunk : npix;
        if (p0 >= p1) return;
        std::vector<char>& v = parts[(size_t)t];
        v.resize((size_t)(p1 - p0) * 3 * 12);
        char* q = v.data();
        for (int64_t p = p0; p < p1; ++p) {
            for (int c = 0; c < 3; ++c) {
                double x = fb_format == VPT_FB_F32 ? (double)((const float*)rgb)[3 * p + c]
                                                   : ((const double*)rgb)[3 * p + c];
                q = put_int(q, to_display(clamp01(x)));
                *q++ = ' ';
            }
        }
        lens[(size_t)t] = q - v.data();
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    int64_t total = hl;
    for (int t = 0; t < nthreads; ++t) total += lens[(size_t)t];
    if (!buf) return total;
    if (cap < total) return vpt_fail(VPT_E_INVALID, "vpt_encode_ppm: buffer too small (%lld < %lld)", (long long)cap,
                                     (long long)total);
    memcpy(buf, header, (size_t)hl);
    int64_t off = hl;
    for (int t = 0; t < nthreads; ++t) {
        if (lens[(size_t)t]) memcpy(buf + off, parts[(size_t)t].data(), (size_t)lens[(size_t)t]);
        off += lens[(size_t)t];
    }
    return total;
}

int vpt_write_ppm(const char* path, const void* rgb, int fb_format, int w, int h)
{
    int64_t n = vpt_encode_ppm(rgb, fb_format, w, h, NULL, 0);
    if (n < 0) return (int)n;
    std::vector<char> buf((size_t)n);
    if (vpt_encode_ppm(rgb, fb_format, w, h, buf.data(), n) != n) return VPT_E_INVALID;
    FILE* f = path ? fopen(path, "w") : NULL;
    if (!f) return vpt_fail(VPT_E_IO, "vpt_write_ppm: cannot open '%s'", path ? path : "(null)");
    size_t wr = fwrite(buf.data(), 1, (size_t)n, f);
    int rc = fclose(f);
    if (wr != (size_t)n || rc != 0) return vpt_fail(VPT_E_IO, "vpt_write_ppm: short write to '%s'", path);
    return VPT_OK;
}

}  // extern "C"
