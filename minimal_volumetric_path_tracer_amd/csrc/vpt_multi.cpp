/*
 * vpt_multi.cpp -- one image on several GPUs of ONE process, through the C ABI (include/vpt.h).
 *
 * The reference renders with one OpenMP loop over the pixels of one host (src/rt.cpp:767-805); a
 * C++ caller replacing that loop with libvpt calls vpt_render_multi (or the persistent vpt_multi_*
 * handle) to use every GPU of the node without a launcher.  Every (pixel, sample) owns its random
 * stream, so the image shards with no data-path exchange: device g renders the file-row bands
 * g, g + n, g + 2n, ... (interleaved bands balance the per-row cost) into one compact strip, and
 * the strips are gathered to device 0 over RCCL -- one communicator per device from
 * ncclCommInitAll, grouped ncclSend / ncclRecv (RCCL has no gather primitive; this is the same
 * pattern torch.distributed.gather issues).  The image is bit-identical to vpt_render for any
 * device count and band size (the chunk layout and the per-sample streams do not depend on them).
 *
 * The Python path (minimal_volumetric_path_tracer_amd/distributed.py: one process per GPU,
 * torch.distributed "nccl") uses the same band layout.
 *
 * Debug mode (vpt_debug_multi_create_shared, not part of include/vpt.h): n logical ranks on ONE device --
 * n contexts, n streams, n strips -- with a same-device stream-ordered copy of each strip in place of
 * the grouped ncclSend / ncclRecv (RCCL refuses two ranks on one device).  Everything else of the n > 1
 * path runs as on n GPUs: buffers, band plan, per-rank renders on their own streams, synchronisation,
 * the reassembly copies; tests/test_gpu_multi.py checks it bit for bit against vpt_render on a
 * one-GPU box.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdint.h>
#include <string.h>

#include <vector>

#include "vpt_internal.h"

#define MULTI_DEFAULT_BAND_ROWS 16

struct vpt_multi {
    int n;                              /* logical ranks 0 .. n-1 */
    std::vector<int> dev;               /* rank g's device: g, or 0 for every rank in the shared debug mode */
    bool shared = false;                /* debug: all ranks on device 0, strips copied instead of sent */
    std::vector<vpt_context*> ctx;
    std::vector<hipStream_t> stream;
    std::vector<ncclComm_t> comm;       /* empty when n == 1 or shared */
    std::vector<void*> strip;           /* device g's strip (g >= 1); device 0 renders into gather */
    std::vector<size_t> strip_bytes;
    void* gather = nullptr;             /* on device 0: n slots of `slot_bytes` */
    size_t gather_bytes = 0;
};

namespace {

int hip_fail(const char* what, hipError_t e) { return vpt_fail(VPT_E_HIP, "%s: %s", what, hipGetErrorString(e)); }
int nccl_fail(const char* what, ncclResult_t r) { return vpt_fail(VPT_E_HIP, "%s: %s", what, ncclGetErrorString(r)); }

/* file rows of band layout (band_rows, stride n, offset g), in output order */
int shard_rows_of(int height, int band_rows, int n, int g)
{
    vpt_params q;
    memset(&q, 0, sizeof q);
    q.height = height;
    q.band_rows = band_rows;
    q.band_stride = n;
    q.band_offset = g;
    return vpt_shard_rows(&q);
}

int ensure_device_buffer(int device, void** buf, size_t* have, size_t want)
{
    if (*have >= want) return VPT_OK;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail("vpt_multi: hipSetDevice", e);
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    e = hipMalloc(buf, want);
    if (e != hipSuccess) return hip_fail("vpt_multi: hipMalloc", e);
    *have = want;
    return VPT_OK;
}

/* waits for every device's stream (error paths: nothing the call enqueued may still run when it
 * returns, since the caller may free or reuse what it passed) */
void sync_all(vpt_multi* m)
{
    for (int g = 0; g < m->n; ++g) {
        if (!m->stream[g]) continue;
        (void)hipSetDevice(m->dev[g]);
        (void)hipStreamSynchronize(m->stream[g]);
    }
}

}  // namespace


namespace {

/* The gathered strips -> file order, as copies: strip g (at g * slot of the gather buffer) holds
 * device g's bands g, g + n, g + 2n, ... of `band` rows each (the last band may be short), rows of
 * row_bytes, so band b is ONE contiguous run in both the strip and the file.  Returns false when a
 * strip would overrun its slot. */
struct BandCopy {
    size_t src, dst, bytes;
};
bool band_plan(size_t slot, int n, int height, int band, size_t row_bytes, std::vector<BandCopy>& plan)
{
    plan.clear();
    const int nbands = (height + band - 1) / band;
    std::vector<size_t> next(n, 0);  /* next strip row per device */
    for (int b = 0; b < nbands; ++b) {
        const int g = b % n, r0 = b * band, r1 = r0 + band < height ? r0 + band : height;
        const size_t rows = (size_t)(r1 - r0);
        if ((next[g] + rows) * row_bytes > slot) return false;
        plan.push_back({(size_t)g * slot + next[g] * row_bytes, (size_t)r0 * row_bytes, rows * row_bytes});
        next[g] += rows;
    }
    return true;
}

}  // namespace

extern "C" {

/* The reassembly plan of vpt_multi_render applied on the host (staging = the gather buffer's bytes).
 * Exported for tests (not part of include/vpt.h): the n > 1 layout is checked on the CPU without
 * RCCL; vpt_multi_render applies the same plan with device-to-host copies. */
int vpt_debug_band_reorder(const void* staging, size_t slot, int n, int height, int band, size_t row_bytes, void* out)
{
    if (!staging || !out || n < 1 || height < 1 || band < 1) return VPT_E_INVALID;
    std::vector<BandCopy> plan;
    if (!band_plan(slot, n, height, band, row_bytes, plan)) return VPT_E_INVALID;
    for (const BandCopy& c : plan) memcpy((unsigned char*)out + c.dst, (const unsigned char*)staging + c.src, c.bytes);
    return VPT_OK;
}

void vpt_multi_destroy(vpt_multi* m)
{
    if (!m) return;
    for (int g = 0; g < m->n; ++g) {
        if (g < (int)m->stream.size() && m->stream[g]) {
            (void)hipSetDevice(m->dev[g]);
            (void)hipStreamSynchronize(m->stream[g]);
        }
    }
    for (ncclComm_t c : m->comm)
        if (c) (void)ncclCommDestroy(c);
    for (int g = 0; g < m->n; ++g) {
        (void)hipSetDevice(m->dev[g]);
        if (g < (int)m->strip.size() && m->strip[g]) (void)hipFree(m->strip[g]);
        if (g < (int)m->stream.size() && m->stream[g]) (void)hipStreamDestroy(m->stream[g]);
        if (g < (int)m->ctx.size() && m->ctx[g]) vpt_context_destroy(m->ctx[g]);
    }
    if (m->gather) {
        (void)hipSetDevice(0);
        (void)hipFree(m->gather);
    }
    delete m;
}

/* n ranks on devices 0 .. n-1 (shared: all on device 0, no communicator) */
static int multi_create(int n_gpus, bool shared, vpt_multi** out)
{
    vpt_clear_error();
    if (!out) return vpt_fail(VPT_E_INVALID, "vpt_multi_create: out is NULL");
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess) return hip_fail("vpt_multi_create: hipGetDeviceCount", e);
    if (n_gpus < 1 || (!shared && n_gpus > ndev) || ndev < 1 || n_gpus > 64)
        return vpt_fail(VPT_E_INVALID, "vpt_multi_create: n_gpus %d of %d devices", n_gpus, ndev);
    vpt_multi* m = new vpt_multi();
    m->n = n_gpus;
    m->shared = shared;
    m->dev.resize(n_gpus);
    for (int g = 0; g < n_gpus; ++g) m->dev[g] = shared ? 0 : g;
    m->ctx.assign(n_gpus, nullptr);
    m->stream.assign(n_gpus, nullptr);
    m->strip.assign(n_gpus, nullptr);
    m->strip_bytes.assign(n_gpus, 0);
    for (int g = 0; g < n_gpus; ++g) {
        int rc = vpt_context_create(m->dev[g], &m->ctx[g]);
        if (rc) {
            vpt_multi_destroy(m);
            return rc;
        }
        e = hipSetDevice(m->dev[g]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->stream[g], hipStreamNonBlocking);
        if (e != hipSuccess) {
            vpt_multi_destroy(m);
            return hip_fail("vpt_multi_create: stream", e);
        }
    }
    if (n_gpus > 1 && !shared) {
        m->comm.assign(n_gpus, nullptr);
        std::vector<int> devs(n_gpus);
        for (int g = 0; g < n_gpus; ++g) devs[g] = g;
        ncclResult_t r = ncclCommInitAll(m->comm.data(), n_gpus, devs.data());
        if (r != ncclSuccess) {
            m->comm.clear();
            vpt_multi_destroy(m);
            return nccl_fail("vpt_multi_create: ncclCommInitAll", r);
        }
    }
    *out = m;
    return VPT_OK;
}

int vpt_multi_create(int n_gpus, vpt_multi** out) { return multi_create(n_gpus, false, out); }

/* debug (tests): n logical ranks on device 0, strips copied on the device instead of sent over RCCL */
int vpt_debug_multi_create_shared(int n_ranks, vpt_multi** out) { return multi_create(n_ranks, true, out); }

int vpt_multi_set_scene(vpt_multi* m, const vpt_sphere* spheres, int n)
{
    vpt_clear_error();
    if (!m) return vpt_fail(VPT_E_INVALID, "vpt_multi_set_scene: NULL handle");
    for (int g = 0; g < m->n; ++g) {
        int rc = vpt_set_scene(m->ctx[g], spheres, n);
        if (rc) return rc;
    }
    return VPT_OK;
}

int vpt_multi_render(vpt_multi* m, const vpt_params* p, void* h_out)
{
    vpt_clear_error();
    if (!m || !p || !h_out) return vpt_fail(VPT_E_INVALID, "vpt_multi_render: NULL argument");
    if (p->band_stride != 1 || p->band_offset != 0 || p->band_rows < 1)
        return vpt_fail(VPT_E_INVALID, "vpt_multi_render: params must describe the whole image (band_stride 1, offset 0)");
    if (p->width < 1 || p->height < 1) return vpt_fail(VPT_E_INVALID, "vpt_multi_render: image %dx%d", p->width, p->height);
    const int n = m->n, H = p->height;
    /* band size: the caller's when it cuts the image, else 16 rows (distributed.py's default) */
    const int band = n == 1 ? H : (p->band_rows < H ? p->band_rows : MULTI_DEFAULT_BAND_ROWS);
    const size_t esize = p->fb_format == VPT_FB_F64 ? sizeof(double) : sizeof(float);
    const size_t row_bytes = (size_t)p->width * 3 * esize;
    std::vector<int> rows(n);
    int cap = 0;
    for (int g = 0; g < n; ++g) {
        rows[g] = shard_rows_of(H, band, n, g);
        cap = rows[g] > cap ? rows[g] : cap;
    }
    const size_t slot = (size_t)cap * row_bytes;
    int rc = ensure_device_buffer(0, &m->gather, &m->gather_bytes, slot * (size_t)n);
    if (rc) return rc;
    for (int g = 1; g < n; ++g) {
        rc = ensure_device_buffer(m->dev[g], &m->strip[g], &m->strip_bytes[g], slot);
        if (rc) return rc;
    }
    /* every device renders its bands on its own stream */
    for (int g = 0; g < n; ++g) {
        if (rows[g] == 0) continue;
        vpt_params q = *p;
        q.band_rows = band;
        q.band_stride = n;
        q.band_offset = g;
        void* dst = g == 0 ? m->gather : m->strip[g];
        rc = vpt_render_device(m->ctx[g], &q, dst, (void*)m->stream[g]);
        if (rc) {
            sync_all(m);
            return rc;
        }
    }
    /* strips -> device 0, slot g (stream-ordered after each render) */
    if (n > 1 && m->shared) {  /* debug: the same movement as the send / recv pairs, on one device */
        hipError_t e = hipSetDevice(0);
        for (int g = 1; g < n && e == hipSuccess; ++g) {
            const size_t bytes = (size_t)rows[g] * row_bytes;
            if (bytes == 0) continue;
            e = hipMemcpyAsync((unsigned char*)m->gather + (size_t)g * slot, m->strip[g], bytes, hipMemcpyDeviceToDevice,
                               m->stream[g]);
        }
        if (e != hipSuccess) {
            sync_all(m);
            return hip_fail("vpt_multi_render: strip copy (shared debug mode)", e);
        }
    } else if (n > 1) {
        ncclResult_t r = ncclGroupStart();
        for (int g = 1; g < n && r == ncclSuccess; ++g) {
            const size_t bytes = (size_t)rows[g] * row_bytes;
            if (bytes == 0) continue;
            r = ncclSend(m->strip[g], bytes, ncclUint8, 0, m->comm[g], m->stream[g]);
            if (r == ncclSuccess)
                r = ncclRecv((unsigned char*)m->gather + (size_t)g * slot, bytes, ncclUint8, g, m->comm[0], m->stream[0]);
        }
        ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess) {
            sync_all(m);
            return r != ncclSuccess ? nccl_fail("vpt_multi_render: send/recv", r) : nccl_fail("vpt_multi_render: ncclGroupEnd", r2);
        }
    }
    for (int g = n - 1; g >= 0; --g) {
        hipError_t e = hipSetDevice(m->dev[g]);
        if (e == hipSuccess) e = hipStreamSynchronize(m->stream[g]);
        if (e != hipSuccess) {
            sync_all(m);
            return hip_fail("vpt_multi_render: synchronize", e);
        }
    }
    /* gathered strips -> file order */
    if (n == 1) {
        hipError_t e = hipMemcpy(h_out, m->gather, (size_t)H * row_bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail("vpt_multi_render: hipMemcpy", e);
        return VPT_OK;
    }
    /* each band straight from the gather buffer into its file rows (no host staging, no host
     * reorder pass): one device-to-host copy per band, queued back to back on device 0's stream */
    std::vector<BandCopy> plan;
    if (!band_plan(slot, n, H, band, row_bytes, plan))
        return vpt_fail(VPT_E_INVALID, "vpt_multi_render: band layout does not fit the strips");
    hipError_t e = hipSetDevice(0);
    for (size_t i = 0; i < plan.size() && e == hipSuccess; ++i)
        e = hipMemcpyAsync((unsigned char*)h_out + plan[i].dst, (const unsigned char*)m->gather + plan[i].src, plan[i].bytes,
                           hipMemcpyDeviceToHost, m->stream[0]);
    if (e == hipSuccess) e = hipStreamSynchronize(m->stream[0]);
    if (e != hipSuccess) {
        sync_all(m);
        return hip_fail("vpt_multi_render: device-to-host copy", e);
    }
    return VPT_OK;
}

int vpt_render_multi(const vpt_sphere* spheres, int n, const vpt_params* p, int n_gpus, void* h_out)
{
    vpt_multi* m = nullptr;
    int rc = vpt_multi_create(n_gpus, &m);
    if (rc == VPT_OK) rc = vpt_multi_set_scene(m, spheres, n);
    if (rc == VPT_OK) rc = vpt_multi_render(m, p, h_out);
    vpt_multi_destroy(m);
    return rc;
}

}  // extern "C"
