/*
 * vpt_chunks.h -- how a pixel's spp samples are cut into partial sums (work units of the pool
 * kernel).  Plain C, shared by the kernels, the host library and the oracle (oracle/vpt_oracle.c),
 * so that the GPU and the oracle sum in the same order.
 *
 * The reference adds a pixel's samples one after the other (acc = L + acc, src/rt.cpp:794).  The
 * build sums each chunk that way and then adds the chunk sums in chunk order.  Layouts:
 *   uniform (taper = 0): chunks of C samples (the last one may be shorter); C >= spp is the
 *     reference's own order;
 *   tapered (taper = 1, the default when vpt_params.chunk_spp == 0): chunks of C over the first
 *     spp - R samples, R = min(spp, 2C), then the last R samples in chunks of a third of what is
 *     left (rounded up): for C = 32, R = 64 -> 22, 14, 10, 6, 4, 3, 2, 1, 1, 1.  spp <= C is one
 *     chunk (the reference's order).
 * Why tapered: a task runs its unit's samples one after the other, one path iteration per pass
 * through the workgroup's task pool (~18 us at full load), so a 32-sample unit takes ~1.4 ms
 * however idle the GPU is.  The pool kernel hands units out chunk-major, and with this layout the
 * work still queued behind any unit is at least twice that unit (sum of later chunks >= 2 x the
 * chunk), which covers its latency down to ~1/8 of a 1024^2 x 256 image per GPU (the 8-GPU split):
 * the launch ends on one- and two-sample units instead of a long sequential tail.
 */
#ifndef VPT_CHUNKS_H
#define VPT_CHUNKS_H

#ifdef __HIPCC__
#define VPT_CK __host__ __device__ static inline
#else
#define VPT_CK static inline
#endif

typedef struct {
    int spp, C;   /* samples per pixel, chunk size */
    int head;     /* samples covered by chunks of C */
    int n_head;   /* number of those chunks */
    int n;        /* chunks in total */
} vpt_chunk_layout;

VPT_CK vpt_chunk_layout vpt_chunks(int spp, int C, int taper)
{
    vpt_chunk_layout L;
    if (C <= 0 || C > spp) C = spp;
    L.spp = spp;
    L.C = C;
    L.head = (taper && spp > C) ? spp - (spp < 2 * C ? spp : 2 * C) : spp;
    L.n_head = (L.head + C - 1) / C;
    L.n = L.n_head;
    for (int rem = spp - L.head; rem > 0; rem -= (rem + 2) / 3) L.n++;
    return L;
}

/* auto chunk size (vpt_params.chunk_spp == 0): 32 samples (A/B at 1024^2 x 256 spp), more
 * above 4096 spp so that a pixel has at most 128 chunks + the taper (4096^2 x 8192 spp on one GPU:
 * 2.3e9 work units < 2^32, 55 GB of partials); spp <= 32 is one chunk */
#ifndef VPT_AUTO_CHUNK_MIN
#define VPT_AUTO_CHUNK_MIN 32
#endif
VPT_CK int vpt_auto_chunk(int spp)
{
    int c = (spp + 127) / 128;
    if (c < VPT_AUTO_CHUNK_MIN) c = VPT_AUTO_CHUNK_MIN;
    return c < spp ? c : spp;
}

/* samples [*s0, *s1) of chunk c */
VPT_CK void vpt_chunk_range(const vpt_chunk_layout* L, int c, int* s0, int* s1)
{
    if (c < L->n_head) {
        *s0 = c * L->C;
        *s1 = *s0 + L->C < L->head ? *s0 + L->C : L->head;
        return;
    }
    int s = L->head, rem = L->spp - L->head, sz = (rem + 2) / 3;
    for (int k = L->n_head; k < c; ++k) {
        s += sz;
        rem -= sz;
        sz = (rem + 2) / 3;
    }
    *s0 = s;
    *s1 = s + sz;
}

/* the chunk whose last sample is s1 - 1 */
VPT_CK int vpt_chunk_of_end(const vpt_chunk_layout* L, int s1)
{
    if (s1 <= L->head) return (s1 - 1) / L->C;
    int c = L->n_head, s = L->head, rem = L->spp - L->head;
    while (1) {
        const int sz = (rem + 2) / 3;
        if (s1 <= s + sz) return c;
        s += sz;
        rem -= sz;
        ++c;
    }
}

#endif
