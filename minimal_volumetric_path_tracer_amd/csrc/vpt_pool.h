/*
 * vpt_pool.h -- workgroup task pool in LDS: cross-wave compaction of pending path events.
 *
 * A task is one (pixel, chunk of samples) work unit in flight: its path state (ray, throughput,
 * radiance, chunk sum, erand48 state, pending event) lives in LDS, not in a lane.  A path loop
 * iteration of the reference (include/vptShadeMethods.h:1278-1336 / :1345-1481) is split into three
 * stages:
 *     A  intersection + light pick + distance sample   (decide(), vpt_device.h)
 *     S  surface event: pLight + MISv2 + bdsf           (surface_event()) + next roulette draw
 *     M  medium event: single scattering + phase sample (medium_event())  + next roulette draw
 * Pending tasks wait in rings keyed by what their next stage will branch on, so that a batch runs
 * one side of the divergent code only:
 *     ring 0     stage A
 *     ring 1..4  stage S: diffuse surface + sphere light, diffuse + point light, metal, other
 *     ring 5..6  stage M: sphere light, point light
 A wave returns its finished tasks to the rings of their next stage (lock-free: one LDS atomic per
 * ring reserves positions), claims up to 64 tasks of the fullest ring (one CAS on its head), runs
 * that ONE stage with (nearly) every lane busy -- an S/M batch then runs stage A on the same lanes --
 * and stores the states back.  The pool is larger than the workgroup (880 tasks for 512 lanes), so
 * there is nearly always a full batch of some ring.
 *
 * Determinism: a task runs its unit's samples strictly in order and adds each sample to the
 * chunk sum as the reference adds to its pixel (acc = L + acc, src/rt.cpp:794); chunk sums are
 * written to a partial buffer and combined in chunk order by reduce_kernel.  Which wave or lane
 * runs a stage changes nothing in the arithmetic, so images are bit-identical to the oracle
 * (oracle/vpt_oracle.c orc_render_chunked) for any schedule, GPU count or pool size.
 */
#ifndef VPT_POOL_H
#define VPT_POOL_H

#include "vpt_chunks.h"
#include "vpt_device.h"

namespace vpt {

#ifndef VPT_POOL_DEBUG
#define VPT_POOL_DEBUG 0
#endif
/* One 512-thread workgroup per CU (8 waves = 2 per SIMD) sharing one pool of 880 tasks (161 KB of
 * LDS), vs two 256-thread workgroups of 440 each: A/B 46.48 -> 46.01 ms at 1024^2 x 256, 1/8 shard
 * 6.76 -> 6.47 ms (more tasks per ring, fuller batches, half the unit rings to drain at the end). */
#ifndef VPT_POOL_THREADS
#define VPT_POOL_THREADS 512  /* threads per workgroup: its waves share one task pool */
#endif
#ifndef VPT_POOL_WGS
#define VPT_POOL_WGS 1      /* workgroups per CU (occupancy target; LDS and VGPR budgets follow) */
#endif
/* Kill-predicting rings: a diffuse surface or medium event whose path the next roulette draw (or the
 * depth cap) will end is known when decide() picks the event -- the draws in between are a fixed
 * number (2 n_mis + 4 for a diffuse surface event: two per MIS light cone, the BSDF sample of MISv2
 * and bdsf's cosine sample; 4 for a medium event: the light cone and the phase sample), and a dead
 * path's stream is never read again (the next sample starts its own).  Such tasks wait in rings of
 * their own, so their batches skip the continuation (bdsf / the phase sample, the throughput and ray
 * updates) -- the same radiance, the same bits. */
#ifndef VPT_KILL_RINGS
#define VPT_KILL_RINGS 1
#endif
#ifndef VPT_SCHED_PRIO
#define VPT_SCHED_PRIO 3    /* s_setprio level of the scheduler's critical section (0: off; A/B 3 vs 0: +0.7 %) */
#endif
#ifndef VPT_PREP_TRIES
#define VPT_PREP_TRIES 3    /* samples a lane may start per preparation round (round 2, A/B 1 / 2 / 4 / 8: FF 52.16 / 52.02 / 53.70 / 53.85 ms, MIS 248.1 / 245.2 / 251.9 / 252.0; round 4, with the kill rings every lane of a dying batch restarts: 2 / 3: FF 42.84 / 42.75, MIS + HG 194.1 / 193.5) */
#endif
#ifndef VPT_PREP_ROUNDS
#define VPT_PREP_ROUNDS 2   /* stage-A preparation rounds per batch before unready lanes park (0: no cap; round-2 A/B 1 / 2 / 3 / none: 4949 / 5104 / 5052 / 5020 Ms/s; round 3: see VPT_PREP_MORE_MIN) */
#endif
#ifndef VPT_PREP_MORE_MIN
/* fewer lanes than this still without a path after a round: parked at once, no further round.  The
 * second round ran in 99.4 % of batches for ~5 lanes and took 7.1 % of the kernel's wave-time
 * (profiles/r03/sections_ff_prep.txt).  A/B (kernel ms FF / MIS+HG, profiles/r03/ab_session2.txt):
 * 0 (always a second round) 49.87 / 222.4; 8 48.46 / 216.1; 16 48.41 / 216.1; 24 48.39 / 215.9;
 * 32 48.39 / 215.9; one round only (VPT_PREP_ROUNDS=1) 48.11 / 218.1 */
#define VPT_PREP_MORE_MIN 24
#endif
constexpr int NF = 18;      /* doubles per task */
/* rings: A; S diffuse x (sphere light, point light), metal, other; M (sphere light, point light);
 * with VPT_KILL_RINGS the four diffuse-surface / medium rings again for tasks the event ends */
constexpr int R_A = 0, R_S = 1, R_M = 5, R_SD = 7, R_MD = 9;
constexpr int NR = VPT_KILL_RINGS ? 11 : 7, R_DONE = NR;
/* the scheduler's counters (TaskPool::ctl): ring tails, ring heads, slots retired, the unit ring's
 * tail, queue exhausted, refill in progress, the unit ring's head (one lane-parallel read fetches all) */
constexpr int C_TAIL = 0, C_HEAD = NR, C_DONE = 2 * NR, C_UTAIL = 2 * NR + 1, C_EXH = 2 * NR + 2, C_RFL = 2 * NR + 3,
              C_UHEAD = 2 * NR + 4, NCTL = 2 * NR + 5;
static_assert(NCTL <= 64, "the counters are read lane-parallel by one wave");
#ifndef VPT_UREFILL
#define VPT_UREFILL 128
#endif
constexpr int UREFILL = VPT_UREFILL, URING = 2 * UREFILL;  /* work-unit ring: one global queue atomic per UREFILL units */
static_assert(URING >= 2 * UREFILL, "a refill (at most UREFILL entries from utail < uhead + UREFILL) must stay below uhead + URING");
/* task slots per workgroup: as many as the CU's 160 KB of LDS hold beside the counters, the unit ring
 * (and the debug build's section timers) -- 182 B each with 7 rings (880 slots), 190 B with 11 */
#ifdef VPT_POOL_SIZE
constexpr int POOL = VPT_POOL_SIZE;
#else
constexpr int POOL = NR == 7 ? 880
                                     : (163840 - 4 * NCTL - 4 * URING - (VPT_SECTIONS ? 8 * 3 * SECT_USED * 4 : 0) - 64) /
                                           (NF * 8 + 8 + 4 * 4 + 2 * NR);
#endif

/* debug statistics, in builds with -DVPT_POOL_DEBUG=1 (=2: top-level cycle split only, cheaper;
 * scripts/build_variant.sh) run with
 * VPT_POOL_STATS=1 (vpt_debug_pool_stats, scripts/pool_stats.py): [0-6] batches per ring, [7-13] lanes
 * per ring, [14] idle polls, [15] claim retries, [16-19] cycles in stage A/S/M/scheduling, [20]
 * stage-A preparation rounds, [21] samples started, [22] cycles preparing, [23] cycles in decide */
constexpr int NSTATS = 24;
/* debug timeline (s_memrealtime, 100 MHz) after the counters: per workgroup b, stats[TL0 + 3b + k] =
 * min over its waves of k=0 start, k=1 first sight of the exhausted work queue, k=2 ~exit time */
constexpr int TL0 = 32, TL_MAXWG = 4096;
__device__ __forceinline__ void dbg_tl(unsigned long long* stats, int k, bool inv)
{
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x < (unsigned)TL_MAXWG) atomicMin(&stats[TL0 + 3 * blockIdx.x + k], inv ? ~t : t);
}
struct ADbg {
    unsigned long long rounds, samples, c_prep, c_decide;
};
__device__ __forceinline__ unsigned long long dbg_clock(bool dbg) { return dbg ? __builtin_amdgcn_s_memtime() : 0; }

/* F_TD: the pending event's distance -- surface t for stage S, sampled distance for stage M (each
 * stage reads only its own); F_KEY: the unit's pixel stream key (vpt_stream_key), as raw bits */
enum { F_OX = 0, F_OY, F_OZ, F_DX, F_DY, F_DZ, F_BX, F_BY, F_BZ, F_LX, F_LY, F_LZ, F_AX, F_AY, F_AZ, F_TD, F_KEY,
       F_PDF };

struct TaskPool {
    double2 f2[NF / 2][POOL]; /* SoA of field pairs (F_OX, F_OY), (F_OZ, F_DX), ...: one 16-B LDS access per pair */
    uint64_t X[POOL];        /* erand48 state */
    uint4 w[POOL];           /* pix (x | camera row << 16), c1 (one past the unit's last sample; 0 = no unit),
                              * samp (next sample | in_path << 31), evw (depth | id << 16 | src << 24 | killed << 31) */
    uint16_t ring[NR][POOL]; /* slots waiting, per ring */
    /* the scheduler's counters, contiguous so that one lane-parallel LDS read fetches them all:
     * monotonic ring tails and heads, slots retired, the unit ring's tail, queue exhausted */
    int ctl[NCTL];
    uint32_t uring[URING];   /* prefetched work units (refilled by one wave at a time under the C_RFL flag, taken by CAS on ctl[C_UHEAD]) */
};

/* Lock-free rings: an entry is the slot and the lap of its ring position,
 * slot | (position / POOL mod 128) << 9.  A producer reserves positions with one atomic add on the
 * ring's tail and then writes the entries; a consumer reads entries from the head, keeps the prefix
 * whose lap tags are current (written), and claims exactly that prefix with one CAS on the head.
 * An entry is read before the claim, and its position cannot be reserved again before the claim
 * (tail - head < POOL), so a claimed entry is never a later lap's. */
constexpr int SLOT_BITS = POOL > 512 ? 10 : 9, SLOT_MASK = (1 << SLOT_BITS) - 1, LAP_MASK = (1 << (16 - SLOT_BITS)) - 1;
static_assert(POOL <= (1 << SLOT_BITS), "slot ids must fit the ring entry");
__device__ __forceinline__ uint16_t ring_entry(int slot, int pos)
{
    return (uint16_t)(slot | (((pos / POOL) & LAP_MASK) << SLOT_BITS));
}

__device__ __forceinline__ int lds_peek(const int* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct PoolParams {
    int w, h, spp, rows;
    int band_rows, band_stride, band_offset;
    int tiles_x, nch;
    vpt_chunk_layout lay;   /* chunks of a pixel's samples (vpt_chunks.h) */
    unsigned level_units;   /* units per chunk index: 64 pixels x tiles */
    unsigned nunits;        /* units of this launch: unit0, unit0 + 1, ... */
    unsigned unit0;
    uint64_t seed;
    double o[3], d[3], cx[3], cy[3];
    /* log2 of level_units, tiles_x, band_rows, band_stride and the chunk size C when they are powers of
     * two, else -1: the unit decode and the partial's address divide by them (a u32 division is ~15
     * VALU instructions; every lane of a wave runs it when one lane takes or finishes a unit) */
    int sh_lu, sh_tx, sh_br, sh_bs, sh_c;
    double rw, rh;          /* 1/w, 1/h when w, h are powers of two (then u / w == u * rw exactly), else 0 */
    double* partials;       /* nch * rows * w * 3: chunk-major, so the units of one chunk level (handed
                             * out together, 8x8 tiles) write neighbouring 24-B records that merge into
                             * whole lines in L2 (pixel-major wrote 24 B per 128-B line: 2x the WRITE_SIZE) */
    unsigned* queue;
    unsigned* guard;        /* the argument-layout guard's flag (VPT_P_KARG): set when the check fails */
    unsigned guard_bias;    /* 0; vpt_debug_karg_guard sets it to make the check fail (its test) */
};

/* VPT_P_KARG: the launch parameters read where they are used, by scalar loads from the kernel-argument
 * segment through an opaque pointer (the kernel's first argument sits at offset 0), instead of held
 * in SGPRs for the whole kernel: the unit hand-out, camera, partial-store and refill blocks use them
 * once per batch or less. */
#ifndef VPT_P_KARG
#define VPT_P_KARG 1
#endif
#if VPT_P_KARG && defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) PoolParams PoolParamsK;
__device__ __forceinline__ PoolParamsK& pool_params_at_use()
{
    uint64_t a = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    __asm__ volatile("" : "+s"(a));
    return *(PoolParamsK*)a;
}
#define VPT_PARAMS(Pin) PoolParamsK& P = pool_params_at_use(); (void)(Pin)
#else
#define VPT_PARAMS(Pin) const PoolParams& P = (Pin)
#endif

/* vpt_chunk_of_end / vpt_chunk_range on a copy of the layout (the parameters may sit in the constant
 * address space, VPT_P_KARG) */
template <class LAY>
__device__ __forceinline__ int vpt_chunk_of_end_lay(const LAY& lay, int c1)
{
    const vpt_chunk_layout l = lay;
    return vpt_chunk_of_end(&l, c1);
}
template <class LAY>
__device__ __forceinline__ void vpt_chunk_range_lay(const LAY& lay, int c, int* s0, int* s1)
{
    const vpt_chunk_layout l = lay;
    vpt_chunk_range(&l, c, s0, s1);
}

/* a / d for a launch constant d = 2^sh (sh >= 0: a shift; the branch is uniform) */
__device__ __forceinline__ unsigned udiv_p(unsigned a, unsigned d, int sh) { return sh >= 0 ? a >> sh : a / d; }

/* work unit -> pixel and chunk.  Chunk-major: all units of chunk 0 (8x8 tiles in order, 64
 * consecutive units per tile), then chunk 1, ...; with the tapered layout the last units handed
 * out are the shortest. */
struct Unit {
    int x, y, c;
    bool valid;
};

__device__ __forceinline__ Unit decode_unit(const PoolParams& P0, unsigned u)
{
    VPT_PARAMS(P0);
    u += P.unit0;
    Unit r;
    const unsigned c = udiv_p(u, P.level_units, P.sh_lu), rem = u - c * P.level_units;
    r.c = (int)c;
    const unsigned tile = rem >> 6, p = rem & 63u;
    const unsigned ty = udiv_p(tile, (unsigned)P.tiles_x, P.sh_tx);
    r.x = (int)(tile - ty * (unsigned)P.tiles_x) * 8 + (int)(p & 7u);
    const int lr = (int)ty * 8 + (int)(p >> 3);  /* row within the shard */
    r.valid = r.x < P.w && lr < P.rows;
    const int k = (int)udiv_p((unsigned)lr, (unsigned)P.band_rows, P.sh_br), rr = lr - k * P.band_rows;
    const int fr = (P.band_offset + k * P.band_stride) * P.band_rows + rr;  /* file row */
    r.y = P.h - 1 - fr;                                                       /* camera row */
    return r;
}

/* camera ray through pixel (x, y) with jitter (jx, jy) -- src/rt.cpp:787-789 */
__device__ __forceinline__ dv3 pool_camera_dir(const PoolParams& P0, double jx, double jy, int x, int y)
{
    VPT_PARAMS(P0);
    const dv3 cd = mk(P.d[0], P.d[1], P.d[2]);
    const dv3 cx = mk(P.cx[0], P.cx[1], P.cx[2]), cy = mk(P.cy[0], P.cy[1], P.cy[2]);
    const double ux = (double)x + jx - 0.5, uy = (double)y + jy - 0.5;
    /* division by a power of two is exact, as is the multiplication by its reciprocal (the operands
     * are far from the subnormal range): the same bits without the division sequences */
    const double fx = P.rw != 0 ? ux * P.rw : ux / P.w, fy = P.rh != 0 ? uy * P.rh : uy / P.h;
    dv3 dir = add(add(scl(cx, (fx - .5)), scl(cy, (fy - .5))), cd);
    return nrm(dir);
}

/* ---- task state <-> registers ----
 * A task in ring A either has a path that has already survived this iteration's roulette draw
 * (in_path; the draw is taken at the end of stage S/M, where it falls in the stream anyway) or
 * needs its next sample.  `killed`: the S/M roulette ended the path, stage A adds L to the sum. */
struct Task {
    Path p;
    Event e;
    dv3 acc;
    uint64_t X;
    uint64_t key;    /* the unit's pixel stream key */
    unsigned pix;    /* x | camera row << 16 */
    unsigned c1;     /* one past the unit's last sample; 0 = the task needs a unit */
    unsigned i;      /* next sample to start */
    bool in_path, killed;
};

/* the task state in 11 LDS accesses (9 field pairs, X, the four words) instead of 23 with one array per
 * field: a batch's slots are scattered, so each access pays bank conflicts, and fewer, wider accesses
 * pay them fewer times (A/B: FF 43.30 -> 42.90 ms) */
__device__ __forceinline__ void load_task(const TaskPool& sh, int s, Task& t, bool)
{
    static_assert(F_OX == 0 && F_DX == 3 && F_BX == 6 && F_LX == 9 && F_AX == 12 && F_TD == 15 && F_KEY == 16 &&
                      F_PDF == 17, "the field pairs below");
    const double2 a = sh.f2[0][s], b = sh.f2[1][s], c = sh.f2[2][s], d = sh.f2[3][s], e = sh.f2[4][s];
    const double2 f = sh.f2[5][s], g = sh.f2[6][s], h = sh.f2[7][s], k = sh.f2[8][s];
    t.p.o = mk(a.x, a.y, b.x);
    t.p.d = mk(b.y, c.x, c.y);
    t.p.beta = mk(d.x, d.y, e.x);
    t.p.L = mk(e.y, f.x, f.y);
    t.acc = mk(g.x, g.y, h.x);
    t.e.t = t.e.dist = h.y;
    t.key = (uint64_t)__double_as_longlong(k.x);
    t.e.pdf = k.y;
    t.X = sh.X[s];
    const uint4 w = sh.w[s];
    t.pix = w.x;
    t.c1 = w.y;
    t.i = w.z & 0x7FFFFFFFu;
    t.in_path = (w.z >> 31) != 0;
    const uint32_t ev = w.w;
    t.p.depth = (int)(ev & 0xFFFFu);
    t.e.id = (int)((ev >> 16) & 0xFFu);
    t.e.src = (int)((ev >> 24) & 0x7Fu);
    t.killed = (ev >> 31) != 0;
}

__device__ __forceinline__ void store_task(TaskPool& sh, int s, const Task& t, bool)
{
    sh.f2[0][s] = double2{t.p.o.x, t.p.o.y};
    sh.f2[1][s] = double2{t.p.o.z, t.p.d.x};
    sh.f2[2][s] = double2{t.p.d.y, t.p.d.z};
    sh.f2[3][s] = double2{t.p.beta.x, t.p.beta.y};
    sh.f2[4][s] = double2{t.p.beta.z, t.p.L.x};
    sh.f2[5][s] = double2{t.p.L.y, t.p.L.z};
    sh.f2[6][s] = double2{t.acc.x, t.acc.y};
    sh.f2[7][s] = double2{t.acc.z, t.e.t};  /* stage_a leaves the distance the next stage reads in e.t */
    sh.f2[8][s] = double2{__longlong_as_double((long long)t.key), t.e.pdf};
    sh.X[s] = t.X;
    sh.w[s] = uint4{t.pix, t.c1, t.i | (t.in_path ? 0x80000000u : 0u),
                    (uint32_t)(t.p.depth & 0xFFFF) | ((uint32_t)t.e.id << 16) | ((uint32_t)t.e.src << 24) |
                        (t.killed ? 0x80000000u : 0u)};
}

/* the finished unit's chunk sum -> partials[chunk][shard row][x] */
__device__ __forceinline__ void store_partial(const PoolParams& P0, const Task& t)
{
    VPT_PARAMS(P0);
    const int x = (int)(t.pix & 0xFFFFu), y = (int)(t.pix >> 16);
    const int fr = P.h - 1 - y;
    const int k = (int)udiv_p((unsigned)fr, (unsigned)P.band_rows, P.sh_br), rr = fr - k * P.band_rows;
    const int lr = (int)udiv_p((unsigned)(k - P.band_offset), (unsigned)P.band_stride, P.sh_bs) * P.band_rows + rr;
    const int c = (int)t.c1 <= P.lay.head ? (int)udiv_p(t.c1 - 1u, (unsigned)P.lay.C, P.sh_c)  /* vpt_chunk_of_end */
                                          : vpt_chunk_of_end_lay(P.lay, (int)t.c1);
    const size_t o = (((size_t)c * (size_t)P.rows + (size_t)lr) * (size_t)P.w + (size_t)x) * 3;
    P.partials[o] = t.acc.x;
    P.partials[o + 1] = t.acc.y;
    P.partials[o + 2] = t.acc.z;
}

/* The S or M event of ring st (1-6) for one task, then the next iteration's roulette draw.  Surface
 * rings are keyed by material -- diffuse (R_S, R_S + 1), metal (R_S + 2), other -- and by light kind:
 * sphere light (R_S, R_M), point light (R_S + 1, R_M + 1). */
template <int EST, bool COUNT>
__device__ __forceinline__ void run_event(const DevScene* __restrict__ S, Sampler<COUNT>& smp, Task& t, const Medium& m, int st)
{
    if constexpr (EST == 5) {  /* iterativePathTracer: the roulette is inside the bounce */
        if (st == R_S + 2) t.killed = surface_event_pt<COUNT, 1>(S, smp, t.p, t.e);
        else if (st == R_S) t.killed = surface_event_pt<COUNT, 0>(S, smp, t.p, t.e);
        else t.killed = surface_event_pt<COUNT, -1>(S, smp, t.p, t.e);
    } else {
        SECT_BEGIN(ev);
        /* a kill-predicted ring (R_SD.., R_MD..) runs its base ring's event without the continuation */
        bool cont = true;
        if (VPT_KILL_RINGS && st >= R_SD) {
            cont = false;
            st = st < R_MD ? st - R_SD + R_S : st - R_MD + R_M;
        }
        /* metal (R_S + 2) and other materials (R_S + 3) are rare: 1.4 % of surface events at the
         * bench scene.  Diffuse-surface and medium events are compiled once for both light kinds (the
         * ring fixes the kind for the whole batch, so its branches are wave-uniform) instead of once per
         * kind: the hot code is what the shared 64 KB instruction cache has to hold (round 5: I-cache
         * misses track code size) */
#if VPT_DUP == DUP_SURF || VPT_DUP == DUP_MED
        if (VPT_DUP == DUP_SURF ? st < R_M : st >= R_M) {
            Path p2 = t.p;
            Event e2 = t.e;
            vpt_opaque(p2);
            vpt_opaque(e2);
            Sampler<COUNT> s2 = smp;
            vpt_opaque(s2.X);
            if (st >= R_M) medium_event<EST, COUNT, -1>(S, s2, p2, e2, m, cont);
            else if (st < R_S + 2) surface_event<EST, COUNT, 0, -1>(S, s2, p2, e2, m, cont, st - R_S);
            else if (st == R_S + 2) surface_event<EST, COUNT, 1, -1>(S, s2, p2, e2, m);
            else surface_event<EST, COUNT, -1, -1>(S, s2, p2, e2, m);
            vpt_sink(p2);
            vpt_sink(s2.X);
        }
#endif
        if (st < R_M) {
            if (st < R_S + 2) surface_event<EST, COUNT, 0, -1>(S, smp, t.p, t.e, m, cont, st - R_S);
            else if (st == R_S + 2) surface_event<EST, COUNT, 1, -1>(S, smp, t.p, t.e, m);
            else surface_event<EST, COUNT, -1, -1>(S, smp, t.p, t.e, m);
        } else {
            medium_event<EST, COUNT, -1>(S, smp, t.p, t.e, m, cont);
        }
        SECT_END(ev, st < R_M ? SECT_S_TOTAL : SECT_M_TOTAL);
        SECT_BEGIN(cp);
        t.killed = !cont || !continue_path(smp, t.p, m);  /* next iteration's roulette draw */
        SECT_END(cp, SECT_CONT);
    }
}

/* the kill prediction (VPT_KILL_RINGS): with the state X after decide(), does the roulette draw that
 * follows the event -- `jump` draws on -- end the path, or does the depth cap (continue_path)? */
template <int EST>
__device__ __forceinline__ constexpr bool kill_predicted_est()
{
    return VPT_KILL_RINGS && (EST == 0 || EST == 1 || EST == 2 || EST == 4);
}
__device__ __forceinline__ bool path_ends_after_event(uint64_t X, int depth, const Medium& m, uint64_t ja, uint64_t jc)
{
    if (m.max_depth > 0 && depth + 1 >= m.max_depth) return true;
    return vpt_erand48_value(vpt_erand48_skip(X, ja, jc)) < 1 - 0.6;
}

/* Stage A for the lanes with `active`: at most ONE decide() per task.  A converged preparation
 * loop first gives every task a path that has survived its roulette draw.  Lanes that need a
 * work unit take them together from the workgroup's unit ring; a finished unit writes its chunk
 * sum; a task without a path starts samples until one survives its first roulette draw.  A camera
 * sample killed by that draw has L = 0 and adds nothing to the sum (acc + 0 = acc exactly), so
 * only its three draws (jitter x, jitter y, roulette; src/rt.cpp:787 + vptShadeMethods.h:1282)
 * are taken and its camera ray is never built.  Then every ready lane runs decide() once; a path
 * that ends there goes back to ring A.  Returns the ring of the task's next stage (R_DONE:
 * retired). */
template <int EST, bool COUNT>
__device__ __forceinline__ int stage_a(TaskPool& sh, const PoolParams& P0, const DevScene* __restrict__ S,
                                       const Medium& m, Sampler<COUNT>& smp, Task& t, bool active, int lane,
                                       uint64_t below, bool dbg, ADbg& D)
{
    VPT_PARAMS(P0);
    bool done = !active, parked = false, fresh = false;
    if (active && t.killed) {  /* the S/M roulette ended the path */
        t.acc = add(t.p.L, t.acc);  /* src/rt.cpp:794 */
        t.in_path = false;
        t.killed = false;
    }
    const unsigned long long c0 = dbg_clock(dbg);
    SECT_BEGIN(pr);
    int round = 0;
    uint32_t t_r2 = 0;
    while (true) {
        if (dbg) ++D.rounds;
        ++round;
        if (round == 2) t_r2 = sect_now();
        const bool need = !done && !parked && t.c1 == 0;
        const uint64_t needm = __ballot(need);
        SECT_BEGIN(un);
        if (needm) {
            const int leader = __ffsll((unsigned long long)needm) - 1;
            const int k = __popcll(needm);
            const int r = __popcll(needm & below);
            int h = 0, got = 0, ex = 0;
            uint32_t ent = 0;
            /* take up to k units from the workgroup's ring: read the entries, then claim exactly
             * them with one CAS on uhead.  Reading before the claim keeps a refill from reusing
             * the entries' positions under a reader: a refill writes below uhead + 2 UREFILL =
             * uhead + URING, and uhead stays h until this CAS succeeds. */
            while (true) {
                if (lane == leader) {
                    ex = __hip_atomic_load(&sh.ctl[C_EXH], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    h = lds_peek(&sh.ctl[C_UHEAD]);
                    const int avail =
                        __hip_atomic_load(&sh.ctl[C_UTAIL], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) - h;
                    got = max(0, min(k, avail));
                }
                /* leader is wave-uniform: v_readlane, not an LDS permute round trip */
                h = __builtin_amdgcn_readlane(h, leader);
                got = __builtin_amdgcn_readlane(got, leader);
                ex = __builtin_amdgcn_readlane(ex, leader);
                if (need && r < got) ent = ((volatile uint32_t*)sh.uring)[(h + r) % URING];
                if (got == 0) break;
                /* the entry reads above must complete before the claim below: a refill may rewrite
                 * those positions (mod URING) once uhead has moved past them.  The release fence
                 * orders them for the compiler and the memory model (one wave's LDS accesses also
                 * execute in order, which this does not rely on). */
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                int won = 0;
                if (lane == leader) {
                    int hh = h;
                    won = __hip_atomic_compare_exchange_strong(&sh.ctl[C_UHEAD], &hh, h + got, __ATOMIC_RELAXED,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if (__builtin_amdgcn_readlane(won, leader)) break;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (need) {
                if (r >= got) {
                    /* ring empty: retire only once the queue is exhausted (the flag was read before
                     * utail, so no unit can still be on its way in); otherwise back to ring A */
                    if (ex) done = true;
                    else parked = true;
                } else {
                    const Unit uu = decode_unit(P0, ent);
                    if (uu.valid) {  /* (an invalid unit -- a tile's padding -- is dropped) */
                        t.pix = (unsigned)uu.x | ((unsigned)uu.y << 16);
                        t.key = vpt_stream_key(P.seed, (uint64_t)(P.h - 1 - uu.y) * (uint64_t)P.w + (uint64_t)uu.x);
                        int s0, s1;
                        if (uu.c < P.lay.n_head) {  /* vpt_chunk_range: a chunk of C */
                            s0 = uu.c * P.lay.C;
                            s1 = s0 + P.lay.C < P.lay.head ? s0 + P.lay.C : P.lay.head;
                        } else {
                            vpt_chunk_range_lay(P.lay, uu.c, &s0, &s1);
                        }
                        t.i = (unsigned)s0;
                        t.c1 = (unsigned)s1;
                        t.in_path = false;
                        t.acc = mk(0, 0, 0);
                    }
                }
            }
        }
        if (needm) SECT_END(un, SECT_A_UNIT);
        if (!done && !parked && !t.in_path && t.c1 != 0) {
            /* up to VPT_PREP_TRIES samples of the unit per round: a sample killed by its first
             * roulette draw costs only its stream start (no LDS, no hand-out), so trying the next
             * one here instead of in the next round keeps the lane from parking (a parked lane
             * idles through this batch's decide) */
            for (int k = 0; k < VPT_PREP_TRIES && !t.in_path && t.i != t.c1; ++k) {
                const uint64_t X0 = vpt_stream_start_key(t.key, (uint64_t)t.i);  /* key: src/rt.cpp:773 idx */
                ++t.i;
                if (dbg) ++D.samples;
                /* the first roulette draw (vptShadeMethods.h:1282, continue_path at depth 0) is the
                 * stream's third, after the jitter pair: decide it from the state three steps on;
                 * the jitter and the camera ray are built after the loop, for survivors only */
                if (EST == 5) {  /* iterativePathTracer draws no roulette before its first intersection */
                    t.X = X0;
                    t.in_path = true;
                    fresh = true;
                } else {
                    if (COUNT) smp.cnt.iterations++;
                    if (!(vpt_erand48_value(vpt_erand48_skip3(X0)) < 1 - 0.6)) {
                        t.X = X0;
                        t.in_path = true;
                        fresh = true;
                    }
                }
            }
            if (VPT_UNLIKELY(!t.in_path && t.i == t.c1)) {  /* the unit is done: its chunk sum out */
                store_partial(P0, t);
                t.c1 = 0;
            }
        }
        const uint64_t waiting = __ballot(!done && !parked && !t.in_path);
        if (waiting == 0) break;
        /* a lane still without a path after VPT_PREP_ROUNDS rounds is parked (back to ring A, it
         * continues from its next sample in a later batch) instead of holding the whole wave in
         * this loop: the wave's round count is the maximum over its lanes of a geometric count.
         * A further round costs the wave the same whatever its number of lanes, so with fewer than
         * VPT_PREP_MORE_MIN lanes waiting they are parked at once */
        if ((VPT_PREP_ROUNDS > 0 && round >= VPT_PREP_ROUNDS) || __popcll(waiting) < VPT_PREP_MORE_MIN) {
            if (!done && !t.in_path) parked = true;
            break;
        }
    }
    if (round >= 2) sect_add(SECT_A_R2, t_r2);
    SECT_END(pr, SECT_A_PREP);
    SECT_BEGIN(cam);
    if (fresh) {  /* camera ray of the surviving sample: src/rt.cpp:787-789 */
        SECT_BEGIN(ci);
        smp.X = t.X;
        const double jx = smp.next();  /* x draw first */
        const double jy = smp.next();
        if (EST != 5) (void)smp.next();  /* the roulette draw, decided above */
        t.p.o = mk(P.o[0], P.o[1], P.o[2]);
#if VPT_DUP == DUP_CAMERA
        {
            double jx2 = jx, jy2 = jy;
            int px = (int)(t.pix & 0xFFFFu), py = (int)(t.pix >> 16);
            vpt_opaque(jx2);
            vpt_opaque(jy2);
            vpt_opaque(px);
            vpt_opaque(py);
            vpt_sink(pool_camera_dir(P0, jx2, jy2, px, py));
        }
#endif
        t.p.d = pool_camera_dir(P0, jx, jy, (int)(t.pix & 0xFFFFu), (int)(t.pix >> 16));
        t.p.beta = mk(1, 1, 1);
        t.p.L = mk(0, 0, 0);
        t.p.depth = 0;
        if (EST == 5) t.e.pdf = 1;  /* iterativePathTracer's `factor` rides in the event's pdf slot */
        t.X = smp.X;
        SECT_END(ci, SECT_A_CAMERA_IN);
    }
    SECT_END(cam, SECT_A_CAMERA);
    const unsigned long long c1 = dbg_clock(dbg);
    int result = parked ? R_A : R_DONE;
    SECT_BEGIN(dc);
    if (!done && !parked) {
        SECT_BEGIN(dci);
        smp.X = t.X;
#if VPT_DUP == DUP_DECIDE
        {
            Path p2 = t.p;
            Event e2 = t.e;
            vpt_opaque(p2);
            vpt_opaque(e2);
            Sampler<COUNT> s2 = smp;
            vpt_opaque(s2.X);
            vpt_sink(decide<EST>(S, s2, p2, e2, m));
            vpt_sink(p2);
            vpt_sink(e2);
            vpt_sink(s2.X);
        }
#endif
        const int ev = decide<EST>(S, smp, t.p, t.e, m);
        t.X = smp.X;
        if (ev == EV_END) {
            t.acc = add(t.p.L, t.acc);
            t.in_path = false;
            result = R_A;
        } else if (ev == EV_SURF) {  /* (the implicit estimator, EST 3, picks no light) */
            const int sk = sph_flag(S->m_skey1, t.e.id) | (sph_flag(S->m_skey2, t.e.id) << 1);
            result = R_S + (sk == 0 ? (EST == 3 || EST == 5 ? 0 : sph_flag(S->m_point, t.e.src)) : sk);
            /* a diffuse surface event: 2 n_mis + 4 draws, then the roulette (S->kp_sa, kp_sc) */
            if (kill_predicted_est<EST>() && !COUNT && sk == 0 &&
                path_ends_after_event(t.X, t.p.depth, m, S->kp_sa, S->kp_sc))
                result += R_SD - R_S;
        } else {
            result = R_M + (EST == 3 ? 0 : sph_flag(S->m_point, t.e.src));
            /* one slot (F_TD): stage M reads the sampled distance -- or, for the deferred
             * equi-angular estimators, tMax (with decide()'s psurf in F_PDF) */
            if (!(EST == 1 || EST == 4)) t.e.t = t.e.dist;
            /* a medium event: the light cone's two draws and the phase sample's two, then the roulette */
            if constexpr (kill_predicted_est<EST>() && !COUNT) {
                uint64_t ja, jc;
                vpt_erand48_jump(5, &ja, &jc);
                if (path_ends_after_event(t.X, t.p.depth, m, ja, jc)) result += R_MD - R_M;
            }
        }
        SECT_END(dci, SECT_A_DECIDE_IN);
    }
    SECT_END(dc, SECT_A_DECIDE);
    if (dbg) {
        D.c_prep += c1 - c0;
        D.c_decide += dbg_clock(dbg) - c1;
    }
    return result;
}

template <int EST, bool COUNT>
__global__ __launch_bounds__(VPT_POOL_THREADS, VPT_POOL_WGS) void pool_kernel(PoolParams P0, Medium m0, const DevScene* __restrict__ S,
                                                   unsigned long long* counters, unsigned long long* stats)
{
    __shared__ TaskPool sh;
#if VPT_P_KARG && defined(__HIP_DEVICE_COMPILE__)
    /* pool_params_at_use() reads P0 at offset 0 of the argument segment: P0 must stay the first argument.
     * If it moves, the launch renders nothing and raises the guard flag: reduce_kernel then writes NaN and
     * the synchronous entry points (vpt_render) return VPT_E_INTERNAL instead of a garbage image. */
    if (pool_params_at_use().nunits != P0.nunits + P0.guard_bias || pool_params_at_use().unit0 != P0.unit0) {
        if (threadIdx.x == 0) atomicOr(P0.guard, 1u);
        return;
    }
#endif
    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int j = tid; j < POOL; j += VPT_POOL_THREADS) {
        sh.w[j] = uint4{0u, 0u, 0u, 0u};
        sh.ring[R_A][j] = (uint16_t)j;  /* = ring_entry(j, j): lap 0 */
        for (int r = 1; r < NR; ++r) sh.ring[r][j] = (uint16_t)(LAP_MASK << SLOT_BITS);  /* no lap-0 entry yet */
    }
    if (tid < NCTL) sh.ctl[tid] = tid == C_TAIL + R_A ? POOL : 0;  /* every slot starts in ring A */
    sect_init();
    __syncthreads();

    Sampler<COUNT> smp;
    smp.X = 0;
    smp.g = m0.g;
    smp.cnt.tests = 0;
    smp.cnt.iterations = 0;
    smp.cnt.draw_mismatch = 0;
    int n = 0, slot = 0, next = R_A;
    unsigned long long st_idle = 0, st_retry = 0, st_sched = 0, st_b[NR] = {}, st_l[NR] = {}, st_c[3] = {};
    ADbg D = {};
    const bool dbg = VPT_POOL_DEBUG && stats != nullptr;  /* compiled out of production builds */
    const bool dbga = VPT_POOL_DEBUG == 1 && dbg;          /* stage-A internals (VPT_POOL_DEBUG=2: top level only) */
    unsigned long long tclk = dbg_clock(dbg);
    bool seen_exh = false;
    if (dbg && tid == 0) dbg_tl(stats, 0, false);
    while (true) {
        SECT_BEGIN(sc);
        /* ---- scheduling without a lock (ring_entry): reserve, publish, claim ---- */
        if (VPT_SCHED_PRIO) __builtin_amdgcn_s_setprio(VPT_SCHED_PRIO);
        if (n > 0) {  /* return the finished tasks: each lane reserves its ring position with one LDS atomic */
            const bool ret = lane < n && next < NR;
            int pos = 0;
            if (ret) pos = __hip_atomic_fetch_add(&sh.ctl[C_TAIL + next], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  /* task states before their entries */
            if (ret) ((volatile uint16_t*)sh.ring[next])[pos % POOL] = ring_entry(slot, pos);
            const uint64_t md = __ballot(lane < n && next == R_DONE);
            if (md && lane == 0)
                __hip_atomic_fetch_add(&sh.ctl[C_DONE], __popcll(md), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        /* keep the unit ring stocked (the queue atomic's latency is paid once per 128 units); one
         * wave at a time, claimed by a flag.  The counters read here serve the first claim attempt
         * below as well (re-read after a refill and on every retry). */
        int vc = lane < NCTL ? lds_peek(&sh.ctl[lane]) : 0;
        int hc = lane < NR ? lds_peek(&sh.ctl[C_HEAD + lane]) : 0;
        {
            const int v = vc;
            if (dbg && !seen_exh && __builtin_amdgcn_readlane(v, C_EXH)) {
                seen_exh = true;
                if (lane == 0) dbg_tl(stats, 1, false);
            }
            if (VPT_UNLIKELY(!__builtin_amdgcn_readlane(v, C_EXH) && !__builtin_amdgcn_readlane(v, C_RFL) &&
                __builtin_amdgcn_readlane(v, C_UTAIL) - __builtin_amdgcn_readlane(v, C_UHEAD) < UREFILL)) {
                int own = 0;
                if (lane == 0) {
                    int z = 0;
                    own = __hip_atomic_compare_exchange_strong(&sh.ctl[C_RFL], &z, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if (__builtin_amdgcn_readfirstlane(own)) {
                    const int t0 = __builtin_amdgcn_readfirstlane(lds_peek(&sh.ctl[C_UTAIL]));
                    if (t0 - __builtin_amdgcn_readfirstlane(lds_peek(&sh.ctl[C_UHEAD])) < UREFILL) {
                        VPT_PARAMS(P0);
                        unsigned ubase = 0;
                        if (lane == 0) ubase = atomicAdd(P.queue, (unsigned)UREFILL);
                        ubase = (unsigned)__builtin_amdgcn_readfirstlane((int)ubase);
                        const unsigned left = ubase < P.nunits ? P.nunits - ubase : 0u;
                        const int nv = (int)(left < (unsigned)UREFILL ? left : (unsigned)UREFILL);
                        for (int j = lane; j < nv; j += 64) sh.uring[(t0 + j) % URING] = ubase + (unsigned)j;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        if (lane == 0) {
                            __hip_atomic_store(&sh.ctl[C_UTAIL], t0 + nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (left <= (unsigned)UREFILL)
                                __hip_atomic_store(&sh.ctl[C_EXH], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                    }
                    if (lane == 0) __hip_atomic_store(&sh.ctl[C_RFL], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                vc = lane < NCTL ? lds_peek(&sh.ctl[lane]) : 0;
                hc = lane < NR ? lds_peek(&sh.ctl[C_HEAD + lane]) : 0;
            }
        }
        /* take a batch of the fullest ring: read its published entries, then claim them by one CAS
         * on the ring's head (a claim never covers an entry that is not yet written) */
        int st = 0, take = 0;
        bool fin = false;
        for (bool first = true;; first = false) {
            const int v = first ? vc : lane < NCTL ? lds_peek(&sh.ctl[lane]) : 0;
            int best = 0;
            st = 0;
            /* the fullest ring, lowest index on ties: lane r < NR holds ring r's count as the key
             * count << 4 | (15 - r); a max over the first 16 lanes (row shifts) leaves it in lane 15 */
            static_assert(NR <= 16, "the ring argmax runs in one DPP row");
            {
                const int hv = first ? hc : lane < NR ? lds_peek(&sh.ctl[C_HEAD + lane]) : 0;
                const int c = v - hv;
                int key = lane < NR && c > 0 ? (c << 4) | (15 - lane) : -1;
                key = max(key, __builtin_amdgcn_update_dpp(-1, key, 0x111, 0xF, 0xF, false));  /* row_shr:1 */
                key = max(key, __builtin_amdgcn_update_dpp(-1, key, 0x112, 0xF, 0xF, false));  /* row_shr:2 */
                key = max(key, __builtin_amdgcn_update_dpp(-1, key, 0x114, 0xF, 0xF, false));  /* row_shr:4 */
                key = max(key, __builtin_amdgcn_update_dpp(-1, key, 0x118, 0xF, 0xF, false));  /* row_shr:8 */
                key = __builtin_amdgcn_readlane(key, 15);
                if (key >= 0) {
                    best = key >> 4;
                    st = 15 - (key & 15);
                }
            }
            if (VPT_UNLIKELY(best <= 0)) {
                if (__builtin_amdgcn_readlane(v, C_DONE) == POOL) {
                    fin = true;
                    break;
                }
                ++st_idle;
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            const int h = __builtin_amdgcn_readlane(v, C_HEAD + st);
            const int want = min(64, best);
            int e = 0;
            bool ok = false;
            if (lane < want) {
                const int p = h + lane;
                e = ((volatile uint16_t*)sh.ring[st])[p % POOL];
                ok = (e >> SLOT_BITS) == ((p / POOL) & LAP_MASK);
            }
            const uint64_t okm = __ballot(ok);
            const int got = okm == ~0ull ? 64 : __builtin_ctzll(~okm);  /* the published prefix */
            if (VPT_UNLIKELY(got == 0)) {
                ++st_retry;
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            int won = 0;
            if (lane == 0) {
                int hh = h;
                won = __hip_atomic_compare_exchange_strong(&sh.ctl[C_HEAD + st], &hh, h + got, __ATOMIC_RELAXED,
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (VPT_UNLIKELY(!__builtin_amdgcn_readfirstlane(won))) {
                ++st_retry;
                continue;
            }
            take = got;
            slot = e & SLOT_MASK;
            break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  /* the claimed tasks' states */
        if (VPT_SCHED_PRIO) __builtin_amdgcn_s_setprio(0);
        SECT_END(sc, SECT_SCHED);
        if (fin) break;
        n = take;
        if (dbg) {  /* debug only; compile-time indices keep the counters in registers */
#pragma unroll
            for (int r = 0; r < NR; ++r)
                if (st == r) {
                    st_b[r] += 1;
                    st_l[r] += (unsigned long long)take;
                }
            const unsigned long long now = dbg_clock(dbg);
            st_sched += now - tclk;
            tclk = now;
        }

        /* ---- run one stage on the batch ---- */
        const Medium& m = m0;
        const bool active = lane < n;
        Task t;
        const int stage = st == R_A ? 0 : st < R_M ? 1 : 2;
        /* one copy of stage A in the code: a batch of ring A runs it alone, a batch of an S/M ring
         * runs its event first and then stage A on the same lanes */
        SECT_BEGIN(ld);
#if VPT_DUP == DUP_LDST
        if (active) {  /* a second load of the task (sunk) and, below, a second store of the same values */
            int slot2 = slot;
            vpt_opaque(slot2);
            Task t2;
            load_task(sh, slot2, t2, true);
            vpt_sink(t2.p);
            vpt_sink(t2.e);
            vpt_sink(t2.acc);
            vpt_sink(t2.X);
            vpt_sink(t2.key);
            vpt_sink((int)(t2.pix ^ t2.c1 ^ t2.i ^ (t2.in_path ? 1 : 0) ^ (t2.killed ? 2 : 0)));
        }
#endif
        if (active) load_task(sh, slot, t, true);
        else {
            t.c1 = 0;
            t.in_path = false;
            t.killed = false;
        }
        SECT_END(ld, SECT_LOAD);
        if (stage != 0 && active) {
            smp.X = t.X;
            run_event<EST, COUNT>(S, smp, t, m, st);
            t.X = smp.X;
        }
        next = stage_a<EST>(sh, P0, S, m, smp, t, active, lane, below, dbga, D);
        SECT_BEGIN(stt);
        if (active) store_task(sh, slot, t, true);
#if VPT_DUP == DUP_LDST
        if (active) {
            int slot2 = slot;
            vpt_opaque(slot2);
            store_task(sh, slot2, t, true);
        }
#endif
        SECT_END(stt, SECT_STORE);
        if (dbg) {
            const unsigned long long now = dbg_clock(dbg);
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (stage == k) st_c[k] += now - tclk;
            tclk = now;
        }
    }
    sect_flush();
    if (COUNT) {
        atomicAdd(&counters[0], (unsigned long long)smp.cnt.tests);
        atomicAdd(&counters[1], (unsigned long long)smp.cnt.iterations);
    }
    if (dbg) {
        if (lane == 0) dbg_tl(stats, 2, true);
        atomicAdd(&stats[21], D.samples);
        if (lane == 0) {
            atomicAdd(&stats[14], st_idle);
            atomicAdd(&stats[15], st_retry);
            atomicAdd(&stats[19], st_sched);
#pragma unroll
            for (int r = 0; r < NR; ++r) {  /* (kill-predicted rings are counted with their base ring) */
                const int rb = r < R_SD ? r : r < R_MD ? r - R_SD + R_S : r - R_MD + R_M;
                atomicAdd(&stats[rb], st_b[r]);
                atomicAdd(&stats[7 + rb], st_l[r]);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) atomicAdd(&stats[16 + k], st_c[k]);
            atomicAdd(&stats[20], D.rounds);
            atomicAdd(&stats[22], D.c_prep);
            atomicAdd(&stats[23], D.c_decide);
        }
    }
}

/* chunk sums -> pixel average, in chunk order (matches orc_render_chunked) */
template <int FB>
__global__ __launch_bounds__(256) void reduce_kernel(PoolParams P, void* out)
{
    const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t npix = (size_t)P.rows * (size_t)P.w;
    if (p >= npix) return;
    const double* q = P.partials + p * 3;
    const size_t plane = npix * 3;  /* one chunk level (chunk-major layout, store_partial) */
    dv3 tot = mk(0, 0, 0);
    for (int c = 0; c < P.nch; ++c) tot = add(mk(q[c * plane], q[c * plane + 1], q[c * plane + 2]), tot);
    tot = scl(tot, (1 / (double)P.spp));  /* src/rt.cpp:800 */
    if (VPT_UNLIKELY(*(volatile unsigned*)P.guard != 0)) tot = mk(__builtin_nan(""), __builtin_nan(""), __builtin_nan(""));
    if (FB == VPT_FB_F32) {
        float* o = (float*)out;
        o[3 * p] = (float)tot.x;
        o[3 * p + 1] = (float)tot.y;
        o[3 * p + 2] = (float)tot.z;
    } else {
        double* o = (double*)out;
        o[3 * p] = tot.x;
        o[3 * p + 1] = tot.y;
        o[3 * p + 2] = tot.z;
    }
}

}  // namespace vpt

#endif
