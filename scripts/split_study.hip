/*
 * split_study.hip -- CPU-only compile study: would the pool kernel's stages, compiled
 * as separate kernels that exchange task state through global memory (a wavefront / "split" design),
 * fit a register budget that allows more than the pool kernel's 2 waves per SIMD?
 *
 * Each kernel below runs exactly one of pool_kernel's stages (vpt_pool.h run_event / stage_a) on tasks
 * read from and written back to SoA arrays in global memory, with the product's flags.  The register
 * budget per occupancy target is set with amdgpu_waves_per_eu(W, W): W waves per SIMD allow
 * 512 / W registers (3: 168, 4: 128 after the 8-register granule).  scripts/split_study.sh compiles
 * every (stage, W) pair and reads VGPR / SGPR / spill counts from the code object's metadata.
 *
 * Stages (estimator EST, 1 = MISVPTTracerRecursive, include/vptShadeMethods.h:1345-1481):
 *   decide   decide(): intersection, light pick, distance sample + the kill prediction
 *   surf_d   diffuse-surface event (pLight + the fused two-light MISv2 + bdsf) + the next roulette draw
 *   med      medium event (equi-angular setup, single scattering, phase sample) + the roulette draw
 *   surf_r   rare-material surface event (metal: microfacet BSDF) + the roulette draw
 */
#include <hip/hip_runtime.h>

#include "vpt_device.h"
#include "vpt_pool.h"

using namespace vpt;

#ifndef SPLIT_W
#define SPLIT_W 2
#endif
#ifndef SPLIT_EST
#define SPLIT_EST 1
#endif

struct TaskSoA {
    double* f[NF];   /* the 18 doubles of a task (vpt_pool.h F_*) */
    uint64_t* X;     /* erand48 state */
    uint32_t* w;     /* depth | id << 16 | src << 24 | killed << 31 */
    int* ring;       /* next ring */
};

__device__ __forceinline__ void ld(const TaskSoA& T, int i, Path& p, Event& e, uint64_t& X)
{
    p.o = mk(T.f[F_OX][i], T.f[F_OY][i], T.f[F_OZ][i]);
    p.d = mk(T.f[F_DX][i], T.f[F_DY][i], T.f[F_DZ][i]);
    p.beta = mk(T.f[F_BX][i], T.f[F_BY][i], T.f[F_BZ][i]);
    p.L = mk(T.f[F_LX][i], T.f[F_LY][i], T.f[F_LZ][i]);
    e.t = e.dist = T.f[F_TD][i];
    e.pdf = T.f[F_PDF][i];
    X = T.X[i];
    const uint32_t ev = T.w[i];
    p.depth = (int)(ev & 0xFFFFu);
    e.id = (int)((ev >> 16) & 0xFFu);
    e.src = (int)((ev >> 24) & 0x7Fu);
}

__device__ __forceinline__ void st(const TaskSoA& T, int i, const Path& p, const Event& e, uint64_t X, bool killed, int ring)
{
    T.f[F_OX][i] = p.o.x, T.f[F_OY][i] = p.o.y, T.f[F_OZ][i] = p.o.z;
    T.f[F_DX][i] = p.d.x, T.f[F_DY][i] = p.d.y, T.f[F_DZ][i] = p.d.z;
    T.f[F_BX][i] = p.beta.x, T.f[F_BY][i] = p.beta.y, T.f[F_BZ][i] = p.beta.z;
    T.f[F_LX][i] = p.L.x, T.f[F_LY][i] = p.L.y, T.f[F_LZ][i] = p.L.z;
    T.f[F_TD][i] = e.t;
    T.f[F_PDF][i] = e.pdf;
    T.X[i] = X;
    T.w[i] = (uint32_t)(p.depth & 0xFFFF) | ((uint32_t)e.id << 16) | ((uint32_t)e.src << 24) | (killed ? 0x80000000u : 0u);
    T.ring[i] = ring;
}

#define SPLIT_ATTR __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SPLIT_W, SPLIT_W)))

SPLIT_ATTR void k_decide(TaskSoA T, Medium m, const DevScene* __restrict__ S, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    Path p;
    Event e;
    Sampler<false> smp;
    smp.g = m.g;
    ld(T, i, p, e, smp.X);
    const int ev = decide<SPLIT_EST>(S, smp, p, e, m);
    int ring = R_A;
    if (ev == EV_SURF) {
        const int sk = sph_flag(S->m_skey1, e.id) | (sph_flag(S->m_skey2, e.id) << 1);
        ring = R_S + (sk == 0 ? sph_flag(S->m_point, e.src) : sk);
        if (sk == 0 && path_ends_after_event(smp.X, p.depth, m, S->kp_sa, S->kp_sc)) ring += R_SD - R_S;
    } else if (ev == EV_MED) {
        ring = R_M + sph_flag(S->m_point, e.src);
        uint64_t ja, jc;
        vpt_erand48_jump(5, &ja, &jc);
        if (path_ends_after_event(smp.X, p.depth, m, ja, jc)) ring += R_MD - R_M;
    }
    st(T, i, p, e, smp.X, false, ring);
}

SPLIT_ATTR void k_surf_d(TaskSoA T, Medium m, const DevScene* __restrict__ S, int n, int lk, int cont)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    Path p;
    Event e;
    Sampler<false> smp;
    smp.g = m.g;
    ld(T, i, p, e, smp.X);
    surface_event<SPLIT_EST, false, 0, -1>(S, smp, p, e, m, cont != 0, lk);
    const bool killed = !cont || !continue_path(smp, p, m);
    st(T, i, p, e, smp.X, killed, R_A);
}

SPLIT_ATTR void k_med(TaskSoA T, Medium m, const DevScene* __restrict__ S, int n, int cont)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    Path p;
    Event e;
    Sampler<false> smp;
    smp.g = m.g;
    ld(T, i, p, e, smp.X);
    medium_event<SPLIT_EST, false, -1>(S, smp, p, e, m, cont != 0);
    const bool killed = !cont || !continue_path(smp, p, m);
    st(T, i, p, e, smp.X, killed, R_A);
}

SPLIT_ATTR void k_surf_r(TaskSoA T, Medium m, const DevScene* __restrict__ S, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    Path p;
    Event e;
    Sampler<false> smp;
    smp.g = m.g;
    ld(T, i, p, e, smp.X);
    surface_event<SPLIT_EST, false, 1, -1>(S, smp, p, e, m);
    const bool killed = !continue_path(smp, p, m);
    st(T, i, p, e, smp.X, killed, R_A);
}
