/*
 * vpt_pool_mis.hip -- the pool kernel of the north-star estimator (MISVPTTracerRecursive, EST = 1,
 * include/vptShadeMethods.h:1345-1481) in a translation unit of its own, so that it can take compile
 * flags of its own (csrc/Makefile MISFLAGS).  The kernel's code is vpt_pool.h's pool_kernel template,
 * unchanged; vpt_kernels.hip declares this instantiation extern and launches it like the others.
 * Round 6: without MachineLICM (-mllvm -disable-machine-licm) the EST = 1 kernel keeps no loop-invariant
 * value in a register across the whole pool loop -- 0 spills instead of 53 -- and is 0.8 % faster, while
 * the free-flight kernel (EST = 0) is 0.2 % slower that way (A/B ab_r06s), hence the separate unit.
 */
#include <hip/hip_runtime.h>

#include "vpt_device.h"
#include "vpt_pool.h"

#ifndef VPT_MIS_TU
#define VPT_MIS_TU 1
#endif
#if VPT_MIS_TU
namespace vpt {
template __global__ void pool_kernel<1, false>(PoolParams P0, Medium m0, const DevScene* __restrict__ S,
                                               unsigned long long* counters, unsigned long long* stats);
}  // namespace vpt

#if VPT_SECTIONS
/* debug (section-timer builds): this unit's timers, added into out and cleared (vpt_debug_sections) */
extern "C" int vpt_mis_sections_add(unsigned long long* out)
{
    unsigned long long v[3 * vpt::SECT_N];
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(vpt::g_vpt_sect), sizeof(v)) != hipSuccess) return 1;
    for (int k = 0; k < 3 * vpt::SECT_N; ++k) out[k] += v[k];
    static const unsigned long long zero[3 * vpt::SECT_N] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(vpt::g_vpt_sect), zero, sizeof(zero)) != hipSuccess;
}
#endif
#endif
