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

namespace vpt {
template __global__ void pool_kernel<1, false>(PoolParams P0, Medium m0, const DevScene* __restrict__ S,
                                               unsigned long long* counters, unsigned long long* stats);
}  // namespace vpt
