// Micro-benchmark of the device libm: calls per second of each function on path-like argument
// distributions, per implementation (gl_*: glibc-exact; vm_*: portable).  64 lanes of a wave draw
// independent arguments, so branchy implementations pay their divergence as they do in the kernel.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I minimal_volumetric_path_tracer_amd/csrc \
//         scripts/ubench_libm.hip -o scripts/ubench_libm.bin && scripts/ubench_libm.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "vpt_math.h"

#ifndef UB_EXTRA
#define UB_EXTRA
#endif

__device__ __forceinline__ double u01(unsigned long long& s)
{
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(s >> 11) * 0x1p-53;
}

enum { F_EXP, F_LOG, F_SIN, F_COS, F_SINCOS, F_TAN, F_ATAN2, F_ACOS, F_SCACOS, F_ATAN, F_DIR, F_DIRCONE, NF };
static const char* NAMES[NF] = {"exp", "log", "sin", "cos", "sincos", "tan", "atan2", "acos", "sincos_acos", "atan", "dir_trig", "dir_cone"};

template <int F, int IMPL>
__global__ __launch_bounds__(256) void bench(double* out, int iters)
{
    unsigned long long s = 0x9E3779B97F4A7C15ull * (blockIdx.x * blockDim.x + threadIdx.x + 1);
    double acc = 0;
    for (int i = 0; i < iters; ++i) {
        const double u = u01(s), v = u01(s);
        double r = 0;
        if (F == F_EXP) r = IMPL ? lm_exp(-5.0 * u) : vm_exp(-5.0 * u);
        if (F == F_LOG) r = IMPL ? lm_log(1.0 - u) : vm_log(1.0 - u);
        if (F == F_SIN) r = IMPL ? lm_sin(6.283185307179586 * u) : vm_sin(6.283185307179586 * u);
        if (F == F_COS) r = IMPL ? lm_cos(6.283185307179586 * u) : vm_cos(6.283185307179586 * u);
        if (F == F_SINCOS) {
            double a, b;
            if (IMPL) lm_sincos(6.283185307179586 * u, &a, &b);
            else vm_sincos(6.283185307179586 * u, &a, &b);
            r = a + b;
        }
        if (F == F_TAN) r = IMPL ? lm_tan(3.0 * u - 1.5) : vm_tan(3.0 * u - 1.5);
        if (F == F_ATAN2) r = IMPL ? lm_atan2(200.0 * u - 100.0, 0.1 + 100.0 * v) : vm_atan2(200.0 * u - 100.0, 0.1 + 100.0 * v);
        if (F == F_ACOS) r = IMPL ? lm_acos(2.0 * u - 1.0) : vm_acos(2.0 * u - 1.0);
        if (F == F_SCACOS) {
            double a, b;
            if (IMPL) lm_sincos_acos(2.0 * u - 1.0, &a, &b);
            else vm_sincos_acos(2.0 * u - 1.0, &a, &b);
            r = a + b;
        }
        if (F == F_DIR || F == F_DIRCONE) {  /* lm_dir_trig: sin/cos of acos(c) and of phi */
            const double c = F == F_DIR ? 2.0 * u - 1.0 : (1.0 - u) + u * 0.9998;
            double a, b, e, f;
            if (IMPL) lm_dir_trig(c, 6.283185307179586 * v, &a, &b, &e, &f);
            else {
                vm_sincos_acos(c, &a, &b);
                vm_sincos(6.283185307179586 * v, &e, &f);
            }
            r = a * e + b * f;
        }
        if (F == F_ATAN) r = IMPL ? lm_atan(20.0 * u - 10.0) : vm_atan(20.0 * u - 10.0);
        acc += r;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int F, int IMPL>
static double run(double* d)
{
    const int blocks = 256 * 8, threads = 256, iters = 256;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    bench<F, IMPL><<<blocks, threads>>>(d, 4);
    (void)hipEventRecord(e0);
    bench<F, IMPL><<<blocks, threads>>>(d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return (double)blocks * threads * iters / (ms * 1e-3) / 1e9;  // Gcalls/s
}

template <int F>
static void row(double* d)
{
    const double vm = run<F, 0>(d), lm = run<F, 1>(d);
    printf("%-12s vm %8.2f Gcalls/s   lm %8.2f Gcalls/s   lm/vm %.2f\n", NAMES[F], vm, lm, lm / vm);
}

int main(int argc, char** argv)
{
    double* d;
    (void)hipMalloc(&d, sizeof(double) * 256 * 8 * 256);
    if (argc > 1) {  /* one function only (for rocprofv3 --pmc): dir */
        row<F_DIR>(d);
        (void)hipFree(d);
        return 0;
    }
    row<F_EXP>(d);
    row<F_LOG>(d);
    row<F_SIN>(d);
    row<F_COS>(d);
    row<F_SINCOS>(d);
    row<F_TAN>(d);
    row<F_ATAN2>(d);
    row<F_ACOS>(d);
    row<F_SCACOS>(d);
    row<F_ATAN>(d);
    row<F_DIR>(d);
    row<F_DIRCONE>(d);
    (void)hipFree(d);
    return 0;
}
