// Micro-benchmark: FP64 VALU issue rate and dependent latency on gfx950, by waves per SIMD and
// independent chains per wave.  hipcc --offload-arch=gfx950 -O3 scripts/ubench_f64.hip -o /tmp/ub
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int K, int OP>
__global__ __launch_bounds__(1024) void chains(double* out, double a, double b, int iters)
{
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x * 1e-3 + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (OP == 0) x[k] = __builtin_fma(x[k], a, b);
                else if (OP == 1) x[k] = x[k] * a;
                else if (OP == 2) x[k] = __builtin_amdgcn_rsq(x[k]);
                else if (OP == 3) x[k] = __builtin_fmaf((float)x[k], (float)a, (float)b);
                else if (OP == 4) {  /* fma with both constants materialised in SGPRs at the use (vm_k) */
                    double ca = 1.0000001 + r * 1e-12, cb = 1e-9 + k * 1e-15;
                    __asm__ volatile("" : "+s"(ca));
                    __asm__ volatile("" : "+s"(cb));
                    x[k] = __builtin_fma(x[k], ca, cb);
                } else if (OP == 5) {  /* one constant materialised per fma */
                    double cb = 1e-9 + r * 1e-15 + k * 1e-17;
                    __asm__ volatile("" : "+s"(cb));
                    x[k] = __builtin_fma(x[k], a, cb);
                }
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int K, int OP>
void run(const char* name, double* d, int wps)
{
    int cus = 256;
    dim3 grid(cus), block(64 * 4 * wps);
    int iters = 8000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    chains<K, OP><<<grid, block>>>(d, 1.0000001, 1e-9, 10);
    hipEventRecord(e0);
    chains<K, OP><<<grid, block>>>(d, 1.0000001, 1e-9, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double insts_per_simd = (double)iters * 16 * K * wps;  // wave-instructions per SIMD
    double cyc = ms * 1e-3 * 2.4e9;
    printf("%-6s waves/SIMD %d chains %d : %.2f cycles per wave-instruction per SIMD (%.3f ms)\n", name, wps, K,
           cyc / insts_per_simd, ms);
}

int main()
{
    double* d;
    hipMalloc(&d, 256 * 1024 * sizeof(double));
    /* dependent-chain latency (1 chain, 1 wave/SIMD) vs issue rate (many chains, 2 waves/SIMD) */
    for (int w = 1; w <= 2; w *= 2) {
        run<1, 0>("fma64", d, w);
        run<2, 0>("fma64", d, w);
        run<4, 0>("fma64", d, w);
        run<8, 0>("fma64", d, w);
        run<1, 1>("mul64", d, w);
        run<4, 1>("mul64", d, w);
        run<1, 2>("rsq64", d, w);
        run<4, 2>("rsq64", d, w);
        run<1, 3>("fma32", d, w);
        run<4, 3>("fma32", d, w);
    }
    run<1, 0>("fma64", d, 4);
    run<4, 0>("fma64", d, 4);
    return 0;
}
