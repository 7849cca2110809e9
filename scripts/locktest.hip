// Debug micro-test: workgroup LDS spin lock (lane 0 CAS) as used by vpt_pool.h.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void lock_kernel(int iters, unsigned long long* out, int variant)
{
    __shared__ int lock;
    __shared__ int counter;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) { lock = 0; counter = 0; }
    __syncthreads();
    unsigned long long retries = 0;
    for (int k = 0; k < iters; ++k) {
        if (lane == 0) {
            int expected = 0;
            while (!__hip_atomic_compare_exchange_strong(&lock, &expected, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP)) {
                expected = 0;
                ++retries;
                if (variant) __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        int c = counter;
        if (lane == 0) counter = c + 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&lock, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&out[0], (unsigned long long)counter);
    if (lane == 0) atomicAdd(&out[1], retries);
}

int main()
{
    unsigned long long* d;
    hipMalloc(&d, 16);
    for (int variant = 0; variant < 2; ++variant) {
        hipMemset(d, 0, 16);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        lock_kernel<<<1, 256>>>(1000, d, variant);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        unsigned long long h[2];
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("variant %d: counter %llu (expect 4000) retries %llu time %.3f ms\n", variant, h[0], h[1], ms);
    }
    return 0;
}
