// Does work on hipStreamPerThread wait for earlier work on the null stream
// (torch's default stream)?  A ~200 ms spin kernel on the null stream sets a
// flag when it ends; a kernel on the per-thread stream, launched right
// after, records whether it saw the flag.  Also the converse, and a
// hipStreamNonBlocking stream for comparison.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void spin_then_set(int *flag, unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
    __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void observe(const int *flag, int *seen) {
    *seen = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static int run(hipStream_t first, hipStream_t second) {
    int *flag = nullptr, *seen = nullptr;
    (void)hipMalloc(&flag, 4);
    (void)hipMalloc(&seen, 4);
    (void)hipMemset(flag, 0, 4);
    (void)hipMemset(seen, 0, 4);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(spin_then_set, dim3(1), dim3(1), 0, first, flag, 20000000ull);  // 200 ms
    hipLaunchKernelGGL(observe, dim3(1), dim3(1), 0, second, flag, seen);
    (void)hipDeviceSynchronize();
    int h = -1;
    (void)hipMemcpy(&h, seen, 4, hipMemcpyDeviceToHost);
    (void)hipFree(flag);
    (void)hipFree(seen);
    return h;
}

int main() {
    hipStream_t nb = nullptr, blk = nullptr;
    (void)hipStreamCreateWithFlags(&nb, hipStreamNonBlocking);
    (void)hipStreamCreate(&blk);
    printf("null -> per-thread: second kernel saw the first's flag: %d\n", run(nullptr, hipStreamPerThread));
    printf("per-thread -> null: %d\n", run(hipStreamPerThread, nullptr));
    printf("null -> blocking stream: %d\n", run(nullptr, blk));
    printf("null -> non-blocking stream: %d\n", run(nullptr, nb));
    return 0;
}
