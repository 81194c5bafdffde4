// Copy-kernel shape probe for the one-sided / point-to-point transfer kernel
// (osc_ipc.hip xfer_kernel), standalone, no torch.
//
// Round 3 measured put at 0.69 of 8 TB/s with a persistent grid of 256
// workgroups (one system-scope acquire per workgroup; a full grid of
// acquires cost 7x on accumulate).  Every thread/unroll shape of that
// persistent loop measured the same (r03_xfer_shape_sweep.txt), so bytes in
// flight per lane are not the limit; this probe tests what is:
//   persist   the shipped loop: P workgroups, acquire each, per pass U
//             loads then U stores
//   pipe      P workgroups, acquire each, software-pipelined: the loads of
//             pass k+1 are issued before the stores of pass k, so a wave
//             never waits for its own store acks before its next loads
//   full      one chunk per workgroup (grid = bytes / chunk), no acquire
//             (the op kernel's shape; the upper bound for a local copy)
//   fullacq   one chunk per workgroup, acquire in every workgroup
// Output: one JSON line per (variant, P).  Rate = 2 x bytes / kernel time.
// Build: hipcc --offload-arch=gfx950 -O3 -o xfer_probe xfer_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int T = 256, U = 4;

__device__ __forceinline__ void acquire_sys() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

__global__ __launch_bounds__(T) void k_persist(const u32x4 *s, u32x4 *d, long n) {
    if (threadIdx.x == 0) acquire_sys();
    __syncthreads();
    constexpr long chunk = (long)T * U;
    for (long base = (long)blockIdx.x * chunk + threadIdx.x; base < n; base += (long)gridDim.x * chunk) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + (long)u * T;
            if (i < n) v[u] = __builtin_nontemporal_load(s + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + (long)u * T;
            if (i < n) __builtin_nontemporal_store(v[u], d + i);
        }
    }
}

__global__ __launch_bounds__(T) void k_pipe(const u32x4 *s, u32x4 *d, long n) {
    if (threadIdx.x == 0) acquire_sys();
    __syncthreads();
    constexpr long chunk = (long)T * U;
    const long stride = (long)gridDim.x * chunk;
    long base = (long)blockIdx.x * chunk + threadIdx.x;
    u32x4 cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * T;
        if (i < n) cur[u] = __builtin_nontemporal_load(s + i);
    }
    while (base < n) {
        const long nb = base + stride;
        u32x4 nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = nb + (long)u * T;
            if (i < n) nxt[u] = __builtin_nontemporal_load(s + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + (long)u * T;
            if (i < n) __builtin_nontemporal_store(cur[u], d + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        base = nb;
    }
}

template <bool ACQ>
__global__ __launch_bounds__(T) void k_full(const u32x4 *s, u32x4 *d, long n) {
    if (ACQ) {
        if (threadIdx.x == 0) acquire_sys();
        __syncthreads();
    }
    const long base = (long)blockIdx.x * T * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * T;
        if (i < n) v[u] = __builtin_nontemporal_load(s + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * T;
        if (i < n) __builtin_nontemporal_store(v[u], d + i);
    }
}

int main(int argc, char **argv) {
    const long bytes = argc > 1 ? atol(argv[1]) : (256l << 20);
    const long n = bytes / 16;
    u32x4 *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 1, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const long full = (n + (long)T * U - 1) / ((long)T * U);
    struct V {
        const char *name;
        int kind;
        long blocks;
    } vs[] = {{"persist", 0, 256}, {"persist", 0, 512}, {"persist", 0, 1024}, {"persist", 0, 2048},
              {"pipe", 1, 256},    {"pipe", 1, 512},    {"pipe", 1, 1024},    {"pipe", 1, 2048},
              {"full", 2, full},   {"fullacq", 3, full}};
    for (const V &v : vs) {
        auto launch = [&] {
            switch (v.kind) {
            case 0: hipLaunchKernelGGL(k_persist, dim3(v.blocks), dim3(T), 0, 0, s, d, n); break;
            case 1: hipLaunchKernelGGL(k_pipe, dim3(v.blocks), dim3(T), 0, 0, s, d, n); break;
            case 2: hipLaunchKernelGGL(k_full<false>, dim3(v.blocks), dim3(T), 0, 0, s, d, n); break;
            default: hipLaunchKernelGGL(k_full<true>, dim3(v.blocks), dim3(T), 0, 0, s, d, n); break;
            }
        };
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int iters = 20;
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < iters; ++i) launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= iters;
        const double gbs = 2.0 * bytes / (ms * 1e-3) / 1e9;
        printf("{\"variant\": \"%s\", \"blocks\": %ld, \"bytes\": %ld, \"ms\": %.4f, \"GBps\": %.1f, "
               "\"frac\": %.4f}\n",
               v.name, v.blocks, bytes, ms, gbs, gbs / 8000.0);
        fflush(stdout);
    }
    CK(hipFree(s));
    CK(hipFree(d));
    return 0;
}
