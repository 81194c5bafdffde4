// Local device-to-device copy (osc_ipc.hip xfer_kernel's body: 16-B
// granules, 4 per lane in flight, non-temporal) over 256 MiB, by the
// workgroup-entry fence it pays and the grid: system-scope acquire (shipped),
// agent-scope acquire, none; persistent 256 workgroups vs one chunk each.
// Output: one JSON line per variant; GB/s = 2 x bytes / time.
// Build: hipcc --offload-arch=gfx950 -O3 -o xfer_acquire_probe xfer_acquire_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int FENCE, int REL>  // FENCE: 0 none, 1 agent acquire, 2 system acquire; REL: per-WG system release
__global__ __launch_bounds__(256) void k_copy(const u32x4 *src, u32x4 *dst, long n) {
    if (FENCE && threadIdx.x == 0) {
        if (FENCE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    const long chunk = 256L * 4;
    for (long base = (long)blockIdx.x * chunk + threadIdx.x; base < n; base += (long)gridDim.x * chunk) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = base + (long)u * 256;
            if (i < n) v[u] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = base + (long)u * 256;
            if (i < n) __builtin_nontemporal_store(v[u], dst + i);
        }
    }
    if (!REL) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// The shipped shape with THREADS x UNROLL per workgroup (system acquire at
// entry, system release per workgroup at exit).
template <int THREADS, int UNROLL>
__global__ __launch_bounds__(THREADS) void k_copy_shape(const u32x4 *src, u32x4 *dst, long n) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const long chunk = (long)THREADS * UNROLL;
    for (long base = (long)blockIdx.x * chunk + threadIdx.x; base < n; base += (long)gridDim.x * chunk) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const long i = base + (long)u * THREADS;
            if (i < n) v[u] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const long i = base + (long)u * THREADS;
            if (i < n) __builtin_nontemporal_store(v[u], dst + i);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

template <int THREADS, int UNROLL>
static void run_shape(const u32x4 *s, u32x4 *d, long n, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((k_copy_shape<THREADS, UNROLL>), dim3(grid), dim3(THREADS), 0, 0, s, d, n);
    CK(hipDeviceSynchronize());
    const int iters = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((k_copy_shape<THREADS, UNROLL>), dim3(grid), dim3(THREADS), 0, 0, s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= iters;
    const double gbs = 2.0 * (double)n * 16 / (ms * 1e-3) / 1e9;
    printf("{\"shape\": \"%dx%d\", \"grid\": %d, \"ms\": %.4f, \"gbs\": %.1f, \"frac_of_8TBs\": %.4f}\n",
           THREADS, UNROLL, grid, ms, gbs, gbs / 8000.0);
    fflush(stdout);
}

// The same body with its stores through a buffer descriptor carrying cache
// policy bits AUX (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16): write-through
// stores (sc1) leave no dirty lines for the per-workgroup system-scope
// release to write back.  Offsets fit 32 bits (256 MiB).
template <int AUX>
__global__ __launch_bounds__(256) void k_copy_wt(const u32x4 *src, u32x4 *dst, long n) {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(n * 16), 0x00020000);
    const long chunk = 256L * 4;
    for (long base = (long)blockIdx.x * chunk + threadIdx.x; base < n; base += (long)gridDim.x * chunk) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = base + (long)u * 256;
            if (i < n) v[u] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = base + (long)u * 256;
            if (i < n) __builtin_amdgcn_raw_buffer_store_b128(v[u], rs, (int)(i * 16), 0, AUX);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// as k_copy_wt with one descriptor per workgroup chunk (the shape a copy of
// any size needs: 32-bit offsets per descriptor)
template <int AUX>
__global__ __launch_bounds__(256) void k_copy_wt_chunk(const u32x4 *src, u32x4 *dst, long n) {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    const long chunk = 256L * 4;
    for (long c0 = (long)blockIdx.x * chunk; c0 < n; c0 += (long)gridDim.x * chunk) {
        const long left = n - c0;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(dst + c0, 0, (int)((left < chunk ? left : chunk) * 16), 0x00020000);
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = c0 + threadIdx.x + (long)u * 256;
            if (i < n) v[u] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = (int)threadIdx.x + u * 256;
            if (c0 + k < n) __builtin_amdgcn_raw_buffer_store_b128(v[u], rs, k * 16, 0, AUX);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

template <int AUX>
static void run_wt_chunk(const char *name, const u32x4 *s, u32x4 *d, long n, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_copy_wt_chunk<AUX>), dim3(grid), dim3(256), 0, 0, s, d, n);
    CK(hipDeviceSynchronize());
    const int iters = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k_copy_wt_chunk<AUX>), dim3(grid), dim3(256), 0, 0, s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= iters;
    const double gbs = 2.0 * (double)n * 16 / (ms * 1e-3) / 1e9;
    printf("{\"fence\": \"system\", \"release\": 1, \"stores\": \"%s, descriptor per chunk\", \"grid\": %d, \"ms\": %.4f, \"gbs\": %.1f, \"frac_of_8TBs\": %.4f}\n",
           name, grid, ms, gbs, gbs / 8000.0);
    fflush(stdout);
}

template <int AUX>
static void run_wt(const char *name, const u32x4 *s, u32x4 *d, long n, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_copy_wt<AUX>), dim3(grid), dim3(256), 0, 0, s, d, n);
    CK(hipDeviceSynchronize());
    const int iters = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k_copy_wt<AUX>), dim3(grid), dim3(256), 0, 0, s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= iters;
    const double gbs = 2.0 * (double)n * 16 / (ms * 1e-3) / 1e9;
    printf("{\"fence\": \"system\", \"release\": 1, \"stores\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"gbs\": %.1f, \"frac_of_8TBs\": %.4f}\n",
           name, grid, ms, gbs, gbs / 8000.0);
    fflush(stdout);
}

template <int FENCE, int REL>
static void run(const char *name, const u32x4 *s, u32x4 *d, long n, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_copy<FENCE, REL>), dim3(grid), dim3(256), 0, 0, s, d, n);
    CK(hipDeviceSynchronize());
    const int iters = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k_copy<FENCE, REL>), dim3(grid), dim3(256), 0, 0, s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= iters;
    const double gbs = 2.0 * (double)n * 16 / (ms * 1e-3) / 1e9;
    printf("{\"fence\": \"%s\", \"release\": %d, \"grid\": %d, \"ms\": %.4f, \"gbs\": %.1f, \"frac_of_8TBs\": %.4f}\n", name, REL, grid,
           ms, gbs, gbs / 8000.0);
    fflush(stdout);
}

int main(int argc, char **argv) {
    // argv[3]: MiB to copy (default 256; 1024+ keeps the destination out of
    // the 256 MB Infinity Cache)
    const long bytes = (argc > 3 ? atol(argv[3]) : 256L) << 20, n = bytes / 16;
    u32x4 *s = nullptr, *d = nullptr;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 1, bytes));
    CK(hipMemset(d, 0, bytes));
    const int full = (int)((n + 1023) / 1024);
    if (argc > 2 && !strcmp(argv[2], "fine")) {  // a fine-grained destination (hipExtMallocWithFlags)
        CK(hipFree(d));
        CK(hipExtMallocWithFlags((void **)&d, bytes, hipDeviceMallocFinegrained));
        CK(hipMemset(d, 0, bytes));
        printf("{\"destination\": \"fine-grained\"}\n");
    }
    if (argc > 1 && !strcmp(argv[1], "shape")) {  // bytes in flight per workgroup, fences in
        for (int grid : {256, 512}) {
            run_shape<256, 4>(s, d, n, grid);
            run_shape<256, 8>(s, d, n, grid);
            run_shape<256, 16>(s, d, n, grid);
            run_shape<512, 4>(s, d, n, grid);
            run_shape<512, 8>(s, d, n, grid);
            run_shape<1024, 4>(s, d, n, grid);
            run_shape<1024, 8>(s, d, n, grid);
        }
        return 0;
    }
    if (argc > 1 && !strcmp(argv[1], "wt")) {  // store cache policy under the shipped release
        for (int grid : {256, 512, 1024}) {
            run<2, 1>("system", s, d, n, grid);
            run_wt<0>("buffer plain", s, d, n, grid);
            run_wt<2>("buffer nt", s, d, n, grid);
            run_wt<16>("buffer sc1", s, d, n, grid);
            run_wt<17>("buffer sc0 sc1", s, d, n, grid);
            run_wt<18>("buffer nt sc1", s, d, n, grid);
            run_wt_chunk<17>("buffer sc0 sc1", s, d, n, grid);
            run_wt_chunk<0>("buffer plain", s, d, n, grid);
            run<2, 0>("system", s, d, n, grid);
        }
        return 0;
    }
    for (int grid : {256, 512, 1024, 2048, 4096, full}) {
        run<2, 1>("system", s, d, n, grid);
        run<2, 0>("system", s, d, n, grid);
        run<0, 0>("none", s, d, n, grid);
    }
    return 0;
}
