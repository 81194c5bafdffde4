// Shape probe for the osc derived-target accumulate (osc_ipc.hip
// ddt_acc_kernel), standalone, no torch, no library.
//
// Round 4's bench row (MPI_Type_vector of single doubles at stride 2 over a
// 256 MiB window, 128 MiB packed f64 origin SUMmed in) ran at 1.70 TB/s of
// algorithmic bytes (1.5 x S).  Its PMC passes (round 5,
// profiles/r05_pmc_*_ddt_acc.csv) count 402.7 MB fetched (the packed origin
// + the target's typed span read whole) and 268.4 MB written (byte-masked
// requests over the whole span) per launch: 671 MB in 0.235 ms = 2.86 TB/s
// of real traffic, below the masked-store probe's rate.  The shipped shape
// is a persistent grid of 256 workgroups x 256 threads (one system-scope
// acquire per workgroup) with 4 elements per lane in flight: one wave per
// SIMD, ~16 KiB of loads in flight per CU.  This probe varies threads per
// workgroup and elements per lane (bytes in flight) and the grid, with the
// kernel's own element -> typed-offset mapping (ddt_device.h).
// Output: one JSON line per (threads, unroll, grid); rate = 1.5 x S / time.
// Build: hipcc --offload-arch=gfx950 -O3 -I.. -o ddt_acc_probe ddt_acc_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../ompi_amd/csrc/ddt_device.h"

using namespace ompi_amd;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__device__ __forceinline__ void acquire_sys() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }
__device__ __forceinline__ void release_sys() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// round 5: the library keeps a single-element type's element in registers
// (osc_ipc.hip ddt_acc_kernel); this loop does the same
template <int THREADS, int UNROLL>
__global__ __launch_bounds__(THREADS) void k_acc(ddt_desc d, char *typed, const double *in, int64_t n) {
    if (threadIdx.x == 0) acquire_sys();
    const ddt_elem e0 = d.elems[0];
    __syncthreads();
    const ddt_elem *el = &e0;
    const int64_t chunk = (int64_t)THREADS * UNROLL;
    const int64_t gs = (int64_t)gridDim.x * chunk;
    for (int64_t b = (int64_t)blockIdx.x * chunk + threadIdx.x; b < n; b += gs) {
        double *t[UNROLL];
        double v[UNROLL], x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t k = b + (int64_t)u * THREADS;
            t[u] = nullptr;
            if (k < n) {
                t[u] = reinterpret_cast<double *>(
                    typed + typed_offset_fast<8>(el, 1, (uint32_t)(d.size / 8), d.sdiv, d.extent,
                                                 (uint32_t)k));
                v[u] = *t[u];
                x[u] = in[k];
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            if (t[u]) *t[u] = v[u] + x[u];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) release_sys();
}

template <int THREADS, int UNROLL>
static void run(const ddt_desc &d, char *typed, const double *in, int64_t n, int64_t S, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((k_acc<THREADS, UNROLL>), dim3(grid), dim3(THREADS), 0, 0, d, typed, in, n);
    CK(hipDeviceSynchronize());
    const int iters = 10;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((k_acc<THREADS, UNROLL>), dim3(grid), dim3(THREADS), 0, 0, d, typed, in, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= iters;
    const double gbs = 1.5 * (double)S / (ms * 1e-3) / 1e9;
    printf("{\"threads\": %d, \"unroll\": %d, \"grid\": %d, \"ms\": %.4f, \"algo_gbs\": %.1f, \"frac_of_8TBs\": %.4f}\n",
           THREADS, UNROLL, grid, ms, gbs, gbs / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main(int argc, char **argv) {
    const int64_t S = (argc > 1 ? atoll(argv[1]) : 256) << 20;
    const int64_t n = S / 16;  // doubles in the packed origin
    char *typed = nullptr;
    double *in = nullptr;
    CK(hipMalloc(&typed, S));
    CK(hipMalloc(&in, S / 2));
    CK(hipMemset(typed, 0, S));
    CK(hipMemset(in, 0, S / 2));
    // MPI_Type_vector(S / 16, 1, 2, MPI_DOUBLE): one element {count, 8 B, 16 B}
    ddt_elem h{};
    h.count = n;
    h.blen = 8;
    h.stride = 16;
    h.disp = 0;
    h.prefix = 0;
    for (int g = 0; g < 5; ++g) h.bdiv[g] = make_fdiv((uint32_t)(8 >> g ? 8 >> g : 1));
    ddt_elem *de = nullptr;
    CK(hipMalloc(&de, sizeof(h)));
    CK(hipMemcpy(de, &h, sizeof(h), hipMemcpyHostToDevice));
    ddt_desc d{};
    d.elems = de;
    d.nelem = 1;
    d.size = S / 2;
    d.extent = (n - 1) * 16 + 8;
    d.sdiv = make_fdiv((uint32_t)(d.size / 8));
    for (int grid : {256, 512, 1024}) {
        run<256, 4>(d, typed, in, n, S, grid);
        run<256, 8>(d, typed, in, n, S, grid);
        run<256, 16>(d, typed, in, n, S, grid);
        run<512, 8>(d, typed, in, n, S, grid);
        run<1024, 4>(d, typed, in, n, S, grid);
        run<1024, 8>(d, typed, in, n, S, grid);
    }
    return 0;
}
