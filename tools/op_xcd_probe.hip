// XCD placement probe for the MPI_Op 3-buffer kernel (standalone, no torch).
//
// The op kernel (op_kernels.hip op_vec_kernel) gives workgroup b the b-th
// chunk of 256 x 4 16-B vectors; the dispatcher deals workgroups round-robin
// to the 8 XCDs, so neighbouring chunks land on different XCDs.  This probe
// measures, for 3-buffer fp32 SUM over 1 GiB operands, whether handing each
// XCD a contiguous eighth of the vector changes the HBM rate:
//   linear   chunk = b                                   (the shipped map)
//   xcd      chunk = (b % 8) * (nblocks / 8) + b / 8     (XCD-contiguous)
//   skewN    linear, with operand b and out displaced by N x 64 KiB inside one
//            allocation (different HBM channel phase between the streams)
// Output: one JSON line per variant.  Rate = 3 x bytes / kernel time.
// Build: hipcc --offload-arch=gfx950 -O3 -o op_xcd_probe op_xcd_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int T = 256, U = 4;

template <bool XCD>
__global__ __launch_bounds__(T) void k_op(const f32x4 *a, const f32x4 *b, f32x4 *o, long n) {
    long blk = blockIdx.x;
    if (XCD) {
        const long per = gridDim.x / 8;  // grid is a multiple of 8
        blk = (blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const long base = blk * T * U + threadIdx.x;
    f32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * T;
        if (i < n) {
            x[u] = __builtin_nontemporal_load(a + i);
            y[u] = __builtin_nontemporal_load(b + i);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * T;
        if (i < n) __builtin_nontemporal_store(x[u] + y[u], o + i);
    }
}

int main() {
    const long bytes = 1l << 30, n = bytes / 16;
    const long skew_unit = 64 << 10;
    char *pool;
    CK(hipMalloc(&pool, 3 * bytes + 16 * skew_unit));
    CK(hipMemset(pool, 0, 3 * bytes + 16 * skew_unit));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const long blocks = (n + (long)T * U - 1) / ((long)T * U);  // 65536, a multiple of 8
    struct V {
        const char *name;
        bool xcd;
        long skew;
    } vs[] = {{"linear", false, 0}, {"xcd", true, 0},      {"skew1", false, 1},
              {"skew3", false, 3},  {"skew5", false, 5},   {"linear", false, 0},
              {"xcd", true, 0}};
    for (const V &v : vs) {
        const f32x4 *a = (const f32x4 *)pool;
        const f32x4 *b = (const f32x4 *)(pool + bytes + v.skew * skew_unit);
        f32x4 *o = (f32x4 *)(pool + 2 * bytes + 2 * v.skew * skew_unit);
        auto launch = [&] {
            if (v.xcd) hipLaunchKernelGGL(k_op<true>, dim3(blocks), dim3(T), 0, 0, a, b, o, n);
            else hipLaunchKernelGGL(k_op<false>, dim3(blocks), dim3(T), 0, 0, a, b, o, n);
        };
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int iters = 20;
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        const double gbs = 3.0 * bytes / (ms * 1e-3) / 1e9;
        printf("{\"variant\": \"%s\", \"skew_bytes\": %ld, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
               v.name, v.skew * skew_unit, ms, gbs, gbs / 8000.0);
        fflush(stdout);
    }
    CK(hipFree(pool));
    return 0;
}
