// Strided-gather pack of a wide-gap vector (MPI_Type_vector(count, bl, 2 bl,
// MPI_DOUBLE), the layout ddt_kernels.hip's ddt_vec_kernel packs when the gap
// is too wide for the staged tile): 256 MiB packed, by kernel shape —
// the shipped walk (one pass per lane, grid = granules / (256 x 8)), the same
// with non-temporal accesses, a capped persistent grid, and the runtime's
// hipMemcpy2DAsync as a reference point.  Output: one JSON line per variant;
// GB/s = 2 x packed bytes / time (the read side touches only run bytes: the
// gaps are >= 128 B).
// Build: hipcc --offload-arch=gfx950 -O3 -o ddt_vec_probe ddt_vec_probe.hip
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

struct walk {
    long count, bg, stride, disp, extent, size_g;
};

// NT: 0 plain, 1 nt loads + stores; the walk of ddt_vec_kernel (G = 16)
template <int U, int NT>
__global__ __launch_bounds__(256) void k_vec(walk v, const char *src, char *dst, long ngran) {
    const long S = (long)gridDim.x * 256;
    const long S_el = S / v.size_g, S_q = S % v.size_g;
    const long S_k = S_q / v.bg, S_w = S_q % v.bg;
    const long j0 = (long)blockIdx.x * 256 + threadIdx.x;
    if (j0 >= ngran) return;
    long el = j0 / v.size_g;
    const long q = j0 - el * v.size_g;
    long k = q / v.bg;
    long ww = q - k * v.bg;
    for (long j = j0; j < ngran; j += S * U) {
        long toff[U];
        u32x4 val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            toff[u] = el * v.extent + v.disp + k * v.stride + ww * 16;
            ww += S_w;
            k += S_k;
            if (ww >= v.bg) { ww -= v.bg; ++k; }
            if (k >= v.count) { k -= v.count; ++el; }
            el += S_el;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long jj = j + u * S;
            if (jj < ngran) {
                const u32x4 *p = reinterpret_cast<const u32x4 *>(src + toff[u]);
                val[u] = NT ? __builtin_nontemporal_load(p) : *p;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long jj = j + u * S;
            if (jj < ngran) {
                u32x4 *p = reinterpret_cast<u32x4 *>(dst + jj * 16);
                if (NT) __builtin_nontemporal_store(val[u], p);
                else *p = val[u];
            }
        }
    }
}

// run-major: a wave's lanes cover consecutive granules; granule j lives in
// run j / bg at typed offset (j / bg) * stride + (j % bg) * 16 (bg a power
// of two: shift and mask); persistent grid-stride over the packed stream
template <int U, int NT>
__global__ __launch_bounds__(256) void k_run(const char *src, char *dst, long ngran, int bg_log,
                                             long stride) {
    const long S = (long)gridDim.x * 256;
    for (long j = (long)blockIdx.x * 256 + threadIdx.x; j < ngran; j += S * U) {
        u32x4 val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long jj = j + u * S;
            if (jj < ngran) {
                const long r = jj >> bg_log, w = jj & ((1L << bg_log) - 1);
                const u32x4 *p = reinterpret_cast<const u32x4 *>(src + r * stride + w * 16);
                val[u] = NT ? __builtin_nontemporal_load(p) : *p;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long jj = j + u * S;
            if (jj < ngran) {
                u32x4 *p = reinterpret_cast<u32x4 *>(dst + jj * 16);
                if (NT) __builtin_nontemporal_store(val[u], p);
                else *p = val[u];
            }
        }
    }
}

// per-lane consecutive chunk inside a workgroup tile: workgroup b owns
// packed granules [b*T, (b+1)*T), lane t moves granules t, t+256, ... (U
// per pass, all loads before the stores)
template <int U, int NT>
__global__ __launch_bounds__(256) void k_tile(const char *src, char *dst, long ngran, int bg_log,
                                              long stride, long per_wg) {
    for (long b = blockIdx.x; b * per_wg < ngran; b += gridDim.x) {
        const long lo = b * per_wg, hi = lo + per_wg < ngran ? lo + per_wg : ngran;
        for (long j = lo + threadIdx.x; j < hi; j += 256L * U) {
            u32x4 val[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long jj = j + u * 256L;
                if (jj < hi) {
                    const long r = jj >> bg_log, w = jj & ((1L << bg_log) - 1);
                    const u32x4 *p = reinterpret_cast<const u32x4 *>(src + r * stride + w * 16);
                    val[u] = NT ? __builtin_nontemporal_load(p) : *p;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long jj = j + u * 256L;
                if (jj < hi) {
                    u32x4 *p = reinterpret_cast<u32x4 *>(dst + jj * 16);
                    if (NT) __builtin_nontemporal_store(val[u], p);
                    else *p = val[u];
                }
            }
        }
    }
}

// chunked walk (the xfer kernels' shape): workgroup b moves chunks b, b + G,
// ... of 256 x U packed granules; lane t granules t, t + 256, ... of each.
// The typed position walks by carries as ddt_vec_kernel does: +256 granules
// between a lane's granules of one chunk, +D2 to its first of the next.
struct step {
    long el, k, w;
};
__device__ __forceinline__ void adv(const walk &v, long &el, long &k, long &w, const step &d) {
    w += d.w;
    k += d.k;
    if (w >= v.bg) { w -= v.bg; ++k; }
    if (k >= v.count) { k -= v.count; ++el; }
    el += d.el;
}
__host__ __device__ inline step split(const walk &v, long D) {
    step s;
    s.el = D / v.size_g;
    const long q = D % v.size_g;
    s.k = q / v.bg;
    s.w = q % v.bg;
    return s;
}
template <int U, int NT>
__global__ __launch_bounds__(256) void k_chunk_walk(walk v, const char *src, char *dst, long ngran,
                                                    step d1, step d2) {
    constexpr long C = 256L * U;
    long j = (long)blockIdx.x * C + threadIdx.x;
    if (j >= ngran) return;
    long el = j / v.size_g;
    const long q = j - el * v.size_g;
    long k = q / v.bg, w = q - k * v.bg;
    for (; j < ngran; j += (long)gridDim.x * C) {
        long toff[U];
        u32x4 val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            toff[u] = el * v.extent + v.disp + k * v.stride + w * 16;
            if (u + 1 < U) adv(v, el, k, w, d1);
        }
        adv(v, el, k, w, d2);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (j + u * 256L < ngran) {
                const u32x4 *p = reinterpret_cast<const u32x4 *>(src + toff[u]);
                val[u] = NT ? __builtin_nontemporal_load(p) : *p;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long jj = j + u * 256L;
            if (jj < ngran) {
                u32x4 *p = reinterpret_cast<u32x4 *>(dst + jj * 16);
                if (NT) __builtin_nontemporal_store(val[u], p);
                else *p = val[u];
            }
        }
    }
}

static hipEvent_t ea, eb;

template <typename F>
static void timeit(const char *name, int bl, long grid, long packed, F fn) {
    for (int i = 0; i < 3; ++i) fn();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        const int iters = 20;
        CK(hipEventRecord(ea));
        for (int i = 0; i < iters; ++i) fn();
        CK(hipEventRecord(eb));
        CK(hipEventSynchronize(eb));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ea, eb));
        ms /= iters;
        if (ms < best) best = ms;
    }
    const double gbs = 2.0 * (double)packed / (best * 1e-3) / 1e9;
    printf("{\"variant\": \"%s\", \"bl\": %d, \"grid\": %ld, \"ms\": %.4f, \"gbs\": %.1f, \"frac_of_8TBs\": %.4f}\n",
           name, bl, grid, best, gbs, gbs / 8000.0);
    fflush(stdout);
}

static void check(const char *name, const char *typed_h, const char *out_d, long packed, long blen,
                  long stride) {
    char *h = (char *)malloc(packed);
    CK(hipMemcpy(h, out_d, packed, hipMemcpyDeviceToHost));
    for (long r = 0; r < packed / blen; ++r)
        if (memcmp(h + r * blen, typed_h + r * stride, blen) != 0) {
            printf("{\"variant\": \"%s\", \"error\": \"mismatch at run %ld\"}\n", name, r);
            exit(1);
        }
    free(h);
}

int main(int argc, char **argv) {
    // argv[1]: packed MiB (default 256; 1024 keeps the buffers out of the
    // 256 MB Infinity Cache)
    const long packed = (argc > 1 ? atol(argv[1]) : 256L) << 20;
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    for (int bl : {64, 256}) {  // doubles per run: 512 B (the bench row), 2 KiB
        const long blen = bl * 8L, stride = 2 * blen, runs = packed / blen, span = runs * stride;
        char *typed = nullptr, *out = nullptr;
        CK(hipMalloc(&typed, span));
        CK(hipMalloc(&out, packed));
        char *typed_h = (char *)malloc(span);
        for (long i = 0; i < span; ++i) typed_h[i] = (char)(i * 131 + (i >> 12));
        CK(hipMemcpy(typed, typed_h, span, hipMemcpyHostToDevice));
        const long ngran = packed / 16;
        const long bg = blen / 16;
        int bg_log = 0;
        while ((1L << bg_log) < bg) ++bg_log;
        const walk v{runs, bg, stride, 0, span, runs * bg};
        const long g0 = (ngran + 256 * 8 - 1) / (256 * 8);
        timeit("shipped_walk_u8", bl, g0, packed, [&] {
            hipLaunchKernelGGL((k_vec<8, 0>), dim3(g0), dim3(256), 0, 0, v, typed, out, ngran);
        });
        check("shipped_walk_u8", typed_h, out, packed, blen, stride);
        const long tiles = (ngran + 4095) / 4096;
        timeit("tile64k_u4_nt", bl, tiles, packed, [&] {
            hipLaunchKernelGGL((k_tile<4, 1>), dim3(tiles), dim3(256), 0, 0, typed, out, ngran,
                               bg_log, stride, 4096L);
        });
        const walk c{1, ngran, 0, 0, 0, ngran};
        for (long g : {256L, 512L, 1024L, 2048L}) {
            for (int U : {4, 8}) {
                const step d1 = split(v, 256), d2 = split(v, g * 256L * U - (U - 1) * 256L);
                const step c1 = split(c, 256), c2 = split(c, g * 256L * U - (U - 1) * 256L);
                CK(hipMemset(out, 0, packed));
                if (U == 4) {
                    timeit("chunk_walk_u4_nt", bl, g, packed, [&] {
                        hipLaunchKernelGGL((k_chunk_walk<4, 1>), dim3(g), dim3(256), 0, 0, v, typed,
                                           out, ngran, d1, d2);
                    });
                    check("chunk_walk_u4_nt", typed_h, out, packed, blen, stride);
                    timeit("chunk_walk_u4_plain", bl, g, packed, [&] {
                        hipLaunchKernelGGL((k_chunk_walk<4, 0>), dim3(g), dim3(256), 0, 0, v, typed,
                                           out, ngran, d1, d2);
                    });
                    timeit("contiguous_chunk_walk_u4_nt", bl, g, packed, [&] {
                        hipLaunchKernelGGL((k_chunk_walk<4, 1>), dim3(g), dim3(256), 0, 0, c, typed,
                                           out, ngran, c1, c2);
                    });
                } else {
                    timeit("chunk_walk_u8_nt", bl, g, packed, [&] {
                        hipLaunchKernelGGL((k_chunk_walk<8, 1>), dim3(g), dim3(256), 0, 0, v, typed,
                                           out, ngran, d1, d2);
                    });
                    check("chunk_walk_u8_nt", typed_h, out, packed, blen, stride);
                    timeit("contiguous_chunk_walk_u8_nt", bl, g, packed, [&] {
                        hipLaunchKernelGGL((k_chunk_walk<8, 1>), dim3(g), dim3(256), 0, 0, c, typed,
                                           out, ngran, c1, c2);
                    });
                }
            }
        }
        free(typed_h);
        CK(hipFree(typed));
        CK(hipFree(out));
    }
    return 0;
}
