// HBM ceiling probe for the MPI_Op streaming kernels (standalone, no torch).
//
// Measures, over 1 GiB operands on one MI355X, what plain 16-B-per-lane
// streaming reaches for the access mixes the op kernels use, so that the
// op kernel's roofline fraction can be read against the achievable rate:
//   rd2    two read streams (a, b), no write (XOR folded, stored only if magic)
//   wr1    one write stream
//   cp     one read + one write stream (copy)
//   op     two reads + one write (out = a + b), the op kernel's shape
//          (threads x unroll, one chunk per workgroup, nt loads + stores)
//   opseq  same, but each workgroup walks SEQ consecutive chunks (longer
//          runs per DRAM page)
//   pstore (argv[2] == 2) the masked partial-line store ceiling the convertor
//          unpack meets: a contiguous packed stream read W bytes per lane and
//          written to a typed layout of period P (W < P: the gap bytes are
//          never written, so every 64-B store request is byte-masked);
//          W/P = 8/16 (vector bl1 of doubles), 16/32 (bl2), 4+8/16
//          (struct {int, double}); "pstore_full" writes the same payload
//          densely (P = W) for comparison.  Rate = 2 x payload bytes / time.
// Output: one JSON line per variant.
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe hbm_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

template <int T, int U>
__global__ __launch_bounds__(T) void k_rd2(const u32x4 *a, const u32x4 *b, u32x4 *out, size_t nvec) {
    const size_t base = (size_t)blockIdx.x * T * U + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * T;
        if (i < nvec) acc ^= __builtin_nontemporal_load(a + i) ^ __builtin_nontemporal_load(b + i);
    }
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) out[base] = acc;
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_wr1(u32x4 *out, size_t nvec) {
    const size_t base = (size_t)blockIdx.x * T * U + threadIdx.x;
    const u32x4 v = {(unsigned)base, 1u, 2u, 3u};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * T;
        if (i < nvec) __builtin_nontemporal_store(v, out + i);
    }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_cp(const u32x4 *a, u32x4 *out, size_t nvec) {
    const size_t base = (size_t)blockIdx.x * T * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * T;
        if (i < nvec) v[u] = __builtin_nontemporal_load(a + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * T;
        if (i < nvec) __builtin_nontemporal_store(v[u], out + i);
    }
}

template <int T, int U, int SEQ>
__global__ __launch_bounds__(T) void k_op(const f32x4 *a, const f32x4 *b, f32x4 *out, size_t nvec) {
    for (int s = 0; s < SEQ; ++s) {
        const size_t base = ((size_t)blockIdx.x * SEQ + s) * T * U + threadIdx.x;
        f32x4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) {
                x[u] = __builtin_nontemporal_load(a + i);
                y[u] = __builtin_nontemporal_load(b + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) __builtin_nontemporal_store(x[u] + y[u], out + i);
        }
    }
}

// Cache-policy variants of the op shape through buffer intrinsics: LP / SP
// are the load / store aux bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1).
template <int T, int U, int LP, int SP>
__global__ __launch_bounds__(T) void k_oppol(const float *a, const float *b, float *out,
                                             size_t nvec) {
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(b), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    const size_t base = (size_t)blockIdx.x * T * U + threadIdx.x;
    f32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * T;
        if (i < nvec) {
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (int)(i * 16), 0, LP);
            y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, (int)(i * 16), 0, LP);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * T;
        if (i < nvec) __builtin_amdgcn_raw_buffer_store_b128(x[u] + y[u], ro, (int)(i * 16), 0, SP);
    }
}

// lane j: W packed bytes at src + j*W -> dst + j*P (+ a second field for
// the struct pattern: 4 bytes at 0 and 8 bytes at 8 of a 16-B period)
template <int W, int P, bool STRUCT>
__global__ __launch_bounds__(256) void k_pstore(const unsigned char *src, unsigned char *dst,
                                                size_t nelem) {
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= nelem) return;
    if (STRUCT) {
        const unsigned *s4 = (const unsigned *)(src + j * 12);
        const unsigned a = __builtin_nontemporal_load(s4);
        const unsigned b = __builtin_nontemporal_load(s4 + 1);
        const unsigned c = __builtin_nontemporal_load(s4 + 2);
        unsigned *d = (unsigned *)(dst + j * 16);
        __builtin_nontemporal_store(a, d);
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(u32x2{b, c}, (u32x2 *)(d + 2));
    } else if (W == 16) {
        const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(src + j * 16));
        __builtin_nontemporal_store(v, (u32x4 *)(dst + j * P));
    } else if (W == 8) {
        const unsigned long long v = __builtin_nontemporal_load((const unsigned long long *)(src + j * 8));
        __builtin_nontemporal_store(v, (unsigned long long *)(dst + j * P));
    } else {
        const unsigned v = __builtin_nontemporal_load((const unsigned *)(src + j * 4));
        __builtin_nontemporal_store(v, (unsigned *)(dst + j * P));
    }
}

template <typename L>
static double time_ms(L &&launch, int reps);

// blacs-indexed unpack stores without the kernel around them (mode 3):
// store op k of period j writes sz[k] bytes from packed offset po[k] of the
// period to typed offset to[k] (a 1548-B period holding 624 B in 18 runs).
// G4: one op per 4-B granule; WIDE: each run cut into naturally aligned 16 /
// 8 / 4-B stores.  NT: non-temporal stores.  TOUCH: every lane first reads
// one byte per 64 B of its period's typed span (brings the lines in before
// the masked stores).
struct bop { unsigned short to, po; unsigned char sz; };
template <bool NT>
__global__ __launch_bounds__(256) void k_blacs(const unsigned char *src, unsigned char *dst,
                                               const bop *ops, int nops, size_t nper, int touch) {
    const size_t j0 = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t total = nper * (size_t)nops;
    unsigned seen = 0;
    if (touch) {
        const size_t per = (size_t)blockIdx.x * 256 / nops;  // first period of this workgroup
        const size_t last = min(nper, ((size_t)blockIdx.x + 1) * 256 / nops + 1);
        for (size_t o = per * 1548 + threadIdx.x * 64; o < last * 1548; o += 256 * 64) seen |= dst[o];
    }
    if (j0 < total) {
        const size_t j = j0 / nops;
        const bop op = ops[j0 - j * nops];
        const unsigned char *s = src + j * 624 + op.po;
        unsigned char *d = dst + j * 1548 + op.to;
        if (op.sz == 16) {
            typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
            u32x4_ v;
            v.x = *(const unsigned *)s; v.y = *(const unsigned *)(s + 4);
            v.z = *(const unsigned *)(s + 8); v.w = *(const unsigned *)(s + 12);
            if (NT) __builtin_nontemporal_store(v, (u32x4_ *)d); else *(u32x4_ *)d = v;
        } else if (op.sz == 8) {
            typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
            u32x2_ v;
            v.x = *(const unsigned *)s; v.y = *(const unsigned *)(s + 4);
            if (NT) __builtin_nontemporal_store(v, (u32x2_ *)d); else *(u32x2_ *)d = v;
        } else {
            const unsigned v = *(const unsigned *)s;
            if (NT) __builtin_nontemporal_store(v, (unsigned *)d); else *(unsigned *)d = v;
        }
    }
    asm volatile("" ::"v"(seen));
}

template <int W, int P, bool STRUCT>
static void run_pstore(void *src, void *dst, size_t dst_bytes, const char *name, int reps) {
    const size_t nelem = dst_bytes / P;
    const size_t payload = nelem * (STRUCT ? 12 : W);
    const unsigned grid = (unsigned)((nelem + 255) / 256);
    const double ms = time_ms([&] {
        hipLaunchKernelGGL((k_pstore<W, P, STRUCT>), dim3(grid), dim3(256), 0, 0,
                           (const unsigned char *)src, (unsigned char *)dst, nelem);
    }, reps);
    const double gbs = 2.0 * payload / (ms * 1e-3) / 1e9;
    printf("{\"variant\": \"%s\", \"W\": %d, \"P\": %d, \"payload_bytes\": %zu, \"ms\": %.4f, "
           "\"GBps\": %.1f, \"frac\": %.4f}\n", name, STRUCT ? 12 : W, P, payload, ms, gbs, gbs / 8000.0);
    fflush(stdout);
}

struct Bufs;

struct Bufs {
    void *a, *b, *c;
    size_t bytes, nvec;
};

template <typename L>
static double time_ms(L &&launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.push_back(ms / reps);
    }
    std::sort(v.begin(), v.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return v[1];
}

static void report(const char *name, int T, int U, int seq, double ms, double bytes) {
    const double gbs = bytes / (ms * 1e-3) / 1e9;
    printf("{\"variant\": \"%s\", \"threads\": %d, \"unroll\": %d, \"seq\": %d, \"ms\": %.4f, "
           "\"GBps\": %.1f, \"frac\": %.4f}\n",
           name, T, U, seq, ms, gbs, gbs / 8000.0);
    fflush(stdout);
}

template <int T, int U>
static void run_basic(const Bufs &B, int reps) {
    const size_t chunk = (size_t)T * U;
    const unsigned grid = (unsigned)((B.nvec + chunk - 1) / chunk);
    const u32x4 *a = (const u32x4 *)B.a, *b = (const u32x4 *)B.b;
    u32x4 *c = (u32x4 *)B.c;
    report("rd2", T, U, 1, time_ms([&] { hipLaunchKernelGGL((k_rd2<T, U>), dim3(grid), dim3(T), 0, 0, a, b, c, B.nvec); }, reps), 2.0 * B.bytes);
    report("wr1", T, U, 1, time_ms([&] { hipLaunchKernelGGL((k_wr1<T, U>), dim3(grid), dim3(T), 0, 0, c, B.nvec); }, reps), 1.0 * B.bytes);
    report("cp", T, U, 1, time_ms([&] { hipLaunchKernelGGL((k_cp<T, U>), dim3(grid), dim3(T), 0, 0, a, c, B.nvec); }, reps), 2.0 * B.bytes);
}

template <int T, int U, int SEQ>
static void run_op(const Bufs &B, int reps) {
    const size_t chunk = (size_t)T * U * SEQ;
    const unsigned grid = (unsigned)((B.nvec + chunk - 1) / chunk);
    const f32x4 *a = (const f32x4 *)B.a, *b = (const f32x4 *)B.b;
    f32x4 *c = (f32x4 *)B.c;
    report(SEQ == 1 ? "op" : "opseq", T, U, SEQ,
           time_ms([&] { hipLaunchKernelGGL((k_op<T, U, SEQ>), dim3(grid), dim3(T), 0, 0, a, b, c, B.nvec); }, reps),
           3.0 * B.bytes);
}

template <int T, int U, int LP, int SP>
static void run_pol(const Bufs &B, int reps) {
    const size_t chunk = (size_t)T * U;
    const unsigned grid = (unsigned)((B.nvec + chunk - 1) / chunk);
    const float *a = (const float *)B.a, *b = (const float *)B.b;
    float *c = (float *)B.c;
    const double ms = time_ms([&] { hipLaunchKernelGGL((k_oppol<T, U, LP, SP>), dim3(grid), dim3(T), 0, 0, a, b, c, B.nvec); }, reps);
    const double gbs = 3.0 * B.bytes / (ms * 1e-3) / 1e9;
    printf("{\"variant\": \"oppol\", \"threads\": %d, \"unroll\": %d, \"load_aux\": %d, \"store_aux\": %d, "
           "\"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n", T, U, LP, SP, ms, gbs, gbs / 8000.0);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const size_t bytes = (argc > 1) ? strtoull(argv[1], nullptr, 0) : (1ull << 30);
    const int reps = 20;
    Bufs B{};
    B.bytes = bytes;
    B.nvec = bytes / 16;
    CK(hipMalloc(&B.a, bytes));
    CK(hipMalloc(&B.b, bytes));
    CK(hipMalloc(&B.c, bytes));
    CK(hipMemset(B.a, 0x11, bytes));
    CK(hipMemset(B.b, 0x22, bytes));
    CK(hipMemset(B.c, 0, bytes));
    CK(hipDeviceSynchronize());
    if (argc > 2 && atoi(argv[2]) == 2) {  // masked partial-line store ceiling only
        // typed destination of `bytes`; the packed source is B.a
        run_pstore<8, 16, false>(B.a, B.c, bytes, "pstore", reps);
        run_pstore<8, 8, false>(B.a, B.c, bytes / 2, "pstore_full", reps);
        run_pstore<16, 32, false>(B.a, B.c, bytes, "pstore", reps);
        run_pstore<16, 16, false>(B.a, B.c, bytes / 2, "pstore_full", reps);
        run_pstore<12, 16, true>(B.a, B.c, bytes, "pstore_struct", reps);
        run_pstore<4, 8, false>(B.a, B.c, bytes, "pstore", reps);
        run_pstore<4, 4, false>(B.a, B.c, bytes / 2, "pstore_full", reps);
        return 0;
    }
    if (argc > 2 && atoi(argv[2]) == 3) {  // blacs-indexed unpack store patterns
        const int lens[18] = {13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1};
        const int disps[18] = {286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603, 626, 649, 672};
        for (int wide = 0; wide < 2; ++wide) {
            std::vector<bop> ops;
            int po = 0;
            for (int r = 0; r < 18; ++r) {
                int to = (disps[r] - 286) * 4, left = lens[r] * 4;
                while (left > 0) {
                    int sz = 4;
                    if (wide) {
                        // widest natural alignment of the typed address (the
                        // typed base of every period is 1548 * j: 4-B aligned
                        // only; the probe's buffer is 16-B aligned, j even
                        // periods keep the alignment of period 0)
                        if (left >= 16 && to % 16 == 0) sz = 16;
                        else if (left >= 8 && to % 8 == 0) sz = 8;
                    }
                    ops.push_back(bop{(unsigned short)to, (unsigned short)po, (unsigned char)sz});
                    to += sz; po += sz; left -= sz;
                }
            }
            bop *dops = nullptr;
            CK(hipMalloc(&dops, ops.size() * sizeof(bop)));
            CK(hipMemcpy(dops, ops.data(), ops.size() * sizeof(bop), hipMemcpyHostToDevice));
            // periods spaced 1548 B would break 8/16-B alignment on odd
            // periods: space them 1552 B? no — keep MPI's layout and use the
            // 4-B ops on every period for wide = 0; wide = 1 is a bound only
            // (run on periods of 1552 B, 16-B aligned)
            const size_t pext = wide ? 1552 : 1548;
            const size_t nper = (bytes - 4096) / pext;
            const int nops = (int)ops.size();
            const unsigned grid = (unsigned)((nper * nops + 255) / 256);
            for (int nt = 0; nt < 2; ++nt)
                for (int touch = 0; touch < 2; ++touch) {
                    const double ms = time_ms([&] {
                        if (nt) hipLaunchKernelGGL((k_blacs<true>), dim3(grid), dim3(256), 0, 0,
                                                   (const unsigned char *)B.a, (unsigned char *)B.c, dops, nops, nper, touch);
                        else hipLaunchKernelGGL((k_blacs<false>), dim3(grid), dim3(256), 0, 0,
                                                (const unsigned char *)B.a, (unsigned char *)B.c, dops, nops, nper, touch);
                    }, reps);
                    const double payload = (double)nper * 624;
                    const double gbs = 2.0 * payload / (ms * 1e-3) / 1e9;
                    printf("{\"variant\": \"blacs_%s%s%s\", \"ops_per_period\": %d, \"period_bytes\": %zu, "
                           "\"payload_bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
                           wide ? "wide" : "g4", nt ? "_nt" : "", touch ? "_touch" : "", nops, pext, payload,
                           ms, gbs, gbs / 8000.0);
                    fflush(stdout);
                }
            CK(hipFree(dops));
        }
        return 0;
    }
    if (argc > 2 && atoi(argv[2]) == 1) {  // cache-policy sweep only
        run_op<256, 4, 1>(B, reps);
        run_pol<256, 4, 2, 2>(B, reps);
        run_pol<256, 4, 0, 0>(B, reps);
        run_pol<256, 4, 2, 17>(B, reps);
        run_pol<256, 4, 2, 19>(B, reps);
        run_pol<256, 4, 2, 16>(B, reps);
        run_pol<256, 4, 2, 18>(B, reps);
        run_pol<256, 4, 16, 2>(B, reps);
        run_pol<256, 4, 19, 2>(B, reps);
        run_pol<256, 4, 18, 18>(B, reps);
        run_pol<256, 4, 1, 1>(B, reps);
        run_pol<256, 8, 2, 2>(B, reps);
        run_pol<256, 8, 2, 17>(B, reps);
        run_pol<512, 4, 2, 17>(B, reps);
        return 0;
    }
    run_basic<256, 4>(B, reps);
    run_basic<256, 8>(B, reps);
    run_basic<512, 4>(B, reps);
    run_op<256, 4, 1>(B, reps);
    run_op<256, 8, 1>(B, reps);
    run_op<512, 4, 1>(B, reps);
    run_op<1024, 2, 1>(B, reps);
    run_op<256, 4, 4>(B, reps);
    run_op<256, 4, 16>(B, reps);
    run_op<256, 2, 8>(B, reps);
    CK(hipFree(B.a));
    CK(hipFree(B.b));
    CK(hipFree(B.c));
    return 0;
}
