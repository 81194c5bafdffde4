// MPI_Op streaming reduction kernels for gfx950 and the op-framework handler
// tables built on them.
//
// Replaces op/base's scalar loops (ompi/mca/op/base/op_base_functions.c:
// 40-104 2-buffer, 654-731 3-buffer, tables 1485-1655).  The work is
// HBM-bound streaming (1 op per 3*sizeof(T) bytes): every lane moves 16 B
// per global access (global_load_dwordx4 / global_store_dwordx4), UNROLL
// independent 16-B vectors per operand are in flight per lane, and the grid
// is capped so every CU stays busy while blocks grid-stride.  No LDS, no
// MFMA: nothing here is reused or contracted.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <array>
#include <utility>

#include "host_mark.h"
#include "op_device.h"
#include "runtime.h"

namespace ompi_amd {

// Build-time tuning knobs (tools/op_tune.py builds variants; the defaults
// are the measured best on MI355X, see DESIGN.md "op kernel").
#ifndef OMPI_AMD_OP_UNROLL
#define OMPI_AMD_OP_UNROLL 4
#endif
#ifndef OMPI_AMD_OP_NT_LOADS
#define OMPI_AMD_OP_NT_LOADS 1
#endif
#ifndef OMPI_AMD_OP_NT_STORES
#define OMPI_AMD_OP_NT_STORES 1
#endif
#ifndef OMPI_AMD_OP_THREADS
#define OMPI_AMD_OP_THREADS 256
#endif
constexpr int kOpThreads = OMPI_AMD_OP_THREADS;
constexpr int kOpUnroll = OMPI_AMD_OP_UNROLL;

__device__ __forceinline__ u32x4 ld16(const u32x4 *p) {
#if OMPI_AMD_OP_NT_LOADS
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
#if OMPI_AMD_OP_NT_STORES
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// dst[i] = f(x[i], y[i]).  2-buffer: x = dst = inout, y = in.
// 3-buffer: x = in1, y = in2, dst = out.  x/dst may alias, so no restrict;
// every lane loads all its vectors before storing any.  The 16-B vectors
// start at element `head` (the operands share their offset within 16 B:
// the head elements before the first boundary and the tail after the last
// whole vector go element by element, in workgroup 0).
template <typename T, int OP, bool THREE>
__global__ __launch_bounds__(kOpThreads) void op_vec_kernel(const T *x, const T *y, T *dst,
                                                            size_t nvec, size_t n, int head) {
    using F = opfn<OP, THREE>;
    constexpr int E = 16 / sizeof(T);
    constexpr size_t chunk = (size_t)kOpThreads * kOpUnroll;
    const u32x4 *xv = reinterpret_cast<const u32x4 *>(x + head);
    const u32x4 *yv = reinterpret_cast<const u32x4 *>(y + head);
    u32x4 *dv = reinterpret_cast<u32x4 *>(dst + head);
    const size_t stride = (size_t)gridDim.x * chunk;

    for (size_t base = (size_t)blockIdx.x * chunk + threadIdx.x; base < nvec; base += stride) {
        vec16<T> a[kOpUnroll], b[kOpUnroll];
#pragma unroll
        for (int u = 0; u < kOpUnroll; ++u) {
            const size_t i = base + (size_t)u * kOpThreads;
            if (i < nvec) {
                a[u].v = ld16(xv + i);
                b[u].v = ld16(yv + i);
            }
        }
#pragma unroll
        for (int u = 0; u < kOpUnroll; ++u) {
            const size_t i = base + (size_t)u * kOpThreads;
            if (i < nvec) {
                vec16<T> r;
                r.v = a[u].v;
#pragma unroll
                for (int e = 0; e < E; ++e) r.e[e] = F::template f<T>(a[u].e[e], b[u].e[e]);
                st16(dv + i, r.v);
            }
        }
    }
    if (blockIdx.x == 0) {
        if ((int)threadIdx.x < head) {  // head: before the first 16-B boundary
            const size_t i = threadIdx.x;
            store_elem<T>(dst + i, F::template f<T>(x[i], y[i]));
        }
        // tail: elements past the last whole 16-B vector
        for (size_t i = (size_t)head + nvec * E + threadIdx.x; i < n; i += kOpThreads)
            store_elem<T>(dst + i, F::template f<T>(x[i], y[i]));
    }
}

// Operands at different offsets within 16 B: elements, kOpUnroll*E per lane
// per pass (coalesced across lanes, every load of a pass issued before its
// stores, so as many bytes are in flight per lane as in op_vec_kernel).
template <typename T, int OP, bool THREE>
__global__ __launch_bounds__(kOpThreads) void op_scalar_kernel(const T *x, const T *y, T *dst,
                                                               size_t n) {
    using F = opfn<OP, THREE>;
    constexpr int K = kOpUnroll * (16 / sizeof(T) < 4 ? 16 / sizeof(T) : 4);
    constexpr size_t chunk = (size_t)kOpThreads * K;
    const size_t stride = (size_t)gridDim.x * chunk;
    for (size_t base = (size_t)blockIdx.x * chunk + threadIdx.x; base < n; base += stride) {
        T a[K], b[K];
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const size_t i = base + (size_t)u * kOpThreads;
            if (i < n) {
                a[u] = x[i];
                b[u] = y[i];
            }
        }
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const size_t i = base + (size_t)u * kOpThreads;
            if (i < n) store_elem<T>(dst + i, F::template f<T>(a[u], b[u]));
        }
    }
}

static int g_max_blocks = -1;

static int op_max_blocks() {
    if (g_max_blocks < 0) {
        const char *s = getenv("OMPI_AMD_OP_MAX_BLOCKS");
        // Default: no cap — one 4-vector-per-lane chunk per workgroup.  On
        // MI355X this beat every grid-stride cap from 512 to 16384 blocks
        // (tools/op_tune.py, profiles/r01_op_tune.jsonl).
        g_max_blocks = (s && atoi(s) > 0) ? atoi(s) : (1 << 24);
    }
    return g_max_blocks;
}

int op_set_max_blocks(int64_t v) {
    if (v <= 0 || v > (1 << 24)) return OMPI_AMD_ERR_BAD_PARAM;
    g_max_blocks = (int)v;
    return OMPI_AMD_SUCCESS;
}

template <typename T, int OP, bool THREE>
static hipError_t launch_typed(const void *x, const void *y, void *dst, size_t n,
                               hipStream_t s) {
    constexpr int E = 16 / sizeof(T);
    const uintptr_t px = (uintptr_t)x & 15, py = (uintptr_t)y & 15, pd = (uintptr_t)dst & 15;
    const size_t max_blocks = (size_t)op_max_blocks();
    // same offset within 16 B (aligned, or e.g. all three displaced by the
    // same element count): peel the head, vectors after it
    if (px == py && px == pd && px % sizeof(T) == 0) {
        size_t head = px ? (16 - px) / sizeof(T) : 0;
        if (head > n) head = n;
        const size_t nvec = (n - head) / E;
        const size_t chunk = (size_t)kOpThreads * kOpUnroll;
        size_t blocks = (nvec + chunk - 1) / chunk;
        if (blocks == 0) blocks = 1;
        if (blocks > max_blocks) blocks = max_blocks;
        hipLaunchKernelGGL((op_vec_kernel<T, OP, THREE>), dim3((unsigned)blocks), dim3(kOpThreads),
                           0, s, (const T *)x, (const T *)y, (T *)dst, nvec, n, (int)head);
    } else {
        constexpr size_t chunk = (size_t)kOpThreads * kOpUnroll * (E < 4 ? E : 4);
        size_t blocks = (n + chunk - 1) / chunk;
        if (blocks == 0) blocks = 1;
        if (blocks > max_blocks) blocks = max_blocks;
        hipLaunchKernelGGL((op_scalar_kernel<T, OP, THREE>), dim3((unsigned)blocks),
                           dim3(kOpThreads), 0, s, (const T *)x, (const T *)y, (T *)dst, n);
    }
    return hipGetLastError();
}

// ---- (op,type) dispatch -------------------------------------------------
template <int OP, int TYPE, bool THREE>
static hipError_t launch_slot(const void *x, const void *y, void *dst, size_t n, hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        return launch_typed<typename type_of<TYPE>::type, OP, THREE>(x, y, dst, n, s);
    } else {
        return hipErrorInvalidValue;
    }
}

using launch_fn = hipError_t (*)(const void *, const void *, void *, size_t, hipStream_t);

template <int OP, bool THREE, int... T>
static constexpr std::array<launch_fn, OMPI_AMD_TYPE_COUNT> make_launch_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &launch_slot<OP, T, THREE> : (launch_fn) nullptr)...}};
}

template <bool THREE, int... O>
static constexpr std::array<std::array<launch_fn, OMPI_AMD_TYPE_COUNT>, OMPI_AMD_OP_COUNT>
make_launch_table(std::integer_sequence<int, O...>) {
    return {{make_launch_row<O, THREE>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}

static const auto g_launch2 =
    make_launch_table<false>(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});
static const auto g_launch3 =
    make_launch_table<true>(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});

int op_launch(int op, int type, bool three, const void *x, const void *y, void *dst,
              size_t n, hipStream_t s) {
    if (op < 0 || op >= OMPI_AMD_OP_COUNT || type < 0 || type >= OMPI_AMD_TYPE_COUNT)
        return OMPI_AMD_ERR_BAD_PARAM;
    launch_fn f = three ? g_launch3[op][type] : g_launch2[op][type];
    if (f == nullptr) return OMPI_AMD_ERR_UNSUPPORTED;
    if (n == 0) return OMPI_AMD_SUCCESS;
    hipError_t e = f(x, y, dst, n, s);
    return record_hip(e, "op kernel launch");
}

// ---- op-framework handlers ----------------------------------------------
struct fallback_slot {
    ompi_amd_op_handler_fn_t fn;
    ompi_op_base_module_1_0_0_t *module;
    ompi_amd_op_3buff_handler_fn_t fn3;
    ompi_op_base_module_1_0_0_t *module3;
};
static fallback_slot g_fallback[OMPI_AMD_OP_COUNT][OMPI_AMD_TYPE_COUNT];

[[noreturn]] static void handler_abort(const char *what, int op, int type) {
    fprintf(stderr, "ompi_amd: op handler (op %d, type %d): %s: %s\n", op, type, what,
            ompi_amd_last_error());
    abort();
}

// kind: 1 = all device, 0 = all host, -1 = mixed
static int buffers_kind(const void *a, const void *b, const void *c) {
    const int da = device_pointer_cached(a), db = device_pointer_cached(b);
    const int dc = c ? device_pointer_cached(c) : db;
    if (da && db && dc) return 1;
    if (!da && !db && !dc) return 0;
    return -1;
}

// Mixed residency: coll/tuned's ring and segmented ring reduce a malloc'd
// host bounce buffer into the caller's device rbuf
// (coll_base_allreduce.c:688-693, 782, 811) whenever coll/rocm declined the
// call (more than OMPI_AMD_MAX_RANKS ranks, a multi-node comm, ranks
// disagreeing on residency).  The handler has no error channel and must not
// abort there: every host operand is staged into a per-thread device
// scratch, the kernel runs on device memory only, and a host output is
// copied back — all on the thread's stream, complete before returning.
struct mixed_scratch {
    char *p = nullptr;
    size_t cap = 0;
};
static thread_local mixed_scratch tls_scratch;  // grown on demand; freed at regrow only

static char *scratch_bytes(size_t bytes) {
    if (bytes <= tls_scratch.cap) return tls_scratch.p;
    const size_t want = std::max(bytes, 2 * tls_scratch.cap);
    if (tls_scratch.p) hip_ignore(hipFree(tls_scratch.p));
    tls_scratch = {};
    void *q = nullptr;
    if (hipMalloc(&q, want) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    tls_scratch = {(char *)q, want};
    return tls_scratch.p;
}

// 2-buffer (three = false): in1 = in, out = inout (also the second operand).
static int reduce_mixed(int op, int type, bool three, const void *in1, const void *in2, void *out,
                        size_t n, hipStream_t s) {
    const size_t bytes = n * ompi_amd_type_extent(type);
    const size_t slot = (bytes + 255) & ~(size_t)255;
    char *scr = scratch_bytes(3 * slot);
    if (!scr) {
        record_msg("op handler: no device scratch for %zu B", 3 * slot);
        return OMPI_AMD_ERR_HIP;
    }
    const void *d1 = in1, *d2 = three ? in2 : out;
    void *dout = out;
    auto stage = [&](const void *host, char *dev) {
        return record_hip(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s),
                          "op handler: stage host operand");
    };
    int rc = OMPI_AMD_SUCCESS;
    if (!ompi_amd_is_device_pointer(in1)) {
        rc = stage(in1, scr);
        d1 = scr;
    }
    if (rc == OMPI_AMD_SUCCESS && three && !ompi_amd_is_device_pointer(in2)) {
        rc = stage(in2, scr + slot);
        d2 = scr + slot;
    }
    if (rc == OMPI_AMD_SUCCESS && !ompi_amd_is_device_pointer(out)) {
        dout = scr + 2 * slot;
        if (!three) {  // inout is an operand too
            rc = stage(out, (char *)dout);
            d2 = dout;
        }
    }
    if (rc == OMPI_AMD_SUCCESS)
        rc = three ? op_launch(op, type, true, d1, d2, dout, n, s)
                   : op_launch(op, type, false, d2, d1, dout, n, s);
    if (rc == OMPI_AMD_SUCCESS && dout != out)
        rc = record_hip(hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, s),
                        "op handler: result to host");
    // the caller reads a host `out` at once: the event wait (host_mark.h)
    if (rc == OMPI_AMD_SUCCESS) rc = record_hip(mark_stream_wait(s, no_idle, dout != out), "op sync");
    return rc;
}

template <int OP, int TYPE>
static void handler2(const void *in, void *inout, int *count, ompi_datatype_t **dtype,
                     ompi_op_base_module_1_0_0_t *module) {
    if (*count <= 0) return;
    const int kind = buffers_kind(in, inout, nullptr);
    const fallback_slot &fb = g_fallback[OP][TYPE];
    if (kind == 0) {
        if (!fb.fn) handler_abort("host buffers and no fallback registered", OP, TYPE);
        fb.fn(in, inout, count, dtype, fb.module);
        return;
    }
    hipStream_t s = thread_stream();
    int rc;
    if (kind == 1) {
        rc = op_launch(OP, TYPE, false, inout, in, inout, (size_t)*count, s);
        if (rc == OMPI_AMD_SUCCESS) rc = record_hip(mark_stream_wait(s, no_idle), "op sync");
    } else {
        rc = reduce_mixed(OP, TYPE, false, in, nullptr, inout, (size_t)*count, s);
    }
    if (rc != OMPI_AMD_SUCCESS) handler_abort("device reduction failed", OP, TYPE);
}

template <int OP, int TYPE>
static void handler3(const void *in1, const void *in2, void *out, int *count,
                     ompi_datatype_t **dtype, ompi_op_base_module_1_0_0_t *module) {
    if (*count <= 0) return;
    const int kind = buffers_kind(in1, in2, out);
    const fallback_slot &fb = g_fallback[OP][TYPE];
    if (kind == 0) {
        if (!fb.fn3) handler_abort("host buffers and no fallback registered", OP, TYPE);
        fb.fn3(in1, in2, out, count, dtype, fb.module3);
        return;
    }
    hipStream_t s = thread_stream();
    int rc;
    if (kind == 1) {
        rc = op_launch(OP, TYPE, true, in1, in2, out, (size_t)*count, s);
        if (rc == OMPI_AMD_SUCCESS) rc = record_hip(mark_stream_wait(s, no_idle), "op sync");
    } else {
        rc = reduce_mixed(OP, TYPE, true, in1, in2, out, (size_t)*count, s);
    }
    if (rc != OMPI_AMD_SUCCESS) handler_abort("device reduction failed", OP, TYPE);
}

template <int OP, int... T>
static constexpr std::array<ompi_amd_op_handler_fn_t, OMPI_AMD_TYPE_COUNT> make_h2_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &handler2<OP, T> : (ompi_amd_op_handler_fn_t) nullptr)...}};
}
template <int OP, int... T>
static constexpr std::array<ompi_amd_op_3buff_handler_fn_t, OMPI_AMD_TYPE_COUNT> make_h3_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &handler3<OP, T>
                                    : (ompi_amd_op_3buff_handler_fn_t) nullptr)...}};
}
template <int... O>
static constexpr std::array<std::array<ompi_amd_op_handler_fn_t, OMPI_AMD_TYPE_COUNT>,
                            OMPI_AMD_OP_COUNT>
make_h2_table(std::integer_sequence<int, O...>) {
    return {{make_h2_row<O>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}
template <int... O>
static constexpr std::array<std::array<ompi_amd_op_3buff_handler_fn_t, OMPI_AMD_TYPE_COUNT>,
                            OMPI_AMD_OP_COUNT>
make_h3_table(std::integer_sequence<int, O...>) {
    return {{make_h3_row<O>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}
static const auto g_h2 = make_h2_table(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});
static const auto g_h3 = make_h3_table(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});

}  // namespace ompi_amd

using namespace ompi_amd;

extern "C" {

int ompi_amd_op_supported(int op, int type) {
    if (op < 0 || op >= OMPI_AMD_OP_COUNT || type < 0 || type >= OMPI_AMD_TYPE_COUNT) return 0;
    return g_launch2[op][type] != nullptr;
}

size_t ompi_amd_type_extent(int type) {
    switch (type) {
    case OMPI_AMD_TYPE_INT8_T: case OMPI_AMD_TYPE_UINT8_T: case OMPI_AMD_TYPE_BOOL:
    case OMPI_AMD_TYPE_BYTE: return 1;
    case OMPI_AMD_TYPE_INT16_T: case OMPI_AMD_TYPE_UINT16_T: case OMPI_AMD_TYPE_SHORT_FLOAT:
        return 2;
    case OMPI_AMD_TYPE_INT32_T: case OMPI_AMD_TYPE_UINT32_T: case OMPI_AMD_TYPE_FLOAT:
    case OMPI_AMD_TYPE_C_SHORT_FLOAT_COMPLEX:
        return 4;
    case OMPI_AMD_TYPE_INT64_T: case OMPI_AMD_TYPE_UINT64_T: case OMPI_AMD_TYPE_DOUBLE: return 8;
    case OMPI_AMD_TYPE_C_FLOAT_COMPLEX: return sizeof(cfloat_t);
    case OMPI_AMD_TYPE_C_DOUBLE_COMPLEX: return sizeof(cdouble_t);
    case OMPI_AMD_TYPE_FLOAT_INT: return sizeof(float_int_t);
    case OMPI_AMD_TYPE_DOUBLE_INT: return sizeof(double_int_t);
    case OMPI_AMD_TYPE_LONG_INT: return sizeof(long_int_t);
    case OMPI_AMD_TYPE_2INT: return sizeof(two_int_t);
    case OMPI_AMD_TYPE_SHORT_INT: return sizeof(short_int_t);
    default: return 0;
    }
}

int ompi_amd_op_reduce(int op, int type, const void *in, void *inout, size_t count,
                       void *stream) {
    if (count && (!in || !inout)) return OMPI_AMD_ERR_BAD_PARAM;
    return op_launch(op, type, false, inout, in, inout, count, as_stream(stream));
}

int ompi_amd_op_reduce_3buff(int op, int type, const void *in1, const void *in2, void *out,
                             size_t count, void *stream) {
    if (count && (!in1 || !in2 || !out)) return OMPI_AMD_ERR_BAD_PARAM;
    return op_launch(op, type, true, in1, in2, out, count, as_stream(stream));
}

const ompi_amd_op_handler_fn_t *ompi_amd_op_handler_row(int op) {
    if (op < 0 || op >= OMPI_AMD_OP_COUNT) return nullptr;
    return g_h2[op].data();
}

const ompi_amd_op_3buff_handler_fn_t *ompi_amd_op_3buff_handler_row(int op) {
    if (op < 0 || op >= OMPI_AMD_OP_COUNT) return nullptr;
    return g_h3[op].data();
}

int ompi_amd_op_set_fallback(int op, int type, ompi_amd_op_handler_fn_t fn,
                             ompi_op_base_module_1_0_0_t *module,
                             ompi_amd_op_3buff_handler_fn_t fn3,
                             ompi_op_base_module_1_0_0_t *module3) {
    if (op < 0 || op >= OMPI_AMD_OP_COUNT || type < 0 || type >= OMPI_AMD_TYPE_COUNT)
        return OMPI_AMD_ERR_BAD_PARAM;
    g_fallback[op][type] = {fn, module, fn3, module3};
    return OMPI_AMD_SUCCESS;
}

}  // extern "C"
