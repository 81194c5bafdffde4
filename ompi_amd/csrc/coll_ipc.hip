// Device-buffer collectives over xGMI for gfx950: allreduce,
// reduce_scatter_block, allgather, bcast (include/ompi_amd_coll.h).
//
// Reference path being replaced (coll/tuned over PML ob1 + btl/sm):
//   allreduce  coll_tuned_decision_fixed.c:45-89 ->
//              ring_segmented coll_base_allreduce.c:618-856 (1 MiB segments,
//              N-1 hops per segment, host bounce buffers, one op call per hop)
// Here each rank owns one ring block (COLL_BASE_COMPUTE_BLOCKCOUNT,
// coll_base_functions.h:425-431) and produces it in ONE pass that loads the
// block from every peer's buffer over xGMI at once (all N-1 links busy) and
// folds the values in exactly the ring's operand order
//     block b = x[b-1] (+) (x[b-2] (+) (... (x[b+1] (+) x[b])))
// with (+) the 2-buffer op rule f(out, in) — so fp results are bit-identical
// to the reference — then every rank pulls the other N-1 finished blocks
// from their owners (again all links at once).  Below 10000 bytes the
// reference runs recursive doubling (coll_base_allreduce.c:130-274); the
// same pass then folds in that algorithm's pairwise-tree order.
//
// Synchronisation: a monotonically increasing epoch per communicator.  A
// barrier is one 64-lane workgroup: lane p stores the epoch into peer p's
// flag slot [me] (system-scope atomic into fine-grained IPC memory) and
// polls its own slot [p] until the peer's epoch arrives, with a wall-clock
// bound (s_memrealtime) that sets a sticky error word instead of hanging.
// Kernel boundaries on the stream order the barrier after the producer of
// the data; every transfer workgroup opens with a system-scope acquire
// (buffer_inv sc0 sc1: drops stale lines of peer memory from this XCD's
// caches) and closes with a system-scope release (buffer_wbl2 sc0 sc1).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "../../include/ompi_amd_coll.h"
#include "bootstrap.h"
#include "op_device.h"
#include "runtime.h"

namespace ompi_amd {

constexpr int kMaxRanks = OMPI_AMD_MAX_RANKS;
constexpr int kXferThreads = 256;

struct ptr_set { const char *p[kMaxRanks]; };
struct flag_set { uint64_t *p[kMaxRanks]; };

enum order_t { ORDER_RING = 0, ORDER_TREE = 1, ORDER_LINEAR = 2 };

// One reduction job: elements [off, off+cnt) of every source, combined in
// `order` and written to dst + off_dst (element units).
struct red_job {
    int64_t off, cnt, off_dst;
    int first;  // ring order: the block id b (sources start at rank b)
    int head;   // elements before the 16-B aligned body; -1: no common alignment
};
struct red_jobs { red_job j[kMaxRanks]; int n; };

struct cp_job { const char *src; char *dst; int64_t bytes; };
struct cp_jobs { cp_job j[kMaxRanks]; int n; };

__device__ __forceinline__ void sys_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }
__device__ __forceinline__ void sys_release() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------- barrier
__global__ __launch_bounds__(64) void barrier_kernel(uint64_t *local, flag_set peers, int rank,
                                                     int size, uint64_t epoch, int *err,
                                                     uint64_t timeout_ticks) {
    const int t = threadIdx.x;
    sys_release();
    if (t < size && t != rank)
        __hip_atomic_store(peers.p[t] + rank, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < size && t != rank) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(local + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
                __hip_atomic_store(err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
    }
    __syncthreads();
    sys_acquire();
}

// ---------------------------------------------------------------- reduce
template <typename T, int OP>
__device__ __forceinline__ T fold(const T (&v)[kMaxRanks], int n, int order) {
    using F = opfn<OP, false>;  // 2-buffer rule: f(out, in)
    if (order == ORDER_RING) {
        // v[j] = x[(b + j) % n]; acc = x[b]; acc = f(x[b+j], acc)
        T acc = v[0];
#pragma unroll
        for (int j = 1; j < kMaxRanks; ++j)
            if (j < n) acc = F::template f<T>(v[j], acc);
        return acc;
    }
    if (order == ORDER_LINEAR) {
        // basic_linear reduce (coll_base_reduce.c:627-700): acc = x[n-1];
        // for i = n-2..0: acc = f(acc, x[i])
        T acc = v[kMaxRanks - 1];
#pragma unroll
        for (int j = kMaxRanks - 1; j >= 0; --j)
            if (j == n - 1) acc = v[j];
            else if (j < n - 1) acc = F::template f<T>(acc, v[j]);
        return acc;
    }
    // recursive doubling (coll_base_allreduce.c:184-236): fold the
    // 2*extra lowest ranks pairwise, then a pairwise tree; every combine is
    // f(out = higher, in = lower).
    int adj = 1;
    while (adj * 2 <= n) adj *= 2;
    const int extra = n - adj;
    T w[kMaxRanks];
#pragma unroll
    for (int i = 0; i < kMaxRanks; ++i) {
        if (i < extra) w[i] = F::template f<T>(v[2 * i + 1], v[2 * i]);
        else if (i < adj) w[i] = v[i + extra];
    }
#pragma unroll
    for (int len = kMaxRanks; len > 1; len >>= 1) {
        if (len <= adj) {
#pragma unroll
            for (int i = 0; i < kMaxRanks / 2; ++i)
                if (2 * i + 1 < len) w[i] = F::template f<T>(w[2 * i + 1], w[2 * i]);
        }
    }
    return w[0];
}

// Gather v[j] for element index e of the sources in the job's order.
template <typename T>
__device__ __forceinline__ void gather_scalar(T (&v)[kMaxRanks], const ptr_set &src, int n,
                                              int order, int first, int64_t e) {
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) {
        if (j < n) {
            const int r = (order == ORDER_RING) ? (first + j) % n : j;
            v[j] = reinterpret_cast<const T *>(src.p[r])[e];
        }
    }
}

template <typename T, int OP>
__global__ __launch_bounds__(kXferThreads) void reduce_kernel(ptr_set src, T *dst, int n,
                                                              int order, red_jobs jobs) {
    sys_acquire();
    const red_job jb = jobs.j[blockIdx.y];
    constexpr int E = 16 / sizeof(T);
    const int64_t gstride = (int64_t)gridDim.x * kXferThreads;
    const int64_t tid = (int64_t)blockIdx.x * kXferThreads + threadIdx.x;
    // vector body [head, head + nvec*E): every source and dst 16-B aligned
    // there (head < 0: no common alignment, all scalar)
    const int64_t head = jb.head < 0 ? jb.cnt : jb.head;
    const int64_t nvec = jb.head < 0 ? 0 : (jb.cnt - head) / E;
    for (int64_t i = tid; i < nvec; i += gstride) {
        vec16<T> v[kMaxRanks];
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j) {
            if (j < n) {
                const int r = (order == ORDER_RING) ? (jb.first + j) % n : j;
                const u32x4 *p = reinterpret_cast<const u32x4 *>(
                    reinterpret_cast<const T *>(src.p[r]) + jb.off + head);
                v[j].v = __builtin_nontemporal_load(p + i);
            }
        }
        vec16<T> out;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            T s[kMaxRanks];
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j) s[j] = v[j].e[e];
            out.e[e] = fold<T, OP>(s, n, order);
        }
        reinterpret_cast<u32x4 *>(dst + jb.off_dst + head)[i] = out.v;
    }
    // scalar head [0, head) and tail [head + nvec*E, cnt)
    const int64_t tail0 = head + nvec * E;
    const int64_t nscalar = head + (jb.cnt - tail0);
    for (int64_t k = tid; k < nscalar; k += gstride) {
        const int64_t e = k < head ? k : tail0 + (k - head);
        T s[kMaxRanks];
        gather_scalar<T>(s, src, n, order, jb.first, jb.off + e);
        store_elem<T>(dst + jb.off_dst + e, fold<T, OP>(s, n, order));
    }
    __syncthreads();
    if (threadIdx.x == 0) sys_release();
}

// ---------------------------------------------------------------- copy
// Byte copy with a peeled head so that the body runs 16 B (or 4 B) per
// lane whenever src and dst share their alignment phase.
__global__ __launch_bounds__(kXferThreads) void copy_kernel(cp_jobs jobs) {
    sys_acquire();
    const cp_job jb = jobs.j[blockIdx.y];
    const int64_t gstride = (int64_t)gridDim.x * kXferThreads;
    const int64_t tid = (int64_t)blockIdx.x * kXferThreads + threadIdx.x;
    const uintptr_t phase = (uintptr_t)jb.src ^ (uintptr_t)jb.dst;
    const int g = (phase & 15) == 0 ? 16 : ((phase & 3) == 0 ? 4 : 1);
    int64_t head = (int64_t)((g - ((uintptr_t)jb.src & (uintptr_t)(g - 1))) & (uintptr_t)(g - 1));
    if (head > jb.bytes) head = jb.bytes;
    const int64_t nbody = (jb.bytes - head) / g;
    const char *sb = jb.src + head;
    char *db = jb.dst + head;
    if (g == 16) {
        const u32x4 *s = reinterpret_cast<const u32x4 *>(sb);
        u32x4 *d = reinterpret_cast<u32x4 *>(db);
        int64_t i = tid;
        for (; i + 3 * gstride < nbody; i += 4 * gstride) {
            const u32x4 a = __builtin_nontemporal_load(s + i);
            const u32x4 b = __builtin_nontemporal_load(s + i + gstride);
            const u32x4 c = __builtin_nontemporal_load(s + i + 2 * gstride);
            const u32x4 e = __builtin_nontemporal_load(s + i + 3 * gstride);
            d[i] = a;
            d[i + gstride] = b;
            d[i + 2 * gstride] = c;
            d[i + 3 * gstride] = e;
        }
        for (; i < nbody; i += gstride) d[i] = __builtin_nontemporal_load(s + i);
    } else if (g == 4) {
        const uint32_t *s = reinterpret_cast<const uint32_t *>(sb);
        uint32_t *d = reinterpret_cast<uint32_t *>(db);
        for (int64_t i = tid; i < nbody; i += gstride) d[i] = s[i];
    } else {
        for (int64_t i = tid; i < nbody; i += gstride) db[i] = sb[i];
    }
    const int64_t tail0 = head + nbody * g;
    const int64_t nrest = head + (jb.bytes - tail0);
    for (int64_t k = tid; k < nrest; k += gstride) {
        const int64_t i = k < head ? k : tail0 + (k - head);
        jb.dst[i] = jb.src[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) sys_release();
}

// ---------------------------------------------------------------- dispatch
using red_launch_fn = hipError_t (*)(dim3, const ptr_set &, void *, int, int, const red_jobs &,
                                     hipStream_t);

template <int OP, int TYPE>
static hipError_t red_launch_slot(dim3 grid, const ptr_set &src, void *dst, int n, int order,
                                  const red_jobs &jobs, hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        using T = typename type_of<TYPE>::type;
        hipLaunchKernelGGL((reduce_kernel<T, OP>), grid, dim3(kXferThreads), 0, s, src, (T *)dst,
                           n, order, jobs);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}

template <int OP, int... T>
static constexpr std::array<red_launch_fn, OMPI_AMD_TYPE_COUNT> make_red_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &red_launch_slot<OP, T> : (red_launch_fn) nullptr)...}};
}
template <int... O>
static constexpr std::array<std::array<red_launch_fn, OMPI_AMD_TYPE_COUNT>, OMPI_AMD_OP_COUNT>
make_red_table(std::integer_sequence<int, O...>) {
    return {{make_red_row<O>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}
static const auto g_red = make_red_table(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});

// MPI type size (bytes of data) — the tuned decision uses it, not the extent
// (ompi_datatype_module.c:404-430: DOUBLE_INT size 12 / extent 16).
static size_t type_size(int type) {
    switch (type) {
    case OMPI_AMD_TYPE_DOUBLE_INT: case OMPI_AMD_TYPE_LONG_INT: return 12;
    case OMPI_AMD_TYPE_SHORT_INT: return 6;
    default: return ompi_amd_type_extent(type);
    }
}

static void blockcount(int64_t count, int n, int64_t *split, int64_t *early, int64_t *late) {
    *early = *late = count / n;
    *split = count % n;
    if (*split) *early += 1;
}
static int64_t block_off(int64_t b, int64_t split, int64_t early, int64_t late) {
    return b < split ? b * early : b * late + split;
}
static int64_t block_cnt(int64_t b, int64_t split, int64_t early, int64_t late) {
    return b < split ? early : late;
}

}  // namespace ompi_amd

using namespace ompi_amd;

// ------------------------------------------------------------------ comm
struct ompi_amd_comm {
    int rank = 0, size = 0, device = 0;
    ShmBoot boot;
    uint64_t *flags = nullptr;            // [kMaxRanks] epochs written by peers
    flag_set peer_flags{};
    char *scratch = nullptr;              // staged-path landing zone: two halves
    size_t scratch_bytes = 0;             // bytes per half
    uint64_t stage_seq = 0;               // staged calls so far (selects the half)
    ptr_set peer_scratch{};
    int *err_host = nullptr, *err_dev = nullptr;
    uint64_t epoch = 0;
    // params
    size_t small_bytes = 1 << 20;
    int zero_copy = 1;
    int64_t timeout_ms = 30000;
    int max_blocks = 1024;
    // IPC caches
    struct exp_entry { void *base; size_t size; unsigned long long id; hipIpcMemHandle_t h; };
    struct imp_entry { int peer; hipIpcMemHandle_t h; void *base; uint64_t last_use; };
    std::vector<exp_entry> exports;
    std::vector<imp_entry> imports;
    uint64_t use_clock = 0;
    void *opened[kMaxRanks][2] = {};      // flags / scratch mappings of peers
    // per-phase kernel timing (param "profile"): event pairs per call
    int profile = 0;
    std::vector<hipEvent_t> ev_free;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_phase[2];
};

namespace ompi_amd {

struct ipc_blob {
    hipIpcMemHandle_t flags, scratch;
};

// What each rank publishes per zero-copy call: its user buffers as
// (allocation handle, offset).
struct buf_desc {
    hipIpcMemHandle_t h;
    uint64_t off;
    uint64_t valid;
};
struct call_blob {
    buf_desc s, r;
};

static int set_dev(ompi_amd_comm_t *c) {
    return record_hip(hipSetDevice(c->device), "hipSetDevice");
}

static int export_buf(ompi_amd_comm_t *c, const void *ptr, buf_desc *d) {
    memset(d, 0, sizeof(*d));
    if (!ptr) return OMPI_AMD_SUCCESS;
    void *base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange((hipDeviceptr_t *)&base, &size, (hipDeviceptr_t)ptr);
    if (e != hipSuccess) return record_hip(e, "hipMemGetAddressRange (buffer not device memory?)");
    unsigned long long id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)ptr) !=
        hipSuccess) {
        (void)hipGetLastError();
        id = 0;
    }
    for (auto &x : c->exports) {
        if (x.base == base && x.size == size && x.id == id) {
            d->h = x.h;
            d->off = (uint64_t)((const char *)ptr - (const char *)base);
            d->valid = 1;
            return OMPI_AMD_SUCCESS;
        }
    }
    ompi_amd_comm::exp_entry x{base, size, id, {}};
    e = hipIpcGetMemHandle(&x.h, base);
    if (e != hipSuccess) return record_hip(e, "hipIpcGetMemHandle");
    // drop stale entries that overlap this allocation
    c->exports.erase(std::remove_if(c->exports.begin(), c->exports.end(),
                                    [&](const ompi_amd_comm::exp_entry &o) {
                                        return (char *)o.base < (char *)base + size &&
                                               (char *)base < (char *)o.base + o.size;
                                    }),
                     c->exports.end());
    c->exports.push_back(x);
    d->h = x.h;
    d->off = (uint64_t)((const char *)ptr - (const char *)base);
    d->valid = 1;
    return OMPI_AMD_SUCCESS;
}

static int import_buf(ompi_amd_comm_t *c, int peer, const buf_desc &d, const char **out) {
    *out = nullptr;
    if (!d.valid) return OMPI_AMD_SUCCESS;
    for (auto &x : c->imports) {
        if (x.peer == peer && memcmp(&x.h, &d.h, sizeof(d.h)) == 0) {
            x.last_use = ++c->use_clock;
            *out = (const char *)x.base + d.off;
            return OMPI_AMD_SUCCESS;
        }
    }
    if (c->imports.size() >= 256) {  // evict the least recently used mapping
        auto it = std::min_element(c->imports.begin(), c->imports.end(),
                                   [](const ompi_amd_comm::imp_entry &a,
                                      const ompi_amd_comm::imp_entry &b) {
                                       return a.last_use < b.last_use;
                                   });
        (void)hipIpcCloseMemHandle(it->base);
        c->imports.erase(it);
    }
    void *base = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&base, d.h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return record_hip(e, "hipIpcOpenMemHandle");
    c->imports.push_back({peer, d.h, base, ++c->use_clock});
    *out = (const char *)base + d.off;
    return OMPI_AMD_SUCCESS;
}

// Swap (sbuf, rbuf) descriptors with every peer and map theirs.
static int exchange_bufs(ompi_amd_comm_t *c, const void *sbuf, const void *rbuf, ptr_set *s,
                         ptr_set *r) {
    call_blob mine{};
    int rc = export_buf(c, sbuf, &mine.s);
    if (rc == OMPI_AMD_SUCCESS) rc = export_buf(c, rbuf, &mine.r);
    if (rc != OMPI_AMD_SUCCESS) return rc;
    call_blob all[kMaxRanks];
    rc = c->boot.allgather(&mine, all, sizeof(call_blob));
    if (rc != OMPI_AMD_SUCCESS) return rc;
    for (int p = 0; p < c->size; ++p) {
        if (p == c->rank) {
            s->p[p] = (const char *)sbuf;
            r->p[p] = (const char *)rbuf;
            continue;
        }
        if ((rc = import_buf(c, p, all[p].s, &s->p[p])) != OMPI_AMD_SUCCESS) return rc;
        if ((rc = import_buf(c, p, all[p].r, &r->p[p])) != OMPI_AMD_SUCCESS) return rc;
    }
    return OMPI_AMD_SUCCESS;
}

static int launch_barrier(ompi_amd_comm_t *c, hipStream_t s) {
    ++c->epoch;
    const uint64_t ticks = (uint64_t)c->timeout_ms * 100000ull;  // s_memrealtime: 100 MHz
    hipLaunchKernelGGL(barrier_kernel, dim3(1), dim3(64), 0, s, c->flags, c->peer_flags, c->rank,
                       c->size, c->epoch, c->err_dev, ticks);
    return record_hip(hipGetLastError(), "barrier launch");
}

static int launch_copy(ompi_amd_comm_t *c, const cp_jobs &jobs, hipStream_t s) {
    if (jobs.n == 0) return OMPI_AMD_SUCCESS;
    int64_t most = 0;
    for (int i = 0; i < jobs.n; ++i) most = std::max(most, jobs.j[i].bytes);
    int64_t blocks = (most / 16 + kXferThreads * 4 - 1) / (kXferThreads * 4);
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, std::max(1, c->max_blocks / jobs.n)));
    hipLaunchKernelGGL(copy_kernel, dim3((unsigned)blocks, (unsigned)jobs.n), dim3(kXferThreads),
                       0, s, jobs);
    return record_hip(hipGetLastError(), "copy launch");
}

static int launch_reduce(ompi_amd_comm_t *c, int op, int type, const ptr_set &src, void *dst,
                         int order, red_jobs jobs, hipStream_t s) {
    red_launch_fn f = g_red[op][type];
    if (!f) return OMPI_AMD_ERR_UNSUPPORTED;
    if (jobs.n == 0) return OMPI_AMD_SUCCESS;
    const size_t ext = ompi_amd_type_extent(type);
    int64_t most = 0;
    for (int i = 0; i < jobs.n; ++i) {
        red_job &j = jobs.j[i];
        // every source and dst must sit at the same phase mod 16 B, and that
        // phase must be a whole number of elements from 16-B alignment
        const uintptr_t ph = (uintptr_t)((const char *)dst + j.off_dst * ext) & 15;
        bool same = ext <= 16 && 16 % ext == 0;
        for (int r = 0; r < c->size; ++r)
            same = same && ((((uintptr_t)(src.p[r] + j.off * ext)) & 15) == ph);
        const int64_t lead = (int64_t)((16 - ph) & 15);
        j.head = (same && lead % (int64_t)ext == 0) ? (int)std::min<int64_t>(lead / (int64_t)ext, j.cnt) : -1;
        most = std::max(most, j.cnt);
    }
    const int64_t per = (int64_t)(16 / ext) * kXferThreads;
    int64_t blocks = (most + per - 1) / per;
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, std::max(1, c->max_blocks / jobs.n)));
    return record_hip(f(dim3((unsigned)blocks, (unsigned)jobs.n), src, dst, c->size, order, jobs, s),
                      "reduce launch");
}

// Bracket one phase launch with timing events when profiling.
static hipEvent_t prof_event(ompi_amd_comm_t *c) {
    if (!c->ev_free.empty()) {
        hipEvent_t e = c->ev_free.back();
        c->ev_free.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

template <typename F>
static int timed_phase(ompi_amd_comm_t *c, int phase, hipStream_t s, F &&launch) {
    if (!c->profile) return launch();
    hipEvent_t a = prof_event(c), b = prof_event(c);
    if (a) (void)hipEventRecord(a, s);
    const int rc = launch();
    if (b) (void)hipEventRecord(b, s);
    if (a && b) c->ev_phase[phase].emplace_back(a, b);
    return rc;
}

static int check_sticky(ompi_amd_comm_t *c) {
    const int e = __atomic_load_n(c->err_host, __ATOMIC_ACQUIRE);
    if (e != 0) {
        record_msg("collective device error %d (a peer did not reach a barrier within %lld ms)",
                   e, (long long)c->timeout_ms);
        return e;
    }
    return OMPI_AMD_SUCCESS;
}

#define TRY(x)                                   \
    do {                                         \
        int rc_ = (x);                           \
        if (rc_ != OMPI_AMD_SUCCESS) return rc_; \
    } while (0)

static bool in_place(const void *sbuf, const void *rbuf) {
    return sbuf == rbuf || sbuf == (const void *)1;
}

// Staged calls alternate between the two scratch halves, so a call never
// needs a trailing barrier: the next call that writes the same half comes
// after the following call's barrier, which every peer passes only once
// its reads of this half are done (stream order).  Every rank makes the
// same sequence of staged calls, so the halves agree.
struct stage_half {
    char *mine;
    ptr_set peers;
};
static stage_half next_half(ompi_amd_comm_t *c) {
    const size_t h = (size_t)(c->stage_seq++ & 1) * c->scratch_bytes;
    stage_half r;
    r.mine = c->scratch + h;
    for (int p = 0; p < kMaxRanks; ++p) r.peers.p[p] = c->peer_scratch.p[p] ? c->peer_scratch.p[p] + h : nullptr;
    return r;
}

// Fill one ring-order job per block in `blocks` (or every block).
static void ring_jobs(int64_t count, int n, red_jobs *jobs, int only_block) {
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    jobs->n = 0;
    for (int b = 0; b < n; ++b) {
        if (only_block >= 0 && b != only_block) continue;
        red_job &j = jobs->j[jobs->n++];
        j.off = block_off(b, split, early, late);
        j.cnt = block_cnt(b, split, early, late);
        j.off_dst = j.off;
        j.first = b;
        j.head = -1;
    }
}

}  // namespace ompi_amd

extern "C" {

int ompi_amd_comm_create(const char *name, int rank, int size, int device,
                         ompi_amd_comm_t **out) {
    if (!out || size < 1 || size > kMaxRanks || rank < 0 || rank >= size)
        return OMPI_AMD_ERR_BAD_PARAM;
    auto *c = new (std::nothrow) ompi_amd_comm;
    if (!c) return OMPI_AMD_ERR_BAD_PARAM;
    c->rank = rank;
    c->size = size;
    if (device < 0 && hipGetDevice(&device) != hipSuccess) {
        (void)hipGetLastError();
        delete c;
        return OMPI_AMD_ERR_HIP;
    }
    c->device = device;
    if (const char *t = getenv("OMPI_AMD_COLL_TIMEOUT_MS")) c->timeout_ms = atoll(t);
    int rc = set_dev(c);
    if (rc == OMPI_AMD_SUCCESS) rc = c->boot.attach(name, rank, size, 120.0);
    if (rc != OMPI_AMD_SUCCESS) { delete c; return rc; }
    // device resources: fine-grained flags, scratch, pinned error word
    c->scratch_bytes = std::max<size_t>(c->small_bytes, 4 << 20);  // per half
    hipError_t e = hipExtMallocWithFlags((void **)&c->flags, 4096, hipDeviceMallocUncached);
    if (e == hipSuccess) e = hipMemset(c->flags, 0, 4096);
    if (e == hipSuccess) e = hipMalloc((void **)&c->scratch, 2 * c->scratch_bytes);
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->err_host, 64, hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&c->err_dev, c->err_host, 0);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        rc = record_hip(e, "comm device resources");
        ompi_amd_comm_destroy(c);
        return rc;
    }
    *c->err_host = 0;
    ipc_blob mine{}, all[kMaxRanks];
    e = hipIpcGetMemHandle(&mine.flags, c->flags);
    if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.scratch, c->scratch);
    if (e != hipSuccess) {
        rc = record_hip(e, "hipIpcGetMemHandle (comm)");
        ompi_amd_comm_destroy(c);
        return rc;
    }
    rc = c->boot.allgather(&mine, all, sizeof(ipc_blob));
    for (int p = 0; rc == OMPI_AMD_SUCCESS && p < size; ++p) {
        if (p == rank) {
            c->peer_flags.p[p] = c->flags;
            c->peer_scratch.p[p] = c->scratch;
            continue;
        }
        void *f = nullptr, *s = nullptr;
        e = hipIpcOpenMemHandle(&f, all[p].flags, hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle(&s, all[p].scratch, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) { rc = record_hip(e, "hipIpcOpenMemHandle (comm)"); break; }
        c->opened[p][0] = f;
        c->opened[p][1] = s;
        c->peer_flags.p[p] = (uint64_t *)f;
        c->peer_scratch.p[p] = (const char *)s;
    }
    if (rc == OMPI_AMD_SUCCESS) rc = c->boot.barrier();  // all mapped before first use
    if (rc != OMPI_AMD_SUCCESS) {
        ompi_amd_comm_destroy(c);
        return rc;
    }
    *out = c;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_destroy(ompi_amd_comm_t *c) {
    if (!c) return OMPI_AMD_SUCCESS;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    (void)c->boot.barrier();  // nobody still reads our memory
    for (auto &x : c->imports) (void)hipIpcCloseMemHandle(x.base);
    for (int p = 0; p < kMaxRanks; ++p)
        for (int k = 0; k < 2; ++k)
            if (c->opened[p][k]) (void)hipIpcCloseMemHandle(c->opened[p][k]);
    (void)c->boot.barrier();
    if (c->flags) (void)hipFree(c->flags);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->err_host) (void)hipHostFree(c->err_host);
    for (int ph = 0; ph < 2; ++ph)
        for (auto &pr : c->ev_phase[ph]) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    for (auto e : c->ev_free) (void)hipEventDestroy(e);
    c->boot.detach();
    delete c;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_coll_block(size_t count, int size, int block, size_t *off, size_t *cnt) {
    if (size < 1 || block < 0 || block >= size || !off || !cnt) return OMPI_AMD_ERR_BAD_PARAM;
    int64_t split, early, late;
    blockcount((int64_t)count, size, &split, &early, &late);
    *off = (size_t)block_off(block, split, early, late);
    *cnt = (size_t)block_cnt(block, split, early, late);
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_coll_owner(int size, int block) {
    if (size < 1 || block < 0 || block >= size) return -1;
    return (block + size - 1) % size;
}

int ompi_amd_comm_phase_ms(ompi_amd_comm_t *c, int phase, double *total_ms, int *calls) {
    if (!c || phase < 0 || phase > 1 || !total_ms || !calls) return OMPI_AMD_ERR_BAD_PARAM;
    double tot = 0.0;
    int n = 0;
    for (auto &pr : c->ev_phase[phase]) {
        float ms = 0.f;
        if (hipEventSynchronize(pr.second) == hipSuccess &&
            hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
            tot += ms;
            ++n;
        }
        c->ev_free.push_back(pr.first);
        c->ev_free.push_back(pr.second);
    }
    c->ev_phase[phase].clear();
    *total_ms = tot;
    *calls = n;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_agree(ompi_amd_comm_t *c, int local_ok, int *all_ok) {
    if (!c || !all_ok) return OMPI_AMD_ERR_BAD_PARAM;
    int mine = local_ok ? 1 : 0, all[kMaxRanks];
    TRY(c->boot.allgather(&mine, all, sizeof(int)));
    int ok = 1;
    for (int p = 0; p < c->size; ++p) ok &= all[p];
    *all_ok = ok;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_sync(ompi_amd_comm_t *c, void *stream) {
    if (!c) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(set_dev(c));
    TRY(record_hip(hipStreamSynchronize(as_stream(stream)), "hipStreamSynchronize"));
    return check_sticky(c);
}

int ompi_amd_comm_rank(const ompi_amd_comm_t *c) { return c ? c->rank : -1; }
int ompi_amd_comm_size(const ompi_amd_comm_t *c) { return c ? c->size : -1; }

int ompi_amd_comm_error(const ompi_amd_comm_t *c) {
    return c ? __atomic_load_n(c->err_host, __ATOMIC_ACQUIRE) : OMPI_AMD_ERR_BAD_PARAM;
}

int ompi_amd_comm_set_param(ompi_amd_comm_t *c, const char *key, int64_t v) {
    if (!c || !key) return OMPI_AMD_ERR_BAD_PARAM;
    if (!strcmp(key, "small_bytes")) {
        if (v < 0) return OMPI_AMD_ERR_BAD_PARAM;
        c->small_bytes = std::min<size_t>((size_t)v, c->scratch_bytes);
    } else if (!strcmp(key, "zero_copy")) {
        c->zero_copy = v ? 1 : 0;
    } else if (!strcmp(key, "timeout_ms")) {
        if (v <= 0) return OMPI_AMD_ERR_BAD_PARAM;
        c->timeout_ms = v;
    } else if (!strcmp(key, "profile")) {
        c->profile = v ? 1 : 0;
    } else if (!strcmp(key, "blocks")) {
        if (v <= 0 || v > 65535) return OMPI_AMD_ERR_BAD_PARAM;
        c->max_blocks = (int)v;
    } else {
        record_msg("unknown coll param '%s'", key);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_allreduce(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                       int op, void *stream) {
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    if (count == 0) return OMPI_AMD_SUCCESS;  // allreduce.c:104
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const size_t ext = ompi_amd_type_extent(type);
    const size_t bytes = count * ext;
    const bool inplace = in_place(sbuf, rbuf);
    const void *src = inplace ? rbuf : sbuf;
    const int n = c->size;
    if (n == 1) {  // coll/self: copy (or nothing in place)
        if (inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, bytes, hipMemcpyDeviceToDevice, s), "copy");
    }
    // order of coll/tuned's fixed decision: < 10000 B recursive doubling
    const bool tree = type_size(type) * count < 10000 || count < (size_t)n;
    const int order = tree ? ORDER_TREE : ORDER_RING;
    red_jobs jobs;
    if (bytes <= c->small_bytes || !c->zero_copy || tree) {
        if (bytes > c->scratch_bytes) {
            record_msg("staged allreduce of %zu B exceeds the %zu B scratch", bytes, c->scratch_bytes);
            return OMPI_AMD_ERR_BAD_PARAM;
        }
        // staged one-shot: my contribution -> my scratch half, barrier,
        // every rank folds all blocks from all scratches (no trailing
        // barrier: see next_half)
        const stage_half sh = next_half(c);
        cp_jobs cj{};
        cj.n = 1;
        cj.j[0] = {(const char *)src, sh.mine, (int64_t)bytes};
        TRY(launch_copy(c, cj, s));
        TRY(launch_barrier(c, s));
        if (tree) {
            jobs.n = 1;
            jobs.j[0] = {0, (int64_t)count, 0, 0, -1};
        } else {
            ring_jobs((int64_t)count, n, &jobs, -1);
        }
        return launch_reduce(c, op, type, sh.peers, rbuf, order, jobs, s);
    }
    // zero-copy: reduce my ring block from every peer's sbuf, then gather
    ptr_set sp{}, rp{};
    TRY(exchange_bufs(c, src, rbuf, &sp, &rp));
    if (inplace) sp = rp;
    const int mine = (c->rank + 1) % n;  // the block the reference ring finishes here
    TRY(launch_barrier(c, s));
    ring_jobs((int64_t)count, n, &jobs, mine);
    TRY(timed_phase(c, 0, s, [&] { return launch_reduce(c, op, type, sp, rbuf, order, jobs, s); }));
    TRY(launch_barrier(c, s));
    int64_t split, early, late;
    blockcount((int64_t)count, n, &split, &early, &late);
    cp_jobs cj{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * (int64_t)ext;
        cj.j[cj.n++] = {rp.p[owner] + off, (char *)rbuf + off,
                        block_cnt(b, split, early, late) * (int64_t)ext};
    }
    TRY(timed_phase(c, 1, s, [&] { return launch_copy(c, cj, s); }));
    return launch_barrier(c, s);
}

int ompi_amd_reduce_scatter_block(ompi_amd_comm_t *c, const void *sbuf, void *rbuf,
                                  size_t rcount, int type, int op, void *stream) {
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    if (rcount == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const int n = c->size;
    const size_t ext = ompi_amd_type_extent(type);
    const size_t total = rcount * (size_t)n * ext;
    const bool inplace = in_place(sbuf, rbuf);
    const void *src = inplace ? rbuf : sbuf;  // in place: the input is rbuf (n*rcount)
    red_jobs jobs;
    jobs.n = 1;
    jobs.j[0] = {(int64_t)(rcount * (size_t)c->rank), (int64_t)rcount, 0, 0, -1};
    if (n == 1) {
        if (inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, rcount * ext, hipMemcpyDeviceToDevice, s), "copy");
    }
    if (total <= c->small_bytes || !c->zero_copy) {
        if (total > c->scratch_bytes) return OMPI_AMD_ERR_BAD_PARAM;
        const stage_half sh = next_half(c);
        cp_jobs cj{};
        cj.n = 1;
        cj.j[0] = {(const char *)src, sh.mine, (int64_t)total};
        TRY(launch_copy(c, cj, s));
        TRY(launch_barrier(c, s));
        return launch_reduce(c, op, type, sh.peers, rbuf, ORDER_LINEAR, jobs, s);
    }
    ptr_set sp{}, rp{};
    TRY(exchange_bufs(c, src, nullptr, &sp, &rp));
    TRY(launch_barrier(c, s));
    TRY(launch_reduce(c, op, type, sp, rbuf, ORDER_LINEAR, jobs, s));
    return launch_barrier(c, s);
}

int ompi_amd_allgather(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                       void *stream) {
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(check_sticky(c));
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const int n = c->size;
    const bool inplace = sbuf == (const void *)1 ||
                         sbuf == (const void *)((const char *)rbuf + (size_t)c->rank * bytes);
    char *my_slot = (char *)rbuf + (size_t)c->rank * bytes;
    cp_jobs cj{};
    if (bytes <= c->small_bytes || !c->zero_copy) {
        if (bytes > c->scratch_bytes) return OMPI_AMD_ERR_BAD_PARAM;
        const stage_half sh = next_half(c);
        cj.n = 1;
        cj.j[0] = {inplace ? my_slot : (const char *)sbuf, sh.mine, (int64_t)bytes};
        TRY(launch_copy(c, cj, s));
        TRY(launch_barrier(c, s));
        cj.n = 0;
        for (int p = 0; p < n; ++p) {
            if (p == c->rank && inplace) continue;
            cj.j[cj.n++] = {sh.peers.p[p], (char *)rbuf + (size_t)p * bytes, (int64_t)bytes};
        }
        return launch_copy(c, cj, s);
    }
    ptr_set sp{}, rp{};
    TRY(exchange_bufs(c, inplace ? my_slot : sbuf, nullptr, &sp, &rp));
    TRY(launch_barrier(c, s));
    for (int p = 0; p < n; ++p) {
        if (p == c->rank && inplace) continue;
        cj.j[cj.n++] = {sp.p[p], (char *)rbuf + (size_t)p * bytes, (int64_t)bytes};
    }
    TRY(launch_copy(c, cj, s));
    return launch_barrier(c, s);
}

int ompi_amd_bcast(ompi_amd_comm_t *c, void *buf, size_t bytes, int root, void *stream) {
    if (!c || !buf || root < 0 || root >= c->size) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(check_sticky(c));
    if (bytes == 0 || c->size == 1) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    cp_jobs cj{};
    if (bytes <= c->small_bytes || !c->zero_copy) {
        if (bytes > c->scratch_bytes) return OMPI_AMD_ERR_BAD_PARAM;
        const stage_half sh = next_half(c);
        if (c->rank == root) {
            cj.n = 1;
            cj.j[0] = {(const char *)buf, sh.mine, (int64_t)bytes};
            TRY(launch_copy(c, cj, s));
        }
        TRY(launch_barrier(c, s));
        if (c->rank != root) {
            cj.n = 1;
            cj.j[0] = {sh.peers.p[root], (char *)buf, (int64_t)bytes};
            TRY(launch_copy(c, cj, s));
        }
        return OMPI_AMD_SUCCESS;
    }
    ptr_set sp{}, rp{};
    TRY(exchange_bufs(c, c->rank == root ? buf : nullptr, nullptr, &sp, &rp));
    TRY(launch_barrier(c, s));
    if (c->rank != root) {
        cj.n = 1;
        cj.j[0] = {sp.p[root], (char *)buf, (int64_t)bytes};
        TRY(launch_copy(c, cj, s));
    }
    return launch_barrier(c, s);
}

}  // extern "C"
