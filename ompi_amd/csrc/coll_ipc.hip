// Device-buffer collectives over xGMI for gfx950: allreduce, reduce,
// reduce_scatter_block, scan, exscan, allgather, bcast
// (include/ompi_amd_coll.h).
//
// Reference path being replaced (coll/tuned + coll/basic over PML ob1 +
// btl/sm):
//   allreduce  coll_tuned_decision_fixed.c:45-89 ->
//              ring_segmented coll_base_allreduce.c:618-856 (1 MiB segments,
//              N-1 hops per segment, host bounce buffers, one op call per hop)
//   reduce     coll_tuned_decision_fixed.c:354-428 -> basic_linear / binomial
//              / pipeline / binary (coll_base_reduce.c:62-735)
//   rsb        coll_base_reduce_scatter_block.c:54-110 (tuned reduce to 0 +
//              scatter)
//   scan/exscan coll_base_scan.c:35-122, coll_base_exscan.c:35-107 (linear)
// Here each rank owns one block of the vector (allreduce: the ring block the
// reference finishes on it, COLL_BASE_COMPUTE_BLOCKCOUNT,
// coll_base_functions.h:425-431) and produces it in ONE pass that loads the
// block from every rank at once (all N-1 links busy) and folds the N values
// in registers in exactly the reference algorithm's operand order, so fp
// results are bit-identical to the reference:
//   ring        block b = x[b-1] (+) (x[b-2] (+) (... (x[b+1] (+) x[b])))
//   recursive doubling, basic_linear, pipeline chain, in-order binomial and
//   binary trees: see fold() (orders restated in oracle/coll_*oracle.c)
// with (+) the 2-buffer op rule f(out, in).
//
// Allreduce data movement (param "algorithm", all ranks alike):
//   0 pull       barrier, reduce my block pulling every rank's sbuf, barrier,
//                pull the N-1 other blocks from their owners, barrier
//   1 pull+push  barrier, reduce my block pulling every rank's sbuf and store
//                it into every rank's rbuf in the same pass, barrier
//   2 push       every rank stores block b of its sbuf into the owner's
//                landing slot (writes only over xGMI), barrier, the owner
//                reduces from local memory and stores the result into every
//                rank's rbuf, barrier
// Below `small_bytes` every rank stages its input in IPC scratch and folds
// all blocks itself (one barrier, no host rendezvous).
//
// Synchronisation: a monotonically increasing epoch per communicator.  A
// barrier is one 64-lane workgroup: lane p stores the epoch into peer p's
// flag slot [me] (system-scope atomic into fine-grained IPC memory) and
// polls its own slot [p] until the peer's epoch arrives, with a wall-clock
// bound (s_memrealtime) that sets a sticky error word instead of hanging.
// Kernel boundaries on the stream order the barrier after the producer of
// the data; every transfer workgroup opens with a system-scope acquire
// (buffer_inv sc0 sc1: drops stale lines of peer memory from this XCD's
// caches) and closes, after every wave has drained its stores, with a
// system-scope release (buffer_wbl2 sc0 sc1).
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <new>
#include <utility>
#include <vector>

#include "../../include/ompi_amd_coll.h"
#include "bootstrap.h"
#include "comm_internal.h"
#include "op_device.h"
#include "runtime.h"

namespace ompi_amd {

constexpr int kMaxRanks = OMPI_AMD_MAX_RANKS;
constexpr int kXferThreads = 256;

struct ptr_set { const char *p[kMaxRanks]; };
struct flag_set { uint64_t *p[kMaxRanks]; };

// Operand orders of the reference's reduction algorithms.  Sources are
// loaded in virtual-rank order v[j] = x[(first + j) % n].
enum order_t {
    ORDER_RING = 0,      // ring / ring_segmented block `first`; linear scan (first 0)
    ORDER_TREE = 1,      // recursive doubling (first 0)
    ORDER_CHAIN = 2,     // pipeline chain rooted at `first`; basic_linear = chain at 0, no swap
    ORDER_BINOMIAL = 3,  // in-order binomial tree rooted at `first`
    ORDER_BINARY = 4,    // binary tree rooted at `first`
    ORDER_HALVING = 5,   // recursive-halving reduce_scatter, owner tmp rank in flags >> 8
};
// The root passed MPI_IN_PLACE: its first combine is f(own, child)
// (coll_base_reduce.c:170-171, 196-199).
constexpr int FOLD_ROOT_INPLACE = 1;

// One reduction job: elements [off, off+cnt) of every source, combined in
// the call's order and written to dst + off_dst (element units).
struct red_job {
    int64_t off, cnt, off_dst;
    int first;  // virtual rank 0 (ring block b, tree root)
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

// The workgroup's acquire: lane 0 issues it (it invalidates the CU's L1 and
// the XCD's L2 for every wave of the CU), the barrier holds the other waves
// until it completed.  One per workgroup instead of one per wave: in a
// 1024-workgroup grid the 4 per workgroup cost measurable bandwidth
// (osc_ipc.hip's grid note).
__device__ __forceinline__ void acquire_once() {
    if (threadIdx.x == 0) sys_acquire();
    __syncthreads();
}

// Every storing wave drains its stores before the workgroup's single
// system-scope release (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ void xfer_epilogue() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sys_release();
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
// Fold v[0..n) (virtual-rank order) with the 2-buffer rule f(out, in).  All
// array indices are compile-time constants after unrolling; n, order and
// flags are wave-uniform.
template <typename T, int OP>
__device__ __forceinline__ T fold(const T (&v)[kMaxRanks], int n, int order, int flags) {
    using F = opfn<OP, false>;
    const bool swap = (flags & FOLD_ROOT_INPLACE) != 0;
    if (order == ORDER_RING) {
        // v[j] = x[(b + j) % n]; acc = x[b]; acc = f(x[b+j], acc)
        T acc = v[0];
#pragma unroll
        for (int j = 1; j < kMaxRanks; ++j)
            if (j < n) acc = F::template f<T>(v[j], acc);
        return acc;
    }
    if (order == ORDER_CHAIN) {
        // chain fanout 1 (coll_base_topo.c:588-600) under the generic reduce
        // (coll_base_reduce.c:206-215): node k's only child is k+1,
        // acc_k = f(acc_(k+1), x_k); basic_linear (:680-721) is the same
        // expression at first = 0.
        T acc = v[kMaxRanks - 1];
#pragma unroll
        for (int j = kMaxRanks - 1; j >= 0; --j) {
            if (j == n - 1) acc = v[j];
            else if (j < n - 1) acc = (j == 0 && swap) ? F::template f<T>(v[0], acc)
                                                       : F::template f<T>(acc, v[j]);
        }
        return acc;
    }
    if (order == ORDER_BINOMIAL) {
        // in-order binomial (coll_base_topo.c:402-458): vrank u's children
        // are u+1, u+2, u+4, ... while the bit is clear; first child:
        // acc = f(child, own), later ones acc = f(acc, child).
        T w[kMaxRanks];
#pragma unroll
        for (int i = 0; i < kMaxRanks; ++i) w[i] = v[i];
#pragma unroll
        for (int u = 0; u + 1 < kMaxRanks; u += 2)
            if (u + 1 < n) w[u] = (u == 0 && swap) ? F::template f<T>(w[0], w[1])
                                                   : F::template f<T>(w[u + 1], w[u]);
#pragma unroll
        for (int m = 2; m < kMaxRanks; m <<= 1) {
#pragma unroll
            for (int u = 0; u + m < kMaxRanks; u += 2 * m)
                if (u + m < n) w[u] = F::template f<T>(w[u], w[u + m]);
        }
        return w[0];
    }
    if (order == ORDER_BINARY) {
        // build_tree(2) (coll_base_topo.c:77-175): shifted rank s has
        // children s + d and s + 2d, d = largest power of two <= s + 1;
        // children have larger s, so descending s sees them finished.
        T w[kMaxRanks];
#pragma unroll
        for (int i = 0; i < kMaxRanks; ++i) w[i] = v[i];
#pragma unroll
        for (int s = kMaxRanks - 1; s >= 0; --s) {
            int d = 1;
            while (2 * d <= s + 1) d *= 2;
            const int c0 = s + d, c1 = s + 2 * d;
            if (c0 < kMaxRanks && c0 < n)
                w[s] = (s == 0 && swap) ? F::template f<T>(w[0], w[c0])
                                        : F::template f<T>(w[c0], w[s]);
            if (c1 < kMaxRanks && c1 < n) w[s] = F::template f<T>(w[s], w[c1]);
        }
        return w[0];
    }
    if (order == ORDER_HALVING) {
        // recursive-halving reduce_scatter (coll_base_reduce_scatter.c:
        // 203-345): the 2*remain lowest ranks fold pairwise (odd keeps:
        // f(odd, even)), then at every mask from the top the rank holding
        // the owner's half does f(mine, partner's).  tb = the owner's tmp
        // rank; holders at mask m agree with tb on bit m, and their
        // partners never do, so the update can run in place.
        int adj = 1;
        while (adj * 2 <= n) adj *= 2;
        const int remain = n - adj;
        const int tb = (flags >> 8) & 0xff;
        T w[kMaxRanks];
#pragma unroll
        for (int u = 0; u < kMaxRanks; ++u) {
            if (2 * u + 1 < kMaxRanks && u < remain) w[u] = F::template f<T>(v[2 * u + 1], v[2 * u]);
            else if (u < adj) w[u] = v[u + remain];
        }
#pragma unroll
        for (int m = kMaxRanks / 2; m >= 1; m >>= 1) {
            if (m < adj) {
#pragma unroll
                for (int u = 0; u < kMaxRanks; ++u)
                    if (u < adj && (u & m) == (tb & m)) w[u] = F::template f<T>(w[u], w[u ^ m]);
            }
        }
        T r = w[0];
#pragma unroll
        for (int u = 1; u < kMaxRanks; ++u)
            if (u == tb) r = w[u];
        return r;
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

// Gather v[j] for element index e of the sources in virtual-rank order.
template <typename T>
__device__ __forceinline__ void gather_scalar(T (&v)[kMaxRanks], const ptr_set &src, int n,
                                              int first, int64_t e) {
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) {
        if (j < n) {
            const int r = (first + j) % n;
            v[j] = reinterpret_cast<const T *>(src.p[r])[e];
        }
    }
}

// n sources (virtual ranks 0..n), result stored to dst.p[0 .. ndst): ndst =
// 1 is a plain reduce into one buffer; ndst = size is the fused push of the
// owner's block into every rank's rbuf (the host orders dst local first,
// then peers rank+1, rank+2, ... so concurrent owners spread their stores
// over the links).
template <typename T, int OP>
__global__ __launch_bounds__(kXferThreads) void reduce_kernel(ptr_set src, ptr_set dst, int ndst,
                                                              int n, int order, int flags,
                                                              red_jobs jobs) {
    acquire_once();
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
                const int r = (jb.first + j) % n;
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
            out.e[e] = fold<T, OP>(s, n, order, flags);
        }
#pragma unroll
        for (int k = 0; k < kMaxRanks; ++k)
            if (k < ndst)
                reinterpret_cast<u32x4 *>(reinterpret_cast<T *>(const_cast<char *>(dst.p[k])) +
                                          jb.off_dst + head)[i] = out.v;
    }
    // scalar head [0, head) and tail [head + nvec*E, cnt)
    const int64_t tail0 = head + nvec * E;
    const int64_t nscalar = head + (jb.cnt - tail0);
    for (int64_t k = tid; k < nscalar; k += gstride) {
        const int64_t e = k < head ? k : tail0 + (k - head);
        T s[kMaxRanks];
        gather_scalar<T>(s, src, n, jb.first, jb.off + e);
        const T r = fold<T, OP>(s, n, order, flags);
#pragma unroll
        for (int d = 0; d < kMaxRanks; ++d)
            if (d < ndst)
                store_elem<T>(reinterpret_cast<T *>(const_cast<char *>(dst.p[d])) + jb.off_dst + e,
                              r);
    }
    xfer_epilogue();
}

// ---------------------------------------------------------------- fused small allreduce
// One launch for small messages (param "fused_bytes"): every workgroup
// stages its slice of my input in my scratch half, signals the peers on its
// own flag row, waits for the same slice of every peer and folds it.
// Workgroup g depends only on the peers' workgroup g (same slice), so there
// is no grid-wide sync.  Flag slot [g * kMaxRanks + p] of rank r holds the
// last epoch peer p's workgroup g signalled to r (row 0 doubles as the
// barrier kernel's row; epochs only grow, so the users never collide).
constexpr int kFusedMaxGroups = 4096 / (int)sizeof(uint64_t) / kMaxRanks;  // 32 rows

struct fused_args {
    const char *src;
    char *dst, *mine;
    ptr_set peers;
    uint64_t *flags;
    flag_set peer_flags;
    int rank, n, order;
    int64_t count, split, early, late;
    uint64_t epoch, timeout_ticks;
    int *err;
};

template <typename T, int OP>
__global__ __launch_bounds__(kXferThreads) void fused_allreduce_kernel(fused_args a) {
    const int t = threadIdx.x;
    const int g = blockIdx.y * gridDim.x + blockIdx.x;
    int64_t off = 0, cnt = a.count;
    int first = 0;
    if (a.order == ORDER_RING) {  // grid row y = ring block y
        const int64_t b = blockIdx.y;
        off = b < a.split ? b * a.early : b * a.late + a.split;
        cnt = b < a.split ? a.early : a.late;
        first = (int)b;
    }
    const int64_t per = (cnt + gridDim.x - 1) / gridDim.x;
    const int64_t lo = off + min(cnt, per * (int64_t)blockIdx.x);
    const int64_t hi = off + min(cnt, per * (int64_t)(blockIdx.x + 1));
    const T *src = reinterpret_cast<const T *>(a.src);
    T *mine = reinterpret_cast<T *>(a.mine);
    for (int64_t e = lo + t; e < hi; e += kXferThreads) mine[e] = src[e];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) sys_release();
    __syncthreads();
    if (t < a.n && t != a.rank) {
        __hip_atomic_store(a.peer_flags.p[t] + g * kMaxRanks + a.rank, a.epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(a.flags + g * kMaxRanks + t, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                __hip_atomic_store(a.err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
    }
    __syncthreads();
    acquire_once();
    T *dst = reinterpret_cast<T *>(a.dst);
    for (int64_t e = lo + t; e < hi; e += kXferThreads) {
        T v[kMaxRanks];
        gather_scalar<T>(v, a.peers, a.n, first, e);
        store_elem<T>(dst + e, fold<T, OP>(v, a.n, a.order, 0));
    }
}

// ---------------------------------------------------------------- copy
// Byte copy with a peeled head so that the body runs 16 B (or 4 B) per
// lane whenever src and dst share their alignment phase.
__global__ __launch_bounds__(kXferThreads) void copy_kernel(cp_jobs jobs) {
    acquire_once();
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
    xfer_epilogue();
}

// ---------------------------------------------------------------- dispatch
using red_launch_fn = hipError_t (*)(dim3, const ptr_set &, const ptr_set &, int, int, int, int,
                                     const red_jobs &, hipStream_t);

template <int OP, int TYPE>
static hipError_t red_launch_slot(dim3 grid, const ptr_set &src, const ptr_set &dst, int ndst,
                                  int n, int order, int flags, const red_jobs &jobs,
                                  hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        using T = typename type_of<TYPE>::type;
        hipLaunchKernelGGL((reduce_kernel<T, OP>), grid, dim3(kXferThreads), 0, s, src, dst, ndst,
                           n, order, flags, jobs);
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

using fused_launch_fn = hipError_t (*)(dim3, const fused_args &, hipStream_t);

template <int OP, int TYPE>
static hipError_t fused_launch_slot(dim3 grid, const fused_args &a, hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        using T = typename type_of<TYPE>::type;
        hipLaunchKernelGGL((fused_allreduce_kernel<T, OP>), grid, dim3(kXferThreads), 0, s, a);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}
template <int OP, int... T>
static constexpr std::array<fused_launch_fn, OMPI_AMD_TYPE_COUNT> make_fused_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &fused_launch_slot<OP, T> : (fused_launch_fn) nullptr)...}};
}
template <int... O>
static constexpr std::array<std::array<fused_launch_fn, OMPI_AMD_TYPE_COUNT>, OMPI_AMD_OP_COUNT>
make_fused_table(std::integer_sequence<int, O...>) {
    return {{make_fused_row<O>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}
static const auto g_fused = make_fused_table(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});

// MPI type size (bytes of data) — the tuned decisions use it, not the
// extent (ompi_datatype_module.c:404-430: DOUBLE_INT size 12 / extent 16).
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

// The operand order of coll/tuned's reduce for a commutative op
// (coll_tuned_decision_fixed.c:354-428; msg = type size * count).
struct red_order { int order, first, flags; };
static red_order tuned_reduce_order(int n, size_t msg, size_t count, int root, bool root_inplace) {
    const double a1 = 0.6016 / 1024.0, b1 = 1.3496;
    const double a2 = 0.0410 / 1024.0, b2 = 9.7128;
    const double a3 = 0.0422 / 1024.0, b3 = 1.1614;
    const int fl = root_inplace ? FOLD_ROOT_INPLACE : 0;
    const double m = (double)msg;
    if (n < 8 && msg < 512) return {ORDER_CHAIN, 0, 0};  // basic_linear
    if ((n < 8 && msg < 20480) || msg < 2048 || count <= 1) return {ORDER_BINOMIAL, root, fl};
    if (n > a1 * m + b1) return {ORDER_BINOMIAL, root, fl};
    if (n > a2 * m + b2) return {ORDER_CHAIN, root, fl};  // pipeline, 1 KiB segments
    if (n > a3 * m + b3) return {ORDER_BINARY, root, fl};
    return {ORDER_CHAIN, root, fl};                      // pipeline, 32/64 KiB segments
}

// What each rank publishes per zero-copy call: its user buffers as
// (allocation handle, offset).
struct buf_desc {
    hipIpcMemHandle_t h;
    uint64_t off;
    uint64_t valid;
};
struct call_blob {
    buf_desc s, r;
    uint64_t flags;  // per-call rank flags (bit 0: MPI_IN_PLACE)
};

// The parameters a path decision reads, captured when a nonblocking call is
// posted so that its deferred launch takes the path every rank agreed on.
struct path_params {
    size_t small_bytes, fused_bytes;
    int zero_copy, algorithm;
};

// A nonblocking collective posted but not launched yet.  Device work must
// enter every rank's stream in the same order (the epoch barriers pair by
// count), so deferred calls launch strictly first-in first-out, and every
// blocking entry point launches the queue first.
struct pending_op {
    uint64_t ticket;  // rendezvous ticket of the handle swap (0: none)
    const void *sbuf;
    void *rbuf;
    size_t count;
    int type, op;
    hipStream_t stream;
    path_params pp;
    ompi_amd_request *req;
};

}  // namespace ompi_amd

using namespace ompi_amd;

// A nonblocking collective's completion (MPI_Request of MPI_Iallreduce).
struct ompi_amd_request {
    ompi_amd_comm_t *c = nullptr;
    hipEvent_t ev = nullptr;
    hipStream_t stream = nullptr;
    bool launched = false;  // its kernels are on `stream`
    bool recorded = false;  // `ev` recorded after them (lazily, at the first test / wait)
    int rc = OMPI_AMD_SUCCESS;
};

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
    char *land = nullptr;                 // grow-on-demand landing buffer (push
    size_t land_bytes = 0;                //   allreduce, large scan/exscan)
    ptr_set peer_land{};
    void *land_opened[kMaxRanks] = {};
    std::vector<void *> land_rejected;  // aliased landing candidates, freed at destroy
    int land_alias_retries = 0;
    int *err_host = nullptr, *err_dev = nullptr;
    uint64_t epoch = 0;
    // params
    size_t small_bytes = 1 << 20;
    size_t fused_bytes = 64 << 10;
    int zero_copy = 1;
    int64_t timeout_ms = 30000;
    int max_blocks = 1024;
    int algorithm = 0;
    // IPC caches
    struct exp_entry { void *base; size_t size; unsigned long long id; hipIpcMemHandle_t h; };
    struct imp_entry { int peer; hipIpcMemHandle_t h; void *base; uint64_t last_use; int pins; };
    std::vector<exp_entry> exports;
    std::vector<imp_entry> imports;
    uint64_t use_clock = 0;
    void *opened[kMaxRanks][2] = {};      // flags / scratch mappings of peers
    // per-phase kernel timing (param "profile"): event pairs per call
    int profile = 0;
    std::vector<hipEvent_t> ev_free;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_phase[2];
    // nonblocking calls not launched yet, and the swapped blobs of the one
    // being launched (exchange_bufs takes them instead of a rendezvous)
    std::deque<pending_op> pending;
    const call_blob *pre = nullptr;
    // point-to-point mailboxes (p2p.cpp)
    p2p_state *p2p = nullptr;
};

// A persistent allreduce (MPI_Allreduce_init, coll.h:349-352): buffers,
// path and peer mappings fixed at init, so a start enqueues device work
// only — no host rendezvous, no handle swap.
struct ompi_amd_plan {
    ompi_amd_comm_t *c = nullptr;
    const void *src = nullptr;
    void *rbuf = nullptr;
    int64_t count = 0;
    int op = 0, type = 0;
    int kind = 0;      // 0: small paths (as a plain call), 1 pull, 2 pull+push, 3 push
    ptr_set sp{}, rp{};
    void *bases[OMPI_AMD_MAX_RANKS][2] = {};  // pinned peer mappings
    // completion: recorded on the start's stream at the first test / wait
    // after a start (a later point in the stream, so never early; keeps an
    // event record out of the start itself)
    hipEvent_t done = nullptr;
    hipStream_t stream = nullptr;
    bool started = false, recorded = false;
};

namespace ompi_amd {

enum { ALG_PULL = 0, ALG_PULL_PUSH = 1, ALG_PUSH = 2, ALG_COUNT = 3 };

struct ipc_blob {
    hipIpcMemHandle_t flags, scratch;
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

// pin: the mapping is held by a persistent plan and never evicted until
// the plan releases it (unpin_import with the returned *base).
static int import_buf(ompi_amd_comm_t *c, int peer, const buf_desc &d, const char **out,
                      bool pin = false, void **base_out = nullptr) {
    *out = nullptr;
    if (base_out) *base_out = nullptr;
    if (!d.valid) return OMPI_AMD_SUCCESS;
    for (auto &x : c->imports) {
        if (x.peer == peer && memcmp(&x.h, &d.h, sizeof(d.h)) == 0) {
            x.last_use = ++c->use_clock;
            x.pins += pin ? 1 : 0;
            *out = (const char *)x.base + d.off;
            if (base_out) *base_out = x.base;
            return OMPI_AMD_SUCCESS;
        }
    }
    if (c->imports.size() >= 256) {  // evict the least recently used unpinned mapping
        auto it = c->imports.end();
        for (auto jt = c->imports.begin(); jt != c->imports.end(); ++jt)
            if (jt->pins == 0 && (it == c->imports.end() || jt->last_use < it->last_use)) it = jt;
        if (it != c->imports.end()) {
            (void)hipIpcCloseMemHandle(it->base);
            c->imports.erase(it);
        }
    }
    void *base = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&base, d.h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return record_hip(e, "hipIpcOpenMemHandle");
    c->imports.push_back({peer, d.h, base, ++c->use_clock, pin ? 1 : 0});
    *out = (const char *)base + d.off;
    if (base_out) *base_out = base;
    return OMPI_AMD_SUCCESS;
}

static void unpin_import(ompi_amd_comm_t *c, void *base) {
    for (auto &x : c->imports)
        if (x.base == base && x.pins > 0) {
            --x.pins;
            return;
        }
}

// Swap (sbuf, rbuf) descriptors with every peer and map theirs (either may
// be NULL: nothing is exported for it).
static int exchange_bufs(ompi_amd_comm_t *c, const void *sbuf, const void *rbuf, ptr_set *s,
                         ptr_set *r, uint64_t myflags = 0, uint64_t *allflags = nullptr,
                         bool pin = false, void *(*bases)[2] = nullptr) {
    call_blob mine{};
    mine.flags = myflags;
    int rc = export_buf(c, sbuf, &mine.s);
    if (rc == OMPI_AMD_SUCCESS) rc = export_buf(c, rbuf, &mine.r);
    if (rc != OMPI_AMD_SUCCESS) return rc;
    call_blob all[kMaxRanks];
    if (c->pre) {  // a deferred nonblocking call: swapped when it was posted
        memcpy(all, c->pre, sizeof(call_blob) * (size_t)c->size);
    } else {
        rc = c->boot.allgather(&mine, all, sizeof(call_blob));
        if (rc != OMPI_AMD_SUCCESS) return rc;
    }
    for (int p = 0; p < c->size; ++p) {
        if (allflags) allflags[p] = all[p].flags;
        if (p == c->rank) {
            s->p[p] = (const char *)sbuf;
            r->p[p] = (const char *)rbuf;
            continue;
        }
        void *b0 = nullptr, *b1 = nullptr;
        if ((rc = import_buf(c, p, all[p].s, &s->p[p], pin, &b0)) != OMPI_AMD_SUCCESS) return rc;
        if ((rc = import_buf(c, p, all[p].r, &r->p[p], pin, &b1)) != OMPI_AMD_SUCCESS) return rc;
        if (bases) {
            bases[p][0] = b0;
            bases[p][1] = b1;
        }
    }
    return OMPI_AMD_SUCCESS;
}

static void release_landing(ompi_amd_comm_t *c) {
    for (int p = 0; p < kMaxRanks; ++p) {
        if (c->land_opened[p]) (void)hipIpcCloseMemHandle(c->land_opened[p]);
        c->land_opened[p] = nullptr;
        c->peer_land.p[p] = nullptr;
    }
    if (c->land) (void)hipFree(c->land);
    c->land = nullptr;
    c->land_bytes = 0;
}

// Collective: every rank reaches it in the same call with the same `need`.
// Growing waits for all earlier work of every rank (no kernel may still
// touch the old buffers), then swaps handles of the new one.  The new buffer
// is allocated (and exported) while the old one is still alive, so it never
// reuses the old one's address range: on ROCm 7.2 an IPC export of a fresh
// allocation at a just-freed range failed with hipErrorInvalidValue (seen
// at 4 ranks, third growth).  Sizes grow geometrically, in 32 MiB steps.
static hipError_t alloc_exportable(size_t bytes, char **out, hipIpcMemHandle_t *h) {
    std::vector<void *> failed;
    hipError_t e = hipErrorInvalidValue;
    for (int attempt = 0; attempt < 3; ++attempt) {
        void *p = nullptr;
        e = hipMalloc(&p, bytes + (size_t)attempt * (2u << 20));
        if (e != hipSuccess) break;
        e = hipIpcGetMemHandle(h, p);
        if (e == hipSuccess) {
            *out = (char *)p;
            break;
        }
        (void)hipGetLastError();
        failed.push_back(p);  // keep it alive so the next try gets another range
    }
    for (void *p : failed) (void)hipFree(p);
    return e;
}

static uint64_t landing_token(int rank) {
    static std::atomic<uint64_t> serial{0};
    uint64_t x = ((uint64_t)getpid() << 32) ^ (++serial << 8) ^ (uint64_t)rank ^
                 (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    x ^= x >> 33;  // splitmix finaliser: spread the bits
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return x | 1;
}

static int ensure_landing(ompi_amd_comm_t *c, size_t need) {
    if (need <= c->land_bytes) return OMPI_AMD_SUCCESS;
    constexpr size_t kStep = 32u << 20, kTag = 64;  // the last kTag bytes hold the token
    const size_t want = std::max((need + kTag + kStep - 1) / kStep * kStep,
                                 c->land_bytes ? 2 * (c->land_bytes + kTag) : 0);
    int rc = record_hip(hipDeviceSynchronize(), "landing: drain");
    if (rc == OMPI_AMD_SUCCESS) rc = c->boot.barrier();
    if (rc != OMPI_AMD_SUCCESS) return rc;
    for (int p = 0; p < kMaxRanks; ++p) {
        if (c->land_opened[p]) (void)hipIpcCloseMemHandle(c->land_opened[p]);
        c->land_opened[p] = nullptr;
        c->peer_land.p[p] = nullptr;
    }
    // Every rank stamps a fresh token into its new buffer and every importer
    // reads it back through its mapping.  A mapping that shows another token
    // aliases an older allocation of that peer (seen on ROCm 7.2 when a new
    // buffer reuses a freed, previously exported address range): then all
    // ranks retry with new buffers, keeping the rejected ones alive so the
    // next ranges differ.
    bool first = true;
    for (int attempt = 0; attempt < 3; ++attempt) {
        struct { hipIpcMemHandle_t h; uint64_t token; int ok; } mine{}, all[kMaxRanks];
        char *fresh = nullptr;
        hipError_t e = alloc_exportable(want, &fresh, &mine.h);
        mine.token = landing_token(c->rank);
        if (e == hipSuccess)
            e = hipMemcpy(fresh + want - kTag, &mine.token, sizeof(mine.token),
                          hipMemcpyHostToDevice);
        mine.ok = e == hipSuccess;
        if (e != hipSuccess) record_hip(e, "landing buffer");
        rc = c->boot.allgather(&mine, all, sizeof(mine));  // also: nobody maps the old one now
        if (rc != OMPI_AMD_SUCCESS) {
            if (fresh) (void)hipFree(fresh);
            return rc;
        }
        if (first) {
            if (c->land) (void)hipFree(c->land);
            c->land = nullptr;
            c->land_bytes = 0;
            first = false;
        }
        bool ok = true, alias = false;
        for (int p = 0; p < c->size; ++p) ok = ok && all[p].ok;
        for (int p = 0; ok && p < c->size; ++p) {
            if (p == c->rank) continue;
            void *m = nullptr;
            e = hipIpcOpenMemHandle(&m, all[p].h, hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess) {
                record_hip(e, "hipIpcOpenMemHandle (landing)");
                ok = false;
                break;
            }
            c->land_opened[p] = m;
            uint64_t seen = 0;
            e = hipMemcpy(&seen, (char *)m + want - kTag, sizeof(seen), hipMemcpyDeviceToHost);
            if (e != hipSuccess || seen != all[p].token) {
                if (e != hipSuccess) record_hip(e, "landing token read");
                else record_msg("landing buffer of rank %d: the IPC mapping aliases an older "
                               "allocation (token %016llx, expected %016llx)", p,
                               (unsigned long long)seen, (unsigned long long)all[p].token);
                ok = false;
                alias = e == hipSuccess;
                break;
            }
        }
        int oks[kMaxRanks], flags = (ok ? 1 : 0) | (alias ? 2 : 0);
        rc = c->boot.allgather(&flags, oks, sizeof(int));
        if (rc != OMPI_AMD_SUCCESS) return rc;
        bool all_ok = true, any_alias = false;
        for (int p = 0; p < c->size; ++p) {
            all_ok = all_ok && (oks[p] & 1);
            any_alias = any_alias || (oks[p] & 2);
        }
        if (all_ok) {
            c->land = fresh;
            for (int p = 0; p < c->size; ++p)
                c->peer_land.p[p] = p == c->rank ? c->land : (const char *)c->land_opened[p];
            c->land_bytes = want - kTag;
            return OMPI_AMD_SUCCESS;
        }
        (void)c->boot.barrier();  // nobody reads the rejected buffers any more
        for (int p = 0; p < kMaxRanks; ++p) {
            if (c->land_opened[p]) (void)hipIpcCloseMemHandle(c->land_opened[p]);
            c->land_opened[p] = nullptr;
        }
        if (!any_alias) {
            if (fresh) (void)hipFree(fresh);
            return OMPI_AMD_ERR_HIP;
        }
        if (fresh) c->land_rejected.push_back(fresh);
        ++c->land_alias_retries;
        if (alias) fprintf(stderr, "ompi_amd[%d]: %s; retrying\n", c->rank, ompi_amd_last_error());
    }
    return OMPI_AMD_ERR_HIP;
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

static ptr_set one_ptr(const void *p) {
    ptr_set r{};
    r.p[0] = (const char *)p;
    return r;
}

// Every rank's buffer in push order: mine first, then rank+1, rank+2, ...
static ptr_set push_order(const ompi_amd_comm_t *c, const ptr_set &bufs) {
    ptr_set r{};
    for (int k = 0; k < c->size; ++k) r.p[k] = bufs.p[(c->rank + k) % c->size];
    return r;
}

// Reduce `nsrc` sources (ranks 0..nsrc of src) in `order`, store to the
// ndst buffers of dst.
static int launch_reduce(ompi_amd_comm_t *c, int op, int type, const ptr_set &src, int nsrc,
                         const ptr_set &dst, int ndst, int order, int flags, red_jobs jobs,
                         hipStream_t s) {
    red_launch_fn f = g_red[op][type];
    if (!f) return OMPI_AMD_ERR_UNSUPPORTED;
    if (jobs.n == 0 || nsrc < 1) return OMPI_AMD_SUCCESS;
    const size_t ext = ompi_amd_type_extent(type);
    int64_t most = 0;
    for (int i = 0; i < jobs.n; ++i) {
        red_job &j = jobs.j[i];
        // every source and dst must sit at the same phase mod 16 B, and that
        // phase must be a whole number of elements from 16-B alignment
        const uintptr_t ph = (uintptr_t)(dst.p[0] + j.off_dst * ext) & 15;
        bool same = ext <= 16 && 16 % ext == 0;
        for (int r = 0; r < nsrc; ++r)
            same = same && ((((uintptr_t)(src.p[r] + j.off * ext)) & 15) == ph);
        for (int d = 1; d < ndst; ++d)
            same = same && ((((uintptr_t)(dst.p[d] + j.off_dst * ext)) & 15) == ph);
        const int64_t lead = (int64_t)((16 - ph) & 15);
        j.head = (same && lead % (int64_t)ext == 0) ? (int)std::min<int64_t>(lead / (int64_t)ext, j.cnt) : -1;
        most = std::max(most, j.cnt);
    }
    if (most == 0) return OMPI_AMD_SUCCESS;
    const int64_t per = (int64_t)(16 / ext) * kXferThreads;
    int64_t blocks = (most + per - 1) / per;
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, std::max(1, c->max_blocks / jobs.n)));
    return record_hip(f(dim3((unsigned)blocks, (unsigned)jobs.n), src, dst, ndst, nsrc, order,
                        flags, jobs, s),
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

// Fill one ring-order job per block (or only `only_block`).
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

static int stage_in(ompi_amd_comm_t *c, const void *src, size_t bytes, stage_half *sh,
                    hipStream_t s) {
    if (bytes > c->scratch_bytes) {
        record_msg("staged collective of %zu B exceeds the %zu B scratch", bytes, c->scratch_bytes);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    *sh = next_half(c);
    cp_jobs cj{};
    cj.n = 1;
    cj.j[0] = {(const char *)src, sh->mine, (int64_t)bytes};
    TRY(launch_copy(c, cj, s));
    return launch_barrier(c, s);
}

// ---- large allreduce, three data-movement schemes (header comment) ----
// ---- small allreduce: one fused launch (flags per workgroup) ----
static int allreduce_fused(ompi_amd_comm_t *c, const void *src, void *rbuf, int64_t count,
                           int op, int type, bool tree, hipStream_t s) {
    fused_launch_fn f = g_fused[op][type];
    if (!f) return OMPI_AMD_ERR_UNSUPPORTED;
    const int n = c->size;
    const stage_half sh = next_half(c);
    fused_args a{};
    a.src = (const char *)src;
    a.dst = (char *)rbuf;
    a.mine = sh.mine;
    a.peers = sh.peers;
    a.flags = c->flags;
    a.peer_flags = c->peer_flags;
    a.rank = c->rank;
    a.n = n;
    a.order = tree ? ORDER_TREE : ORDER_RING;
    a.count = count;
    blockcount(count, n, &a.split, &a.early, &a.late);
    a.epoch = ++c->epoch;
    a.timeout_ticks = (uint64_t)c->timeout_ms * 100000ull;  // s_memrealtime: 100 MHz
    a.err = c->err_dev;
    const int rows = tree ? 1 : n;
    const int64_t most = tree ? count : a.early;
    const int64_t cols = std::max<int64_t>(
        1, std::min<int64_t>((most + 4 * kXferThreads - 1) / (4 * kXferThreads),
                             kFusedMaxGroups / rows));
    return record_hip(f(dim3((unsigned)cols, (unsigned)rows), a, s), "fused allreduce launch");
}

// ---- medium allreduce, staged two-shot: my input -> my scratch, barrier,
// my ring block folded from every scratch into my rbuf and into a result
// area of my scratch, barrier, the other blocks pulled from their owners'
// result areas.  No host rendezvous; no trailing barrier (next_half).
static size_t two_shot_result_off(size_t bytes) { return (bytes + 255) & ~(size_t)255; }

static bool two_shot_fits(const ompi_amd_comm_t *c, int64_t count, size_t ext) {
    int64_t split, early, late;
    blockcount(count, c->size, &split, &early, &late);
    return two_shot_result_off((size_t)count * ext) + (size_t)early * ext + 16 <= c->scratch_bytes;
}

static int allreduce_staged_two_shot(ompi_amd_comm_t *c, const void *src, void *rbuf,
                                     int64_t count, int op, int type, hipStream_t s) {
    const int n = c->size, mine = (c->rank + 1) % n;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    const size_t res = two_shot_result_off((size_t)count * ext);
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    stage_half sh;
    TRY(stage_in(c, src, (size_t)(count * ext), &sh, s));
    const int64_t offm = block_off(mine, split, early, late) * ext;
    ptr_set dst{};
    dst.p[0] = (const char *)rbuf;
    dst.p[1] = sh.mine + res + (offm & 15) - offm;
    red_jobs jobs;
    ring_jobs(count, n, &jobs, mine);
    TRY(launch_reduce(c, op, type, sh.peers, n, dst, 2, ORDER_RING, 0, jobs, s));
    TRY(launch_barrier(c, s));
    cp_jobs cj{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * ext;
        cj.j[cj.n++] = {sh.peers.p[owner] + res + (off & 15), (char *)rbuf + off,
                        block_cnt(b, split, early, late) * ext};
    }
    return launch_copy(c, cj, s);
}

// sp / rp: every rank's input and rbuf as this rank maps them (sp = rp in
// place); push needs rp only, and the landing buffer sized by push_slot.
static int allreduce_pull(ompi_amd_comm_t *c, const ptr_set &sp, const ptr_set &rp, void *rbuf,
                          int64_t count, int op, int type, hipStream_t s) {
    const int n = c->size, mine = (c->rank + 1) % n;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    TRY(launch_barrier(c, s));
    red_jobs jobs;
    ring_jobs(count, n, &jobs, mine);
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, sp, n, one_ptr(rbuf), 1, ORDER_RING, 0, jobs, s);
    }));
    TRY(launch_barrier(c, s));
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    cp_jobs cj{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * ext;
        cj.j[cj.n++] = {rp.p[owner] + off, (char *)rbuf + off, block_cnt(b, split, early, late) * ext};
    }
    TRY(timed_phase(c, 1, s, [&] { return launch_copy(c, cj, s); }));
    return launch_barrier(c, s);
}

static int allreduce_pull_push(ompi_amd_comm_t *c, const ptr_set &sp, const ptr_set &rp,
                               int64_t count, int op, int type, hipStream_t s) {
    // in place, sp = rp: only the owner of a block touches it
    const int n = c->size, mine = (c->rank + 1) % n;
    TRY(launch_barrier(c, s));
    red_jobs jobs;
    ring_jobs(count, n, &jobs, mine);
    const ptr_set dsts = push_order(c, rp);
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, sp, n, dsts, n, ORDER_RING, 0, jobs, s);
    }));
    return launch_barrier(c, s);
}

// slot r of the owner's landing buffer receives rank r's copy of the
// owner's block, at the block's own phase mod 16 B
static size_t push_slot(int64_t count, int n, int type) {
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    return ((size_t)(early * (int64_t)ompi_amd_type_extent(type)) + 16 + 255) & ~(size_t)255;
}

static int allreduce_push(ompi_amd_comm_t *c, const void *src, const ptr_set &rp, int64_t count,
                          int op, int type, hipStream_t s) {
    const int n = c->size, mine = (c->rank + 1) % n;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    const size_t slot = push_slot(count, n, type);
    cp_jobs cj{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * ext;
        char *dst = const_cast<char *>(c->peer_land.p[owner]) + (size_t)c->rank * slot + (off & 15);
        cj.j[cj.n++] = {(const char *)src + off, dst, block_cnt(b, split, early, late) * ext};
    }
    // the owner's previous reads of its landing ended before the previous
    // push call's trailing barrier, so the scatter needs no leading one
    TRY(timed_phase(c, 1, s, [&] { return launch_copy(c, cj, s); }));
    TRY(launch_barrier(c, s));
    const int64_t offm = block_off(mine, split, early, late) * ext;
    ptr_set srcs{};
    for (int r = 0; r < n; ++r)
        srcs.p[r] = (r == c->rank) ? (const char *)src
                                   : c->land + (size_t)r * slot + (offm & 15) - offm;
    red_jobs jobs;
    ring_jobs(count, n, &jobs, mine);
    const ptr_set dsts = push_order(c, rp);
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, srcs, n, dsts, n, ORDER_RING, 0, jobs, s);
    }));
    return launch_barrier(c, s);
}

// reduce_scatter_block / reduce_scatter: my block [off, off + cnt) of the
// full vector folded from every rank's input into rbuf[0, cnt).
// Staged: inputs in the scratch halves.  Zero-copy: peers' inputs read in
// place; a rank that passed MPI_IN_PLACE must not overwrite its rbuf (a
// peer may still read its own block there), so every rank learns the
// in-place flags with the handle swap and in-place ranks fold into their
// landing buffer and copy after the trailing barrier.
static int reduce_my_block(ompi_amd_comm_t *c, const void *src, void *rbuf, size_t total_bytes,
                           int64_t off, int64_t cnt, int64_t max_cnt, int op, int type,
                           red_order ro, bool inplace, hipStream_t s) {
    red_jobs jobs;
    jobs.n = 1;
    jobs.j[0] = {off, cnt, 0, ro.first, -1};
    const int n = c->size;
    const size_t ext = ompi_amd_type_extent(type);
    if (total_bytes <= c->small_bytes || !c->zero_copy) {
        stage_half sh;
        TRY(stage_in(c, src, total_bytes, &sh, s));
        return launch_reduce(c, op, type, sh.peers, n, one_ptr(rbuf), 1, ro.order, ro.flags, jobs, s);
    }
    ptr_set sp{}, rp{};
    uint64_t fl[kMaxRanks] = {};
    TRY(exchange_bufs(c, src, nullptr, &sp, &rp, inplace ? 1 : 0, fl));
    bool any_inplace = false;
    for (int p = 0; p < n; ++p) any_inplace = any_inplace || (fl[p] & 1);
    if (any_inplace)  // collective: every rank sees the same flags and max_cnt
        TRY(ensure_landing(c, (size_t)max_cnt * ext + 256));
    TRY(launch_barrier(c, s));
    void *dst = inplace ? (void *)c->land : rbuf;
    TRY(launch_reduce(c, op, type, sp, n, one_ptr(dst), 1, ro.order, ro.flags, jobs, s));
    TRY(launch_barrier(c, s));
    if (inplace && cnt > 0)
        return record_hip(hipMemcpyAsync(rbuf, c->land, (size_t)cnt * ext, hipMemcpyDeviceToDevice, s),
                          "in-place result copy");
    return OMPI_AMD_SUCCESS;
}

// scan (exclusive = false) / exscan: rank r folds ranks 0..r (0..r-1) in
// the linear scan's order, which is the ring fold at first = 0.
static int scan_common(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                       int op, void *stream, bool exclusive) {
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    if (count == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const size_t bytes = count * ompi_amd_type_extent(type);
    const bool inplace = in_place(sbuf, rbuf);
    const void *src = inplace ? rbuf : sbuf;
    const int nsrc = exclusive ? c->rank : c->rank + 1;
    red_jobs jobs;
    jobs.n = 1;
    jobs.j[0] = {0, (int64_t)count, 0, 0, -1};
    if (c->size == 1) {
        if (exclusive || inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, bytes, hipMemcpyDeviceToDevice, s), "copy");
    }
    if (bytes <= c->small_bytes || !c->zero_copy) {
        stage_half sh;
        TRY(stage_in(c, src, bytes, &sh, s));
        return launch_reduce(c, op, type, sh.peers, nsrc, one_ptr(rbuf), 1, ORDER_RING, 0, jobs, s);
    }
    // large: inputs go through the landing buffers (a peer may still read
    // my input while I write my result in place), then one fold per rank
    TRY(ensure_landing(c, bytes + 256));
    cp_jobs cj{};
    cj.n = 1;
    cj.j[0] = {(const char *)src, c->land, (int64_t)bytes};
    TRY(launch_copy(c, cj, s));
    TRY(launch_barrier(c, s));
    TRY(launch_reduce(c, op, type, c->peer_land, nsrc, one_ptr(rbuf), 1, ORDER_RING, 0, jobs, s));
    return launch_barrier(c, s);
}

}  // namespace ompi_amd

static path_params params_of(const ompi_amd_comm_t *c) {
    return {c->small_bytes, c->fused_bytes, c->zero_copy, c->algorithm};
}

// Whether an allreduce of `count` elements takes a zero-copy path (and so
// swaps buffer handles): the complement of the fused / staged conditions of
// allreduce_impl.
static bool allreduce_swaps(const ompi_amd_comm_t *c, const path_params &pp, size_t count,
                            int type) {
    const int n = c->size;
    if (n == 1 || count == 0) return false;
    const size_t bytes = count * ompi_amd_type_extent(type);
    const bool tree = type_size(type) * count < 10000 || count < (size_t)n;
    if (bytes <= pp.fused_bytes && bytes <= c->scratch_bytes) return false;
    return !(bytes <= pp.small_bytes || !pp.zero_copy || tree);
}

static int allreduce_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                          int op, hipStream_t s, const path_params &pp);

// Launch deferred nonblocking calls in posting order, each once every rank
// has posted its handle-swap half; block = wait for them (the blocking entry
// points do, so their device work follows the deferred calls' on every rank).
static int progress(ompi_amd_comm_t *c, bool block) {
    while (!c->pending.empty()) {
        pending_op o = c->pending.front();
        call_blob all[kMaxRanks];
        int rc = OMPI_AMD_SUCCESS;
        if (o.ticket) {
            bool ready = false;
            rc = c->boot.test(o.ticket, all, sizeof(call_blob), block, &ready);
            if (rc == OMPI_AMD_SUCCESS && !ready) return OMPI_AMD_SUCCESS;
        }
        c->pending.pop_front();
        if (rc == OMPI_AMD_SUCCESS) {
            c->pre = o.ticket ? all : nullptr;
            rc = allreduce_impl(c, o.sbuf, o.rbuf, o.count, o.type, o.op, o.stream, o.pp);
            c->pre = nullptr;
        }
        o.req->stream = o.stream;
        o.req->rc = rc;
        o.req->launched = true;
        if (rc != OMPI_AMD_SUCCESS) return rc;
    }
    return OMPI_AMD_SUCCESS;
}

static int drain(ompi_amd_comm_t *c) {
    return c->pending.empty() ? OMPI_AMD_SUCCESS : progress(c, true);
}

static int allreduce_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                          int op, hipStream_t s, const path_params &pp) {
    if (count == 0) return OMPI_AMD_SUCCESS;  // allreduce.c:104
    TRY(set_dev(c));
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
    if (bytes <= pp.fused_bytes && bytes <= c->scratch_bytes)
        return allreduce_fused(c, src, rbuf, (int64_t)count, op, type, tree, s);
    if (!tree && (bytes <= pp.small_bytes || !pp.zero_copy) &&
        two_shot_fits(c, (int64_t)count, ext))
        return allreduce_staged_two_shot(c, src, rbuf, (int64_t)count, op, type, s);
    if (bytes <= pp.small_bytes || !pp.zero_copy || tree) {
        // staged one-shot: my contribution -> my scratch half, barrier,
        // every rank folds all blocks from all scratches (no trailing
        // barrier: see next_half)
        stage_half sh;
        TRY(stage_in(c, src, bytes, &sh, s));
        red_jobs jobs;
        if (tree) {
            jobs.n = 1;
            jobs.j[0] = {0, (int64_t)count, 0, 0, -1};
        } else {
            ring_jobs((int64_t)count, n, &jobs, -1);
        }
        return launch_reduce(c, op, type, sh.peers, n, one_ptr(rbuf), 1,
                             tree ? ORDER_TREE : ORDER_RING, 0, jobs, s);
    }
    ptr_set sp{}, rp{};
    if (pp.algorithm == ALG_PUSH) {
        TRY(ensure_landing(c, push_slot((int64_t)count, n, type) * (size_t)n));
        TRY(exchange_bufs(c, nullptr, rbuf, &sp, &rp));
        return allreduce_push(c, src, rp, (int64_t)count, op, type, s);
    }
    TRY(exchange_bufs(c, src, rbuf, &sp, &rp));
    if (inplace) sp = rp;
    if (pp.algorithm == ALG_PULL_PUSH)
        return allreduce_pull_push(c, sp, rp, (int64_t)count, op, type, s);
    return allreduce_pull(c, sp, rp, rbuf, (int64_t)count, op, type, s);
}

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
    if (const char *a = getenv("OMPI_AMD_COLL_ALGORITHM")) {
        const int v = atoi(a);
        if (v >= 0 && v < ALG_COUNT) c->algorithm = v;
    }
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
    if (rank == 0) rc = p2p_create(c, name, rank, size, 0, &c->p2p);
    if (rc == OMPI_AMD_SUCCESS) rc = c->boot.allgather(&mine, all, sizeof(ipc_blob));
    if (rc == OMPI_AMD_SUCCESS && rank != 0) rc = p2p_create(c, name, rank, size, 1, &c->p2p);
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
    if (rank == 0 && c->p2p) p2p_unlink(c->p2p);  // every rank has it mapped
    *out = c;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_destroy(ompi_amd_comm_t *c) {
    if (!c) return OMPI_AMD_SUCCESS;
    (void)hipSetDevice(c->device);
    (void)drain(c);  // deferred nonblocking calls every peer will also launch
    (void)hipDeviceSynchronize();
    (void)c->boot.barrier();  // nobody still reads our memory
    for (auto &x : c->imports) (void)hipIpcCloseMemHandle(x.base);
    for (int p = 0; p < kMaxRanks; ++p) {
        for (int k = 0; k < 2; ++k)
            if (c->opened[p][k]) (void)hipIpcCloseMemHandle(c->opened[p][k]);
        if (c->land_opened[p]) (void)hipIpcCloseMemHandle(c->land_opened[p]);
        c->land_opened[p] = nullptr;
    }
    (void)c->boot.barrier();
    if (c->flags) (void)hipFree(c->flags);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->land) (void)hipFree(c->land);
    for (void *p : c->land_rejected) (void)hipFree(p);
    if (c->err_host) (void)hipHostFree(c->err_host);
    for (int ph = 0; ph < 2; ++ph)
        for (auto &pr : c->ev_phase[ph]) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    for (auto e : c->ev_free) (void)hipEventDestroy(e);
    if (c->p2p) p2p_destroy(c->p2p);
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

int ompi_amd_coll_reduce_order(int size, size_t msg_bytes, size_t count, int root,
                               int root_inplace, int *order, int *first) {
    if (size < 1 || root < 0 || root >= size || !order || !first) return OMPI_AMD_ERR_BAD_PARAM;
    const red_order ro = tuned_reduce_order(size, msg_bytes, count, root, root_inplace != 0);
    *order = ro.order;
    *first = ro.first;
    return OMPI_AMD_SUCCESS;
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
    TRY(drain(c));
    TRY(c->boot.allgather(&mine, all, sizeof(int)));
    int ok = 1;
    for (int p = 0; p < c->size; ++p) ok &= all[p];
    *all_ok = ok;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_sync(ompi_amd_comm_t *c, void *stream) {
    if (!c) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(set_dev(c));
    TRY(drain(c));
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
    } else if (!strcmp(key, "fused_bytes")) {
        if (v < 0) return OMPI_AMD_ERR_BAD_PARAM;
        c->fused_bytes = std::min<size_t>((size_t)v, c->scratch_bytes);
    } else if (!strcmp(key, "algorithm")) {
        if (v < 0 || v >= ALG_COUNT) return OMPI_AMD_ERR_BAD_PARAM;
        c->algorithm = (int)v;
    } else {
        record_msg("unknown coll param '%s'", key);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_get_param(const ompi_amd_comm_t *c, const char *key, int64_t *v) {
    if (!c || !key || !v) return OMPI_AMD_ERR_BAD_PARAM;
    if (!strcmp(key, "small_bytes")) *v = (int64_t)c->small_bytes;
    else if (!strcmp(key, "zero_copy")) *v = c->zero_copy;
    else if (!strcmp(key, "timeout_ms")) *v = (int64_t)c->timeout_ms;
    else if (!strcmp(key, "profile")) *v = c->profile;
    else if (!strcmp(key, "blocks")) *v = c->max_blocks;
    else if (!strcmp(key, "fused_bytes")) *v = (int64_t)c->fused_bytes;
    else if (!strcmp(key, "algorithm")) *v = c->algorithm;
    else if (!strcmp(key, "landing_bytes")) *v = (int64_t)c->land_bytes;
    else if (!strcmp(key, "landing_alias_retries")) *v = c->land_alias_retries;
    else if (!strcmp(key, "imports")) *v = (int64_t)c->imports.size();
    else {
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
    TRY(drain(c));
    return allreduce_impl(c, sbuf, rbuf, count, type, op, as_stream(stream), params_of(c));
}

int ompi_amd_iallreduce(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                        int op, void *stream, ompi_amd_request_t **out) {
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(set_dev(c));
    auto *req = new (std::nothrow) ompi_amd_request;
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    req->c = c;
    int rc = record_hip(hipEventCreateWithFlags(&req->ev, hipEventDisableTiming), "request event");
    if (rc != OMPI_AMD_SUCCESS) {
        delete req;
        return rc;
    }
    const path_params pp = params_of(c);
    const bool inplace = in_place(sbuf, rbuf);
    pending_op o{0, inplace ? rbuf : sbuf, rbuf, count, type, op, as_stream(stream), pp, req};
    if (allreduce_swaps(c, pp, count, type)) {
        // post this rank's half of the handle swap now; the launch waits for
        // the peers' halves (progress / the next collective call)
        const bool push = pp.algorithm == ALG_PUSH;
        if (push) {
            const size_t need = push_slot((int64_t)count, c->size, type) * (size_t)c->size;
            if (need > c->land_bytes) {  // collective growth: every rank decides alike
                rc = drain(c);
                if (rc == OMPI_AMD_SUCCESS) rc = ensure_landing(c, need);
            }
        }
        call_blob mine{};
        if (rc == OMPI_AMD_SUCCESS && !push) rc = export_buf(c, o.sbuf, &mine.s);
        if (rc == OMPI_AMD_SUCCESS) rc = export_buf(c, rbuf, &mine.r);
        if (rc == OMPI_AMD_SUCCESS) rc = c->boot.post(&mine, sizeof(mine), &o.ticket);
        if (rc != OMPI_AMD_SUCCESS) {
            (void)hipEventDestroy(req->ev);
            delete req;
            return rc;
        }
    }
    c->pending.push_back(o);
    *out = req;
    return progress(c, false);
}

int ompi_amd_reduce(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                    int op, int root, void *stream) {
    if (!c || root < 0 || root >= c->size || (c->rank == root && !rbuf))
        return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    if (count == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const int n = c->size;
    const size_t bytes = count * ompi_amd_type_extent(type);
    const bool root_inplace = c->rank == root && in_place(sbuf, rbuf);
    const void *src = root_inplace ? rbuf : sbuf;
    if (!src) return OMPI_AMD_ERR_BAD_PARAM;
    if (n == 1) {
        if (root_inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, bytes, hipMemcpyDeviceToDevice, s), "copy");
    }
    // the in-place flag only changes the root's first combine; every rank
    // must fold the same expression, so the root's choice is made known
    int flag = root_inplace ? 1 : 0, flags_all[kMaxRanks];
    TRY(c->boot.allgather(&flag, flags_all, sizeof(int)));
    const red_order ro = tuned_reduce_order(n, type_size(type) * count, count, root,
                                            flags_all[root] != 0);
    red_jobs jobs;
    if (bytes <= c->small_bytes || !c->zero_copy) {
        // staged: everyone stages, the root folds everything
        stage_half sh;
        TRY(stage_in(c, src, bytes, &sh, s));
        if (c->rank != root) return OMPI_AMD_SUCCESS;
        jobs.n = 1;
        jobs.j[0] = {0, (int64_t)count, 0, ro.first, -1};
        return launch_reduce(c, op, type, sh.peers, n, one_ptr(rbuf), 1, ro.order, ro.flags, jobs, s);
    }
    // zero-copy: every rank folds one block of the vector from every
    // rank's sbuf and stores it straight into the root's rbuf
    ptr_set sp{}, rp{};
    TRY(exchange_bufs(c, src, c->rank == root ? rbuf : nullptr, &sp, &rp));
    TRY(launch_barrier(c, s));
    int64_t split, early, late;
    blockcount((int64_t)count, n, &split, &early, &late);
    jobs.n = 1;
    jobs.j[0].off = block_off(c->rank, split, early, late);
    jobs.j[0].cnt = block_cnt(c->rank, split, early, late);
    jobs.j[0].off_dst = jobs.j[0].off;
    jobs.j[0].first = ro.first;
    jobs.j[0].head = -1;
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, sp, n, one_ptr(rp.p[root]), 1, ro.order, ro.flags, jobs, s);
    }));
    return launch_barrier(c, s);
}

int ompi_amd_reduce_scatter_block(ompi_amd_comm_t *c, const void *sbuf, void *rbuf,
                                  size_t rcount, int type, int op, void *stream) {
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    if (rcount == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const int n = c->size;
    const size_t ext = ompi_amd_type_extent(type);
    const size_t total = rcount * (size_t)n * ext;
    const bool inplace = in_place(sbuf, rbuf);
    const void *src = inplace ? rbuf : sbuf;  // in place: the input is rbuf (n*rcount)
    if (n == 1) {
        if (inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, rcount * ext, hipMemcpyDeviceToDevice, s), "copy");
    }
    // basic_linear rsb = tuned reduce of the whole vector to rank 0 (never
    // in place at that level) + scatter: my block folds in that order
    const size_t tcount = rcount * (size_t)n;
    const red_order ro = tuned_reduce_order(n, type_size(type) * tcount, tcount, 0, false);
    return reduce_my_block(c, src, rbuf, total, (int64_t)(rcount * (size_t)c->rank),
                           (int64_t)rcount, (int64_t)rcount, op, type, ro, inplace, s);
}

// coll/tuned's reduce_scatter decision (coll_tuned_decision_fixed.c:
// 466-512, commutative): recursive halving for small totals or
// power-of-two sizes up to 256 KiB, else the ring.
static red_order tuned_reduce_scatter_order(int n, size_t total_bytes, int block) {
    int pow2 = 1;
    while (pow2 < n) pow2 <<= 1;
    if (total_bytes <= 12 * 1024 || (total_bytes <= 256 * 1024 && pow2 == n) ||
        (double)n >= 0.0012 * (double)total_bytes + 8.0) {
        int adj = 1;
        while (adj * 2 <= n) adj *= 2;
        const int remain = n - adj;
        const int tb = block < 2 * remain ? block / 2 : block - remain;
        return {ORDER_HALVING, 0, tb << 8};
    }
    // ring: block b starts at rank b+1 and ends at b (coll_base_reduce_scatter.c:551-605)
    return {ORDER_RING, (block + 1) % n, 0};
}

int ompi_amd_reduce_scatter(ompi_amd_comm_t *c, const void *sbuf, void *rbuf,
                            const size_t *rcounts, int type, int op, void *stream) {
    if (!c || !rbuf || !rcounts) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    const int n = c->size;
    size_t total = 0, off = 0, maxc = 0;
    for (int p = 0; p < n; ++p) {
        if (p < c->rank) off += rcounts[p];
        total += rcounts[p];
        maxc = std::max(maxc, rcounts[p]);
    }
    if (total == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const size_t ext = ompi_amd_type_extent(type);
    const bool inplace = in_place(sbuf, rbuf);
    const void *src = inplace ? rbuf : sbuf;
    if (n == 1) {
        if (inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, rcounts[0] * ext, hipMemcpyDeviceToDevice, s),
                          "copy");
    }
    const red_order ro = tuned_reduce_scatter_order(n, total * type_size(type), c->rank);
    return reduce_my_block(c, src, rbuf, total * ext, (int64_t)off, (int64_t)rcounts[c->rank],
                           (int64_t)maxc, op, type, ro, inplace, s);
}

int ompi_amd_scan(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                  int op, void *stream) {
    if (c) TRY(drain(c));
    return scan_common(c, sbuf, rbuf, count, type, op, stream, false);
}

int ompi_amd_exscan(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                    int op, void *stream) {
    if (c) TRY(drain(c));
    return scan_common(c, sbuf, rbuf, count, type, op, stream, true);
}

int ompi_amd_allgather(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                       void *stream) {
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(check_sticky(c));
    TRY(drain(c));
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    const int n = c->size;
    const bool inplace = sbuf == (const void *)1 ||
                         sbuf == (const void *)((const char *)rbuf + (size_t)c->rank * bytes);
    char *my_slot = (char *)rbuf + (size_t)c->rank * bytes;
    cp_jobs cj{};
    if (bytes <= c->small_bytes || !c->zero_copy) {
        stage_half sh;
        TRY(stage_in(c, inplace ? my_slot : sbuf, bytes, &sh, s));
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
    TRY(drain(c));
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

int ompi_amd_allreduce_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count,
                            int type, int op, ompi_amd_plan_t **out) {
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    TRY(set_dev(c));
    auto *pl = new (std::nothrow) ompi_amd_plan;
    if (!pl) return OMPI_AMD_ERR_BAD_PARAM;
    const size_t bytes = count * ompi_amd_type_extent(type);
    const bool inplace = in_place(sbuf, rbuf);
    const int n = c->size;
    pl->c = c;
    pl->src = inplace ? rbuf : sbuf;
    pl->rbuf = rbuf;
    pl->count = (int64_t)count;
    pl->op = op;
    pl->type = type;
    const bool tree = type_size(type) * count < 10000 || count < (size_t)n;
    const bool small = n == 1 || count == 0 || (bytes <= c->fused_bytes && bytes <= c->scratch_bytes) ||
                       bytes <= c->small_bytes || !c->zero_copy || tree;
    int rc = OMPI_AMD_SUCCESS;
    if (!small) {
        pl->kind = c->algorithm == ALG_PUSH ? 3 : c->algorithm == ALG_PULL_PUSH ? 2 : 1;
        if (pl->kind == 3) rc = ensure_landing(c, push_slot(pl->count, n, type) * (size_t)n);
        if (rc == OMPI_AMD_SUCCESS)
            rc = exchange_bufs(c, pl->kind == 3 ? nullptr : pl->src, rbuf, &pl->sp, &pl->rp, 0,
                               nullptr, true, pl->bases);
        if (inplace) pl->sp = pl->rp;
    }
    if (rc == OMPI_AMD_SUCCESS)
        rc = record_hip(hipEventCreateWithFlags(&pl->done, hipEventDisableTiming), "plan event");
    if (rc != OMPI_AMD_SUCCESS) {
        (void)ompi_amd_plan_free(pl);
        return rc;
    }
    *out = pl;
    return OMPI_AMD_SUCCESS;
}

static int plan_enqueue(ompi_amd_plan_t *pl, void *stream) {
    ompi_amd_comm_t *c = pl->c;
    if (pl->kind == 0)
        return ompi_amd_allreduce(c, pl->src == pl->rbuf ? (const void *)1 : pl->src, pl->rbuf,
                                  (size_t)pl->count, pl->type, pl->op, stream);
    TRY(check_sticky(c));
    TRY(set_dev(c));
    hipStream_t s = as_stream(stream);
    if (pl->kind == 3) {
        // another call may have grown (and so moved) the landing buffer:
        // its size only grows, so the slots still fit
        return allreduce_push(c, pl->src, pl->rp, pl->count, pl->op, pl->type, s);
    }
    if (pl->kind == 2) return allreduce_pull_push(c, pl->sp, pl->rp, pl->count, pl->op, pl->type, s);
    return allreduce_pull(c, pl->sp, pl->rp, pl->rbuf, pl->count, pl->op, pl->type, s);
}

int ompi_amd_plan_start(ompi_amd_plan_t *pl, void *stream) {
    if (!pl || !pl->c) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(drain(pl->c));  // device order: deferred nonblocking calls first
    TRY(plan_enqueue(pl, stream));
    pl->started = true;
    pl->recorded = false;
    pl->stream = as_stream(stream);
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_plan_test(ompi_amd_plan_t *pl, int *done) {
    if (!pl || !done) return OMPI_AMD_ERR_BAD_PARAM;
    *done = 1;
    if (!pl->started) return OMPI_AMD_SUCCESS;
    if (!pl->recorded) {
        TRY(record_hip(hipEventRecord(pl->done, pl->stream), "plan completion event"));
        pl->recorded = true;
    }
    const hipError_t e = hipEventQuery(pl->done);
    if (e == hipErrorNotReady) {
        *done = 0;
        return OMPI_AMD_SUCCESS;
    }
    if (e != hipSuccess) return record_hip(e, "plan test");
    return check_sticky(pl->c);
}

int ompi_amd_plan_wait(ompi_amd_plan_t *pl) {
    if (!pl) return OMPI_AMD_ERR_BAD_PARAM;
    if (!pl->started) return OMPI_AMD_SUCCESS;
    if (!pl->recorded) {
        TRY(record_hip(hipEventRecord(pl->done, pl->stream), "plan completion event"));
        pl->recorded = true;
    }
    TRY(record_hip(hipEventSynchronize(pl->done), "plan wait"));
    return check_sticky(pl->c);
}

int ompi_amd_plan_free(ompi_amd_plan_t *pl) {
    if (!pl) return OMPI_AMD_SUCCESS;
    if (pl->c)
        for (int p = 0; p < OMPI_AMD_MAX_RANKS; ++p)
            for (int k = 0; k < 2; ++k)
                if (pl->bases[p][k]) unpin_import(pl->c, pl->bases[p][k]);
    if (pl->done) (void)hipEventDestroy(pl->done);
    delete pl;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_request_test(ompi_amd_request_t *r, int *done) {
    if (!r || !done) return OMPI_AMD_ERR_BAD_PARAM;
    *done = 0;
    if (!r->launched) {
        TRY(set_dev(r->c));
        TRY(progress(r->c, false));
        if (!r->launched) return OMPI_AMD_SUCCESS;
    }
    if (r->rc != OMPI_AMD_SUCCESS) return r->rc;
    if (!r->recorded) {
        TRY(record_hip(hipEventRecord(r->ev, r->stream), "request event"));
        r->recorded = true;
    }
    const hipError_t e = hipEventQuery(r->ev);
    if (e == hipErrorNotReady) return OMPI_AMD_SUCCESS;
    if (e != hipSuccess) return record_hip(e, "request test");
    *done = 1;
    return check_sticky(r->c);
}

int ompi_amd_request_wait(ompi_amd_request_t *r) {
    if (!r) return OMPI_AMD_ERR_BAD_PARAM;
    if (!r->launched) {
        TRY(set_dev(r->c));
        TRY(progress(r->c, true));
    }
    if (r->rc != OMPI_AMD_SUCCESS) return r->rc;
    if (!r->recorded) {
        TRY(record_hip(hipEventRecord(r->ev, r->stream), "request event"));
        r->recorded = true;
    }
    TRY(record_hip(hipEventSynchronize(r->ev), "request wait"));
    return check_sticky(r->c);
}

int ompi_amd_request_free(ompi_amd_request_t *r) {
    if (!r) return OMPI_AMD_SUCCESS;
    // the peers launch it whatever this rank does: launch and finish it too
    const int rc = ompi_amd_request_wait(r);
    if (r->ev) (void)hipEventDestroy(r->ev);
    delete r;
    return rc;
}

}  // extern "C"

// ------------------------------------------------ services for p2p / osc
namespace ompi_amd {

static_assert(sizeof(ipc_desc) == sizeof(buf_desc), "ipc_desc mirrors buf_desc");

int comm_rank(const ompi_amd_comm_t *c) { return c->rank; }
int comm_size(const ompi_amd_comm_t *c) { return c->size; }
int comm_device(const ompi_amd_comm_t *c) { return c->device; }
int64_t comm_timeout_ms(const ompi_amd_comm_t *c) { return c->timeout_ms; }
int *comm_err_dev(ompi_amd_comm_t *c) { return c->err_dev; }
p2p_state *comm_p2p(ompi_amd_comm_t *c) { return c->p2p; }

int comm_allgather(ompi_amd_comm_t *c, const void *mine, void *all, size_t len) {
    return c->boot.allgather(mine, all, len);
}

int comm_export(ompi_amd_comm_t *c, const void *ptr, ipc_desc *d) {
    buf_desc b{};
    const int rc = export_buf(c, ptr, &b);
    memcpy(d, &b, sizeof(b));
    return rc;
}

int comm_import(ompi_amd_comm_t *c, int peer, const ipc_desc &d, const char **out, bool pin,
                void **base) {
    buf_desc b;
    memcpy(&b, &d, sizeof(b));
    return import_buf(c, peer, b, out, pin, base);
}

void comm_unpin(ompi_amd_comm_t *c, void *base) { unpin_import(c, base); }

int comm_drain(ompi_amd_comm_t *c) { return drain(c); }

int comm_barrier(ompi_amd_comm_t *c, hipStream_t s) {
    TRY(drain(c));
    return launch_barrier(c, s);
}

int comm_sticky(ompi_amd_comm_t *c) { return check_sticky(c); }

int comm_copy(ompi_amd_comm_t *c, const void *src, void *dst, size_t bytes, hipStream_t s) {
    cp_jobs jobs{};
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    jobs.j[0] = {(const char *)src, (char *)dst, (int64_t)bytes};
    jobs.n = 1;
    return launch_copy(c, jobs, s);
}

}  // namespace ompi_amd
