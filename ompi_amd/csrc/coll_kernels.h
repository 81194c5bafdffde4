// Device side of the xGMI collectives (coll_ipc.hip): the shared job and
// pointer-set types, the memory-ordering helpers, the reduction fold in the
// reference algorithms' operand orders, and the reduce / fused-allreduce
// kernel templates.  The kernels are instantiated per op by coll_kern.hip
// (one object per op, compiled in parallel) and reached through the
// per-op launch rows declared at the end.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/ompi_amd_coll.h"
#include "op_device.h"

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
    ORDER_RABEN = 6,     // Rabenseifner allreduce (redscat_allgather), owner vrank in flags >> 8
};
// The root passed MPI_IN_PLACE: its first combine is f(own, child)
// (coll_base_reduce.c:170-171, 196-199).
constexpr int FOLD_ROOT_INPLACE = 1;
// Launch flag, not a fold rule: the vector body stores non-temporally
// (param "copy_nt", the 8-GPU bench's A/B; fold() never reads bit 16).
constexpr int FOLD_NT_STORE = 1 << 16;

// One reduction job: elements [off, off+cnt) of every source, combined in
// the call's order and written to dst + off_dst (element units).
struct red_job {
    int64_t off, cnt, off_dst;
    int first;  // virtual rank 0 (ring block b, tree root)
    int head;   // elements before the 16-B aligned body; -1: no common alignment
    int aux = 0;  // per-job fold flags, or-ed into the launch's (ORDER_RABEN: owner vrank << 8)
};
// a ring block cut at the Rabenseifner pieces: up to kMaxRanks + 1 jobs
struct red_jobs { red_job j[2 * kMaxRanks]; int n; };

struct cp_job { const char *src; char *dst; int64_t bytes; };
struct cp_jobs { cp_job j[kMaxRanks]; int n; };

// the acquiring lane waits for its invalidate before the barrier that
// lets the other waves load (Guideline 16: the fence itself does not wait)
__device__ __forceinline__ void sys_acquire() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
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

// Wait until *flag >= epoch (a peer's barrier store).  Bounded: past
// `ticks` (s_memrealtime, 100 MHz) the communicator's sticky error word (host
// memory, written only — a spinning wave never reads host memory) is set and
// the communicator's abort word (in its own flag page, device memory) is
// raised.  Every ~1 ms of waiting the abort word is read, so once any wait
// of this communicator has given up — or a failing peer raised the word
// (abort_peers) — every later wait gives up within 1 ms: a rank whose peer
// failed a call it had already launched drains its queued collectives in one
// timeout instead of one per barrier, and reaches comm_destroy's host
// rendezvous while that peer is still there to keep its memory alive.
// Returns false when the wait gave up.
// The flag page: 32 rows x 16 ranks of epochs (4 KiB), then the abort word.
constexpr int kAbortWord = 512;               // uint64 index in the flag page
constexpr size_t kFlagPageBytes = 8192;

// seen (debug, OMPI_AMD_DEBUG_PROGRESS=1; else null): the flag value read
// at every ~1 ms check, in host-mapped memory a watchdog can print.
__device__ __forceinline__ bool wait_epoch(const uint64_t *flag, uint64_t epoch, int *err,
                                           uint64_t ticks, uint64_t *abort_word,
                                           uint64_t *seen = nullptr) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t check = t0 + 100000;  // 1 ms
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
        __builtin_amdgcn_s_sleep(1);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (now - t0 > ticks) {
            __hip_atomic_store(err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(abort_word, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
        if (now >= check) {
            if (seen)
                __hip_atomic_store(seen, __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
                __hip_atomic_store(err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
            check = now + 100000;
        }
    }
    return true;
}

// Every storing wave drains its stores before the workgroup's single
// system-scope release (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ void xfer_epilogue() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sys_release();
}

// ---------------------------------------------------------------- reduce
// Fold v[0..n) (virtual-rank order) with the 2-buffer rule f(out, in).  All
// array indices are compile-time constants after unrolling; n, order and
// flags are wave-uniform.
template <typename T, int OP, int NM = kMaxRanks>
__device__ __forceinline__ T fold(const T (&v)[NM], int n, int order, int flags) {
    using F = opfn<OP, false>;
    const bool swap = (flags & FOLD_ROOT_INPLACE) != 0;
    if (order == ORDER_RING) {
        // v[j] = x[(b + j) % n]; acc = x[b]; acc = f(x[b+j], acc)
        T acc = v[0];
#pragma unroll
        for (int j = 1; j < NM; ++j)
            if (j < n) acc = F::template f<T>(v[j], acc);
        return acc;
    }
    if (order == ORDER_CHAIN) {
        // chain fanout 1 (coll_base_topo.c:588-600) under the generic reduce
        // (coll_base_reduce.c:206-215): node k's only child is k+1,
        // acc_k = f(acc_(k+1), x_k); basic_linear (:680-721) is the same
        // expression at first = 0.
        T acc = v[NM - 1];
#pragma unroll
        for (int j = NM - 1; j >= 0; --j) {
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
        T w[NM];
#pragma unroll
        for (int i = 0; i < NM; ++i) w[i] = v[i];
#pragma unroll
        for (int u = 0; u + 1 < NM; u += 2)
            if (u + 1 < n) w[u] = (u == 0 && swap) ? F::template f<T>(w[0], w[1])
                                                   : F::template f<T>(w[u + 1], w[u]);
#pragma unroll
        for (int m = 2; m < NM; m <<= 1) {
#pragma unroll
            for (int u = 0; u + m < NM; u += 2 * m)
                if (u + m < n) w[u] = F::template f<T>(w[u], w[u + m]);
        }
        return w[0];
    }
    if (order == ORDER_BINARY) {
        // build_tree(2) (coll_base_topo.c:77-175): shifted rank s has
        // children s + d and s + 2d, d = largest power of two <= s + 1;
        // children have larger s, so descending s sees them finished.
        T w[NM];
#pragma unroll
        for (int i = 0; i < NM; ++i) w[i] = v[i];
#pragma unroll
        for (int s = NM - 1; s >= 0; --s) {
            int d = 1;
            while (2 * d <= s + 1) d *= 2;
            const int c0 = s + d, c1 = s + 2 * d;
            if (c0 < NM && c0 < n)
                w[s] = (s == 0 && swap) ? F::template f<T>(w[0], w[c0])
                                        : F::template f<T>(w[c0], w[s]);
            if (c1 < NM && c1 < n) w[s] = F::template f<T>(w[s], w[c1]);
        }
        return w[0];
    }
    if (order == ORDER_RABEN) {
        // redscat_allgather (coll_base_allreduce.c:970-1243).  Step 1: the
        // 2*rem lowest ranks pair up; the even one keeps the left half of
        // the vector as f(even, odd), the odd one the right half as
        // f(odd, even) (:1031-1080) — the owner's bit 0 says which half
        // this element is in.  Step 2: recursive halving over the p' vranks
        // with masks 1, 2, 4, ... (:1122-1171): at every mask the vrank
        // keeping the element's part does f(mine, partner's).  o = the
        // vrank the element ends on.
        int adj = 1;
        while (adj * 2 <= n) adj *= 2;
        const int rem = n - adj;
        const int o = (flags >> 8) & 0xff;
        const bool right = (o & 1) != 0;
        T w[NM];
#pragma unroll
        for (int u = 0; u < NM; ++u) {
            if (2 * u + 1 < NM && u < rem)
                w[u] = right ? F::template f<T>(v[2 * u + 1], v[2 * u])
                             : F::template f<T>(v[2 * u], v[2 * u + 1]);
            else if (u < adj)
                w[u] = v[u + rem < NM ? u + rem : 0];
        }
#pragma unroll
        for (int m = 1; m < NM; m <<= 1) {
            if (m < adj) {
#pragma unroll
                for (int u = 0; u < NM; ++u)
                    if (u < adj && (u & m) == (o & m)) w[u] = F::template f<T>(w[u], w[u ^ m]);
            }
        }
        T r = w[0];
#pragma unroll
        for (int u = 1; u < NM; ++u)
            if (u == o) r = w[u];
        return r;
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
        T w[NM];
#pragma unroll
        for (int u = 0; u < NM; ++u) {
            if (2 * u + 1 < NM && u < remain) w[u] = F::template f<T>(v[2 * u + 1], v[2 * u]);
            else if (u < adj) w[u] = v[u + remain];
        }
#pragma unroll
        for (int m = NM / 2; m >= 1; m >>= 1) {
            if (m < adj) {
#pragma unroll
                for (int u = 0; u < NM; ++u)
                    if (u < adj && (u & m) == (tb & m)) w[u] = F::template f<T>(w[u], w[u ^ m]);
            }
        }
        T r = w[0];
#pragma unroll
        for (int u = 1; u < NM; ++u)
            if (u == tb) r = w[u];
        return r;
    }
    // recursive doubling (coll_base_allreduce.c:184-236): fold the
    // 2*extra lowest ranks pairwise, then a pairwise tree; every combine is
    // f(out = higher, in = lower).
    int adj = 1;
    while (adj * 2 <= n) adj *= 2;
    const int extra = n - adj;
    T w[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        if (i < extra) w[i] = F::template f<T>(v[2 * i + 1], v[2 * i]);
        else if (i < adj) w[i] = v[i + extra];
    }
#pragma unroll
    for (int len = NM; len > 1; len >>= 1) {
        if (len <= adj) {
#pragma unroll
            for (int i = 0; i < NM / 2; ++i)
                if (2 * i + 1 < len) w[i] = F::template f<T>(w[2 * i + 1], w[2 * i]);
        }
    }
    return w[0];
}

// Gather v[j] for element index e of the sources in virtual-rank order.
template <typename T, int NM = kMaxRanks>
__device__ __forceinline__ void gather_scalar(T (&v)[NM], const ptr_set &src, int n,
                                              int first, int64_t e) {
#pragma unroll
    for (int j = 0; j < NM; ++j) {
        if (j < n) {
            const int r = (first + j) % n;
            v[j] = reinterpret_cast<const T *>(src.p[r])[e];
        }
    }
}

// NM: the register arrays' size, a compile-time bound >= n (8 for up to 8
// ranks, else 16: at N <= 8 the kernel holds half the vectors, 109 -> fewer
// VGPRs and more waves per SIMD).
// n sources (virtual ranks 0..n), result stored to dst.p[0 .. ndst): ndst =
// 1 is a plain reduce into one buffer; ndst = size is the fused push of the
// owner's block into every rank's rbuf (the host orders dst local first,
// then peers rank+1, rank+2, ... so concurrent owners spread their stores
// over the links).
template <typename T, int OP, int NM = kMaxRanks>
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
        vec16<T> v[NM];
#pragma unroll
        for (int j = 0; j < NM; ++j) {
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
            T s[NM];
#pragma unroll
            for (int j = 0; j < NM; ++j) s[j] = v[j].e[e];
            out.e[e] = fold<T, OP, NM>(s, n, order, flags | jb.aux);
        }
        if (flags & FOLD_NT_STORE) {
#pragma unroll
            for (int k = 0; k < NM; ++k)
                if (k < ndst)
                    __builtin_nontemporal_store(
                        out.v, reinterpret_cast<u32x4 *>(reinterpret_cast<T *>(const_cast<char *>(dst.p[k])) +
                                                         jb.off_dst + head) + i);
        } else {
#pragma unroll
            for (int k = 0; k < NM; ++k)
                if (k < ndst)
                    reinterpret_cast<u32x4 *>(reinterpret_cast<T *>(const_cast<char *>(dst.p[k])) +
                                              jb.off_dst + head)[i] = out.v;
        }
    }
    // scalar head [0, head) and tail [head + nvec*E, cnt)
    const int64_t tail0 = head + nvec * E;
    const int64_t nscalar = head + (jb.cnt - tail0);
    for (int64_t k = tid; k < nscalar; k += gstride) {
        const int64_t e = k < head ? k : tail0 + (k - head);
        T s[NM];
        gather_scalar<T, NM>(s, src, n, jb.first, jb.off + e);
        const T r = fold<T, OP, NM>(s, n, order, flags | jb.aux);
#pragma unroll
        for (int d = 0; d < NM; ++d)
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
    // ompi_amd_allreduce_wait: the last workgroup to finish stores mark_v
    // into the pinned host word `mark` (done: a zeroed counter in my flag
    // page) — the host's wait needs no mark kernel after this one
    uint32_t *done;
    uint64_t *mark;
    uint64_t mark_v;
};

// flag-page word (uint32 index) of the fused kernel's finished-workgroup counter
constexpr int kFusedDoneWord = 8192 / (int)sizeof(uint32_t);
// completion counters of fused launches that store their own mark: slot k
// at word kFusedDoneWord + kFusedDoneStride * k (own 64-B line), slot 0 the
// blocking call's, the others persistent plans' (up to kPipeFlagOff)
constexpr int kFusedDoneStride = 64 / (int)sizeof(uint32_t);
constexpr int kFusedDoneSlots = (64 << 10) / 64 - 8192 / 64;

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
    __shared__ int gave_up;
    if (t == 0) gave_up = 0;
    __syncthreads();
    if (t < a.n && t != a.rank) {
        __hip_atomic_store(a.peer_flags.p[t] + g * kMaxRanks + a.rank, a.epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        if (!wait_epoch(a.flags + g * kMaxRanks + t, a.epoch, a.err, a.timeout_ticks,
                        a.flags + kAbortWord))
            gave_up = 1;
    }
    __syncthreads();
    if (gave_up) return;  // a peer never arrived: its scratch is not ours to read
    acquire_once();
    T *dst = reinterpret_cast<T *>(a.dst);
    for (int64_t e = lo + t; e < hi; e += kXferThreads) {
        T v[kMaxRanks];
        gather_scalar<T>(v, a.peers, a.n, first, e);
        store_elem<T>(dst + e, fold<T, OP>(v, a.n, a.order, 0));
    }
    if (a.mark) {  // the host-observed completion, by the last workgroup
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // my results, device-wide
            const uint32_t total = gridDim.x * gridDim.y;
            if (__hip_atomic_fetch_add(a.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == total - 1) {
                __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(a.mark, a.mark_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// ---------------------------------------------------------------- pipelined large allreduce
// The two-shot schemes' three phases — send (C: my input's blocks to where
// their owners fold them), fold (F: the owner folds its block and stores the
// result where the others gather it), gather (G: the other blocks into my
// rbuf) — in ONE launch with per-slice flags instead of a device barrier
// between phases.  Every block is cut into slices; workgroup w owns slices
// w, w + G, w + 2G, ... of every block, and at its iteration p it runs C of
// its slice p, F of slice p - 1 and G of slice p - 2, then drains its
// stores, releases once, and tells every peer "C(p) and F(p - 1) done" on
// its own flag row.  Before iteration p it waits only for the SAME
// workgroup of every peer to have finished iteration p - 1 (its C(p - 1)
// feeds my F(p - 1), its F(p - 2) my G(p - 2)): no grid-wide sync, and
// copy, fold and gather traffic of different slices is in flight together
// (the staging copy of pull, the scatter of push, overlap the transfers
// instead of preceding them behind a barrier).  Which buffers the phases
// touch is the host's choice (coll_ipc.hip: staged pull, push-gather,
// push-land).  Element e of the vector sits at p + e * sizeof(T) for every
// pointer below (the host biases landing-slot pointers by their block's
// offset).  Flag rows live kPipeFlagOff bytes into each rank's flag
// allocation: [phase C / F][workgroup][peer] of uint64 counters,
// (seq << 20) + (iterations done), seq the same on every rank per call.
constexpr int kPipeMaxGroups = 1024;
constexpr size_t kPipeFlagOff = 64 << 10;
constexpr size_t kPipeFlagBytes = 2 * (size_t)kPipeMaxGroups * kMaxRanks * sizeof(uint64_t);

struct pipe_args {
    const char *src;
    ptr_set dst_c;  // per block: where C sends it (null: not sent — my own block)
    ptr_set src_f;  // per rank: the fold's sources (virtual order from `first`)
    ptr_set dst_f;  // the fold's destinations [0, ndst)
    ptr_set src_g;  // per block: where G gathers it from (null: not gathered)
    char *rbuf;
    uint64_t *flags;      // my pipe rows
    flag_set peer_flags;  // every peer's pipe rows as mapped here
    int rank, n, mine, ndst, order, first, fold_flags, nt;
    int colocated;  // most ranks of this communicator sharing one GPU (co-residency cap)
    int64_t split, early, late;  // ring blocks (blockcount)
    int64_t per, nslices;        // elements per slice (a multiple of 16 B), slices per block
    uint64_t seq, timeout_ticks;
    int *err;
    uint64_t *abort_word;
};

__device__ __forceinline__ size_t pipe_row(int phase, int w, int r) {
    return ((size_t)phase * kPipeMaxGroups + (size_t)w) * kMaxRanks + (size_t)r;
}

// Bytes [lo, hi) from s to d by one workgroup: 16-B vectors, 4 in flight
// per lane, when s and d share their phase mod 16; else bytewise.
__device__ __forceinline__ void pipe_copy(const char *s, char *d, int64_t lo, int64_t hi, bool nt) {
    const int t = threadIdx.x;
    if (hi <= lo) return;
    int64_t head = hi - lo, nv = 0;
    if ((((uintptr_t)(s + lo) ^ (uintptr_t)(d + lo)) & 15) == 0) {
        head = min(hi - lo, (int64_t)((16 - ((uintptr_t)(s + lo) & 15)) & 15));
        nv = (hi - lo - head) / 16;
    }
    const u32x4 *sv = reinterpret_cast<const u32x4 *>(s + lo + head);
    u32x4 *dv = reinterpret_cast<u32x4 *>(d + lo + head);
    constexpr int S = kXferThreads;
    int64_t i = t;
    for (; i + 3 * S < nv; i += 4 * S) {
        const u32x4 a = __builtin_nontemporal_load(sv + i);
        const u32x4 b = __builtin_nontemporal_load(sv + i + S);
        const u32x4 c = __builtin_nontemporal_load(sv + i + 2 * S);
        const u32x4 e = __builtin_nontemporal_load(sv + i + 3 * S);
        if (nt) {
            __builtin_nontemporal_store(a, dv + i);
            __builtin_nontemporal_store(b, dv + i + S);
            __builtin_nontemporal_store(c, dv + i + 2 * S);
            __builtin_nontemporal_store(e, dv + i + 3 * S);
        } else {
            dv[i] = a;
            dv[i + S] = b;
            dv[i + 2 * S] = c;
            dv[i + 3 * S] = e;
        }
    }
    for (; i < nv; i += S) {
        if (nt) __builtin_nontemporal_store(__builtin_nontemporal_load(sv + i), dv + i);
        else dv[i] = __builtin_nontemporal_load(sv + i);
    }
    const int64_t tail0 = lo + head + nv * 16;
    const int64_t nrest = head + (hi - tail0);
    for (int64_t k = t; k < nrest; k += S) {
        const int64_t b = k < head ? lo + k : tail0 + (k - head);
        d[b] = s[b];
    }
}

// Elements [lo, hi) of the fold by one workgroup (reduce_kernel's body).
template <typename T, int OP, int NM>
__device__ __forceinline__ void pipe_fold(const pipe_args &a, int64_t lo, int64_t hi) {
    constexpr int E = 16 / sizeof(T);
    const int t = threadIdx.x;
    if (hi <= lo) return;
    // vector body where every source and destination is 16-B aligned
    const uintptr_t ph = (uintptr_t)(a.dst_f.p[0] + lo * (int64_t)sizeof(T)) & 15;
    bool same = true;
#pragma unroll
    for (int j = 0; j < NM; ++j)
        if (j < a.n) same = same && (((uintptr_t)(a.src_f.p[j] + lo * (int64_t)sizeof(T)) & 15) == ph);
#pragma unroll
    for (int k = 1; k < NM; ++k)
        if (k < a.ndst) same = same && (((uintptr_t)(a.dst_f.p[k] + lo * (int64_t)sizeof(T)) & 15) == ph);
    const int64_t lead = (int64_t)((16 - ph) & 15);
    int64_t head = hi - lo, nv = 0;
    if (same && lead % (int64_t)sizeof(T) == 0) {
        head = min(hi - lo, lead / (int64_t)sizeof(T));
        nv = (hi - lo - head) / E;
    }
    const int64_t v0 = lo + head;
    for (int64_t i = t; i < nv; i += kXferThreads) {
        vec16<T> v[NM];
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            if (j < a.n) {
                const int r = (a.first + j) % a.n;
                const u32x4 *p = reinterpret_cast<const u32x4 *>(reinterpret_cast<const T *>(a.src_f.p[r]) + v0);
                v[j].v = __builtin_nontemporal_load(p + i);
            }
        }
        vec16<T> out;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            T s[NM];
#pragma unroll
            for (int j = 0; j < NM; ++j) s[j] = v[j].e[e];
            out.e[e] = fold<T, OP, NM>(s, a.n, a.order, a.fold_flags);
        }
#pragma unroll
        for (int k = 0; k < NM; ++k) {
            if (k < a.ndst) {
                u32x4 *q = reinterpret_cast<u32x4 *>(reinterpret_cast<T *>(const_cast<char *>(a.dst_f.p[k])) + v0) + i;
                if (a.nt) __builtin_nontemporal_store(out.v, q);
                else *q = out.v;
            }
        }
    }
    const int64_t tail0 = v0 + nv * E;
    const int64_t nrest = head + (hi - tail0);
    for (int64_t k = t; k < nrest; k += kXferThreads) {
        const int64_t e = k < head ? lo + k : tail0 + (k - head);
        T s[NM];
        gather_scalar<T, NM>(s, a.src_f, a.n, a.first, e);
        const T r = fold<T, OP, NM>(s, a.n, a.order, a.fold_flags);
#pragma unroll
        for (int d = 0; d < NM; ++d)
            if (d < a.ndst) store_elem<T>(reinterpret_cast<T *>(const_cast<char *>(a.dst_f.p[d])) + e, r);
    }
}

template <typename T, int OP, int NM>
__global__ __launch_bounds__(kXferThreads) void pipe_allreduce_kernel(pipe_args a) {
    const int t = threadIdx.x, w = blockIdx.x, G = gridDim.x;
    const int64_t P = (a.nslices - w + G - 1) / G;  // my slices (the host sizes G <= nslices)
    constexpr int64_t ext = sizeof(T);
    __shared__ int gave_up;
    if (t == 0) gave_up = 0;
    __syncthreads();
    for (int64_t p = 0; p < P + 2; ++p) {
        const bool doC = p < P, doF = p >= 1 && p <= P, doG = p >= 2;
        if (p >= 1) {
            if (t < a.n && t != a.rank) {
                bool ok = true;
                if (doF)  // peer t's C(p - 1): its share of my block's slice p - 1
                    ok = wait_epoch(a.flags + pipe_row(0, w, t), a.seq + (uint64_t)p, a.err,
                                    a.timeout_ticks, a.abort_word);
                if (ok && doG)  // peer t's F(p - 2): its block's slice p - 2 folded
                    ok = wait_epoch(a.flags + pipe_row(1, w, t), a.seq + (uint64_t)(p - 1), a.err,
                                    a.timeout_ticks, a.abort_word);
                if (!ok) gave_up = 1;
            }
            __syncthreads();
            if (gave_up) return;  // a peer never arrived: its memory is not ours to read
            acquire_once();
        }
        if (doC) {
            const int64_t s = w + p * G;
#pragma unroll
            for (int b = 0; b < NM; ++b) {
                if (b >= a.n || !a.dst_c.p[b]) continue;
                const int64_t off = b < a.split ? b * a.early : b * a.late + a.split;
                const int64_t cnt = b < a.split ? a.early : a.late;
                const int64_t lo = off + min(cnt, s * a.per), hi = off + min(cnt, (s + 1) * a.per);
                pipe_copy(a.src, const_cast<char *>(a.dst_c.p[b]), lo * ext, hi * ext, a.nt);
            }
        }
        if (doF) {
            const int64_t s = w + (p - 1) * G;
            const int b = a.mine;
            const int64_t off = b < a.split ? b * a.early : b * a.late + a.split;
            const int64_t cnt = b < a.split ? a.early : a.late;
            pipe_fold<T, OP, NM>(a, off + min(cnt, s * a.per), off + min(cnt, (s + 1) * a.per));
        }
        if (doG) {
            const int64_t s = w + (p - 2) * G;
#pragma unroll
            for (int b = 0; b < NM; ++b) {
                if (b >= a.n || !a.src_g.p[b]) continue;
                const int64_t off = b < a.split ? b * a.early : b * a.late + a.split;
                const int64_t cnt = b < a.split ? a.early : a.late;
                const int64_t lo = off + min(cnt, s * a.per), hi = off + min(cnt, (s + 1) * a.per);
                pipe_copy(a.src_g.p[b], a.rbuf, lo * ext, hi * ext, a.nt);
            }
        }
        if (doC || doF) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) sys_release();
            __syncthreads();
            if (t < a.n && t != a.rank) {
                if (doC)
                    __hip_atomic_store(a.peer_flags.p[t] + pipe_row(0, w, a.rank), a.seq + (uint64_t)(p + 1),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (doF)
                    __hip_atomic_store(a.peer_flags.p[t] + pipe_row(1, w, a.rank), a.seq + (uint64_t)p,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    xfer_epilogue();
}

// ---------------------------------------------------------------- launch rows
using red_launch_fn = hipError_t (*)(dim3, const ptr_set &, const ptr_set &, int, int, int, int,
                                     const red_jobs &, hipStream_t);
using fused_launch_fn = hipError_t (*)(dim3, const fused_args &, hipStream_t);
using pipe_launch_fn = hipError_t (*)(unsigned, const pipe_args &, hipStream_t);

// Row `op` of the launch tables: OMPI_AMD_TYPE_COUNT entries, NULL where
// op/base has no handler (slot_supported).  Defined by coll_kern.hip built
// once per op with -DCOLL_OP=<op>.
#define OMPI_AMD_COLL_OPS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
#define OMPI_AMD_COLL_ROW_DECL(k)          \
    const red_launch_fn *red_row_##k();    \
    const fused_launch_fn *fused_row_##k(); \
    const pipe_launch_fn *pipe_row_##k();
OMPI_AMD_COLL_OPS(OMPI_AMD_COLL_ROW_DECL)
#undef OMPI_AMD_COLL_ROW_DECL

}  // namespace ompi_amd
