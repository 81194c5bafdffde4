// One-sided communication on device windows (include/ompi_amd_osc.h).
//
// Reference: osc/sm (ompi/mca/osc/sm/).  Its window is one shared segment;
// an accumulate takes the target's accumulate spinlock and runs
// ompi_op_reduce(op, origin, target) on the host (osc_sm_comm.c:271-309 ->
// osc_base_obj_convert.c ompi_osc_base_sndrcv_op); passive-target locks are
// a ticket lock of three counters per rank (osc_sm_passive_target.c:23-110);
// a fence is a barrier (osc_sm_active_target.c:95-115).
//
// Here each rank's window is device memory that every peer maps with
// hipIpcOpenMemHandle, plus one fine-grained control page per rank (the
// accumulate lock word and the ticket-lock counters).  Every operation is
// kernels on the origin's stream:
//   lock kernels    one lane; system-scope atomics on the target's control
//                   page, polled with s_sleep and a wall-clock bound that
//                   sets the communicator's sticky error word;
//   acc_kernel      target[i] = f(target[i], origin[i]) with op/base's
//                   2-buffer element rule (op_device.h), 16-B granules when
//                   both sides are 16-B aligned; target is peer memory, so
//                   its loads and stores cross xGMI once each;
//   xfer_kernel     put / get / the fetch of get_accumulate (and the p2p
//                   receive): byte copy, 16-B granules.
// Grids are persistent (kOscMaxBlocks): a system-scope acquire invalidates
// the XCD's L2, so paying it once per workgroup in a 65k-workgroup grid
// cost 7x (tools/osc_probe.py: accumulate 0.89 TB/s uncapped, 6.26 at 256).
// Every transfer workgroup opens with a system-scope acquire and closes
// with a drained system-scope release, as the collectives do
// (coll_ipc.hip header): the lock hand-off then orders one origin's
// stores before the next holder's loads.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "host_mark.h"
#include "../../include/ompi_amd_osc.h"
#include "comm_internal.h"
#include "ddt_device.h"
#include "ipc_registry.h"
#include "op_device.h"
#include "runtime.h"

namespace ompi_amd {

constexpr int kOscThreads = 256;
constexpr int kOscMaxRanks = OMPI_AMD_MAX_RANKS;

// control page words (uint32 each)
enum { CTL_ACC = 0, CTL_COUNTER = 16, CTL_WRITE = 32, CTL_READ = 48, CTL_BYTES = 4096 };
// Origin-side words of the rank's own control page: whether this rank's
// last lock kernel toward target t actually holds the lock — 0 no (skipped
// after a sticky error, or timed out), 1 yes, 2 a ticket was drawn but never
// granted.  Unlock kernels and the data kernels of the epoch read them, so a
// lock that was not taken is never released on someone else's behalf and
// no data moves without it.
enum { CTL_TAKEN_ACC = 256, CTL_TAKEN_EPOCH = 512 };
// General active target synchronisation (osc_sm_active_target.c:126-330):
// word CTL_POST + 16 p of a rank's control page counts the exposure epochs
// rank p opened toward it (MPI_Win_post; osc/sm's posts[] bit per rank, a
// counter here so that repeated epochs need no clearing); CTL_COMPLETE
// counts the access epochs origins closed toward it (MPI_Win_complete;
// osc/sm's complete_count).  Each on its own 64-B line.
enum { CTL_POST = 640, CTL_COMPLETE = 960 };
constexpr int kPscwLane = 16;  // words between two CTL_POST counters
static_assert(CTL_POST + kPscwLane * OMPI_AMD_MAX_RANKS <= CTL_COMPLETE, "pscw words overlap");

// the peers' control pages, by value (a kernel argument)
struct peer_ctl_set {
    uint32_t *p[OMPI_AMD_MAX_RANKS];
};

// The acquiring lane waits for its invalidate before the workgroup barrier
// that usually follows: the other waves' loads must not pass it (the
// fence's own lowering does not wait; cdna_hip_programming.md Guideline 16).
__device__ __forceinline__ void osc_acquire() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void osc_release() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void osc_epilogue() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) osc_release();
}

__device__ __forceinline__ uint32_t ld_sys(uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Poll until *p == want (or the bound passes: sticky error, give up).
__device__ __forceinline__ bool wait_eq(uint32_t *p, uint32_t want, int *err, uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (ld_sys(p) != want) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            __hip_atomic_store(err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
    }
    return true;
}

__device__ __forceinline__ void st_sys(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A data kernel of a locked epoch runs only if its lock was taken
// (gate = the origin's CTL_TAKEN_* word; NULL: no lock involved).
__device__ __forceinline__ bool gate_open(const uint32_t *gate) {
    __shared__ uint32_t open;
    if (threadIdx.x == 0)
        open = gate ? __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 1u : 1u;
    __syncthreads();
    return open != 0;
}

// The target's accumulate lock (opal_atomic_lock, osc_sm_comm.c:296-305):
// spin on a compare-and-swap 0 -> 1 of its CTL_ACC word, bounded (sticky
// timeout); false at once when the communicator already failed.
__device__ __forceinline__ bool acc_lock_take(uint32_t *ctl, int *err, uint64_t ticks) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return false;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        uint32_t expect = 0;
        if (__hip_atomic_compare_exchange_strong(ctl + CTL_ACC, &expect, 1u, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
            return true;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            __hip_atomic_store(err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
    }
}

// kind: 0 accumulate lock, 1 accumulate unlock, 2 start_exclusive,
// 3 end_exclusive, 4 start_shared, 5 end_shared (osc_sm_passive_target.c:57-110)
// taken: this rank's CTL_TAKEN_* word for the target (its own control page).
__global__ __launch_bounds__(64) void lock_kernel(uint32_t *ctl, int kind, int *err,
                                                  uint64_t ticks, uint32_t *taken) {
    if (threadIdx.x != 0) return;
    // fail fast: once a lock or barrier of this communicator timed out, the
    // later acquisitions do not wait again (the error is already sticky)
    if ((kind == 0 || kind == 2 || kind == 4) &&
        __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
        st_sys(taken, 0u);
        return;
    }
    // a release of a lock this rank does not hold is a no-op (the unlock
    // would otherwise free another rank's lock)
    if ((kind == 1 || kind == 3 || kind == 5) && ld_sys(taken) != 1u) return;
    switch (kind) {
    case 0:  // opal_atomic_lock
        st_sys(taken, acc_lock_take(ctl, err, ticks) ? 1u : 0u);
        osc_acquire();
        break;
    case 1:
        osc_release();
        __hip_atomic_store(ctl + CTL_ACC, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st_sys(taken, 0u);
        break;
    case 2: {  // start_exclusive: take a ticket, wait until every earlier holder ended
        const uint32_t me = __hip_atomic_fetch_add(ctl + CTL_COUNTER, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM);
        // a ticket drawn but never granted cannot be given back (the holders
        // after it wait for it); the communicator's error is sticky by then
        st_sys(taken, wait_eq(ctl + CTL_WRITE, me, err, ticks) ? 1u : 2u);
        osc_acquire();
        break;
    }
    case 3:  // end_exclusive
        osc_release();
        __hip_atomic_fetch_add(ctl + CTL_WRITE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_add(ctl + CTL_READ, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st_sys(taken, 0u);
        break;
    case 4: {  // start_shared: wait until every earlier ticket has started (shared) or ended
        const uint32_t me = __hip_atomic_fetch_add(ctl + CTL_COUNTER, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM);
        const bool ok = wait_eq(ctl + CTL_READ, me, err, ticks);
        if (ok)
            __hip_atomic_fetch_add(ctl + CTL_READ, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st_sys(taken, ok ? 1u : 2u);
        osc_acquire();
        break;
    }
    case 5:  // end_shared
        osc_release();
        __hip_atomic_fetch_add(ctl + CTL_WRITE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st_sys(taken, 0u);
        break;
    }
}

// PSCW on the stream (one lane per group member):
//   0 post      release this rank's window; +1 on CTL_POST[me] of each origin
//   1 start     wait until each target's CTL_POST[target] here reached the
//               epoch's count, then acquire
//   2 complete  release (the epoch's RMA kernels precede on the stream); +1
//               on CTL_COMPLETE of each target
//   3 wait      wait until CTL_COMPLETE here reached the count, then acquire
struct pscw_group {
    int n;
    int rank[kOscMaxRanks];
    uint32_t want[kOscMaxRanks];  // start: per target; wait: want[0]
};

__global__ __launch_bounds__(64) void pscw_kernel(uint32_t *own, peer_ctl_set peers, pscw_group g,
                                                  int kind, int me, int *err, uint64_t ticks) {
    const int t = threadIdx.x;
    if (kind == 0 || kind == 2) {
        if (t == 0) osc_release();
        __syncthreads();
        if (t < g.n)
            __hip_atomic_fetch_add(peers.p[g.rank[t]] + (kind == 0 ? CTL_POST + kPscwLane * me : CTL_COMPLETE),
                                   1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
    const int lanes = kind == 1 ? g.n : 1;
    if (t < lanes) {
        uint32_t *w = kind == 1 ? own + CTL_POST + kPscwLane * g.rank[t] : own + CTL_COMPLETE;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while ((int32_t)(ld_sys(w) - g.want[t]) < 0) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                __hip_atomic_store(err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
    }
    __syncthreads();
    if (t == 0) osc_acquire();
}

// target[i] = f(target[i], origin[i]) — the 2-buffer rule with out = target,
// in = origin (ompi_osc_base_sndrcv_op -> ompi_op_reduce(op, origin, target)).
// Aligned operands: 4 16-B vectors of each in flight per lane, one chunk
// per workgroup (the op kernel's tuned shape, op_kernels.hip); the target's
// loads and stores cross xGMI.  Unaligned: one element per lane.
constexpr int kOscUnroll = 4;
// Grid cap: a persistent grid-stride grid, so the per-workgroup L2
// invalidation of the acquire is paid a bounded number of times
// (tools/osc_probe.py; env OMPI_AMD_OSC_MAX_BLOCKS overrides).
constexpr int kOscMaxBlocks = 256;  // one per CU: 6.26 TB/s vs 3.40 at 2048 (256 MiB fp32 SUM)

// sys: the target is another GPU's memory — every workgroup ends with a
// system-scope release (as xfer_kernel's SYS); this GPU's memory is covered
// by the kernel boundary's release.
template <typename T, int OP>
__global__ __launch_bounds__(kOscThreads) void acc_kernel(const T *__restrict__ origin, T *target,
                                                          int64_t n, int vec,
                                                          const uint32_t *gate, int sys) {
    if (!gate_open(gate)) return;
    // one system-scope acquire per workgroup (it invalidates this CU's L1
    // and the XCD's L2 for every wave of the CU): lane 0, then the barrier
    if (threadIdx.x == 0) osc_acquire();
    __syncthreads();
    using F = opfn<OP, false>;
    int64_t done = 0;
    if constexpr (16 % sizeof(T) == 0) {
        constexpr int E = 16 / sizeof(T);
        constexpr int64_t chunk = (int64_t)kOscThreads * kOscUnroll;
        if (vec) {
            const int64_t nv = n / E;
            const u32x4 *o = reinterpret_cast<const u32x4 *>(origin);
            u32x4 *t = reinterpret_cast<u32x4 *>(target);
            for (int64_t base = (int64_t)blockIdx.x * chunk + threadIdx.x; base < nv;
                 base += (int64_t)gridDim.x * chunk) {
                vec16<T> a[kOscUnroll], b[kOscUnroll];
#pragma unroll
                for (int u = 0; u < kOscUnroll; ++u) {
                    const int64_t i = base + (int64_t)u * kOscThreads;
                    if (i < nv) {
                        a[u].v = t[i];
                        b[u].v = __builtin_nontemporal_load(o + i);
                    }
                }
#pragma unroll
                for (int u = 0; u < kOscUnroll; ++u) {
                    const int64_t i = base + (int64_t)u * kOscThreads;
                    if (i < nv) {
                        vec16<T> r;
                        r.v = a[u].v;
#pragma unroll
                        for (int e = 0; e < E; ++e) r.e[e] = F::f(a[u].e[e], b[u].e[e]);
                        t[i] = r.v;
                    }
                }
            }
            done = nv * E;
        }
    }
    const int64_t gs = (int64_t)gridDim.x * kOscThreads;
    for (int64_t i = done + (int64_t)blockIdx.x * kOscThreads + threadIdx.x; i < n; i += gs) {
        const T r = F::f(target[i], origin[i]);
        store_elem(target + i, r);
    }
    if (sys) osc_epilogue();
}

// Byte copy for put / get / fetches and the p2p receive: 16-B granules
// (UNROLL in flight per lane) when src and dst share their phase mod 16,
// else 4-B or 1-B granules; one acquire per workgroup, persistent grid (as
// acc_kernel).
template <int THREADS, int UNROLL>
__device__ __forceinline__ void xfer_body(const char *src, char *dst, int64_t bytes) {
    const uintptr_t phase = (uintptr_t)src ^ (uintptr_t)dst;
    const int g = (phase & 15) == 0 ? 16 : ((phase & 3) == 0 ? 4 : 1);
    int64_t head = (int64_t)((g - ((uintptr_t)src & (uintptr_t)(g - 1))) & (uintptr_t)(g - 1));
    if (head > bytes) head = bytes;
    const int64_t nbody = (bytes - head) / g;
    const int64_t tid = (int64_t)blockIdx.x * THREADS + threadIdx.x;
    if (g == 16) {
        const u32x4 *sv = reinterpret_cast<const u32x4 *>(src + head);
        u32x4 *dv = reinterpret_cast<u32x4 *>(dst + head);
        constexpr int64_t chunk = (int64_t)THREADS * UNROLL;
        for (int64_t base = (int64_t)blockIdx.x * chunk + threadIdx.x; base < nbody;
             base += (int64_t)gridDim.x * chunk) {
            u32x4 v[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const int64_t i = base + (int64_t)u * THREADS;
                if (i < nbody) v[u] = __builtin_nontemporal_load(sv + i);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const int64_t i = base + (int64_t)u * THREADS;
                if (i < nbody) __builtin_nontemporal_store(v[u], dv + i);
            }
        }
    } else if (g == 4) {
        const uint32_t *sw = reinterpret_cast<const uint32_t *>(src + head);
        uint32_t *dw = reinterpret_cast<uint32_t *>(dst + head);
        for (int64_t i = tid; i < nbody; i += (int64_t)gridDim.x * THREADS) dw[i] = sw[i];
    } else {
        for (int64_t i = tid; i < nbody; i += (int64_t)gridDim.x * THREADS)
            dst[head + i] = src[head + i];
    }
    const int64_t tail0 = head + nbody * g;
    const int64_t nrest = head + (bytes - tail0);
    for (int64_t k = tid; k < nrest; k += (int64_t)gridDim.x * THREADS) {
        const int64_t i = k < head ? k : tail0 + (k - head);
        dst[i] = src[i];
    }
}

// SYS: every workgroup ends with a system-scope release of its stores —
// for a destination on another GPU (a peer's window over xGMI), where a
// write-back at the runtime's end-of-dispatch scope is not known here to
// cover the remote lines.  A destination on this GPU (the caller's own
// buffer, a window of a rank on the same device) is consumed after a kernel
// boundary, whose release covers it: no per-workgroup release (~10 % of a
// 256 MiB copy).
template <int THREADS, int UNROLL, bool SYS>
__global__ __launch_bounds__(THREADS) void xfer_kernel(const char *src, char *dst, int64_t bytes,
                                                       const uint32_t *gate) {
    if (!gate_open(gate)) return;
    if (threadIdx.x == 0) osc_acquire();
    __syncthreads();
    xfer_body<THREADS, UNROLL>(src, dst, bytes);
    if constexpr (SYS) osc_epilogue();
}

// xfer_kernel with the signalling of comm_internal.h's xfer_sig.
template <int THREADS, int UNROLL>
__global__ __launch_bounds__(THREADS) void xfer_sig_kernel(const char *src, char *dst, int64_t bytes,
                                                           xfer_sig sg) {
    __shared__ int ok;
    if (threadIdx.x == 0) {
        ok = 1;
        if (sg.wait) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(sg.wait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != sg.wait_v) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > sg.ticks) {
                    __hip_atomic_store(sg.err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                    ok = 0;
                    break;
                }
            }
        }
        osc_acquire();
    }
    __syncthreads();
    if (ok) xfer_body<THREADS, UNROLL>(src, dst, bytes);
    osc_epilogue();  // this workgroup's stores released at system scope
    if (threadIdx.x != 0 || (!sg.flag && !sg.mark)) return;
    if (gridDim.x > 1) {
        // the last workgroup to finish signals (its acquire-release RMW
        // orders every other workgroup's released stores before the flag)
        const uint32_t prev = __hip_atomic_fetch_add(sg.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
        if (prev != gridDim.x - 1) return;
        __hip_atomic_store(sg.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        osc_release();
    }
    if (sg.flag) __hip_atomic_store(sg.flag, sg.flag_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (sg.mark) __hip_atomic_store(sg.mark, sg.mark_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Compare-and-swap of one element of `size` data bytes (osc_sm_comm.c:386-396).
// Under the target's accumulate lock, taken and released in this one launch
// (as rma_small_kernel).
__global__ __launch_bounds__(64) void cas_kernel(const unsigned char *origin,
                                                 const unsigned char *compare,
                                                 unsigned char *result, unsigned char *target,
                                                 int size, uint32_t *ctl, int *err, uint64_t ticks) {
    if (threadIdx.x != 0) return;
    if (!acc_lock_take(ctl, err, ticks)) return;
    osc_acquire();
    unsigned char old[16];
    bool same = true;
    for (int b = 0; b < size; ++b) {
        old[b] = target[b];
        result[b] = old[b];
        same = same && old[b] == compare[b];
    }
    if (same)
        for (int b = 0; b < size; ++b) target[b] = origin[b];
    osc_release();
    __hip_atomic_store(ctl + CTL_ACC, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

using acc_launch_fn = hipError_t (*)(dim3, const void *, void *, int64_t, int, const uint32_t *,
                                     int, hipStream_t);

template <int OP, int TYPE>
static hipError_t acc_launch_slot(dim3 grid, const void *o, void *t, int64_t n, int vec,
                                  const uint32_t *gate, int sys, hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        using T = typename type_of<TYPE>::type;
        hipLaunchKernelGGL((acc_kernel<T, OP>), grid, dim3(kOscThreads), 0, s,
                           static_cast<const T *>(o), static_cast<T *>(t), n, vec, gate, sys);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}
template <int OP, int... T>
static constexpr std::array<acc_launch_fn, OMPI_AMD_TYPE_COUNT> make_acc_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &acc_launch_slot<OP, T> : (acc_launch_fn) nullptr)...}};
}
template <int... O>
static constexpr std::array<std::array<acc_launch_fn, OMPI_AMD_TYPE_COUNT>, OMPI_AMD_OP_COUNT>
make_acc_table(std::integer_sequence<int, O...>) {
    return {{make_acc_row<O>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}
static const auto g_acc = make_acc_table(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});

// Small accumulate-lock operations in ONE single-workgroup launch: take the
// target's accumulate lock, fetch the old elements (get_accumulate /
// fetch_and_op), combine or replace, release, unlock — osc_sm_comm.c's
// opal_atomic_lock / copy + ompi_op_reduce / opal_atomic_unlock sequence
// (:296-305, :340-356, :424-438) with the lock held inside one kernel
// instead of across three or four launches (lock, fetch copy, op, unlock).
// MODE: 0 replace, 1 combine with OP, 2 fetch only (NO_OP).  T: the
// element type (MODE 1) or the widest granule both pointers and the byte
// count allow (MODE 0 / 2: bytes move unchanged).
enum { RMA_REPLACE = 0, RMA_COMBINE = 1, RMA_FETCH = 2 };
constexpr size_t kRmaSmallBytes = 16 << 10;

template <typename T, int OP, int MODE>
__global__ __launch_bounds__(kOscThreads) void rma_small_kernel(const T *origin, T *result, T *target,
                                                                int64_t n, uint32_t *ctl, int *err,
                                                                uint64_t ticks) {
    __shared__ int ok;
    if (threadIdx.x == 0) {
        ok = acc_lock_take(ctl, err, ticks) ? 1 : 0;
        if (ok) osc_acquire();
    }
    __syncthreads();
    if (!ok) return;
    for (int64_t i = threadIdx.x; i < n; i += kOscThreads) {
        const T old = target[i];
        if (result) result[i] = old;
        if constexpr (MODE == RMA_REPLACE) {
            target[i] = origin[i];
        } else if constexpr (MODE == RMA_COMBINE) {
            store_elem(target + i, opfn<OP, false>::f(old, origin[i]));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        osc_release();
        __hip_atomic_store(ctl + CTL_ACC, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

using rma_small_fn = hipError_t (*)(const void *, void *, void *, int64_t, uint32_t *, int *, uint64_t,
                                    hipStream_t);

template <typename T, int OP, int MODE>
static hipError_t rma_small_launch(const void *o, void *r, void *t, int64_t n, uint32_t *ctl, int *err,
                                   uint64_t ticks, hipStream_t s) {
    hipLaunchKernelGGL((rma_small_kernel<T, OP, MODE>), dim3(1), dim3(kOscThreads), 0, s,
                       static_cast<const T *>(o), static_cast<T *>(r), static_cast<T *>(t), n, ctl, err,
                       ticks);
    return hipGetLastError();
}
template <int OP, int TYPE>
static constexpr rma_small_fn rma_small_slot() {
    if constexpr (slot_supported(OP, TYPE))
        return &rma_small_launch<typename type_of<TYPE>::type, OP, RMA_COMBINE>;
    else
        return nullptr;
}
template <int OP, int... T>
static constexpr std::array<rma_small_fn, OMPI_AMD_TYPE_COUNT> make_small_row(std::integer_sequence<int, T...>) {
    return {{rma_small_slot<OP, T>()...}};
}
template <int... O>
static constexpr std::array<std::array<rma_small_fn, OMPI_AMD_TYPE_COUNT>, OMPI_AMD_OP_COUNT>
make_small_table(std::integer_sequence<int, O...>) {
    return {{make_small_row<O>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}
static const auto g_rma_small = make_small_table(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});

// replace / fetch-only by granule (16, 8, 4, 2, 1 bytes)
template <int MODE>
static rma_small_fn rma_small_bytes_fn(int g) {
    switch (g) {
    case 16: return &rma_small_launch<u32x4, 0, MODE>;
    case 8: return &rma_small_launch<uint64_t, 0, MODE>;
    case 4: return &rma_small_launch<uint32_t, 0, MODE>;
    case 2: return &rma_small_launch<uint16_t, 0, MODE>;
    default: return &rma_small_launch<uint8_t, 0, MODE>;
    }
}

// ---- derived datatypes at the target (ompi_osc_base_sndrcv_op,
// osc_base_obj_convert.c:160-245): the origin's packed stream of primitive
// elements is combined in order into the primitive slots the target
// datatype describes.  Element k of the stream sits at
// typed_offset(k * sizeof(T)) of the target; one lane per element, the
// datatype program in LDS (ddt_kernel's position -> address mapping).
// old (get_accumulate; else null): the target's elements before the update,
// packed.  OP 0: replace (REPLACE), -1: none (NO_OP: fetch only).
// Target position k (in elements of T) -> typed byte offset.  FAST: every
// quantity in element units fits 32 bits and each run length has its
// multiply-high divisor (ddt_device.h), instead of two 64-bit divisions
// per element.
template <typename T, bool FAST>
__device__ __forceinline__ int64_t acc_offset(const ddt_desc &d, const ddt_elem *el, int nelem,
                                              int64_t k) {
    if constexpr (FAST)
        return typed_offset_fast<(int)sizeof(T)>(el, nelem, (uint32_t)(d.size / (int64_t)sizeof(T)),
                                                 d.sdiv, d.extent, (uint32_t)k);
    else
        return typed_offset<uint64_t>(el, nelem, (uint64_t)d.size, d.extent, (uint64_t)k * sizeof(T));
}

// Derived-target accumulate: element k of the packed origin stream `in`
// combines into the k-th primitive slot of the target datatype.  Four
// elements per lane per pass, their loads issued before any store.
constexpr int kAccUnroll = 4;
template <typename T, int OP, bool FAST>
__device__ __forceinline__ void ddt_acc_body(const ddt_desc &d, const ddt_elem *el, int nelem, char *typed,
                                             const T *in, T *old, int64_t n) {
    const int64_t chunk = (int64_t)kOscThreads * kAccUnroll;
    const int64_t gs = (int64_t)gridDim.x * chunk;
    for (int64_t b = (int64_t)blockIdx.x * chunk + threadIdx.x; b < n; b += gs) {
        T *t[kAccUnroll];
        T v[kAccUnroll], x[kAccUnroll];
#pragma unroll
        for (int u = 0; u < kAccUnroll; ++u) {
            const int64_t k = b + (int64_t)u * kOscThreads;
            t[u] = nullptr;
            if (k < n) {
                t[u] = reinterpret_cast<T *>(typed + acc_offset<T, FAST>(d, el, nelem, k));
                v[u] = *t[u];
                if constexpr (OP >= 0) x[u] = in[k];
            }
        }
#pragma unroll
        for (int u = 0; u < kAccUnroll; ++u) {
            const int64_t k = b + (int64_t)u * kOscThreads;
            if (!t[u]) continue;
            if (old) old[k] = v[u];
            if constexpr (OP == 0) {
                *t[u] = x[u];
            } else if constexpr (OP > 0) {
                store_elem(t[u], opfn<OP, false>::f(v[u], x[u]));
            }
        }
    }
}

// The element table's address space must be known where the loop reads it
// (else every read is a flat load, five per element: 1.70 TB/s on the
// bench's vector target, against 2.73 TB/s for the same loop reading LDS,
// tools/ddt_acc_probe.hip): a single-element type (every vector) keeps its
// element in registers (a constant nelem of 1 lets the compiler scalarise
// it), up to kDdtLdsElems stage in LDS, longer tables stay in global memory.
template <typename T, int OP, bool FAST>
__global__ __launch_bounds__(kOscThreads) void ddt_acc_kernel(ddt_desc d, char *typed, const T *in,
                                                              T *old, int64_t n,
                                                              const uint32_t *gate, int sys) {
    if (!gate_open(gate)) return;
    __shared__ ddt_elem lds[kDdtLdsElems];
    if (threadIdx.x == 0) osc_acquire();
    if (d.nelem == 1) {
        const ddt_elem e0 = d.elems[0];
        __syncthreads();
        ddt_acc_body<T, OP, FAST>(d, &e0, 1, typed, in, old, n);
    } else if (d.nelem <= kDdtLdsElems) {
        for (int i = threadIdx.x; i < d.nelem; i += kOscThreads) lds[i] = d.elems[i];
        __syncthreads();
        ddt_acc_body<T, OP, FAST>(d, lds, d.nelem, typed, in, old, n);
    } else {
        __syncthreads();
        ddt_acc_body<T, OP, FAST>(d, d.elems, d.nelem, typed, in, old, n);
    }
    if (sys) osc_epilogue();  // sys: the target is another GPU's memory (acc_kernel)
}

using ddt_acc_fn = hipError_t (*)(dim3, const ddt_desc &, char *, const void *, void *, int64_t,
                                  const uint32_t *, bool, hipStream_t, int);

// ---- derived datatypes of pair type (MAXLOC / MINLOC operands) ----
// ompi_osc_base_sndrcv_op (osc_base_obj_convert.c:73-245) converts the
// origin into the target's primitive slots element by element; a pair's
// packed element is its members back to back (DOUBLE_INT: 8 + 4 = 12 bytes)
// while its memory element carries the struct's padding (16 bytes, the
// int at offset 8; SHORT_INT: the int at offset 4 after 2 bytes of gap).
// One lane per pair: each member is located on its own — through the
// target program (the member's packed position -> typed offset, so a
// program whose runs split a pair still maps each member), or at
// k * extent + its struct offset for a contiguous side — loaded bytewise
// (a packed double need not be 8-byte aligned), combined with op/base's
// LOC rule (f(target, origin), the 2-buffer form), and only the members'
// bytes are stored: a pair's gap bytes in the window stay as they were.
// OP 0 replace, -1 fetch only.
struct pair_side {
    char *p;        // the stream or buffer
    int64_t stride; // bytes per pair: the packed size, or the extent
    int32_t koff;   // byte offset of the index member within one pair
};

template <typename S>
__device__ __forceinline__ void pair_ld(const char *a, const char *b, S *x) {
    __builtin_memcpy(&x->v, a, sizeof(x->v));
    __builtin_memcpy(&x->k, b, sizeof(x->k));
}

template <typename S, int OP>
__global__ __launch_bounds__(kOscThreads) void ddt_pair_kernel(ddt_desc d, char *typed, pair_side in,
                                                               pair_side old, int64_t n,
                                                               const uint32_t *gate) {
    if (!gate_open(gate)) return;
    if (threadIdx.x == 0) osc_acquire();
    __syncthreads();
    constexpr int64_t P = (int64_t)(sizeof(S::v) + sizeof(S::k));  // packed pair
    const int64_t gs = (int64_t)gridDim.x * kOscThreads;
    for (int64_t k = (int64_t)blockIdx.x * kOscThreads + threadIdx.x; k < n; k += gs) {
        char *tv, *tk;
        if (d.nelem > 0) {
            tv = typed + typed_offset<uint64_t>(d.elems, d.nelem, (uint64_t)d.size, d.extent, (uint64_t)(k * P));
            tk = typed + typed_offset<uint64_t>(d.elems, d.nelem, (uint64_t)d.size, d.extent,
                                                (uint64_t)(k * P + (int64_t)sizeof(S::v)));
        } else {  // contiguous target: memory pairs
            tv = typed + k * (int64_t)sizeof(S);
            tk = tv + offsetof(S, k);
        }
        S x;
        pair_ld(tv, tk, &x);
        if (old.p) {
            char *o = old.p + k * old.stride;
            __builtin_memcpy(o, &x.v, sizeof(x.v));
            __builtin_memcpy(o + old.koff, &x.k, sizeof(x.k));
        }
        if constexpr (OP >= 0) {
            const char *ip = in.p + k * in.stride;
            S y;
            pair_ld(ip, ip + in.koff, &y);
            S r = y;
            if constexpr (OP > 0) r = opfn<OP, false>::f(x, y);
            __builtin_memcpy(tv, &r.v, sizeof(r.v));
            __builtin_memcpy(tk, &r.k, sizeof(r.k));
        }
    }
    osc_epilogue();
}

using pair_fn = void (*)(dim3, const ddt_desc &, char *, pair_side, pair_side, int64_t, const uint32_t *,
                         hipStream_t);
template <typename S, int OP>
static void pair_launch(dim3 grid, const ddt_desc &d, char *typed, pair_side in, pair_side old, int64_t n,
                        const uint32_t *gate, hipStream_t s) {
    hipLaunchKernelGGL((ddt_pair_kernel<S, OP>), grid, dim3(kOscThreads), 0, s, d, typed, in, old, n, gate);
}
template <typename S>
static pair_fn pair_fn_of(int op) {
    switch (op) {
    case OMPI_AMD_OP_MAXLOC: return &pair_launch<S, OMPI_AMD_OP_MAXLOC>;
    case OMPI_AMD_OP_MINLOC: return &pair_launch<S, OMPI_AMD_OP_MINLOC>;
    case OMPI_AMD_OP_REPLACE: return &pair_launch<S, 0>;
    case OMPI_AMD_OP_NO_OP: return &pair_launch<S, -1>;
    default: return nullptr;
    }
}
// (fn, packed pair size, struct size, index member offset) of a pair type
static bool pair_info(int type, int op, pair_fn *f, int64_t *packed, int64_t *ext, int32_t *koff) {
    switch (type) {
#define PAIR(T, S)                                                     \
    case T:                                                            \
        *f = pair_fn_of<S>(op);                                        \
        *packed = (int64_t)(sizeof(S::v) + sizeof(S::k));              \
        *ext = (int64_t)sizeof(S);                                     \
        *koff = (int32_t)offsetof(S, k);                               \
        return *f != nullptr;
        PAIR(OMPI_AMD_TYPE_FLOAT_INT, float_int_t)
        PAIR(OMPI_AMD_TYPE_DOUBLE_INT, double_int_t)
        PAIR(OMPI_AMD_TYPE_LONG_INT, long_int_t)
        PAIR(OMPI_AMD_TYPE_2INT, two_int_t)
        PAIR(OMPI_AMD_TYPE_SHORT_INT, short_int_t)
#undef PAIR
    default: return false;
    }
}

template <typename T, int OP>
static hipError_t ddt_acc_launch(dim3 grid, const ddt_desc &d, char *typed, const void *in,
                                 void *old, int64_t n, const uint32_t *gate, bool fast, hipStream_t s,
                                 int sys) {
    if (fast)  // d.sdiv holds size / sizeof(T)
        hipLaunchKernelGGL((ddt_acc_kernel<T, OP, true>), grid, dim3(kOscThreads), 0, s, d, typed,
                           static_cast<const T *>(in), static_cast<T *>(old), n, gate, sys);
    else
        hipLaunchKernelGGL((ddt_acc_kernel<T, OP, false>), grid, dim3(kOscThreads), 0, s, d, typed,
                           static_cast<const T *>(in), static_cast<T *>(old), n, gate, sys);
    return hipGetLastError();
}
template <int OP, int TYPE>
static constexpr ddt_acc_fn ddt_acc_slot() {
    if constexpr (slot_supported(OP, TYPE) && !is_pair_type(TYPE))
        return &ddt_acc_launch<typename type_of<TYPE>::type, OP>;
    else
        return nullptr;
}
template <int OP, int... T>
static constexpr std::array<ddt_acc_fn, OMPI_AMD_TYPE_COUNT> make_ddt_acc_row(
    std::integer_sequence<int, T...>) {
    return {{ddt_acc_slot<OP, T>()...}};
}
template <int... O>
static constexpr std::array<std::array<ddt_acc_fn, OMPI_AMD_TYPE_COUNT>, OMPI_AMD_OP_COUNT>
make_ddt_acc_table(std::integer_sequence<int, O...>) {
    return {{make_ddt_acc_row<O>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{})...}};
}
static const auto g_ddt_acc = make_ddt_acc_table(std::make_integer_sequence<int, OMPI_AMD_OP_COUNT>{});

// replace / fetch-only by element size (any non-pair type of that size)
template <int SZ> struct sized;
template <> struct sized<1> { using t = uint8_t; };
template <> struct sized<2> { using t = uint16_t; };
template <> struct sized<4> { using t = uint32_t; };
template <> struct sized<8> { using t = uint64_t; };
template <> struct sized<16> { typedef unsigned int t __attribute__((ext_vector_type(4))); };
static ddt_acc_fn ddt_rw_fn(size_t size, bool replace) {
    switch (size) {
#define RW(SZ) case SZ: return replace ? &ddt_acc_launch<sized<SZ>::t, 0> : &ddt_acc_launch<sized<SZ>::t, -1>;
        RW(1) RW(2) RW(4) RW(8) RW(16)
#undef RW
    default: return nullptr;
    }
}

struct win_blob {
    ipc_desc base;
    uint64_t bytes;
    int64_t disp_unit;
    int64_t failed;    // this rank could not set up its side
    int64_t shadowed;  // this rank's window runs through a public copy (separate model)
};

}  // namespace ompi_amd

using namespace ompi_amd;

// A request-based RMA call (MPI_Rput / _Rget / _Raccumulate /
// _Rget_accumulate): an event recorded after the call's kernels.
struct ompi_amd_rma_request {
    hipEvent_t ev = nullptr;
    ompi_amd_win_t *w = nullptr;
};

struct ompi_amd_win {
    ompi_amd_comm_t *c = nullptr;
    int rank = 0, size = 0;
    char *base = nullptr;
    size_t bytes = 0;
    bool owns_base = false;   // hipMalloc'd by win_allocate (past the arena's limit)
    bool arena_base = false;  // from the communicator's exported arena
    uint32_t *ctl = nullptr;
    char *peer_base[kOscMaxRanks] = {};
    uint32_t *peer_ctl[kOscMaxRanks] = {};
    uint64_t peer_bytes[kOscMaxRanks] = {};
    int64_t peer_disp[kOscMaxRanks] = {};
    // target's window memory on another GPU than this rank's: copies into it
    // end with a per-workgroup system-scope release (xfer_kernel SYS)
    bool peer_remote[kOscMaxRanks] = {};
    void *pinned[kOscMaxRanks] = {};
    int ctl_slot = -1;  // this window's page in the communicator's control arena
    std::vector<hipStream_t> streams;  // every stream an epoch or RMA call ran on (win_free waits)
    int held[kOscMaxRanks] = {};  // outstanding passive lock per target (0 none)
    // general active target synchronisation (host side of the counters)
    bool posted = false, started = false;
    uint32_t post_seen[kOscMaxRanks] = {};  // exposure epochs of rank t this rank started toward
    uint32_t complete_want = 0;             // access epochs origins must have closed here
    std::vector<int> start_group;
    hipStream_t query = nullptr;  // MPI_Win_test's counter reads
    // MPI_Win_allocate_shared: one allocation on rank 0 holds every rank's
    // segment back to back; the others map it once
    bool shared = false;
    char *shared_seg = nullptr;   // rank 0: the allocation; others: their mapping
    void *shared_pin = nullptr;   // others: the pinned import of rank 0's allocation
    bool shared_owner = false;    // rank 0: frees shared_seg (arena or hipFree)
    bool shared_arena = false;
    // MPI_Win_create over memory peers cannot map reliably (no IPC-safe
    // size, or older than an IPC close of this process):
    // the window runs in MPI's separate memory model — peers' RMA reaches a
    // public copy in the exported arena (shadow), the owner's own loads and
    // stores the private copy (base), and every synchronisation merges them
    // against the state of the last one (snap).  separate: some rank of the
    // window has a shadow (every rank then takes part in the fence's merge
    // step and reports MPI_WIN_SEPARATE).
    char *shadow = nullptr;
    char *snap = nullptr;
    bool owns_shadow = false;  // past the arena's limit: hipFree'd, not returned to the arena
    bool separate = false;
    // MPI_Win_create_dynamic: every rank's attached regions in a host
    // shared-memory table (one slot per rank, a sequence lock each), and
    // this process's mappings of peers' regions (pinned until win_free)
    bool dynamic = false;
    struct dyn_table *dyn = nullptr;
    size_t dyn_bytes = 0;
    struct dyn_map {
        int target;
        uint64_t base, size, id, abase;
        const char *p;
        void *pin;
    };
    std::vector<dyn_map> dyn_maps;
    // packed-stream scratch of the derived-datatype calls (osc_scratch)
    char *scr[2] = {};
    size_t scr_cap[2] = {};
    std::vector<char *> scr_old;  // buffers a growth replaced (kernels may still read them)
    hipEvent_t scr_ev = nullptr;  // after the last call's use, on scr_last
    hipStream_t scr_last = nullptr;
};

#define OSC_TRY(x)                               \
    do {                                         \
        int rc_ = (x);                           \
        if (rc_ != OMPI_AMD_SUCCESS) return rc_; \
    } while (0)

// Scratch of a derived-datatype call (the origin's packed stream, the
// fetched result stream): two regions kept for the window's life and grown
// geometrically, ordered between calls by stream order — a call on another
// stream than the previous user's first waits for that use (an event).
// Not the stream-ordered pool (hipMallocAsync / hipFreeAsync): with it, a
// derived get at N = 3 on one GPU intermittently unpacked zeros for part of
// the fetched stream (1 of 12 repeats, 4 of 12 with a one-workgroup fetch);
// with this scratch 0 of 48 (tools/osc_flake_probe.sh).
static int osc_scratch(ompi_amd_win_t *w, hipStream_t s, int slot, size_t bytes, void **out) {
    *out = nullptr;
    if (w->scr_last && w->scr_last != s && w->scr_ev)
        OSC_TRY(record_hip(hipStreamWaitEvent(s, w->scr_ev, 0), "hipStreamWaitEvent (osc scratch)"));
    w->scr_last = nullptr;  // until osc_scratch_done records this call's use
    if (bytes > w->scr_cap[slot]) {
        const size_t want = std::max(bytes, 2 * w->scr_cap[slot]);
        void *p = nullptr;
        ipc_desc d;  // recycled memory (comm_release_exportable), not exported
        OSC_TRY(comm_alloc_exportable(want, false, &p, &d));
        if (w->scr[slot]) w->scr_old.push_back(w->scr[slot]);
        w->scr[slot] = static_cast<char *>(p);
        w->scr_cap[slot] = want;
    }
    *out = w->scr[slot];
    return OMPI_AMD_SUCCESS;
}

static void osc_scratch_done(ompi_amd_win_t *w, hipStream_t s) {
    if (!w->scr_ev && hipEventCreateWithFlags(&w->scr_ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        w->scr_ev = nullptr;
    }
    if (w->scr_ev && hipEventRecord(w->scr_ev, s) == hipSuccess) {
        w->scr_last = s;
    } else {
        (void)hipGetLastError();
        hip_ignore(hipStreamSynchronize(s));  // no event: the next user must not overtake this one
    }
}

// ---- dynamic windows (MPI_Win_create_dynamic / _attach / _detach;
// osc/rdma's region table, osc_rdma_dynamic.c:162-300, in host shared
// memory here: every attach is local, and an origin finds the target's
// region — its absolute address is the displacement — when it accesses it)
constexpr int kDynRegions = 64;
struct dyn_region {
    uint64_t base, size;
    ompi_amd::ipc_desc d;  // the attached device memory, exported at attach
};
struct dyn_table {
    std::atomic<uint64_t> version;  // odd while the owner edits its regions
    uint32_t n, pad;
    dyn_region r[kDynRegions];
};

namespace ompi_amd {

enum { HELD_NONE = 0, HELD_EXCLUSIVE = 1, HELD_SHARED = 2, HELD_NOCHECK = 3 };

// A consistent copy of rank t's region table (the owner's sequence lock).
static int dyn_read(ompi_amd_win_t *w, int t, dyn_table *out) {
    const dyn_table &src = w->dyn[t];
    for (int spin = 0; spin < (1 << 20); ++spin) {
        const uint64_t v1 = src.version.load(std::memory_order_acquire);
        if (v1 & 1) continue;
        out->n = std::min<uint32_t>(src.n, kDynRegions);
        memcpy(out->r, src.r, sizeof(dyn_region) * out->n);
        std::atomic_thread_fence(std::memory_order_acquire);
        if (src.version.load(std::memory_order_relaxed) == v1) return OMPI_AMD_SUCCESS;
    }
    record_msg("osc: rank %d's dynamic region table stayed busy", t);
    return OMPI_AMD_ERR_TIMEOUT;
}

static int dyn_resolve(ompi_amd_win_t *w, int target, int64_t lo, int64_t hi, char **out) {
    static thread_local dyn_table tab;
    OSC_TRY(dyn_read(w, target, &tab));
    for (uint32_t i = 0; i < tab.n; ++i) {
        const dyn_region &r = tab.r[i];
        if ((uint64_t)lo < r.base || (uint64_t)hi > r.base + r.size) continue;
        if (target == w->rank) {  // own memory: the address itself
            *out = reinterpret_cast<char *>((uintptr_t)lo);
            return OMPI_AMD_SUCCESS;
        }
        for (const auto &m : w->dyn_maps)
            if (m.target == target && m.base == r.base && m.size == r.size && m.id == r.d.id &&
                m.abase == r.d.base) {
                *out = const_cast<char *>(m.p) + (lo - (int64_t)r.base);
                return OMPI_AMD_SUCCESS;
            }
        ompi_amd_win::dyn_map m{target, r.base, r.size, r.d.id, r.d.base, nullptr, nullptr};
        OSC_TRY(comm_import(w->c, target, r.d, &m.p, true, &m.pin));
        w->dyn_maps.push_back(m);
        *out = const_cast<char *>(m.p) + (lo - (int64_t)r.base);
        return OMPI_AMD_SUCCESS;
    }
    record_msg("osc: [0x%llx, 0x%llx) is not inside a region rank %d attached to the dynamic window",
               (unsigned long long)lo, (unsigned long long)hi, target);
    return OMPI_AMD_ERR_BAD_PARAM;
}

static uint64_t ticks_of(ompi_amd_win_t *w) {
    return (uint64_t)comm_timeout_ms(w->c) * 100000ull;  // s_memrealtime: 100 MHz
}

// The origin's CTL_TAKEN_* word for (lock kind, target).
static uint32_t *taken_word(ompi_amd_win_t *w, int target, bool acc) {
    return w->ctl + (acc ? CTL_TAKEN_ACC : CTL_TAKEN_EPOCH) + target;
}

// The gate of a data kernel toward `target` inside a passive-target epoch
// this rank locked (NULL: fence / NOCHECK / no epoch — nothing to check).
static const uint32_t *epoch_gate(ompi_amd_win_t *w, int target);

static int launch_lock(ompi_amd_win_t *w, int target, int kind, hipStream_t s) {
    hipLaunchKernelGGL(lock_kernel, dim3(1), dim3(64), 0, s, w->peer_ctl[target], kind,
                       comm_err_dev(w->c), ticks_of(w), taken_word(w, target, kind <= 1));
    return record_hip(hipGetLastError(), "osc lock launch");
}

static const uint32_t *epoch_gate(ompi_amd_win_t *w, int target) {
    const int h = w->held[target];
    return (h == HELD_EXCLUSIVE || h == HELD_SHARED) ? taken_word(w, target, false) : nullptr;
}

static int dyn_resolve(ompi_amd_win_t *w, int target, int64_t lo, int64_t hi, char **out);

// The address, in this process, of byte `base` of target's window, after
// checking that [base + lo, base + hi) lies inside it: inside the window's
// bytes, or — a dynamic window (MPI_Win_create_dynamic), whose
// displacements are the target's absolute addresses — inside one region the
// target attached.
static int target_span(ompi_amd_win_t *w, int target, int64_t base, int64_t lo, int64_t hi, char **out) {
    if (target < 0 || target >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    if (w->dynamic) {
        char *p = nullptr;
        OSC_TRY(dyn_resolve(w, target, base + lo, base + hi, &p));
        *out = p - lo;
        return OMPI_AMD_SUCCESS;
    }
    if (base + lo < 0 || base + hi > (int64_t)w->peer_bytes[target] || !w->peer_base[target]) {
        record_msg("osc: target %d range [%lld, %lld) outside its %llu-byte window", target,
                   (long long)(base + lo), (long long)(base + hi), (unsigned long long)w->peer_bytes[target]);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    *out = w->peer_base[target] + base;
    return OMPI_AMD_SUCCESS;
}

// Whether p (a mapping of a peer's window, or an origin buffer) is device
// memory of GPU `dev`; host memory and anything unknown count as not (the
// conservative copy, with the system-scope release).
static bool on_this_device(const void *p, int dev) {
    if (!p) return true;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice && a.device == dev;
}

// A copy into target's window needs the system-scope release (another
// GPU's memory, or a dynamic window's region, not classified).
static bool remote_dst(const ompi_amd_win_t *w, int target) {
    return w->dynamic || w->peer_remote[target];
}

// Target address of (target, disp) with room for `bytes`.
static int target_ptr(ompi_amd_win_t *w, int target, size_t disp, size_t bytes, char **out) {
    if (target < 0 || target >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    const int64_t off = (int64_t)((uint64_t)disp * (uint64_t)w->peer_disp[target]);
    if (bytes == 0) {  // an empty access (at the window's end, or anywhere in a dynamic window)
        if (w->dynamic) {
            *out = nullptr;
            return OMPI_AMD_SUCCESS;
        }
        if (off < 0 || (uint64_t)off > w->peer_bytes[target]) return OMPI_AMD_ERR_BAD_PARAM;
        *out = w->peer_base[target] ? w->peer_base[target] + off : nullptr;
        return OMPI_AMD_SUCCESS;
    }
    return target_span(w, target, off, 0, (int64_t)bytes, out);
}


static int64_t osc_grid_cap() {
    static const int64_t cap = [] {
        const char *e = getenv("OMPI_AMD_OSC_MAX_BLOCKS");
        return (e && atoll(e) > 0) ? atoll(e) : (int64_t)kOscMaxBlocks;
    }();
    return cap;
}

// Copy shape: 256 threads x 4 16-B vectors per lane.  256x8, 256x16, 512x8,
// 1024x4 and 1024x8 measured within noise of it (put 5.26-5.59 TB/s,
// profiles/r03_xfer_shape_sweep.txt): bytes in flight are not the limit,
// and neither is the store-acknowledgement wait (a software-pipelined body,
// loads of pass k+1 before stores of pass k, measured the same: 0.726 vs
// 0.722 of 8 TB/s, profiles/r03_xfer_probe.jsonl).  The limit is the grid:
// one chunk per workgroup reaches 0.775 without an acquire but 0.456 with
// one per workgroup, so the persistent grid (one acquire per CU) stays.
constexpr int kXferThreads = 256, kXferUnroll = 4;

int xfer_copy(const void *src, void *dst, size_t bytes, hipStream_t s, const uint32_t *gate,
              bool remote_dst) {
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    const int64_t units = (int64_t)(bytes / 16) + 1;
    const int64_t per = (int64_t)kXferThreads * kXferUnroll;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((units + per - 1) / per,
                                                                  osc_grid_cap()));
    if (remote_dst)
        hipLaunchKernelGGL((xfer_kernel<kXferThreads, kXferUnroll, true>), dim3((unsigned)blocks),
                           dim3(kXferThreads), 0, s, static_cast<const char *>(src),
                           static_cast<char *>(dst), (int64_t)bytes, gate);
    else
        hipLaunchKernelGGL((xfer_kernel<kXferThreads, kXferUnroll, false>), dim3((unsigned)blocks),
                           dim3(kXferThreads), 0, s, static_cast<const char *>(src),
                           static_cast<char *>(dst), (int64_t)bytes, gate);
    return record_hip(hipGetLastError(), "xfer copy launch");
}

// p2p eager cells (p2p.cpp).  One workgroup: at most 4 KiB, 16-B granules
// when both sides are 16-B aligned, else bytes.
__device__ __forceinline__ void eager_bytes(const char *src, char *dst, int64_t bytes) {
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
        const int64_t nv = bytes / 16;
        for (int64_t i = threadIdx.x; i < nv; i += blockDim.x)
            reinterpret_cast<u32x4 *>(dst)[i] = reinterpret_cast<const u32x4 *>(src)[i];
        for (int64_t i = nv * 16 + threadIdx.x; i < bytes; i += blockDim.x) dst[i] = src[i];
    } else {
        for (int64_t i = threadIdx.x; i < bytes; i += blockDim.x) dst[i] = src[i];
    }
}

// The sender's copy into its cell, then the cell's flag = v (system scope,
// after a release): the message is posted before this kernel runs, and the
// receiver's copy waits for the flag on the device instead of the sender
// waiting for this kernel on the host.
__global__ __launch_bounds__(256) void eager_put_kernel(const char *src, char *cell, int64_t bytes,
                                                        uint64_t *flag, uint64_t v, uint64_t *mark,
                                                        uint64_t mark_v) {
    eager_bytes(src, cell, bytes);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        osc_release();
        __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (mark) __hip_atomic_store(mark, mark_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The receiver's copy out of the sender's cell once its flag is v (bounded:
// past `ticks` the communicator's sticky error, nothing copied).
__global__ __launch_bounds__(256) void eager_get_kernel(const char *cell, char *dst, int64_t bytes,
                                                        const uint64_t *flag, uint64_t v, int *err,
                                                        uint64_t ticks, uint64_t *mark, uint64_t mark_v) {
    __shared__ int ok;
    if (threadIdx.x == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        ok = 1;
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != v) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                __hip_atomic_store(err, (int)OMPI_AMD_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                ok = 0;
                break;
            }
        }
        osc_acquire();
    }
    __syncthreads();
    if (ok) eager_bytes(cell, dst, bytes);
    osc_epilogue();
    // the host's completion word (also after a timeout: the host then reads
    // the communicator's sticky error)
    if (threadIdx.x == 0 && mark) __hip_atomic_store(mark, mark_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int eager_put(const void *src, char *cell, size_t bytes, uint64_t *flag, uint64_t v, uint64_t *mark,
              uint64_t mark_v, hipStream_t s) {
    hipLaunchKernelGGL(eager_put_kernel, dim3(1), dim3(256), 0, s, static_cast<const char *>(src), cell,
                       (int64_t)bytes, flag, v, mark, mark_v);
    return record_hip(hipGetLastError(), "p2p eager copy launch");
}

int eager_get(const char *cell, void *dst, size_t bytes, const uint64_t *flag, uint64_t v, int *err,
              uint64_t ticks, uint64_t *mark, uint64_t mark_v, hipStream_t s) {
    hipLaunchKernelGGL(eager_get_kernel, dim3(1), dim3(256), 0, s, cell, static_cast<char *>(dst),
                       (int64_t)bytes, flag, v, err, ticks, mark, mark_v);
    return record_hip(hipGetLastError(), "p2p eager receive launch");
}

int xfer_copy_sig(const void *src, void *dst, size_t bytes, hipStream_t s, const xfer_sig &sig) {
    const int64_t units = (int64_t)(bytes / 16) + 1;
    const int64_t per = (int64_t)kXferThreads * kXferUnroll;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((units + per - 1) / per,
                                                                  osc_grid_cap()));
    if (blocks > 1 && (sig.flag || sig.mark) && !sig.done) {
        record_msg("xfer_copy_sig: a multi-workgroup copy that signals needs a counter");
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    hipLaunchKernelGGL((xfer_sig_kernel<kXferThreads, kXferUnroll>), dim3((unsigned)blocks),
                       dim3(kXferThreads), 0, s, static_cast<const char *>(src), static_cast<char *>(dst),
                       (int64_t)bytes, sig);
    return record_hip(hipGetLastError(), "signalled copy launch");
}

static int launch_acc(ompi_amd_win_t *w, int op, int type, const void *origin, void *target,
                      size_t count, const uint32_t *gate, hipStream_t s, bool remote) {
    acc_launch_fn f = (op >= 0 && op < OMPI_AMD_OP_COUNT && type >= 0 && type < OMPI_AMD_TYPE_COUNT)
                          ? g_acc[op][type]
                          : nullptr;
    if (!f) {
        record_msg("osc accumulate: op %d on type %d is not provided", op, type);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    const size_t ext = ompi_amd_type_extent(type);
    const int vec = (16 % ext == 0 && ((uintptr_t)origin & 15) == 0 && ((uintptr_t)target & 15) == 0);
    const int64_t per = vec ? (int64_t)kOscThreads * kOscUnroll : (int64_t)kOscThreads;
    const int64_t units = vec ? (int64_t)(count * ext / 16) : (int64_t)count;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((units + per - 1) / per,
                                                                  osc_grid_cap()));
    return record_hip(f(dim3((unsigned)blocks), origin, target, (int64_t)count, vec, gate, remote ? 1 : 0, s),
                      "osc accumulate launch");
}


// The stream of a window call, remembered so that win_free waits for this
// window's work only (not for every stream of the device).
static hipStream_t win_stream(ompi_amd_win_t *w, void *stream) {
    const hipStream_t s = comm_call_stream(w->c, stream);
    if (std::find(w->streams.begin(), w->streams.end(), s) == w->streams.end()) w->streams.push_back(s);
    return s;
}

// rma_op's single-launch form (rma_small_kernel) up to this many bytes;
// OMPI_AMD_OSC_SMALL_BYTES overrides, 0 turns it off.
static size_t rma_small_bytes() {
    static const size_t v = [] {
        const char *e = getenv("OMPI_AMD_OSC_SMALL_BYTES");
        return e ? (size_t)atoll(e) : (size_t)kRmaSmallBytes;
    }();
    return v;
}

// accumulate / get_accumulate / fetch_and_op under the accumulate lock
// (osc_sm_comm.c:296-305, :340-356, :424-438).
static int rma_op(ompi_amd_win_t *w, const void *origin, void *result, size_t count, int type,
                  int target, size_t disp, int op, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    if (type < 0 || type >= OMPI_AMD_TYPE_COUNT || ompi_amd_type_extent(type) == 0)
        return OMPI_AMD_ERR_BAD_PARAM;
    if (op != OMPI_AMD_OP_REPLACE && op != OMPI_AMD_OP_NO_OP &&
        (op <= 0 || op >= OMPI_AMD_OP_COUNT || !g_acc[op][type])) {
        record_msg("osc accumulate: op %d on type %d is not provided", op, type);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    if (count == 0) return OMPI_AMD_SUCCESS;
    const size_t bytes = count * ompi_amd_type_extent(type);
    char *t = nullptr;
    OSC_TRY(target_ptr(w, target, disp, bytes, &t));
    hipStream_t s = win_stream(w, stream);
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    if (bytes <= rma_small_bytes()) {  // lock, fetch, combine, unlock: one launch
        rma_small_fn f = nullptr;
        int64_t n = (int64_t)count;
        if (op == OMPI_AMD_OP_REPLACE || op == OMPI_AMD_OP_NO_OP) {
            const uintptr_t a = (uintptr_t)origin | (uintptr_t)result | (uintptr_t)t | (uintptr_t)bytes;
            int g = 16;
            while (g > 1 && (a & (uintptr_t)(g - 1))) g >>= 1;
            f = op == OMPI_AMD_OP_REPLACE ? rma_small_bytes_fn<RMA_REPLACE>(g) : rma_small_bytes_fn<RMA_FETCH>(g);
            n = (int64_t)(bytes / (size_t)g);
        } else {
            f = g_rma_small[op][type];
        }
        if (f)
            return record_hip(f(origin, result, t, n, w->peer_ctl[target], comm_err_dev(w->c), ticks_of(w), s),
                              "osc small accumulate launch");
    }
    OSC_TRY(launch_lock(w, target, 0, s));
    const uint32_t *gate = taken_word(w, target, true);
    int rc = OMPI_AMD_SUCCESS;
    const bool remote = remote_dst(w, target);
    if (result) rc = xfer_copy(t, result, bytes, s, gate, !on_this_device(result, comm_device(w->c)));
    if (rc == OMPI_AMD_SUCCESS) {
        if (op == OMPI_AMD_OP_REPLACE) rc = xfer_copy(origin, t, bytes, s, gate, remote);
        else if (op != OMPI_AMD_OP_NO_OP) rc = launch_acc(w, op, type, origin, t, count, gate, s, remote);
    }
    const int urc = launch_lock(w, target, 1, s);  // always release
    return rc != OMPI_AMD_SUCCESS ? rc : urc;
}

// ---- control pages: one arena per communicator ----
// Every window needs a control page that every peer maps.  One exportable
// allocation per window meant one IPC open per peer per window, and opens
// of freshly recycled exporter ranges are what ROCm 7.2 refused ("invalid
// device pointer").  The pages come instead from an arena
// of the communicator — kCtlPerChunk pages per exportable, fine-grained
// allocation, mapped by every peer once, released with the communicator.
// Windows are created and freed collectively, in one order, so every rank
// takes the same slot; a freed window's page is zeroed before its slot is
// reused.
constexpr int kCtlPerChunk = 64;
constexpr size_t kCtlWords = CTL_BYTES / sizeof(uint32_t);

struct ctl_chunk {
    uint32_t *mine = nullptr;
    uint32_t *peer[kOscMaxRanks] = {};
    ipc_ref *ref[kOscMaxRanks] = {};
};

struct ctl_arena {
    std::vector<ctl_chunk> chunks;
    std::vector<char> used;  // per slot
    void *owner = nullptr;   // the communicator holding the chunks' mappings
};

static void ctl_arena_release(void *state, int phase) {
    auto *a = static_cast<ctl_arena *>(state);
    if (!a) return;
    if (phase == 0) {  // nobody reads our pages any more: drop the peers' mappings
        for (auto &ch : a->chunks)
            for (auto &r : ch.ref) {
                ipc_unmap(r, a->owner);
                r = nullptr;
            }
        return;
    }
    for (auto &ch : a->chunks)  // every peer dropped its mappings of ours
        if (ch.mine) comm_release_exportable(ch.mine);
    delete a;
}

// The lowest free slot (every rank alike), growing the arena by one chunk —
// a collective step every rank reaches at the same window — when none is
// free.  rc_in: this rank's state so far (it joins the rendezvous anyway).
static int ctl_take(ompi_amd_comm_t *c, int rc_in, int *slot) {
    *slot = -1;
    auto *a = static_cast<ctl_arena *>(comm_osc_state(c));
    if (!a) {
        a = new (std::nothrow) ctl_arena;
        if (!a) return OMPI_AMD_ERR_BAD_PARAM;  // every rank: the same allocation failure
        a->owner = c;
        comm_set_osc_state(c, a, ctl_arena_release);
    }
    for (size_t k = 0; k < a->used.size(); ++k)
        if (!a->used[k]) {
            a->used[k] = 1;
            *slot = (int)k;
            return rc_in;
        }
    const int me = comm_rank(c), n = comm_size(c);
    struct chunk_blob {
        ipc_desc d;
        int64_t failed;
    } mine{}, all[kOscMaxRanks];
    ctl_chunk ch;
    int rc = rc_in;
    if (rc == OMPI_AMD_SUCCESS) {
        rc = comm_alloc_exportable(CTL_BYTES * kCtlPerChunk, true, (void **)&ch.mine, &mine.d);
        if (rc == OMPI_AMD_SUCCESS)
            rc = record_hip(hipMemset(ch.mine, 0, CTL_BYTES * kCtlPerChunk), "osc control arena");
        if (rc == OMPI_AMD_SUCCESS)
            rc = record_hip(hipStreamSynchronize(nullptr), "osc control arena");
    }
    mine.failed = rc == OMPI_AMD_SUCCESS ? 0 : 1;
    const int arc = comm_allgather(c, &mine, all, sizeof(chunk_blob));
    if (rc == OMPI_AMD_SUCCESS) rc = arc;
    for (int p = 0; rc == OMPI_AMD_SUCCESS && p < n; ++p) {
        if (all[p].failed) {
            record_msg("osc control arena: rank %d could not allocate its chunk", p);
            rc = OMPI_AMD_ERR_BOOTSTRAP;
        } else if (p == me) {
            ch.peer[p] = ch.mine;
        } else {  // one attempt (a refused open is an error)
            void *m = nullptr;
            const ipc_desc &d = all[p].d;
            rc = ipc_map(ipc_alloc{d.h, d.pid, d.id, d.base, d.size}, c, &ch.ref[p], &m);
            ch.peer[p] = reinterpret_cast<uint32_t *>(static_cast<char *>(m) + d.off);
        }
    }
    int all_ok = 0;  // the chunk joins the arena on every rank or on none
    const int grc = ompi_amd_comm_agree(c, rc == OMPI_AMD_SUCCESS, &all_ok);
    if (rc == OMPI_AMD_SUCCESS && (grc != OMPI_AMD_SUCCESS || !all_ok))
        rc = grc != OMPI_AMD_SUCCESS ? grc : OMPI_AMD_ERR_BOOTSTRAP;
    if (rc != OMPI_AMD_SUCCESS) {
        for (auto &r : ch.ref) ipc_unmap(r, c);
        (void)comm_allgather(c, nullptr, nullptr, 0);  // every mapping closed before the free
        if (ch.mine) comm_release_exportable(ch.mine);
        return rc;
    }
    *slot = (int)a->used.size();
    a->chunks.push_back(ch);
    a->used.resize(a->used.size() + kCtlPerChunk, 0);
    a->used[(size_t)*slot] = 1;
    return OMPI_AMD_SUCCESS;
}

// rank p's control page of slot `slot` as this process maps it
static uint32_t *ctl_page(ompi_amd_comm_t *c, int slot, int p) {
    auto *a = static_cast<ctl_arena *>(comm_osc_state(c));
    return a->chunks[(size_t)slot / kCtlPerChunk].peer[p] + (size_t)(slot % kCtlPerChunk) * kCtlWords;
}

// after the window's last use everywhere: zero this rank's page, free the slot
static int ctl_give(ompi_amd_comm_t *c, int slot) {
    if (slot < 0) return OMPI_AMD_SUCCESS;
    auto *a = static_cast<ctl_arena *>(comm_osc_state(c));
    int rc = record_hip(hipMemset(ctl_page(c, slot, comm_rank(c)), 0, CTL_BYTES), "osc control page reset");
    if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipStreamSynchronize(nullptr), "osc control page reset");
    a->used[(size_t)slot] = 0;
    return rc;
}

// Three-way merge of a separate-model window (ompi_amd_win.shadow): byte b
// changed in the private copy since the last merge (p != s) -> the public
// copy takes it; else changed in the public copy (q != s) -> the private
// copy takes it; the snapshot becomes the merged value.  MPI forbids a
// local store and an RMA update of one location in the same epoch, so no
// byte changes on both sides.  Only changed bytes are stored into the two
// copies: an RMA of a passive epoch may still be updating other bytes of
// the public copy during MPI_Win_sync, and a stale rewrite would undo it.
// Words whose bytes all agree (the common case) cost three loads and no
// store.  HBM-bound: 3 x bytes read per merge, plus the changed words.
__global__ __launch_bounds__(kOscThreads) void win_merge_kernel(char *priv, char *pub, char *snap,
                                                                int64_t bytes) {
    if (threadIdx.x == 0) osc_acquire();  // the peers' released RMA into pub
    __syncthreads();
    const int64_t words = bytes / 4;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    uint32_t *p = reinterpret_cast<uint32_t *>(priv), *q = reinterpret_cast<uint32_t *>(pub),
             *sn = reinterpret_cast<uint32_t *>(snap);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words + (bytes % 4); i += gs) {
        if (i < words) {
            const uint32_t pv = p[i], qv = q[i], sv = sn[i];
            if (pv == sv && qv == sv) continue;
            uint32_t mv = 0;
            for (int k = 0; k < 4; ++k) {
                const uint32_t sh = 8u * (uint32_t)k;
                const uint8_t pb = (uint8_t)(pv >> sh), qb = (uint8_t)(qv >> sh), sb = (uint8_t)(sv >> sh);
                const uint8_t mb = pb != sb ? pb : qb;
                mv |= (uint32_t)mb << sh;
                if (pb != sb) reinterpret_cast<uint8_t *>(q + i)[k] = pb;
                else if (qb != sb) reinterpret_cast<uint8_t *>(p + i)[k] = qb;
            }
            sn[i] = mv;
        } else {  // the last bytes past the whole words
            const int64_t b = words * 4 + (i - words);
            const char pb = priv[b], qb = pub[b], sb = snap[b];
            if (pb != sb) pub[b] = pb;
            else if (qb != sb) priv[b] = qb;
            snap[b] = pb != sb ? pb : qb;
        }
    }
    osc_epilogue();  // the public copy's new bytes, to the peers
}

static void win_release_shadow(ompi_amd_win_t *w) {
    if (w->snap) comm_release_exportable(w->snap);
    if (w->shadow) {
        if (w->owns_shadow) comm_release_exportable(w->shadow);
        else comm_arena_free(w->c, w->shadow);
    }
    w->snap = w->shadow = nullptr;
}

// this rank's copies merged (a no-op for a window without a shadow here)
static int win_merge(ompi_amd_win_t *w, hipStream_t s) {
    if (!w->shadow || !w->bytes) return OMPI_AMD_SUCCESS;
    const int64_t units = (int64_t)(w->bytes / 4) + (int64_t)(w->bytes % 4);
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((units + kOscThreads - 1) / kOscThreads,
                                                                  osc_grid_cap()));
    hipLaunchKernelGGL(win_merge_kernel, dim3((unsigned)blocks), dim3(kOscThreads), 0, s, w->base, w->shadow,
                       w->snap, (int64_t)w->bytes);
    return record_hip(hipGetLastError(), "osc window merge launch");
}


// shared: every rank's base as this process maps it (MPI_Win_allocate_shared),
// so nothing is exported or imported for the bases.
// user: the caller's memory (MPI_Win_create), shadowed when peers cannot
// map it reliably.
static int win_setup(ompi_amd_comm_t *c, void *base, size_t bytes, int disp_unit, bool owns,
                     ompi_amd_win_t **out, char *const *shared = nullptr, bool user = false,
                     bool failed_here = false) {
    auto *w = new (std::nothrow) ompi_amd_win;
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    w->c = c;
    w->rank = ompi_amd_comm_rank(c);
    w->size = ompi_amd_comm_size(c);
    w->base = static_cast<char *>(base);
    w->bytes = bytes;
    w->owns_base = owns;
    int rc = comm_drain(c);  // collective order: deferred nonblocking calls first
    if (failed_here && rc == OMPI_AMD_SUCCESS) rc = OMPI_AMD_ERR_BOOTSTRAP;  // still joins the rendezvous
    rc = ctl_take(c, rc, &w->ctl_slot);
    if (rc == OMPI_AMD_SUCCESS) w->ctl = ctl_page(c, w->ctl_slot, w->rank);
    win_blob mine{}, all[kOscMaxRanks];
    mine.bytes = bytes;
    mine.disp_unit = disp_unit;
    // the caller's memory (MPI_Win_create) that peers could not map
    // reliably: a public copy in the exported arena, the separate model
    const bool need_copy = rc == OMPI_AMD_SUCCESS && bytes && user && comm_win_needs_shadow(c, base);
    if (need_copy && !comm_win_separate_ok(c)) {
        record_msg("osc window: memory peers cannot map as it is (not an IPC-safe size, or older than "
                   "an IPC close of this process) and the separate model is off (osc_win_separate 0)");
        rc = OMPI_AMD_ERR_UNSUPPORTED;  // joins the rendezvous: every rank fails alike
    }
    if (rc == OMPI_AMD_SUCCESS && need_copy) {
        void *pub = nullptr;
        rc = comm_arena_alloc(c, bytes, &pub);
        if (rc == OMPI_AMD_ERR_UNSUPPORTED) {  // past the arena's limit: an allocation of its own
            ipc_desc d;
            rc = comm_alloc_exportable(bytes, false, &pub, &d);
            w->owns_shadow = rc == OMPI_AMD_SUCCESS;
        }
        if (rc == OMPI_AMD_SUCCESS) {
            w->shadow = static_cast<char *>(pub);
            ipc_desc sd;  // recycled memory (comm_release_exportable), not exported
            void *snap = nullptr;
            rc = comm_alloc_exportable(bytes, false, &snap, &sd);
            w->snap = static_cast<char *>(snap);
        }
        // both copies complete before this rank joins the rendezvous below:
        // peers may put into the public copy as soon as the window exists.
        // (hipMemcpy device-to-device returns before the copy is done; that
        // was the round-5 "one-sided mismatch after point-to-point traffic":
        // an epoch-0 put landed in the public copy and the still-running
        // initial copy overwrote it — DESIGN.md §4.9.)  A stream of its own,
        // non-blocking: the legacy stream would also wait for this process's
        // blocking streams, whose kernels may be waiting for these peers.
        if (rc == OMPI_AMD_SUCCESS) {
            hipStream_t z = nullptr;
            rc = record_hip(hipStreamCreateWithFlags(&z, hipStreamNonBlocking), "window copy stream");
            if (rc == OMPI_AMD_SUCCESS)
                rc = record_hip(hipMemcpyAsync(w->shadow, base, bytes, hipMemcpyDeviceToDevice, z),
                                "window public copy");
            if (rc == OMPI_AMD_SUCCESS)
                rc = record_hip(hipMemcpyAsync(w->snap, base, bytes, hipMemcpyDeviceToDevice, z),
                                "window snapshot");
            if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipStreamSynchronize(z), "window copies");
            if (z) hip_ignore(hipStreamDestroy(z));
        }
        mine.shadowed = 1;
    }
    if (rc == OMPI_AMD_SUCCESS && bytes && !shared)
        rc = comm_export(c, w->shadow ? w->shadow : static_cast<char *>(base), &mine.base);
    // every rank takes part in the rendezvous, whatever failed locally
    mine.failed = rc == OMPI_AMD_SUCCESS ? 0 : 1;
    const int arc = comm_allgather(c, &mine, all, sizeof(win_blob));
    if (rc == OMPI_AMD_SUCCESS) rc = arc;
    for (int p = 0; rc == OMPI_AMD_SUCCESS && p < w->size; ++p) {
        if (all[p].failed) {
            record_msg("osc window: rank %d failed to set up its window", p);
            rc = OMPI_AMD_ERR_BOOTSTRAP;
            break;
        }
        w->peer_bytes[p] = all[p].bytes;
        w->peer_disp[p] = all[p].disp_unit;
        w->separate = w->separate || all[p].shadowed != 0;
        if (p == w->rank) {
            w->peer_base[p] = w->shadow ? w->shadow : w->base;  // RMA reaches the public copy
            w->peer_ctl[p] = w->ctl;
            continue;
        }
        if (shared) {
            w->peer_base[p] = shared[p];
        } else if (all[p].bytes) {
            const char *pb = nullptr;
            rc = comm_import(c, p, all[p].base, &pb, true, &w->pinned[p]);
            w->peer_base[p] = const_cast<char *>(pb);
        }
        w->peer_ctl[p] = ctl_page(c, w->ctl_slot, p);
        w->peer_remote[p] = !on_this_device(w->peer_base[p], comm_device(c));
    }
    // agree: all mapped (or all give up together)
    int ok = rc == OMPI_AMD_SUCCESS, all_ok = 0;
    const int grc = ompi_amd_comm_agree(c, ok, &all_ok);
    if (rc == OMPI_AMD_SUCCESS && (grc != OMPI_AMD_SUCCESS || !all_ok))
        rc = grc != OMPI_AMD_SUCCESS ? grc : OMPI_AMD_ERR_BOOTSTRAP;
    if (rc != OMPI_AMD_SUCCESS) {
        for (int p = 0; p < w->size; ++p)
            if (w->pinned[p]) comm_unpin(c, w->pinned[p]);
        (void)ctl_give(c, w->ctl_slot);  // nobody used it: every rank failed here together
        win_release_shadow(w);
        delete w;
        return rc;
    }
    *out = w;
    return OMPI_AMD_SUCCESS;
}

}  // namespace ompi_amd

extern "C" {

int ompi_amd_win_create(ompi_amd_comm_t *c, void *base, size_t bytes, int disp_unit,
                        ompi_amd_win_t **out) {
    if (!c || !out || disp_unit <= 0 || (bytes && !base)) return OMPI_AMD_ERR_BAD_PARAM;
    if (bytes && !ompi_amd_is_device_pointer(base)) {
        record_msg("osc window base is not device memory");
        return OMPI_AMD_ERR_NOT_DEVICE;
    }
    int rc = record_hip(hipSetDevice(comm_device(c)), "hipSetDevice");
    if (rc != OMPI_AMD_SUCCESS) return rc;
    return win_setup(c, bytes ? base : nullptr, bytes, disp_unit, false, out, nullptr, true);
}

int ompi_amd_win_allocate(ompi_amd_comm_t *c, size_t bytes, int disp_unit, void **base,
                          ompi_amd_win_t **out) {
    if (!c || !out || !base || disp_unit <= 0) return OMPI_AMD_ERR_BAD_PARAM;
    int rc = record_hip(hipSetDevice(comm_device(c)), "hipSetDevice");
    void *m = nullptr;
    bool arena = false;
    if (rc == OMPI_AMD_SUCCESS && bytes) {
        // library-owned, from the communicator's exported arena: its chunks
        // are exported once and every peer maps each chunk once, so a new
        // window costs no IPC open at all (each open of a fresh small
        // allocation was a chance for ROCm 7.2's "invalid device pointer"
        // refusal).  Past the arena's IPC size limit: an
        // allocation of its own, padded so that its handle is not a freed
        // window's again.
        rc = comm_arena_alloc(c, bytes, &m);
        arena = rc == OMPI_AMD_SUCCESS;
        if (rc == OMPI_AMD_ERR_UNSUPPORTED) {
            ipc_desc d;
            rc = comm_alloc_exportable(bytes, false, &m, &d);
        }
        if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipMemset(m, 0, bytes), "hipMemset (window)");
        if (rc == OMPI_AMD_SUCCESS)
            rc = record_hip(hipStreamSynchronize(nullptr), "hipStreamSynchronize (window memset)");
    }
    auto release = [&] {
        if (!m) return;
        if (arena) comm_arena_free(c, m);
        else comm_release_exportable(m);
    };
    // a local failure still joins the rendezvous (as a zero-byte window) so
    // that no peer waits; the collective result reports it
    if (rc != OMPI_AMD_SUCCESS) {
        release();
        ompi_amd_win_t *w = nullptr;
        if (win_setup(c, nullptr, 0, disp_unit, false, &w) == OMPI_AMD_SUCCESS)
            (void)ompi_amd_win_free(w);
        return rc;
    }
    rc = win_setup(c, m, bytes, disp_unit, !arena, out);
    if (rc != OMPI_AMD_SUCCESS) {
        release();
        return rc;
    }
    (*out)->arena_base = arena;
    *base = m;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_create_dynamic(ompi_amd_comm_t *c, ompi_amd_win_t **out) {
    if (!c || !out) return OMPI_AMD_ERR_BAD_PARAM;
    int rc = record_hip(hipSetDevice(comm_device(c)), "hipSetDevice");
    // the region tables: one POSIX shared-memory segment, rank 0 creates it
    // and names it in a rendezvous, the others map it, rank 0 unlinks it
    const int me = comm_rank(c), n = comm_size(c);
    const size_t bytes = sizeof(dyn_table) * (size_t)n;
    struct name_blob {
        char name[64];
        int64_t failed;
    } mine{}, all[kOscMaxRanks];
    static std::atomic<unsigned> serial{0};
    dyn_table *map = nullptr;
    if (me == 0 && rc == OMPI_AMD_SUCCESS) {
        snprintf(mine.name, sizeof(mine.name), "/ompi_amd_dyn_%d_%u", (int)getpid(), serial++);
        const int fd = shm_open(mine.name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) rc = OMPI_AMD_ERR_BOOTSTRAP;
        if (rc == OMPI_AMD_SUCCESS) {
            void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            map = m == MAP_FAILED ? nullptr : static_cast<dyn_table *>(m);
            if (!map) rc = OMPI_AMD_ERR_BOOTSTRAP;
        }
        if (fd >= 0) close(fd);
        if (rc != OMPI_AMD_SUCCESS) record_msg("osc dynamic window: cannot create %s", mine.name);
    }
    mine.failed = rc == OMPI_AMD_SUCCESS ? 0 : 1;
    const int arc = comm_allgather(c, &mine, all, sizeof(name_blob));
    if (rc == OMPI_AMD_SUCCESS) rc = arc;
    if (rc == OMPI_AMD_SUCCESS && all[0].failed) rc = OMPI_AMD_ERR_BOOTSTRAP;
    if (rc == OMPI_AMD_SUCCESS && me != 0) {
        const int fd = shm_open(all[0].name, O_RDWR, 0600);
        if (fd >= 0) {
            void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            map = m == MAP_FAILED ? nullptr : static_cast<dyn_table *>(m);
            close(fd);
        }
        if (!map) {
            record_msg("osc dynamic window: cannot map %s", all[0].name);
            rc = OMPI_AMD_ERR_BOOTSTRAP;
        }
    }
    ompi_amd_win_t *w = nullptr;
    // the window proper (control pages, no memory); its rendezvous also
    // tells rank 0 that every rank has mapped the tables
    const int src = win_setup(c, nullptr, 0, 1, false, &w, nullptr, false, rc != OMPI_AMD_SUCCESS);
    if (me == 0 && mine.name[0]) shm_unlink(mine.name);
    if (rc == OMPI_AMD_SUCCESS) rc = src;
    if (rc != OMPI_AMD_SUCCESS) {
        if (map) munmap(map, bytes);
        if (w) (void)ompi_amd_win_free(w);
        return rc;
    }
    w->dynamic = true;
    w->dyn = map;
    w->dyn_bytes = bytes;
    for (int p = 0; p < n; ++p) w->peer_disp[p] = 1;  // displacements are addresses
    *out = w;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_attach(ompi_amd_win_t *w, void *base, size_t size) {
    if (!w || (size && !base)) return OMPI_AMD_ERR_BAD_PARAM;
    if (!w->dynamic) return OMPI_AMD_ERR_UNSUPPORTED;  // another flavor (MPI_ERR_RMA_ATTACH)
    if (size == 0) return OMPI_AMD_SUCCESS;
    if (!ompi_amd_is_device_pointer(base)) {  // osc/rdma's host path cannot reach device peers
        record_msg("osc dynamic window: attached memory is not device memory");
        return OMPI_AMD_ERR_NOT_DEVICE;
    }
    // peers map it as it is: it must be exportable (an IPC-safe allocation
    // that predates no IPC close of this process); a dynamic
    // window has no public copy to fall back on
    if (!comm_ipc_safe(base)) {
        record_msg("osc dynamic window: memory at %p cannot be exported reliably (not an IPC-safe size, "
                   "or older than an IPC close of this process)", base);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    dyn_region r{};
    r.base = (uint64_t)(uintptr_t)base;
    r.size = size;
    OSC_TRY(comm_export(w->c, base, &r.d));
    dyn_table &t = w->dyn[w->rank];
    if (t.n >= (uint32_t)kDynRegions) {
        record_msg("osc dynamic window: more than %d attached regions", kDynRegions);
        return OMPI_AMD_ERR_UNSUPPORTED;  // osc/rdma's limit is a parameter too
    }
    for (uint32_t i = 0; i < t.n; ++i)
        if (r.base < t.r[i].base + t.r[i].size && t.r[i].base < r.base + r.size) {
            record_msg("osc dynamic window: region overlaps an attached one");
            return OMPI_AMD_ERR_BAD_PARAM;
        }
    t.version.fetch_add(1, std::memory_order_acq_rel);
    t.r[t.n] = r;
    std::atomic_thread_fence(std::memory_order_release);
    t.n = t.n + 1;
    t.version.fetch_add(1, std::memory_order_release);
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_detach(ompi_amd_win_t *w, const void *base) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    if (!w->dynamic) return OMPI_AMD_ERR_UNSUPPORTED;  // another flavor (MPI_ERR_RMA_ATTACH)
    dyn_table &t = w->dyn[w->rank];
    for (uint32_t i = 0; i < t.n; ++i)
        if (t.r[i].base == (uint64_t)(uintptr_t)base) {
            t.version.fetch_add(1, std::memory_order_acq_rel);
            for (uint32_t j = i + 1; j < t.n; ++j) t.r[j - 1] = t.r[j];
            t.n = t.n - 1;
            t.version.fetch_add(1, std::memory_order_release);
            return OMPI_AMD_SUCCESS;
        }
    record_msg("osc dynamic window: no region attached at %p", base);
    return OMPI_AMD_ERR_BAD_PARAM;  // MPI_ERR_RMA_RANGE at the MPI level
}

int ompi_amd_win_free(ompi_amd_win_t *w) {
    if (!w) return OMPI_AMD_SUCCESS;
    ompi_amd_comm_t *c = w->c;
    hip_ignore(hipSetDevice(comm_device(c)));
    int rc = comm_drain(c);
    for (hipStream_t s : w->streams) {  // this window's epochs and RMA kernels
        const int src = record_hip(hipStreamSynchronize(s), "hipStreamSynchronize (win_free)");
        if (rc == OMPI_AMD_SUCCESS) rc = src;
    }
    const int brc = comm_allgather(c, nullptr, nullptr, 0);  // nobody still touches the windows
    if (rc == OMPI_AMD_SUCCESS) rc = brc;
    for (int p = 0; p < w->size; ++p)
        if (w->pinned[p]) comm_unpin(c, w->pinned[p]);
    for (auto &m : w->dyn_maps)
        if (m.pin) comm_unpin(c, m.pin);
    w->dyn_maps.clear();
    if (w->dyn) munmap(w->dyn, w->dyn_bytes);
    w->dyn = nullptr;
    const int crc = ctl_give(c, w->ctl_slot);  // the peers' last kernels on it are done
    if (rc == OMPI_AMD_SUCCESS) rc = crc;
    if (w->shared_pin) comm_unpin(c, w->shared_pin);
    const int brc2 = comm_allgather(c, nullptr, nullptr, 0);  // mappings released before frees
    if (rc == OMPI_AMD_SUCCESS) rc = brc2;
    if (w->shared_owner && w->shared_seg) {
        if (w->shared_arena) comm_arena_free(c, w->shared_seg);
        else comm_release_exportable(w->shared_seg);
    }
    if (w->query) hip_ignore(hipStreamDestroy(w->query));
    if (w->owns_base && w->base) comm_release_exportable(w->base);
    if (w->arena_base && w->base) comm_arena_free(c, w->base);  // nobody maps it per window
    win_release_shadow(w);  // no peer maps the public copy any more
    for (char *q : w->scr) if (q) comm_release_exportable(q);  // the streams were synchronised above
    for (char *q : w->scr_old) comm_release_exportable(q);
    if (w->scr_ev) hip_ignore(hipEventDestroy(w->scr_ev));
    if (rc == OMPI_AMD_SUCCESS) rc = comm_sticky(c);
    delete w;
    return rc;
}

int ompi_amd_win_fence(ompi_amd_win_t *w, int assert_, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    const hipStream_t s = win_stream(w, stream);
    OSC_TRY(comm_barrier(w->c, s));
    if (!w->separate) return OMPI_AMD_SUCCESS;
    // separate model: every epoch's RMA into the public copies is done;
    // merge them with the private copies, and let no peer start the next
    // epoch before every rank merged (a second device barrier)
    OSC_TRY(win_merge(w, s));
    return comm_barrier(w->c, s);
}

int ompi_amd_win_sync(ompi_amd_win_t *w, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    return win_merge(w, win_stream(w, stream));
}

int ompi_amd_win_model(const ompi_amd_win_t *w) {
    return !w ? OMPI_AMD_ERR_BAD_PARAM : w->separate ? OMPI_AMD_WIN_SEPARATE : OMPI_AMD_WIN_UNIFIED;
}

int ompi_amd_win_copies(const ompi_amd_win_t *w, void **priv, void **pub, void **snap) {
    if (!w || !priv || !pub || !snap) return OMPI_AMD_ERR_BAD_PARAM;
    *priv = w->base;
    *pub = w->shadow;
    *snap = w->snap;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_peer_base(const ompi_amd_win_t *w, int peer, void **base) {
    if (!w || !base || peer < 0 || peer >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    *base = w->peer_base[peer];
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_lock(ompi_amd_win_t *w, int lock_type, int target, int assert_, void *stream) {
    if (!w || target < 0 || target >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    if (lock_type != OMPI_AMD_LOCK_EXCLUSIVE && lock_type != OMPI_AMD_LOCK_SHARED)
        return OMPI_AMD_ERR_BAD_PARAM;
    if (w->held[target] != HELD_NONE) {
        record_msg("osc: target %d is already locked by this rank", target);
        return OMPI_AMD_ERR_BAD_PARAM;  // MPI_ERR_RMA_SYNC (osc_sm_passive_target.c:122-124)
    }
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    const bool excl = lock_type == OMPI_AMD_LOCK_EXCLUSIVE;
    if (assert_ & OMPI_AMD_MODE_NOCHECK) {
        w->held[target] = HELD_NOCHECK;
    } else {
        OSC_TRY(launch_lock(w, target, excl ? 2 : 4, win_stream(w, stream)));
        w->held[target] = excl ? HELD_EXCLUSIVE : HELD_SHARED;
    }
    // separate model: a lock of one's own window synchronises its copies
    if (target == w->rank) OSC_TRY(win_merge(w, win_stream(w, stream)));
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_unlock(ompi_amd_win_t *w, int target, void *stream) {
    if (!w || target < 0 || target >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    const int h = w->held[target];
    if (h == HELD_NONE) {
        record_msg("osc: target %d is not locked by this rank", target);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    int rc = target == w->rank ? win_merge(w, win_stream(w, stream)) : OMPI_AMD_SUCCESS;
    if (rc != OMPI_AMD_SUCCESS) return rc;
    if (h == HELD_EXCLUSIVE) rc = launch_lock(w, target, 3, win_stream(w, stream));
    else if (h == HELD_SHARED) rc = launch_lock(w, target, 5, win_stream(w, stream));
    w->held[target] = HELD_NONE;
    return rc;
}

int ompi_amd_win_lock_all(ompi_amd_win_t *w, int assert_, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    for (int p = 0; p < w->size; ++p)  // osc_sm_passive_target.c:191-206
        OSC_TRY(ompi_amd_win_lock(w, OMPI_AMD_LOCK_SHARED, p, assert_, stream));
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_unlock_all(ompi_amd_win_t *w, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    for (int p = 0; p < w->size; ++p) OSC_TRY(ompi_amd_win_unlock(w, p, stream));
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_flush(ompi_amd_win_t *w, int target, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    OSC_TRY(record_hip(mark_stream_wait(win_stream(w, stream), no_idle), "hipStreamSynchronize (flush)"));
    return comm_sticky(w->c);
}

int ompi_amd_put(ompi_amd_win_t *w, const void *origin, size_t bytes, int target, size_t disp,
                 void *stream) {
    if (!w || (bytes && !origin)) return OMPI_AMD_ERR_BAD_PARAM;
    char *t = nullptr;
    OSC_TRY(target_ptr(w, target, disp, bytes, &t));
    if (!bytes) return OMPI_AMD_SUCCESS;
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    return xfer_copy(origin, t, bytes, win_stream(w, stream), epoch_gate(w, target), remote_dst(w, target));
}

int ompi_amd_get(ompi_amd_win_t *w, void *origin, size_t bytes, int target, size_t disp,
                 void *stream) {
    if (!w || (bytes && !origin)) return OMPI_AMD_ERR_BAD_PARAM;
    char *t = nullptr;
    OSC_TRY(target_ptr(w, target, disp, bytes, &t));
    if (!bytes) return OMPI_AMD_SUCCESS;
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    return xfer_copy(t, origin, bytes, win_stream(w, stream), epoch_gate(w, target),
                     !on_this_device(origin, comm_device(w->c)));
}

int ompi_amd_accumulate(ompi_amd_win_t *w, const void *origin, size_t count, int type, int target,
                        size_t disp, int op, void *stream) {
    if (op == OMPI_AMD_OP_NO_OP) return OMPI_AMD_ERR_BAD_PARAM;  // MPI_Accumulate forbids it
    if (count && !origin) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_op(w, origin, nullptr, count, type, target, disp, op, stream);
}

int ompi_amd_get_accumulate(ompi_amd_win_t *w, const void *origin, void *result, size_t count,
                            int type, int target, size_t disp, int op, void *stream) {
    if (count && (!result || (!origin && op != OMPI_AMD_OP_NO_OP))) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_op(w, origin, result, count, type, target, disp, op, stream);
}

// Derived datatypes on any side (osc_sm_comm.c:135, 191, 301, 350 ->
// ompi_osc_base_sndrcv_op): a non-contiguous origin is packed on the
// device first (local, before the lock); under the target's accumulate
// lock one gated kernel walks the target datatype's element slots, fetching
// the old elements packed (get_accumulate) and combining the packed origin
// into them; a non-contiguous result is unpacked from the fetched stream
// afterwards (local).  Null odt / rdt / tdt: `type` contiguous.  The packed
// streams live in the window's scratch (osc_scratch).
// acc_ddt for MAXLOC / MINLOC operand types (ddt_pair_kernel above): every
// side's signature counts packed pairs; a contiguous side (NULL program)
// holds `count` memory pairs (extent apart), a derived one the packed
// stream its program describes (the origin packed, the result unpacked, by
// the convertor's kernels, as for the other types).
static int acc_ddt_pair(ompi_amd_win_t *w, const void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                        void *result, size_t rcount, const ompi_amd_ddt_t *rdt, int target, size_t disp,
                        size_t tcount, const ompi_amd_ddt_t *tdt, int type, int op, void *stream) {
    pair_fn f = nullptr;
    int64_t P = 0, E = 0;
    int32_t koff = 0;
    if (!pair_info(type, op, &f, &P, &E, &koff)) {
        record_msg("osc accumulate: op %d on pair type %d is not provided", op, type);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    const bool fetch = result != nullptr;
    const size_t tsig = tdt ? ompi_amd_ddt_size(tdt) * tcount : (size_t)P * tcount;
    if (tsig == 0) return OMPI_AMD_SUCCESS;
    if (tsig % (size_t)P != 0 ||
        (op != OMPI_AMD_OP_NO_OP && (odt ? ompi_amd_ddt_size(odt) * ocount : (size_t)P * ocount) != tsig) ||
        (fetch && (rdt ? ompi_amd_ddt_size(rdt) * rcount : (size_t)P * rcount) != tsig) ||
        (op != OMPI_AMD_OP_NO_OP && !origin)) {
        record_msg("osc accumulate: origin / result / target type signatures differ (pair type %d)", type);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    const int64_t n = (int64_t)(tsig / (size_t)P);
    ddt_view tv{};
    if (tdt && !ddt_view_of(tdt, &tv)) return OMPI_AMD_ERR_BAD_PARAM;
    if (target < 0 || target >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    const int64_t base = (int64_t)disp * (int64_t)w->peer_disp[target];
    const int64_t last = (int64_t)(tcount - 1) * (tdt ? tv.d.extent : E);
    const int64_t lo = base + (tdt ? tv.lo + std::min<int64_t>(0, last) : 0);
    const int64_t hi = base + (tdt ? tv.hi + std::max<int64_t>(0, last) : n * E);
    char *t = nullptr;
    OSC_TRY(target_span(w, target, base, lo - base, hi - base, &t));
    hipStream_t s = win_stream(w, stream);
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    const int32_t pk = (int32_t)(P - (int64_t)sizeof(int));  // packed: the index right after the value
    pair_side in{const_cast<char *>(static_cast<const char *>(origin)), E, koff};
    pair_side old{static_cast<char *>(result), E, koff};
    void *po = nullptr, *pr = nullptr;
    int rc = OMPI_AMD_SUCCESS;
    if (odt && op != OMPI_AMD_OP_NO_OP) {  // the origin's packed pairs (local; before the lock)
        rc = osc_scratch(w, s, 0, tsig, &po);
        size_t done = 0;
        if (rc == OMPI_AMD_SUCCESS) rc = ompi_amd_ddt_pack(odt, ocount, origin, po, 0, tsig, &done, s);
        if (rc == OMPI_AMD_SUCCESS && done != tsig) rc = OMPI_AMD_ERR_BAD_PARAM;
        in = pair_side{static_cast<char *>(po), P, pk};
    }
    if (op == OMPI_AMD_OP_NO_OP) in.p = nullptr;
    if (rc == OMPI_AMD_SUCCESS && fetch && rdt) {
        rc = osc_scratch(w, s, 1, tsig, &pr);
        old = pair_side{static_cast<char *>(pr), P, pk};
    }
    if (rc == OMPI_AMD_SUCCESS) rc = launch_lock(w, target, 0, s);
    if (rc == OMPI_AMD_SUCCESS) {
        const uint32_t *gate = taken_word(w, target, true);
        ddt_desc dd{};
        if (tdt) dd = tv.d;  // else nelem 0: a contiguous target
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n + kOscThreads - 1) / kOscThreads,
                                                                      osc_grid_cap()));
        f(dim3((unsigned)blocks), dd, t, in, old, n, gate, s);
        rc = record_hip(hipGetLastError(), "osc pair accumulate launch");
        const int urc = launch_lock(w, target, 1, s);  // always release
        if (rc == OMPI_AMD_SUCCESS) rc = urc;
    }
    if (rc == OMPI_AMD_SUCCESS && pr) {  // the fetched pairs into the result layout (local)
        size_t done = 0;
        rc = ompi_amd_ddt_unpack(rdt, rcount, pr, result, 0, tsig, &done, s);
        if (rc == OMPI_AMD_SUCCESS && done != tsig) rc = OMPI_AMD_ERR_BAD_PARAM;
    }
    if (po || pr) osc_scratch_done(w, s);
    return rc;
}

static int acc_ddt(ompi_amd_win_t *w, const void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                   void *result, size_t rcount, const ompi_amd_ddt_t *rdt, int target, size_t disp,
                   size_t tcount, const ompi_amd_ddt_t *tdt, int type, int op, void *stream) {
    if (!w || type < 0 || type >= OMPI_AMD_TYPE_COUNT || ompi_amd_type_extent(type) == 0)
        return OMPI_AMD_ERR_BAD_PARAM;
    const size_t ext = ompi_amd_type_extent(type);
    const bool fetch = result != nullptr;
    if ((odt || rdt || tdt) && is_pair_type(type))
        return acc_ddt_pair(w, origin, ocount, odt, result, rcount, rdt, target, disp, tcount, tdt, type, op,
                            stream);
    const size_t tbytes = (tdt ? ompi_amd_ddt_size(tdt) : ext) * tcount;
    if (tbytes == 0) return OMPI_AMD_SUCCESS;
    if (tbytes % ext != 0 ||
        (op != OMPI_AMD_OP_NO_OP && (odt ? ompi_amd_ddt_size(odt) : ext) * ocount != tbytes) ||
        (fetch && (rdt ? ompi_amd_ddt_size(rdt) : ext) * rcount != tbytes) ||
        (op != OMPI_AMD_OP_NO_OP && !origin)) {
        record_msg("osc accumulate: origin / result / target type signatures differ");
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    const int64_t n = (int64_t)(tbytes / ext);
    if (!tdt && !odt && !rdt) return rma_op(w, origin, result, (size_t)n, type, target, disp, op, stream);
    ddt_acc_fn f = nullptr;
    if (op == OMPI_AMD_OP_REPLACE || op == OMPI_AMD_OP_NO_OP) f = ddt_rw_fn(ext, op == OMPI_AMD_OP_REPLACE);
    else if (op > 0 && op < OMPI_AMD_OP_COUNT) f = g_ddt_acc[op][type];
    if (!f || (op != OMPI_AMD_OP_REPLACE && op != OMPI_AMD_OP_NO_OP && !g_acc[op][type])) {
        record_msg("osc accumulate: op %d on type %d is not provided", op, type);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    // the target's typed span, inside its window
    ddt_view tv{};
    if (tdt && !ddt_view_of(tdt, &tv)) return OMPI_AMD_ERR_BAD_PARAM;
    if (target < 0 || target >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    const int64_t base = (int64_t)disp * (int64_t)w->peer_disp[target];
    const int64_t last = (int64_t)(tcount - 1) * (tdt ? tv.d.extent : (int64_t)ext);
    const int64_t lo = base + (tdt ? tv.lo + std::min<int64_t>(0, last) : 0);
    const int64_t hi = base + (tdt ? tv.hi + std::max<int64_t>(0, last) : (int64_t)tbytes);
    char *t = nullptr;
    OSC_TRY(target_span(w, target, base, lo - base, hi - base, &t));
    hipStream_t s = win_stream(w, stream);
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    // origin stream, packed (local; before the lock)
    const void *in = origin;
    void *po = nullptr, *pr = nullptr;
    int rc = OMPI_AMD_SUCCESS;
    if (odt && op != OMPI_AMD_OP_NO_OP) {
        rc = osc_scratch(w, s, 0, tbytes, &po);
        size_t done = 0;
        if (rc == OMPI_AMD_SUCCESS) rc = ompi_amd_ddt_pack(odt, ocount, origin, po, 0, tbytes, &done, s);
        if (rc == OMPI_AMD_SUCCESS && done != tbytes) rc = OMPI_AMD_ERR_BAD_PARAM;
        in = po;
    }
    void *old = result;
    if (rc == OMPI_AMD_SUCCESS && fetch && rdt) {
        rc = osc_scratch(w, s, 1, tbytes, &pr);
        old = pr;
    }
    if (rc == OMPI_AMD_SUCCESS) rc = launch_lock(w, target, 0, s);
    if (rc == OMPI_AMD_SUCCESS) {
        const uint32_t *gate = taken_word(w, target, true);
        if (tdt) {
            const int64_t blocks = std::max<int64_t>(
                1, std::min<int64_t>((n + kOscThreads * kAccUnroll - 1) / (kOscThreads * kAccUnroll),
                                     osc_grid_cap()));
            // element-unit arithmetic in 32 bits when everything fits and every
            // run, displacement and stride is a multiple of the element
            ddt_desc dd = tv.d;
            const int64_t e = (int64_t)ext;
            static const bool fast_on = !(getenv("OMPI_AMD_OSC_DDT_FAST") &&
                                          atoi(getenv("OMPI_AMD_OSC_DDT_FAST")) == 0);
            const bool fast = fast_on && (e == 1 || e == 2 || e == 4 || e == 8 || e == 16) && tv.gran % e == 0 &&
                              n < (1ll << 32) && dd.size / e < (1ll << 32) && tv.max_blen / e < (1ll << 32);
            if (fast) dd.sdiv = make_fdiv((uint32_t)(dd.size / e));
            rc = record_hip(f(dim3((unsigned)blocks), dd, t, in, old, n, gate, fast, s,
                              remote_dst(w, target) ? 1 : 0),
                            "osc derived accumulate launch");
        } else {  // contiguous target: the plain kernels on the packed streams
            if (fetch) rc = xfer_copy(t, old, tbytes, s, gate, !on_this_device(old, comm_device(w->c)));
            if (rc == OMPI_AMD_SUCCESS) {
                if (op == OMPI_AMD_OP_REPLACE) rc = xfer_copy(in, t, tbytes, s, gate, remote_dst(w, target));
                else if (op != OMPI_AMD_OP_NO_OP)
                    rc = launch_acc(w, op, type, in, t, (size_t)n, gate, s, remote_dst(w, target));
            }
        }
        const int urc = launch_lock(w, target, 1, s);  // always release
        if (rc == OMPI_AMD_SUCCESS) rc = urc;
    }
    if (rc == OMPI_AMD_SUCCESS && pr) {  // the fetched stream into the result layout (local)
        size_t done = 0;
        rc = ompi_amd_ddt_unpack(rdt, rcount, pr, result, 0, tbytes, &done, s);
        if (rc == OMPI_AMD_SUCCESS && done != tbytes) rc = OMPI_AMD_ERR_BAD_PARAM;
    }
    if (po || pr) osc_scratch_done(w, s);
    return rc;
}

// MPI_Put / MPI_Get with derived datatypes (osc_sm_comm.c:24-100, 209-270:
// ompi_datatype_sndrcv of any origin / target pair).  The origin side is a
// packed byte stream on this GPU (a non-contiguous origin is packed before
// a put, and unpacked from it after a get, by the convertor's kernels); the
// target side moves in one launch of ddt_acc_kernel over G-byte granules (G
// the widest power of two dividing every run, displacement, stride and
// extent of the target type and both addresses): REPLACE stores granule k
// of the stream into the k-th granule slot of the target type, NO_OP loads
// it out — the derived accumulate's element walk with no element type, its
// per-workgroup system-scope acquire / release and the epoch gate, and no
// accumulate lock (put and get are not atomic, osc/sm takes none either).
// A side's program NULL: `count` contiguous bytes.
static int rma_ddt(ompi_amd_win_t *w, void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                   int target, size_t disp, size_t tcount, const ompi_amd_ddt_t *tdt, bool put,
                   void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    const size_t obytes = odt ? ompi_amd_ddt_size(odt) * ocount : ocount;
    const size_t tbytes = tdt ? ompi_amd_ddt_size(tdt) * tcount : tcount;
    if (obytes != tbytes) {
        record_msg("osc %s: origin (%zu bytes) and target (%zu bytes) type signatures differ",
                   put ? "put" : "get", obytes, tbytes);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    if (tbytes == 0) return OMPI_AMD_SUCCESS;
    if (!origin) return OMPI_AMD_ERR_BAD_PARAM;
    if (!odt && !tdt)
        return put ? ompi_amd_put(w, origin, tbytes, target, disp, stream)
                   : ompi_amd_get(w, origin, tbytes, target, disp, stream);
    ddt_view tv{};
    if (tdt && !ddt_view_of(tdt, &tv)) return OMPI_AMD_ERR_BAD_PARAM;
    if (target < 0 || target >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    const int64_t base = (int64_t)disp * (int64_t)w->peer_disp[target];
    const int64_t last = tdt ? (int64_t)(tcount - 1) * tv.d.extent : 0;
    const int64_t lo = base + (tdt ? tv.lo + std::min<int64_t>(0, last) : 0);
    const int64_t hi = base + (tdt ? tv.hi + std::max<int64_t>(0, last) : (int64_t)tbytes);
    char *t = nullptr;
    OSC_TRY(target_span(w, target, base, lo - base, hi - base, &t));
    hipStream_t s = win_stream(w, stream);
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    const uint32_t *gate = epoch_gate(w, target);
    int rc = OMPI_AMD_SUCCESS;
    char *packed = static_cast<char *>(origin);
    void *tmp = nullptr;
    if (odt) {  // the origin's packed stream, local
        rc = osc_scratch(w, s, 0, tbytes, &tmp);
        packed = static_cast<char *>(tmp);
        if (rc == OMPI_AMD_SUCCESS && put) {
            size_t done = 0;
            rc = ompi_amd_ddt_pack(odt, ocount, origin, tmp, 0, tbytes, &done, s);
            if (rc == OMPI_AMD_SUCCESS && done != tbytes) rc = OMPI_AMD_ERR_BAD_PARAM;
        }
    }
    if (rc == OMPI_AMD_SUCCESS && !tdt) {  // contiguous target: one copy
        rc = put ? xfer_copy(packed, t, tbytes, s, gate, remote_dst(w, target))
                 : xfer_copy(t, packed, tbytes, s, gate, !on_this_device(packed, comm_device(w->c)));
    } else if (rc == OMPI_AMD_SUCCESS) {
        int64_t g = tv.gran;
        while (g > 1 && (((uintptr_t)t | (uintptr_t)packed) & (uintptr_t)(g - 1))) g >>= 1;
        g = std::min<int64_t>(g, 16);
        const ddt_acc_fn f = ddt_rw_fn((size_t)g, put);
        const int64_t n = (int64_t)tbytes / g;
        const int64_t blocks = std::max<int64_t>(
            1, std::min<int64_t>((n + kOscThreads * kAccUnroll - 1) / (kOscThreads * kAccUnroll),
                                 osc_grid_cap()));
        ddt_desc dd = tv.d;
        const bool fast = tv.gran % g == 0 && n < (1ll << 32) && dd.size / g < (1ll << 32) &&
                          tv.max_blen / g < (1ll << 32);
        if (fast) dd.sdiv = make_fdiv((uint32_t)(dd.size / g));
        rc = record_hip(f(dim3((unsigned)blocks), dd, t, put ? packed : nullptr, put ? nullptr : packed, n,
                          gate, fast, s,
                          (put ? remote_dst(w, target) : !on_this_device(packed, comm_device(w->c))) ? 1 : 0),
                        put ? "osc derived put launch" : "osc derived get launch");
    }
    if (rc == OMPI_AMD_SUCCESS && odt && !put) {  // the fetched stream into the origin's layout
        size_t done = 0;
        rc = ompi_amd_ddt_unpack(odt, ocount, tmp, origin, 0, tbytes, &done, s);
        if (rc == OMPI_AMD_SUCCESS && done != tbytes) rc = OMPI_AMD_ERR_BAD_PARAM;
    }
    if (tmp) osc_scratch_done(w, s);
    return rc;
}

int ompi_amd_put_ddt(ompi_amd_win_t *w, const void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                     int target, size_t disp, size_t tcount, const ompi_amd_ddt_t *tdt, void *stream) {
    return rma_ddt(w, const_cast<void *>(origin), ocount, odt, target, disp, tcount, tdt, true, stream);
}

int ompi_amd_get_ddt(ompi_amd_win_t *w, void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                     int target, size_t disp, size_t tcount, const ompi_amd_ddt_t *tdt, void *stream) {
    return rma_ddt(w, origin, ocount, odt, target, disp, tcount, tdt, false, stream);
}

int ompi_amd_accumulate_ddt(ompi_amd_win_t *w, const void *origin, size_t ocount,
                            const ompi_amd_ddt_t *odt, int target, size_t disp, size_t tcount,
                            const ompi_amd_ddt_t *tdt, int type, int op, void *stream) {
    if (op == OMPI_AMD_OP_NO_OP) return OMPI_AMD_ERR_BAD_PARAM;  // MPI_Accumulate forbids it
    return acc_ddt(w, origin, ocount, odt, nullptr, 0, nullptr, target, disp, tcount, tdt, type, op,
                   stream);
}

int ompi_amd_get_accumulate_ddt(ompi_amd_win_t *w, const void *origin, size_t ocount,
                                const ompi_amd_ddt_t *odt, void *result, size_t rcount,
                                const ompi_amd_ddt_t *rdt, int target, size_t disp, size_t tcount,
                                const ompi_amd_ddt_t *tdt, int type, int op, void *stream) {
    if (!result && tcount) return OMPI_AMD_ERR_BAD_PARAM;
    return acc_ddt(w, origin, ocount, odt, result, rcount, rdt, target, disp, tcount, tdt, type, op,
                   stream);
}

int ompi_amd_fetch_and_op(ompi_amd_win_t *w, const void *origin, void *result, int type,
                          int target, size_t disp, int op, void *stream) {
    return ompi_amd_get_accumulate(w, origin, result, 1, type, target, disp, op, stream);
}

int ompi_amd_compare_and_swap(ompi_amd_win_t *w, const void *origin, const void *compare,
                              void *result, int type, int target, size_t disp, void *stream) {
    if (!w || !origin || !compare || !result) return OMPI_AMD_ERR_BAD_PARAM;
    if (type < 0 || type >= OMPI_AMD_TYPE_COUNT || ompi_amd_type_extent(type) == 0 ||
        is_pair_type(type))
        return OMPI_AMD_ERR_BAD_PARAM;  // integer, logical and byte types (MPI-3.1 §11.3.4)
    const size_t size = ompi_amd_type_extent(type);  // no gaps in these types
    char *t = nullptr;
    OSC_TRY(target_ptr(w, target, disp, size, &t));
    hipStream_t s = win_stream(w, stream);
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    hipLaunchKernelGGL(cas_kernel, dim3(1), dim3(64), 0, s,
                       static_cast<const unsigned char *>(origin),
                       static_cast<const unsigned char *>(compare),
                       static_cast<unsigned char *>(result), reinterpret_cast<unsigned char *>(t),
                       (int)size, w->peer_ctl[target], comm_err_dev(w->c), ticks_of(w));
    return record_hip(hipGetLastError(), "osc compare_and_swap launch");
}

// ---- shared windows (osc_sm_component.c:244-360, 455-485) ----

int ompi_amd_win_allocate_shared(ompi_amd_comm_t *c, size_t bytes, int disp_unit, int noncontig,
                                 void **base, ompi_amd_win_t **out) {
    if (!c || !out || !base || disp_unit <= 0) return OMPI_AMD_ERR_BAD_PARAM;
    const int me = ompi_amd_comm_rank(c), n = ompi_amd_comm_size(c);
    int rc = record_hip(hipSetDevice(comm_device(c)), "hipSetDevice");
    if (rc == OMPI_AMD_SUCCESS) rc = comm_drain(c);
    // segment sizes: exact, or whole pages with alloc_shared_noncontig
    // (osc_sm_component.c:265-268)
    uint64_t seg = noncontig ? (bytes + 4095) / 4096 * 4096 : bytes, segs[kOscMaxRanks] = {};
    const int src = comm_allgather(c, &seg, segs, sizeof(seg));
    if (rc == OMPI_AMD_SUCCESS) rc = src;
    uint64_t prefix[kOscMaxRanks + 1] = {};
    for (int p = 0; p < n; ++p) prefix[p + 1] = prefix[p] + segs[p];
    // rank 0 allocates the whole window; everyone learns its descriptor
    struct seg_blob {
        ipc_desc d;
        int64_t failed;
    } mine{}, all[kOscMaxRanks];
    char *m = nullptr;
    bool arena = false;
    if (me == 0 && rc == OMPI_AMD_SUCCESS) {
        // from rank 0's exported arena (peers map its chunk once, §4.6), or
        // an allocation of its own past the arena's IPC size limit
        rc = comm_arena_alloc(c, prefix[n] ? prefix[n] : 1, (void **)&m);
        arena = rc == OMPI_AMD_SUCCESS;
        if (arena) rc = comm_export(c, m, &mine.d);
        else if (rc == OMPI_AMD_ERR_UNSUPPORTED)
            rc = comm_alloc_exportable(prefix[n] ? prefix[n] : 1, false, (void **)&m, &mine.d);
        if (rc == OMPI_AMD_SUCCESS && prefix[n])
            rc = record_hip(hipMemset(m, 0, prefix[n]), "hipMemset (shared window)");
        if (rc == OMPI_AMD_SUCCESS)
            rc = record_hip(hipStreamSynchronize(nullptr), "hipStreamSynchronize (shared window)");
    }
    mine.failed = rc == OMPI_AMD_SUCCESS ? 0 : 1;
    const int arc = comm_allgather(c, &mine, all, sizeof(seg_blob));
    if (rc == OMPI_AMD_SUCCESS) rc = arc;
    if (rc == OMPI_AMD_SUCCESS && all[0].failed) {
        record_msg("osc shared window: rank 0 could not allocate %llu bytes",
                   (unsigned long long)prefix[n]);
        rc = OMPI_AMD_ERR_BOOTSTRAP;
    }
    void *pin = nullptr;
    if (rc == OMPI_AMD_SUCCESS && me != 0) {
        const char *mb = nullptr;
        rc = comm_import(c, 0, all[0].d, &mb, true, &pin);
        if (rc == OMPI_AMD_SUCCESS) m = const_cast<char *>(mb);
    }
    auto release_owner = [&] {
        if (me != 0 || !m) return;
        if (arena) comm_arena_free(c, m);
        else comm_release_exportable(m);
    };
    int all_ok = 0;
    const int grc = ompi_amd_comm_agree(c, rc == OMPI_AMD_SUCCESS, &all_ok);
    if (rc == OMPI_AMD_SUCCESS && (grc != OMPI_AMD_SUCCESS || !all_ok))
        rc = grc != OMPI_AMD_SUCCESS ? grc : OMPI_AMD_ERR_BOOTSTRAP;
    char *bases[kOscMaxRanks] = {};
    for (int p = 0; p < n && m; ++p) bases[p] = m + prefix[p];
    ompi_amd_win_t *w = nullptr;
    if (rc == OMPI_AMD_SUCCESS) rc = win_setup(c, bases[me], bytes, disp_unit, false, &w, bases);
    if (rc != OMPI_AMD_SUCCESS) {
        if (pin) comm_unpin(c, pin);
        (void)comm_allgather(c, nullptr, nullptr, 0);  // every mapping released before the free
        release_owner();
        return rc;
    }
    for (int p = 0; p < n; ++p) w->peer_bytes[p] = segs[p];  // queried sizes (padded if noncontig)
    w->bytes = segs[me];
    w->shared = true;
    w->shared_seg = m;
    w->shared_pin = pin;
    w->shared_owner = me == 0;
    w->shared_arena = arena;
    *base = bases[me];
    *out = w;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_shared_query(ompi_amd_win_t *w, int rank, size_t *size, int *disp_unit,
                              void **baseptr) {
    if (!w || !size || !disp_unit || !baseptr) return OMPI_AMD_ERR_BAD_PARAM;
    if (!w->shared) {  // osc_sm_component.c:460-462
        record_msg("osc: MPI_Win_shared_query on a window not made by MPI_Win_allocate_shared");
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    if (rank >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
    *size = 0;
    *disp_unit = 0;
    *baseptr = nullptr;
    for (int p = rank < 0 ? 0 : rank; p < (rank < 0 ? w->size : rank + 1); ++p) {
        if (rank < 0 && w->peer_bytes[p] == 0) continue;  // MPI_PROC_NULL: first nonzero segment
        *size = w->peer_bytes[p];
        *disp_unit = (int)w->peer_disp[p];
        *baseptr = w->peer_base[p];
        break;
    }
    return OMPI_AMD_SUCCESS;
}

// ---- general active target synchronisation (osc_sm_active_target.c) ----

static int pscw_launch(ompi_amd_win_t *w, int kind, const pscw_group &g, hipStream_t s) {
    peer_ctl_set peers{};
    for (int p = 0; p < w->size; ++p) peers.p[p] = w->peer_ctl[p];
    hipLaunchKernelGGL(pscw_kernel, dim3(1), dim3(64), 0, s, w->ctl, peers, g, kind, w->rank,
                       comm_err_dev(w->c), ticks_of(w));
    return record_hip(hipGetLastError(), "osc pscw launch");
}

static int pscw_group_of(ompi_amd_win_t *w, const int *ranks, int n, pscw_group *g) {
    if (n < 0 || n > w->size || (n && !ranks)) return OMPI_AMD_ERR_BAD_PARAM;
    *g = pscw_group{};
    g->n = n;
    for (int i = 0; i < n; ++i) {
        if (ranks[i] < 0 || ranks[i] >= w->size) return OMPI_AMD_ERR_BAD_PARAM;
        g->rank[i] = ranks[i];
    }
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_post(ompi_amd_win_t *w, const int *ranks, int n, int assert_, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    if (w->posted) {  // osc_sm_active_target.c:230-233
        record_msg("osc: MPI_Win_post while an exposure epoch is open");
        return OMPI_AMD_ERR_RMA_SYNC;
    }
    pscw_group g;
    OSC_TRY(pscw_group_of(w, ranks, n, &g));
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    // MPI_MODE_NOCHECK: the origins start without waiting for this post
    // (osc_sm_active_target.c:239); the window is still released
    if (assert_ & OMPI_AMD_MODE_NOCHECK) g.n = 0;
    OSC_TRY(win_merge(w, win_stream(w, stream)));  // separate model: the exposed copy up to date
    OSC_TRY(pscw_launch(w, 0, g, win_stream(w, stream)));
    w->posted = true;
    w->complete_want += (uint32_t)n;  // every origin of the group completes once
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_start(ompi_amd_win_t *w, const int *ranks, int n, int assert_, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    if (w->started) {  // osc_sm_active_target.c:137-140
        record_msg("osc: MPI_Win_start while an access epoch is open");
        return OMPI_AMD_ERR_RMA_SYNC;
    }
    pscw_group g;
    OSC_TRY(pscw_group_of(w, ranks, n, &g));
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    // MPI_MODE_NOCHECK: the targets' posts are not waited for (nor counted:
    // they posted with NOCHECK too, osc_sm_active_target.c:142)
    if (!(assert_ & OMPI_AMD_MODE_NOCHECK)) {
        for (int i = 0; i < n; ++i) g.want[i] = w->post_seen[ranks[i]] + 1;
        OSC_TRY(pscw_launch(w, 1, g, win_stream(w, stream)));
        for (int i = 0; i < n; ++i) ++w->post_seen[ranks[i]];
    }
    w->started = true;
    w->start_group.assign(ranks, ranks + n);
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_complete(ompi_amd_win_t *w, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    if (!w->started) {
        record_msg("osc: MPI_Win_complete without MPI_Win_start");
        return OMPI_AMD_ERR_RMA_SYNC;
    }
    pscw_group g;
    OSC_TRY(pscw_group_of(w, w->start_group.data(), (int)w->start_group.size(), &g));
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    OSC_TRY(pscw_launch(w, 2, g, win_stream(w, stream)));
    w->started = false;
    w->start_group.clear();
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_wait(ompi_amd_win_t *w, void *stream) {
    if (!w) return OMPI_AMD_ERR_BAD_PARAM;
    if (!w->posted) {
        record_msg("osc: MPI_Win_wait without MPI_Win_post");
        return OMPI_AMD_ERR_RMA_SYNC;
    }
    pscw_group g{};
    g.want[0] = w->complete_want;
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    OSC_TRY(pscw_launch(w, 3, g, win_stream(w, stream)));
    OSC_TRY(win_merge(w, win_stream(w, stream)));  // separate model: the origins' RMA, private too
    w->posted = false;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_win_test(ompi_amd_win_t *w, int *flag) {
    if (!w || !flag) return OMPI_AMD_ERR_BAD_PARAM;
    *flag = 0;
    if (!w->posted) {
        record_msg("osc: MPI_Win_test without MPI_Win_post");
        return OMPI_AMD_ERR_RMA_SYNC;
    }
    OSC_TRY(record_hip(hipSetDevice(comm_device(w->c)), "hipSetDevice"));
    // read the counter on a stream of its own: this rank's streams may hold
    // a start kernel that waits for a peer (and the legacy stream would
    // order the read behind it)
    if (!w->query) OSC_TRY(record_hip(hipStreamCreateWithFlags(&w->query, hipStreamNonBlocking),
                                      "osc test stream"));
    uint32_t seen = 0;
    OSC_TRY(record_hip(hipMemcpyAsync(&seen, w->ctl + CTL_COMPLETE, sizeof(seen),
                                      hipMemcpyDeviceToHost, w->query), "osc test (complete counter)"));
    OSC_TRY(record_hip(hipStreamSynchronize(w->query), "osc test (complete counter)"));
    if ((int32_t)(seen - w->complete_want) >= 0) {
        // the exposure epoch ends (osc_sm_active_target.c:320-330); the wait
        // kernel (already satisfied) acquires what the origins released
        pscw_group g{};
        g.want[0] = w->complete_want;
        OSC_TRY(pscw_launch(w, 3, g, win_stream(w, nullptr)));
        OSC_TRY(win_merge(w, win_stream(w, nullptr)));
        *flag = 1;
        w->posted = false;
    }
    return comm_sticky(w->c);
}

// ---- request-based RMA (osc.h:384-393) ----

static int rma_request(ompi_amd_win_t *w, void *stream, int rc, ompi_amd_rma_request_t **out) {
    *out = nullptr;
    if (rc != OMPI_AMD_SUCCESS) return rc;
    auto *r = new (std::nothrow) ompi_amd_rma_request;
    if (!r) return OMPI_AMD_ERR_BAD_PARAM;
    r->w = w;
    rc = record_hip(hipEventCreateWithFlags(&r->ev, hipEventDisableTiming), "rma request event");
    if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipEventRecord(r->ev, win_stream(w, stream)), "rma request record");
    if (rc != OMPI_AMD_SUCCESS) {
        if (r->ev) hip_ignore(hipEventDestroy(r->ev));
        delete r;
        return rc;
    }
    *out = r;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_rput(ompi_amd_win_t *w, const void *origin, size_t bytes, int target, size_t disp,
                  void *stream, ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream, ompi_amd_put(w, origin, bytes, target, disp, stream), req);
}

int ompi_amd_rget(ompi_amd_win_t *w, void *origin, size_t bytes, int target, size_t disp,
                  void *stream, ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream, ompi_amd_get(w, origin, bytes, target, disp, stream), req);
}

int ompi_amd_raccumulate(ompi_amd_win_t *w, const void *origin, size_t count, int type, int target,
                         size_t disp, int op, void *stream, ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream,
                       ompi_amd_accumulate(w, origin, count, type, target, disp, op, stream), req);
}

int ompi_amd_rget_accumulate(ompi_amd_win_t *w, const void *origin, void *result, size_t count,
                             int type, int target, size_t disp, int op, void *stream,
                             ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream,
                       ompi_amd_get_accumulate(w, origin, result, count, type, target, disp, op,
                                               stream), req);
}

int ompi_amd_rput_ddt(ompi_amd_win_t *w, const void *origin, size_t ocount,
                      const ompi_amd_ddt_t *odt, int target, size_t disp, size_t tcount,
                      const ompi_amd_ddt_t *tdt, void *stream, ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream, ompi_amd_put_ddt(w, origin, ocount, odt, target, disp, tcount, tdt, stream),
                       req);
}

int ompi_amd_rget_ddt(ompi_amd_win_t *w, void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                      int target, size_t disp, size_t tcount, const ompi_amd_ddt_t *tdt, void *stream,
                      ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream, ompi_amd_get_ddt(w, origin, ocount, odt, target, disp, tcount, tdt, stream),
                       req);
}

int ompi_amd_raccumulate_ddt(ompi_amd_win_t *w, const void *origin, size_t ocount,
                             const ompi_amd_ddt_t *odt, int target, size_t disp, size_t tcount,
                             const ompi_amd_ddt_t *tdt, int type, int op, void *stream,
                             ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream,
                       ompi_amd_accumulate_ddt(w, origin, ocount, odt, target, disp, tcount, tdt,
                                               type, op, stream), req);
}

int ompi_amd_rget_accumulate_ddt(ompi_amd_win_t *w, const void *origin, size_t ocount,
                                 const ompi_amd_ddt_t *odt, void *result, size_t rcount,
                                 const ompi_amd_ddt_t *rdt, int target, size_t disp,
                                 size_t tcount, const ompi_amd_ddt_t *tdt, int type, int op,
                                 void *stream, ompi_amd_rma_request_t **req) {
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    return rma_request(w, stream,
                       ompi_amd_get_accumulate_ddt(w, origin, ocount, odt, result, rcount, rdt,
                                                   target, disp, tcount, tdt, type, op, stream),
                       req);
}

int ompi_amd_rma_test(ompi_amd_rma_request_t *r, int *done) {
    if (!r || !done) return OMPI_AMD_ERR_BAD_PARAM;
    const hipError_t e = hipEventQuery(r->ev);
    *done = 0;
    if (e == hipErrorNotReady) return OMPI_AMD_SUCCESS;
    if (e != hipSuccess) return record_hip(e, "rma request test");
    *done = 1;
    return comm_sticky(r->w->c);
}

int ompi_amd_rma_wait(ompi_amd_rma_request_t *r) {
    if (!r) return OMPI_AMD_ERR_BAD_PARAM;
    OSC_TRY(record_hip(hipEventSynchronize(r->ev), "rma request wait"));
    return comm_sticky(r->w->c);
}

int ompi_amd_rma_free(ompi_amd_rma_request_t *r) {
    if (!r) return OMPI_AMD_SUCCESS;
    const int rc = ompi_amd_rma_wait(r);
    hip_ignore(hipEventDestroy(r->ev));
    delete r;
    return rc;
}

}  // extern "C"
