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
//                rank's rbuf, barrier (staged, user_ipc 0: push-gather — the
//                owner keeps its result, every rank then pulls the others)
//   3 push-land  staged push whose second phase stores too: the owner
//                stores its result into every rank's landing buffer,
//                barrier, each rank copies the results into its rbuf
//                locally, barrier (with user_ipc: as 2)
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

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

#include "../../include/ompi_amd_coll.h"
#include "bootstrap.h"
#include "comm_internal.h"
#include "host_mark.h"
#include "coll_kernels.h"
#include "ipc_registry.h"
#include "op_device.h"
#include "runtime.h"

namespace ompi_amd {

#define TRY(x)                                   \
    do {                                         \
        int rc_ = (x);                           \
        if (rc_ != OMPI_AMD_SUCCESS) return rc_; \
    } while (0)

// Largest allocation the library exports or maps: on ROCm 7.2
// hipIpcOpenMemHandle of a 2 GiB + 2 MiB allocation never returned (four
// ranks on one MI355X, OMPI_AMD_TRACE=1); 1 GiB opened in < 1 ms.
constexpr size_t kMaxIpcBytes = (2ull << 30) - (4u << 20);

// ---------------------------------------------------------------- barrier
// A rank that fails a call its peers may already have launched (a deferred
// nonblocking call whose IPC open was refused) raises every peer's abort
// word, so their waits give up within ~1 ms instead of timing out.
__global__ void abort_kernel(flag_set peers, uint64_t *local, int rank, int size) {
    const int t = threadIdx.x;
    if (t < size && t != rank)
        __hip_atomic_store(peers.p[t] + kAbortWord, (uint64_t)1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (t == rank)
        __hip_atomic_store(local + kAbortWord, (uint64_t)1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    sys_release();
}

// dbg (OMPI_AMD_DEBUG_PROGRESS=1, else null; host-mapped): [0] the last
// epoch whose barrier started, [1] the last that ended, [2 + p] peer p's
// flag as last seen by a wait still running (a hang names the missing peer).
__global__ __launch_bounds__(64) void barrier_kernel(uint64_t *local, flag_set peers, int rank,
                                                     int size, uint64_t epoch, int *err,
                                                     uint64_t timeout_ticks, uint64_t *dbg) {
    const int t = threadIdx.x;
    if (dbg && t == 0)
        __hip_atomic_store(dbg, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    sys_release();
    if (t < size && t != rank)
        __hip_atomic_store(peers.p[t] + rank, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < size && t != rank)
        (void)wait_epoch(local + t, epoch, err, timeout_ticks, local + kAbortWord,
                         dbg ? dbg + 2 + t : nullptr);
    __syncthreads();
    sys_acquire();
    if (dbg && t == 0)
        __hip_atomic_store(dbg + 1, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------- copy
// Byte copy with a peeled head so that the body runs 16 B (or 4 B) per
// lane whenever src and dst share their alignment phase.
// one 8-byte load through a peer mapping, by the GPU's own page tables (the
// landing token check; hipMemcpy resolves the pointer through the runtime's
// memory-object map instead)
__global__ void peek_kernel(const uint64_t *src, uint64_t *dst) {
    *dst = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A deferred landing growth's token stamp and check (grow_launch), on the
// stream of the call it was queued for: land_stamp_kernel stores this
// rank's token into the last bytes of its new buffer, a device barrier of
// the communicator follows (every rank's stamp is out before any check),
// then land_check_kernel reads every peer's token through this process's
// new mapping of that peer's buffer.  A mapping that shows another token —
// it reaches another allocation — raises the communicator's error word and
// the peers' abort word.  No host wait and no stream of its own.
struct tok_set { uint64_t t[kMaxRanks]; };
struct tok_ptrs { const uint64_t *p[kMaxRanks]; };
__global__ void land_stamp_kernel(uint64_t *mine, uint64_t token) {
    __hip_atomic_store(mine, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    sys_release();
}
__global__ __launch_bounds__(64) void land_check_kernel(tok_ptrs peers, tok_set expect, int rank, int size,
                                                        int *err, uint64_t *abort_word) {
    const int t = threadIdx.x;
    sys_acquire();
    if (t >= size || t == rank) return;
    if (__hip_atomic_load(peers.p[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != expect.t[t]) {
        __hip_atomic_store(err, (int)OMPI_AMD_ERR_HIP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(abort_word, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// NT: non-temporal stores (streaming cache policy) — param "copy_nt" (which
// also sets the fold kernels' FOLD_NT_STORE), an A/B the 8-GPU bench
// measures for the remote stores of the scatter and push phases
template <bool NT>
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
            if constexpr (NT) {
                __builtin_nontemporal_store(a, d + i);
                __builtin_nontemporal_store(b, d + i + gstride);
                __builtin_nontemporal_store(c, d + i + 2 * gstride);
                __builtin_nontemporal_store(e, d + i + 3 * gstride);
            } else {
                d[i] = a;
                d[i + gstride] = b;
                d[i + 2 * gstride] = c;
                d[i + 3 * gstride] = e;
            }
        }
        for (; i < nbody; i += gstride) {
            if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
            else d[i] = __builtin_nontemporal_load(s + i);
        }
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
static red_launch_fn red_fn(int op, int type) {
    if (type < 0 || type >= OMPI_AMD_TYPE_COUNT) return nullptr;
    switch (op) {
#define CASE(k) case k: return red_row_##k()[type];
        OMPI_AMD_COLL_OPS(CASE)
#undef CASE
    default: return nullptr;
    }
}
static pipe_launch_fn pipe_fn(int op, int type) {
    if (type < 0 || type >= OMPI_AMD_TYPE_COUNT) return nullptr;
    switch (op) {
#define CASE(k) case k: return pipe_row_##k()[type];
        OMPI_AMD_COLL_OPS(CASE)
#undef CASE
    default: return nullptr;
    }
}
static fused_launch_fn fused_fn(int op, int type) {
    if (type < 0 || type >= OMPI_AMD_TYPE_COUNT) return nullptr;
    switch (op) {
#define CASE(k) case k: return fused_row_##k()[type];
        OMPI_AMD_COLL_OPS(CASE)
#undef CASE
    default: return nullptr;
    }
}

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
// forced: coll_tuned_reduce_algorithm under coll_tuned_use_dynamic_rules
// (coll_tuned_reduce_decision.c:146-179) — 1 basic_linear, 3 pipeline,
// 4 binary, 5 binomial; segmentation does not change an element's operand
// order (coll_base_reduce.c:62-260 folds each segment child by child), so
// the segment size is irrelevant here.  0 (and every value the library does
// not implement, which set_param refuses): the fixed decision.
// coll/tuned's forced-algorithm numbers the device path implements
// (coll_tuned_reduce_decision.c:35-44, coll_tuned_reduce_scatter_decision.c:
// 36-42, coll_tuned_reduce_scatter_block_decision.c:34-40).
enum { TUNED_RED_LINEAR = 1, TUNED_RED_PIPELINE = 3, TUNED_RED_BINARY = 4, TUNED_RED_BINOMIAL = 5 };
enum { TUNED_RS_NONOVERLAPPING = 1, TUNED_RS_HALVING = 2, TUNED_RS_RING = 3 };
enum { TUNED_RSB_BASIC_LINEAR = 1 };
static bool tuned_red_alg_ok(int64_t v) {
    return v == 0 || v == TUNED_RED_LINEAR || v == TUNED_RED_PIPELINE || v == TUNED_RED_BINARY ||
           v == TUNED_RED_BINOMIAL;
}

static red_order tuned_reduce_order(int n, size_t msg, size_t count, int root, bool root_inplace,
                                    int forced = 0) {
    const int flr = root_inplace ? FOLD_ROOT_INPLACE : 0;
    switch (forced) {
    case TUNED_RED_LINEAR: return {ORDER_CHAIN, 0, 0};
    case TUNED_RED_PIPELINE: return {ORDER_CHAIN, root, flr};
    case TUNED_RED_BINARY: return {ORDER_BINARY, root, flr};
    case TUNED_RED_BINOMIAL: return {ORDER_BINOMIAL, root, flr};
    default: break;
    }
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
    uint64_t id;    // HIP_POINTER_ATTRIBUTE_BUFFER_ID of the allocation in the exporter
    uint64_t base;  // the allocation's range in the exporter's address space
    uint64_t size;
    uint64_t pid;   // the exporter process (the registry's key, ipc_registry.h)
};
struct call_blob {
    buf_desc s, r;
    uint64_t flags;  // per-call rank flags (bit 0: MPI_IN_PLACE)
};
// a landing-buffer growth's contribution: the new buffer, the token stamped
// into its last bytes, whether this rank's allocation / export worked
struct land_blob {
    buf_desc d;
    uint64_t token;
    int ok;
};

// The parameters a path decision reads, captured when a nonblocking call is
// posted so that its deferred launch takes the path every rank agreed on.
struct fold_plan {
    int order;   // ORDER_*
    int first;   // virtual rank 0 of the uniform orders
    int flags;   // FOLD_ROOT_INPLACE (the reduce of nonoverlapping)
};
enum {
    TUNED_AR_FIXED = 0, TUNED_AR_BASIC_LINEAR = 1, TUNED_AR_NONOVERLAPPING = 2,
    TUNED_AR_RECURSIVE_DOUBLING = 3, TUNED_AR_RING = 4, TUNED_AR_RING_SEGMENTED = 5,
    TUNED_AR_RABENSEIFNER = 6, TUNED_AR_COUNT = 7
};

struct path_params {
    size_t small_bytes, fused_bytes;
    int zero_copy, algorithm;
    int tuned_alg;      // coll_tuned_allreduce_algorithm the user forced (0: fixed decision)
    int root0_inplace;  // forced nonoverlapping only: rank 0 passed MPI_IN_PLACE
    int push_gather;    // push / push-land scheme, staged (user_ipc 0): no handle swap at all
    int blocks = 0;     // transfer grid of a deferred call (nb_tuned); 0: the communicator's
    int copy_nt = -1;   // store kind of the copy / fold kernels (autotune); -1: the communicator's
    int red_alg = 0;    // coll_tuned_reduce_algorithm forced (nonoverlapping's reduce), 0: fixed
};

// Export fallback.  hipIpcGetMemHandle sometimes refuses a live device
// allocation (hipErrorInvalidValue on ROCm 7.2, seen for torch tensors after
// the caching allocator returned and re-took segments; not reproducible in
// a two-process probe, tools/ipc_alias_probe.hip S7-S12).  A zero-copy call
// then runs on this rank through a "shadow": an exportable buffer of the
// communicator that takes the user buffer's place for the peers — the send
// side is copied in before the call, the receive side copied out after its
// trailing barrier.  Purely local: the peers just map another allocation.
struct shadow_set {
    cp_jobs in{};          // user -> shadow, before the collective
    cp_job out{};          // shadow -> user rbuf, after its trailing barrier
    char *mem = nullptr;   // owned shadow memory (nonblocking / persistent calls)
    char *mem2 = nullptr;  //   its result region when input + result exceed one allocation
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
    shadow_set sh;  // export fallback of this call (sbuf / rbuf above are then the shadows)
    int kind = 0;   // PEND_*: which collective
    int root = 0;   // bcast, reduce
    bool inplace = false;  // rsb without a swap (staged push): MPI_IN_PLACE
    bool exclusive = false;        // scan: exscan
    bool land = false;             // allgather / bcast through the landing buffers (no swap)
    std::vector<size_t> rcounts;   // reduce_scatter
    // the ticket's blob while the rendezvous ring is full (nb_ticket): it is
    // posted from progress, in queue order, once every rank read the slot
    bool unposted = false;
    size_t blob_len = 0;
    union {
        call_blob call;
        land_blob land;
    } blob{};
    // PEND_GROW: this rank's new landing buffer (allocated at post time,
    // stamped on the device at launch), its size and token
    char *grow = nullptr;
    size_t grow_bytes = 0;
    uint64_t grow_token = 0;
};

enum { PEND_ALLREDUCE = 0, PEND_RSB = 1, PEND_ALLGATHER = 2, PEND_BCAST = 3, PEND_REDUCE = 4,
       PEND_SCAN = 5, PEND_RS = 6, PEND_GROW = 7 };

}  // namespace ompi_amd

using namespace ompi_amd;

// A nonblocking collective's completion (MPI_Request of MPI_Iallreduce).
struct ompi_amd_request {
    ~ompi_amd_request() { mark_word_put(mark); }  // freed after its wait: the mark has landed
    ompi_amd_comm_t *c = nullptr;
    hipEvent_t ev = nullptr;
    hipStream_t stream = nullptr;
    bool launched = false;  // its kernels are on `stream`
    bool recorded = false;  // `ev` recorded after them (lazily, at the first test / wait)
    uint64_t *mark = nullptr;  // host-observed completion word (below), with `ev`
    uint64_t mark_seq = 0;     //   the value it reaches; 0: no mark launched
    int rc = OMPI_AMD_SUCCESS;
    char *shadow = nullptr;  // export-fallback memory of the call, freed with the request
    char *shadow2 = nullptr; //   and its separate result region, if any
    // a small allreduce launched on the fused kernel that stores `mark`
    // itself: the value (0: none), its completion-counter slot, polls
    uint64_t embedded = 0;
    int done_slot = -1;
    unsigned polls = 0;
};

// ------------------------------------------------------------------ comm
// Autotuning of large staged allreduces (param "autotune"): the first
// kTuneRounds x kTuneCands blocking calls of a size bucket run the
// candidates (scheme x grid) in turn, each call timed with events on its
// stream after a device barrier (host skew between the ranks is not
// timed); a candidate's time is its best round (the bucket's first call
// also pays the one-time setup — landing growth, peer mappings).  At the
// last call the
// ranks allgather their times and every rank takes the candidate whose
// slowest rank was fastest — the same choice everywhere, since every rank
// makes the same calls.  coll/tuned's dynamic rules pick from a table;
// this picks from measurements on the machine it runs on (xGMI loads vs
// stores and the grid that saturates the links are not knowable offline).
// The store kind of the copy and fold kernels (non-temporal or plain) is a
// third dimension unless param copy_nt fixed it: remote xGMI stores may
// prefer either, and one GPU cannot tell — 18 candidates
// then, 18 with it fixed.  Schemes: push-gather, push-land, staged pull and
// their pipelined launches (round 4: phases overlapped by per-slice flags).
constexpr int kTuneGrid = 18, kTuneCands = 2 * kTuneGrid, kTuneRounds = 2,
              kTuneCalls = kTuneCands * kTuneRounds;
struct tune_cand {
    int algorithm, blocks, nt;  // nt: 1 non-temporal stores, 0 plain
};
static const tune_cand kTune[kTuneCands] = {
    {2, 1024, 1}, {2, 512, 1}, {2, 256, 1}, {3, 1024, 1}, {3, 512, 1}, {3, 256, 1},
    {0, 1024, 1}, {0, 512, 1}, {0, 256, 1}, {4, 1024, 1}, {4, 512, 1}, {4, 256, 1},
    {5, 1024, 1}, {5, 512, 1}, {5, 256, 1}, {6, 1024, 1}, {6, 512, 1}, {6, 256, 1},
    {2, 1024, 0}, {2, 512, 0}, {2, 256, 0}, {3, 1024, 0}, {3, 512, 0}, {3, 256, 0},
    {0, 1024, 0}, {0, 512, 0}, {0, 256, 0}, {4, 1024, 0}, {4, 512, 0}, {4, 256, 0},
    {5, 1024, 0}, {5, 512, 0}, {5, 256, 0}, {6, 1024, 0}, {6, 512, 0}, {6, 256, 0}};
struct tune_bucket {
    int ncand = kTuneCands;  // candidates tried: kTuneGrid when copy_nt is fixed
    int next = 0;            // calls made so far; call k runs candidate k % ncand
    bool done = false;
    int choice = 0;
    hipEvent_t ev[2 * kTuneCalls] = {};
    float worst_ms[kTuneCands] = {};
};

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
    ipc_ref *land_ref[kMaxRanks] = {};   // peers' landing buffers (IPC registry references)
    // Deferred growth (nonblocking calls, PEND_GROW): land_planned is the
    // size once every queued growth has launched — what a post compares
    // against.  The buffers any growth replaced stay allocated (and mapped)
    // until destroy: land_retired / land_ref_retired (hipFree and IPC
    // closes may wait for every kernel of the device).
    size_t land_planned = 0;
    std::vector<char *> land_retired;
    std::vector<ipc_ref *> land_ref_retired;
    bool land_failed = false;             // a deferred growth failed: nothing after it launches
    int unposted = 0;                     // pending ops whose ticket waits for a ring slot
    int64_t deferred_growths = 0;         // landing growths taken from progress (counter)
    std::vector<uint64_t> land_tokens;    // every rank's token of every landing growth (diagnostics)
    int memcpy_token_mismatch = 0;        // landing tokens right by kernel load, wrong by hipMemcpy
    int bcast_split = 0;                  // bcasts that ran as scatter + allgather
    size_t bcast_split_bytes = 4u << 20;  // from this size on (0: never)
    int64_t exports_new = 0, imports_new = 0;  // runtime export / open calls made (cache misses)
    int recycled_exports = 0;             // exports refused: recycled handle bytes (shadowed)
    int64_t reused_exports = 0;           // not exported: an address exported before under another id (shadowed)
    int reuse_shadow = 1;                 // param "reuse_shadow": 0 exports such allocations (registry tests)
    int unsafe_exports = 0;               // application buffers of no IPC-safe size (shadowed)
    int aged_exports = 0;                 // application buffers older than an IPC close (shadowed)
    // streams this communicator launched work on: the current one, plus an
    // event recorded on each earlier one when the calls moved away from it
    // (quiesce() waits for exactly that work, not for the whole device)
    // (stream_mu: quiesce() also runs on other threads, from the IPC
    // registry's retirement of a mapping this communicator holds)
    std::mutex stream_mu;
    // api_mu: held by every entry point for its whole call (recursive: entry
    // points call each other); progress_others() takes it with try_lock
    std::recursive_mutex api_mu;
    std::atomic<int> npending{0};  // deferred calls not yet launched (pending.size())
    bool has_stream = false;
    hipStream_t cur_stream = nullptr;
    // param own_stream (coll/rocm sets it): every call runs on `own`, a
    // stream on a hardware queue of its own (comm_stream)
    int own_stream = 0;
    hipStream_t own = nullptr;
    // another communicator launched on cur_stream after this one's last
    // launch there: stream_evs holds the mark of this one's end on it, and
    // quiesce() must not synchronise the stream (note_stream)
    bool cur_closed = false;
    std::vector<hipEvent_t> stream_evs;
    char *shadow = nullptr;               // export fallback of blocking calls (shadow_set)
    size_t shadow_bytes = 0;
    char *shadow2 = nullptr;              //   its result region when both exceed one allocation
    size_t shadow2_bytes = 0;
    // Shadow arena: every shadow (blocking, nonblocking, persistent) is a
    // range of a chunk that is exported once and freed only with the
    // communicator, so peers map each chunk once and no exported address is
    // ever freed and handed out again (the churn behind the runtime's stale
    // import answers).
    struct arena_chunk {
        char *base;
        size_t size;
        std::map<size_t, size_t> free;  // offset -> bytes, coalesced
        std::map<size_t, size_t> used;  // offset -> bytes
    };
    std::mutex arena_mu;
    std::vector<arena_chunk> arena;
    size_t arena_bytes = 0;
    int shadowed = 0;                     // zero-copy calls that needed it
    int force_shadow = 0;                 // param "force_shadow": take the fallback always (tests)
    int win_shadow = 0;                   // param "osc_win_shadow": 1 = every MPI_Win_create shadowed (tests)
    int win_separate = 1;                 // param "osc_win_separate": 0 = refuse a window that needs a public copy
    int64_t shadow_windows = 0;           // MPI_Win_create windows in the separate model (osc_ipc.hip)
    // param "user_ipc" (env OMPI_AMD_USER_IPC): export the caller's buffers
    // to peers (zero-copy).  Off by default: every zero-copy-size call stages
    // through the shadow arena (exported once, never freed), because on ROCm
    // 7.2 an IPC mapping of an application buffer names (pid, address), not
    // the allocation — after the application frees and reallocates, cached
    // or freshly opened mappings were seen to reach other memory (DESIGN.md
    // §4.6: wrong blocks, illegal-address faults, refused opens).
    int user_ipc = 0;
    int *err_host = nullptr, *err_dev = nullptr;
    uint64_t *dbg_host = nullptr, *dbg_dev = nullptr;  // OMPI_AMD_DEBUG_PROGRESS=1 (barrier_kernel)
    uint64_t epoch = 0;
    // ompi_amd_allreduce_wait: the fused launch stores its own host mark
    // (fused_mark: this communicator's pinned word; want_mark set for the
    // duration of that call; mark_embedded the value it stores, 0 none)
    uint64_t *fused_mark = nullptr;
    bool want_mark = false;
    uint64_t mark_embedded = 0;
    // the word and completion-counter slot the next fused launch signals
    // (want_mark): fused_mark and slot 0 for the blocking call, a plan's own
    // word and slot for a persistent start (plan_enqueue)
    uint64_t *mark_word = nullptr;
    int mark_slot = 0;
    std::vector<int> done_free;  // counter slots of freed plans
    int done_next = 1;           // slot 0: the blocking call
    // params
    size_t small_bytes = 1 << 20;
    size_t fused_bytes = 64 << 10;
    int zero_copy = 1;
    int64_t timeout_ms = 30000;
    int max_blocks = 1024;
    // pipelined schemes: every workgroup of the grid runs pipe_passes
    // slices of each block (param "pipe_passes"), none under pipe_slice
    // bytes (param "pipe_slice"; smaller messages use fewer workgroups);
    // pipe_seq numbers the pipelined calls (flag values)
    int64_t pipe_slice = 64 << 10;
    int pipe_passes = 1;
    uint64_t pipe_seq = 0;
    int colocated = 1;  // most ranks of this communicator on one GPU (pipe_args.colocated)
    int algorithm = 2;                    // push: push-gather in the staged mode (no staging copy)
    // param "autotune" (0 here; coll/rocm turns it on): large blocking
    // allreduces pick their scheme and grid by measurement (tune_bucket)
    int autotune = 0;
    std::map<int, struct tune_bucket> tune;  // by floor(log2(bytes))
    int tune_last = 0;                       // last bucket touched: 0 none, 1 tuning, 2 decided
    int tune_last_key = -1;
    // the scheme / grid the last nonblocking or persistent allreduce of an
    // autotuned size took (nb_tuned; -1: none yet)
    int nb_tuned_alg = -1, nb_tuned_blocks = -1, nb_tuned_nt = -1;
    int64_t land_ag_bcast = 0;  // allgathers / bcasts run through the landing buffers
    // param "land_blocking" (0): blocking allgather / bcast of a zero-copy
    // size take the landing path too (an A/B the 8-GPU bench measures)
    int land_blocking = 0;
    // param "copy_nt": 1 the copy and fold kernels store non-temporally —
    // measured no slower on one GPU at N = 2 / 4 / 8 (scatter, gather and fold
    // kernels 1-5 % faster) — 0 plain stores; -1 (default)
    // non-temporal, and the autotune measures both (copy_nt_fixed 0)
    int copy_nt = 1;
    int copy_nt_fixed = 0;
    int tuned_alg = 0;                    // coll_tuned_allreduce_algorithm (forced), 0 = fixed
    int tuned_red_alg = 0;                // coll_tuned_reduce_algorithm (forced, TUNED_RED_*)
    int tuned_rs_alg = 0;                 // coll_tuned_reduce_scatter_algorithm (TUNED_RS_*)
    int tuned_rsb_alg = 0;                // coll_tuned_reduce_scatter_block_algorithm (TUNED_RSB_*)
    // this communicator's references to peer mappings (the mappings
    // themselves are process-wide: ipc_registry.h), least recently used
    // evicted past 256
    struct imp_entry {
        int peer;
        hipIpcMemHandle_t h;
        uint64_t id, rbase, rsize;  // the allocation in the exporter (buf_desc)
        ipc_ref *ref;
        void *base;                 // its mapping here
        uint64_t last_use;
        int pins;
    };
    std::vector<imp_entry> imports;
    uint64_t use_clock = 0;
    ipc_ref *opened[kMaxRanks][2] = {};   // peers' flag pages / scratch
    // per-phase kernel timing (param "profile"): event pairs per call
    int profile = 0;
    std::vector<hipEvent_t> ev_free;
    std::vector<hipEvent_t> req_ev_free;  // nonblocking requests' completion events, reused
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_phase[3];  // fold, gather, scatter
    // nonblocking calls not launched yet, and the swapped blobs of the one
    // being launched (exchange_bufs takes them instead of a rendezvous)
    std::deque<pending_op> pending;
    const call_blob *pre = nullptr;
    // point-to-point mailboxes (p2p.cpp)
    p2p_state *p2p = nullptr;
    // per-communicator state of the one-sided part (osc_ipc.hip): released
    // by destroy in two phases (comm_internal.h comm_set_osc_state)
    void *osc_state = nullptr;
    void (*osc_release)(void *, int) = nullptr;
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
    ompi_amd::path_params pp{};  // the parameters (and forced algorithm) fixed at init
    ompi_amd::fold_plan fp{};
    ptr_set sp{}, rp{};
    void *bases[OMPI_AMD_MAX_RANKS][2] = {};  // pinned peer mappings
    // completion: recorded on the start's stream at the first test / wait
    // after a start (a later point in the stream, so never early; keeps an
    // event record out of the start itself)
    hipEvent_t done = nullptr;
    hipStream_t stream = nullptr;
    bool started = false, recorded = false;
    uint64_t *mark = nullptr;  // host-observed completion word, with `done`
    uint64_t mark_seq = 0;
    // a small-path start whose fused kernel stores `mark` itself: the value
    // (0: none — the event and a mark kernel at the first test / wait), the
    // plan's completion-counter slot in the flag page, backstop poll count
    uint64_t embedded = 0;
    int done_slot = -1;
    unsigned polls = 0;
    ~ompi_amd_plan() { mark_word_put(mark); }
    shadow_set sh;  // export fallback (src / rbuf above are then the shadows)
    // kind 4: a persistent reduce_scatter_block / allgather / bcast — every
    // start posts the nonblocking call with the init's arguments (PEND_*
    // below), whose request the plan's test / wait / free follow
    int nb_kind = -1;
    int root = 0;
    size_t bytes = 0;
    bool exclusive = false;        // PEND_SCAN: exscan
    std::vector<size_t> rcounts;   // PEND_RS: the init's counts
    ompi_amd_request *req = nullptr;
};

namespace ompi_amd {

enum {
    ALG_PULL = 0, ALG_PULL_PUSH = 1, ALG_PUSH = 2, ALG_PUSH_LAND = 3,
    // the staged schemes' phases in one pipelined launch (pipe_allreduce_kernel)
    ALG_PUSH_PIPE = 4, ALG_LAND_PIPE = 5, ALG_PULL_PIPE = 6,
    ALG_COUNT = 7
};
// push-land is the staged push whose second phase also stores (the owners
// push their results into every rank's landing buffer) instead of loading;
// with user_ipc it is the push scheme (results stored into the rbufs)
static inline bool is_push(int alg) {
    return alg == ALG_PUSH || alg == ALG_PUSH_LAND || alg == ALG_PUSH_PIPE || alg == ALG_LAND_PIPE;
}
static inline bool is_land(int alg) { return alg == ALG_PUSH_LAND || alg == ALG_LAND_PIPE; }
static inline bool is_pipe(int alg) { return alg >= ALG_PUSH_PIPE; }

struct ipc_blob {
    buf_desc flags, scratch;
    int pci[3];  // the rank's GPU (domain, bus, device): ranks sharing one GPU
};


static int set_dev(ompi_amd_comm_t *c) {
    return record_hip(hipSetDevice(c->device), "hipSetDevice");
}

// Every IPC handle this process has exported, with the allocation it
// named.  On ROCm 7.2 with dmabuf IPC a new allocation can be handed the
// very handle bytes of a freed one (profiles/r02_coll_free_realloc*: most
// re-allocations at a freed address did), and a peer that still maps — or
// just closed — the freed one may then get the old memory back for the new
// handle (round 1's stale landing data; round 2's free/realloc push cases
// with all peer blocks missing).  A handle is therefore never published
// for a second allocation: export_buf sends such a buffer through its
// shadow, alloc_exportable retries while holding the colliding allocation.
// The process's IPC exports, one per allocation (base, size, HIP buffer
// id): every export — user buffers, shadows, landing, scratch, flag pages
// — goes through export_alloc, so an allocation is exported once and its
// handle stays the one peers already know (a second hipIpcGetMemHandle on
// the same allocation can return other bytes).  Records of freed
// allocations are kept as the handle history: an allocation whose handle
// bytes equal an older record's is "recycled" and never published.
struct export_rec {
    void *base;
    size_t size;
    unsigned long long id;
    hipIpcMemHandle_t h;
    bool recycled;
};
static std::mutex g_exp_mu;
static std::vector<export_rec> g_exp;

// 0: *h exported (fresh if *fresh), 1: recycled handle bytes, <0: the
// runtime refused (*e).
static int quiesce(ompi_amd_comm_t *c, const char *why = "quiesce");

// OMPI_AMD_IPC_TRACE=1: one stderr line per new export and per new import
// (handle words 0-15), for diagnosing mapping mix-ups after the fact.
static bool ipc_trace() {
    static const bool on = [] {
        const char *v = getenv("OMPI_AMD_IPC_TRACE");
        return v && *v == '1';
    }();
    return on;
}

// OMPI_AMD_TRACE=1: one stderr line before and after each host step that
// can block (allocations, exports, opens, rendezvous, stream drains), with
// its duration — a stuck rank names the step it sits in.
static bool host_trace() {
    static const bool on = [] {
        const char *v = getenv("OMPI_AMD_TRACE");
        return v && *v == '1';
    }();
    return on;
}

struct host_step {
    const char *what;
    size_t arg;
    std::chrono::steady_clock::time_point t0;
    host_step(const char *w, size_t a = 0) : what(w), arg(a), t0(std::chrono::steady_clock::now()) {
        if (host_trace()) fprintf(stderr, "[trace pid %d] %s %zu ...\n", (int)getpid(), what, arg);
    }
    ~host_step() {
        if (!host_trace()) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        fprintf(stderr, "[trace pid %d] %s %zu done %.3f ms\n", (int)getpid(), what, arg, ms);
    }
};

static void trace_handle(const char *what, const hipIpcMemHandle_t &h, const char *fmt, ...) {
    if (!ipc_trace()) return;
    char head[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(head, sizeof(head), fmt, ap);
    va_end(ap);
    unsigned w[16];
    memcpy(w, &h, sizeof(w));
    fprintf(stderr, "[ipc pid %d] %s %s h=", (int)getpid(), what, head);
    for (int i = 0; i < 16; ++i) fprintf(stderr, "%08x%s", w[i], i == 15 ? "\n" : ".");
}

// Handle identity: all 64 bytes.  On ROCm 7.2 words 0-12 are (exporter
// address, pid, descriptor, size, offset, pid) and words 13-15 vary between
// exports of one allocation (tools/ipc_handle_dump.hip, OMPI_AMD_IPC_TRACE);
// comparing words 0-12 only would call every same-size reallocation at a
// reused address "recycled" — round 2 tried that: the export history then
// refuses most library reallocations (osc control pages) and sends far more
// calls through the shadow fallback.  The full comparison flags the
// allocations whose whole handle repeats, as measured in round 1.
static bool same_handle(const hipIpcMemHandle_t &a, const hipIpcMemHandle_t &b) {
    return memcmp(&a, &b, sizeof(a)) == 0;
}

static int export_alloc(void *base, size_t size, unsigned long long id, hipIpcMemHandle_t *h,
                        hipError_t *e, bool *fresh) {
    std::lock_guard<std::mutex> g(g_exp_mu);
    *fresh = false;
    *e = hipSuccess;
    for (const auto &r : g_exp)
        if (r.base == base && r.size == size && r.id == id) {
            *h = r.h;
            return r.recycled ? 1 : 0;
        }
    {
        host_step st("hipIpcGetMemHandle", size);
        *e = hipIpcGetMemHandle(h, base);
    }
    if (*e != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    *fresh = true;
    bool recycled = false;
    for (const auto &r : g_exp) recycled = recycled || same_handle(r.h, *h);
    trace_handle("export", *h, "%p+%zu id %llu%s", base, size, id, recycled ? " RECYCLED" : "");
    g_exp.push_back({base, size, id, *h, recycled});
    return recycled ? 1 : 0;
}

// Whether this process exported (base, size, id) before: its handle was
// made before any later close, so it stays valid (ipc_close_watermark).
static bool export_known(void *base, size_t size, unsigned long long id) {
    std::lock_guard<std::mutex> g(g_exp_mu);
    for (const auto &r : g_exp)
        if (r.base == base && r.size == size && r.id == id) return true;
    return false;
}

// An allocation at an address this process exported before under another
// buffer id (the earlier allocation freed, the address handed out again):
// a peer that mapped the earlier one retires that mapping and opens this
// one's handle right after the close, and ROCm 7.2 refused such an open
// ("invalid device pointer") about once in several hundred re-imports of a
// 20 MiB torch segment (round 4's N = 8 user_ipc_free_realloc, round 5's
// ipc-share realloc step) — no replay order reproduces it on demand, so the
// sequence is avoided instead: such an allocation is never exported where
// the caller has somewhere else to put the bytes (shadow, stage, public
// window copy).  Library allocations never reuse an exported address
// (alloc_exportable keeps a repeated one alive).
static bool export_reused(void *base, unsigned long long id) {
    std::lock_guard<std::mutex> g(g_exp_mu);
    for (const auto &r : g_exp)
        if (r.base == base && r.id != id) return true;
    return false;
}

// An allocation this process may not export any more: it predates a close
// of one of its IPC mappings (ROCm 7.2 then refuses its export, for good,
// 10-30 % of the time — ipc_registry.h) and was not exported before.
static bool export_aged(void *base, size_t size, unsigned long long id) {
    return id < ipc_close_watermark() && !export_known(base, size, id);
}

// IPC-safe allocation sizes on ROCm 7.2 (tools/ipc_replay_probe.py,
// profiles/r04_ipc_replay*.jsonl, N = 4 / 8 processes on one MI355X):
//  - below 2 MiB hipMalloc sub-allocates from a shared chunk, and the import
//    of such a buffer is refused ("invalid device pointer", the runtime
//    printing "IPC Attach: Invalid IPC handle! <id> and 0") every time once
//    another exported buffer of the chunk was freed, and 1-2 times in 400
//    opens even when none was; an exactly 2 MiB one 1-2 times in 500;
//  - an allocation whose size is not a multiple of 2 MiB, freed and its
//    address reused by the next one, gets that one's import refused 2-5 times
//    in 500 (the registry's retire-then-open order);
//  - multiples of 2 MiB from 4 MiB up: no refusal in any order (thousands of
//    opens).
// Every library allocation peers map is sized accordingly (alloc_exportable),
// and an application buffer that is not (user_ipc) goes through a shadow.
constexpr size_t kIpcGrain = 2u << 20, kIpcMinBytes = 4u << 20;
static size_t ipc_size_for(size_t bytes) {
    return std::max(kIpcMinBytes, (bytes + kIpcGrain - 1) / kIpcGrain * kIpcGrain);
}
static bool ipc_safe_size(size_t size) { return size >= kIpcMinBytes && size % kIpcGrain == 0; }

static unsigned long long buffer_id(const void *p) {
    unsigned long long id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return id;
}

// The descriptor peers map an exported library allocation by (the handle
// is already in d->h): the allocation's real range, buffer id and process.
static void describe_alloc(void *p, buf_desc *d) {
    void *ab = p;
    size_t as = 0;
    if (hipMemGetAddressRange((hipDeviceptr_t *)&ab, &as, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        ab = p;
    }
    d->off = (uint64_t)((char *)p - (char *)ab);
    d->valid = 1;
    d->id = buffer_id(p);
    d->base = (uint64_t)(uintptr_t)ab;
    d->size = as;
    d->pid = (uint64_t)getpid();
}

// ipc_failed: set when the runtime refused to export a live device
// allocation, or handed it recycled handle bytes (the shadow fallback
// applies); other failures are errors.
static int export_buf(ompi_amd_comm_t *c, const void *ptr, buf_desc *d, bool *ipc_failed = nullptr) {
    memset(d, 0, sizeof(*d));
    if (ipc_failed) *ipc_failed = false;
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
    d->id = id;
    d->base = (uint64_t)(uintptr_t)base;
    d->size = (uint64_t)size;
    if (size > kMaxIpcBytes) {  // peers could not open it: the shadow path
        if (ipc_failed) *ipc_failed = true;
        record_msg("allocation %p + %zu exceeds the %zu-byte IPC mapping limit", base, size,
                   kMaxIpcBytes);
        return OMPI_AMD_ERR_HIP;
    }
    if (ipc_failed && !ipc_safe_size(size)) {  // a caller with a shadow: use it
        *ipc_failed = true;
        ++c->unsafe_exports;
        record_msg("allocation %p + %zu is not an IPC-safe size (a multiple of 2 MiB from 4 MiB)",
                   base, size);
        return OMPI_AMD_ERR_HIP;
    }
    // A caller with a shadow never offers an allocation a close spoiled
    // (ipc_registry.h).  One without (a window over the caller's memory)
    // tries: most such exports work, and a refusal fails every rank alike.
    if (ipc_failed && c->reuse_shadow && export_reused(base, id)) {
        *ipc_failed = true;
        ++c->reused_exports;
        record_msg("allocation %p + %zu (id %llu) reuses an address this process exported before: not "
                   "exported (DESIGN.md §4.6)", base, size, id);
        return OMPI_AMD_ERR_HIP;
    }
    if (ipc_failed && export_aged(base, size, id)) {
        *ipc_failed = true;
        ++c->aged_exports;
        record_msg("allocation %p + %zu (id %llu) predates an IPC close of this process: not exported "
                   "(DESIGN.md §4.6)", base, size, id);
        return OMPI_AMD_ERR_HIP;
    }
    hipIpcMemHandle_t h;
    bool fresh = false;
    const int rc = export_alloc(base, size, id, &h, &e, &fresh);
    c->exports_new += fresh ? 1 : 0;
    if (rc < 0) {
        hipPointerAttribute_t at{};
        const hipError_t ea = hipPointerGetAttributes(&at, ptr);
        (void)hipGetLastError();
        record_msg("hipIpcGetMemHandle: %s (ptr %p in allocation %p + %zu, buffer id %llu, "
                   "attr rc %d type %d device %d)",
                   hipGetErrorString(e), ptr, base, size, (unsigned long long)id, (int)ea,
                   (int)at.type, at.device);
        if (ipc_failed) *ipc_failed = true;
        return OMPI_AMD_ERR_HIP;
    }
    if (rc == 1) {
        c->recycled_exports += fresh ? 1 : 0;
        if (ipc_failed) *ipc_failed = true;
        record_msg("allocation %p + %zu (id %llu) carries a recycled IPC handle", base, size, id);
        return OMPI_AMD_ERR_HIP;
    }
    d->h = h;
    d->off = (uint64_t)((const char *)ptr - (const char *)base);
    d->valid = 1;
    d->pid = (uint64_t)getpid();
    return OMPI_AMD_SUCCESS;
}

static ipc_alloc alloc_of(const buf_desc &d) { return ipc_alloc{d.h, d.pid, d.id, d.base, d.size}; }

// This rank failed a call its peers may have launched: make the failure
// sticky here and raise every peer's abort word (their barrier waits then
// give up within ~1 ms and their calls fail with OMPI_AMD_ERR_TIMEOUT).
static void abort_peers(ompi_amd_comm_t *c, int rc) {
    int expect = 0;
    (void)__atomic_compare_exchange_n(c->err_host, &expect, rc, false, __ATOMIC_ACQ_REL,
                                      __ATOMIC_ACQUIRE);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    hipLaunchKernelGGL(abort_kernel, dim3(1), dim3(64), 0, s, c->peer_flags, c->flags, c->rank,
                       c->size);
    if (hipGetLastError() == hipSuccess) hip_ignore(hipStreamSynchronize(s));
    (void)hipGetLastError();
    hip_ignore(hipStreamDestroy(s));
}

// Drop this communicator's references to mappings the registry retired
// (their exporter freed the allocation).  A pinned one is reported: a
// persistent operation of this communicator still uses it.
static int drop_retired(ompi_amd_comm_t *c) {
    for (auto it = c->imports.begin(); it != c->imports.end();) {
        if (!ipc_retired(it->ref)) {
            ++it;
            continue;
        }
        if (it->pins > 0) {
            record_msg("rank %d freed a buffer (id %llu) that a persistent collective still maps",
                       it->peer, (unsigned long long)it->id);
            return OMPI_AMD_ERR_BAD_PARAM;
        }
        ipc_unmap(it->ref, c);
        it = c->imports.erase(it);
    }
    return OMPI_AMD_SUCCESS;
}

// Map peer `peer`'s buffer `d` (cached per communicator; the mapping itself
// is the process's, shared through the IPC registry).  One attempt: a
// refused or wrong answer from the runtime is an error, never retried.
static int import_buf(ompi_amd_comm_t *c, int peer, const buf_desc &d, const char **out,
                      bool pin = false, void **base_out = nullptr) {
    *out = nullptr;
    if (base_out) *base_out = nullptr;
    if (!d.valid) return OMPI_AMD_SUCCESS;
    TRY(drop_retired(c));
    for (auto &x : c->imports) {
        if (x.peer == peer && x.id == d.id && x.rbase == d.base && x.rsize == d.size &&
            same_handle(x.h, d.h)) {
            x.last_use = ++c->use_clock;
            if (pin) {
                ++x.pins;
                ipc_pin(x.ref, 1);
            }
            *out = (const char *)x.base + d.off;
            if (base_out) *base_out = x.base;
            return OMPI_AMD_SUCCESS;
        }
    }
    if (c->imports.size() >= 256) {  // evict the least recently used unpinned reference
        auto it = c->imports.end();
        for (auto jt = c->imports.begin(); jt != c->imports.end(); ++jt)
            if (jt->pins == 0 && (it == c->imports.end() || jt->last_use < it->last_use)) it = jt;
        if (it != c->imports.end()) {
            TRY(quiesce(c, "quiesce (import eviction)"));  // an earlier call's kernel may still read it
            ipc_unmap(it->ref, c);
            c->imports.erase(it);
        }
    }
    ipc_ref *ref = nullptr;
    void *base = nullptr;
    {
        host_step st("ipc_map", (size_t)d.size);
        TRY(ipc_map(alloc_of(d), c, &ref, &base));
    }
    ++c->imports_new;
    if (pin) ipc_pin(ref, 1);
    c->imports.push_back({peer, d.h, d.id, d.base, d.size, ref, base, ++c->use_clock, pin ? 1 : 0});
    *out = (const char *)base + d.off;
    if (base_out) *base_out = base;
    return OMPI_AMD_SUCCESS;
}

static void unpin_import(ompi_amd_comm_t *c, void *base) {
    for (auto &x : c->imports)
        if (x.base == base && x.pins > 0) {
            --x.pins;
            ipc_pin(x.ref, -1);
            return;
        }
}

static int import_all(ompi_amd_comm_t *c, const call_blob *all, const void *sbuf, const void *rbuf,
                      ptr_set *s, ptr_set *r, uint64_t *allflags, bool pin, void *(*bases)[2]);

// Swap (sbuf, rbuf) descriptors with every peer and map theirs (either may
// be NULL: nothing is exported for it).
static int exchange_bufs(ompi_amd_comm_t *c, const void *sbuf, const void *rbuf, ptr_set *s,
                         ptr_set *r, uint64_t myflags = 0, uint64_t *allflags = nullptr,
                         bool pin = false, void *(*bases)[2] = nullptr) {
    call_blob mine{};
    mine.flags = myflags;
    int rc = export_buf(c, sbuf, &mine.s);
    if (rc == OMPI_AMD_SUCCESS) rc = export_buf(c, rbuf, &mine.r);
    if (rc != OMPI_AMD_SUCCESS && !c->pre) {
        // still take part in the swap (peers must not wait for this rank at
        // the rendezvous), then stop their device work
        call_blob all_[kMaxRanks];
        mine = call_blob{};
        (void)c->boot.allgather(&mine, all_, sizeof(call_blob));
        abort_peers(c, rc);
        return rc;
    }
    if (rc != OMPI_AMD_SUCCESS) return rc;
    call_blob all[kMaxRanks];
    if (c->pre) {  // a deferred nonblocking call: swapped when it was posted
        memcpy(all, c->pre, sizeof(call_blob) * (size_t)c->size);
    } else {
        host_step st("exchange allgather");
        rc = c->boot.allgather(&mine, all, sizeof(call_blob));
        if (rc != OMPI_AMD_SUCCESS) return rc;
    }
    return import_all(c, all, sbuf, rbuf, s, r, allflags, pin, bases);
}

// Map every peer's (s, r) descriptors of `all`.  A failure is final for
// this communicator: the peers' device work of the call is stopped through
// their abort words (abort_peers) instead of a confirmation rendezvous.
static int import_all(ompi_amd_comm_t *c, const call_blob *all, const void *sbuf, const void *rbuf,
                      ptr_set *s, ptr_set *r, uint64_t *allflags, bool pin,
                      void *(*bases)[2]) {
    int rc = OMPI_AMD_SUCCESS;
    for (int p = 0; p < c->size; ++p) {
        if (allflags) allflags[p] = all[p].flags;
        if (p == c->rank) {
            s->p[p] = (const char *)sbuf;
            r->p[p] = (const char *)rbuf;
            continue;
        }
        if (rc != OMPI_AMD_SUCCESS) continue;
        void *b0 = nullptr, *b1 = nullptr;
        rc = import_buf(c, p, all[p].s, &s->p[p], pin, &b0);
        if (rc == OMPI_AMD_SUCCESS) rc = import_buf(c, p, all[p].r, &r->p[p], pin, &b1);
        if (rc != OMPI_AMD_SUCCESS && b0 && pin) unpin_import(c, b0);
        if (rc == OMPI_AMD_SUCCESS && bases) {
            bases[p][0] = b0;
            bases[p][1] = b1;
        }
    }
    if (rc != OMPI_AMD_SUCCESS) abort_peers(c, rc);
    return rc;
}

// Work this communicator put on a stream: note the stream; when the calls
// move to another stream, an event marks the end of the old one's work.
// The communicator that launched last on each stream (process-wide): when
// another one launches there, an event marks where the first one's work on
// that stream ends, so that quiescing it (the IPC registry retiring a
// mapping it holds) waits for its own kernels only — not for a later
// communicator's, which may be waiting on device for peers that are
// themselves waiting for this rank (a deferred call of A
// launched here, B retiring a mapping on the same stream).
static std::mutex g_stream_owner_mu;
static std::vector<std::pair<hipStream_t, ompi_amd_comm_t *>> g_stream_owner;

static void mark_end(ompi_amd_comm_t *o, hipStream_t s) {
    std::lock_guard<std::mutex> g(o->stream_mu);
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
        if (hipEventRecord(e, s) == hipSuccess) o->stream_evs.push_back(e);
        else hip_ignore(hipEventDestroy(e));
    }
    (void)hipGetLastError();
    if (o->has_stream && o->cur_stream == s) o->cur_closed = true;
}

static void forget_streams(ompi_amd_comm_t *c) {
    std::lock_guard<std::mutex> g(g_stream_owner_mu);
    g_stream_owner.erase(std::remove_if(g_stream_owner.begin(), g_stream_owner.end(),
                                        [&](const std::pair<hipStream_t, ompi_amd_comm_t *> &p) {
                                            return p.second == c;
                                        }),
                         g_stream_owner.end());
}

static void note_stream(ompi_amd_comm_t *c, hipStream_t s) {
    {
        std::lock_guard<std::mutex> g(g_stream_owner_mu);
        bool found = false;
        for (auto &p : g_stream_owner)
            if (p.first == s) {
                if (p.second != c) mark_end(p.second, s);
                p.second = c;
                found = true;
                break;
            }
        if (!found) g_stream_owner.emplace_back(s, c);
    }
    std::lock_guard<std::mutex> g(c->stream_mu);
    if (c->has_stream && c->cur_stream == s) {
        c->cur_closed = false;
        return;
    }
    if (c->has_stream) {
        // the communicator's calls run one after the other on the device
        // whatever streams they were issued on (MPI orders a communicator's
        // collectives; the staged calls' scratch halves, the barrier rows and
        // the landing buffers are reused call after call on that premise):
        // the new stream waits for the last one's work so far
        // (hipStreamLegacy, the C ABI's spelling of the legacy null
        // stream, as the null handle: hipStreamWaitEvent does not take it)
        auto plain = [](hipStream_t x) { return x == hipStreamLegacy ? nullptr : x; };
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
            if (hipEventRecord(e, plain(c->cur_stream)) == hipSuccess) {
                hip_ignore(hipStreamWaitEvent(plain(s), e, 0));
                c->stream_evs.push_back(e);
            } else {
                hip_ignore(hipEventDestroy(e));
            }
        }
        // forget marks that have fired
        for (auto it = c->stream_evs.begin(); c->stream_evs.size() > 8 && it != c->stream_evs.end();) {
            if (hipEventQuery(*it) == hipSuccess) {
                hip_ignore(hipEventDestroy(*it));
                it = c->stream_evs.erase(it);
            } else {
                ++it;
            }
        }
        (void)hipGetLastError();
    }
    c->cur_stream = s;
    c->has_stream = true;
    c->cur_closed = false;
}

// Wait until every kernel this communicator launched has finished (its
// streams only: an application's unrelated work on the device is not
// waited for, unlike hipDeviceSynchronize).
}  // namespace ompi_amd
// (defined below, outside the namespace, beside progress_others)
static hipError_t wait_stream(hipStream_t s);
static hipError_t wait_event(hipEvent_t ev);
namespace ompi_amd {

static int quiesce_user(void *c) {
    return quiesce(static_cast<ompi_amd_comm_t *>(c), "quiesce (holder of a stale IPC mapping)");
}

static int quiesce(ompi_amd_comm_t *c, const char *why) {
    host_step st(why);
    std::vector<hipEvent_t> evs;
    hipStream_t cur = nullptr;
    bool has = false;
    {  // the marks are this call's from here on (note_stream may add new ones)
        std::lock_guard<std::mutex> g(c->stream_mu);
        evs.swap(c->stream_evs);
        cur = c->cur_stream;
        has = c->has_stream && !c->cur_closed;  // closed: a mark in evs bounds it
    }
    // the waits launch other communicators' ready deferred calls meanwhile
    // (progress_others): this communicator's kernels may be waiting for a
    // peer that waits for this rank's launch of another communicator's call
    int rc = OMPI_AMD_SUCCESS;
    for (hipEvent_t e : evs) {
        const hipError_t r = ::wait_event(e);
        hip_ignore(hipEventDestroy(e));
        if (r != hipSuccess && rc == OMPI_AMD_SUCCESS)
            rc = record_hip(r, "hipEventSynchronize (communicator streams)");
    }
    TRY(rc);
    if (has) TRY(record_hip(::wait_stream(cur), "hipStreamSynchronize (communicator stream)"));
    return OMPI_AMD_SUCCESS;
}

// Collective: every rank reaches it in the same call with the same `need`.
// Growing waits for all earlier work of every rank (no kernel may still
// touch the old buffers), then swaps descriptors of the new one.  The new
// buffer is allocated (and exported) while the old one is still alive, so it
// never reuses the old one's address range: on ROCm 7.2 an IPC export of a
// fresh allocation at a just-freed range failed with hipErrorInvalidValue
// (seen at 4 ranks, third growth).  Sizes grow geometrically, in 32 MiB steps.
// The allocation must also get handle bytes no earlier allocation had
// (export_alloc): a colliding one is kept alive while the next is made,
// so that the runtime cannot hand out the same handle again.
// uncached: fine-grained memory (flag pages) instead of ordinary device memory.
// Library allocations peers map (flag pages, staging scratch, landing
// buffers, shadow arena chunks, osc control pages and public copies) are
// recycled, not freed: release_exportable keeps them for the next request
// of the same size and kind, which gets the same address, buffer id and
// handle, so a peer still mapping it shares that mapping.  A hipFree — and
// the IPC close a peer must make before it opens a new allocation at a
// freed address — waits for every kernel of the device, and with other
// communicators' kernels waiting on peers that wait for this rank, that
// stalled a nonblocking post until the device timeout.
// Past kRecycleCap bytes kept, a release frees.
struct recycled_block {
    char *p;
    size_t size;
    bool uncached;
    int device;
};
static std::mutex g_recycle_mu;
static std::vector<recycled_block> g_recycle_free;
static std::map<char *, recycled_block> g_recycle_used;
static size_t g_recycle_free_bytes = 0;
constexpr size_t kRecycleCap = 16ull << 30;

static void release_exportable(void *ptr) {
    if (!ptr) return;
    char *p = static_cast<char *>(ptr);
    {
        std::lock_guard<std::mutex> g(g_recycle_mu);
        auto it = g_recycle_used.find(p);
        if (it != g_recycle_used.end()) {
            const recycled_block b = it->second;
            g_recycle_used.erase(it);
            if (g_recycle_free_bytes + b.size <= kRecycleCap) {
                g_recycle_free.push_back(b);
                g_recycle_free_bytes += b.size;
                return;
            }
        }
    }
    hip_ignore(hipFree(p));
}

static hipError_t alloc_exportable(size_t bytes, char **out, hipIpcMemHandle_t *h,
                                   bool uncached = false) {
    // Sized as ipc_safe_size() demands (a multiple of 2 MiB, at least 4 MiB:
    // smaller or odd-sized allocations are the ones ROCm 7.2 refuses to
    // import).  The handle names (pid, address, size): a
    // same-size allocation at a freed allocation's address gets its handle
    // again; such a repeat is kept alive (for good: freeing it would wait for
    // the device, see above) while the next attempt allocates elsewhere.
    static std::vector<void *> g_quarantine;  // under g_recycle_mu
    const size_t want_sz = ipc_size_for(bytes);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) (void)hipGetLastError();
    {
        std::lock_guard<std::mutex> g(g_recycle_mu);
        for (auto it = g_recycle_free.begin(); it != g_recycle_free.end(); ++it)
            if (it->size == want_sz && it->uncached == uncached && it->device == dev) {
                const recycled_block b = *it;
                g_recycle_free.erase(it);
                g_recycle_free_bytes -= b.size;
                g_recycle_used[b.p] = b;
                *out = b.p;
                void *base = nullptr;
                size_t range = 0;
                if (hipMemGetAddressRange((hipDeviceptr_t *)&base, &range, (hipDeviceptr_t)b.p) != hipSuccess) {
                    (void)hipGetLastError();
                    base = b.p;
                    range = b.size;
                }
                bool fresh = false;
                hipError_t e = hipSuccess;
                // exported before: the recorded handle comes back
                if (export_alloc(base, range, buffer_id(b.p), h, &e, &fresh) == 0) return hipSuccess;
                g_recycle_used.erase(b.p);  // not expected: fall through to a new allocation
                g_quarantine.push_back(b.p);
                break;
            }
    }
    std::vector<void *> failed;
    hipError_t e = hipErrorInvalidValue;
    for (int attempt = 0; attempt < 8; ++attempt) {
        void *p = nullptr;
        const size_t sz = want_sz;
        {
            host_step st("hipMalloc", sz);
            e = uncached ? hipExtMallocWithFlags(&p, sz, hipDeviceMallocUncached) : hipMalloc(&p, sz);
        }
        if (e != hipSuccess) break;
        void *base = nullptr;
        size_t range = 0;
        if (hipMemGetAddressRange((hipDeviceptr_t *)&base, &range, (hipDeviceptr_t)p) != hipSuccess) {
            (void)hipGetLastError();
            base = p;
            range = sz;
        }
        bool fresh = false;
        const int rc = export_alloc(base, range, buffer_id(p), h, &e, &fresh);
        if (rc == 0) {
            *out = (char *)p;
            std::lock_guard<std::mutex> g(g_recycle_mu);
            g_recycle_used[(char *)p] = recycled_block{(char *)p, sz, uncached, dev};
            break;
        }
        if (rc == 1) e = hipErrorInvalidValue;  // recycled handle bytes
        (void)hipGetLastError();
        failed.push_back(p);  // keep it alive so the next try gets another range and handle
    }
    if (!failed.empty()) {
        std::lock_guard<std::mutex> g(g_recycle_mu);
        g_quarantine.insert(g_quarantine.end(), failed.begin(), failed.end());
    }
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

// The landing buffers travel as full descriptors (process, handle, buffer
// id, exporter range) and are mapped through the IPC registry, which
// retires any mapping of the peer's freed allocations that the new one
// could collide with before opening it.  The token the owner stamps into
// its buffer is read back through every new mapping, as an assertion: a
// mismatch fails the growth on every rank with the peer and both tokens
// named (no retry).
constexpr size_t kLandTag = 64;  // a landing buffer's last kLandTag bytes hold its token

// the allocation a growth from `cur` usable bytes to `need` makes (32 MiB
// steps, at least doubling); every rank computes it alike
static size_t landing_want(size_t cur, size_t need) {
    constexpr size_t kStep = 32u << 20;
    return std::max((need + kLandTag + kStep - 1) / kStep * kStep,
                    cur ? std::min(2 * (cur + kLandTag), kMaxIpcBytes) : 0);
}

// a new landing buffer's descriptor (its handle is already in d->h)
static void land_desc(char *fresh, size_t want, buf_desc *d) {
    d->id = buffer_id(fresh);
    d->base = (uint64_t)(uintptr_t)fresh;
    d->size = want;
    d->pid = (uint64_t)getpid();
    d->valid = 1;
    // the registry keys on the allocation's real range (alloc_exportable pads it)
    void *ab = nullptr;
    size_t as = 0;
    if (hipMemGetAddressRange((hipDeviceptr_t *)&ab, &as, (hipDeviceptr_t)fresh) == hipSuccess) {
        d->base = (uint64_t)(uintptr_t)ab;
        d->size = as;
    } else {
        (void)hipGetLastError();
    }
}

static int ensure_landing(ompi_amd_comm_t *c, size_t need) {
    if (need <= c->land_bytes) return OMPI_AMD_SUCCESS;
    constexpr size_t kTag = kLandTag;
    const size_t want = landing_want(c->land_bytes, need);
    if (want > kMaxIpcBytes) {  // every rank decides alike (same need)
        record_msg("landing buffer of %zu bytes exceeds the %zu-byte IPC mapping limit", want,
                   kMaxIpcBytes);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    if (host_trace())
        fprintf(stderr, "[trace pid %d] blocking landing growth: need %zu, have %zu, planned %zu, %zu queued\n",
                (int)getpid(), need, c->land_bytes, c->land_planned, c->pending.size());
    TRY(quiesce(c, "quiesce (landing growth)"));
    TRY(c->boot.barrier());  // every rank's earlier kernels are done
    // the old mappings stay open until the new ones are (so the new ones
    // get fresh addresses in this process), then close
    ipc_ref *old_land[kMaxRanks];
    for (int p = 0; p < kMaxRanks; ++p) {
        old_land[p] = c->land_ref[p];
        c->land_ref[p] = nullptr;
        c->peer_land.p[p] = nullptr;
    }
    // the old mappings are kept with the communicator (their buffers stay
    // allocated until destroy: see below), not closed here — a close may
    // wait for every kernel of the device
    auto close_old = [&] {
        for (int p = 0; p < kMaxRanks; ++p)
            if (old_land[p]) c->land_ref_retired.push_back(old_land[p]);
    };
    land_blob mine{}, all[kMaxRanks];
    char *fresh = nullptr;
    hipError_t e = alloc_exportable(want, &fresh, &mine.d.h);
    mine.token = landing_token(c->rank);
    if (e == hipSuccess) land_desc(fresh, want, &mine.d);
    else record_hip(e, "landing buffer: hipMalloc / hipIpcGetMemHandle");
    // hipMemcpy from pageable memory may return once the bytes are staged,
    // before they reach the device: a peer reading through its mapping right
    // after the rendezvous below would see whatever the memory held before
    // (round 2 saw exactly that as a "token mismatch").  Wait for the copy.
    // A stream the communicator already ran on (drained above): its own
    // queue on the MPI path, else the stream of its last call (the null
    // stream before any).  Not the null stream by choice — a null-stream
    // operation also waits for every blocking stream of the process, other
    // communicators' queues on the MPI path, whose kernels may be waiting on
    // peers — and not a stream this process has not used yet: a first use
    // gives the process one more hardware queue, which on a shared GPU cost
    // the MPI path 4x in latency.
    hipStream_t ls = nullptr;
    {
        std::lock_guard<std::mutex> g(c->stream_mu);
        ls = c->own ? c->own : (c->has_stream ? c->cur_stream : nullptr);
    }
    if (e == hipSuccess)
        e = hipMemcpyAsync(fresh + want - kTag, &mine.token, sizeof(mine.token),
                           hipMemcpyHostToDevice, ls);
    if (e == hipSuccess) e = ::wait_stream(ls);
    if (e != hipSuccess && mine.d.valid) record_hip(e, "landing token write");
    mine.ok = e == hipSuccess;
    int rc = c->boot.allgather(&mine, all, sizeof(mine));  // also: nobody uses the old one now
    // freed with the communicator, not here: hipFree waits for every kernel
    // of the device, other communicators' spinning ones included
    if (c->land) c->land_retired.push_back(c->land);
    c->land = nullptr;
    c->land_bytes = c->land_planned = 0;
    if (rc != OMPI_AMD_SUCCESS) {
        close_old();
        release_exportable(fresh);
        return rc;
    }
    int status = mine.ok ? 0 : 1;  // 0 ok, 1 local HIP failure, 2 token mismatch
    for (int p = 0; p < c->size && status == 0; ++p) {
        if (p == c->rank) continue;
        if (!all[p].ok) {
            record_msg("landing buffer: rank %d failed to allocate or export its buffer", p);
            status = 1;
            break;
        }
        void *m = nullptr;
        if (ipc_map(alloc_of(all[p].d), c, &c->land_ref[p], &m) != OMPI_AMD_SUCCESS) {
            status = 1;
            break;
        }
        // the token sits `want` - kTag bytes from the allocation's start
        // (alloc_exportable's pointer is the allocation's base); read it by a kernel load through the mapping (what the
        // collectives' kernels see) into this communicator's own scratch,
        // and by hipMemcpy from the mapping, to tell the two apart
        uint64_t seen = 0, seen_memcpy = 0;
        hipLaunchKernelGGL(peek_kernel, dim3(1), dim3(1), 0, ls,
                           (const uint64_t *)((char *)m + want - kTag), (uint64_t *)c->scratch);
        e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemcpyAsync(&seen, c->scratch, sizeof(seen), hipMemcpyDeviceToHost, ls);
        if (e == hipSuccess)
            e = hipMemcpyAsync(&seen_memcpy, (char *)m + want - kTag, sizeof(seen), hipMemcpyDeviceToHost, ls);
        if (e == hipSuccess) e = ::wait_stream(ls);
        if (e == hipSuccess && seen == all[p].token && seen_memcpy != seen) {
            ++c->memcpy_token_mismatch;  // the kernel sees the right buffer; hipMemcpy does not
            record_msg("landing buffer of rank %d: kernel load sees the token, hipMemcpy through "
                       "the same mapping sees %016llx", p, (unsigned long long)seen_memcpy);
        }
        if (e != hipSuccess) {
            record_hip(e, "landing token read");
            status = 1;
        } else if (seen != all[p].token) {
            // whose token is it: another rank's new buffer, or an older one?
            int whose = -1;
            for (int q = 0; q < c->size; ++q)
                if (all[q].token == seen) whose = q;
            int old_gen = -1;
            for (size_t g = 0; g < c->land_tokens.size(); ++g)
                if (c->land_tokens[g] == seen) old_gen = (int)g;
            record_msg("landing buffer of rank %d (id %llu, %p + %llu): the IPC mapping %p shows "
                       "token %016llx, expected %016llx (it aliases another allocation: new buffer "
                       "of rank %d, earlier growth %d)", p, (unsigned long long)all[p].d.id,
                       (void *)(uintptr_t)all[p].d.base, (unsigned long long)all[p].d.size, m,
                       (unsigned long long)seen, (unsigned long long)all[p].token, whose, old_gen);
            status = 2;
        }
    }
    close_old();
    for (int q = 0; q < c->size; ++q) c->land_tokens.push_back(all[q].token);
    int st[kMaxRanks];
    rc = c->boot.allgather(&status, st, sizeof(int));
    int worst = 0;
    for (int p = 0; rc == OMPI_AMD_SUCCESS && p < c->size; ++p) worst = std::max(worst, st[p]);
    if (rc == OMPI_AMD_SUCCESS && worst == 0) {
        c->land = fresh;
        for (int p = 0; p < c->size; ++p)
            c->peer_land.p[p] = p == c->rank ? c->land : (const char *)ipc_ref_base(c->land_ref[p]);
        c->land_bytes = c->land_planned = want - kTag;
        return OMPI_AMD_SUCCESS;
    }
    (void)c->boot.barrier();  // nobody reads the new buffers any more
    for (int p = 0; p < kMaxRanks; ++p) {
        ipc_unmap(c->land_ref[p], c);
        c->land_ref[p] = nullptr;
    }
    release_exportable(fresh);
    if (rc == OMPI_AMD_SUCCESS && status == 0)
        record_msg("landing buffer growth failed on another rank (%s)",
                   worst == 2 ? "stale IPC mapping" : "HIP error");
    return rc != OMPI_AMD_SUCCESS ? rc : OMPI_AMD_ERR_HIP;
}

// ---- deferred landing growth (nonblocking calls) ----
// A nonblocking call that needs a bigger landing buffer cannot grow it at
// post time: ensure_landing is a rendezvous of the communicator, and MPI
// lets ranks post different communicators' calls in different orders — two
// growths posted in opposite orders wait for each other.
// So the post does only local work: it allocates this rank's new buffer,
// posts the descriptor and token as a ticket and queues a PEND_GROW ahead
// of the call.  Progress, once the growth is at the queue front and every
// rank's descriptor is in, maps the peers' new buffers, queues the token
// stamp and check on the call's stream (device work only: a host-side
// check would need a stream of its own, and one more stream cost a
// hardware queue) and switches the communicator over.
// Every rank switches at the same queue position, so a call launched
// before the switch uses the old buffers on every rank; those stay
// allocated and mapped until the communicator is destroyed (as a blocking
// growth keeps the buffers it replaces: hipFree and IPC closes may wait for
// every kernel of the device).  Nothing here waits for device work.

// Post a deferred call's ticket now — or, while the rendezvous ring is full
// (or earlier tickets still wait), keep the blob for progress to post in
// queue order: a full ring would otherwise hold the post until peers launch
// older calls, and they may be held in another communicator's call.
static int nb_ticket(ompi_amd_comm_t *c, pending_op &o, const void *blob, size_t len) {
    memcpy(&o.blob, blob, len);
    o.blob_len = len;
    if (c->unposted == 0 && c->boot.can_post()) return c->boot.post(blob, len, &o.ticket);
    o.unposted = true;
    ++c->unposted;
    return OMPI_AMD_SUCCESS;
}

// Post the queued tickets that fit the ring, in queue order; block_front:
// the queue's front one is posted even if that waits for a ring slot.
static int post_queued(ompi_amd_comm_t *c, bool block_front) {
    for (auto &p : c->pending) {
        if (c->unposted == 0) break;
        if (!p.unposted) continue;
        if (!(block_front && &p == &c->pending.front()) && !c->boot.can_post()) break;
        TRY(c->boot.post(&p.blob, p.blob_len, &p.ticket));
        p.unposted = false;
        --c->unposted;
    }
    return OMPI_AMD_SUCCESS;
}

// Queue a growth to `need` usable bytes unless the queued ones reach it,
// ahead of a call on stream `s`.
// Every rank decides alike: the same calls are posted on every rank.  Only
// local work here — no stream is touched (a stream created for it alone
// costs a hardware queue: on a shared GPU that took 8-B sendrecvs from 31
// to 96 µs at 2 ranks, tools/p2p_osc_rows.py ROWS_PRE=iar_big).
static int nb_grow(ompi_amd_comm_t *c, size_t need, hipStream_t s) {
    if (need <= c->land_planned) return OMPI_AMD_SUCCESS;
    const size_t want = landing_want(c->land_planned, need);
    if (want > kMaxIpcBytes) {
        record_msg("landing buffer of %zu bytes exceeds the %zu-byte IPC mapping limit", want,
                   kMaxIpcBytes);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    land_blob mine{};
    char *fresh = nullptr;
    const hipError_t e = alloc_exportable(want, &fresh, &mine.d.h);
    mine.token = landing_token(c->rank);
    if (e == hipSuccess) land_desc(fresh, want, &mine.d);
    else record_hip(e, "landing buffer (deferred growth): hipMalloc / hipIpcGetMemHandle");
    mine.ok = e == hipSuccess;  // a failure is posted too: every rank fails the growth alike
    pending_op g{};
    g.kind = PEND_GROW;
    g.stream = s;
    g.grow = fresh;
    g.grow_bytes = want;
    g.grow_token = mine.token;
    const int rc = nb_ticket(c, g, &mine, sizeof(mine));
    if (rc != OMPI_AMD_SUCCESS) {
        release_exportable(fresh);
        return rc;
    }
    c->pending.push_back(g);
    c->npending.fetch_add(1);
    c->land_planned = want - kLandTag;
    return OMPI_AMD_SUCCESS;
}

// A queued growth at the front of the queue with every rank's descriptor
// (`all`): map the peers' new buffers, queue the token stamp / barrier /
// check on the growth's stream, switch.  On failure nothing after it
// launches (land_failed): those calls were sized for the new buffers.
static int launch_barrier(ompi_amd_comm_t *c, hipStream_t s);

static int grow_launch(ompi_amd_comm_t *c, const pending_op &g, const land_blob *all) {
    const size_t want = g.grow_bytes;
    ipc_ref *refs[kMaxRanks] = {};
    void *maps[kMaxRanks] = {};
    int status = all[c->rank].ok ? 0 : 1;
    for (int p = 0; p < c->size && status == 0; ++p) {
        if (p == c->rank) continue;
        if (!all[p].ok) {
            record_msg("landing buffer: rank %d failed to allocate or export its buffer", p);
            status = 1;
        } else if (ipc_map(alloc_of(all[p].d), c, &refs[p], &maps[p]) != OMPI_AMD_SUCCESS) {
            status = 1;
        }
    }
    if (status == 0) {
        tok_ptrs peers{};
        tok_set expect{};
        for (int p = 0; p < c->size; ++p) {
            expect.t[p] = all[p].token;
            if (p != c->rank) peers.p[p] = (const uint64_t *)((char *)maps[p] + want - kLandTag);
        }
        note_stream(c, g.stream);
        hipLaunchKernelGGL(land_stamp_kernel, dim3(1), dim3(1), 0, g.stream,
                           (uint64_t *)(g.grow + want - kLandTag), g.grow_token);
        int rc = record_hip(hipGetLastError(), "landing stamp launch (deferred growth)");
        if (rc == OMPI_AMD_SUCCESS) rc = launch_barrier(c, g.stream);
        if (rc == OMPI_AMD_SUCCESS) {
            hipLaunchKernelGGL(land_check_kernel, dim3(1), dim3(64), 0, g.stream, peers, expect, c->rank,
                               c->size, c->err_dev, c->flags + kAbortWord);
            rc = record_hip(hipGetLastError(), "landing check launch (deferred growth)");
        }
        if (rc != OMPI_AMD_SUCCESS) status = 1;
    }
    for (int q = 0; q < c->size; ++q) c->land_tokens.push_back(all[q].token);
    if (status != 0) {
        for (int p = 0; p < kMaxRanks; ++p) ipc_unmap(refs[p], c);
        if (g.grow) c->land_retired.push_back(g.grow);  // peers may have mapped it
        c->land_failed = true;
        return OMPI_AMD_ERR_HIP;
    }
    if (c->land) c->land_retired.push_back(c->land);
    for (int p = 0; p < kMaxRanks; ++p) {
        if (c->land_ref[p]) c->land_ref_retired.push_back(c->land_ref[p]);
        c->land_ref[p] = refs[p];
    }
    c->land = g.grow;
    for (int p = 0; p < c->size; ++p)
        c->peer_land.p[p] = p == c->rank ? c->land : (const char *)ipc_ref_base(c->land_ref[p]);
    c->land_bytes = want - kLandTag;
    ++c->deferred_growths;
    return OMPI_AMD_SUCCESS;
}

static int launch_barrier(ompi_amd_comm_t *c, hipStream_t s) {
    note_stream(c, s);
    ++c->epoch;
    const uint64_t ticks = (uint64_t)c->timeout_ms * 100000ull;  // s_memrealtime: 100 MHz
    hipLaunchKernelGGL(barrier_kernel, dim3(1), dim3(64), 0, s, c->flags, c->peer_flags, c->rank,
                       c->size, c->epoch, c->err_dev, ticks, c->dbg_dev);
    return record_hip(hipGetLastError(), "barrier launch");
}

static int launch_copy(ompi_amd_comm_t *c, const cp_jobs &jobs, hipStream_t s) {
    if (jobs.n == 0) return OMPI_AMD_SUCCESS;
    note_stream(c, s);
    int64_t most = 0;
    for (int i = 0; i < jobs.n; ++i) most = std::max(most, jobs.j[i].bytes);
    int64_t blocks = (most / 16 + kXferThreads * 4 - 1) / (kXferThreads * 4);
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, std::max(1, c->max_blocks / jobs.n)));
    if (c->copy_nt)
        hipLaunchKernelGGL(copy_kernel<true>, dim3((unsigned)blocks, (unsigned)jobs.n),
                           dim3(kXferThreads), 0, s, jobs);
    else
        hipLaunchKernelGGL(copy_kernel<false>, dim3((unsigned)blocks, (unsigned)jobs.n),
                           dim3(kXferThreads), 0, s, jobs);
    return record_hip(hipGetLastError(), "copy launch");
}

// ---- shadow arena ----

// First fit over the chunks (256-B granules, never across a chunk: peers map
// each chunk separately); a new chunk of max(need, min_chunk, everything so
// far) when none fits (64 MiB for collective shadows; windows ask for 2 MiB:
// the osc component gives every window a communicator of its own).
static int arena_alloc(ompi_amd_comm_t *c, size_t need, char **out,
                       size_t min_chunk = (size_t)64 << 20) {
    host_step st("arena_alloc", need);
    const size_t n = (std::max<size_t>(need, 1) + 255) & ~(size_t)255;
    std::lock_guard<std::mutex> g(c->arena_mu);
    for (auto &ch : c->arena) {
        for (auto it = ch.free.begin(); it != ch.free.end(); ++it) {
            if (it->second < n) continue;
            const size_t off = it->first, left = it->second - n;
            ch.free.erase(it);
            if (left) ch.free[off + n] = left;
            ch.used[off] = n;
            *out = ch.base + off;
            return OMPI_AMD_SUCCESS;
        }
    }
    if (n > kMaxIpcBytes) {
        record_msg("shadow of %zu bytes exceeds the %zu-byte IPC allocation limit", n, kMaxIpcBytes);
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    const size_t want = std::min(kMaxIpcBytes,
                                 (std::max({n, min_chunk, c->arena_bytes}) + (2u << 20) - 1) &
                                     ~(size_t)((2u << 20) - 1));
    char *mem = nullptr;
    hipIpcMemHandle_t h;
    const hipError_t e = alloc_exportable(want, &mem, &h);
    if (e != hipSuccess) return record_hip(e, "shadow arena: hipMalloc / hipIpcGetMemHandle");
    c->arena.push_back({mem, want, {}, {}});
    auto &ch = c->arena.back();
    if (want > n) ch.free[n] = want - n;
    ch.used[0] = n;
    c->arena_bytes += want;
    *out = mem;
    return OMPI_AMD_SUCCESS;
}

// The caller guarantees no peer still reads the range (the call that used it
// passed its trailing barrier on this rank's stream).
static void arena_free(ompi_amd_comm_t *c, char *p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(c->arena_mu);
    for (auto &ch : c->arena) {
        if (p < ch.base || p >= ch.base + ch.size) continue;
        const size_t off = (size_t)(p - ch.base);
        auto u = ch.used.find(off);
        if (u == ch.used.end()) return;
        size_t lo = off, len = u->second;
        ch.used.erase(u);
        auto nx = ch.free.lower_bound(off);
        if (nx != ch.free.end() && nx->first == off + len) {  // merge the next free range
            len += nx->second;
            nx = ch.free.erase(nx);
        }
        if (nx != ch.free.begin()) {  // and the previous one
            auto pv = std::prev(nx);
            if (pv->first + pv->second == lo) {
                lo = pv->first;
                len += pv->second;
                ch.free.erase(pv);
            }
        }
        ch.free[lo] = len;
        return;
    }
}

// ---- export fallback (shadow_set) ----
// k: the communicator's shadow k (0, and 1 for a result region that does
// not fit beside the input in one IPC allocation).
static int shadow_reserve(ompi_amd_comm_t *c, size_t need, char **out, int k = 0) {
    char *&sh = k ? c->shadow2 : c->shadow;
    size_t &bytes = k ? c->shadow2_bytes : c->shadow_bytes;
    if (need <= bytes) {
        *out = sh;
        return OMPI_AMD_SUCCESS;
    }
    // the old shadow's last readers are the peers of an earlier call, done
    // once this rank's stream passed that call's trailing barrier
    TRY(quiesce(c, "quiesce (shadow growth)"));
    arena_free(c, sh);
    const size_t want = std::max(need, std::min(2 * bytes, kMaxIpcBytes));
    sh = nullptr;
    bytes = 0;
    TRY(arena_alloc(c, want, &sh));
    bytes = want;
    *out = sh;
    return OMPI_AMD_SUCCESS;
}

// Decide the shadows of one zero-copy call and substitute the pointers:
// *src (sbytes read by peers) and *rbuf (rbytes read or written by peers;
// rbuf_in: its content is an input).  src == rbuf is in place (one region).
// owned: fresh memory for this call (post->mem) instead of the
// communicator's.  Nothing is enqueued here (shadow_in / shadow_out).
static int shadow_plan(ompi_amd_comm_t *c, const void **src, size_t sbytes, void **rbuf,
                       size_t rbytes, bool rbuf_in, bool owned, shadow_set *post,
                       bool split_inplace = false) {
    *post = shadow_set{};
    bool inplace = *src && *src == (const void *)*rbuf;
    bool fs = false, fr = false;
    buf_desc d;
    if (*src && sbytes) {
        if (c->force_shadow || !c->user_ipc) {
            fs = true;
        } else {
            const int rc = export_buf(c, *src, &d, &fs);
            if (rc != OMPI_AMD_SUCCESS && !fs) return rc;
        }
    }
    if (inplace && fs && split_inplace) {
        // two shadows: the input (copied in) and the result (copied out)
        inplace = false;
        fr = true;
        rbuf_in = false;
    } else if (inplace) {
        fr = fs;
        fs = false;
        rbytes = std::max(rbytes, sbytes);
        rbuf_in = true;
    } else if (*rbuf && rbytes) {
        if (c->force_shadow || !c->user_ipc) {
            fr = true;
        } else {
            const int rc = export_buf(c, *rbuf, &d, &fr);
            if (rc != OMPI_AMD_SUCCESS && !fr) return rc;
        }
    }
    if (!fs && !fr) return OMPI_AMD_SUCCESS;
    // each region keeps its user pointer's phase mod 256 (the kernels'
    // vector paths need the sources' and destinations' 16-B phases to agree)
    const size_t so = fs ? ((uintptr_t)*src & 255) : 0;
    const size_t rbase = fs ? ((so + sbytes + 255) & ~(size_t)255) : 0;
    const size_t ro = fr ? rbase + ((uintptr_t)*rbuf & 255) : rbase;
    size_t need = (fr ? ro + rbytes : so + sbytes) + 256;
    // input and result in separate allocations when together they pass the
    // IPC size limit (the result region then starts at offset 0 of its own)
    const bool split2 = fs && fr && need > kMaxIpcBytes;
    if (split2) need = so + sbytes + 256;
    char *mem = nullptr, *mem2 = nullptr;
    if (owned) {
        TRY(arena_alloc(c, need, &mem));
        post->mem = mem;
        if (split2) {
            TRY(arena_alloc(c, ((uintptr_t)*rbuf & 255) + rbytes + 256, &mem2));
            post->mem2 = mem2;
        }
    } else {
        TRY(shadow_reserve(c, need, &mem));
        if (split2) TRY(shadow_reserve(c, ((uintptr_t)*rbuf & 255) + rbytes + 256, &mem2, 1));
    }
    if (fs) {
        post->in.j[post->in.n++] = {(const char *)*src, mem + so, (int64_t)sbytes};
        *src = mem + so;
    }
    if (fr) {
        char *r = split2 ? mem2 + ((uintptr_t)*rbuf & 255) : mem + ro;
        if (rbuf_in) post->in.j[post->in.n++] = {(const char *)*rbuf, r, (int64_t)rbytes};
        post->out = {r, (char *)*rbuf, (int64_t)rbytes};
        *rbuf = r;
        if (inplace) *src = r;
    }
    ++c->shadowed;
    return OMPI_AMD_SUCCESS;
}

static int shadow_in(ompi_amd_comm_t *c, const shadow_set &sh, hipStream_t s) {
    return launch_copy(c, sh.in, s);
}

static int shadow_out(ompi_amd_comm_t *c, const shadow_set &sh, hipStream_t s) {
    if (sh.out.bytes <= 0) return OMPI_AMD_SUCCESS;
    cp_jobs cj{};
    cj.j[0] = sh.out;
    cj.n = 1;
    return launch_copy(c, cj, s);
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
    red_launch_fn f = red_fn(op, type);
    if (!f) return OMPI_AMD_ERR_UNSUPPORTED;
    if (jobs.n == 0 || nsrc < 1) return OMPI_AMD_SUCCESS;
    note_stream(c, s);
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
                        flags | (c->copy_nt ? FOLD_NT_STORE : 0), jobs, s),
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
    if (a) hip_ignore(hipEventRecord(a, s));
    const int rc = launch();
    if (b) hip_ignore(hipEventRecord(b, s));
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

// The operand order of one allreduce: the algorithm coll/tuned runs for
// these arguments — its fixed decision (coll_tuned_decision_fixed.c:45-89)
// or the one the user forced with coll_tuned_use_dynamic_rules +
// coll_tuned_allreduce_algorithm (coll_tuned_allreduce_decision.c:37-147),
// with each algorithm's own fallbacks.  Every path below folds every
// element in this order, whichever rank computes it.
static int pof2_floor(int n) {
    int a = 1;
    while (a * 2 <= n) a *= 2;
    return a;
}

static fold_plan allreduce_fold(int n, int tuned_alg, size_t count, int type, bool root0_inplace,
                                int red_alg = 0) {
    const size_t msg = type_size(type) * count;
    const fold_plan tree{ORDER_TREE, 0, 0}, ring{ORDER_RING, 0, 0};
    // basic_linear: basic linear reduce to 0 (acc = x[n-1]; acc = f(acc, x[i]),
    // i = n-2 .. 0, coll_base_reduce.c:680-721) + bcast (:881-912)
    const fold_plan linear{ORDER_CHAIN, 0, 0};
    switch (tuned_alg) {
    case TUNED_AR_BASIC_LINEAR: return linear;
    case TUNED_AR_NONOVERLAPPING: {  // tuned reduce to 0 + bcast (:54-86)
        const red_order ro = tuned_reduce_order(n, msg, count, 0, root0_inplace, red_alg);
        return {ro.order, ro.first, ro.flags};
    }
    case TUNED_AR_RECURSIVE_DOUBLING: return tree;
    case TUNED_AR_RING:               // count < size: recursive doubling (:371-377)
    case TUNED_AR_RING_SEGMENTED:     // too few segments: ring (:652-656), then as ring
        return count < (size_t)n ? tree : ring;
    case TUNED_AR_RABENSEIFNER:       // count < p': basic linear (:988-995)
        return count < (size_t)pof2_floor(n) ? linear : fold_plan{ORDER_RABEN, 0, 0};
    default:                          // the fixed decision: < 10000 B recursive doubling
        return (msg < 10000 || count < (size_t)n) ? tree : ring;
    }
}

// Rabenseifner: the piece of the vector vrank o ends up owning — the
// recursive vector halving of :1122-1171 (the lower vrank of a pair keeps
// the left floor(w/2) elements of the window).
static void raben_piece(int64_t count, int n, int o, int64_t *lo, int64_t *cnt) {
    int64_t l = 0, w = count;
    for (int m = 1; m < pof2_floor(n); m <<= 1) {
        const int64_t half = w / 2;
        if (o & m) { l += half; w -= half; }
        else w = half;
    }
    *lo = l;
    *cnt = w;
}

// Jobs folding the elements of ring block `block` (every element: -1)
// in plan p's order.
static void fold_jobs(const fold_plan &p, int64_t count, int n, int block, red_jobs *jobs) {
    if (p.order == ORDER_RING) {
        ring_jobs(count, n, jobs, block);
        return;
    }
    int64_t lo = 0, hi = count;
    if (block >= 0) {
        int64_t split, early, late;
        blockcount(count, n, &split, &early, &late);
        lo = block_off(block, split, early, late);
        hi = lo + block_cnt(block, split, early, late);
    }
    jobs->n = 0;
    if (p.order != ORDER_RABEN) {
        red_job &j = jobs->j[jobs->n++];
        j = red_job{lo, hi - lo, lo, p.first, -1};
        return;
    }
    const int adj = pof2_floor(n);
    for (int o = 0; o < adj; ++o) {  // one job per piece the range meets
        int64_t plo, pcnt;
        raben_piece(count, n, o, &plo, &pcnt);
        const int64_t a = std::max(lo, plo), b = std::min(hi, plo + pcnt);
        if (a >= b) continue;
        red_job &j = jobs->j[jobs->n++];
        j = red_job{a, b - a, a, 0, -1};
        j.aux = o << 8;
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
    fused_launch_fn f = fused_fn(op, type);
    if (!f) return OMPI_AMD_ERR_UNSUPPORTED;
    note_stream(c, s);
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
    if (c->want_mark && c->mark_word) {  // the call's completion, by the kernel itself
        a.done = reinterpret_cast<uint32_t *>(c->flags) + kFusedDoneWord + kFusedDoneStride * c->mark_slot;
        a.mark = c->mark_word;
        a.mark_v = mark_reserve();
    }
    TRY(record_hip(f(dim3((unsigned)cols, (unsigned)rows), a, s), "fused allreduce launch"));
    if (a.mark) c->mark_embedded = a.mark_v;
    return OMPI_AMD_SUCCESS;
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
                                     int64_t count, int op, int type, const fold_plan &fp,
                                     hipStream_t s) {
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
    fold_jobs(fp, count, n, mine, &jobs);
    TRY(launch_reduce(c, op, type, sh.peers, n, dst, 2, fp.order, fp.flags, jobs, s));
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
                          int64_t count, int op, int type, const fold_plan &fp, hipStream_t s) {
    const int n = c->size, mine = (c->rank + 1) % n;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    TRY(launch_barrier(c, s));
    red_jobs jobs;
    fold_jobs(fp, count, n, mine, &jobs);
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, sp, n, one_ptr(rbuf), 1, fp.order, fp.flags, jobs, s);
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

// The pull scheme staged through this rank's shadow `sh` (user_ipc off):
// peers read only shadows.  The caller copied the input into `sh` and
// swapped shadows (sp[r] = rank r's).  The owner of block b folds it from
// every shadow and stores the result into its rbuf AND into block b of its
// own shadow (nobody else reads that block of it during the fold), so the
// gather phase pulls results from the shadows: one local copy of the input
// is the whole price of staging (no result shadow, no copy out).
static int allreduce_pull_staged(ompi_amd_comm_t *c, const ptr_set &sp, char *sh, void *rbuf,
                                 int64_t count, int op, int type, const fold_plan &fp,
                                 hipStream_t s) {
    const int n = c->size, mine = (c->rank + 1) % n;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    TRY(launch_barrier(c, s));
    red_jobs jobs;
    fold_jobs(fp, count, n, mine, &jobs);
    ptr_set dsts{};
    dsts.p[0] = (const char *)rbuf;
    dsts.p[1] = sh;
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, sp, n, dsts, 2, fp.order, fp.flags, jobs, s);
    }));
    TRY(launch_barrier(c, s));
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    cp_jobs cj{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * ext;
        cj.j[cj.n++] = {sp.p[owner] + off, (char *)rbuf + off, block_cnt(b, split, early, late) * ext};
    }
    TRY(timed_phase(c, 1, s, [&] { return launch_copy(c, cj, s); }));
    return launch_barrier(c, s);
}

static int allreduce_pull_push(ompi_amd_comm_t *c, const ptr_set &sp, const ptr_set &rp,
                               int64_t count, int op, int type, const fold_plan &fp,
                               hipStream_t s) {
    // in place, sp = rp: only the owner of a block touches it
    const int n = c->size, mine = (c->rank + 1) % n;
    TRY(launch_barrier(c, s));
    red_jobs jobs;
    fold_jobs(fp, count, n, mine, &jobs);
    const ptr_set dsts = push_order(c, rp);
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, sp, n, dsts, n, fp.order, fp.flags, jobs, s);
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
                          int op, int type, const fold_plan &fp, hipStream_t s) {
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
    TRY(timed_phase(c, 2, s, [&] { return launch_copy(c, cj, s); }));
    TRY(launch_barrier(c, s));
    const int64_t offm = block_off(mine, split, early, late) * ext;
    ptr_set srcs{};
    for (int r = 0; r < n; ++r)
        srcs.p[r] = (r == c->rank) ? (const char *)src
                                   : c->land + (size_t)r * slot + (offm & 15) - offm;
    red_jobs jobs;
    fold_jobs(fp, count, n, mine, &jobs);
    const ptr_set dsts = push_order(c, rp);
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, srcs, n, dsts, n, fp.order, fp.flags, jobs, s);
    }));
    return launch_barrier(c, s);
}

// ---- pipelined staged schemes (pipe_allreduce_kernel): one launch whose
// per-slice flags replace the barriers between send, fold and gather, then
// the trailing barrier every landing / shadow call ends with.  The phases'
// buffers: dst_c[b] where my block b goes (null: my own block), src_f[r]
// rank r's share of my block, dst_f the fold's results, src_g[b] where
// block b's result is gathered from.  Element e sits at ptr + e * ext.
static int launch_pipe(ompi_amd_comm_t *c, int op, int type, const void *src, void *rbuf,
                       int64_t count, const fold_plan &fp, const ptr_set &dst_c,
                       const ptr_set &src_f, const ptr_set &dst_f, int ndst,
                       const ptr_set &src_g, hipStream_t s) {
    pipe_launch_fn f = pipe_fn(op, type);
    if (!f) return OMPI_AMD_ERR_UNSUPPORTED;
    note_stream(c, s);
    const int n = c->size;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    pipe_args a{};
    a.src = (const char *)src;
    a.rbuf = (char *)rbuf;
    a.dst_c = dst_c;
    a.src_f = src_f;
    a.dst_f = dst_f;
    a.ndst = ndst;
    a.src_g = src_g;
    a.flags = c->flags + kPipeFlagOff / sizeof(uint64_t);
    for (int p = 0; p < n; ++p) a.peer_flags.p[p] = c->peer_flags.p[p] + kPipeFlagOff / sizeof(uint64_t);
    a.rank = c->rank;
    a.n = n;
    a.mine = (c->rank + 1) % n;
    a.order = fp.order;
    a.first = fp.order == ORDER_RING ? a.mine : fp.first;
    a.fold_flags = fp.flags;
    a.nt = c->copy_nt ? 1 : 0;
    a.colocated = c->colocated;
    blockcount(count, n, &a.split, &a.early, &a.late);
    // slices: whole 16-B vectors, pipe_passes per workgroup of the grid,
    // none under pipe_slice bytes.  Each pass costs the workgroup one
    // system-scope release and acquire (L2 write-back / invalidate): on one
    // shared GPU, 16 KiB slices (32 passes) ran 2.7x the phased scheme,
    // >= 1 MiB slices (one pass) 0.89x it for the staged pull at N = 2,
    // 256 MiB (profiles/r04_pipe_slices_n2.jsonl)
    const int64_t E = std::max<int64_t>(1, 16 / ext);
    const int64_t groups_max = std::max(1, std::min(c->max_blocks, kPipeMaxGroups));
    const int64_t want = groups_max * std::max(1, c->pipe_passes);
    int64_t per = ((a.early + want - 1) / want + E - 1) / E * E;
    per = std::max<int64_t>(per, std::max<int64_t>(E, (c->pipe_slice / ext + E - 1) / E * E));
    a.per = per;
    a.nslices = std::max<int64_t>(1, (a.early + per - 1) / per);
    const int64_t groups = std::min(groups_max, a.nslices);
    a.seq = (++c->pipe_seq) << 20;
    a.timeout_ticks = (uint64_t)c->timeout_ms * 100000ull;  // s_memrealtime: 100 MHz
    a.err = c->err_dev;
    a.abort_word = c->flags + kAbortWord;
    return record_hip(f((unsigned)groups, a, s), "pipelined allreduce launch");
}

// Whether the pipelined kernel runs this call: one job per block
// (Rabenseifner's pieces carry per-piece owners) and at most 8 ranks (one
// node's GPUs; the kernel is built for 8 sources): else the phased schemes.
static bool pipe_fits(const ompi_amd_comm_t *c, const fold_plan &fp) {
    return fp.order != ORDER_RABEN && c->size <= 8;
}

// Push-gather / push-land pipelined: C stores my block b into slot [me] of
// its owner's landing buffer, F folds my block from my input and my landing
// slots into rbuf and the result slot [n] (push-land: into slot [n + mine]
// of every peer's landing buffer instead), G gathers the other blocks from
// the owners' result slots (push-land: from my own result slots).
static int allreduce_push_pipe(ompi_amd_comm_t *c, const void *src, void *rbuf, int64_t count,
                               int op, int type, const fold_plan &fp, hipStream_t s, bool land) {
    const int n = c->size, mine = (c->rank + 1) % n;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    const size_t slot = push_slot(count, n, type);
    ptr_set dst_c{}, src_f{}, dst_f{}, src_g{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * ext;
        dst_c.p[b] = c->peer_land.p[owner] + (size_t)c->rank * slot + (off & 15) - off;
        src_g.p[b] = land ? c->land + (size_t)(n + b) * slot + (off & 15) - off
                          : c->peer_land.p[owner] + (size_t)n * slot + (off & 15) - off;
    }
    const int64_t offm = block_off(mine, split, early, late) * ext;
    for (int r = 0; r < n; ++r)
        src_f.p[r] = r == c->rank ? (const char *)src : c->land + (size_t)r * slot + (offm & 15) - offm;
    dst_f.p[0] = (const char *)rbuf;
    int ndst = 2;
    if (land) {
        for (int k = 1; k < n; ++k) {
            const int q = (c->rank + k) % n;
            dst_f.p[k] = c->peer_land.p[q] + (size_t)(n + mine) * slot + (offm & 15) - offm;
        }
        ndst = n;
    } else {
        dst_f.p[1] = c->land + (size_t)n * slot + (offm & 15) - offm;
    }
    // the previous landing call's trailing barrier ended every reader of
    // these slots: no leading barrier
    TRY(timed_phase(c, 0, s, [&] {
        return launch_pipe(c, op, type, src, rbuf, count, fp, dst_c, src_f, dst_f, ndst, src_g, s);
    }));
    return launch_barrier(c, s);
}

// Staged pull pipelined: C copies my blocks other than my own into my
// shadow `sh` (peers' shadows in sp after the swap), F folds my block from
// my input and the peers' shadows into rbuf and my shadow, G gathers the
// other blocks from their owners' shadows.  The staging copy of slice k
// runs while slices < k are folded and gathered.
static int allreduce_pull_pipe(ompi_amd_comm_t *c, const ptr_set &sp, char *sh, const void *src,
                               void *rbuf, int64_t count, int op, int type, const fold_plan &fp,
                               hipStream_t s) {
    const int n = c->size, mine = (c->rank + 1) % n;
    ptr_set dst_c{}, src_f{}, dst_f{}, src_g{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        dst_c.p[b] = sh;
        src_g.p[b] = sp.p[(b + n - 1) % n];
    }
    for (int r = 0; r < n; ++r) src_f.p[r] = r == c->rank ? (const char *)src : sp.p[r];
    dst_f.p[0] = (const char *)rbuf;
    dst_f.p[1] = sh;
    TRY(timed_phase(c, 0, s, [&] {
        return launch_pipe(c, op, type, src, rbuf, count, fp, dst_c, src_f, dst_f, 2, src_g, s);
    }));
    return launch_barrier(c, s);
}

// Landing bytes of the staged push schemes: push-gather needs n input slots
// and its result slot [n]; push-land n input slots and n result slots (one
// per block).  Push-land falls back to push-gather when its 2n slots would
// pass the IPC size limit (every rank computes the same for the same count).
static size_t staged_push_landing(int n, int algorithm, int64_t count, int type, bool *land) {
    const size_t slot = push_slot(count, n, type);
    const bool l = is_land(algorithm) && slot * (size_t)(2 * n) <= kMaxIpcBytes;
    if (land) *land = l;
    return slot * (size_t)(l ? 2 * n : n + 1);
}

// The push scheme with a gather instead of remote result stores: nothing
// of the caller's is exported (the default, user_ipc = 0).  Scatter: block b
// of my input into slot [me] of its owner's landing buffer (remote stores,
// library memory).  Barrier.  The owner folds its block from its own input
// and its landing slots (local reads) into its rbuf and into its landing
// result slot [n].  Barrier.  Every rank pulls the other blocks from their
// owners' result slots into its rbuf.  Barrier.  Same xGMI bytes as the
// zero-copy pull ((N-1)/N·S out, (N-1)/N·S in), no staging copy.
//
// Push-land (algorithm 3): the same scatter and barrier; then the owner
// folds its block into its rbuf AND stores the result into slot [n + b] of
// every peer's landing buffer in the same pass (remote stores, spread over
// the links: local first, then rank+1, rank+2, ...).  Barrier.  Every rank
// copies the other blocks from its own result slots into its rbuf (local
// HBM).  Barrier (every landing call ends with one: the next landing call of
// any collective may scatter into these bytes without a leading barrier).
// Both xGMI phases store; the price is one local copy of (N-1)/N of the
// vector.
static int allreduce_push_gather(ompi_amd_comm_t *c, const void *src, void *rbuf, int64_t count,
                                 int op, int type, const fold_plan &fp, hipStream_t s,
                                 int algorithm) {
    const int n = c->size, mine = (c->rank + 1) % n;
    const int64_t ext = (int64_t)ompi_amd_type_extent(type);
    int64_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    const size_t slot = push_slot(count, n, type);
    bool land = false;
    TRY(ensure_landing(c, staged_push_landing(n, algorithm, count, type, &land)));
    if (is_pipe(algorithm) && pipe_fits(c, fp))
        return allreduce_push_pipe(c, src, rbuf, count, op, type, fp, s, land);
    cp_jobs cj{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * ext;
        char *dst = const_cast<char *>(c->peer_land.p[owner]) + (size_t)c->rank * slot + (off & 15);
        cj.j[cj.n++] = {(const char *)src + off, dst, block_cnt(b, split, early, late) * ext};
    }
    // the owner's reads of its slots and the peers' reads of its result slot
    // from the previous landing call ended before that call's trailing
    // barrier, so the scatter needs no leading one
    TRY(timed_phase(c, 2, s, [&] { return launch_copy(c, cj, s); }));
    TRY(launch_barrier(c, s));
    const int64_t offm = block_off(mine, split, early, late) * ext;
    ptr_set srcs{};
    for (int r = 0; r < n; ++r)
        srcs.p[r] = (r == c->rank) ? (const char *)src
                                   : c->land + (size_t)r * slot + (offm & 15) - offm;
    red_jobs jobs;
    fold_jobs(fp, count, n, mine, &jobs);
    ptr_set dsts{};
    dsts.p[0] = (const char *)rbuf;
    if (land) {
        for (int k = 1; k < n; ++k) {
            const int q = (c->rank + k) % n;
            dsts.p[k] = c->peer_land.p[q] + (size_t)(n + mine) * slot + (offm & 15) - offm;
        }
        TRY(timed_phase(c, 0, s, [&] {
            return launch_reduce(c, op, type, srcs, n, dsts, n, fp.order, fp.flags, jobs, s);
        }));
        TRY(launch_barrier(c, s));
        cj = cp_jobs{};
        for (int b = 0; b < n; ++b) {
            if (b == mine) continue;
            const int64_t off = block_off(b, split, early, late) * ext;
            cj.j[cj.n++] = {c->land + (size_t)(n + b) * slot + (off & 15), (char *)rbuf + off,
                            block_cnt(b, split, early, late) * ext};
        }
        TRY(timed_phase(c, 1, s, [&] { return launch_copy(c, cj, s); }));
        return launch_barrier(c, s);
    }
    dsts.p[1] = c->land + (size_t)n * slot + (offm & 15) - offm;
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, srcs, n, dsts, 2, fp.order, fp.flags, jobs, s);
    }));
    TRY(launch_barrier(c, s));
    cj = cp_jobs{};
    for (int b = 0; b < n; ++b) {
        if (b == mine) continue;
        const int owner = (b + n - 1) % n;
        const int64_t off = block_off(b, split, early, late) * ext;
        const char *res = c->peer_land.p[owner] + (size_t)n * slot + (off & 15);
        cj.j[cj.n++] = {res, (char *)rbuf + off, block_cnt(b, split, early, late) * ext};
    }
    TRY(timed_phase(c, 1, s, [&] { return launch_copy(c, cj, s); }));
    return launch_barrier(c, s);
}

// reduce_scatter_block / reduce_scatter: my block [off, off + cnt) of the
// full vector folded from every rank's input into rbuf[0, cnt).
// Staged: inputs in the scratch halves.  Zero-copy: peers' inputs read in
// place; a rank that passed MPI_IN_PLACE must not overwrite its rbuf (a
// peer may still read its own block there), so every rank learns the
// in-place flags with the handle swap and in-place ranks fold into their
// landing buffer and copy after the trailing barrier.
// rcounts: every rank's block length (reduce_scatter), or null for equal
// blocks of cnt (reduce_scatter_block).
static int reduce_my_block(ompi_amd_comm_t *c, const void *src, void *rbuf, size_t total_bytes,
                           int64_t off, int64_t cnt, int64_t max_cnt, int op, int type,
                           red_order ro, bool inplace, hipStream_t s,
                           const size_t *rcounts = nullptr) {
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
    if (!c->pre && !c->user_ipc && !c->force_shadow) {
        // Staged push (nothing of the caller's exported, no staging copy):
        // block b of my input into slot [me] of rank b's landing buffer
        // (at its own phase mod 16), barrier, fold my block from my input
        // and my landing slots, barrier (peers then may reuse the slots).
        // In place, the result goes through landing slot [n] (it may
        // overlap my own block of the input, reduce_scatter's uneven counts).
        const size_t slot = ((size_t)max_cnt * ext + 16 + 255) & ~(size_t)255;
        TRY(ensure_landing(c, slot * (size_t)(n + 1)));
        cp_jobs cj{};
        int64_t ob = 0;
        for (int b = 0; b < n; ++b) {
            const int64_t cb = rcounts ? (int64_t)rcounts[b] : cnt;
            if (b != c->rank && cb > 0) {
                const int64_t bytes_off = ob * (int64_t)ext;
                char *dst = const_cast<char *>(c->peer_land.p[b]) + (size_t)c->rank * slot + (bytes_off & 15);
                cj.j[cj.n++] = {(const char *)src + bytes_off, dst, cb * (int64_t)ext};
            }
            ob += cb;
        }
        // the previous landing call's trailing barrier ended every reader of
        // these slots: no leading barrier
        TRY(launch_copy(c, cj, s));
        TRY(launch_barrier(c, s));
        const int64_t offb = off * (int64_t)ext;
        ptr_set srcs{};
        for (int r = 0; r < n; ++r)
            srcs.p[r] = (r == c->rank) ? (const char *)src
                                       : c->land + (size_t)r * slot + (offb & 15) - offb;
        char *res = inplace ? c->land + (size_t)n * slot + (offb & 15) : (char *)rbuf;
        jobs.j[0].off_dst = 0;
        if (cnt > 0)
            TRY(launch_reduce(c, op, type, srcs, n, one_ptr(res), 1, ro.order, ro.flags, jobs, s));
        if (inplace && cnt > 0) {
            cj = cp_jobs{};
            cj.n = 1;
            cj.j[0] = {res, (char *)rbuf, cnt * (int64_t)ext};
            TRY(launch_copy(c, cj, s));
        }
        return launch_barrier(c, s);
    }
    ptr_set sp{}, rp{};
    uint64_t fl[kMaxRanks] = {};
    void *none = nullptr;
    shadow_set sh;  // peers only read src; this rank's result stays local
    if (!c->pre)    // a deferred call posted its (shadow) descriptor already
        TRY(shadow_plan(c, &src, total_bytes, &none, 0, false, false, &sh));
    TRY(shadow_in(c, sh, s));
    TRY(exchange_bufs(c, src, nullptr, &sp, &rp, inplace ? 1 : 0, fl));
    bool any_inplace = false;
    for (int p = 0; p < n; ++p) any_inplace = any_inplace || (fl[p] & 1);
    if (any_inplace)  // collective: every rank sees the same flags and max_cnt
        TRY(ensure_landing(c, (size_t)max_cnt * ext + 256));
    TRY(launch_barrier(c, s));
    void *dst = inplace ? (void *)c->land : rbuf;
    TRY(launch_reduce(c, op, type, sp, n, one_ptr(dst), 1, ro.order, ro.flags, jobs, s));
    TRY(launch_barrier(c, s));
    if (!any_inplace) return OMPI_AMD_SUCCESS;
    // the result leaves the landing buffer after the barrier (peers may read
    // this rank's input in rbuf until then); one more barrier keeps the
    // peers' next landing call from storing into it while the copy runs
    // (every rank sees the same flags, so every rank takes it)
    if (inplace && cnt > 0)
        TRY(record_hip(hipMemcpyAsync(rbuf, c->land, (size_t)cnt * ext, hipMemcpyDeviceToDevice, s),
                       "in-place result copy"));
    return launch_barrier(c, s);
}

// scan (exclusive = false) / exscan: rank r folds ranks 0..r (0..r-1) in
// the linear scan's order, which is the ring fold at first = 0.
// The stream a call of c runs on.  By default the caller's (stream-ordered
// after its producers).  With param own_stream — coll/rocm sets it: MPI
// callers hand over buffers that are ready at the call — every call of the
// communicator runs on one stream of its own, created with a CU mask of
// every CU so that HIP gives it a hardware queue of its own instead of one
// of the GPU_MAX_HW_QUEUES it shares among a process's streams.  A device
// wait of one communicator (a barrier spinning on its peers) then never sits
// in front of another communicator's kernels in one in-order queue: MPI lets
// ranks issue different communicators' collectives — and point-to-point
// traffic — in different orders (two nonblocking collectives posted in
// opposite orders), and with one queue per process that was a
// cycle of waits across ranks.  No event joins the caller's stream: the
// buffers are ready when the call is made.
static hipStream_t comm_stream(ompi_amd_comm_t *c, void *stream) {
    if (!c || !c->own_stream) return as_stream(stream);
    if (!c->own) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
            cus <= 0)
            cus = 256;
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xffffffffu);
        if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
        if (hipExtStreamCreateWithCUMask(&c->own, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
            (void)hipGetLastError();
            c->own = nullptr;
            if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
                (void)hipGetLastError();
                c->own = nullptr;
                return as_stream(stream);
            }
        }
    }
    return c->own;
}

static int scan_common(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                       int op, void *stream, bool exclusive) {
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    if (count == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    hipStream_t s = comm_stream(c, stream);
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
    path_params pp{c->small_bytes, c->fused_bytes, c->zero_copy, c->algorithm, c->tuned_alg, 0,
                   is_push(c->algorithm) && !c->user_ipc && !c->force_shadow ? 1 : 0, 0};
    pp.red_alg = c->tuned_red_alg;
    return pp;
}

// Whether an allreduce of `count` elements takes a zero-copy path (and so
// swaps buffer handles): the complement of the fused / staged conditions of
// allreduce_impl.
static bool allreduce_swaps(const ompi_amd_comm_t *c, const path_params &pp, size_t count,
                            int type) {
    const int n = c->size;
    if (n == 1 || count == 0) return false;
    const size_t bytes = count * ompi_amd_type_extent(type);
    const fold_plan fp = allreduce_fold(n, pp.tuned_alg, count, type, pp.root0_inplace != 0, pp.red_alg);
    const bool tree = fp.order == ORDER_TREE;
    if ((tree || fp.order == ORDER_RING) && bytes <= pp.fused_bytes && bytes <= c->scratch_bytes)
        return false;
    return !(bytes <= pp.small_bytes || !pp.zero_copy || (tree && bytes <= c->scratch_bytes));
}

// A zero-copy-size allreduce that runs push-gather: no handle swap (so a
// nonblocking or persistent one needs no host rendezvous), only a landing
// buffer of n + 1 slots, grown beforehand (growth is collective).
static bool allreduce_push_gathers(const ompi_amd_comm_t *c, const path_params &pp, size_t count,
                                   int type) {
    return pp.push_gather && allreduce_swaps(c, pp, count, type);
}

// Nonblocking and persistent allreduces of a size bucket the autotune has
// decided take the fastest measured candidate among the schemes that swap
// no handles (push-gather, push-land: the deferred launch needs no host
// rendezvous) with its grid; a bucket that chose the staged pull (which
// swaps) still gives its best push-type candidate.  Before the bucket is
// decided they keep the communicator's scheme.  Every rank made the same
// blocking calls before this one (MPI orders collectives alike on every
// rank), so every rank finds the same bucket state and takes the same path.
static void nb_tuned(ompi_amd_comm_t *c, path_params *pp, size_t count, int type) {
    if (!c->autotune || pp->tuned_alg != 0 || c->user_ipc || c->force_shadow ||
        !allreduce_swaps(c, *pp, count, type))
        return;
    const size_t bytes = count * ompi_amd_type_extent(type);
    const auto it = c->tune.find(63 - __builtin_clzll((unsigned long long)bytes));
    if (it == c->tune.end() || !it->second.done) return;
    int best = -1;
    for (int k = 0; k < it->second.ncand; ++k)
        if (is_push(kTune[k].algorithm) &&
            (best < 0 || it->second.worst_ms[k] < it->second.worst_ms[best]))
            best = k;
    if (best < 0) return;
    pp->algorithm = kTune[best].algorithm;
    pp->blocks = kTune[best].blocks;
    if (it->second.ncand == kTuneCands) pp->copy_nt = kTune[best].nt;
    pp->push_gather = 1;
    c->nb_tuned_alg = pp->algorithm;
    c->nb_tuned_blocks = pp->blocks;
    c->nb_tuned_nt = pp->copy_nt >= 0 ? pp->copy_nt : c->copy_nt;
}

static int allreduce_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                          int op, hipStream_t s, const path_params &pp);
static int rsb_impl(ompi_amd_comm_t *c, const void *src, void *rbuf, size_t rcount, int type,
                    int op, bool inplace, hipStream_t s);
static int allgather_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                          hipStream_t s);
static int bcast_impl(ompi_amd_comm_t *c, void *buf, const void *root_src, size_t bytes, int root,
                      hipStream_t s);
static int allgather_land(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                          hipStream_t s);
static int bcast_land(ompi_amd_comm_t *c, void *buf, size_t bytes, int root, hipStream_t s);
static size_t ag_landing_need(const ompi_amd_comm_t *c, size_t bytes);
static size_t bcast_landing_need(const ompi_amd_comm_t *c, size_t bytes);
static int reduce_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                       int op, int root, bool root_inplace, hipStream_t s);
static int rs_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, const size_t *rcounts,
                   int type, int op, hipStream_t s);

// Forced nonoverlapping only: every rank must know whether rank 0 passed
// MPI_IN_PLACE (it changes rank 0's first combine of the reduce,
// coll_base_allreduce.c:54-86); one host exchange, then in pp.
static int agree_root0_inplace(ompi_amd_comm_t *c, path_params *pp, bool inplace) {
    pp->root0_inplace = 0;
    if (pp->tuned_alg != TUNED_AR_NONOVERLAPPING || c->size == 1) return OMPI_AMD_SUCCESS;
    int mine = inplace ? 1 : 0, all[kMaxRanks];
    TRY(c->boot.allgather(&mine, all, sizeof(int)));
    pp->root0_inplace = all[0];
    return OMPI_AMD_SUCCESS;
}

// Launch deferred nonblocking calls in posting order, each once every rank
// has posted its handle-swap half; block = wait for them (the blocking entry
// points do, so their device work follows the deferred calls' on every rank).
// max_launch: stop after launching that many deferred calls (-1: no limit).
// Whether fused small allreduces store their own completion marks (env
// OMPI_AMD_FUSED_MARK=0: a mark kernel behind them instead, for A/B runs).
static bool fused_mark_on() {
    static const bool on = !(getenv("OMPI_AMD_FUSED_MARK") && atoi(getenv("OMPI_AMD_FUSED_MARK")) == 0);
    return on;
}

// A completion-counter slot of the flag page for a fused launch that
// signals its own mark (kFusedDoneSlots; slot 0 is the blocking call's);
// -1 when all are taken (the call then waits through a mark kernel).
static int done_slot_take(ompi_amd_comm_t *c) {
    if (!fused_mark_on()) return -1;
    if (!c->done_free.empty()) {
        const int k = c->done_free.back();
        c->done_free.pop_back();
        return k;
    }
    return c->done_next < kFusedDoneSlots ? c->done_next++ : -1;
}

static void done_slot_give(ompi_amd_comm_t *c, int k) {
    if (k > 0) c->done_free.push_back(k);
}

static int progress(ompi_amd_comm_t *c, bool block, int max_launch = -1);

// ---- progress across communicators (MPI's progress rule for nonblocking
// collectives).  A nonblocking call of communicator A launched on this rank
// waits on device for its peers; a peer may be blocked in a call of
// communicator B that only completes once this rank gets through B — and
// this rank may itself be held in B by the runtime (hipIpcCloseMemHandle
// of a retired mapping waits for every kernel of the device, A's spinning
// one included: measured 20 s, the device timeout, tests/ipc_share_worker.py
// step 5).  So every blocking wait of the library (host rendezvous, stream
// and event waits) launches the other communicators' ready deferred calls
// while it waits, as opal_progress drives libnbc's schedules.
static std::mutex g_comms_mu;
static std::vector<ompi_amd_comm_t *> g_comms;
static thread_local std::vector<const ompi_amd_comm_t *> tl_held;  // entry points this thread is in
static thread_local bool tl_in_progress = false;

struct api_guard {
    ompi_amd_comm_t *c;
    explicit api_guard(ompi_amd_comm_t *cc) : c(cc) {
        if (!c) return;
        c->api_mu.lock();
        tl_held.push_back(c);
    }
    ~api_guard() {
        if (!c) return;
        tl_held.pop_back();
        c->api_mu.unlock();
    }
    api_guard(const api_guard &) = delete;
    api_guard &operator=(const api_guard &) = delete;
};

// Launch what is ready among the other communicators' deferred calls (never
// blocks on a peer; skips a communicator another thread is in, and the ones
// this thread is in).
static void progress_others() {
    if (tl_in_progress) return;
    std::unique_lock<std::mutex> g(g_comms_mu, std::try_to_lock);
    if (!g.owns_lock()) return;
    tl_in_progress = true;
    for (ompi_amd_comm_t *o : g_comms) {
        if (o->npending.load() == 0 ||
            std::find(tl_held.begin(), tl_held.end(), o) != tl_held.end() || !o->api_mu.try_lock())
            continue;
        tl_held.push_back(o);
        if (set_dev(o) == OMPI_AMD_SUCCESS) (void)progress(o, false);
        tl_held.pop_back();
        o->api_mu.unlock();
    }
    tl_in_progress = false;
    if (!tl_held.empty()) (void)set_dev(const_cast<ompi_amd_comm_t *>(tl_held.back()));
}

// bootstrap.cpp's idle hook (its rendezvous spin loops)
static void boot_idle() { progress_others(); }
static const bool g_boot_idle_set = [] {
    set_boot_idle_hook(boot_idle);
    return true;
}();

// The library's waits (host_mark.h) run the other communicators' ready
// deferred calls between polls.
static hipError_t wait_stream(hipStream_t s) { return mark_stream_wait(s, progress_others); }

static hipError_t wait_event(hipEvent_t ev) {
    return mark_event_wait(ev, nullptr, 0, progress_others);
}
static hipError_t wait_marked(hipEvent_t ev, const uint64_t *w, uint64_t v) {
    return mark_event_wait(ev, w, v, progress_others);
}

// a nonblocking request's completion event: from the communicator's pool
// (hipEventCreate on every MPI_I* call costs more than the call's launch)
static hipError_t req_event_get(ompi_amd_comm_t *c, hipEvent_t *ev) {
    if (!c->req_ev_free.empty()) {
        *ev = c->req_ev_free.back();
        c->req_ev_free.pop_back();
        return hipSuccess;
    }
    return hipEventCreateWithFlags(ev, hipEventDisableTiming);
}
static void req_event_put(ompi_amd_comm_t *c, hipEvent_t ev) {
    if (ev) c->req_ev_free.push_back(ev);
}

static int progress(ompi_amd_comm_t *c, bool block, int max_launch) {
    while (!c->pending.empty() && max_launch-- != 0) {
        if (c->unposted) {  // tickets the full ring held back (nb_ticket)
            std::unique_ptr<host_step> st(block ? new host_step("post queued tickets (blocking)") : nullptr);
            TRY(post_queued(c, block && c->pending.front().unposted));
            if (c->pending.front().unposted) return OMPI_AMD_SUCCESS;
        }
        if (c->land_failed) {
            // a deferred growth failed (every peer was told: abort_peers):
            // the calls behind it were sized for the buffers it would have
            // made, so they complete with the error, unlaunched
            pending_op o = c->pending.front();
            c->pending.pop_front();
            c->npending.fetch_sub(1);
            if (o.grow) c->land_retired.push_back(o.grow);
            if (o.req) {
                o.req->rc = OMPI_AMD_ERR_HIP;
                o.req->launched = true;
            }
            continue;
        }
        if (c->pending.front().kind == PEND_GROW) {
            const pending_op g = c->pending.front();
            land_blob lall[kMaxRanks];
            bool ready = false;
            int rc = c->boot.test(g.ticket, lall, sizeof(land_blob), block, &ready);
            if (rc == OMPI_AMD_SUCCESS && !ready) return OMPI_AMD_SUCCESS;
            c->pending.pop_front();
            c->npending.fetch_sub(1);
            if (rc == OMPI_AMD_SUCCESS) rc = grow_launch(c, g, lall);
            else c->land_failed = true;
            if (rc != OMPI_AMD_SUCCESS) {
                abort_peers(c, rc);
                return rc;
            }
            continue;
        }
        pending_op o = c->pending.front();
        call_blob all[kMaxRanks];
        int rc = OMPI_AMD_SUCCESS;
        if (o.ticket) {
            bool ready = false;
            std::unique_ptr<host_step> st(block ? new host_step("ticket test (blocking)", o.ticket) : nullptr);
            rc = c->boot.test(o.ticket, all, sizeof(call_blob), block, &ready);
            if (rc == OMPI_AMD_SUCCESS && !ready) return OMPI_AMD_SUCCESS;
        }
        c->pending.pop_front();
        c->npending.fetch_sub(1);
        if (rc == OMPI_AMD_SUCCESS) {
            c->pre = o.ticket ? all : nullptr;
            rc = shadow_in(c, o.sh, o.stream);
            if (rc == OMPI_AMD_SUCCESS) {
                switch (o.kind) {
                case PEND_RSB:
                    rc = rsb_impl(c, o.sbuf, o.rbuf, o.count, o.type, o.op, o.inplace, o.stream);
                    break;
                case PEND_ALLGATHER:
                    rc = o.land ? allgather_land(c, o.sbuf, o.rbuf, o.count, o.stream)
                                : allgather_impl(c, o.sbuf, o.rbuf, o.count, o.stream);
                    break;
                case PEND_BCAST:
                    rc = o.land ? bcast_land(c, o.rbuf, o.count, o.root, o.stream)
                                : bcast_impl(c, o.rbuf, o.sbuf, o.count, o.root, o.stream);
                    break;
                case PEND_REDUCE:
                case PEND_SCAN:
                case PEND_RS: {
                    // these post no buffer descriptors: they launch on the
                    // staged / landing paths only (no handle swap at launch)
                    const int ui = c->user_ipc, fs = c->force_shadow;
                    c->user_ipc = 0;
                    c->force_shadow = 0;
                    if (o.kind == PEND_REDUCE)
                        rc = reduce_impl(c, o.sbuf, o.rbuf, o.count, o.type, o.op, o.root,
                                         o.ticket && (all[o.root].flags & 1), o.stream);
                    else if (o.kind == PEND_SCAN)
                        rc = scan_common(c, o.sbuf, o.rbuf, o.count, o.type, o.op, o.stream,
                                         o.exclusive);
                    else
                        rc = rs_impl(c, o.sbuf, o.rbuf, o.rcounts.data(), o.type, o.op, o.stream);
                    c->user_ipc = ui;
                    c->force_shadow = fs;
                    break;
                }
                default: {
                    // a fused launch stores the request's mark itself
                    const int slot = o.req->mark ? done_slot_take(c) : -1;
                    c->want_mark = slot >= 0;
                    c->mark_word = o.req->mark;
                    c->mark_slot = std::max(slot, 0);
                    c->mark_embedded = 0;
                    rc = allreduce_impl(c, o.sbuf, o.rbuf, o.count, o.type, o.op, o.stream, o.pp);
                    c->want_mark = false;
                    o.req->embedded = c->mark_embedded;
                    c->mark_embedded = 0;
                    if (o.req->embedded) o.req->done_slot = slot;
                    else done_slot_give(c, slot);  // not a fused launch: unused
                }
                }
            }
            if (rc == OMPI_AMD_SUCCESS) rc = shadow_out(c, o.sh, o.stream);
            c->pre = nullptr;
        }
        o.req->stream = o.stream;
        o.req->rc = rc;
        o.req->launched = true;
        if (rc != OMPI_AMD_SUCCESS) {
            // peers launch this call from their own progress and would wait
            // for this rank's device work until their timeout
            abort_peers(c, rc);
            return rc;
        }
    }
    return OMPI_AMD_SUCCESS;
}

// After a nonblocking post: launch what is ready, here and on the other
// communicators (any call into the library progresses them all, as
// opal_progress does: a peer's kernels of another communicator may be
// waiting for this rank's launch of them).
static int post_progress(ompi_amd_comm_t *c) {
    const int rc = progress(c, false);
    progress_others();
    return rc;
}

static int drain(ompi_amd_comm_t *c) {
    return c->pending.empty() ? OMPI_AMD_SUCCESS : progress(c, true);
}

static int allreduce_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                          int op, hipStream_t s, const path_params &pp) {
    if (count == 0) return OMPI_AMD_SUCCESS;  // allreduce.c:104
    TRY(set_dev(c));
    // a deferred call's own grid (nb_tuned) for the launches below
    struct grid_scope {
        ompi_amd_comm_t *c;
        int saved, saved_nt;
        ~grid_scope() {
            c->max_blocks = saved;
            c->copy_nt = saved_nt;
        }
    } grid{c, c->max_blocks, c->copy_nt};
    if (pp.blocks > 0) c->max_blocks = pp.blocks;
    if (pp.copy_nt >= 0) c->copy_nt = pp.copy_nt;
    const size_t ext = ompi_amd_type_extent(type);
    const size_t bytes = count * ext;
    const bool inplace = in_place(sbuf, rbuf);
    const void *src = inplace ? rbuf : sbuf;
    const int n = c->size;
    if (n == 1) {  // coll/self: copy (or nothing in place)
        if (inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, bytes, hipMemcpyDeviceToDevice, s), "copy");
    }
    // the operand order coll/tuned would use (fixed decision or forced)
    const fold_plan fp = allreduce_fold(n, pp.tuned_alg, count, type, pp.root0_inplace != 0, pp.red_alg);
    const bool tree = fp.order == ORDER_TREE;
    if ((tree || fp.order == ORDER_RING) && bytes <= pp.fused_bytes && bytes <= c->scratch_bytes)
        return allreduce_fused(c, src, rbuf, (int64_t)count, op, type, tree, s);
    if (!tree && (bytes <= pp.small_bytes || !pp.zero_copy) &&
        two_shot_fits(c, (int64_t)count, ext))
        return allreduce_staged_two_shot(c, src, rbuf, (int64_t)count, op, type, fp, s);
    if (bytes <= pp.small_bytes || !pp.zero_copy || (tree && bytes <= c->scratch_bytes)) {
        // staged one-shot: my contribution -> my scratch half, barrier,
        // every rank folds all blocks from all scratches (no trailing
        // barrier: see next_half)
        stage_half sh;
        TRY(stage_in(c, src, bytes, &sh, s));
        red_jobs jobs;
        fold_jobs(fp, (int64_t)count, n, -1, &jobs);
        return launch_reduce(c, op, type, sh.peers, n, one_ptr(rbuf), 1, fp.order, fp.flags, jobs, s);
    }
    ptr_set sp{}, rp{};
    if (!c->pre && pp.push_gather)
        return allreduce_push_gather(c, src, rbuf, (int64_t)count, op, type, fp, s, pp.algorithm);
    if (!c->pre && (pp.algorithm == ALG_PULL || pp.algorithm == ALG_PULL_PIPE) && !c->user_ipc &&
        !c->force_shadow) {
        // staged pull: the input into this rank's shadow (rbuf's phase mod
        // 256, so results and shadows line up for 16-B vectors), swap
        // shadows, fold / gather through them
        char *base = nullptr;
        TRY(shadow_reserve(c, bytes + 256, &base));
        char *sh = base + ((uintptr_t)rbuf & 255);
        if (pp.algorithm == ALG_PULL_PIPE && pipe_fits(c, fp)) {  // the copy runs inside the pipeline
            TRY(exchange_bufs(c, sh, nullptr, &sp, &rp));
            return allreduce_pull_pipe(c, sp, sh, src, rbuf, (int64_t)count, op, type, fp, s);
        }
        cp_jobs cj{};
        cj.n = 1;
        cj.j[0] = {(const char *)src, sh, (int64_t)bytes};
        TRY(launch_copy(c, cj, s));
        TRY(exchange_bufs(c, sh, nullptr, &sp, &rp));
        return allreduce_pull_staged(c, sp, sh, rbuf, (int64_t)count, op, type, fp, s);
    }
    // export fallback (shadow_plan); a deferred call substituted its
    // shadows when it was posted, so these export and plan nothing
    const bool push = is_push(pp.algorithm);
    const void *xs = push ? nullptr : src;
    void *xr = rbuf;
    shadow_set sh;
    if (c->pre) {
        // deferred: the posted descriptors are final (progress() runs the
        // call's own shadow copies around it)
    } else if (push) {
        TRY(shadow_plan(c, &xs, 0, &xr, bytes, false, false, &sh));
    } else {
        TRY(shadow_plan(c, &xs, bytes, &xr, bytes, inplace, false, &sh));
        src = xs;
    }
    rbuf = xr;
    TRY(shadow_in(c, sh, s));
    int rc;
    if (push) {
        TRY(ensure_landing(c, push_slot((int64_t)count, n, type) * (size_t)n));
        TRY(exchange_bufs(c, nullptr, rbuf, &sp, &rp));
        rc = allreduce_push(c, src, rp, (int64_t)count, op, type, fp, s);
    } else {
        TRY(exchange_bufs(c, src, rbuf, &sp, &rp));
        if (inplace) sp = rp;
        rc = pp.algorithm == ALG_PULL_PUSH
                 ? allreduce_pull_push(c, sp, rp, (int64_t)count, op, type, fp, s)
                 : allreduce_pull(c, sp, rp, rbuf, (int64_t)count, op, type, fp, s);
    }
    TRY(rc);
    return shadow_out(c, sh, s);
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
    // coll/tuned's own forcing variables (coll_tuned_allreduce_decision.c:
    // 37-101): honoured when dynamic rules are on, as tuned does
    // (the environment form, for callers outside Open MPI; coll/rocm reads
    // them through the MCA variable system and sets them per communicator)
    if (const char *d = getenv("OMPI_MCA_coll_tuned_use_dynamic_rules")) {
        const char *a = getenv("OMPI_MCA_coll_tuned_allreduce_algorithm");
        if (atoi(d) && a && atoi(a) >= 0 && atoi(a) < TUNED_AR_COUNT) c->tuned_alg = atoi(a);
        const char *r = getenv("OMPI_MCA_coll_tuned_reduce_algorithm");
        if (atoi(d) && r && tuned_red_alg_ok(atoi(r))) c->tuned_red_alg = atoi(r);
        const char *rs = getenv("OMPI_MCA_coll_tuned_reduce_scatter_algorithm");
        if (atoi(d) && rs && atoi(rs) >= 0 && atoi(rs) <= TUNED_RS_RING) c->tuned_rs_alg = atoi(rs);
    }
    if (const char *u = getenv("OMPI_AMD_USER_IPC")) c->user_ipc = atoi(u) ? 1 : 0;
    if (const char *a = getenv("OMPI_AMD_COLL_ALGORITHM")) {
        const int v = atoi(a);
        if (v >= 0 && v < ALG_COUNT) c->algorithm = v;
    }
    int rc = set_dev(c);
    if (rc == OMPI_AMD_SUCCESS) rc = c->boot.attach(name, rank, size, 120.0);
    if (rc != OMPI_AMD_SUCCESS) { delete c; return rc; }
    // device resources: fine-grained flags, scratch, pinned error word
    c->scratch_bytes = std::max<size_t>(c->small_bytes, 4 << 20);  // per half
    ipc_blob mine{}, all[kMaxRanks];
    // the flag page, then the pipelined schemes' rows (kPipeFlagOff)
    const size_t flag_bytes = kPipeFlagOff + kPipeFlagBytes;
    hipError_t e;
    {
        host_step st("comm_create device resources", (size_t)rank);
        e = alloc_exportable(flag_bytes, (char **)&c->flags, &mine.flags.h, true);
        if (e == hipSuccess) e = hipMemsetAsync(c->flags, 0, flag_bytes, nullptr);
        if (e == hipSuccess) e = alloc_exportable(2 * c->scratch_bytes, &c->scratch, &mine.scratch.h);
        if (e == hipSuccess) e = hipHostMalloc((void **)&c->err_host, 64, hipHostMallocMapped);
        if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&c->err_dev, c->err_host, 0);
        if (e == hipSuccess && getenv("OMPI_AMD_DEBUG_PROGRESS") && atoi(getenv("OMPI_AMD_DEBUG_PROGRESS"))) {
            e = hipHostMalloc((void **)&c->dbg_host, (2 + kMaxRanks) * sizeof(uint64_t), hipHostMallocMapped);
            if (e == hipSuccess) {
                memset(c->dbg_host, 0, (2 + kMaxRanks) * sizeof(uint64_t));
                e = hipHostGetDevicePointer((void **)&c->dbg_dev, c->dbg_host, 0);
            }
        }
        if (e == hipSuccess) e = hipStreamSynchronize(nullptr);  // the flag page is zero
    }
    if (e != hipSuccess) {
        rc = record_hip(e, "comm device resources");
        ompi_amd_comm_destroy(c);
        return rc;
    }
    describe_alloc(c->flags, &mine.flags);
    describe_alloc(c->scratch, &mine.scratch);
    if (hipDeviceGetAttribute(&mine.pci[0], hipDeviceAttributePciDomainID, device) != hipSuccess ||
        hipDeviceGetAttribute(&mine.pci[1], hipDeviceAttributePciBusId, device) != hipSuccess ||
        hipDeviceGetAttribute(&mine.pci[2], hipDeviceAttributePciDeviceId, device) != hipSuccess) {
        (void)hipGetLastError();
        mine.pci[0] = mine.pci[1] = mine.pci[2] = -1;  // unknown: counted as shared
    }
    *c->err_host = 0;
    c->fused_mark = mark_word_get();  // nullptr with marks off: ompi_amd_allreduce_wait syncs instead
    ipc_add_user(c, quiesce_user);
    if (rank == 0) rc = p2p_create(c, name, rank, size, 0, &c->p2p);
    if (rc == OMPI_AMD_SUCCESS) rc = c->boot.allgather(&mine, all, sizeof(ipc_blob));
    if (rc == OMPI_AMD_SUCCESS && rank != 0) rc = p2p_create(c, name, rank, size, 1, &c->p2p);
    for (int p = 0; rc == OMPI_AMD_SUCCESS && p < size; ++p) {
        int same = 0;
        for (int q = 0; q < size; ++q)
            same += (all[q].pci[0] < 0 || memcmp(all[q].pci, all[p].pci, sizeof(all[p].pci)) == 0) ? 1 : 0;
        c->colocated = std::max(c->colocated, same);
    }
    for (int p = 0; rc == OMPI_AMD_SUCCESS && p < size; ++p) {
        if (p == rank) {
            c->peer_flags.p[p] = c->flags;
            c->peer_scratch.p[p] = c->scratch;
            continue;
        }
        void *f = nullptr, *s = nullptr;
        host_step st("comm_create map peer", (size_t)p);
        rc = ipc_map(alloc_of(all[p].flags), c, &c->opened[p][0], &f);
        if (rc == OMPI_AMD_SUCCESS) rc = ipc_map(alloc_of(all[p].scratch), c, &c->opened[p][1], &s);
        if (rc != OMPI_AMD_SUCCESS) break;
        c->peer_flags.p[p] = (uint64_t *)f;
        c->peer_scratch.p[p] = (const char *)s;
    }
    if (rc == OMPI_AMD_SUCCESS) rc = c->boot.barrier();  // all mapped before first use
    if (rc != OMPI_AMD_SUCCESS) {
        ompi_amd_comm_destroy(c);
        return rc;
    }
    if (rank == 0 && c->p2p) p2p_unlink(c->p2p);  // every rank has it mapped
    {
        std::lock_guard<std::mutex> g(g_comms_mu);
        g_comms.push_back(c);
    }
    *out = c;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_destroy(ompi_amd_comm_t *c) {
    if (!c) return OMPI_AMD_SUCCESS;
    {  // no progress_others() reaches it from here on
        std::lock_guard<std::mutex> g(g_comms_mu);
        g_comms.erase(std::remove(g_comms.begin(), g_comms.end(), c), g_comms.end());
    }
    { std::lock_guard<std::recursive_mutex> w(c->api_mu); }  // (and none is still in it)
    hip_ignore(hipSetDevice(c->device));
    (void)drain(c);  // deferred nonblocking calls every peer will also launch
    for (auto &o : c->pending)  // left by a failed drain: queued growths' buffers
        if (o.grow) c->land_retired.push_back(o.grow);
    (void)quiesce(c, "quiesce (destroy)");
    (void)c->boot.barrier();  // nobody still reads our memory
    ipc_remove_user(c);
    for (auto &x : c->imports) ipc_unmap(x.ref, c);  // the process's mapping stays while others hold it
    c->imports.clear();
    if (c->osc_release) c->osc_release(c->osc_state, 0);  // its peer mappings
    for (int p = 0; p < kMaxRanks; ++p) {
        for (int k = 0; k < 2; ++k) ipc_unmap(c->opened[p][k], c);
        ipc_unmap(c->land_ref[p], c);
        c->land_ref[p] = nullptr;
    }
    for (ipc_ref *r : c->land_ref_retired) ipc_unmap(r, c);
    c->land_ref_retired.clear();
    (void)c->boot.barrier();
    if (c->osc_release) c->osc_release(c->osc_state, 1);  // its own memory
    // recycled for later communicators, not freed (release_exportable)
    release_exportable(c->flags);
    release_exportable(c->scratch);
    release_exportable(c->land);
    for (char *q : c->land_retired) release_exportable(q);
    c->land_retired.clear();
    for (auto &ch : c->arena) release_exportable(ch.base);  // shadows included
    c->arena.clear();
    if (c->err_host) hip_ignore(hipHostFree(c->err_host));
    if (c->dbg_host) hip_ignore(hipHostFree(c->dbg_host));
    for (int ph = 0; ph < 3; ++ph)
        for (auto &pr : c->ev_phase[ph]) {
            hip_ignore(hipEventDestroy(pr.first));
            hip_ignore(hipEventDestroy(pr.second));
        }
    mark_word_put(c->fused_mark);  // its last wait is over (destroy drained the streams)
    for (auto e : c->ev_free) hip_ignore(hipEventDestroy(e));
    for (auto e : c->req_ev_free) hip_ignore(hipEventDestroy(e));
    for (auto &kv : c->tune)
        for (auto e : kv.second.ev)
            if (e) hip_ignore(hipEventDestroy(e));
    if (c->p2p) p2p_destroy(c->p2p);
    c->boot.detach();
    forget_streams(c);
    if (c->own) hip_ignore(hipStreamDestroy(c->own));  // drained above
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

int ompi_amd_coll_reduce_order_forced(int size, size_t msg_bytes, size_t count, int root,
                                      int root_inplace, int forced, int *order, int *first) {
    if (size < 1 || root < 0 || root >= size || !order || !first) return OMPI_AMD_ERR_BAD_PARAM;
    if (!tuned_red_alg_ok(forced)) return OMPI_AMD_ERR_UNSUPPORTED;
    const red_order ro = tuned_reduce_order(size, msg_bytes, count, root, root_inplace != 0, forced);
    *order = ro.order;
    *first = ro.first;
    return OMPI_AMD_SUCCESS;
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
    api_guard api_(c);
    if (!c || phase < 0 || phase > 2 || !total_ms || !calls) return OMPI_AMD_ERR_BAD_PARAM;
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
    api_guard api_(c);
    if (!c || !all_ok) return OMPI_AMD_ERR_BAD_PARAM;
    int mine = local_ok ? 1 : 0, all[kMaxRanks];
    TRY(drain(c));
    TRY(c->boot.allgather(&mine, all, sizeof(int)));
    int ok = 1;
    for (int p = 0; p < c->size; ++p) ok &= all[p];
    *all_ok = ok;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_vote(ompi_amd_comm_t *c, int local_yes, int *n_yes) {
    api_guard api_(c);
    if (!c || !n_yes) return OMPI_AMD_ERR_BAD_PARAM;
    int mine = local_yes ? 1 : 0, all[kMaxRanks];
    TRY(drain(c));
    TRY(c->boot.allgather(&mine, all, sizeof(int)));
    int k = 0;
    for (int p = 0; p < c->size; ++p) k += all[p];
    *n_yes = k;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_allreduce_wait(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                            int op) {
    if (!c) return OMPI_AMD_ERR_BAD_PARAM;
    c->want_mark = fused_mark_on();
    c->mark_word = c->fused_mark;
    c->mark_slot = 0;
    c->mark_embedded = 0;
    const int rc = ompi_amd_allreduce(c, sbuf, rbuf, count, type, op, nullptr);
    c->want_mark = false;
    const uint64_t v = c->mark_embedded;
    c->mark_embedded = 0;
    if (rc != OMPI_AMD_SUCCESS || !v) return rc != OMPI_AMD_SUCCESS ? rc : ompi_amd_comm_sync(c, nullptr);
    // the fused kernel was the call's last launch on the per-thread stream,
    // and it stores the mark itself: no mark kernel behind it
    api_guard api_(c);
    TRY(record_hip(mark_value_wait(comm_stream(c, nullptr), c->fused_mark, v, progress_others), "allreduce wait"));
    return check_sticky(c);
}

int ompi_amd_comm_abort(ompi_amd_comm_t *c, int rc) {
    api_guard api_(c);
    if (!c || rc >= 0) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(set_dev(c));
    abort_peers(c, rc);
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_comm_sync(ompi_amd_comm_t *c, void *stream) {
    api_guard api_(c);
    if (!c) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(set_dev(c));
    TRY(drain(c));
    TRY(record_hip(wait_stream(comm_stream(c, stream)), "hipStreamSynchronize"));
    return check_sticky(c);
}

int ompi_amd_comm_rank(const ompi_amd_comm_t *c) { return c ? c->rank : -1; }
int ompi_amd_comm_size(const ompi_amd_comm_t *c) { return c ? c->size : -1; }

int ompi_amd_comm_error(const ompi_amd_comm_t *c) {
    return c ? __atomic_load_n(c->err_host, __ATOMIC_ACQUIRE) : OMPI_AMD_ERR_BAD_PARAM;
}

int ompi_amd_comm_set_param(ompi_amd_comm_t *c, const char *key, int64_t v) {
    api_guard api_(c);
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
    } else if (!strcmp(key, "bcast_split_bytes")) {
        if (v < 0) return OMPI_AMD_ERR_BAD_PARAM;
        c->bcast_split_bytes = (size_t)v;
    } else if (!strcmp(key, "blocks")) {
        if (v <= 0 || v > 65535) return OMPI_AMD_ERR_BAD_PARAM;
        c->max_blocks = (int)v;
        c->autotune = 0;  // an explicit grid is not second-guessed
    } else if (!strcmp(key, "autotune")) {
        c->autotune = v ? 1 : 0;
    } else if (!strcmp(key, "land_blocking")) {
        c->land_blocking = v ? 1 : 0;
    } else if (!strcmp(key, "copy_nt")) {
        c->copy_nt_fixed = v >= 0;
        c->copy_nt = v != 0 ? 1 : 0;
    } else if (!strcmp(key, "fused_bytes")) {
        if (v < 0) return OMPI_AMD_ERR_BAD_PARAM;
        c->fused_bytes = std::min<size_t>((size_t)v, c->scratch_bytes);
    } else if (!strcmp(key, "algorithm")) {
        if (v < 0 || v >= ALG_COUNT) return OMPI_AMD_ERR_BAD_PARAM;
        c->algorithm = (int)v;
        c->autotune = 0;  // an explicit scheme is not second-guessed
    } else if (!strcmp(key, "pipe_slice")) {
        if (v < 16 || v > (64 << 20)) return OMPI_AMD_ERR_BAD_PARAM;
        c->pipe_slice = v;
    } else if (!strcmp(key, "pipe_passes")) {
        if (v < 1 || v > 4096) return OMPI_AMD_ERR_BAD_PARAM;
        c->pipe_passes = (int)v;
    } else if (!strcmp(key, "force_shadow")) {
        c->force_shadow = v ? 1 : 0;
    } else if (!strcmp(key, "reuse_shadow")) {
        c->reuse_shadow = v ? 1 : 0;
    } else if (!strcmp(key, "osc_win_shadow")) {
        c->win_shadow = v ? 1 : 0;
    } else if (!strcmp(key, "osc_win_separate")) {
        c->win_separate = v ? 1 : 0;
    } else if (!strcmp(key, "user_ipc")) {
        c->user_ipc = v ? 1 : 0;
        c->autotune = 0;
    } else if (!strcmp(key, "tuned_allreduce_algorithm")) {
        if (v < 0 || v >= TUNED_AR_COUNT) return OMPI_AMD_ERR_BAD_PARAM;
        c->tuned_alg = (int)v;
    } else if (!strcmp(key, "own_stream")) {
        c->own_stream = v ? 1 : 0;
    } else if (!strcmp(key, "tuned_reduce_algorithm")) {
        if (!tuned_red_alg_ok(v)) return OMPI_AMD_ERR_UNSUPPORTED;  // the caller keeps tuned's path
        c->tuned_red_alg = (int)v;
    } else if (!strcmp(key, "tuned_reduce_scatter_algorithm")) {
        if (v < 0 || v > TUNED_RS_RING) return OMPI_AMD_ERR_UNSUPPORTED;
        c->tuned_rs_alg = (int)v;
    } else if (!strcmp(key, "tuned_reduce_scatter_block_algorithm")) {
        if (v < 0 || v > TUNED_RSB_BASIC_LINEAR) return OMPI_AMD_ERR_UNSUPPORTED;
        c->tuned_rsb_alg = (int)v;
    } else if (!strncmp(key, "p2p_", 4) && p2p_set_param(c->p2p, key, v) != OMPI_AMD_ERR_UNSUPPORTED) {
        return p2p_set_param(c->p2p, key, v);
    } else {
        record_msg("unknown coll param '%s'", key);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    return OMPI_AMD_SUCCESS;
}

// the store kind candidate k of a bucket ran with (a fixed copy_nt: that)
static int tune_nt(const ompi_amd_comm_t *c, const tune_bucket &tb, int k) {
    return tb.ncand == kTuneCands ? kTune[k].nt : c->copy_nt;
}

int ompi_amd_comm_get_param(const ompi_amd_comm_t *c, const char *key, int64_t *v) {
    if (!c || !key || !v) return OMPI_AMD_ERR_BAD_PARAM;
    if (!strcmp(key, "small_bytes")) *v = (int64_t)c->small_bytes;
    else if (!strcmp(key, "zero_copy")) *v = c->zero_copy;
    else if (!strcmp(key, "pipe_slice")) *v = c->pipe_slice;
    else if (!strcmp(key, "pipe_passes")) *v = c->pipe_passes;
    else if (!strcmp(key, "pipe_calls")) *v = (int64_t)c->pipe_seq;
    else if (!strcmp(key, "colocated")) *v = c->colocated;
    else if (!strcmp(key, "timeout_ms")) *v = (int64_t)c->timeout_ms;
    else if (!strcmp(key, "profile")) *v = c->profile;
    else if (!strcmp(key, "blocks")) *v = c->max_blocks;
    else if (!strcmp(key, "fused_bytes")) *v = (int64_t)c->fused_bytes;
    else if (!strcmp(key, "algorithm")) *v = c->algorithm;
    else if (!strcmp(key, "autotune")) *v = c->autotune;
    else if (!strcmp(key, "autotune_state")) *v = c->tune_last;
    else if (!strcmp(key, "nb_tuned_algorithm")) *v = c->nb_tuned_alg;
    else if (!strcmp(key, "nb_tuned_blocks")) *v = c->nb_tuned_blocks;
    else if (!strcmp(key, "nb_tuned_copy_nt")) *v = c->nb_tuned_nt;
    else if (!strcmp(key, "landing_ag_bcast")) *v = c->land_ag_bcast;
    else if (!strcmp(key, "land_blocking")) *v = c->land_blocking;
    else if (!strcmp(key, "copy_nt")) *v = c->copy_nt;
    else if (!strcmp(key, "copy_nt_fixed")) *v = c->copy_nt_fixed;
    else if (!strcmp(key, "unsafe_exports")) *v = c->unsafe_exports;
    else if (!strcmp(key, "aged_exports")) *v = c->aged_exports;
    else if (!strncmp(key, "autotune_", 9) && c->tune_last_key >= 0 &&
             c->tune.count(c->tune_last_key) && c->tune.at(c->tune_last_key).done) {
        // the last decided bucket: its choice and every candidate's worst rank
        const tune_bucket &tb = c->tune.at(c->tune_last_key);
        const auto idx = [&](int at) { return atoi(key + at) >= 0 && atoi(key + at) < tb.ncand; };
        if (!strcmp(key, "autotune_algorithm")) *v = kTune[tb.choice].algorithm;
        else if (!strcmp(key, "autotune_blocks")) *v = kTune[tb.choice].blocks;
        else if (!strcmp(key, "autotune_copy_nt")) *v = tune_nt(c, tb, tb.choice);
        else if (!strcmp(key, "autotune_ncand")) *v = tb.ncand;
        else if (!strncmp(key, "autotune_us", 11) && idx(11))
            *v = (int64_t)(tb.worst_ms[atoi(key + 11)] * 1000.f);
        else if (!strncmp(key, "autotune_alg", 12) && idx(12))
            *v = kTune[atoi(key + 12)].algorithm;
        else if (!strncmp(key, "autotune_grid", 13) && idx(13))
            *v = kTune[atoi(key + 13)].blocks;
        else if (!strncmp(key, "autotune_nt", 11) && idx(11))
            *v = tune_nt(c, tb, atoi(key + 11));
        else return OMPI_AMD_ERR_BAD_PARAM;
    }
    else if (!strcmp(key, "tuned_allreduce_algorithm")) *v = c->tuned_alg;
    else if (!strcmp(key, "tuned_reduce_algorithm")) *v = c->tuned_red_alg;
    else if (!strcmp(key, "own_stream")) *v = c->own_stream;
    else if (!strcmp(key, "tuned_reduce_scatter_algorithm")) *v = c->tuned_rs_alg;
    else if (!strcmp(key, "tuned_reduce_scatter_block_algorithm")) *v = c->tuned_rsb_alg;
    else if (!strcmp(key, "landing_bytes")) *v = (int64_t)c->land_bytes;
    else if (!strcmp(key, "landing_deferred_growths")) *v = c->deferred_growths;
    else if (!strcmp(key, "landing_retired")) *v = (int64_t)c->land_retired.size();
    else if (!strcmp(key, "boot_calls")) *v = (int64_t)c->boot.posted();
    else if (!strcmp(key, "ipc_opens")) *v = ipc_get_stats().opens;
    else if (!strcmp(key, "ipc_refusals")) *v = ipc_get_stats().refusals;
    else if (!strcmp(key, "ipc_close_watermark")) *v = (int64_t)ipc_close_watermark();
    else if (!strcmp(key, "ipc_closes")) *v = ipc_get_stats().closes;
    else if (!strcmp(key, "ipc_shared")) *v = ipc_get_stats().shared;
    else if (!strcmp(key, "ipc_retired")) *v = ipc_get_stats().retired;
    else if (!strcmp(key, "ipc_live")) *v = ipc_get_stats().live;
    else if (!strcmp(key, "ipc_refs")) *v = ipc_get_stats().refs;
    else if (!strcmp(key, "bcast_split")) *v = c->bcast_split;
    else if (!strcmp(key, "bcast_split_bytes")) *v = (int64_t)c->bcast_split_bytes;
    else if (!strcmp(key, "memcpy_token_mismatch")) *v = c->memcpy_token_mismatch;
    else if (!strcmp(key, "shadowed")) *v = c->shadowed;
    else if (!strcmp(key, "epoch")) *v = (int64_t)c->epoch;
    else if (!strncmp(key, "dbg_", 4) && c->dbg_host) {  // dbg_entered / dbg_left / dbg_seenP
        volatile uint64_t *d = c->dbg_host;
        if (!strcmp(key, "dbg_entered")) *v = (int64_t)d[0];
        else if (!strcmp(key, "dbg_left")) *v = (int64_t)d[1];
        else if (!strncmp(key, "dbg_seen", 8) && atoi(key + 8) >= 0 && atoi(key + 8) < kMaxRanks)
            *v = (int64_t)d[2 + atoi(key + 8)];
        else return OMPI_AMD_ERR_BAD_PARAM;
    }
    else if (!strcmp(key, "exports_new")) *v = c->exports_new;
    else if (!strcmp(key, "recycled_exports")) *v = c->recycled_exports;
    else if (!strcmp(key, "imports_new")) *v = c->imports_new;
    else if (!strcmp(key, "force_shadow")) *v = c->force_shadow;
    else if (!strcmp(key, "osc_win_shadow")) *v = c->win_shadow;
    else if (!strcmp(key, "osc_win_separate")) *v = c->win_separate;
    else if (!strcmp(key, "reuse_shadow")) *v = c->reuse_shadow;
    else if (!strcmp(key, "reused_exports")) *v = c->reused_exports;
    else if (!strcmp(key, "osc_shadow_windows")) *v = c->shadow_windows;
    else if (!strcmp(key, "user_ipc")) *v = c->user_ipc;
    else if (!strcmp(key, "imports")) *v = (int64_t)c->imports.size();
    else if (!strncmp(key, "p2p_", 4) && p2p_get_param(c->p2p, key, v) == OMPI_AMD_SUCCESS) return OMPI_AMD_SUCCESS;
    else if (!strcmp(key, "ipc_mode_legacy_env")) *v = ipc_mode_env_at_load();
    else if (!strcmp(key, "ipc_mode_legacy")) *v = *ipc_mode_env_now() ? atoi(ipc_mode_env_now()) : -1;
    else {
        record_msg("unknown coll param '%s'", key);
        return OMPI_AMD_ERR_BAD_PARAM;
    }
    return OMPI_AMD_SUCCESS;
}


int ompi_amd_allreduce(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                       int op, void *stream) {
    api_guard api_(c);
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    path_params pp = params_of(c);
    TRY(agree_root0_inplace(c, &pp, in_place(sbuf, rbuf)));
    const hipStream_t s = comm_stream(c, stream);
    tune_bucket *tb = nullptr;
    int cand = -1;
    const int save_alg = c->algorithm, save_blocks = c->max_blocks;
    if (c->autotune && pp.tuned_alg == 0 && !c->user_ipc && !c->force_shadow &&
        allreduce_swaps(c, pp, count, type)) {
        const size_t bytes = count * ompi_amd_type_extent(type);
        const int key = 63 - __builtin_clzll((unsigned long long)bytes);
        const bool fresh = !c->tune.count(key);
        tb = &c->tune[key];
        if (fresh) tb->ncand = c->copy_nt_fixed ? kTuneGrid : kTuneCands;
        c->tune_last_key = key;
        cand = tb->done ? -1 : tb->next;  // the call's slot; candidate cand % ncand
        const tune_cand &tc = kTune[tb->done ? tb->choice : cand % tb->ncand];
        c->algorithm = tc.algorithm;
        c->max_blocks = tc.blocks;
        pp = params_of(c);
        if (tb->ncand == kTuneCands) pp.copy_nt = tc.nt;
        if (cand >= 0) {
            for (int k = 0; k < 2; ++k)
                if (!tb->ev[2 * cand + k])
                    TRY(record_hip(hipEventCreate(&tb->ev[2 * cand + k]), "autotune event"));
            // a device barrier first, so the timed region starts with every
            // rank present: host skew between the ranks' calls is not
            // charged to the candidate (every rank makes this call)
            TRY(set_dev(c));
            TRY(launch_barrier(c, s));
            TRY(record_hip(hipEventRecord(tb->ev[2 * cand], s), "autotune event"));
        }
    }
    int rc = allreduce_impl(c, sbuf, rbuf, count, type, op, s, pp);
    c->algorithm = save_alg;
    c->max_blocks = save_blocks;
    if (cand >= 0) {
        if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipEventRecord(tb->ev[2 * cand + 1], s), "autotune event");
        if (++tb->next == tb->ncand * kTuneRounds) {  // every rank is at this call: decide together
            float mine[kTuneCands], all[kMaxRanks][kTuneCands];
            for (int k = 0; k < kTuneCands; ++k) mine[k] = 1e30f;
            for (int call = 0; call < tb->ncand * kTuneRounds; ++call) {
                float ms = 1e30f;
                if (rc == OMPI_AMD_SUCCESS && hipEventSynchronize(tb->ev[2 * call + 1]) == hipSuccess &&
                    hipEventElapsedTime(&ms, tb->ev[2 * call], tb->ev[2 * call + 1]) != hipSuccess)
                    ms = 1e30f;
                (void)hipGetLastError();
                mine[call % tb->ncand] = std::min(mine[call % tb->ncand], ms);
            }
            const int arc = comm_allgather(c, mine, all, sizeof(mine));
            if (rc == OMPI_AMD_SUCCESS) rc = arc;
            int best = 0;
            for (int k = 0; k < tb->ncand; ++k) {
                float w = 0.f;
                for (int p = 0; p < c->size; ++p) w = std::max(w, arc == OMPI_AMD_SUCCESS ? all[p][k] : 0.f);
                tb->worst_ms[k] = w;
                if (w < tb->worst_ms[best]) best = k;
            }
            tb->choice = arc == OMPI_AMD_SUCCESS ? best : 0;  // a failed rendezvous fails every rank
            tb->done = true;
            for (auto &e : tb->ev)
                if (e) {
                    hip_ignore(hipEventDestroy(e));
                    e = nullptr;
                }
        }
    }
    if (tb) c->tune_last = tb->done ? 2 : 1;
    return rc;
}

int ompi_amd_iallreduce(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                        int op, void *stream, ompi_amd_request_t **out) {
    api_guard api_(c);
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(set_dev(c));
    auto *req = new (std::nothrow) ompi_amd_request;
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    req->c = c;
    req->mark = mark_word_get();
    int rc = record_hip(req_event_get(c, &req->ev), "request event");
    if (rc != OMPI_AMD_SUCCESS) {
        delete req;
        return rc;
    }
    path_params pp = params_of(c);
    nb_tuned(c, &pp, count, type);
    const bool inplace = in_place(sbuf, rbuf);
    if (pp.tuned_alg == TUNED_AR_NONOVERLAPPING) {  // a host exchange, in order with the others
        rc = drain(c);
        if (rc == OMPI_AMD_SUCCESS) rc = agree_root0_inplace(c, &pp, inplace);
        if (rc != OMPI_AMD_SUCCESS) {
            req_event_put(req->c, req->ev);
            delete req;
            return rc;
        }
    }
    pending_op o{0, inplace ? rbuf : sbuf, rbuf, count, type, op, comm_stream(c, stream), pp, req};
    if (allreduce_push_gathers(c, pp, count, type)) {
        // no swap: only the landing buffer must be big enough at the launch
        // (a growth queued ahead of this call: nb_grow)
        rc = nb_grow(c, staged_push_landing(c->size, pp.algorithm, (int64_t)count, type, nullptr), o.stream);
        if (rc != OMPI_AMD_SUCCESS) {
            req_event_put(req->c, req->ev);
            delete req;
            return rc;
        }
    } else if (allreduce_swaps(c, pp, count, type)) {
        // post this rank's half of the handle swap now; the launch waits for
        // the peers' halves (progress / the next collective call)
        const bool push = is_push(pp.algorithm);
        if (push) rc = nb_grow(c, push_slot((int64_t)count, c->size, type) * (size_t)c->size, o.stream);
        // export fallback with memory of its own (several calls may be
        // outstanding): the posted descriptors are the shadows'
        const size_t bytes = count * ompi_amd_type_extent(type);
        if (rc == OMPI_AMD_SUCCESS) {
            const void *xs = push ? nullptr : o.sbuf;
            void *xr = o.rbuf;
            rc = push ? shadow_plan(c, &xs, 0, &xr, bytes, false, true, &o.sh)
                      : shadow_plan(c, &xs, bytes, &xr, bytes, inplace, true, &o.sh);
            if (!push) o.sbuf = xs;
            o.rbuf = xr;
            req->shadow = o.sh.mem;
            req->shadow2 = o.sh.mem2;
        }
        call_blob mine{};
        if (rc == OMPI_AMD_SUCCESS && !push) rc = export_buf(c, o.sbuf, &mine.s);
        if (rc == OMPI_AMD_SUCCESS) rc = export_buf(c, o.rbuf, &mine.r);
        if (rc == OMPI_AMD_SUCCESS) rc = nb_ticket(c, o, &mine, sizeof(mine));
        if (rc != OMPI_AMD_SUCCESS) {
            req_event_put(req->c, req->ev);
            arena_free(c, req->shadow);
            arena_free(c, req->shadow2);
            delete req;
            return rc;
        }
    }
    c->pending.push_back(o);
    c->npending.fetch_add(1);
    *out = req;
    return post_progress(c);
}

// ---- nonblocking reduce_scatter_block / allgather / bcast ----
// The iallreduce machinery (post now, launch from progress in posting
// order): a staged size is enqueued at once; a zero-copy size posts this
// rank's descriptor of what peers read (`exp`, `bytes`; an owned shadow
// when the runtime refuses the export, or when `force` asks for one) and
// launches once every peer has posted.
static int nb_begin(ompi_amd_comm_t *c, ompi_amd_request **out) {
    *out = nullptr;
    TRY(check_sticky(c));
    TRY(set_dev(c));
    auto *req = new (std::nothrow) ompi_amd_request;
    if (!req) return OMPI_AMD_ERR_BAD_PARAM;
    req->c = c;
    req->mark = mark_word_get();
    const int rc = record_hip(req_event_get(c, &req->ev), "request event");
    if (rc != OMPI_AMD_SUCCESS) {
        delete req;
        return rc;
    }
    *out = req;
    return OMPI_AMD_SUCCESS;
}

static int nb_post(ompi_amd_comm_t *c, pending_op &o, const void **exp, size_t bytes, bool force,
                   ompi_amd_request_t **out) {
    int rc = OMPI_AMD_SUCCESS;
    ompi_amd_request *req = o.req;
    if (exp) {
        void *none = nullptr;
        const int saved = c->force_shadow;
        if (force) c->force_shadow = 1;
        if (rc == OMPI_AMD_SUCCESS) rc = shadow_plan(c, exp, bytes, &none, 0, false, true, &o.sh);
        c->force_shadow = saved;
        req->shadow = o.sh.mem;
        req->shadow2 = o.sh.mem2;
        call_blob mine{};
        if (rc == OMPI_AMD_SUCCESS) rc = export_buf(c, *exp, &mine.s);
        if (rc == OMPI_AMD_SUCCESS) rc = nb_ticket(c, o, &mine, sizeof(mine));
    }
    if (rc != OMPI_AMD_SUCCESS) {
        req_event_put(req->c, req->ev);
        arena_free(c, req->shadow);
        arena_free(c, req->shadow2);
        delete req;
        return rc;
    }
    c->pending.push_back(o);
    c->npending.fetch_add(1);
    *out = req;
    return post_progress(c);
}

static bool nb_swaps(const ompi_amd_comm_t *c, size_t bytes) {
    return c->size > 1 && bytes > 0 && bytes > c->small_bytes && c->zero_copy;
}

// A deferred call's landing buffer grown at post time (growth is collective
// and blocking: every rank posts the same call alike); on failure the
// request is released.
static int nb_grow_landing(ompi_amd_comm_t *c, size_t need, ompi_amd_request *req, hipStream_t s) {
    const int rc = nb_grow(c, need, s);
    if (rc != OMPI_AMD_SUCCESS) {
        req_event_put(req->c, req->ev);
        delete req;
    }
    return rc;
}

int ompi_amd_ireduce_scatter_block(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t rcount,
                                   int type, int op, void *stream, ompi_amd_request_t **out) {
    api_guard api_(c);
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    ompi_amd_request *req = nullptr;
    TRY(nb_begin(c, &req));
    const bool inplace = in_place(sbuf, rbuf);
    const size_t total = rcount * (size_t)c->size * ompi_amd_type_extent(type);
    pending_op o{0, inplace ? rbuf : sbuf, rbuf, rcount, type, op, comm_stream(c, stream), params_of(c), req};
    o.kind = PEND_RSB;
    const bool swap = nb_swaps(c, total);
    if (swap && !c->user_ipc && !c->force_shadow) {
        // staged push (reduce_my_block): no swap, so no host rendezvous at
        // launch; only the landing buffer must be big enough beforehand
        // (its growth is collective: every rank posts this call alike)
        const size_t slot = (rcount * ompi_amd_type_extent(type) + 16 + 255) & ~(size_t)255;
        TRY(nb_grow_landing(c, slot * (size_t)(c->size + 1), req, o.stream));
        o.inplace = inplace;
        return nb_post(c, o, nullptr, 0, false, out);
    }
    // in place at a zero-copy size: peers read this rank's input from an
    // owned shadow, so the result can go straight into rbuf (no landing)
    return nb_post(c, o, swap ? &o.sbuf : nullptr, total, inplace, out);
}

int ompi_amd_iallgather(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                        void *stream, ompi_amd_request_t **out) {
    api_guard api_(c);
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    ompi_amd_request *req = nullptr;
    TRY(nb_begin(c, &req));
    char *my_slot = (char *)rbuf + (size_t)c->rank * bytes;
    const bool inplace = sbuf == (const void *)1 || sbuf == (const void *)my_slot;
    pending_op o{0, inplace ? (const void *)my_slot : sbuf, rbuf, bytes, 0, 0, comm_stream(c, stream),
                 params_of(c), req};
    o.kind = PEND_ALLGATHER;
    // in place: keep the (void *)1 spelling unless peers read a shadow
    if (inplace) o.sbuf = (const void *)1;
    if (!nb_swaps(c, bytes)) return nb_post(c, o, nullptr, 0, false, out);
    if (const size_t need = ag_landing_need(c, bytes)) {
        TRY(nb_grow_landing(c, need, req, o.stream));
        o.land = true;  // stores into the peers' landing buffers: nothing to post
        return nb_post(c, o, nullptr, 0, false, out);
    }
    o.sbuf = inplace ? (const void *)my_slot : sbuf;
    return nb_post(c, o, &o.sbuf, bytes, false, out);
}

int ompi_amd_ibcast(ompi_amd_comm_t *c, void *buf, size_t bytes, int root, void *stream,
                    ompi_amd_request_t **out) {
    api_guard api_(c);
    if (!c || !buf || !out || root < 0 || root >= c->size) return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    ompi_amd_request *req = nullptr;
    TRY(nb_begin(c, &req));
    pending_op o{0, buf, buf, bytes, 0, 0, comm_stream(c, stream), params_of(c), req};
    o.kind = PEND_BCAST;
    o.root = root;
    if (nb_swaps(c, bytes)) {
        if (const size_t need = bcast_landing_need(c, bytes)) {
            TRY(nb_grow_landing(c, need, req, o.stream));
            o.land = true;  // stores into the peers' landing buffers: nothing to post
            return nb_post(c, o, nullptr, 0, false, out);
        }
    }
    if (!nb_swaps(c, bytes) || c->rank != root) {
        // non-roots export nothing, but post their (empty) half all the same
        if (!nb_swaps(c, bytes)) return nb_post(c, o, nullptr, 0, false, out);
        const void *nothing = nullptr;
        return nb_post(c, o, &nothing, 0, false, out);
    }
    return nb_post(c, o, &o.sbuf, bytes, false, out);
}

// ---- nonblocking reduce / scan / exscan / reduce_scatter ----
// They post no buffer descriptors and launch (in posting order, from
// progress) on the staged or landing paths, which need no handle swap; the
// landing buffer is grown at post time when a zero-copy size needs it
// (collective and blocking, as for iallreduce: every rank posts alike).
// ireduce posts one ticket carrying the root's MPI_IN_PLACE flag (it
// changes the root's first combine, coll_base_reduce.c:170-171), so no
// rank waits for a peer at post time.

int ompi_amd_ireduce(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                     int op, int root, void *stream, ompi_amd_request_t **out) {
    api_guard api_(c);
    if (!c || !out || root < 0 || root >= c->size || (c->rank == root && !rbuf))
        return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    ompi_amd_request *req = nullptr;
    TRY(nb_begin(c, &req));
    const int n = c->size;
    const size_t bytes = count * ompi_amd_type_extent(type);
    pending_op o{0, sbuf, rbuf, count, type, op, comm_stream(c, stream), params_of(c), req};
    o.kind = PEND_REDUCE;
    o.root = root;
    if (n > 1 && count > 0 && bytes > c->small_bytes && c->zero_copy) {
        int64_t split, early, late;
        blockcount((int64_t)count, n, &split, &early, &late);
        const size_t slot = ((size_t)early * ompi_amd_type_extent(type) + 16 + 255) & ~(size_t)255;
        TRY(nb_grow_landing(c, slot * (size_t)n + ((bytes + 255) & ~(size_t)255), req, o.stream));
    }
    if (n == 1 || count == 0) return nb_post(c, o, nullptr, 0, false, out);
    call_blob mine{};
    mine.flags = (c->rank == root && in_place(sbuf, rbuf)) ? 1 : 0;
    const int rc = nb_ticket(c, o, &mine, sizeof(mine));
    if (rc != OMPI_AMD_SUCCESS) {
        req_event_put(req->c, req->ev);
        delete req;
        return rc;
    }
    c->pending.push_back(o);
    c->npending.fetch_add(1);
    *out = req;
    return post_progress(c);
}

static int iscan_common(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                        int op, void *stream, bool exclusive, ompi_amd_request_t **out) {
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    ompi_amd_request *req = nullptr;
    TRY(nb_begin(c, &req));
    const size_t bytes = count * ompi_amd_type_extent(type);
    pending_op o{0, sbuf, rbuf, count, type, op, comm_stream(c, stream), params_of(c), req};
    o.kind = PEND_SCAN;
    o.exclusive = exclusive;
    if (c->size > 1 && count > 0 && bytes > c->small_bytes && c->zero_copy)
        TRY(nb_grow_landing(c, bytes + 256, req, o.stream));
    return nb_post(c, o, nullptr, 0, false, out);
}

int ompi_amd_iscan(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                   int op, void *stream, ompi_amd_request_t **out) {
    api_guard api_(c);
    return iscan_common(c, sbuf, rbuf, count, type, op, stream, false, out);
}

int ompi_amd_iexscan(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                     int op, void *stream, ompi_amd_request_t **out) {
    api_guard api_(c);
    return iscan_common(c, sbuf, rbuf, count, type, op, stream, true, out);
}

int ompi_amd_ireduce_scatter(ompi_amd_comm_t *c, const void *sbuf, void *rbuf,
                             const size_t *rcounts, int type, int op, void *stream,
                             ompi_amd_request_t **out) {
    api_guard api_(c);
    if (!c || !rbuf || !rcounts || !out) return OMPI_AMD_ERR_BAD_PARAM;
    *out = nullptr;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    ompi_amd_request *req = nullptr;
    TRY(nb_begin(c, &req));
    const size_t ext = ompi_amd_type_extent(type);
    pending_op o{0, sbuf, rbuf, 0, type, op, comm_stream(c, stream), params_of(c), req};
    o.kind = PEND_RS;
    o.rcounts.assign(rcounts, rcounts + c->size);
    size_t total = 0, maxc = 0;
    for (size_t v : o.rcounts) {
        total += v;
        maxc = std::max(maxc, v);
    }
    if (c->size > 1 && total * ext > c->small_bytes && c->zero_copy) {  // reduce_my_block's staged push
        const size_t slot = (maxc * ext + 16 + 255) & ~(size_t)255;
        TRY(nb_grow_landing(c, slot * (size_t)(c->size + 1), req, o.stream));
    }
    return nb_post(c, o, nullptr, 0, false, out);
}

int ompi_amd_reduce(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                    int op, int root, void *stream) {
    api_guard api_(c);
    if (!c || root < 0 || root >= c->size || (c->rank == root && !rbuf))
        return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    if (count == 0) return OMPI_AMD_SUCCESS;
    // the in-place flag only changes the root's first combine; every rank
    // must fold the same expression, so the root's choice is made known
    const bool root_inplace = c->rank == root && in_place(sbuf, rbuf);
    int flag = root_inplace ? 1 : 0, flags_all[kMaxRanks];
    if (c->size > 1) TRY(c->boot.allgather(&flag, flags_all, sizeof(int)));
    return reduce_impl(c, sbuf, rbuf, count, type, op, root, c->size > 1 ? flags_all[root] != 0 : root_inplace,
                       comm_stream(c, stream));
}

// root_inplace_all: whether the root passed MPI_IN_PLACE (known to every rank)
static int reduce_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                       int op, int root, bool root_inplace_all, hipStream_t s) {
    if (count == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    const int n = c->size;
    const size_t bytes = count * ompi_amd_type_extent(type);
    const bool root_inplace = c->rank == root && in_place(sbuf, rbuf);
    const void *src = root_inplace ? rbuf : sbuf;
    if (!src) return OMPI_AMD_ERR_BAD_PARAM;
    if (n == 1) {
        if (root_inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, bytes, hipMemcpyDeviceToDevice, s), "copy");
    }
    const red_order ro = tuned_reduce_order(n, type_size(type) * count, count, root, root_inplace_all,
                                            c->tuned_red_alg);
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
    int64_t split, early, late;
    blockcount((int64_t)count, n, &split, &early, &late);
    if (!c->user_ipc && !c->force_shadow) {
        // Staged push (nothing of the caller's exported, no staging copy on
        // the non-roots): block b of my input into slot [me] of rank b's
        // landing buffer, barrier, rank b folds block b locally and stores
        // it into the root's landing result area, barrier, the root copies
        // the result into rbuf, barrier (the next landing call's scatter
        // may land where this result area was).
        const int64_t ext = (int64_t)ompi_amd_type_extent(type);
        const size_t slot = ((size_t)early * (size_t)ext + 16 + 255) & ~(size_t)255;
        const size_t res_off = slot * (size_t)n;
        TRY(ensure_landing(c, res_off + ((bytes + 255) & ~(size_t)255)));
        cp_jobs cj{};
        for (int b = 0; b < n; ++b) {
            const int64_t off = block_off(b, split, early, late) * ext, cb = block_cnt(b, split, early, late);
            if (b == c->rank || cb == 0) continue;
            char *dst = const_cast<char *>(c->peer_land.p[b]) + (size_t)c->rank * slot + (off & 15);
            cj.j[cj.n++] = {(const char *)src + off, dst, cb * ext};
        }
        TRY(launch_copy(c, cj, s));
        TRY(launch_barrier(c, s));
        const int64_t offm = block_off(c->rank, split, early, late) * ext;
        ptr_set srcs{};
        for (int r = 0; r < n; ++r)
            srcs.p[r] = (r == c->rank) ? (const char *)src
                                       : c->land + (size_t)r * slot + (offm & 15) - offm;
        jobs.n = 1;
        jobs.j[0].off = block_off(c->rank, split, early, late);
        jobs.j[0].cnt = block_cnt(c->rank, split, early, late);
        jobs.j[0].off_dst = jobs.j[0].off;
        jobs.j[0].first = ro.first;
        jobs.j[0].head = -1;
        const char *res = c->peer_land.p[root] + res_off;  // my own landing when I am the root
        if (jobs.j[0].cnt > 0)
            TRY(timed_phase(c, 0, s, [&] {
                return launch_reduce(c, op, type, srcs, n, one_ptr(res), 1, ro.order, ro.flags, jobs, s);
            }));
        TRY(launch_barrier(c, s));
        if (c->rank == root) {
            cj = cp_jobs{};
            cj.n = 1;
            cj.j[0] = {c->land + res_off, (char *)rbuf, (int64_t)bytes};
            TRY(launch_copy(c, cj, s));
        }
        return launch_barrier(c, s);
    }
    // zero-copy: every rank folds one block of the vector from every
    // rank's sbuf and stores it straight into the root's rbuf
    ptr_set sp{}, rp{};
    void *xr = c->rank == root ? rbuf : nullptr;
    shadow_set sh;  // peers read src and write the root's rbuf
    TRY(shadow_plan(c, &src, bytes, &xr, c->rank == root ? bytes : 0, root_inplace, false, &sh));
    TRY(shadow_in(c, sh, s));
    TRY(exchange_bufs(c, src, xr, &sp, &rp));
    TRY(launch_barrier(c, s));
    jobs.n = 1;
    jobs.j[0].off = block_off(c->rank, split, early, late);
    jobs.j[0].cnt = block_cnt(c->rank, split, early, late);
    jobs.j[0].off_dst = jobs.j[0].off;
    jobs.j[0].first = ro.first;
    jobs.j[0].head = -1;
    TRY(timed_phase(c, 0, s, [&] {
        return launch_reduce(c, op, type, sp, n, one_ptr(rp.p[root]), 1, ro.order, ro.flags, jobs, s);
    }));
    TRY(launch_barrier(c, s));
    return shadow_out(c, sh, s);
}

int ompi_amd_reduce_scatter_block(ompi_amd_comm_t *c, const void *sbuf, void *rbuf,
                                  size_t rcount, int type, int op, void *stream) {
    api_guard api_(c);
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    const bool inplace = in_place(sbuf, rbuf);
    return rsb_impl(c, inplace ? rbuf : sbuf, rbuf, rcount, type, op, inplace, comm_stream(c, stream));
}

// src: the input (rbuf itself in place, n * rcount elements)
static int rsb_impl(ompi_amd_comm_t *c, const void *src, void *rbuf, size_t rcount, int type,
                    int op, bool inplace, hipStream_t s) {
    if (rcount == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    const int n = c->size;
    const size_t ext = ompi_amd_type_extent(type);
    const size_t total = rcount * (size_t)n * ext;
    if (n == 1) {
        if (inplace || src == rbuf) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, rcount * ext, hipMemcpyDeviceToDevice, s), "copy");
    }
    // basic_linear rsb = tuned reduce of the whole vector to rank 0 (never
    // in place at that level) + scatter: my block folds in that order
    const size_t tcount = rcount * (size_t)n;
    const red_order ro = tuned_reduce_order(n, type_size(type) * tcount, tcount, 0, false, c->tuned_red_alg);
    return reduce_my_block(c, src, rbuf, total, (int64_t)(rcount * (size_t)c->rank),
                           (int64_t)rcount, (int64_t)rcount, op, type, ro, inplace, s);
}

// coll/tuned's reduce_scatter decision (coll_tuned_decision_fixed.c:
// 466-512, commutative): recursive halving for small totals or
// power-of-two sizes up to 256 KiB, else the ring.
// forced (coll_tuned_reduce_scatter_algorithm, :135-145): 2 recursive
// halving, 3 ring; 1 non-overlapping is a tuned reduce of the whole vector
// to rank 0 + scatterv (coll_base_reduce_scatter.c:42-92), rank 0 in place
// exactly when every rank is; rs_impl builds that one.
static red_order tuned_reduce_scatter_order(int n, size_t total_bytes, int block, int forced = 0) {
    int pow2 = 1;
    while (pow2 < n) pow2 <<= 1;
    const bool halving = forced == TUNED_RS_HALVING ||
        (forced != TUNED_RS_RING &&
         (total_bytes <= 12 * 1024 || (total_bytes <= 256 * 1024 && pow2 == n) ||
          (double)n >= 0.0012 * (double)total_bytes + 8.0));
    if (halving) {
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
    api_guard api_(c);
    if (!c || !rbuf || !rcounts) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(check_sticky(c));
    TRY(drain(c));
    return rs_impl(c, sbuf, rbuf, rcounts, type, op, comm_stream(c, stream));
}

static int rs_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, const size_t *rcounts,
                   int type, int op, hipStream_t s) {
    const int n = c->size;
    size_t total = 0, off = 0, maxc = 0;
    for (int p = 0; p < n; ++p) {
        if (p < c->rank) off += rcounts[p];
        total += rcounts[p];
        maxc = std::max(maxc, rcounts[p]);
    }
    if (total == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    const size_t ext = ompi_amd_type_extent(type);
    const bool inplace = in_place(sbuf, rbuf);
    const void *src = inplace ? rbuf : sbuf;
    if (n == 1) {
        if (inplace) return OMPI_AMD_SUCCESS;
        return record_hip(hipMemcpyAsync(rbuf, src, rcounts[0] * ext, hipMemcpyDeviceToDevice, s),
                          "copy");
    }
    const red_order ro = c->tuned_rs_alg == TUNED_RS_NONOVERLAPPING
                             ? tuned_reduce_order(n, type_size(type) * total, total, 0, inplace, c->tuned_red_alg)
                             : tuned_reduce_scatter_order(n, total * type_size(type), c->rank, c->tuned_rs_alg);
    return reduce_my_block(c, src, rbuf, total * ext, (int64_t)off, (int64_t)rcounts[c->rank],
                           (int64_t)maxc, op, type, ro, inplace, s, rcounts);
}

int ompi_amd_scan(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                  int op, void *stream) {
    api_guard api_(c);
    if (c) TRY(drain(c));
    return scan_common(c, sbuf, rbuf, count, type, op, stream, false);
}

int ompi_amd_exscan(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                    int op, void *stream) {
    api_guard api_(c);
    if (c) TRY(drain(c));
    return scan_common(c, sbuf, rbuf, count, type, op, stream, true);
}

int ompi_amd_allgather(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                       void *stream) {
    api_guard api_(c);
    if (!c || !rbuf) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(check_sticky(c));
    TRY(drain(c));
    if (c->land_blocking && ag_landing_need(c, bytes))  // grown here: collective, every rank alike
        return allgather_land(c, sbuf, rbuf, bytes, comm_stream(c, stream));
    return allgather_impl(c, sbuf, rbuf, bytes, comm_stream(c, stream));
}

static int allgather_impl(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                          hipStream_t s) {
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
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
    const void *mine = inplace ? my_slot : sbuf;
    void *none = nullptr;
    shadow_set sh;
    if (!c->pre) TRY(shadow_plan(c, &mine, bytes, &none, 0, false, false, &sh));
    TRY(shadow_in(c, sh, s));
    TRY(exchange_bufs(c, mine, nullptr, &sp, &rp));
    TRY(launch_barrier(c, s));
    for (int p = 0; p < n; ++p) {
        if (p == c->rank && inplace) continue;
        cj.j[cj.n++] = {sp.p[p], (char *)rbuf + (size_t)p * bytes, (int64_t)bytes};
    }
    TRY(launch_copy(c, cj, s));
    return launch_barrier(c, s);
}

int ompi_amd_bcast(ompi_amd_comm_t *c, void *buf, size_t bytes, int root, void *stream) {
    api_guard api_(c);
    if (!c || !buf || root < 0 || root >= c->size) return OMPI_AMD_ERR_BAD_PARAM;
    TRY(check_sticky(c));
    TRY(drain(c));
    if (c->land_blocking && bcast_landing_need(c, bytes))
        return bcast_land(c, buf, bytes, root, comm_stream(c, stream));
    return bcast_impl(c, buf, buf, bytes, root, comm_stream(c, stream));
}

// root_src: what the root's peers read (buf, or a deferred call's shadow)
static int bcast_impl(ompi_amd_comm_t *c, void *buf, const void *root_src, size_t bytes, int root,
                      hipStream_t s) {
    if (bytes == 0 || c->size == 1) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
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
    // Large: scatter + allgather (the data flow of coll_base_bcast.c:768's
    // scatter_allgather, one hop per phase on the fully connected xGMI
    // mesh): rank r copies block r from the root, barrier, then block b from
    // rank b for every other b.  Every link carries about 2·bytes/N instead
    // of each of the root's links carrying `bytes`.  What peers read is
    // every rank's buffer itself (user_ipc, when every export succeeds) or
    // every rank's communicator shadow (the root copies its buffer in; rank
    // r keeps block r there too); a blocking call only, else the root-pull.
    if (!c->pre && c->bcast_split_bytes > 0 && bytes >= c->bcast_split_bytes) {
        bool every = false;
        char *mine_sh = nullptr;  // staged: this rank's shadow (buf's phase mod 256)
        if (c->user_ipc) {
            call_blob me{}, all[kMaxRanks];
            bool refused = false;
            if (export_buf(c, buf, &me.s, &refused) != OMPI_AMD_SUCCESS) me.s = buf_desc{};
            TRY(c->boot.allgather(&me, all, sizeof(call_blob)));
            every = true;
            for (int p = 0; p < c->size; ++p) every = every && all[p].s.valid;
            if (every) TRY(import_all(c, all, buf, nullptr, &sp, &rp, nullptr, false, nullptr));
        } else {
            char *base = nullptr;
            TRY(shadow_reserve(c, bytes + 256, &base));
            mine_sh = base + ((uintptr_t)buf & 255);
            if (c->rank == root) {
                cj.n = 1;
                cj.j[0] = {(const char *)buf, mine_sh, (int64_t)bytes};
                TRY(launch_copy(c, cj, s));
            }
            TRY(exchange_bufs(c, mine_sh, nullptr, &sp, &rp));
            every = true;
        }
        if (every) {
            const int n = c->size;
            const size_t blk = ((bytes + (size_t)n - 1) / (size_t)n + 255) & ~(size_t)255;
            auto block = [&](int b, size_t *off, size_t *len) {
                *off = std::min(bytes, (size_t)b * blk);
                *len = std::min(bytes, *off + blk) - *off;
            };
            TRY(launch_barrier(c, s));  // the root's data is final
            size_t off, len;
            block(c->rank, &off, &len);
            if (c->rank != root && len) {
                cj.n = 0;
                cj.j[cj.n++] = {sp.p[root] + off, (char *)buf + off, (int64_t)len};
                if (mine_sh) cj.j[cj.n++] = {sp.p[root] + off, mine_sh + off, (int64_t)len};
                TRY(launch_copy(c, cj, s));
            }
            TRY(launch_barrier(c, s));  // every block is at its owner
            if (c->rank != root) {
                cj.n = 0;
                for (int b = 0; b < n; ++b) {
                    block(b, &off, &len);
                    if (b == c->rank || !len) continue;
                    cj.j[cj.n++] = {sp.p[b] + off, (char *)buf + off, (int64_t)len};
                }
                TRY(launch_copy(c, cj, s));
            }
            ++c->bcast_split;
            return launch_barrier(c, s);
        }
        // someone's export was refused: the root-pull path, with its own swap
    }
    const void *mine = c->rank == root ? root_src : nullptr;
    void *none = nullptr;
    shadow_set sh;
    if (!c->pre) TRY(shadow_plan(c, &mine, bytes, &none, 0, false, false, &sh));
    TRY(shadow_in(c, sh, s));
    TRY(exchange_bufs(c, mine, nullptr, &sp, &rp));
    TRY(launch_barrier(c, s));
    if (c->rank != root) {
        cj.n = 1;
        cj.j[0] = {sp.p[root], (char *)buf, (int64_t)bytes};
        TRY(launch_copy(c, cj, s));
    }
    return launch_barrier(c, s);
}

// ---- allgather / bcast through the landing buffers (deferred calls) ----
// Nonblocking and persistent allgathers and bcasts of a zero-copy size in
// the staged mode move their data by remote STORES into the peers' landing
// buffers (library memory, mapped once), so they post no buffer descriptor:
// no host rendezvous at post or at launch, the same as the push-gather
// allreduce.  Landing layout: the allgather puts rank p's block in slot p;
// the bcast mirrors the buffer (offset o of the buffer at offset o).  Data
// sits at the phase mod 16 the receiver's rbuf offset has when rbuf itself
// is 16-B aligned (the copies stay 16-B vectors for aligned buffers).
// Every landing call ends with a barrier (the next landing call of any
// collective may store into these bytes without a leading one).
static size_t ag_land_slot(size_t bytes) { return (bytes + 16 + 255) & ~(size_t)255; }

// Landing bytes a deferred allgather (bcast) needs, or 0 when it does not
// take the landing path (user_ipc / force_shadow, a staged size, or past
// the IPC size limit); every rank computes the same for the same call.
static size_t ag_landing_need(const ompi_amd_comm_t *c, size_t bytes) {
    if (c->user_ipc || c->force_shadow || c->size == 1 || bytes <= c->small_bytes || !c->zero_copy)
        return 0;
    const size_t need = ag_land_slot(bytes) * (size_t)c->size;
    return need + (64u << 20) <= kMaxIpcBytes ? need : 0;
}
static size_t bcast_landing_need(const ompi_amd_comm_t *c, size_t bytes) {
    if (c->user_ipc || c->force_shadow || c->size == 1 || bytes <= c->small_bytes || !c->zero_copy)
        return 0;
    const size_t need = ((bytes + 255) & ~(size_t)255) + 256;
    return need + (64u << 20) <= kMaxIpcBytes ? need : 0;
}

// Store my block into slot [me] of every peer's landing buffer (local rbuf
// first, then peers rank+1, rank+2, ... so concurrent ranks spread over the
// links), barrier, copy the peers' slots of my landing buffer into rbuf,
// barrier.  xGMI bytes as the pull ((N-1)·B out and in per rank); the price
// is one local copy of (N-1)·B.
static int allgather_land(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                          hipStream_t s) {
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    const int n = c->size;
    const size_t slot = ag_land_slot(bytes);
    TRY(ensure_landing(c, slot * (size_t)n));  // grown at post time: a no-op here
    ++c->land_ag_bcast;
    char *my_slot = (char *)rbuf + (size_t)c->rank * bytes;
    const bool inplace = sbuf == (const void *)1 || sbuf == (const void *)my_slot;
    const char *mine = inplace ? my_slot : (const char *)sbuf;
    const size_t ph_me = ((size_t)c->rank * bytes) & 15;
    cp_jobs cj{};
    if (!inplace) cj.j[cj.n++] = {mine, my_slot, (int64_t)bytes};
    for (int k = 1; k < n; ++k) {
        const int q = (c->rank + k) % n;
        cj.j[cj.n++] = {mine, const_cast<char *>(c->peer_land.p[q]) + (size_t)c->rank * slot + ph_me,
                        (int64_t)bytes};
    }
    TRY(launch_copy(c, cj, s));
    TRY(launch_barrier(c, s));
    cj = cp_jobs{};
    for (int p = 0; p < n; ++p) {
        if (p == c->rank) continue;
        const size_t ph = ((size_t)p * bytes) & 15;
        cj.j[cj.n++] = {c->land + (size_t)p * slot + ph, (char *)rbuf + (size_t)p * bytes,
                        (int64_t)bytes};
    }
    TRY(launch_copy(c, cj, s));
    return launch_barrier(c, s);
}

// Scatter + allgather by stores (the data flow of the blocking split bcast,
// coll_base_bcast.c:768's scatter_allgather): the root stores block b into
// rank b's landing buffer and its own block into every peer's; barrier;
// every other rank stores its block from its landing buffer into every
// non-root peer's and copies it into its buffer; barrier; every non-root
// copies the other blocks from its landing buffer; barrier.  The root's
// links carry about 2·bytes/N each instead of `bytes`.
static int bcast_land(ompi_amd_comm_t *c, void *buf, size_t bytes, int root, hipStream_t s) {
    if (bytes == 0 || c->size == 1) return OMPI_AMD_SUCCESS;
    TRY(set_dev(c));
    const int n = c->size, me = c->rank;
    TRY(ensure_landing(c, ((bytes + 255) & ~(size_t)255) + 256));
    ++c->land_ag_bcast;
    const size_t blk = ((bytes + (size_t)n - 1) / (size_t)n + 255) & ~(size_t)255;
    auto block = [&](int b, size_t *off, size_t *len) {
        *off = std::min(bytes, (size_t)b * blk);
        *len = std::min(bytes, *off + blk) - *off;
    };
    size_t off, len;
    cp_jobs cj{};
    if (me == root) {
        for (int k = 1; k < n; ++k) {  // block b to its distributor b
            const int b = (me + k) % n;
            block(b, &off, &len);
            if (len) cj.j[cj.n++] = {(const char *)buf + off, const_cast<char *>(c->peer_land.p[b]) + off,
                                     (int64_t)len};
        }
        TRY(launch_copy(c, cj, s));
        cj = cp_jobs{};
        block(root, &off, &len);  // the root distributes its own block
        for (int k = 1; k < n && len; ++k) {
            const int q = (me + k) % n;
            cj.j[cj.n++] = {(const char *)buf + off, const_cast<char *>(c->peer_land.p[q]) + off,
                            (int64_t)len};
        }
        TRY(launch_copy(c, cj, s));
    }
    TRY(launch_barrier(c, s));  // block b is in rank b's landing buffer
    if (me != root) {
        block(me, &off, &len);
        if (len) {
            cj.j[cj.n++] = {c->land + off, (char *)buf + off, (int64_t)len};
            for (int k = 1; k < n; ++k) {
                const int q = (me + k) % n;
                if (q == root) continue;
                cj.j[cj.n++] = {c->land + off, const_cast<char *>(c->peer_land.p[q]) + off, (int64_t)len};
            }
        }
        TRY(launch_copy(c, cj, s));
    }
    TRY(launch_barrier(c, s));  // every block is in every non-root's landing buffer
    if (me != root) {
        cj = cp_jobs{};
        for (int b = 0; b < n; ++b) {
            block(b, &off, &len);
            if (b == me || !len) continue;
            cj.j[cj.n++] = {c->land + off, (char *)buf + off, (int64_t)len};
        }
        TRY(launch_copy(c, cj, s));
    }
    return launch_barrier(c, s);
}

int ompi_amd_allreduce_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count,
                            int type, int op, ompi_amd_plan_t **out) {
    api_guard api_(c);
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
    pl->pp = params_of(c);
    nb_tuned(c, &pl->pp, count, type);
    int rc = agree_root0_inplace(c, &pl->pp, inplace);
    if (rc != OMPI_AMD_SUCCESS) {
        delete pl;
        return rc;
    }
    // kind 0 (a start re-runs the plain call): the fused / staged sizes, and
    // the push-gather scheme at any size — it swaps no handles (library
    // landing buffers only), so a re-run has no host rendezvous once the
    // landing buffer is sized here for its n + 1 slots
    const bool push_gather = allreduce_push_gathers(c, pl->pp, count, type);
    const bool small = n == 1 || count == 0 || !allreduce_swaps(c, pl->pp, count, type) || push_gather;
    if (rc == OMPI_AMD_SUCCESS && push_gather)
        rc = ensure_landing(c, staged_push_landing(n, pl->pp.algorithm, (int64_t)count, type, nullptr));
    pl->fp = allreduce_fold(n, pl->pp.tuned_alg, count, type, pl->pp.root0_inplace != 0, pl->pp.red_alg);
    if (!small) {
        pl->kind = is_push(c->algorithm) ? 3 : c->algorithm == ALG_PULL_PUSH ? 2 : 1;
        if (pl->kind == 3) rc = ensure_landing(c, push_slot(pl->count, n, type) * (size_t)n);
        if (rc == OMPI_AMD_SUCCESS) {  // export fallback: shadows of the plan's own
            const void *xs = pl->kind == 3 ? nullptr : pl->src;
            void *xr = pl->rbuf;
            // an in-place plan that needs shadows gets two (input, result)
            // and runs as not in place: round 2 saw in-place owned shadows
            // read wrong peer data after long handle-recycling histories on a
            // shared GPU; separate shadows pass those cases
            rc = shadow_plan(c, &xs, pl->kind == 3 ? 0 : bytes, &xr, bytes, inplace, true, &pl->sh,
                             true);
            if (pl->kind != 3) pl->src = xs;
            pl->rbuf = xr;
        }
        if (rc == OMPI_AMD_SUCCESS)
            rc = exchange_bufs(c, pl->kind == 3 ? nullptr : pl->src, pl->rbuf, &pl->sp, &pl->rp, 0,
                               nullptr, true, pl->bases);
        if (pl->src == pl->rbuf) pl->sp = pl->rp;
    }
    if (rc == OMPI_AMD_SUCCESS)
        rc = record_hip(hipEventCreateWithFlags(&pl->done, hipEventDisableTiming), "plan event");
    if (rc == OMPI_AMD_SUCCESS) pl->mark = mark_word_get();
    if (rc != OMPI_AMD_SUCCESS) {
        (void)ompi_amd_plan_free(pl);
        return rc;
    }
    *out = pl;
    return OMPI_AMD_SUCCESS;
}

static int plan_enqueue(ompi_amd_plan_t *pl, void *stream) {
    ompi_amd_comm_t *c = pl->c;
    if (pl->kind == 0) {  // the small paths: a plain call with the parameters of the init
        TRY(check_sticky(c));
        TRY(drain(c));
        // a fused launch stores the plan's mark itself (its own counter slot:
        // plans of one communicator may be in flight together)
        if (pl->done_slot < 0 && pl->mark) pl->done_slot = done_slot_take(c);
        c->want_mark = pl->done_slot >= 0;
        c->mark_word = pl->mark;
        c->mark_slot = std::max(pl->done_slot, 0);
        c->mark_embedded = 0;
        const int rc = allreduce_impl(c, pl->src == pl->rbuf ? (const void *)1 : pl->src, pl->rbuf,
                                      (size_t)pl->count, pl->type, pl->op, comm_stream(c, stream), pl->pp);
        c->want_mark = false;
        pl->embedded = c->mark_embedded;
        c->mark_embedded = 0;
        return rc;
    }
    TRY(check_sticky(c));
    TRY(set_dev(c));
    hipStream_t s = comm_stream(c, stream);
    TRY(shadow_in(c, pl->sh, s));
    int rc;
    if (pl->kind == 3) {
        // another call may have grown (and so moved) the landing buffer:
        // its size only grows, so the slots still fit
        rc = allreduce_push(c, pl->src, pl->rp, pl->count, pl->op, pl->type, pl->fp, s);
    } else if (pl->kind == 2) {
        rc = allreduce_pull_push(c, pl->sp, pl->rp, pl->count, pl->op, pl->type, pl->fp, s);
    } else {
        rc = allreduce_pull(c, pl->sp, pl->rp, pl->rbuf, pl->count, pl->op, pl->type, pl->fp, s);
    }
    TRY(rc);
    return shadow_out(c, pl->sh, s);
}

int ompi_amd_plan_kind(const ompi_amd_plan_t *pl) { return pl ? pl->kind : -1; }

static int plan_nb_post(ompi_amd_plan_t *pl, void *stream) {
    ompi_amd_comm_t *c = pl->c;
    if (pl->req) {  // MPI: a start follows the completion of the previous one
        const int frc = ompi_amd_request_free(pl->req);
        pl->req = nullptr;
        TRY(frc);
    }
    switch (pl->nb_kind) {
    case PEND_RSB:
        return ompi_amd_ireduce_scatter_block(c, pl->src, pl->rbuf, (size_t)pl->count, pl->type, pl->op,
                                              stream, &pl->req);
    case PEND_ALLGATHER:
        return ompi_amd_iallgather(c, pl->src, pl->rbuf, pl->bytes, stream, &pl->req);
    case PEND_BCAST:
        return ompi_amd_ibcast(c, pl->rbuf, pl->bytes, pl->root, stream, &pl->req);
    case PEND_REDUCE:
        return ompi_amd_ireduce(c, pl->src, pl->rbuf, (size_t)pl->count, pl->type, pl->op, pl->root,
                                stream, &pl->req);
    case PEND_SCAN:
        return (pl->exclusive ? ompi_amd_iexscan : ompi_amd_iscan)(c, pl->src, pl->rbuf, (size_t)pl->count,
                                                                   pl->type, pl->op, stream, &pl->req);
    case PEND_RS:
        return ompi_amd_ireduce_scatter(c, pl->src, pl->rbuf, pl->rcounts.data(), pl->type, pl->op, stream,
                                        &pl->req);
    default:
        return OMPI_AMD_ERR_BAD_PARAM;
    }
}

static int plan_nb_new(ompi_amd_comm_t *c, int nb_kind, const void *src, void *rbuf, size_t count,
                       int type, int op, int root, size_t bytes, ompi_amd_plan_t **out) {
    *out = nullptr;
    TRY(check_sticky(c));
    auto *pl = new (std::nothrow) ompi_amd_plan;
    if (!pl) return OMPI_AMD_ERR_BAD_PARAM;
    pl->c = c;
    pl->kind = 4;
    pl->nb_kind = nb_kind;
    pl->src = src;
    pl->rbuf = rbuf;
    pl->count = (int64_t)count;
    pl->type = type;
    pl->op = op;
    pl->root = root;
    pl->bytes = bytes;
    *out = pl;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_reduce_scatter_block_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf,
                                       size_t rcount, int type, int op, ompi_amd_plan_t **out) {
    api_guard api_(c);
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    return plan_nb_new(c, PEND_RSB, sbuf, rbuf, rcount, type, op, 0, 0, out);
}

int ompi_amd_allgather_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t bytes,
                            ompi_amd_plan_t **out) {
    api_guard api_(c);
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    return plan_nb_new(c, PEND_ALLGATHER, sbuf, rbuf, 0, 0, 0, 0, bytes, out);
}

int ompi_amd_bcast_init(ompi_amd_comm_t *c, void *buf, size_t bytes, int root,
                        ompi_amd_plan_t **out) {
    api_guard api_(c);
    if (!c || !buf || !out || root < 0 || root >= c->size) return OMPI_AMD_ERR_BAD_PARAM;
    return plan_nb_new(c, PEND_BCAST, buf, buf, 0, 0, 0, root, bytes, out);
}

int ompi_amd_reduce_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                         int op, int root, ompi_amd_plan_t **out) {
    api_guard api_(c);
    if (!c || !out || root < 0 || root >= c->size || (c->rank == root && !rbuf))
        return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    return plan_nb_new(c, PEND_REDUCE, sbuf, rbuf, count, type, op, root, 0, out);
}

int ompi_amd_reduce_scatter_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf,
                                 const size_t *rcounts, int type, int op, ompi_amd_plan_t **out) {
    api_guard api_(c);
    if (!c || !rbuf || !rcounts || !out) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(plan_nb_new(c, PEND_RS, sbuf, rbuf, 0, type, op, 0, 0, out));
    (*out)->rcounts.assign(rcounts, rcounts + c->size);
    return OMPI_AMD_SUCCESS;
}

static int scan_init_common(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                            int op, bool exclusive, ompi_amd_plan_t **out) {
    if (!c || !rbuf || !out) return OMPI_AMD_ERR_BAD_PARAM;
    if (!ompi_amd_op_supported(op, type)) return OMPI_AMD_ERR_UNSUPPORTED;
    TRY(plan_nb_new(c, PEND_SCAN, sbuf, rbuf, count, type, op, 0, 0, out));
    (*out)->exclusive = exclusive;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_scan_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op,
                       ompi_amd_plan_t **out) {
    api_guard api_(c);
    return scan_init_common(c, sbuf, rbuf, count, type, op, false, out);
}

int ompi_amd_exscan_init(ompi_amd_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type,
                         int op, ompi_amd_plan_t **out) {
    api_guard api_(c);
    return scan_init_common(c, sbuf, rbuf, count, type, op, true, out);
}

int ompi_amd_plan_start(ompi_amd_plan_t *pl, void *stream) {
    api_guard api_(pl ? pl->c : nullptr);
    if (!pl || !pl->c) return OMPI_AMD_ERR_BAD_PARAM;
    if (pl->kind == 4) {  // posts a nonblocking call: never waits for a peer
        TRY(plan_nb_post(pl, stream));
        pl->started = true;
        return OMPI_AMD_SUCCESS;
    }
    TRY(drain(pl->c));  // device order: deferred nonblocking calls first
    pl->embedded = 0;
    pl->polls = 0;
    TRY(plan_enqueue(pl, stream));
    pl->started = true;
    pl->recorded = false;
    pl->stream = comm_stream(pl->c, stream);
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_plan_test(ompi_amd_plan_t *pl, int *done) {
    api_guard api_(pl ? pl->c : nullptr);
    if (!pl || !done) return OMPI_AMD_ERR_BAD_PARAM;
    *done = 1;
    if (!pl->started) return OMPI_AMD_SUCCESS;
    if (pl->kind == 4) return pl->req ? ompi_amd_request_test(pl->req, done) : OMPI_AMD_SUCCESS;
    if (pl->embedded) {  // the fused kernel's own mark; the stream backs it up now and then
        if (mark_seen(pl->mark, pl->embedded)) return check_sticky(pl->c);
        if (++pl->polls % 64 == 0) {
            const hipError_t e = hipStreamQuery(pl->stream);
            if (e == hipSuccess) return check_sticky(pl->c);
            if (e != hipErrorNotReady) return record_hip(e, "plan test");
        }
        *done = 0;
        return OMPI_AMD_SUCCESS;
    }
    if (!pl->recorded) {
        TRY(record_hip(hipEventRecord(pl->done, pl->stream), "plan completion event"));
        pl->mark_seq = mark_launch(pl->mark, pl->stream);
        pl->recorded = true;
    }
    if (mark_seen(pl->mark, pl->mark_seq)) return check_sticky(pl->c);
    const hipError_t e = hipEventQuery(pl->done);
    if (e == hipErrorNotReady) {
        *done = 0;
        return OMPI_AMD_SUCCESS;
    }
    if (e != hipSuccess) return record_hip(e, "plan test");
    return check_sticky(pl->c);
}

int ompi_amd_plan_wait(ompi_amd_plan_t *pl) {
    api_guard api_(pl ? pl->c : nullptr);
    if (!pl) return OMPI_AMD_ERR_BAD_PARAM;
    if (!pl->started) return OMPI_AMD_SUCCESS;
    if (pl->kind == 4) return pl->req ? ompi_amd_request_wait(pl->req) : OMPI_AMD_SUCCESS;
    if (pl->embedded) {
        TRY(record_hip(mark_value_wait(pl->stream, pl->mark, pl->embedded, progress_others), "plan wait"));
        return check_sticky(pl->c);
    }
    if (!pl->recorded) {
        TRY(record_hip(hipEventRecord(pl->done, pl->stream), "plan completion event"));
        pl->mark_seq = mark_launch(pl->mark, pl->stream);
        pl->recorded = true;
    }
    TRY(record_hip(wait_marked(pl->done, pl->mark, pl->mark_seq), "plan wait"));
    return check_sticky(pl->c);
}

int ompi_amd_plan_free(ompi_amd_plan_t *pl) {
    api_guard api_(pl ? pl->c : nullptr);
    if (!pl) return OMPI_AMD_SUCCESS;
    if (pl->kind == 4) {
        const int rc = pl->req ? ompi_amd_request_free(pl->req) : OMPI_AMD_SUCCESS;
        delete pl;
        return rc;
    }
    if (pl->c)
        for (int p = 0; p < OMPI_AMD_MAX_RANKS; ++p)
            for (int k = 0; k < 2; ++k)
                if (pl->bases[p][k]) unpin_import(pl->c, pl->bases[p][k]);
    if (pl->sh.mem || pl->sh.mem2) {  // the plan's last start must be over before its shadow goes
        if (pl->started && pl->done) (void)ompi_amd_plan_wait(pl);
        arena_free(pl->c, pl->sh.mem);
        arena_free(pl->c, pl->sh.mem2);
    }
    if (pl->done) hip_ignore(hipEventDestroy(pl->done));
    if (pl->c && pl->done_slot >= 0) {  // its last start was waited for (MPI_Request_free of a started plan: above)
        if (pl->started && pl->embedded) (void)ompi_amd_plan_wait(pl);
        done_slot_give(pl->c, pl->done_slot);
    }
    delete pl;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_request_test(ompi_amd_request_t *r, int *done) {
    api_guard api_(r ? r->c : nullptr);
    if (!r || !done) return OMPI_AMD_ERR_BAD_PARAM;
    *done = 0;
    if (!r->launched) {
        TRY(set_dev(r->c));
        TRY(progress(r->c, false));
        if (!r->launched) return OMPI_AMD_SUCCESS;
    }
    if (r->rc != OMPI_AMD_SUCCESS) return r->rc;
    if (r->embedded) {  // the fused kernel's own mark; the stream backs it up now and then
        if (mark_seen(r->mark, r->embedded)) {
            *done = 1;
            return check_sticky(r->c);
        }
        if (++r->polls % 64 == 0) {
            const hipError_t e = hipStreamQuery(r->stream);
            if (e != hipSuccess && e != hipErrorNotReady) return record_hip(e, "request test");
            if (e == hipSuccess) {
                *done = 1;
                return check_sticky(r->c);
            }
        }
        return OMPI_AMD_SUCCESS;
    }
    if (!r->recorded) {
        TRY(record_hip(hipEventRecord(r->ev, r->stream), "request event"));
        r->mark_seq = mark_launch(r->mark, r->stream);
        r->recorded = true;
    }
    if (mark_seen(r->mark, r->mark_seq)) {
        *done = 1;
        return check_sticky(r->c);
    }
    const hipError_t e = hipEventQuery(r->ev);
    if (e == hipErrorNotReady) return OMPI_AMD_SUCCESS;
    if (e != hipSuccess) return record_hip(e, "request test");
    *done = 1;
    return check_sticky(r->c);
}

int ompi_amd_request_wait(ompi_amd_request_t *r) {
    api_guard api_(r ? r->c : nullptr);
    if (!r) return OMPI_AMD_ERR_BAD_PARAM;
    if (!r->launched) {
        TRY(set_dev(r->c));
        TRY(progress(r->c, true));
    }
    if (r->rc != OMPI_AMD_SUCCESS) return r->rc;
    if (r->embedded) {
        TRY(record_hip(mark_value_wait(r->stream, r->mark, r->embedded, progress_others), "request wait"));
        return check_sticky(r->c);
    }
    if (!r->recorded) {
        TRY(record_hip(hipEventRecord(r->ev, r->stream), "request event"));
        r->mark_seq = mark_launch(r->mark, r->stream);
        r->recorded = true;
    }
    TRY(record_hip(wait_marked(r->ev, r->mark, r->mark_seq), "request wait"));
    return check_sticky(r->c);
}

int ompi_amd_request_free(ompi_amd_request_t *r) {
    api_guard api_(r ? r->c : nullptr);
    if (!r) return OMPI_AMD_SUCCESS;
    // the peers launch it whatever this rank does: launch and finish it too
    const int rc = ompi_amd_request_wait(r);
    req_event_put(r->c, r->ev);  // its wait is over
    done_slot_give(r->c, r->done_slot);  // its kernel finished (the wait above)
    // the call's trailing barrier has passed: no peer reads the shadow any more
    arena_free(r->c, r->shadow);
    arena_free(r->c, r->shadow2);
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

void *comm_osc_state(ompi_amd_comm_t *c) { return c->osc_state; }

void comm_set_osc_state(ompi_amd_comm_t *c, void *state, void (*release)(void *, int)) {
    c->osc_state = state;
    c->osc_release = release;
}

int comm_allgather(ompi_amd_comm_t *c, const void *mine, void *all, size_t len) {
    return c->boot.allgather(mine, all, len);
}

void comm_release_exportable(void *p) { release_exportable(p); }

int comm_alloc_exportable(size_t bytes, bool uncached, void **out, ipc_desc *d) {
    memset(d, 0, sizeof(*d));
    char *p = nullptr;
    const hipError_t e = alloc_exportable(bytes, &p, &d->h, uncached);
    if (e != hipSuccess) return record_hip(e, "exportable allocation");
    *out = p;
    buf_desc b{};
    b.h = d->h;
    describe_alloc(p, &b);
    memcpy(d, &b, sizeof(b));
    return OMPI_AMD_SUCCESS;
}

int comm_arena_alloc(ompi_amd_comm_t *c, size_t bytes, void **out) {
    char *p = nullptr;
    const int rc = arena_alloc(c, bytes, &p, (size_t)2 << 20);
    *out = p;
    return rc;
}

void comm_arena_free(ompi_amd_comm_t *c, void *p) { arena_free(c, static_cast<char *>(p)); }

int comm_export(ompi_amd_comm_t *c, const void *ptr, ipc_desc *d) {
    buf_desc b{};
    const int rc = export_buf(c, ptr, &b);
    memcpy(d, &b, sizeof(b));
    return rc;
}

bool comm_ipc_safe(const void *ptr) {
    void *base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange((hipDeviceptr_t *)&base, &size, (hipDeviceptr_t)ptr) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const unsigned long long id = buffer_id(ptr);
    return ipc_safe_size(size) && size <= kMaxIpcBytes && !export_aged(base, size, id) &&
           !export_reused(base, id);
}

bool comm_win_separate_ok(ompi_amd_comm_t *c) { return c->win_separate != 0 || c->win_shadow != 0; }

bool comm_win_needs_shadow(ompi_amd_comm_t *c, const void *base) {
    if (c->win_shadow || !comm_ipc_safe(base)) {
        ++c->shadow_windows;
        return true;
    }
    return false;
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

hipStream_t comm_call_stream(ompi_amd_comm_t *c, void *stream) { return comm_stream(c, stream); }

int comm_copy(ompi_amd_comm_t *c, const void *src, void *dst, size_t bytes, hipStream_t s) {
    cp_jobs jobs{};
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    jobs.j[0] = {(const char *)src, (char *)dst, (int64_t)bytes};
    jobs.n = 1;
    return launch_copy(c, jobs, s);
}

}  // namespace ompi_amd
