// Point-to-point messages between device buffers (include/ompi_amd_p2p.h).
//
// Reference path replaced for device memory: PML ob1's rendezvous for CUDA
// buffers (pml_ob1_cuda.c:56-101: the sender registers its buffer and sends
// an RGET header; the receiver "gets" it with btl/smcuda,
// btl_smcuda.c:1077-1250, which opens the sender's CUDA IPC handle and
// issues cuMemcpyAsync, then sends a FIN; common_cuda.c:1008-1320).
//
// Here:
//   mailbox  one POSIX shared-memory segment per communicator holding, for
//            every ordered (src, dst) pair, a ring of kSlots message
//            descriptors {tag, bytes, IPC handle + offset of the send
//            buffer} and a published-count word.  Only the sender writes a
//            descriptor and the count; only the receiver moves a slot from
//            POSTED to MATCHED to DONE; the sender recycles a DONE slot.
//   match    on the receiver's host, in MPI order: per source, messages in
//            sequence order; posted receives in posting order (each takes
//            the earliest matching message), wildcards allowed.
//   data     the receiver launches one copy kernel (osc_ipc.hip's
//            xfer_kernel: 16-B granules, system-scope acquire/release) that
//            loads the sender's buffer through its IPC mapping over xGMI
//            straight into the receive buffer: one HBM read on the sender's
//            GPU, one HBM write on the receiver's, no staging.
//   FIN      the receiver marks the slot DONE once the copy's event has
//            completed; the send completes when it sees DONE.
//   eager    messages of at most kEager bytes (btl/smcuda's 4 KiB eager
//            limit, btl_smcuda_component.c:197) are first copied into the
//            sender's device eager area (one cell per ring slot, the area
//            exported once), as ob1's eager protocol does: MPI_Send of a
//            small message never waits for the receiver.  From a device
//            buffer the copy kernel itself publishes the cell (a flag word
//            after the data = sequence + 1) and the message is posted as
//            soon as the kernel is launched: the receiver's copy kernel waits
//            for the flag on the device, so the sender's copy and the
//            receiver's match and launch overlap instead of the sender
//            synchronising its stream first; the send
//            completes when its copy kernel has run.  The cell is reused
//            only after the slot is DONE.
//   staged   larger messages are copied into a library-owned send stage
//            (a pool of exported device buffers, never freed while the
//            communicator lives) and the receiver pulls from there, so no
//            peer ever maps an application buffer — the (process, address)
//            identity of an IPC handle cannot go stale under the
//            application's frees.  From a device buffer
//            the stage copy signals like an eager cell (its last workgroup
//            sets the slot's cell flag), the message is posted at launch and
//            the receiver's copy waits for the flag on the device; a
//            standard send completes once staged (ob1 may buffer a standard
//            send too);
//            MPI_Ssend still completes at the receiver's FIN.  Past the
//            pool's cap (param p2p_stage_mib), or with p2p_user_ipc = 1, the
//            receiver maps the send buffer itself (rendezvous, as before).
//   host     a host send buffer of at most kInline bytes travels inside
//            its mailbox slot, one of at most kHostMax bytes through the
//            sender's host stage (a ring of kHostStage bytes per rank: its
//            own shared segment, created and reserved with posix_fallocate at
//            the rank's first such send, mapped by a receiver at the first
//            message through it; a reservation /dev/shm cannot hold turns the
//            ring off for that rank) — ob1 / btl/sm's path for host memory:
//            one copy in, one copy out (or one host-to-device copy into a
//            device receive buffer), no device work on the sender (round 4,
//            profiles/r04_pml_host_path_ab*.jsonl); larger host send buffers,
//            or a full ring, go through a device stage (eager cell or pool:
//            the copy kernel cannot read pageable memory); a staged message
//            received into host memory lands in a device receive stage first
//            and is copied out before it completes.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/ompi_amd_p2p.h"
#include "comm_internal.h"
#include "host_mark.h"
#include "runtime.h"

namespace ompi_amd {

constexpr int kSlots = 64;
constexpr size_t kEager = 4096;
constexpr size_t kCell = kEager + 64;  // the data, then the cell's flag word (its own line)
constexpr size_t kInline = 1024;  // host payload carried in the slot itself
constexpr size_t kHostStage = 8u << 20;  // per rank, its own segment (created at first use)
constexpr size_t kHostMax = 2u << 20;    // largest message through it

enum : uint32_t { S_FREE = 0, S_POSTED = 1, S_MATCHED = 2, S_DONE = 3 };

struct alignas(64) msg_slot {
    std::atomic<uint32_t> state;
    int32_t tag;
    uint64_t seq;
    uint64_t bytes;
    uint64_t raw;  // the send buffer's address (messages to self)
    ipc_desc d;    // the send buffer for peers
    uint32_t inl;  // 1: payload in `inline_data`; 2: in the sender's host stage at offset `raw`;
                   // 3: in an eager cell whose flag (cell + kEager) becomes seq + 1;
                   // 4: in a send stage (d) whose copy kernel sets the slot's cell flag (fd)
    ipc_desc fd;   // inl 4: the sender's eager cell of this slot (its flag word)
    char inline_data[kInline];
};

struct alignas(64) pair_q {
    std::atomic<uint64_t> posted;  // descriptors published by the sender
    char pad[56];
    msg_slot slot[kSlots];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory atomics");
static_assert(std::atomic<uint32_t>::is_always_lock_free, "shared-memory atomics");

// A library-owned device buffer of the send-stage pool (exported once) or
// of the receive-stage pool (local only).
struct stage {
    char *buf = nullptr;
    size_t cap = 0;
    ipc_desc d{};
    bool arena = false;  // a range of the communicator's exported arena (freed with it)
};

struct p2p_state {
    ompi_amd_comm_t *c = nullptr;
    int64_t timeout_ms = -1;  // param p2p_timeout_ms: -1 the communicator's, 0 none
    int user_ipc = 0;         // param p2p_user_ipc: large sends map the caller's buffer
    size_t stage_cap = 1ull << 30;  // param p2p_stage_mib: send-stage pool limit
    size_t stage_bytes = 0;         //   allocated so far
    std::vector<stage> send_free, recv_free;
    struct inflight { int dst; uint64_t seq; stage st; };
    std::deque<inflight> staged;  // sends whose stage the receiver may still read
    int64_t staged_sends = 0, direct_sends = 0, host_sends = 0, host_recvs = 0;
    int rank = 0, size = 0;
    char name[256] = {0};
    pair_q *q = nullptr;
    size_t bytes = 0;
    bool unlinked = false;
    std::vector<uint64_t> scan_from;  // per source: first sequence possibly still POSTED
    std::deque<ompi_amd_p2p_request *> recvs;  // posted receives not matched yet
    // matched receives whose copy may still run: progress completes them
    // (FIN to the sender) whatever call drives it, so a rank blocked in a
    // send on a full ring still frees its peers' slots (MPI progress)
    std::vector<ompi_amd_p2p_request *> matched;
    std::recursive_mutex mu;
    // [size][kSlots] cells of kCell bytes, then [size][kSlots] 64-B lines of
    // receive copy counters (zeroed), allocated at first use
    char *eager = nullptr;
    ipc_desc eager_d{};  // its export (made at allocation): a cell's is this one at the cell's offset
    ipc_desc cell_desc(const char *cell) const {
        ipc_desc d = eager_d;
        d.off += (uint64_t)(cell - eager);
        return d;
    }
    uint32_t *recv_done(int src, uint64_t seq) {
        return reinterpret_cast<uint32_t *>(eager + (size_t)size * kSlots * kCell +
                                            ((size_t)src * kSlots + seq % kSlots) * 64);
    }
    // this rank's host stage ring (bytes [htail, hhead) in flight, monotonic
    // counters) and the messages holding it, oldest first
    uint64_t hhead = 0, htail = 0;
    struct hchunk { int dst; uint64_t seq, end; };
    std::deque<hchunk> hflight;
    int64_t host_stage_sends = 0;
    int64_t unsafe_sends = 0;  // user_ipc sends staged: no IPC-safe size, or older than an IPC close
    int age_all = 0;           // test hook (param p2p_age_all): treat every buffer as older
    std::vector<hipEvent_t> ev_free;  // receive copies' events, reused
    // host stage rings: [rank] this process's mapping (nullptr: not yet);
    // this rank's own is created at its first host-staged send
    std::vector<char *> hring;
    bool hring_off = false;  // this rank's could not be reserved: device stages instead
    void ring_name(int r, char *out, size_t n) const { snprintf(out, n, "%s.h%d", name, r); }
    // rank r's ring, mapped on first use (r's sender created it before it
    // posted the message that names it); nullptr when it cannot be mapped
    char *host_stage(int r) {
        if (hring[(size_t)r]) return hring[(size_t)r];
        char nm[300];
        ring_name(r, nm, sizeof(nm));
        const int fd = shm_open(nm, O_RDWR, 0600);
        if (fd < 0) return nullptr;
        void *m = mmap(nullptr, kHostStage, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m == MAP_FAILED) return nullptr;
        return hring[(size_t)r] = static_cast<char *>(m);
    }
    // this rank's ring, created and reserved (posix_fallocate: the pages
    // exist, so no later store can SIGBUS on a full /dev/shm); false when
    // /dev/shm cannot hold it — the ring stays off and device stages carry
    // host messages instead
    bool own_ring() {
        if (hring[(size_t)rank]) return true;
        if (hring_off) return false;
        char nm[300];
        ring_name(rank, nm, sizeof(nm));
        shm_unlink(nm);
        const int fd = shm_open(nm, O_CREAT | O_EXCL | O_RDWR, 0600);
        bool ok = fd >= 0 && ftruncate(fd, (off_t)kHostStage) == 0 &&
                  posix_fallocate(fd, 0, (off_t)kHostStage) == 0;
        void *m = ok ? mmap(nullptr, kHostStage, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
        if (fd >= 0) close(fd);
        if (m == MAP_FAILED) {
            if (fd >= 0) shm_unlink(nm);
            hring_off = true;
            return false;
        }
        hring[(size_t)rank] = static_cast<char *>(m);
        return true;
    }

    pair_q &pair(int src, int dst) { return q[(size_t)src * (size_t)size + (size_t)dst]; }
};

}  // namespace ompi_amd

using namespace ompi_amd;

struct ompi_amd_p2p_request {
    p2p_state *p = nullptr;
    bool is_send = false;
    bool done = false;
    int rc = OMPI_AMD_SUCCESS;
    // send
    int peer = 0;
    uint64_t seq = 0;
    // receive
    void *buf = nullptr;
    size_t cap = 0;
    int src = OMPI_AMD_ANY_SOURCE, tag = OMPI_AMD_ANY_TAG;
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;
    // an eager copy kernel's completion word (pinned host memory, host_mark.h):
    // done once *mark >= mark_v; no event is recorded then
    uint64_t *mark = nullptr;
    uint64_t mark_v = 0;
    unsigned polls = 0;
    bool matched = false;
    msg_slot *slot = nullptr;  // matched message
    void *pinned = nullptr;    // sender mapping held during the copy
    void *pinned2 = nullptr;   // inl 4: the sender's eager area (the stage's flag)
    ompi_amd_status_t st{};
    void *host_dst = nullptr;  // a host receive buffer: the copy lands in `rstage` first
    stage rstage{};
    bool has_rstage = false;
};

namespace ompi_amd {

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

int p2p_set_param(p2p_state *p, const char *key, int64_t v) {
    if (!p) return OMPI_AMD_ERR_BAD_PARAM;
    std::lock_guard<std::recursive_mutex> g(p->mu);
    if (!strcmp(key, "p2p_timeout_ms")) {
        if (v < -1) return OMPI_AMD_ERR_BAD_PARAM;
        p->timeout_ms = v;
    } else if (!strcmp(key, "p2p_user_ipc")) {
        p->user_ipc = v ? 1 : 0;
    } else if (!strcmp(key, "p2p_stage_mib")) {
        if (v < 0) return OMPI_AMD_ERR_BAD_PARAM;
        p->stage_cap = (size_t)v << 20;
    } else if (!strcmp(key, "p2p_age_all")) {  // test hook: as if every buffer predated an IPC close
        p->age_all = v ? 1 : 0;
    } else {
        return OMPI_AMD_ERR_UNSUPPORTED;  // not a p2p key
    }
    return OMPI_AMD_SUCCESS;
}

int p2p_get_param(p2p_state *p, const char *key, int64_t *v) {
    if (!p) return OMPI_AMD_ERR_BAD_PARAM;
    std::lock_guard<std::recursive_mutex> g(p->mu);
    if (!strcmp(key, "p2p_timeout_ms")) *v = p->timeout_ms;
    else if (!strcmp(key, "p2p_user_ipc")) *v = p->user_ipc;
    else if (!strcmp(key, "p2p_stage_mib")) *v = (int64_t)(p->stage_cap >> 20);
    else if (!strcmp(key, "p2p_stage_bytes")) *v = (int64_t)p->stage_bytes;
    else if (!strcmp(key, "p2p_staged_sends")) *v = p->staged_sends;
    else if (!strcmp(key, "p2p_direct_sends")) *v = p->direct_sends;
    else if (!strcmp(key, "p2p_host_sends")) *v = p->host_sends;
    else if (!strcmp(key, "p2p_host_recvs")) *v = p->host_recvs;
    else if (!strcmp(key, "p2p_host_stage_sends")) *v = p->host_stage_sends;
    else if (!strcmp(key, "p2p_unsafe_sends")) *v = p->unsafe_sends;
    else return OMPI_AMD_ERR_UNSUPPORTED;
    return OMPI_AMD_SUCCESS;
}

int p2p_create(ompi_amd_comm_t *c, const char *name, int rank, int size, int phase,
               p2p_state **out) {
    auto *p = new (std::nothrow) p2p_state;
    if (!p) return OMPI_AMD_ERR_BOOTSTRAP;
    p->c = c;
    p->rank = rank;
    p->size = size;
    p->scan_from.assign((size_t)size, 0);
    snprintf(p->name, sizeof(p->name), "/ompi_amd_%s.p2p", name);
    for (char *ch = p->name + 1; *ch; ++ch)
        if (*ch == '/') *ch = '_';
    p->bytes = sizeof(pair_q) * (size_t)size * (size_t)size;
    p->hring.assign((size_t)size, nullptr);
    int fd = -1;
    if (phase == 0) {  // rank 0, before the communicator's first rendezvous
        shm_unlink(p->name);
        fd = shm_open(p->name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd >= 0 && ftruncate(fd, (off_t)p->bytes) != 0) {
            close(fd);
            fd = -1;
        }
    } else {  // the others, after it
        fd = shm_open(p->name, O_RDWR, 0600);
    }
    if (fd < 0) {
        record_msg("p2p mailbox %s: %s", p->name, strerror(errno));
        delete p;
        return OMPI_AMD_ERR_BOOTSTRAP;
    }
    void *m = mmap(nullptr, p->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        record_msg("mmap %s: %s", p->name, strerror(errno));
        if (phase == 0) shm_unlink(p->name);
        delete p;
        return OMPI_AMD_ERR_BOOTSTRAP;
    }
    p->q = static_cast<pair_q *>(m);  // zero-filled by ftruncate: all slots FREE
    *out = p;
    return OMPI_AMD_SUCCESS;
}

void p2p_unlink(p2p_state *p) {
    if (p && !p->unlinked) {
        shm_unlink(p->name);
        p->unlinked = true;
    }
}

void p2p_destroy(p2p_state *p) {
    if (!p) return;
    if (p->q) munmap(p->q, p->bytes);
    for (char *h : p->hring)
        if (h) munmap(h, kHostStage);
    if (p->hring[(size_t)p->rank]) {  // every peer's receive from it completed (final rendezvous)
        char nm[300];
        p->ring_name(p->rank, nm, sizeof(nm));
        shm_unlink(nm);
    }
    if (p->eager) comm_release_exportable(p->eager);  // recycled: a hipFree waits for the device
    for (hipEvent_t e : p->ev_free) hip_ignore(hipEventDestroy(e));
    // the communicator's final rendezvous has passed: no peer reads a stage
    // (arena stages went with the communicator's arena)
    for (auto &f : p->staged)
        if (!f.st.arena) comm_release_exportable(f.st.buf);
    for (auto &st : p->send_free)
        if (!st.arena) comm_release_exportable(st.buf);
    for (auto &st : p->recv_free) comm_release_exportable(st.buf);
    if (p->rank == 0) p2p_unlink(p);
    delete p;
}

// Seconds a host wait may last (0: no limit; the PML glue's blocking calls
// never time out, MPI semantics).
static double limit_s(const p2p_state *p) {
    const int64_t ms = p->timeout_ms < 0 ? comm_timeout_ms(p->c) : p->timeout_ms;
    return ms == 0 ? 0.0 : (double)ms / 1000.0;
}

static bool over(const p2p_state *p, double t0) {
    const double l = limit_s(p);
    return l > 0 && now_s() - t0 > l;
}

// size classes: powers of two from 64 KiB (2 MiB multiples past 1 GiB)
static size_t stage_class(size_t bytes) {
    if (bytes > (1ull << 30)) return (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    size_t c = 64u << 10;
    while (c < bytes) c <<= 1;
    return c;
}

// Send stages whose message the receiver finished (slot DONE or recycled)
// go back to the pool.  Under p->mu.
static void reclaim(p2p_state *p) {
    for (auto it = p->staged.begin(); it != p->staged.end();) {
        msg_slot &m = p->pair(p->rank, it->dst).slot[it->seq % kSlots];
        if (m.seq != it->seq || m.state.load(std::memory_order_acquire) == S_DONE) {
            p->send_free.push_back(it->st);
            it = p->staged.erase(it);
        } else {
            ++it;
        }
    }
}

// Host-stage chunks whose message the receiver finished (oldest first: the
// ring frees in order).  Under p->mu.
static void reclaim_host(p2p_state *p) {
    while (!p->hflight.empty()) {
        const auto &h = p->hflight.front();
        msg_slot &m = p->pair(p->rank, h.dst).slot[h.seq % kSlots];
        if (m.seq == h.seq && m.state.load(std::memory_order_acquire) != S_DONE) break;
        p->htail = h.end;
        p->hflight.pop_front();
    }
}

// A contiguous chunk of `bytes` of this rank's host stage (offset in *off),
// or false when the ring has no room now.  Under p->mu.
static bool take_host(p2p_state *p, size_t bytes, uint64_t *off, uint64_t *end) {
    if (!p->own_ring()) return false;
    reclaim_host(p);
    uint64_t at = p->hhead;
    const uint64_t pos = at % kHostStage;
    if (pos + bytes > kHostStage) at += kHostStage - pos;  // no wrap inside a chunk
    if (at + bytes - p->htail > kHostStage) return false;
    *off = at % kHostStage;
    *end = at + bytes;
    return true;
}

// The smallest free stage of `pool` that holds `bytes`, or a new one
// (exported when `exported`); false past the send pool's cap.  Under p->mu.
static bool take_stage(p2p_state *p, std::vector<stage> &pool, size_t bytes, bool exported,
                       stage *out) {
    auto best = pool.end();
    for (auto it = pool.begin(); it != pool.end(); ++it)
        if (it->cap >= bytes && (best == pool.end() || it->cap < best->cap)) best = it;
    if (best != pool.end()) {
        *out = *best;
        pool.erase(best);
        return true;
    }
    const size_t cls = stage_class(bytes);
    if (exported && p->stage_bytes + cls > p->stage_cap) return false;
    stage st;
    st.cap = cls;
    if (exported) {
        // from the communicator's exported arena: its chunks grow
        // geometrically and each is exported once, so a receiver maps a
        // handful of chunks instead of one allocation (of at least the 4 MiB
        // IPC minimum) per stage; past the arena's limit, one of its own
        void *m = nullptr;
        if (comm_arena_alloc(p->c, cls, &m) == OMPI_AMD_SUCCESS && comm_export(p->c, m, &st.d) == OMPI_AMD_SUCCESS) {
            st.buf = static_cast<char *>(m);
            st.arena = true;
        } else {
            if (m) comm_arena_free(p->c, m);
            if (comm_alloc_exportable(cls, false, (void **)&st.buf, &st.d) != OMPI_AMD_SUCCESS) return false;
        }
        p->stage_bytes += cls;
    } else if (hipMalloc((void **)&st.buf, cls) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    *out = st;
    return true;
}

static bool is_device(const void *ptr) { return ompi_amd_is_device_pointer(ptr) != 0; }

// The eager area (exportable: peers read its cells and flags), allocated
// zeroed at the first device send or signalled receive.  Under p->mu.
static int eager_area(p2p_state *p) {
    if (p->eager) return OMPI_AMD_SUCCESS;
    const size_t area = (size_t)p->size * kSlots * (kCell + 64);
    int rc = comm_alloc_exportable(area, false, (void **)&p->eager, &p->eager_d);
    if (rc == OMPI_AMD_SUCCESS) {  // every flag 0 (no sequence + 1 yet), every counter 0
        // on a stream of its own that waits for nothing else: this can run
        // inside a receive's progress while this process's earlier copy
        // kernels still wait for peers (a device-wide or null-stream
        // synchronisation here could wait on them, and they on this rank)
        hipStream_t z = nullptr;
        rc = record_hip(hipStreamCreateWithFlags(&z, hipStreamNonBlocking), "hipStreamCreate (eager area)");
        if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipMemsetAsync(p->eager, 0, area, z), "hipMemset (p2p eager area)");
        if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipStreamSynchronize(z), "hipStreamSynchronize (eager area)");
        if (z) hip_ignore(hipStreamDestroy(z));
        if (rc != OMPI_AMD_SUCCESS) hip_ignore(hipFree(p->eager));
    }
    if (rc != OMPI_AMD_SUCCESS) p->eager = nullptr;
    return rc;
}

static bool tag_ok(int want, int have) { return want == OMPI_AMD_ANY_TAG || want == have; }

// The earliest POSTED message from `s` a receive with `tag` matches.
// snap: the published counts one matching pass works with (loaded at the
// pass's first look at each source, ~0 = not yet): senders publish
// concurrently, and a message published while the pass is between two
// receives must not go to the later one when the earlier one also matches
// it (MPI's posting order; found by the ring-wrap test at N = 8).  NULL:
// the count as it is now (a probe).
constexpr uint64_t kNoSnap = ~0ull;
static msg_slot *find_from(p2p_state *p, int s, int tag, uint64_t *snap) {
    pair_q &q = p->pair(s, p->rank);
    if (snap && snap[s] == kNoSnap) snap[s] = q.posted.load(std::memory_order_acquire);
    const uint64_t posted = snap ? snap[s] : q.posted.load(std::memory_order_acquire);
    uint64_t &from = p->scan_from[(size_t)s];
    // skip the prefix that is no longer POSTED (matched or recycled)
    while (from < posted) {
        msg_slot &m = q.slot[from % kSlots];
        if (m.state.load(std::memory_order_acquire) == S_POSTED && m.seq == from) break;
        ++from;
    }
    for (uint64_t k = from; k < posted; ++k) {
        msg_slot &m = q.slot[k % kSlots];
        if (m.state.load(std::memory_order_acquire) == S_POSTED && m.seq == k && tag_ok(tag, m.tag))
            return &m;
    }
    return nullptr;
}

static msg_slot *find(p2p_state *p, int src, int tag, int *from_rank, uint64_t *snap = nullptr) {
    if (src != OMPI_AMD_ANY_SOURCE) {
        *from_rank = src;
        return find_from(p, src, tag, snap);
    }
    for (int k = 0; k < p->size; ++k) {
        const int s = (p->rank + k) % p->size;  // self first, then rank+1, ...
        if (msg_slot *m = find_from(p, s, tag, snap)) {
            *from_rank = s;
            return m;
        }
    }
    return nullptr;
}

// The copy's completion on r->stream: an event from the state's pool.  (No
// host mark here: with the send stage's copy on the same stream, the extra
// kernel per message cost more than it saved — device sendrecv 37 -> 52 µs
// at 8 B, 2 ranks on one GPU.)
static int record_copy(p2p_state *p, ompi_amd_p2p_request *r) {
    int rc = OMPI_AMD_SUCCESS;
    if (!r->ev) {
        if (!p->ev_free.empty()) {
            r->ev = p->ev_free.back();
            p->ev_free.pop_back();
        } else {
            rc = record_hip(hipEventCreateWithFlags(&r->ev, hipEventDisableTiming), "hipEventCreate (p2p)");
        }
    }
    if (rc == OMPI_AMD_SUCCESS) rc = record_hip(hipEventRecord(r->ev, r->stream), "hipEventRecord (p2p)");
    return rc;
}

// A completion word for an eager copy kernel of `r` (none: the event).
static void take_mark(ompi_amd_p2p_request *r) {
    r->mark = mark_word_get();
    r->mark_v = r->mark ? mark_reserve() : 0;
}

// Whether r's copy kernel stored its mark.  Every 64th unanswered poll the
// stream backs it up: idle with no mark means the kernel never ran (its
// launch failed after all): the request ends with an error instead of
// waiting for ever (the PML glue's waits have no time limit).
static bool mark_landed(ompi_amd_p2p_request *r) {
    if (__atomic_load_n(r->mark, __ATOMIC_ACQUIRE) >= r->mark_v) return true;
    if (++r->polls % 64 != 0) return false;
    const hipError_t e = hipStreamQuery(r->stream);
    if (e == hipErrorNotReady) return false;
    if (__atomic_load_n(r->mark, __ATOMIC_ACQUIRE) >= r->mark_v) return true;
    r->rc = r->st.error = e != hipSuccess ? record_hip(e, "p2p copy")
                                          : (record_msg("p2p copy kernel ended without its mark"), OMPI_AMD_ERR_HIP);
    return true;
}

// OMPI_AMD_P2P_TRACE=1 (diagnostics): one stderr line per post, match and FIN.
static bool p2p_trace() {
    static const bool on = [] {
        const char *v = getenv("OMPI_AMD_P2P_TRACE");
        return v && atoi(v) != 0;
    }();
    return on;
}

// Claim `m` for receive `r` and launch its copy.
static void start_recv(p2p_state *p, ompi_amd_p2p_request *r, msg_slot *m, int s) {
    if (p2p_trace())
        fprintf(stderr, "[p2p %d] match req %p cap %zu <- src %d seq %llu tag %d bytes %llu inl %u state %u\n",
                p->rank, (void *)r, r->cap, s, (unsigned long long)m->seq, m->tag, (unsigned long long)m->bytes,
                m->inl, m->state.load());
    m->state.store(S_MATCHED, std::memory_order_release);
    r->matched = true;
    r->slot = m;
    r->st.source = s;
    r->st.tag = m->tag;
    r->st.bytes = m->bytes;
    size_t n = (size_t)m->bytes;
    if (n > r->cap) {  // MPI_ERR_TRUNCATE: copy what fits (ob1 does the same)
        n = r->cap;
        r->rc = OMPI_AMD_ERR_TRUNCATE;
        record_msg("p2p receive truncated: message %llu bytes, buffer %zu (source %d, tag %d, seq %llu)",
                   (unsigned long long)m->bytes, r->cap, s, m->tag, (unsigned long long)m->seq);
    }
    r->st.error = r->rc;
    if (n == 0) return;
    int rc = OMPI_AMD_SUCCESS;
    if (m->inl == 1 || m->inl == 2) {  // a host send out of the slot or the sender's host stage (host: done now)
        const char *ring = m->inl == 2 ? p->host_stage(s) : nullptr;
        if (m->inl == 2 && !ring) {
            r->rc = r->st.error = OMPI_AMD_ERR_BOOTSTRAP;
            record_msg("p2p: cannot map rank %d's host stage", s);
            return;
        }
        const char *from = m->inl == 1 ? m->inline_data : ring + m->raw;
        if (r->host_dst) {
            memcpy(r->host_dst, from, n);
            return;
        }
        rc = record_hip(hipMemcpyAsync(r->buf, from, n, hipMemcpyHostToDevice, r->stream),
                        "hipMemcpyAsync (p2p host-stage receive)");
        if (rc == OMPI_AMD_SUCCESS) rc = record_copy(p, r);
        if (rc != OMPI_AMD_SUCCESS) r->rc = r->st.error = rc;
        return;
    }
    const char *src = nullptr;
    if (s == p->rank) {
        src = reinterpret_cast<const char *>(m->raw);
    } else {
        rc = comm_import(p->c, s, m->d, &src, true, &r->pinned);
    }
    char *dst = static_cast<char *>(r->buf);
    if (rc == OMPI_AMD_SUCCESS && r->host_dst) {  // lands in a device stage, then to host
        if (take_stage(p, p->recv_free, n, false, &r->rstage)) {
            r->has_rstage = true;
            dst = r->rstage.buf;
        } else {
            rc = record_hip(hipErrorOutOfMemory, "p2p receive stage");
        }
    }
    if (rc == OMPI_AMD_SUCCESS) {
        if (m->inl == 3) {  // an eager cell: the copy waits for the sender's kernel to publish it
            const int64_t ms = comm_timeout_ms(p->c);
            const uint64_t ticks = ms > 0 ? (uint64_t)ms * 100000ull : (1ull << 62);  // 100 MHz
            if (!r->host_dst) take_mark(r);  // a host receive's copy out still needs the event
            rc = eager_get(src, dst, n, reinterpret_cast<const uint64_t *>(src + kEager), m->seq + 1,
                           comm_err_dev(p->c), ticks, r->mark, r->mark_v, r->stream);
        } else if (m->inl == 4) {  // a signalled stage: the copy waits for the sender's flag
            const char *fc = nullptr;
            rc = comm_import(p->c, s, m->fd, &fc, true, &r->pinned2);
            if (rc == OMPI_AMD_SUCCESS) rc = eager_area(p);  // this rank's copy counters
            if (rc == OMPI_AMD_SUCCESS) {
                const int64_t ms = comm_timeout_ms(p->c);
                xfer_sig sg;
                sg.wait = reinterpret_cast<const uint64_t *>(fc + kEager);
                sg.wait_v = m->seq + 1;
                sg.err = comm_err_dev(p->c);
                sg.ticks = ms > 0 ? (uint64_t)ms * 100000ull : (1ull << 62);
                if (!r->host_dst) take_mark(r);
                sg.mark = r->mark;
                sg.mark_v = r->mark_v;
                sg.done = p->recv_done(s, m->seq);
                rc = xfer_copy_sig(src, dst, n, r->stream, sg);
            }
        } else {
            rc = xfer_copy(src, dst, n, r->stream, nullptr, false);  // dst: this GPU's memory
        }
    }
    if (rc == OMPI_AMD_SUCCESS && r->host_dst)
        rc = record_hip(hipMemcpyAsync(r->host_dst, dst, n, hipMemcpyDeviceToHost, r->stream),
                        "hipMemcpyAsync (p2p receive to host)");
    if (rc == OMPI_AMD_SUCCESS && !r->mark) rc = record_copy(p, r);
    if (rc != OMPI_AMD_SUCCESS) r->rc = r->st.error = rc;
}

// Match posted receives against published messages, in posting order.
// A matched receive whose copy finished: release what it held, check the
// communicator's error (an eager wait that timed out copied nothing), FIN.
// false while the copy still runs.  Under p->mu.
static bool finish_recv(p2p_state *p, ompi_amd_p2p_request *r) {
    bool copied = true;
    if (r->mark) {
        copied = mark_landed(r);
    } else if (r->ev) {
        const hipError_t e = hipEventQuery(r->ev);
        if (e == hipErrorNotReady) {
            copied = false;
        } else if (e != hipSuccess) {
            r->rc = r->st.error = record_hip(e, "p2p copy");
        }
    }
    if (!copied) return false;
    if (r->pinned) comm_unpin(p->c, r->pinned);
    if (r->pinned2) comm_unpin(p->c, r->pinned2);
    r->pinned = r->pinned2 = nullptr;
    if (r->has_rstage) {
        p->recv_free.push_back(r->rstage);
        r->has_rstage = false;
    }
    if ((r->slot->inl == 3 || r->slot->inl == 4) && r->rc == OMPI_AMD_SUCCESS) {
        const int se = comm_sticky(p->c);
        if (se != OMPI_AMD_SUCCESS) r->rc = r->st.error = se;
    }
    if (p2p_trace())
        fprintf(stderr, "[p2p %d] FIN req %p seq %llu state %u\n", p->rank, (void *)r,
                (unsigned long long)r->slot->seq, r->slot->state.load());
    r->slot->state.store(S_DONE, std::memory_order_release);  // the FIN
    r->done = true;
    return true;
}

// Match posted receives against published messages, in posting order, and
// complete matched receives whose copies are over.  Under p->mu.
static void progress(p2p_state *p) {
    uint64_t snap[OMPI_AMD_MAX_RANKS];
    for (int k = 0; k < p->size; ++k) snap[k] = kNoSnap;
    for (auto it = p->recvs.begin(); it != p->recvs.end();) {
        ompi_amd_p2p_request *r = *it;
        int s = -1;
        msg_slot *m = find(p, r->src, r->tag, &s, snap);
        if (!m) {
            ++it;
            continue;
        }
        start_recv(p, r, m, s);
        p->matched.push_back(r);
        it = p->recvs.erase(it);
    }
    for (size_t i = 0; i < p->matched.size();) {
        if (finish_recv(p, p->matched[i])) {
            p->matched[i] = p->matched.back();
            p->matched.pop_back();
        } else {
            ++i;
        }
    }
}

// Non-blocking completion check of one request.
static int test_one(ompi_amd_p2p_request *r, bool *done) {
    p2p_state *p = r->p;
    std::lock_guard<std::recursive_mutex> g(p->mu);
    progress(p);
    if (r->done) {
        *done = true;
        return r->rc;
    }
    *done = false;
    if (r->is_send && r->mark) {  // a device eager send: complete once its copy into the cell ran
        r->done = mark_landed(r);
    } else if (r->is_send && r->ev) {
        const hipError_t e = hipEventQuery(r->ev);
        if (e != hipErrorNotReady) {
            if (e != hipSuccess) r->rc = record_hip(e, "p2p eager copy");
            r->done = true;
        }
    } else if (r->is_send) {
        msg_slot &m = p->pair(p->rank, r->peer).slot[r->seq % kSlots];
        if (m.seq != r->seq || m.state.load(std::memory_order_acquire) == S_DONE) r->done = true;
    }
    // a matched receive completes in progress() above (finish_recv)
    *done = r->done;
    return r->done ? r->rc : OMPI_AMD_SUCCESS;
}

static int wait_one(ompi_amd_p2p_request *r) {
    const double t0 = now_s();
    unsigned spins = 0;
    for (;;) {
        bool done = false;
        const int rc = test_one(r, &done);
        if (done) return rc;
        if (++spins > 64) sched_yield();
        if (over(r->p, t0)) {
            // what the request was waiting for, for the report
            p2p_state *p = r->p;
            std::lock_guard<std::recursive_mutex> g(p->mu);
            const int peer = r->is_send ? r->peer : r->src;
            unsigned long long posted = 0, scan = 0;
            int st = -1;
            if (peer >= 0 && peer < p->size) {
                const pair_q &q = r->is_send ? p->pair(p->rank, peer) : p->pair(peer, p->rank);
                posted = (unsigned long long)q.posted.load(std::memory_order_acquire);
                scan = r->is_send ? 0 : (unsigned long long)p->scan_from[(size_t)peer];
                if (r->is_send) st = (int)q.slot[r->seq % kSlots].state.load(std::memory_order_acquire);
            }
            const int ev = r->ev ? (int)hipEventQuery(r->ev) : -1;
            (void)hipGetLastError();
            record_msg("p2p %s timed out after %.1f s (peer %d, tag %d; matched %d, copy event %d, "
                       "posted %llu, scanned from %llu, slot state %d, seq %llu)",
                       r->is_send ? "send" : "receive", limit_s(r->p), peer,
                       r->is_send ? -1 : r->tag, r->matched ? 1 : 0, ev, posted, scan, st,
                       (unsigned long long)r->seq);
            return OMPI_AMD_ERR_TIMEOUT;
        }
    }
}

// A receive that never matched is taken out of the match list (cancel
// semantics, after a timeout or at free): a message that arrives later must
// not be copied into a buffer whose MPI_Recv already returned.  Matched
// receives (the copy is on the stream) and sends cannot be withdrawn.
static bool cancel_recv(ompi_amd_p2p_request *r) {
    p2p_state *p = r->p;
    std::lock_guard<std::recursive_mutex> g(p->mu);
    progress(p);  // a message that did arrive by now is still taken
    if (r->is_send || r->matched || r->done) return false;
    for (auto it = p->recvs.begin(); it != p->recvs.end(); ++it)
        if (*it == r) {
            p->recvs.erase(it);
            break;
        }
    r->done = true;
    r->rc = r->st.error = OMPI_AMD_ERR_TIMEOUT;
    return true;
}

static void fill_status(const ompi_amd_p2p_request *r, ompi_amd_status_t *st) {
    if (!st) return;
    if (r->is_send) {
        st->source = r->p->rank;
        st->tag = 0;
        st->error = r->rc;
        st->bytes = 0;
    } else {
        *st = r->st;
    }
}

}  // namespace ompi_amd

extern "C" {

int ompi_amd_isend(ompi_amd_comm_t *c, const void *buf, size_t bytes, int dst, int tag, int mode,
                   void *stream, ompi_amd_p2p_request_t **out) {
    if (!c || !out || tag < 0 || (bytes && !buf)) return OMPI_AMD_ERR_BAD_PARAM;
    p2p_state *p = comm_p2p(c);
    if (!p || dst < 0 || dst >= p->size) return OMPI_AMD_ERR_BAD_PARAM;
    if (mode == OMPI_AMD_SEND_BUFFERED) {
        record_msg("MPI_Bsend of device buffers is not provided");
        return OMPI_AMD_ERR_UNSUPPORTED;
    }
    if (mode < OMPI_AMD_SEND_SYNCHRONOUS || mode > OMPI_AMD_SEND_STANDARD)
        return OMPI_AMD_ERR_BAD_PARAM;
    int rc = record_hip(hipSetDevice(comm_device(c)), "hipSetDevice");
    const hipStream_t s = comm_call_stream(c, stream);
    const bool host = bytes && !is_device(buf);
    const bool eager = bytes <= kEager && mode != OMPI_AMD_SEND_SYNCHRONOUS;  // Ssend: rendezvous
    const bool inl = host && eager && bytes <= kInline;  // no device work at all
    const bool hostable = host && !inl && mode != OMPI_AMD_SEND_SYNCHRONOUS && bytes <= kHostMax;
    std::unique_lock<std::recursive_mutex> alloc_guard(p->mu);
    if (rc == OMPI_AMD_SUCCESS && !inl) rc = eager_area(p);  // peers read its cells and flags
    alloc_guard.unlock();
    if (rc != OMPI_AMD_SUCCESS) return rc;
    // A copy into an eager cell or a stage runs on `s`, after the buffer's
    // producers in stream order; only a message the receiver reads from the
    // buffer itself (direct, or to self) needs them done first — a host wait
    // the eager and staged paths no longer pay (one hipStreamSynchronize of
    // the two per small device message).
    auto producers_done = [&]() -> int {
        return host ? OMPI_AMD_SUCCESS : record_hip(hipStreamSynchronize(s), "hipStreamSynchronize (send)");
    };
    auto *r = new (std::nothrow) ompi_amd_p2p_request;
    if (!r) return OMPI_AMD_ERR_BAD_PARAM;
    r->p = p;
    r->is_send = true;
    r->peer = dst;
    std::lock_guard<std::recursive_mutex> g(p->mu);
    pair_q &q = p->pair(p->rank, dst);
    const uint64_t seq = q.posted.load(std::memory_order_relaxed);
    msg_slot &m = q.slot[seq % kSlots];
    // the ring slot must be free: its previous message completed (DONE) or
    // was never used; wait for the receiver otherwise (bounded only by
    // p2p_timeout_ms)
    const double t0 = now_s();
    for (;;) {
        const uint32_t st = m.state.load(std::memory_order_acquire);
        if (st == S_FREE || st == S_DONE) break;
        progress(p);  // our own receives keep flowing meanwhile
        sched_yield();
        if (over(p, t0)) {
            record_msg("p2p send to %d: %d messages unmatched for %.1f s", dst, kSlots, limit_s(p));
            delete r;
            return OMPI_AMD_ERR_TIMEOUT;
        }
    }
    reclaim(p);
    const void *src = buf;
    ipc_desc d{}, fd{};
    bool staged = false, sflagged = false;
    auto copy_in = [&](char *to) {
        const int crc = host ? record_hip(hipMemcpyAsync(to, buf, bytes, hipMemcpyHostToDevice, s),
                                          "hipMemcpyAsync (p2p send stage)")
                             : xfer_copy(buf, to, bytes, s, nullptr, false);  // a stage of this GPU
        return crc == OMPI_AMD_SUCCESS ? record_hip(hipStreamSynchronize(s), "hipStreamSynchronize (stage)")
                                       : crc;
    };
    // The message into a library stage (peers read library memory).  must: a
    // host buffer, or a device buffer peers cannot map reliably — wait
    // for a stage, past the cap once if nothing is in flight; otherwise one
    // try, and without a stage the message goes from the buffer itself.
    auto stage_send = [&](bool must, bool must_if_unsafe = false) -> int {
        stage st;
        bool got = take_stage(p, p->send_free, bytes, true, &st);
        if (!got && !must && must_if_unsafe && (p->age_all || !comm_ipc_safe(src))) {
            // no stage free and the buffer cannot go out by itself: a stage
            // past the cap rather than a wait (an MPI_Isend must return
            // whether or not the receiver has posted yet)
            ++p->unsafe_sends;
            const size_t cap = p->stage_cap;
            p->stage_cap = p->stage_bytes + stage_class(bytes);
            got = take_stage(p, p->send_free, bytes, true, &st);
            p->stage_cap = cap;
            if (!got) return record_hip(hipErrorOutOfMemory, "p2p send stage (device buffer past the cap)");
        }
        if (!got && must) {
            const double t1 = now_s();
            while (!got) {
                progress(p);
                reclaim(p);
                got = take_stage(p, p->send_free, bytes, true, &st);
                if (!got && p->staged.empty()) {  // nothing to wait for: past the cap once
                    const size_t cap = p->stage_cap;
                    p->stage_cap = p->stage_bytes + stage_class(bytes);
                    got = take_stage(p, p->send_free, bytes, true, &st);
                    p->stage_cap = cap;
                    if (!got) break;
                }
                if (!got) sched_yield();
                if (!got && over(p, t1)) break;
            }
            if (!got)
                return record_hip(hipErrorOutOfMemory,
                                  host ? "p2p send stage (host buffer)" : "p2p send stage (device buffer)");
        }
        if (!got) return OMPI_AMD_SUCCESS;
        int crc;
        if (!host && mode != OMPI_AMD_SEND_SYNCHRONOUS) {
            // posted at once: the stage copy sets this slot's cell flag when
            // its last workgroup is done, and the receiver's copy waits for it
            char *cell = p->eager + ((size_t)dst * kSlots + seq % kSlots) * kCell;
            xfer_sig sg;
            sg.flag = reinterpret_cast<uint64_t *>(cell + kEager);
            sg.flag_v = seq + 1;
            sg.done = reinterpret_cast<uint32_t *>(cell + kEager + 8);
            r->stream = s;
            take_mark(r);
            sg.mark = r->mark;
            sg.mark_v = r->mark_v;
            crc = xfer_copy_sig(buf, st.buf, bytes, s, sg);
            if (crc == OMPI_AMD_SUCCESS && !r->mark) crc = record_copy(p, r);
            fd = p->cell_desc(cell);
            sflagged = true;
        } else {
            crc = copy_in(st.buf);
        }
        if (crc != OMPI_AMD_SUCCESS) {
            p->send_free.push_back(st);
            return crc;
        }
        src = st.buf;
        d = st.d;
        staged = true;
        p->staged.push_back({dst, seq, st});
        ++p->staged_sends;
        return OMPI_AMD_SUCCESS;
    };
    uint64_t hoff = 0, hend = 0;
    const bool hstaged = hostable && take_host(p, bytes, &hoff, &hend);
    bool flagged = false;  // a device eager send: the copy kernel publishes the cell
    if (inl) {  // into the slot itself; the send completes now
        memcpy(m.inline_data, buf, bytes);
    } else if (hstaged) {  // into this rank's host stage; the send completes now
        memcpy(p->host_stage(p->rank) + hoff, buf, bytes);
        p->hflight.push_back({dst, seq, hend});
        p->hhead = hend;
        ++p->host_stage_sends;
    } else if (eager && bytes) {  // stage into this slot's cell
        char *cell = p->eager + ((size_t)dst * kSlots + seq % kSlots) * kCell;
        if (host) {  // a host buffer past the host ring: copied in now
            rc = copy_in(cell);
        } else {  // posted at once; the receiver's copy waits for the flag
            r->stream = s;
            take_mark(r);
            rc = eager_put(buf, cell, bytes, reinterpret_cast<uint64_t *>(cell + kEager), seq + 1, r->mark,
                           r->mark_v, s);
            if (rc == OMPI_AMD_SUCCESS && !r->mark) rc = record_copy(p, r);
            flagged = true;
        }
        src = cell;
    } else if (bytes && (host || (dst != p->rank && !p->user_ipc))) {
        // one try at a stage; a device buffer that cannot go out by itself
        // (not IPC-safe, or older than an IPC close) waits for one instead
        rc = stage_send(host, !host);
    } else if (bytes && dst != p->rank && (p->age_all || !comm_ipc_safe(src))) {
        // p2p_user_ipc: an allocation peers could not map reliably — not an
        // IPC-safe size, or older than an IPC close of this process, which
        // ROCm 7.2 may refuse to export — goes through a
        // stage, as the collectives send such a buffer through a shadow
        ++p->unsafe_sends;
        rc = stage_send(true);
    }
    if (host) ++p->host_sends;
    if (rc == OMPI_AMD_SUCCESS && bytes && dst != p->rank && !staged && !inl && !hstaged) {
        // library memory (eager cells, stages: exported at allocation) or an
        // application buffer comm_ipc_safe() accepted: the runtime answers
        // (DESIGN.md §4.6); a refusal is an error
        if (!eager) rc = producers_done();  // the receiver reads the buffer itself
        if (rc == OMPI_AMD_SUCCESS)
            rc = eager ? (d = p->cell_desc(static_cast<const char *>(src)), OMPI_AMD_SUCCESS)
                       : comm_export(c, src, &d);
        if (!eager && !staged) ++p->direct_sends;
    } else if (rc == OMPI_AMD_SUCCESS && bytes && dst == p->rank && !staged && !inl && !hstaged &&
               !eager) {
        rc = producers_done();  // a receive of this process copies from the buffer
    }
    if (rc != OMPI_AMD_SUCCESS) {
        if (r->ev) p->ev_free.push_back(r->ev);
        mark_word_put(r->mark);  // its kernel never launched (or failed to)
        delete r;
        return rc;
    }
    m.tag = tag;
    m.seq = seq;
    m.bytes = bytes;
    m.raw = hstaged ? hoff : reinterpret_cast<uint64_t>(src);
    m.d = d;
    m.fd = fd;
    m.inl = inl ? 1u : hstaged ? 2u : flagged ? 3u : sflagged ? 4u : 0u;
    if (p2p_trace())
        fprintf(stderr, "[p2p %d] post -> dst %d seq %llu tag %d bytes %zu inl %u\n", p->rank, dst,
                (unsigned long long)seq, tag, bytes, m.inl);
    m.state.store(S_POSTED, std::memory_order_release);
    q.posted.store(seq + 1, std::memory_order_release);
    r->seq = seq;
    // the user's buffer is free again once staged (Ssend: at the FIN)
    // (a device eager send: once its copy kernel ran, test_one)
    r->done = (eager && !flagged) || hstaged || (staged && !sflagged && mode != OMPI_AMD_SEND_SYNCHRONOUS);
    *out = r;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_irecv(ompi_amd_comm_t *c, void *buf, size_t bytes, int src, int tag, void *stream,
                   ompi_amd_p2p_request_t **out) {
    if (!c || !out || (bytes && !buf) || tag < OMPI_AMD_ANY_TAG) return OMPI_AMD_ERR_BAD_PARAM;
    p2p_state *p = comm_p2p(c);
    if (!p || src < OMPI_AMD_ANY_SOURCE || src >= p->size) return OMPI_AMD_ERR_BAD_PARAM;
    const int rc = record_hip(hipSetDevice(comm_device(c)), "hipSetDevice");
    if (rc != OMPI_AMD_SUCCESS) return rc;
    auto *r = new (std::nothrow) ompi_amd_p2p_request;
    if (!r) return OMPI_AMD_ERR_BAD_PARAM;
    r->p = p;
    r->buf = buf;
    if (bytes && !is_device(buf)) {
        r->host_dst = buf;
        ++p->host_recvs;
    }
    r->cap = bytes;
    r->src = src;
    r->tag = tag;
    if (p2p_trace())
        fprintf(stderr, "[p2p %d] irecv req %p cap %zu src %d tag %d\n", p->rank, (void *)r, bytes, src, tag);
    r->stream = comm_call_stream(c, stream);
    std::lock_guard<std::recursive_mutex> g(p->mu);
    p->recvs.push_back(r);
    progress(p);
    *out = r;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_p2p_test(ompi_amd_p2p_request_t *r, int *done, ompi_amd_status_t *st) {
    if (!r || !done) return OMPI_AMD_ERR_BAD_PARAM;
    bool d = false;
    const int rc = test_one(r, &d);
    *done = d ? 1 : 0;
    if (d) fill_status(r, st);
    return rc;
}

int ompi_amd_p2p_wait(ompi_amd_p2p_request_t *r, ompi_amd_status_t *st) {
    if (!r) return OMPI_AMD_ERR_BAD_PARAM;
    const int rc = wait_one(r);
    fill_status(r, st);
    return rc;
}

int ompi_amd_p2p_free(ompi_amd_p2p_request_t *r) {
    if (!r) return OMPI_AMD_SUCCESS;
    int rc = OMPI_AMD_SUCCESS;
    if (!r->done) {
        rc = wait_one(r);
        if (!r->done) cancel_recv(r);
    }
    if (!r->done) return rc;  // a matched copy or a send the mailbox still references: keep it
    if (r->ev) {  // done: its copy is over
        std::lock_guard<std::recursive_mutex> g(r->p->mu);
        r->p->ev_free.push_back(r->ev);
    }
    mark_word_put(r->mark);  // done: its mark landed
    delete r;
    return rc;
}

int ompi_amd_send(ompi_amd_comm_t *c, const void *buf, size_t bytes, int dst, int tag, int mode,
                  void *stream) {
    ompi_amd_p2p_request_t *r = nullptr;
    int rc = ompi_amd_isend(c, buf, bytes, dst, tag, mode, stream, &r);
    if (rc != OMPI_AMD_SUCCESS) return rc;
    return ompi_amd_p2p_free(r);
}

int ompi_amd_recv(ompi_amd_comm_t *c, void *buf, size_t bytes, int src, int tag, void *stream,
                  ompi_amd_status_t *st) {
    ompi_amd_p2p_request_t *r = nullptr;
    int rc = ompi_amd_irecv(c, buf, bytes, src, tag, stream, &r);
    if (rc != OMPI_AMD_SUCCESS) return rc;
    rc = wait_one(r);
    if (rc != OMPI_AMD_SUCCESS && !r->done) cancel_recv(r);  // one timeout, not two
    fill_status(r, st);
    const int frc = ompi_amd_p2p_free(r);
    return rc != OMPI_AMD_SUCCESS ? rc : frc;
}

int ompi_amd_sendrecv(ompi_amd_comm_t *c, const void *sbuf, size_t sbytes, int dst, int stag,
                      void *rbuf, size_t rbytes, int src, int rtag, void *stream,
                      ompi_amd_status_t *st) {
    ompi_amd_p2p_request_t *rr = nullptr, *sr = nullptr;
    int rc = ompi_amd_irecv(c, rbuf, rbytes, src, rtag, stream, &rr);
    if (rc != OMPI_AMD_SUCCESS) return rc;
    rc = ompi_amd_isend(c, sbuf, sbytes, dst, stag, OMPI_AMD_SEND_STANDARD, stream, &sr);
    if (rc != OMPI_AMD_SUCCESS) {
        (void)ompi_amd_p2p_free(rr);
        return rc;
    }
    const int rrc = wait_one(rr);
    if (rrc != OMPI_AMD_SUCCESS && !rr->done) cancel_recv(rr);
    fill_status(rr, st);
    const int src_ = wait_one(sr);
    (void)ompi_amd_p2p_free(rr);
    (void)ompi_amd_p2p_free(sr);
    return rrc != OMPI_AMD_SUCCESS ? rrc : src_;
}

int ompi_amd_iprobe(ompi_amd_comm_t *c, int src, int tag, int *flag, ompi_amd_status_t *st) {
    if (!c || !flag) return OMPI_AMD_ERR_BAD_PARAM;
    p2p_state *p = comm_p2p(c);
    if (!p || src < OMPI_AMD_ANY_SOURCE || src >= p->size) return OMPI_AMD_ERR_BAD_PARAM;
    std::lock_guard<std::recursive_mutex> g(p->mu);
    progress(p);  // posted receives match first
    int s = -1;
    msg_slot *m = find(p, src, tag, &s);
    *flag = m ? 1 : 0;
    if (m && st) {
        st->source = s;
        st->tag = m->tag;
        st->error = OMPI_AMD_SUCCESS;
        st->bytes = m->bytes;
    }
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_probe(ompi_amd_comm_t *c, int src, int tag, ompi_amd_status_t *st) {
    if (!c || !comm_p2p(c)) return OMPI_AMD_ERR_BAD_PARAM;
    const double t0 = now_s();
    for (;;) {
        int flag = 0;
        const int rc = ompi_amd_iprobe(c, src, tag, &flag, st);
        if (rc != OMPI_AMD_SUCCESS || flag) return rc;
        sched_yield();
        if (over(comm_p2p(c), t0)) {
            record_msg("probe(%d, %d) timed out after %.1f s", src, tag, limit_s(comm_p2p(c)));
            return OMPI_AMD_ERR_TIMEOUT;
        }
    }
}

}  // extern "C"
