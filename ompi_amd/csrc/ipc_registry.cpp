// Process-wide IPC mapping registry (ipc_registry.h).
#include "ipc_registry.h"

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

#include "runtime.h"

namespace ompi_amd {

struct ipc_ref {
    ipc_alloc a;
    int device;
    void *base;      // the mapping in this process
    int refs = 0;
    int pins = 0;
    bool retired = false;  // closed: the exporter freed the allocation
    std::vector<std::pair<void *, int>> holders;  // (owner, references)
};

namespace {

// g_mu guards the tables below; it is never held across a runtime call that
// can block (an open, a close, a quiesce): those run with it released, and
// an allocation being opened sits in g_opening so that a second thread
// asking for it waits for the first open instead of opening it twice.
std::mutex g_mu;
std::condition_variable g_cv;
std::vector<ipc_ref *> g_live;     // open mappings
std::vector<ipc_alloc> g_opening;  // opens in progress (g_mu released)
std::vector<ipc_alloc> g_closing;  // retired mappings not closed yet (g_mu released)
struct user {
    void *owner;
    int (*quiesce)(void *);
    int busy;  // quiesces of it in progress: ipc_remove_user waits for them
};
std::vector<user> g_users;
ipc_stats g_st{};
std::atomic<uint64_t> g_close_mark{0};  // ipc_close_watermark()
std::mutex g_probe_mu;
std::vector<void *> g_probes;  // watermark probes, freed in batches (not here)

// After a close: the buffer id of a fresh allocation — every allocation
// with a lower id existed at the close (ipc_registry.h).  The probe is
// allocated now (an allocation made later must not count as older) but not
// freed here: closes run inside point-to-point progress and LRU evictions,
// and hipFree synchronises the whole device, which could wait on this
// process's kernels that wait on peers.  ipc_close_watermark(),
// called on host paths before an export, frees the probes 256 at a time.
void note_close() {
    std::lock_guard<std::mutex> g(g_probe_mu);
    void *p = nullptr;
    if (hipMalloc(&p, 4096) != hipSuccess) {
        (void)hipGetLastError();
        g_close_mark.store(UINT64_MAX);  // no id to compare with: spoil everything older
        return;
    }
    unsigned long long id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        id = UINT64_MAX;
    }
    g_probes.push_back(p);
    uint64_t cur = g_close_mark.load();
    while (cur < id && !g_close_mark.compare_exchange_weak(cur, id)) {
    }
}

void free_probes() {
    std::lock_guard<std::mutex> g(g_probe_mu);
    if (g_probes.size() < 256) return;
    for (void *q : g_probes) hip_ignore(hipFree(q));
    g_probes.clear();
}

bool same_handle(const hipIpcMemHandle_t &x, const hipIpcMemHandle_t &y) {
    return memcmp(&x, &y, sizeof(x)) == 0;
}

bool same_alloc(const ipc_alloc &x, const ipc_alloc &y) {
    return x.pid == y.pid && x.id == y.id && x.base == y.base && x.size == y.size &&
           same_handle(x.h, y.h);
}

// the exporter's allocations x and y cannot both be alive
bool collide(const ipc_alloc &x, const ipc_alloc &y) {
    return x.pid == y.pid && ((x.base < y.base + y.size && y.base < x.base + x.size) ||
                              same_handle(x.h, y.h));
}

bool trace() {
    static const bool on = [] {
        const char *v = getenv("OMPI_AMD_IPC_TRACE");
        return v && *v == '1';
    }();
    return on;
}

void hold(ipc_ref *r, void *owner) {
    ++r->refs;
    ++g_st.refs;
    for (auto &h : r->holders)
        if (h.first == owner) {
            ++h.second;
            return;
        }
    r->holders.push_back({owner, 1});
}

// (g_mu released) the runtime close; the stats under the lock
// OMPI_AMD_TRACE=1: the runtime's IPC opens and closes with their duration
// (a close may wait for every kernel of the device)
struct reg_step {
    const char *what;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit reg_step(const char *w) : what(w) {
        static const bool on = getenv("OMPI_AMD_TRACE") && *getenv("OMPI_AMD_TRACE") == '1';
        if (on) fprintf(stderr, "[trace pid %d] %s ...\n", (int)getpid(), what);
    }
    ~reg_step() {
        static const bool on = getenv("OMPI_AMD_TRACE") && *getenv("OMPI_AMD_TRACE") == '1';
        if (!on) return;
        const double ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        fprintf(stderr, "[trace pid %d] %s done %.3f ms\n", (int)getpid(), what, ms);
    }
};

void close_mapping(ipc_ref *r) {
    reg_step st("hipIpcCloseMemHandle");
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipIpcCloseMemHandle(r->base);
    hip_ignore(e);
    note_close();
    if (trace())
        fprintf(stderr, "[ipc pid %d] close pid %llu id %llu %p+%llu -> %p%s (%.3f ms)\n", (int)getpid(),
                (unsigned long long)r->a.pid, (unsigned long long)r->a.id,
                (void *)(uintptr_t)r->a.base, (unsigned long long)r->a.size, r->base,
                r->retired ? " (retired)" : "",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    std::lock_guard<std::mutex> g(g_mu);
    ++g_st.closes;
    --g_st.live;
}

void done_opening(const ipc_alloc &a) {
    for (auto it = g_opening.begin(); it != g_opening.end(); ++it)
        if (same_alloc(*it, a)) {
            g_opening.erase(it);
            break;
        }
    g_cv.notify_all();
}

}  // namespace

int ipc_map(const ipc_alloc &a, void *owner, ipc_ref **ref, void **base) {
    *ref = nullptr;
    *base = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return record_hip(hipErrorInvalidDevice, "hipGetDevice (ipc_map)");
    std::vector<ipc_ref *> stale;
    std::vector<user> quiet;  // the stale mappings' holders, quiesced before the close
    {
        std::unique_lock<std::mutex> g(g_mu);
        for (;;) {
            for (ipc_ref *r : g_live)
                if (r->device == dev && same_alloc(r->a, a)) {
                    hold(r, owner);
                    ++g_st.shared;
                    *ref = r;
                    *base = r->base;
                    return OMPI_AMD_SUCCESS;
                }
            // another thread opens this allocation or one it collides with:
            // wait for that open to finish, then look again
            // (or a retired mapping it collides with is still being closed:
            // the runtime would answer the open with that mapping)
            bool busy = false;
            for (const ipc_alloc &o : g_opening) busy = busy || collide(o, a);
            for (const ipc_alloc &o : g_closing) busy = busy || collide(o, a);
            if (!busy) break;
            g_cv.wait(g);
        }
        // The exporter's live allocations never overlap and never share
        // handle bytes: a mapping that does either belongs to an allocation
        // it freed.  It must be closed BEFORE the new handle is opened (the
        // runtime would answer the open with it).  A pinned one is a program
        // error.
        for (ipc_ref *r : g_live)
            if (r->device == dev && collide(r->a, a)) stale.push_back(r);
        for (ipc_ref *r : stale)
            if (r->pins > 0) {
                record_msg("process %llu freed a device buffer (id %llu, %p + %llu) that a persistent "
                           "operation of this process still maps", (unsigned long long)a.pid,
                           (unsigned long long)r->a.id, (void *)(uintptr_t)r->a.base,
                           (unsigned long long)r->a.size);
                return OMPI_AMD_ERR_BAD_PARAM;
            }
        for (ipc_ref *r : stale) {  // nobody shares it from now on
            r->retired = true;
            g_closing.push_back(r->a);
            ++r->refs;  // this retirement's own, until the close below
            ++g_st.retired;
            g_live.erase(std::find(g_live.begin(), g_live.end(), r));
            for (auto &h : r->holders)
                for (auto &u : g_users)
                    if (u.owner == h.first &&
                        std::none_of(quiet.begin(), quiet.end(),
                                     [&](const user &q) { return q.owner == u.owner; })) {
                        ++u.busy;
                        quiet.push_back(u);
                    }
        }
        g_opening.push_back(a);
    }
    // Only the holders of the stale mappings can have device work reading
    // through them: each drains its own streams (not every communicator's —
    // one with a deferred call waiting for a peer must not be waited for
    // here, and the exporter's free already implies the holders' reads of
    // the freed buffer completed: every collective ends with a barrier).
    int rc = OMPI_AMD_SUCCESS;
    for (const user &u : quiet) {
        const int q = u.quiesce(u.owner);
        if (rc == OMPI_AMD_SUCCESS) rc = q;
    }
    {
        std::lock_guard<std::mutex> g(g_mu);
        for (const user &q : quiet)
            for (auto &u : g_users)
                if (u.owner == q.owner) --u.busy;
        g_cv.notify_all();
    }
    for (ipc_ref *r : stale) {
        close_mapping(r);
        std::lock_guard<std::mutex> g(g_mu);
        for (auto it = g_closing.begin(); it != g_closing.end(); ++it)
            if (same_alloc(*it, r->a)) {
                g_closing.erase(it);
                break;
            }
        g_cv.notify_all();
        if (--r->refs == 0) delete r;  // else freed by its last holder's ipc_unmap
    }
    if (rc != OMPI_AMD_SUCCESS) {
        std::lock_guard<std::mutex> g(g_mu);
        done_opening(a);
        return rc;
    }
    // One open, never retried: the exportable allocations are sized so that
    // the runtime answers, and no exporter hands out an
    // allocation a close of its own spoiled (ipc_close_watermark) — a
    // refusal is an error, reported with the buffer.
    void *m = nullptr;
    const auto t_open = std::chrono::steady_clock::now();
    hipError_t e;
    {
        reg_step st("hipIpcOpenMemHandle");
        e = hipIpcOpenMemHandle(&m, a.h, hipIpcMemLazyEnablePeerAccess);
    }
    const double open_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_open).count();
    std::lock_guard<std::mutex> g(g_mu);
    ++g_st.opens;
    done_opening(a);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        ++g_st.refusals;
        record_msg("hipIpcOpenMemHandle: %s (process %llu buffer id %llu at %p + %llu)",
                   hipGetErrorString(e), (unsigned long long)a.pid, (unsigned long long)a.id,
                   (void *)(uintptr_t)a.base, (unsigned long long)a.size);
        return OMPI_AMD_ERR_HIP;
    }
    // The answer must be a new mapping of the advertised allocation: not
    // inside one the process holds, with the exporter's base and size (the
    // runtime rounds the mapping up to its 2 MiB page).
    for (ipc_ref *r : g_live)
        if ((const char *)m >= (const char *)r->base &&
            (const char *)m < (const char *)r->base + r->a.size) {
            // not closed: that could unmap the live mapping it aliases
            record_msg("hipIpcOpenMemHandle returned %p for process %llu buffer id %llu, which is "
                       "this process's mapping of buffer id %llu of process %llu",
                       m, (unsigned long long)a.pid, (unsigned long long)a.id,
                       (unsigned long long)r->a.id, (unsigned long long)r->a.pid);
            return OMPI_AMD_ERR_HIP;
        }
    void *mb = nullptr;
    size_t ms = 0;
    if (hipMemGetAddressRange((hipDeviceptr_t *)&mb, &ms, (hipDeviceptr_t)m) == hipSuccess) {
        const uint64_t up = (a.size + (2u << 20) - 1) & ~(uint64_t)((2u << 20) - 1);
        if (mb != m || ms < a.size || ms > up) {
            hip_ignore(hipIpcCloseMemHandle(m));
            note_close();
            ++g_st.closes;
            record_msg("hipIpcOpenMemHandle for process %llu buffer id %llu (%llu bytes) returned "
                       "a mapping of %zu bytes at %p", (unsigned long long)a.pid,
                       (unsigned long long)a.id, (unsigned long long)a.size, ms, mb);
            return OMPI_AMD_ERR_HIP;
        }
    } else {
        (void)hipGetLastError();
    }
    auto *r = new ipc_ref;
    r->a = a;
    r->device = dev;
    r->base = m;
    hold(r, owner);
    g_live.push_back(r);
    ++g_st.live;
    if (trace())
        fprintf(stderr, "[ipc pid %d] open pid %llu id %llu %p+%llu -> %p (%.3f ms)\n", (int)getpid(),
                (unsigned long long)a.pid, (unsigned long long)a.id, (void *)(uintptr_t)a.base,
                (unsigned long long)a.size, m, open_ms);
    *ref = r;
    *base = m;
    return OMPI_AMD_SUCCESS;
}

void ipc_unmap(ipc_ref *r, void *owner) {
    if (!r) return;
    bool close = false;
    {
        std::lock_guard<std::mutex> g(g_mu);
        --g_st.refs;
        for (auto it = r->holders.begin(); it != r->holders.end(); ++it)
            if (it->first == owner) {
                if (--it->second == 0) r->holders.erase(it);
                break;
            }
        if (--r->refs > 0) return;
        if (r->retired) {  // already closed by the open that retired it
            delete r;
            return;
        }
        g_live.erase(std::find(g_live.begin(), g_live.end(), r));
        close = true;
    }
    if (close) {
        close_mapping(r);
        delete r;
    }
}

void ipc_pin(ipc_ref *r, int delta) {
    if (!r) return;
    std::lock_guard<std::mutex> g(g_mu);
    r->pins += delta;
}

bool ipc_retired(const ipc_ref *r) {
    std::lock_guard<std::mutex> g(g_mu);
    return r && r->retired;
}

void *ipc_ref_base(const ipc_ref *r) { return r ? r->base : nullptr; }

void ipc_add_user(void *owner, int (*quiesce)(void *)) {
    std::lock_guard<std::mutex> g(g_mu);
    g_users.push_back({owner, quiesce, 0});
}

void ipc_remove_user(void *owner) {
    std::unique_lock<std::mutex> g(g_mu);
    // another thread's open may be draining this user's streams right now
    g_cv.wait(g, [&] {
        for (const user &u : g_users)
            if (u.owner == owner && u.busy > 0) return false;
        return true;
    });
    g_users.erase(std::remove_if(g_users.begin(), g_users.end(),
                                 [&](const user &u) { return u.owner == owner; }),
                  g_users.end());
}

uint64_t ipc_close_watermark() {
    free_probes();
    return g_close_mark.load();
}

ipc_stats ipc_get_stats() {
    std::lock_guard<std::mutex> g(g_mu);
    return g_st;
}

}  // namespace ompi_amd
