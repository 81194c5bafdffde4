// Host-observed completion marks and the library's host-side waits.
//
// A one-wave kernel enqueued after a call's work stores a sequence number
// into a word of pinned, coherent host memory (system scope, written through);
// the host spins on that word.  Launch to observed completion of a tiny
// kernel on MI355X: 6.3 µs this way, 11.8 µs polling hipEventQuery, 11.2 µs
// inside hipStreamSynchronize, 17.6 µs polling hipStreamQuery
// (tools/sync_latency_probe.hip, profiles/r04_sync_latency_probe.jsonl).
// Stream order puts the mark after every earlier kernel of the stream — the
// point an event recorded there marks — and a query of the stream or of an
// event recorded beside the mark stays the backstop (errors, a mark that
// never arrives).  OMPI_AMD_HOST_MARKS=0 turns marks off (events only).
#pragma once
#include <hip/hip_runtime.h>
#include <sched.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>

namespace ompi_amd {

uint64_t *mark_word_get();      // nullptr when marks are off or pinned memory is refused
void mark_word_put(uint64_t *w);
// enqueue the mark on `s`: the value to wait for, 0 if none was launched
uint64_t mark_launch(uint64_t *w, hipStream_t s);
// the next mark value, for a kernel that stores its own mark (the fused
// small allreduce's last workgroup, ompi_amd_allreduce_wait)
uint64_t mark_reserve();

inline bool mark_seen(const uint64_t *w, uint64_t v) {
    return w && v && __atomic_load_n(w, __ATOMIC_ACQUIRE) >= v;
}

// Poll `query(spins)` until it answers something other than NotReady,
// running `idle()` between polls.  The first 2 ms poll with the core
// yielded: a small call completes in a few µs and any sleep costs at least
// the kernel's timer slack (50 µs by default; usleep(20) measured 77 µs per
// wait, tools/nb_latency_probe.py).  Longer waits sleep 50 µs per poll.
template <class Q, class I>
hipError_t poll_wait(Q query, I idle) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 0;; ++spins) {
        const hipError_t e = query(spins);
        if (e != hipErrorNotReady) return e;
        idle();
        if (spins < 256) continue;
        if (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2))
            sched_yield();
        else
            usleep(50);
    }
}

// Everything enqueued on `s` so far is done: through this thread's mark
// word (hipStreamQuery every 64 polls reports errors and an idle stream),
// or, without marks, an event recorded on `s`.
//
// host_reads: the caller reads host memory the GPU wrote on `s` (a
// device-to-host copy) once this returns.  A mark then proves nothing: the
// copy's kernel may have ended with an agent-scope release (the runtime
// relaxes it when a kernel follows on the stream), leaving host lines in
// some XCD's L2 — and a fence inside the one-wave mark kernel writes back
// only its own XCD's L2.  Such waits use the event, whose completion the
// runtime makes host-visible.
template <class I>
hipError_t mark_stream_wait(hipStream_t s, I idle, bool host_reads = false) {
    static thread_local uint64_t *word = mark_word_get();
    const uint64_t v = host_reads ? 0 : mark_launch(word, s);
    if (v)
        return poll_wait(
            [s, v](unsigned spins) {
                if (mark_seen(word, v)) return hipSuccess;
                return spins % 64 == 63 ? hipStreamQuery(s) : hipErrorNotReady;
            },
            idle);
    static thread_local hipEvent_t evs[64] = {};
    int dev = 0;
    hipDevice_t sdev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess && hipStreamGetDevice(s, &sdev) != hipSuccess) {
        (void)hipGetLastError();
        sdev = -1;
    }
    // an event of this device records only into this device's streams
    if (e != hipSuccess || dev < 0 || dev >= 64 || sdev != dev)
        return poll_wait([s](unsigned) { return hipStreamQuery(s); }, idle);
    if (!evs[dev]) {
        e = hipEventCreateWithFlags(&evs[dev], hipEventDisableTiming);
        if (e != hipSuccess) {
            evs[dev] = nullptr;
            return e;
        }
    }
    hipEvent_t ev = evs[dev];
    e = hipEventRecord(ev, s);
    if (e != hipSuccess) return e;
    return poll_wait([ev](unsigned) { return hipEventQuery(ev); }, idle);
}

// A mark some kernel already on `s` stores itself: its value, or the
// stream's own completion (hipStreamQuery every 64 polls: errors, and a
// kernel that gave up before its mark).
template <class I>
hipError_t mark_value_wait(hipStream_t s, const uint64_t *w, uint64_t v, I idle) {
    return poll_wait(
        [s, w, v](unsigned spins) {
            if (mark_seen(w, v)) return hipSuccess;
            return spins % 64 == 63 ? hipStreamQuery(s) : hipErrorNotReady;
        },
        idle);
}

// An event and the mark (value v in w) enqueued right after it: whichever
// shows first.
template <class I>
hipError_t mark_event_wait(hipEvent_t ev, const uint64_t *w, uint64_t v, I idle) {
    if (!v) return poll_wait([ev](unsigned) { return hipEventQuery(ev); }, idle);
    return poll_wait(
        [ev, w, v](unsigned spins) {
            if (mark_seen(w, v)) return hipSuccess;
            return spins % 64 == 63 ? hipEventQuery(ev) : hipErrorNotReady;
        },
        idle);
}

inline void no_idle() {}

}  // namespace ompi_amd
