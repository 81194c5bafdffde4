// Services of the communicator (coll_ipc.hip) used by the point-to-point
// (p2p.cpp) and one-sided (osc_ipc.hip) parts of libompi_amd.so.  Internal:
// not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/ompi_amd_coll.h"

namespace ompi_amd {

// A device buffer as peers see it: its allocation's IPC handle + offset,
// plus the allocation's identity in the exporter (process, HIP buffer id,
// base address, size).  Mappings are shared process-wide through the IPC
// registry (ipc_registry.h), which retires a mapping once the exporter's
// newer allocation overlaps its range (live allocations never overlap).
struct ipc_desc {
    hipIpcMemHandle_t h;
    uint64_t off;
    uint64_t valid;
    uint64_t id;
    uint64_t base;
    uint64_t size;
    uint64_t pid;
};

struct p2p_state;  // p2p.cpp

int comm_rank(const ompi_amd_comm_t *c);
int comm_size(const ompi_amd_comm_t *c);
int comm_device(const ompi_amd_comm_t *c);
int64_t comm_timeout_ms(const ompi_amd_comm_t *c);
int *comm_err_dev(ompi_amd_comm_t *c);
// Host rendezvous: every rank contributes len (<= 2048) bytes.
int comm_allgather(ompi_amd_comm_t *c, const void *mine, void *all, size_t len);
// A fresh device allocation whose IPC handle no earlier allocation of this
// process had (uncached: fine-grained), described in *d.
int comm_alloc_exportable(size_t bytes, bool uncached, void **out, ipc_desc *d);
// Give back memory from comm_alloc_exportable (kept for a later request of
// the same size instead of freed; anything else is freed).
void comm_release_exportable(void *p);
// Device memory from the communicator's exported arena (the shadow arena:
// chunks exported once, mapped by each peer once, freed at comm_destroy),
// so a peer maps nothing new per buffer.  comm_arena_free: once no peer
// touches the range any more.
int comm_arena_alloc(ompi_amd_comm_t *c, size_t bytes, void **out);
void comm_arena_free(ompi_amd_comm_t *c, void *p);
// Export a device buffer (cached per allocation).
int comm_export(ompi_amd_comm_t *c, const void *ptr, ipc_desc *d);
// Whether peers can map ptr's allocation as it is: an IPC-safe size (a
// multiple of 2 MiB from 4 MiB) within the mapping limit,
// and not spoiled by a later IPC close of this process unless exported
// before it (ipc_close_watermark).  A caller with a library stage sends
// other allocations through it.
bool comm_ipc_safe(const void *ptr);
// MPI_Win_create over base: run it through a public copy (separate model)?
// Not IPC-safe (above), or param osc_win_shadow; counted (osc_shadow_windows).
// Whether a window may run in the separate model (param osc_win_separate;
// osc/rocm's osc_rocm_separate_model): otherwise a window that needs a
// public copy fails on every rank.
bool comm_win_separate_ok(ompi_amd_comm_t *c);
bool comm_win_needs_shadow(ompi_amd_comm_t *c, const void *base);
// Map a peer's exported buffer (cached, LRU).  pin: held until comm_unpin.
int comm_import(ompi_amd_comm_t *c, int peer, const ipc_desc &d, const char **out, bool pin,
                void **base);
void comm_unpin(ompi_amd_comm_t *c, void *base);
// Launch the deferred nonblocking collectives (device work keeps one order).
int comm_drain(ompi_amd_comm_t *c);
// Device barrier over every rank of c on stream s (stream-ordered epoch).
int comm_barrier(ompi_amd_comm_t *c, hipStream_t s);
// The stream a call of c runs on: the caller's, or the communicator's own
// (param own_stream; coll_ipc.hip comm_stream).
hipStream_t comm_call_stream(ompi_amd_comm_t *c, void *stream);
// The sticky device error word (a barrier or lock that timed out).
int comm_sticky(ompi_amd_comm_t *c);
// Byte copy kernel (16-/4-/1-byte granules by the common phase of src and
// dst; src or dst may be peer memory), system-scope acquire/release.
int comm_copy(ompi_amd_comm_t *c, const void *src, void *dst, size_t bytes, hipStream_t s);
// p2p eager cells (osc_ipc.hip, one workgroup, bytes <= 4 KiB): eager_put
// copies src into the cell, then stores v into *flag (system scope, after a
// release); eager_get waits (bounded by ticks of s_memrealtime: err set,
// nothing copied) until *flag == v, then copies the cell out.  Both store
// mark_v into the pinned host word *mark (when not null) as their last
// action, so the host sees completion without an event (host_mark.h).
int eager_put(const void *src, char *cell, size_t bytes, uint64_t *flag, uint64_t v, uint64_t *mark,
              uint64_t mark_v, hipStream_t s);
int eager_get(const char *cell, void *dst, size_t bytes, const uint64_t *flag, uint64_t v, int *err,
              uint64_t ticks, uint64_t *mark, uint64_t mark_v, hipStream_t s);
// osc_ipc.hip: the byte copy of put / get and the p2p receive (persistent
// grid, one acquire per workgroup; src or dst may be peer memory).
// gate: a CTL_TAKEN_* word that must read 1 for the copy to run (NULL: none).
// remote_dst: dst is memory of another GPU (a per-workgroup system-scope
// release ends the copy); false: this GPU's memory (the kernel boundary's
// release covers it).
int xfer_copy(const void *src, void *dst, size_t bytes, hipStream_t s,
              const uint32_t *gate = nullptr, bool remote_dst = true);
// The same copy with device-side signalling (p2p staged messages): every
// workgroup first waits until *wait == wait_v (bounded by ticks: *err set,
// nothing copied; wait NULL: no wait); after the last workgroup finished
// (counter *done, zero at rest, reset by that workgroup) *flag = flag_v
// (system scope, after a release) and the pinned host word *mark = mark_v,
// each when not NULL.
struct xfer_sig {
    const uint64_t *wait = nullptr;
    uint64_t wait_v = 0;
    int *err = nullptr;
    uint64_t ticks = 0;
    uint64_t *flag = nullptr;
    uint64_t flag_v = 0;
    uint64_t *mark = nullptr;
    uint64_t mark_v = 0;
    uint32_t *done = nullptr;
};
int xfer_copy_sig(const void *src, void *dst, size_t bytes, hipStream_t s, const xfer_sig &sig);
// Point-to-point mailboxes of the communicator (created with it).
p2p_state *comm_p2p(ompi_amd_comm_t *c);
// The one-sided part's per-communicator state (NULL until it sets one).
// ompi_amd_comm_destroy calls release(state, 0) after its first barrier
// (nobody reads this rank's memory any more: drop peer mappings) and
// release(state, 1) after its second (every peer dropped its mappings:
// free this rank's memory).
void *comm_osc_state(ompi_amd_comm_t *c);
void comm_set_osc_state(ompi_amd_comm_t *c, void *state, void (*release)(void *, int));

// p2p.cpp: created by ompi_amd_comm_create in two phases around its first
// rendezvous (rank 0 creates the segment before it, the others map it
// after), released by ompi_amd_comm_destroy.
int p2p_create(ompi_amd_comm_t *c, const char *name, int rank, int size, int phase,
               p2p_state **out);
void p2p_unlink(p2p_state *p);
// Point-to-point parameters / counters ("p2p_*" keys of comm set/get_param);
// OMPI_AMD_ERR_UNSUPPORTED for a key that is not one of them.
int p2p_set_param(p2p_state *p, const char *key, int64_t v);
int p2p_get_param(p2p_state *p, const char *key, int64_t *v);
void p2p_destroy(p2p_state *p);

}  // namespace ompi_amd
