// Process-wide registry of the IPC mappings this process holds of its peers'
// device allocations.  Internal (not part of the C ABI).
//
// ROCm 7.2 answers hipIpcOpenMemHandle for an exporter address this process
// already maps with that existing mapping, so a mapping is
// a property of the process, not of the communicator, window or message
// that opened it.  Every open in libompi_amd.so goes through ipc_map and
// every close through ipc_unmap: one mapping per peer allocation, shared by
// every communicator, window and point-to-point transfer that uses it,
// refcounted, and closed only when the last user lets go — the reference's
// per-endpoint registration cache (btl_smcuda.c:519, :1083-1136;
// common_cuda.c:1127-1135 treats CUDA_ERROR_ALREADY_MAPPED as exactly this
// sharing).  An allocation the exporter freed (a newer allocation of that
// process overlaps its range or repeats its handle bytes) is retired here,
// once, for every holder: its mapping is closed after every registered user
// has drained its device work, before the newer allocation is opened.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ompi_amd {

// A peer allocation as its exporter described it (buf_desc / ipc_desc).
struct ipc_alloc {
    hipIpcMemHandle_t h;
    uint64_t pid;   // exporter process
    uint64_t id;    // HIP_POINTER_ATTRIBUTE_BUFFER_ID in the exporter
    uint64_t base;  // the allocation's range in the exporter's address space
    uint64_t size;
};

struct ipc_ref;  // one registry entry (opaque)

// Map a peer allocation, or share the mapping the process already holds of
// it: one more reference, held by `owner` (a registered user, see below).
// *base = the mapping of the allocation's first byte.  Mappings the new
// allocation collides with are retired first: only their holders are
// quiesced, and no lock is held across the quiesce, the close or the open.
int ipc_map(const ipc_alloc &a, void *owner, ipc_ref **ref, void **base);
// Drop one of owner's references; the last one closes the mapping (the
// caller has made sure none of its own device work still uses it).
void ipc_unmap(ipc_ref *ref, void *owner);
// A persistent operation holds the mapping (MPI_Allreduce_init, a window):
// an exporter that frees the allocation meanwhile is a program error that
// the next open of its newer allocation reports instead of unmapping.
void ipc_pin(ipc_ref *ref, int delta);
// The exporter freed the allocation (retired): the holder must drop it.
bool ipc_retired(const ipc_ref *ref);
void *ipc_ref_base(const ipc_ref *ref);

// Users of mappings (communicators) register a function that waits for all
// of their device work; retiring a mapping runs it for each user holding a
// reference to the mapping.  The function may run on another thread than
// the user's own (it must be safe against the user's concurrent calls).
void ipc_add_user(void *owner, int (*quiesce)(void *owner));
void ipc_remove_user(void *owner);

// Closing an IPC mapping spoils the exportability of device allocations
// this process already has: ROCm 7.2's hipIpcGetMemHandle then refuses
// ("invalid argument"), for good, 10-30 % of the allocations that existed
// at the close, and none made after it (tools/ipc_p2p_replay.py,
// profiles/r05_ipc_p2p_replay*.jsonl: the round-4 refused exports).  Every
// close here records the buffer id of an allocation made right after it
// (HIP_POINTER_ATTRIBUTE_BUFFER_ID grows with every allocation): an
// allocation with a lower id predates a close and is not exported unless it
// was exported before (its handle stays valid); callers send it through a
// library stage or shadow instead.
uint64_t ipc_close_watermark();

struct ipc_stats {
    int64_t opens;        // hipIpcOpenMemHandle calls made
    int64_t refusals;     // opens the runtime refused (each one failed its call)
    int64_t closes;       // hipIpcCloseMemHandle calls made
    int64_t shared;       // ipc_map answered from a mapping the process held
    int64_t retired;      // mappings retired because the exporter freed the allocation
    int64_t live;         // mappings open now
    int64_t refs;         // references held now
};
ipc_stats ipc_get_stats();

}  // namespace ompi_amd
