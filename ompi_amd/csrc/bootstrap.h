// Node-local rendezvous over a POSIX shared-memory segment.
//
// The reference bootstraps through PMIx/the runtime and moves every byte
// through btl/sm's shared segments (opal/mca/btl/sm/btl_sm_component.c).
// Here the segment carries only control data: each rank's slot holds a
// posted-sequence word, a consumed-sequence word and a ring of kRing
// exchange blobs, which is enough for an allgather of IPC handles and a host
// barrier.  Payload never goes through it.
//
// An allgather can be split: post() publishes this rank's blob and returns
// its ticket without waiting; test() completes tickets in order once every
// rank has posted.  Up to kRing - 1 tickets may be outstanding (a post
// waits only for ring slots every rank has consumed) — the nonblocking
// collectives post at call time (or, while the ring is full, from progress:
// can_post) and complete from progress.
#pragma once

#include <cstddef>
#include <cstdint>

namespace ompi_amd {

// Called while a rendezvous waits for a peer (coll_ipc.hip: launches other
// communicators' ready nonblocking calls, MPI's progress rule).
void set_boot_idle_hook(void (*fn)());

class ShmBoot {
  public:
    static constexpr size_t kBlob = 2048;
    static constexpr uint64_t kRing = 8;

    ShmBoot() = default;
    ~ShmBoot();
    ShmBoot(const ShmBoot &) = delete;
    ShmBoot &operator=(const ShmBoot &) = delete;

    // Attach (rank 0 creates).  Returns OMPI_AMD_* status.
    int attach(const char *name, int rank, int size, double timeout_s);
    void detach();
    // Every rank contributes `len` (<= kBlob) bytes; `all` receives size*len.
    int allgather(const void *mine, void *all, size_t len);
    int barrier() { return allgather(nullptr, nullptr, 0); }
    // Split allgather.  post(): *ticket = this contribution's sequence.
    // test(): tickets complete in posting order; *ready = 1 once every rank
    // posted `ticket` (then `all` holds the blobs), 0 if not yet.  With
    // block = true it waits (bounded by the attach timeout).
    int post(const void *mine, size_t len, uint64_t *ticket);
    int test(uint64_t ticket, void *all, size_t len, bool block, bool *ready);
    // post() would not wait: the ring slot it overwrites was read by every rank
    bool can_post() const;
    uint64_t posted() const { return seq_; }
    uint64_t consumed() const { return done_; }

  private:
    struct Slot;
    Slot *slot(int r) const;
    char name_[256] = {0};
    void *map_ = nullptr;
    size_t bytes_ = 0;
    int rank_ = -1, size_ = 0;
    uint64_t seq_ = 0, done_ = 0;
    double timeout_s_ = 60.0;
    bool unlinked_ = false;
};

}  // namespace ompi_amd
