// Node-local rendezvous over a POSIX shared-memory segment.
//
// The reference bootstraps through PMIx/the runtime and moves every byte
// through btl/sm's shared segments (opal/mca/btl/sm/btl_sm_component.c).
// Here the segment carries only control data: each rank's slot holds a
// sequence word and two exchange blobs (double-buffered by sequence
// parity), which is enough for an allgather of IPC handles and a host
// barrier.  Payload never goes through it.
#pragma once

#include <cstddef>
#include <cstdint>

namespace ompi_amd {

class ShmBoot {
  public:
    static constexpr size_t kBlob = 2048;

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

  private:
    struct Slot;
    Slot *slot(int r) const;
    char name_[256] = {0};
    void *map_ = nullptr;
    size_t bytes_ = 0;
    int rank_ = -1, size_ = 0;
    uint64_t seq_ = 0;
    double timeout_s_ = 60.0;
    bool unlinked_ = false;
};

}  // namespace ompi_amd
