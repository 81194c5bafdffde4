// POSIX shared-memory rendezvous (see bootstrap.h).
#include "bootstrap.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>

#include "../../include/ompi_amd.h"
#include "runtime.h"

namespace ompi_amd {

namespace {
constexpr uint64_t kMagic = 0x6f6d70695f616d64ull;  // "ompi_amd"

struct Header {
    std::atomic<uint64_t> magic;
    uint64_t size;
    char pad[48];
};

double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
}  // namespace

struct ShmBoot::Slot {
    std::atomic<uint64_t> seq;   // last posted ticket
    std::atomic<uint64_t> done;  // last ticket whose blobs this rank has read
    char pad[48];
    char blob[kRing][kBlob];
};

ShmBoot::Slot *ShmBoot::slot(int r) const {
    return reinterpret_cast<Slot *>(static_cast<char *>(map_) + sizeof(Header) +
                                    (size_t)r * sizeof(Slot));
}

ShmBoot::~ShmBoot() { detach(); }

int ShmBoot::attach(const char *name, int rank, int size, double timeout_s) {
    if (!name || rank < 0 || size <= 0 || rank >= size) return OMPI_AMD_ERR_BAD_PARAM;
    snprintf(name_, sizeof(name_), "/ompi_amd_%s", name);
    for (char *c = name_ + 1; *c; ++c)
        if (*c == '/') *c = '_';
    rank_ = rank;
    size_ = size;
    timeout_s_ = timeout_s;
    bytes_ = sizeof(Header) + (size_t)size * sizeof(Slot);
    int fd = -1;
    const double t0 = now_s();
    if (rank == 0) {
        shm_unlink(name_);  // a stale segment of an old job with this name
        fd = shm_open(name_, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)bytes_) != 0) {
            record_msg("shm_open/ftruncate %s: %s", name_, strerror(errno));
            if (fd >= 0) close(fd);
            return OMPI_AMD_ERR_BOOTSTRAP;
        }
    } else {
        for (;;) {
            fd = shm_open(name_, O_RDWR, 0600);
            if (fd >= 0) {
                struct stat st;
                if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes_) break;
                close(fd);
                fd = -1;
            }
            if (now_s() - t0 > timeout_s) {
                record_msg("timed out waiting for %s", name_);
                return OMPI_AMD_ERR_BOOTSTRAP;
            }
            usleep(1000);
        }
    }
    map_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (map_ == MAP_FAILED) {
        map_ = nullptr;
        record_msg("mmap %s: %s", name_, strerror(errno));
        return OMPI_AMD_ERR_BOOTSTRAP;
    }
    Header *h = static_cast<Header *>(map_);
    if (rank == 0) {
        h->size = (uint64_t)size;
        h->magic.store(kMagic, std::memory_order_release);
    } else {
        while (h->magic.load(std::memory_order_acquire) != kMagic) {
            if (now_s() - t0 > timeout_s) {
                record_msg("timed out waiting for rank 0 to initialise %s", name_);
                return OMPI_AMD_ERR_BOOTSTRAP;
            }
            usleep(200);
        }
        if (h->size != (uint64_t)size) {
            record_msg("%s: size mismatch %llu vs %d", name_, (unsigned long long)h->size, size);
            return OMPI_AMD_ERR_BOOTSTRAP;
        }
    }
    seq_ = done_ = 0;
    int rc = barrier();  // everyone attached
    if (rc == OMPI_AMD_SUCCESS && rank == 0) {
        shm_unlink(name_);  // the mappings keep it alive; nothing leaks on a crash
        unlinked_ = true;
    }
    return rc;
}

void ShmBoot::detach() {
    if (map_) {
        munmap(map_, bytes_);
        map_ = nullptr;
    }
    if (rank_ == 0 && !unlinked_ && name_[0]) shm_unlink(name_);
    unlinked_ = true;
}

static void (*g_idle)() = nullptr;
void set_boot_idle_hook(void (*fn)()) { g_idle = fn; }

int ShmBoot::post(const void *mine, size_t len, uint64_t *ticket) {
    if (!map_ || len > kBlob) return OMPI_AMD_ERR_BAD_PARAM;
    const uint64_t s = seq_ + 1;
    // ring slot s % kRing last held ticket s - kRing: every rank must have
    // read it before it is overwritten
    const double t0 = now_s();
    if (s > kRing) {
        for (int r = 0; r < size_; ++r) {
            unsigned spins = 0;
            while (slot(r)->done.load(std::memory_order_acquire) < s - kRing) {
                if (++spins > 1024) {
                    if (now_s() - t0 > timeout_s_) {
                        record_msg("%s: rank %d never consumed rendezvous %llu", name_, r,
                                   (unsigned long long)(s - kRing));
                        return OMPI_AMD_ERR_TIMEOUT;
                    }
                    if (g_idle) g_idle();
                    sched_yield();
                }
            }
        }
    }
    Slot *me = slot(rank_);
    if (len) memcpy(me->blob[s % kRing], mine, len);
    me->seq.store(s, std::memory_order_release);
    seq_ = s;
    *ticket = s;
    return OMPI_AMD_SUCCESS;
}

bool ShmBoot::can_post() const {
    if (!map_) return false;
    const uint64_t s = seq_ + 1;
    if (s <= kRing) return true;
    for (int r = 0; r < size_; ++r)
        if (slot(r)->done.load(std::memory_order_acquire) < s - kRing) return false;
    return true;
}

int ShmBoot::test(uint64_t ticket, void *all, size_t len, bool block, bool *ready) {
    *ready = false;
    if (!map_ || len > kBlob || ticket != done_ + 1 || ticket > seq_) return OMPI_AMD_ERR_BAD_PARAM;
    const double t0 = now_s();
    for (int r = 0; r < size_; ++r) {
        Slot *p = slot(r);
        unsigned spins = 0;
        while (p->seq.load(std::memory_order_acquire) < ticket) {
            if (!block) return OMPI_AMD_SUCCESS;
            if (++spins > 1024) {
                if (now_s() - t0 > timeout_s_) {
                    record_msg("%s: rank %d never reached rendezvous %llu", name_, r,
                               (unsigned long long)ticket);
                    return OMPI_AMD_ERR_TIMEOUT;
                }
                if (g_idle) g_idle();
                sched_yield();
            }
        }
    }
    for (int r = 0; r < size_ && len; ++r)
        memcpy(static_cast<char *>(all) + (size_t)r * len, slot(r)->blob[ticket % kRing], len);
    done_ = ticket;
    slot(rank_)->done.store(ticket, std::memory_order_release);
    *ready = true;
    return OMPI_AMD_SUCCESS;
}

int ShmBoot::allgather(const void *mine, void *all, size_t len) {
    uint64_t t = 0;
    bool ready = false;
    int rc = post(mine, len, &t);
    if (rc == OMPI_AMD_SUCCESS) rc = test(t, all, len, true, &ready);
    return rc;
}

}  // namespace ompi_amd
