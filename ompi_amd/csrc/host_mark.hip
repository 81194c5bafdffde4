// Host-observed completion marks (host_mark.h): the mark kernel and the
// pool of pinned host words.
#include "host_mark.h"

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace ompi_amd {

// A relaxed system-scope store (written through to host memory): the
// earlier kernels of the stream completed, with their own end-of-dispatch
// release, before this one started, so no fence is needed here — a release
// fence at system scope writes back the L2 first (3.2 µs average kernel
// time with it, profiles/r04_seam_kernel_stats_release.csv).
__global__ void host_mark_kernel(uint64_t *word, uint64_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static std::mutex g_mark_mu;
static std::vector<uint64_t *> g_mark_free;  // words of pinned pages (never returned)
static std::atomic<uint64_t> g_mark_seq{0};  // monotonic: a reused word only grows

uint64_t *mark_word_get() {
    static const bool on = [] {
        const char *e = getenv("OMPI_AMD_HOST_MARKS");
        return !(e && atoi(e) == 0);
    }();
    if (!on) return nullptr;
    std::lock_guard<std::mutex> g(g_mark_mu);
    if (g_mark_free.empty()) {
        void *pg = nullptr;
        if (hipHostMalloc(&pg, 4096, hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        auto *w = static_cast<uint64_t *>(pg);
        for (int k = 0; k < 4096 / 64; ++k) {  // one word per 64-B line
            w[k * 8] = 0;
            g_mark_free.push_back(w + k * 8);
        }
    }
    uint64_t *w = g_mark_free.back();
    g_mark_free.pop_back();
    return w;
}

// A word goes back once its holder's wait is over (its mark landed, or the
// wait failed: a late mark then only writes a smaller value, which a later
// holder's backstop query covers).
void mark_word_put(uint64_t *w) {
    if (!w) return;
    std::lock_guard<std::mutex> g(g_mark_mu);
    g_mark_free.push_back(w);
}

uint64_t mark_reserve() { return g_mark_seq.fetch_add(1) + 1; }

uint64_t mark_launch(uint64_t *w, hipStream_t s) {
    if (!w) return 0;
    const uint64_t v = mark_reserve();
    hipLaunchKernelGGL(host_mark_kernel, dim3(1), dim3(64), 0, s, w, v);
    if (hipGetLastError() != hipSuccess) return 0;
    return v;
}

}  // namespace ompi_amd
