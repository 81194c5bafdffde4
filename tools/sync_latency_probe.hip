// Launch-to-host-observed completion latency of one tiny kernel, by the way
// the host waits: hipStreamSynchronize, hipEventSynchronize, or polling
// hipStreamQuery / hipEventQuery (with and without sched_yield).  One JSON
// line per mode (mean and median over the iterations, µs).
//
// build: hipcc --offload-arch=gfx950 -O2 tools/sync_latency_probe.hip -o tools/sync_latency_probe
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void tiny(int *p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

// the same work, then a system-scope store of `v` into host memory the CPU
// spins on (vector store; the host sees it over PCIe)
__global__ void tiny_flag(int *p, int *hflag, int v) {
    if (threadIdx.x == 0) {
        p[blockIdx.x] += 1;
        __hip_atomic_store(hflag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main() {
    int *buf = nullptr;
    CK(hipMalloc(&buf, 4096));
    CK(hipMemset(buf, 0, 4096));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    int *hflag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&hflag), 64, hipHostMallocCoherent));
    *hflag = 0;
    const char *names[] = {"stream_sync", "event_sync", "stream_query_spin", "event_query_spin",
                           "event_query_yield", "host_flag_spin", "launch_only"};
    const int iters = 2000;
    for (int mode = 0; mode < 7; ++mode) {
        std::vector<double> t;
        for (int i = 0; i < iters + 50; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            const int v = mode * 100000 + i + 1;
            if (mode == 5)
                hipLaunchKernelGGL(tiny_flag, dim3(1), dim3(64), 0, s, buf, hflag, v);
            else
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, buf);
            if (mode == 5) {
                while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != v) {
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                        fprintf(stderr, "host flag never arrived\n");
                        return 1;
                    }
                }
            } else if (mode == 6) {
                // launch cost alone (host side of hipLaunchKernelGGL)
            } else if (mode == 0) {
                CK(hipStreamSynchronize(s));
            } else if (mode == 1) {
                CK(hipEventRecord(ev, s));
                CK(hipEventSynchronize(ev));
            } else if (mode == 2) {
                while (hipStreamQuery(s) == hipErrorNotReady) {
                }
            } else {
                CK(hipEventRecord(ev, s));
                while (hipEventQuery(ev) == hipErrorNotReady)
                    if (mode == 4) sched_yield();
            }
            const double us =
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (i >= 50) t.push_back(us);
            if (mode >= 5) CK(hipStreamSynchronize(s));
        }
        double sum = 0;
        for (double v : t) sum += v;
        std::sort(t.begin(), t.end());
        printf("{\"mode\": \"%s\", \"mean_us\": %.2f, \"median_us\": %.2f, \"p90_us\": %.2f}\n",
               names[mode], sum / t.size(), t[t.size() / 2], t[t.size() * 9 / 10]);
    }
    CK(hipStreamSynchronize(s));
    CK(hipEventDestroy(ev));
    CK(hipStreamDestroy(s));
    CK(hipFree(buf));
    CK(hipHostFree(hflag));
    return 0;
}
