// Host runtime helpers: error capture, per-thread streams, pointer queries.
#include "host_mark.h"
#include "runtime.h"

#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace ompi_amd {

static thread_local char tls_err[512] = "";
static thread_local hipStream_t tls_stream = nullptr;

// OMPI_AMD_TRACE=1: every recorded error also goes to stderr when it is
// recorded (a rank that fails inside progress names its cause even if the
// call that reports it never comes)
static bool trace_errors() {
    static const bool on = getenv("OMPI_AMD_TRACE") && *getenv("OMPI_AMD_TRACE") == '1';
    return on;
}

int record_hip(hipError_t e, const char *what) {
    if (e == hipSuccess) return OMPI_AMD_SUCCESS;
    (void)hipGetLastError();  // reported through the status: not left for the application's checks
    snprintf(tls_err, sizeof(tls_err), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    if (trace_errors()) fprintf(stderr, "[trace pid %d] error: %s\n", (int)getpid(), tls_err);
    return OMPI_AMD_ERR_HIP;
}

void record_msg(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(tls_err, sizeof(tls_err), fmt, ap);
    va_end(ap);
    if (trace_errors()) fprintf(stderr, "[trace pid %d] error: %s\n", (int)getpid(), tls_err);
}

hipStream_t thread_stream() { return tls_stream ? tls_stream : hipStreamPerThread; }

// Deployment requirement: peers map each other's memory
// with hipIpcOpenMemHandle, which on this driver stack works only in the
// dmabuf IPC mode (HSA_ENABLE_IPC_MODE_LEGACY=0; the legacy mode fails with
// "hipIpcGetMemHandle: invalid argument").  The HSA runtime reads the
// variable once, when it initialises, so the library sets it when it is
// loaded unless the environment already says otherwise — before any HIP
// call this library makes.  A process whose GPU was initialised before
// the library was loaded keeps the mode it started with; the communicator
// reports both (param "ipc_mode_legacy_env").
static int g_ipc_env_at_load = -2;

__attribute__((constructor)) static void ipc_mode_default() {
    const char *v = getenv("HSA_ENABLE_IPC_MODE_LEGACY");
    g_ipc_env_at_load = v ? atoi(v) : -1;
    if (!v) setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0);
}

int ipc_mode_env_at_load() { return g_ipc_env_at_load; }

// OMPI_AMD_BACKTRACE=1 (diagnostics): a host SIGSEGV / SIGBUS prints the
// raw call stack (library offsets, for addr2line on the same .so) to stderr
// before the default action.
static void crash_trace(int sig) {
    void *pc[64];
    const int n = backtrace(pc, 64);
    static const char head[] = "[ompi_amd] fatal signal, call stack:\n";
    (void)!write(2, head, sizeof(head) - 1);
    backtrace_symbols_fd(pc, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

// ... and SIGUSR2 prints the main thread's stack and continues (a hung
// rank's launcher sends it before the kill: tests/test_coll_gpu.py run_ranks)
static void stack_dump(int sig) {
    if (syscall(SYS_gettid) != getpid()) {  // delivered to another thread: pass it on
        syscall(SYS_tgkill, getpid(), getpid(), sig);
        return;
    }
    void *pc[64];
    const int n = backtrace(pc, 64);
    static const char head[] = "[ompi_amd] SIGUSR2 call stack:\n";
    (void)!write(2, head, sizeof(head) - 1);
    backtrace_symbols_fd(pc, n, 2);
}

__attribute__((constructor)) static void crash_trace_init() {
    const char *v = getenv("OMPI_AMD_BACKTRACE");
    if (!v || atoi(v) == 0) return;
    void *warm[2];
    (void)backtrace(warm, 2);  // loads the unwinder outside a handler
    signal(SIGSEGV, crash_trace);
    signal(SIGBUS, crash_trace);
    signal(SIGUSR2, stack_dump);
}

const char *ipc_mode_env_now() {
    const char *v = getenv("HSA_ENABLE_IPC_MODE_LEGACY");
    return v ? v : "";
}

}  // namespace ompi_amd

using namespace ompi_amd;

extern "C" {

const char *ompi_amd_version(void) { return "ompi_amd 0.1 gfx950"; }

const char *ompi_amd_last_error(void) { return tls_err; }

int ompi_amd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int ompi_amd_set_tuning(const char *key, int64_t value) {
    if (!key) return OMPI_AMD_ERR_BAD_PARAM;
    if (strcmp(key, "op_max_blocks") == 0) return op_set_max_blocks(value);
    record_msg("unknown tuning key '%s'", key);
    return OMPI_AMD_ERR_BAD_PARAM;
}

int ompi_amd_set_thread_stream(void *stream) {
    tls_stream = static_cast<hipStream_t>(stream);
    return OMPI_AMD_SUCCESS;
}

// hipPointerGetAttributes: device and managed memory run on the GPU;
// anything else (pageable or pinned host) is host memory for the handlers
// (common_cuda.c:1739-1792 counterpart).
int ompi_amd_is_device_pointer(const void *ptr) {
    if (ptr == nullptr) return 0;
    hipPointerAttribute_t attr;
    memset(&attr, 0, sizeof(attr));
    hipError_t e = hipPointerGetAttributes(&attr, ptr);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // unregistered host memory
        return 0;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

int ompi_amd_pointer_range(const void *ptr, void **base, size_t *size) {
    if (!base || !size) return OMPI_AMD_ERR_BAD_PARAM;
    *base = nullptr;
    *size = 0;
    if (!ompi_amd_is_device_pointer(ptr)) return 0;
    if (hipMemGetAddressRange((hipDeviceptr_t *)base, size, (hipDeviceptr_t)ptr) != hipSuccess) {
        (void)hipGetLastError();
        *base = const_cast<void *>(ptr);  // device, range unknown: this byte only
        *size = 1;
    }
    return 1;
}

}  // extern "C"

namespace ompi_amd {

// The op handlers classify every operand on every call (ompi_op_reduce has
// no residency hint).  A pure-host reduction (op/avx or op/base underneath)
// should not pay a runtime pointer query per operand per call: each thread
// remembers the last 8 host regions it classified, at 2 MiB granularity —
// only memory the runtime does not know at all (unregistered pageable:
// hipPointerGetAttributes fails), never pinned, registered or managed
// memory — and each remembered region is queried again after 1024 hits.
// Limitation: if such a region is unmapped and its addresses
// reused by an allocation the runtime does know (hipMallocManaged,
// hipHostRegister, an imported allocation), up to 1024 further calls of
// that thread may still classify it as host and take the host path; device
// pointers proper (the GPU's own aperture) are always queried.
int device_pointer_cached(const void *p) {
    static thread_local uintptr_t host_gran[8];  // granule + 1 (0 = empty)
    static thread_local unsigned hits[8];
    static thread_local unsigned next;
    if (!p) return 0;
    const uintptr_t g = ((uintptr_t)p >> 21) + 1;
    for (int i = 0; i < 8; ++i)
        if (host_gran[i] == g) {
            if (++hits[i] < 1024) return 0;
            host_gran[i] = 0;  // stale for too long: ask the runtime again
            break;
        }
    hipPointerAttribute_t attr;
    memset(&attr, 0, sizeof(attr));
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {  // unregistered host memory
        (void)hipGetLastError();
        const unsigned k = next++ & 7;
        host_gran[k] = g;
        hits[k] = 0;
        return 0;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

}  // namespace ompi_amd

extern "C" {

int ompi_amd_memcpy_async(void *dst, const void *src, size_t bytes, void *stream) {
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    if (!dst || !src) return OMPI_AMD_ERR_BAD_PARAM;
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : thread_stream();
    return record_hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s), "hipMemcpyAsync");
}

// The convertor's synchronous fAdvance waits here, and a send window's
// bytes are read from pinned host memory right after (fill_win): a host
// read, so the event wait (host_mark.h).
int ompi_amd_stream_synchronize(void *stream) {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : thread_stream();
    return record_hip(mark_stream_wait(s, no_idle, true), "hipStreamSynchronize");
}

int ompi_amd_memcpy(void *dst, const void *src, size_t bytes) {
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    if (!dst || !src) return OMPI_AMD_ERR_BAD_PARAM;
    hipStream_t s = thread_stream();
    int rc = record_hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s), "hipMemcpyAsync");
    if (rc == OMPI_AMD_SUCCESS)  // the host may read dst now: the event wait
        rc = record_hip(mark_stream_wait(s, no_idle, !ompi_amd_is_device_pointer(dst)),
                        "hipStreamSynchronize");
    return rc;
}

// Overlap-safe: through a temporary device buffer when the ranges overlap
// (the reference's cuda memmove does the same, common_cuda.c:1715-1737).
int ompi_amd_memmove(void *dst, void *src, size_t bytes) {
    if (bytes == 0 || dst == src) return OMPI_AMD_SUCCESS;
    const char *d = static_cast<const char *>(dst), *s = static_cast<const char *>(src);
    if (d + bytes <= s || s + bytes <= d) return ompi_amd_memcpy(dst, src, bytes);
    void *tmp = nullptr;
    int rc = record_hip(hipMalloc(&tmp, bytes), "hipMalloc (memmove)");
    if (rc == OMPI_AMD_SUCCESS) rc = ompi_amd_memcpy(tmp, src, bytes);
    if (rc == OMPI_AMD_SUCCESS) rc = ompi_amd_memcpy(dst, tmp, bytes);
    if (tmp) (void)hipFree(tmp);
    return rc;
}

int ompi_amd_device_alloc(void **ptr, size_t bytes) {
    if (!ptr) return OMPI_AMD_ERR_BAD_PARAM;
    *ptr = nullptr;
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    return record_hip(hipMalloc(ptr, bytes), "hipMalloc");
}

int ompi_amd_device_free(void *ptr) {
    if (!ptr) return OMPI_AMD_SUCCESS;
    return record_hip(hipFree(ptr), "hipFree");
}

int ompi_amd_host_alloc(void **ptr, size_t bytes) {
    if (!ptr) return OMPI_AMD_ERR_BAD_PARAM;
    *ptr = nullptr;
    if (bytes == 0) return OMPI_AMD_SUCCESS;
    return record_hip(hipHostMalloc(ptr, bytes, hipHostMallocDefault), "hipHostMalloc");
}

int ompi_amd_host_free(void *ptr) {
    if (!ptr) return OMPI_AMD_SUCCESS;
    return record_hip(hipHostFree(ptr), "hipHostFree");
}

int ompi_amd_event_record(void **event, void *stream) {
    if (!event) return OMPI_AMD_ERR_BAD_PARAM;
    if (!*event) {
        hipEvent_t e = nullptr;
        const int rc = record_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        if (rc != OMPI_AMD_SUCCESS) return rc;
        *event = e;
    }
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : thread_stream();
    return record_hip(hipEventRecord(static_cast<hipEvent_t>(*event), s), "hipEventRecord");
}

int ompi_amd_event_query(void *event) {
    if (!event) return OMPI_AMD_ERR_BAD_PARAM;
    const hipError_t e = hipEventQuery(static_cast<hipEvent_t>(event));
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        return 0;
    }
    return e == hipSuccess ? 1 : record_hip(e, "hipEventQuery");
}

int ompi_amd_event_synchronize(void *event) {
    if (!event) return OMPI_AMD_ERR_BAD_PARAM;
    return record_hip(hipEventSynchronize(static_cast<hipEvent_t>(event)), "hipEventSynchronize");
}

int ompi_amd_event_destroy(void *event) {
    if (!event) return OMPI_AMD_SUCCESS;
    return record_hip(hipEventDestroy(static_cast<hipEvent_t>(event)), "hipEventDestroy");
}

}  // extern "C"
