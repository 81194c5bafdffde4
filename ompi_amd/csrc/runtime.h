// Shared host-side runtime helpers of libompi_amd.so (error capture, streams).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/ompi_amd.h"

namespace ompi_amd {

// Record a HIP error (thread-local message) and map it to a status code.
int record_hip(hipError_t e, const char *what);
// Record a non-HIP failure message.
void record_msg(const char *fmt, ...);
// A HIP call whose failure is tolerated: clear the thread's last-error slot
// when (and only when) it failed, so that the application's next error check
// (torch reads hipGetLastError after its own launches) does not inherit our
// failure — and an error the application left pending is not wiped.
inline void hip_ignore(hipError_t e) {
    if (e != hipSuccess) (void)hipGetLastError();
}

// The HSA IPC mode this process runs under: HSA_ENABLE_IPC_MODE_LEGACY as
// the library found it when it was loaded (-1: unset, then set to 0 by the
// library's constructor, before any HIP call of its own).
int ipc_mode_env_at_load();
const char *ipc_mode_env_now();

// The stream handlers of this thread run on (ompi_amd_set_thread_stream).
hipStream_t thread_stream();
// `void *` stream argument of the C ABI -> hipStream_t (NULL = per-thread).
// The C ABI's stream argument: NULL = this thread's per-thread stream;
// hipStreamLegacy (1) = the legacy null stream, passed on as the null handle
// (hipStreamWaitEvent does not accept the special handle; this library is
// built with the legacy default stream, so both name the same stream).
inline hipStream_t as_stream(void *s) {
    if (!s) return hipStreamPerThread;
    return static_cast<hipStream_t>(s) == hipStreamLegacy ? nullptr : static_cast<hipStream_t>(s);
}

int op_set_max_blocks(int64_t v);
// ompi_amd_is_device_pointer with a per-thread cache of host regions (op
// handlers: a pure-host call makes no runtime query once its buffers' 2 MiB
// granules are known)
int device_pointer_cached(const void *p);
int op_launch(int op, int type, bool three, const void *x, const void *y, void *dst,
              size_t n, hipStream_t s);

}  // namespace ompi_amd
