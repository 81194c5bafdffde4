/*
 * ompi_amd — MI355X-native reduction-collective hot path for Open MPI.
 *
 * C ABI of libompi_amd.so.  Plain pointers and sizes only; every entry point
 * returns an int status (no C++ exceptions cross this boundary).  Streams are
 * passed as `void *` (a hipStream_t; NULL = the calling thread's per-thread
 * stream).  Device pointers are HIP device (or managed) allocations.
 *
 * Each group of entry points names the reference interface it replaces.
 */
#ifndef OMPI_AMD_H
#define OMPI_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ */
/* Status codes (mapped to OMPI_ERR_* by the MCA glue)                 */
/* ------------------------------------------------------------------ */
#define OMPI_AMD_SUCCESS            0
#define OMPI_AMD_ERR_UNSUPPORTED   (-1)  /* (op,type) slot not provided   */
#define OMPI_AMD_ERR_BAD_PARAM     (-2)
#define OMPI_AMD_ERR_HIP           (-3)  /* a HIP runtime call failed      */
#define OMPI_AMD_ERR_TIMEOUT       (-4)  /* a peer never reached a flag    */
#define OMPI_AMD_ERR_NOT_DEVICE    (-5)  /* buffer is not device memory    */
#define OMPI_AMD_ERR_BOOTSTRAP     (-6)  /* shared-memory rendezvous failed */
#define OMPI_AMD_ERR_RMA_SYNC      (-7)  /* RMA epoch call out of order (OMPI_ERR_RMA_SYNC) */

/* ------------------------------------------------------------------ */
/* Op and type codes — numerically identical to the reference enums so */
/* the MCA glue passes them straight through:                          */
/*   op   = OMPI_OP_BASE_FORTRAN_*  (ompi/mca/op/op.h:203-237)         */
/*   type = OMPI_OP_BASE_TYPE_*     (ompi/mca/op/op.h:104-190)         */
/* ------------------------------------------------------------------ */
enum {
    OMPI_AMD_OP_NULL = 0, OMPI_AMD_OP_MAX = 1, OMPI_AMD_OP_MIN = 2,
    OMPI_AMD_OP_SUM = 3, OMPI_AMD_OP_PROD = 4, OMPI_AMD_OP_LAND = 5,
    OMPI_AMD_OP_BAND = 6, OMPI_AMD_OP_LOR = 7, OMPI_AMD_OP_BOR = 8,
    OMPI_AMD_OP_LXOR = 9, OMPI_AMD_OP_BXOR = 10, OMPI_AMD_OP_MAXLOC = 11,
    OMPI_AMD_OP_MINLOC = 12, OMPI_AMD_OP_REPLACE = 13, OMPI_AMD_OP_NO_OP = 14,
    OMPI_AMD_OP_COUNT = 15             /* OMPI_OP_BASE_FORTRAN_OP_MAX */
};

enum {
    OMPI_AMD_TYPE_INT8_T = 0, OMPI_AMD_TYPE_UINT8_T = 1,
    OMPI_AMD_TYPE_INT16_T = 2, OMPI_AMD_TYPE_UINT16_T = 3,
    OMPI_AMD_TYPE_INT32_T = 4, OMPI_AMD_TYPE_UINT32_T = 5,
    OMPI_AMD_TYPE_INT64_T = 6, OMPI_AMD_TYPE_UINT64_T = 7,
    /* short float = opal_short_float_t (_Float16 wherever the compiler has
     * it, config/opal_check_alt_short_float.m4:27-35); its complex is
     * opal_short_float_t[2] (MPIX_C_FLOAT16 / MPIX_C_FLOAT16_COMPLEX) */
    OMPI_AMD_TYPE_SHORT_FLOAT = 14,
    OMPI_AMD_TYPE_FLOAT = 15, OMPI_AMD_TYPE_DOUBLE = 16,
    OMPI_AMD_TYPE_BOOL = 25,
    OMPI_AMD_TYPE_C_SHORT_FLOAT_COMPLEX = 26,
    OMPI_AMD_TYPE_C_FLOAT_COMPLEX = 27, OMPI_AMD_TYPE_C_DOUBLE_COMPLEX = 28,
    OMPI_AMD_TYPE_BYTE = 30,
    OMPI_AMD_TYPE_FLOAT_INT = 34, OMPI_AMD_TYPE_DOUBLE_INT = 35,
    OMPI_AMD_TYPE_LONG_INT = 36, OMPI_AMD_TYPE_2INT = 37,
    OMPI_AMD_TYPE_SHORT_INT = 38,
    OMPI_AMD_TYPE_COUNT = 41           /* OMPI_OP_BASE_TYPE_MAX */
};

/* Library identity / build check. */
const char *ompi_amd_version(void);
/* Number of visible HIP devices (0 on a host without a GPU). */
int ompi_amd_device_count(void);
/* Last HIP error string seen by this thread (diagnostics only). */
const char *ompi_amd_last_error(void);
/* hipPointerGetAttributes: 1 device/managed, 0 host — replaces
 * mca_common_cuda_is_gpu_buffer (opal/mca/common/cuda/common_cuda.c:
 * 1739-1792) used by the convertor and the handlers to pick the path. */
int ompi_amd_is_device_pointer(const void *ptr);
/* The same answer, and for device memory the allocation holding ptr
 * (hipMemGetAddressRange): 1 device (*base, *size set), 0 host, <0 error. */
int ompi_amd_pointer_range(const void *ptr, void **base, size_t *size);

/* The HIP side of the convertor's GPU function table
 * (opal_common_cuda_function_table_t, opal/datatype/opal_datatype_cuda.h:
 * 16-21: gpu_is_gpu_buffer / gpu_cu_memcpy_async / gpu_cu_memcpy /
 * gpu_memmove; filled by common_cuda.c:1739-1792, :1648-1700).  Any mix of
 * host and device pointers.  memcpy_async is ordered on `stream` (NULL:
 * the calling thread's stream); memcpy and memmove complete before they
 * return; memmove is correct for overlapping ranges. */
int ompi_amd_memcpy_async(void *dst, const void *src, size_t bytes, void *stream);
int ompi_amd_memcpy(void *dst, const void *src, size_t bytes);
int ompi_amd_memmove(void *dst, void *src, size_t bytes);
/* Wait for `stream` (NULL: the calling thread's stream). */
int ompi_amd_stream_synchronize(void *stream);
/* Device memory for callers that stage host operands (coll/rocm's
 * residency staging): hipMalloc / hipFree.  bytes == 0 gives NULL. */
int ompi_amd_device_alloc(void **ptr, size_t bytes);
int ompi_amd_device_free(void *ptr);
/* Page-locked host memory (hipHostMalloc / hipHostFree) for staging
 * windows the device reads and writes directly (the convertor seam's
 * host-fragment windows).  bytes == 0 gives NULL. */
int ompi_amd_host_alloc(void **ptr, size_t bytes);
int ompi_amd_host_free(void *ptr);
/* Completion markers on a stream — the counterparts of common/cuda's
 * record / progress of its dtoh / htod events (common_cuda.c:1008-1320)
 * for a convertor run asynchronously.  ompi_amd_event_record creates the
 * event at *event the first time (NULL: create) and records it on
 * `stream` (NULL: the calling thread's); ompi_amd_event_query returns 1
 * once the work before it finished, 0 while pending, <0 on error. */
int ompi_amd_event_record(void **event, void *stream);
int ompi_amd_event_query(void *event);
int ompi_amd_event_synchronize(void *event);
int ompi_amd_event_destroy(void *event);

/* ================================================================== */
/* 1. MPI_Op kernels — replaces op/base's handler loops                */
/*    ompi/mca/op/base/op_base_functions.c:40-104 (2-buffer),          */
/*    :654-731 (3-buffer); tables :1485-1655.                          */
/* ================================================================== */

/* 1 if this library provides a device kernel for (op,type). */
int ompi_amd_op_supported(int op, int type);
/* Element stride (datatype extent) in bytes; 0 for unknown types. */
size_t ompi_amd_type_extent(int type);

/* inout[i] = inout[i] (op) in[i]  — 2-buffer handler semantics.
 * Stream-ordered; returns before the kernel completes. */
int ompi_amd_op_reduce(int op, int type, const void *in, void *inout,
                       size_t count, void *stream);
/* out[i] = in1[i] (op) in2[i]     — 3-buffer handler semantics. */
int ompi_amd_op_reduce_3buff(int op, int type, const void *in1,
                             const void *in2, void *out, size_t count,
                             void *stream);

/* --- the op framework seam (ompi/mca/op/op.h:258-273, 362-378) ---- */
/* Handler signatures are exactly ompi_op_base_handler_fn_1_0_0_t and
 * ompi_op_base_3buff_handler_fn_1_0_0_t.  The handlers run the device
 * kernel on the calling thread's stream and synchronise before returning
 * (the caller sends the result immediately; handlers return void).  When
 * the buffers are host memory they call the fallback registered for the
 * slot (the previous, lower-priority handler — op_example_module_max.c
 * pattern); with no fallback registered they abort loudly.  Mixed host and
 * device operands (coll/tuned's ring reducing a malloc'd bounce buffer
 * into a device rbuf, coll_base_allreduce.c:688-693) are staged through a
 * per-thread device scratch and run on the GPU. */
struct ompi_datatype_t;
struct ompi_op_base_module_1_0_0_t;
typedef void (*ompi_amd_op_handler_fn_t)(const void *, void *, int *,
                                         struct ompi_datatype_t **,
                                         struct ompi_op_base_module_1_0_0_t *);
typedef void (*ompi_amd_op_3buff_handler_fn_t)(const void *, const void *,
                                               void *, int *,
                                               struct ompi_datatype_t **,
                                               struct ompi_op_base_module_1_0_0_t *);

/* Row `op` of the 2-/3-buffer handler tables: OMPI_AMD_TYPE_COUNT entries,
 * NULL where this library provides no kernel (keep the lower priority
 * slot, op_base_op_select.c:137-178). NULL for an unknown op. */
const ompi_amd_op_handler_fn_t *ompi_amd_op_handler_row(int op);
const ompi_amd_op_3buff_handler_fn_t *ompi_amd_op_3buff_handler_row(int op);

/* Register the host-memory fallback for a slot (what the glue finds in
 * op->o_func.intrinsic.fns[type] / .modules[type] at query time). */
int ompi_amd_op_set_fallback(int op, int type, ompi_amd_op_handler_fn_t fn,
                             struct ompi_op_base_module_1_0_0_t *module,
                             ompi_amd_op_3buff_handler_fn_t fn3,
                             struct ompi_op_base_module_1_0_0_t *module3);

/* Process-wide tuning knobs, the MCA-parameter surface of the component
 * (op_rocm_max_blocks ...).  Keys: "op_max_blocks" (grid cap of the
 * streaming op kernels; default: uncapped, one chunk per workgroup). */
int ompi_amd_set_tuning(const char *key, int64_t value);

/* Stream the handlers of the calling thread use (NULL = per-thread). */
int ompi_amd_set_thread_stream(void *stream);

#ifdef __cplusplus
}
#endif
#endif /* OMPI_AMD_H */
