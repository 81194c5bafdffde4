/*
 * The convertor's GPU seam for device buffers through libompi_amd.so.
 *
 * Two hook points of the reference (SURVEY.md §8b "convertor offload"):
 *  - the GPU function table (opal_common_cuda_function_table_t,
 *    opal/datatype/opal_datatype_cuda.h:16-21), registered with
 *    opal_cuda_add_initialization_function (opal_datatype_cuda.c:34-36):
 *    mca_common_rocm_fill_table fills it with HIP implementations;
 *  - the convertor's advance function (convertor_advance_fct_t,
 *    opal/datatype/opal_convertor.h:64-67), chosen in
 *    opal_convertor_prepare_for_send / _recv (opal_convertor.c:565-653):
 *    opal_rocm_convertor_select replaces the generic pack / unpack by
 *    opal_rocm_pack / opal_rocm_unpack when the user buffer is device
 *    memory (CONVERTOR_CUDA, set by mca_cuda_convertor_init through the
 *    table's gpu_is_gpu_buffer).
 * Nothing here depends on OPAL_CUDA_SUPPORT except the function table and
 * the convertor's stream field, which exist only in such a build
 * (opal_convertor.h:120-123): a ROCm-only build compiles the seam with
 * OPAL_CUDA_SUPPORT 0 and gets the offload through the select / set-
 * position hooks alone.  INTEGRATION.md §3 shows the lines a maintainer
 * adds to the reference's prepare and set-position functions.
 */
#ifndef OPAL_DATATYPE_ROCM_H
#define OPAL_DATATYPE_ROCM_H

#include <stdint.h>
#include <sys/uio.h>

#include "opal/datatype/opal_convertor.h"
#include "ompi_amd_ddt.h"
#if OPAL_CUDA_SUPPORT
#include "opal/datatype/opal_datatype_cuda.h"

/* opal_cuda_add_initialization_function's callback: fill the GPU table
 * (a CUDA-support build only: the table exists nowhere else). */
int mca_common_rocm_fill_table(opal_common_cuda_function_table_t *ftable);
#endif

/* After prepare_for_send / _recv chose fAdvance: offload it when the
 * convertor is a device conversion the library can run.  Returns 1 when
 * fAdvance now points at opal_rocm_pack / opal_rocm_unpack (or, ROCm-only
 * build, opal_rocm_refuse for a device description too irregular to
 * flatten), 0 when the reference's choice stays (host buffer, NO_OP
 * contiguous fast path; a CUDA-support build's irregular description, whose
 * host walker copies through cbmemcpy).  Device residency: CONVERTOR_CUDA
 * in an OPAL_CUDA_SUPPORT build; otherwise this seam's own pointer query
 * (so a ROCm-only build, where nothing sets CONVERTOR_CUDA, offloads too). */
int opal_rocm_convertor_select(opal_convertor_t *convertor);

/* The convertor runs on this seam (its fAdvance is ours). */
int opal_rocm_convertor_owns(const opal_convertor_t *convertor);

/* opal_convertor_set_position_nocheck for an owned convertor (the third
 * hook line): bConverted = *position for a receive, the
 * start of the enclosing predefined element for a non-contiguous send, as
 * the reference; *position updated.  Returns 0. */
int32_t opal_rocm_set_position(opal_convertor_t *convertor, size_t *position);

/* convertor_advance_fct_t implementations: iov[0 .. *out_size) filled
 * (pack) or drained (unpack) from bConverted on — device fragments in one
 * kernel launch (or recorded, after opal_rocm_set_copy_function_async),
 * host fragments through page-locked windows of up to 16 MiB of the stream
 * (a send packs a window ahead and serves the next fragments from it; a
 * receive gathers fragments and unpacks a window at a time, the last one
 * before the call that completes the stream returns); returns 1 complete,
 * 0 more data pending, -1 error. */
int32_t opal_rocm_pack(opal_convertor_t *convertor, struct iovec *iov, uint32_t *out_size,
                       size_t *max_data);
int32_t opal_rocm_unpack(opal_convertor_t *convertor, struct iovec *iov, uint32_t *out_size,
                         size_t *max_data);
#if !OPAL_CUDA_SUPPORT
/* A ROCm-only build's fAdvance for a device buffer whose description has no
 * device program (select returns 1 with it): returns -1 and touches
 * nothing, since that build has no cbmemcpy for the host walker to use. */
int32_t opal_rocm_refuse(opal_convertor_t *convertor, struct iovec *iov, uint32_t *out_size,
                         size_t *max_data);
#endif

/* Asynchronous conversion (the ROCm counterpart of
 * opal_cuda_set_copy_function_async, opal_datatype_cuda.c:216-219, which
 * ob1 calls at pml_ob1_recvfrag.c:598 / pml_ob1_recvreq.c:868): sets
 * CONVERTOR_CUDA_ASYNC and the stream, and from now on fAdvance records
 * device fragments instead of launching them — the caller must flush
 * (opal_rocm_record_event, the counterpart of common_cuda's
 * mca_common_cuda_record_dtoh_event / _htod_event) before it reads a packed
 * fragment or reuses a received one.  Host fragments stay synchronous.
 * Valid until the convertor is prepared again. */
int opal_rocm_set_copy_function_async(opal_convertor_t *convertor, void *stream);
/* Launch what the convertor recorded (device fragments; a receive's
 * gathered host window, waited for).  0 or -1. */
int opal_rocm_convertor_flush(opal_convertor_t *convertor);
/* Flush, then mark the point on the convertor's stream: *event (NULL:
 * created) completes once every fragment converted so far is in place
 * (ompi_amd_event_query / _synchronize / _destroy).  0 or -1. */
int opal_rocm_record_event(opal_convertor_t *convertor, void **event);
/* Forget the convertor's state (its windows return to a pool); prepare
 * does it by itself — for a convertor destroyed before it completed. */
void opal_rocm_convertor_release(opal_convertor_t *convertor);

/* count elements of dt at src (device memory) packed into the device
 * buffer `packed` (dt->size * count bytes), or unpacked from it into dst:
 * one kernel launch, complete on return.  0 done, 1 not offloadable (host
 * memory, or no device program: the caller keeps its host path), -1 error.
 * pml/rocm's non-contiguous device messages (no host round trip). */
int opal_rocm_pack_device(const opal_datatype_t *dt, size_t count, const void *src, void *packed,
                          void *stream);
/* 1 when dt has a device program (the two calls above can take it) */
int opal_rocm_device_program(const opal_datatype_t *dt);
/* dt's device program itself (NULL: none) — osc/rocm's derived-datatype
 * accumulates (ompi_amd_accumulate_ddt) */
const ompi_amd_ddt_t *opal_rocm_device_ddt(const opal_datatype_t *dt);
int opal_rocm_unpack_device(const opal_datatype_t *dt, size_t count, const void *packed, void *dst,
                            void *stream);

/* Device programs cached per datatype description (tests / finalize). */
int opal_rocm_program_cache_size(void);
void opal_rocm_program_cache_clear(void);

#endif
