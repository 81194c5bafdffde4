/*
 * ompi_amd — datatype pack/unpack offload for device buffers.
 *
 * Replaces the convertor's per-run memcpy / cuMemcpy on device memory
 * (opal/datatype/opal_datatype_pack.h:37-206, opal_datatype_unpack.c:
 * 245-428, opal/datatype/opal_datatype_cuda.c:121-145: one cuMemcpy per
 * contiguous block) with one kernel launch per convertor call.
 */
#ifndef OMPI_AMD_DDT_H
#define OMPI_AMD_DDT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One contiguous run of a committed datatype's typemap. */
typedef struct {
    int64_t disp;   /* byte displacement from the element base */
    int64_t len;    /* bytes (> 0) */
} ompi_amd_ddt_block_t;

/* One element of the device program: `count` runs of `blocklen` bytes,
 * `stride` bytes apart, the first at `disp` — the shape of opal's optimized
 * ddt_elem_desc {count, blocklen, extent, disp} (opal_datatype_internal.h:
 * 157-164).  MPI_Type_vector(n, bl, st, MPI_DOUBLE) is ONE such element. */
typedef struct {
    int64_t count;
    int64_t blocklen;
    int64_t stride;
    int64_t disp;
} ompi_amd_ddt_elem_t;

typedef struct ompi_amd_ddt ompi_amd_ddt_t;

/* Build the device program of a datatype from its typemap (nblocks runs in
 * typemap order, element stride `extent`).  Runs are merged and equal-length
 * runs at a constant stride folded into one {count, blocklen, stride, disp}
 * element, the shape of opal's optimized description (ddt_elem_desc,
 * opal_datatype_internal.h:157-164; opal_datatype_optimize.c:261). */
int ompi_amd_ddt_create(const ompi_amd_ddt_block_t *blocks, int nblocks,
                        int64_t extent, ompi_amd_ddt_t **ddt);
/* Same, from an already-optimized element list (typemap order). */
int ompi_amd_ddt_create_elems(const ompi_amd_ddt_elem_t *elems, int nelems,
                              int64_t extent, ompi_amd_ddt_t **ddt);
int ompi_amd_ddt_destroy(ompi_amd_ddt_t *ddt);
/* packed bytes per datatype element (the MPI type size) */
size_t ompi_amd_ddt_size(const ompi_amd_ddt_t *ddt);
/* number of {count, blocklen, stride, disp} elements after folding */
int ompi_amd_ddt_nelems(const ompi_amd_ddt_t *ddt);

/* Pack stream bytes [offset, offset+bytes) of `count` datatype elements
 * based at device address `src` into contiguous device memory `dst`.
 * *done = bytes produced (bytes, or fewer at the end of the stream).
 * `offset` may split a run or a predefined element: the convertor's
 * bConverted position (opal_convertor.c:218-273).  Stream-ordered. */
int ompi_amd_ddt_pack(const ompi_amd_ddt_t *ddt, size_t count, const void *src,
                      void *dst, size_t offset, size_t bytes, size_t *done,
                      void *stream);
/* Inverse: scatter packed `src` bytes (stream positions [offset,
 * offset+bytes)) into the typed layout at `dst`. */
int ompi_amd_ddt_unpack(const ompi_amd_ddt_t *ddt, size_t count,
                        const void *src, void *dst, size_t offset,
                        size_t bytes, size_t *done, void *stream);

/* An iovec entry, layout-identical to struct iovec (sys/uio.h): the glue
 * passes the convertor's iovec array straight through. */
typedef struct {
    void *iov_base;
    size_t iov_len;
} ompi_amd_iovec_t;

/* The convertor's advance step over an iovec array, with the contract of
 * convertor_advance_fct_t (opal/datatype/opal_convertor.h:64-67) as
 * opal_generic_simple_pack / _unpack implement it (opal_datatype_pack.c:
 * 235-370, opal_datatype_unpack.c:245-428): starting at stream byte
 * `position` (the convertor's bConverted; any byte, mid-element included),
 * fill (pack) or drain (unpack) iov[0 .. *out_size) in order, each up to its
 * iov_len; on return iov_len = bytes used per entry, *out_size = entries
 * used (all, unless the stream ended inside one), *max_data = total bytes.
 * Returns 1 when the stream is complete, 0 when data remains, a negative
 * OMPI_AMD_ERR_* on error.  All entries move in ONE kernel launch
 * (stream-ordered on `stream`; the caller synchronises unless it runs the
 * convertor asynchronously). */
int ompi_amd_ddt_pack_iov(const ompi_amd_ddt_t *ddt, size_t count,
                          const void *typed, size_t position,
                          ompi_amd_iovec_t *iov, uint32_t *out_size,
                          size_t *max_data, void *stream);
int ompi_amd_ddt_unpack_iov(const ompi_amd_ddt_t *ddt, size_t count,
                            void *typed, size_t position,
                            ompi_amd_iovec_t *iov, uint32_t *out_size,
                            size_t *max_data, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* OMPI_AMD_DDT_H */
