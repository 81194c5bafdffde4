/* TEST HARNESS ONLY: device buffers for the harnesses, and (coll
 * harness) the datatype engine's sndrcv over the stand-in types. */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdint.h>

/* A copy from pageable memory may return before the bytes reach the
 * device (the DMA from the staging buffer still runs): wait for it, so a
 * peer's RMA that follows the next rendezvous cannot be overwritten. */
int harness_dev_copy_in(void *d, const void *h, size_t bytes)
{
    if (hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int harness_dev_alloc_copy(void **d, const void *h, size_t bytes)
{
    if (hipMalloc(d, bytes) != hipSuccess) return -1;
    return harness_dev_copy_in(*d, h, bytes);
}

int harness_dev_copy_back(void *h, const void *d, size_t bytes)
{
    return hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

int harness_dev_free(void *d)
{
    return hipFree(d) == hipSuccess ? 0 : -1;
}

#ifdef HARNESS_COLL
#include "ompi/datatype/ompi_datatype.h"
/* typed <-> typed copy of equal signatures, element by element, through
 * hipMemcpyDefault so that either side may be device memory */
int32_t ompi_datatype_sndrcv(const void *sbuf, int32_t scount, const ompi_datatype_t *sdtype,
                             void *rbuf, int32_t rcount, const ompi_datatype_t *rdtype)
{
    const size_t bytes = sdtype->size * (size_t) scount;
    size_t done = 0;
    if (bytes != rdtype->size * (size_t) rcount) return -1;
    while (done < bytes) {
        /* the next contiguous run on each side */
        const size_t se = sdtype->size, re = rdtype->size;
        const size_t soff = sdtype->contiguous ? done : (done / se) * 2 * se + done % se;
        const size_t roff = rdtype->contiguous ? done : (done / re) * 2 * re + done % re;
        size_t run = bytes - done;
        if (!sdtype->contiguous && se - done % se < run) run = se - done % se;
        if (!rdtype->contiguous && re - done % re < run) run = re - done % re;
        if (hipMemcpy((char *) rbuf + roff, (const char *) sbuf + soff, run, hipMemcpyDefault) !=
            hipSuccess)
            return -1;
        done += run;
    }
    return 0;
}

/* common/rocm's whole-buffer device pack / unpack (opal_datatype_rocm.c)
 * over the stand-in types, for the pml harness: one 2-D device copy (a
 * stand-in type is `size` data bytes every `size` or 2 * `size` bytes);
 * harness_device_packs counts the calls so a test can see the path taken.
 * The real implementation is exercised by the ddt harness. */
int harness_device_packs;
struct opal_datatype_t;
int opal_rocm_device_program(const struct opal_datatype_t *dt) { return dt != NULL; }
static int whole2d(const ompi_datatype_t *d, size_t count, void *typed, void *packed, int unpack)
{
    const size_t pitch = d->contiguous ? d->size : 2 * d->size;
    hipError_t e;
    if (count == 0) return 0;
    ++harness_device_packs;
    e = unpack ? hipMemcpy2D(typed, pitch, packed, d->size, d->size, count, hipMemcpyDeviceToDevice)
               : hipMemcpy2D(packed, d->size, typed, pitch, d->size, count, hipMemcpyDeviceToDevice);
    return e == hipSuccess ? 0 : -1;
}
int opal_rocm_pack_device(const struct opal_datatype_t *dt, size_t count, const void *src,
                          void *packed, void *stream)
{
    return whole2d((const ompi_datatype_t *) dt, count, (void *) src, packed, 0);
}
int opal_rocm_unpack_device(const struct opal_datatype_t *dt, size_t count, const void *packed,
                            void *dst, void *stream)
{
    return whole2d((const ompi_datatype_t *) dt, count, dst, (void *) packed, 1);
}
#endif

#ifdef HARNESS_OSC
#include "ompi/datatype/ompi_datatype.h"
#include "ompi_amd_ddt.h"
/* ompi_datatype_args.c:825-865 over the stand-in types: a predefined type
 * is its own primitive; a gapped stand-in (contiguous == 0: `size` data
 * bytes every 2 * `size`) is built from the predefined type of its id */
ompi_datatype_t *ompi_datatype_get_single_predefined_type_from_args(ompi_datatype_t *type)
{
    static ompi_datatype_t prim[64];
    if (type->predefined) return type;
    if (type->id < 0 || type->id >= 64) return (ompi_datatype_t *) 0;
    prim[type->id] = (ompi_datatype_t){type->id, type->size, 1, 1};
    return &prim[type->id];
}

/* common/rocm's device program of a datatype (opal_datatype_rocm.c) for the
 * stand-in types: one run of `size` bytes, extent 2 * `size` (gapped) */
struct opal_datatype_t;
int harness_device_ddts;
const ompi_amd_ddt_t *opal_rocm_device_ddt(const struct opal_datatype_t *dt)
{
    static struct { const void *dt; ompi_amd_ddt_t *prog; } cache[16];
    static int n;
    const ompi_datatype_t *d = (const ompi_datatype_t *) dt;
    for (int i = 0; i < n; ++i)
        if (cache[i].dt == dt) return cache[i].prog;
    ompi_amd_ddt_elem_t e = {1, (int64_t) d->size, (int64_t) d->size, 0};
    ompi_amd_ddt_t *prog = 0;
    if (n == 16 || ompi_amd_ddt_create_elems(&e, 1, (int64_t) (d->contiguous ? d->size : 2 * d->size),
                                             &prog) != 0)
        return 0;
    ++harness_device_ddts;
    cache[n].dt = dt;
    cache[n++].prog = prog;
    return prog;
}
#endif
