/* TEST HARNESS ONLY: device buffers for the harnesses, and (coll
 * harness) the datatype engine's sndrcv over the stand-in types. */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdint.h>

int harness_dev_alloc_copy(void **d, const void *h, size_t bytes)
{
    if (hipMalloc(d, bytes) != hipSuccess) return -1;
    return hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

int harness_dev_copy_in(void *d, const void *h, size_t bytes)
{
    return hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
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
#endif
