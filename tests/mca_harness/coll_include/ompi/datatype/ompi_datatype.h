/* TEST HARNESS ONLY: predefined datatypes as (id, size, predefined,
 * contiguous).  A stand-in type with contiguous == 0 lays each element out
 * as `size` data bytes followed by a `size`-byte gap (extent 2 * size): the
 * smallest layout that exercises packing. */
#ifndef HARNESS_OMPI_DATATYPE_H
#define HARNESS_OMPI_DATATYPE_H
#include <stddef.h>
#include <stdint.h>
typedef struct ompi_datatype_t {
    int id;
    size_t size;
    int predefined;
    int contiguous;
} ompi_datatype_t;
static inline int ompi_datatype_is_predefined(const ompi_datatype_t *d) { return d->predefined; }
static inline int ompi_datatype_type_size(const ompi_datatype_t *d, size_t *s)
{
    *s = d->size;
    return 0;
}
static inline int ompi_datatype_is_contiguous_memory_layout(const ompi_datatype_t *d, int count)
{
    (void) count;
    return d->contiguous;
}
static inline int ompi_datatype_get_extent(const ompi_datatype_t *d, ptrdiff_t *lb, ptrdiff_t *ext)
{
    *lb = 0;
    *ext = (ptrdiff_t) (d->contiguous ? d->size : 2 * d->size);
    return 0;
}
static inline int ompi_datatype_get_true_extent(const ompi_datatype_t *d, ptrdiff_t *lb,
                                                ptrdiff_t *ext)
{
    *lb = 0;
    *ext = (ptrdiff_t) d->size;
    return 0;
}
/* ompi/datatype/ompi_datatype.h (ompi_datatype_args.c:825; harness:
 * dev_helpers.c, HARNESS_OSC) */
ompi_datatype_t *ompi_datatype_get_single_predefined_type_from_args(ompi_datatype_t *type);
/* ompi/datatype/ompi_datatype.h:303-304 (harness: dev_helpers.c, any
 * residency) */
int32_t ompi_datatype_sndrcv(const void *sbuf, int32_t scount, const ompi_datatype_t *sdtype,
                             void *rbuf, int32_t rcount, const ompi_datatype_t *rdtype);
#endif
