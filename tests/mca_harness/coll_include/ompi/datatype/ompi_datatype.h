/* TEST HARNESS ONLY: predefined datatypes as (id, size, contiguous). */
#ifndef HARNESS_OMPI_DATATYPE_H
#define HARNESS_OMPI_DATATYPE_H
#include <stddef.h>
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
#endif
