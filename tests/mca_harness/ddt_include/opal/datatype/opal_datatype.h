/* TEST HARNESS ONLY: opal_datatype_t's fields the convertor seam reads
 * (opal/datatype/opal_datatype.h:55-145), restated with the reference's
 * field list and order. */
#ifndef HARNESS_OPAL_DATATYPE_H
#define HARNESS_OPAL_DATATYPE_H
#include <stddef.h>
#include <stdint.h>

#include "opal/class/opal_object.h"

#define OPAL_DATATYPE_MAX_PREDEFINED 26
#define OPAL_DATATYPE_FLAG_CONTIGUOUS 0x0010
#define OPAL_DATATYPE_FLAG_NO_GAPS 0x0020
#define OPAL_DATATYPE_FLAG_DATA 0x0100

typedef union dt_elem_desc dt_elem_desc_t;
typedef size_t opal_datatype_count_t;

typedef struct dt_type_desc_t {
    opal_datatype_count_t length;
    opal_datatype_count_t used;
    dt_elem_desc_t *desc;
} dt_type_desc_t;

#define OPAL_MAX_OBJECT_NAME 64

/* the reference's field list and order (opal_datatype.h:97-134) */
typedef struct opal_datatype_t {
    opal_object_t super;
    uint16_t flags;
    uint16_t id;
    uint32_t bdt_used;
    size_t size;
    ptrdiff_t true_lb, true_ub, lb, ub;
    size_t nbElems;
    uint32_t align, loops;
    char name[OPAL_MAX_OBJECT_NAME];
    dt_type_desc_t desc;
    dt_type_desc_t opt_desc;
    size_t *ptypes;
} opal_datatype_t;

extern const opal_datatype_t *opal_datatype_basicDatatypes[OPAL_DATATYPE_MAX_PREDEFINED];
#endif
