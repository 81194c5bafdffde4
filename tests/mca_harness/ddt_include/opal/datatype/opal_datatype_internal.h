/* TEST HARNESS ONLY: the description elements of opal/datatype
 * (opal_datatype_internal.h:104-190) restated with the reference's field
 * names and meanings, for compiling ompi_amd/mca/common/rocm. */
#ifndef HARNESS_OPAL_DATATYPE_INTERNAL_H
#define HARNESS_OPAL_DATATYPE_INTERNAL_H
#include <stddef.h>
#include <stdint.h>

#define OPAL_DATATYPE_LOOP 0
#define OPAL_DATATYPE_END_LOOP 1
#define OPAL_DATATYPE_LB 2
#define OPAL_DATATYPE_UB 3
#define OPAL_DATATYPE_INT1 4
#define OPAL_DATATYPE_INT2 5
#define OPAL_DATATYPE_INT4 6
#define OPAL_DATATYPE_INT8 7
#define OPAL_DATATYPE_UINT1 9
#define OPAL_DATATYPE_FLOAT4 15
#define OPAL_DATATYPE_FLOAT8 16
#define OPAL_DATATYPE_FLOAT16 18

typedef struct ddt_elem_id_description {
    uint16_t flags;
    uint16_t type;
} ddt_elem_id_description;

typedef struct ddt_elem_desc {   /* count blocks of blocklen basic elements */
    ddt_elem_id_description common;
    uint32_t count;
    size_t blocklen;
    ptrdiff_t extent;            /* bytes between blocks */
    ptrdiff_t disp;              /* bytes to the first block */
} ddt_elem_desc_t;

typedef struct ddt_loop_desc {   /* loops repetitions of the next items-1 entries */
    ddt_elem_id_description common;
    uint32_t items;
    uint32_t loops;
    size_t unused;
    ptrdiff_t extent;
} ddt_loop_desc_t;

typedef struct ddt_endloop_desc {
    ddt_elem_id_description common;
    uint32_t items;
    uint32_t unused;
    size_t size;
    ptrdiff_t first_elem_disp;
} ddt_endloop_desc_t;

union dt_elem_desc {
    ddt_elem_desc_t elem;
    ddt_loop_desc_t loop;
    ddt_endloop_desc_t end_loop;
};
#endif
