/* TEST HARNESS ONLY: the ompi_op_t fields the coll glue reads
 * (ompi/op/op.h:145-195, 99-117; ompi_op_ddt_map op.c:102). */
#ifndef HARNESS_COLL_OMPI_OP_H
#define HARNESS_COLL_OMPI_OP_H
#define OMPI_OP_FLAGS_INTRINSIC 0x0001
typedef struct ompi_op_t {
    int o_flags;
    int o_f_to_c_index;
} ompi_op_t;
extern int ompi_op_ddt_map[64];
static inline int ompi_op_is_intrinsic(const ompi_op_t *op)
{
    return (op->o_flags & OMPI_OP_FLAGS_INTRINSIC) != 0;
}
#endif
