/* TEST HARNESS ONLY: the ompi_op_t fields the op glue reads
 * (ompi/op/op.h:145-195 of the reference). */
#ifndef HARNESS_OMPI_OP_H
#define HARNESS_OMPI_OP_H
#include "ompi/mca/op/op.h"
#define OMPI_OP_FLAGS_INTRINSIC 0x0001
typedef struct ompi_op_t {
    int o_flags;
    int o_f_to_c_index;
    struct {
        struct {
            ompi_op_base_handler_fn_t fns[OMPI_OP_BASE_TYPE_MAX];
            ompi_op_base_module_t *modules[OMPI_OP_BASE_TYPE_MAX];
        } intrinsic;
    } o_func;
    struct {
        ompi_op_base_3buff_handler_fn_t fns[OMPI_OP_BASE_TYPE_MAX];
        ompi_op_base_module_t *modules[OMPI_OP_BASE_TYPE_MAX];
    } o_3buff_intrinsic;
} ompi_op_t;
#endif
