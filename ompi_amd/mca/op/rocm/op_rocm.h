/*
 * op/rocm — MI355X op component for Open MPI's op framework.
 *
 * Drop-in: copy this directory to ompi/mca/op/rocm/ of an Open MPI tree
 * (see INTEGRATION.md §1).  The component fills the 2-buffer / 3-buffer
 * handler slots (ompi/mca/op/op.h:362-378) with libompi_amd.so's HIP
 * handlers for every (op, type) both op/base and the library provide, and
 * registers op/base's handler of the same slot as the host-memory fallback
 * (the op_example_module_max.c pattern).
 */
#ifndef MCA_OP_ROCM_EXPORT_H
#define MCA_OP_ROCM_EXPORT_H

#include "ompi_config.h"

#include "ompi/mca/mca.h"
#include "ompi/mca/op/op.h"
#include "opal/class/opal_object.h"

BEGIN_C_DECLS

typedef struct {
    ompi_op_base_component_1_0_0_t super;
    /* MCA params: op_rocm_priority, op_rocm_max_blocks */
    int priority;
    int max_blocks;
    /* set by init_query: a HIP device is visible */
    bool have_gpu;
} ompi_op_rocm_component_t;

OMPI_DECLSPEC extern ompi_op_rocm_component_t mca_op_rocm_component;

END_C_DECLS

#endif /* MCA_OP_ROCM_EXPORT_H */
