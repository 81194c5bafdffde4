/* TEST HARNESS ONLY: the op framework interface (restated from the
 * reference's ompi/mca/op/op.h:104-378 layouts, not copied). */
#ifndef HARNESS_OMPI_MCA_OP_H
#define HARNESS_OMPI_MCA_OP_H
#include "ompi_config.h"
#include "ompi/mca/mca.h"
#include "opal/class/opal_object.h"
#define OMPI_OP_BASE_TYPE_MAX 41
#define OMPI_OP_BASE_FORTRAN_OP_MAX 15
#define OMPI_OP_BASE_TYPE_FLOAT 15
struct ompi_datatype_t;
struct ompi_op_t;
struct ompi_op_base_module_1_0_0_t;
typedef struct ompi_op_base_module_1_0_0_t ompi_op_base_module_t;
typedef void (*ompi_op_base_handler_fn_t)(const void *, void *, int *, struct ompi_datatype_t **,
                                          struct ompi_op_base_module_1_0_0_t *);
typedef void (*ompi_op_base_3buff_handler_fn_t)(const void *, const void *, void *, int *,
                                                struct ompi_datatype_t **,
                                                struct ompi_op_base_module_1_0_0_t *);
typedef int (*ompi_op_base_component_init_query_fn_t)(bool, bool);
typedef struct ompi_op_base_module_1_0_0_t *(*ompi_op_base_component_op_query_1_0_0_fn_t)(
    struct ompi_op_t *op, int *priority);
typedef struct ompi_op_base_component_1_0_0_t {
    mca_base_component_t opc_version;
    mca_base_component_data_t opc_data;
    ompi_op_base_component_init_query_fn_t opc_init_query;
    ompi_op_base_component_op_query_1_0_0_fn_t opc_op_query;
} ompi_op_base_component_1_0_0_t;
typedef int (*ompi_op_base_module_enable_1_0_0_fn_t)(struct ompi_op_base_module_1_0_0_t *,
                                                     struct ompi_op_t *);
struct ompi_op_base_module_1_0_0_t {
    opal_object_t super;
    ompi_op_base_module_enable_1_0_0_fn_t opm_enable;
    struct ompi_op_t *opm_op;
    ompi_op_base_handler_fn_t opm_fns[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_3buff_handler_fn_t opm_3buff_fns[OMPI_OP_BASE_TYPE_MAX];
};
#define OMPI_OP_BASE_VERSION_1_0_0 OMPI_MCA_BASE_VERSION_2_1_0("op", 1, 0, 0)
#endif
