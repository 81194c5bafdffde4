/*
 * op/rocm component: query / enable glue between Open MPI's op framework
 * (ompi/mca/op/op.h:294-378, selection ompi/mca/op/base/op_base_op_select.c:
 * 90-211) and libompi_amd.so (include/ompi_amd.h).
 *
 * For each intrinsic MPI_Op the query builds one module whose slot i is
 * libompi_amd's handler when BOTH op/base and the library have slot i
 * (op_base_op_select.c:182-204 requires the NULL pattern to stay op/base's;
 * NULL = keep the lower-priority handler).  The host-buffer fallback of a
 * slot is captured in the module's opm_enable, not in the query: the base
 * queries every component first (check_components, :133) and then enables
 * and installs them in ascending priority (:137-178), so at op/rocm's
 * enable the slot already holds whatever a lower-priority component (op/avx
 * at 50) installed over op/base — host reductions keep that handler and
 * its semantics.
 */
#include "ompi_config.h"

#include "ompi/constants.h"
#include "ompi/op/op.h"
#include "ompi/mca/op/op.h"
#include "ompi/mca/op/base/base.h"
#include "opal/class/opal_object.h"
#include "opal/mca/base/mca_base_var.h"

#include "op_rocm.h"
#include "ompi_amd.h"

static int rocm_component_open(void);
static int rocm_component_close(void);
static int rocm_component_register(void);
static int rocm_component_init_query(bool enable_progress_threads,
                                     bool enable_mpi_thread_multiple);
static struct ompi_op_base_module_1_0_0_t *
rocm_component_op_query(struct ompi_op_t *op, int *priority);

ompi_op_rocm_component_t mca_op_rocm_component = {
    .super = {
        .opc_version = {
            OMPI_OP_BASE_VERSION_1_0_0,
            .mca_component_name = "rocm",
            MCA_BASE_MAKE_VERSION(component, OMPI_MAJOR_VERSION, OMPI_MINOR_VERSION,
                                  OMPI_RELEASE_VERSION),
            .mca_open_component = rocm_component_open,
            .mca_close_component = rocm_component_close,
            .mca_register_component_params = rocm_component_register,
        },
        .opc_data = {
            /* the component is checkpoint-ready */
            MCA_BASE_METADATA_PARAM_CHECKPOINT
        },
        .opc_init_query = rocm_component_init_query,
        .opc_op_query = rocm_component_op_query,
    },
    .priority = 60,     /* above op/avx (50): device buffers are ours */
    .max_blocks = 0,    /* 0 = library default (uncapped grid) */
    .have_gpu = false,
};

static int rocm_component_register(void)
{
    (void) mca_base_component_var_register(&mca_op_rocm_component.super.opc_version,
                                           "priority",
                                           "Priority of the op/rocm component",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0,
                                           OPAL_INFO_LVL_9, MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_op_rocm_component.priority);
    (void) mca_base_component_var_register(&mca_op_rocm_component.super.opc_version,
                                           "max_blocks",
                                           "Grid cap of the streaming op kernels (0 = uncapped)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0,
                                           OPAL_INFO_LVL_9, MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_op_rocm_component.max_blocks);
    return OMPI_SUCCESS;
}

static int rocm_component_open(void)
{
    return OMPI_SUCCESS;
}

static int rocm_component_close(void)
{
    return OMPI_SUCCESS;
}

static int rocm_component_init_query(bool enable_progress_threads,
                                     bool enable_mpi_thread_multiple)
{
    /* Handlers keep no global mutable state beyond the fallback table
       written here at init, and run on the calling thread's HIP stream, so
       MPI_THREAD_MULTIPLE is fine. */
    mca_op_rocm_component.have_gpu = ompi_amd_device_count() > 0;
    if (!mca_op_rocm_component.have_gpu) {
        return OMPI_ERR_NOT_SUPPORTED;
    }
    if (mca_op_rocm_component.max_blocks > 0) {
        (void) ompi_amd_set_tuning("op_max_blocks", mca_op_rocm_component.max_blocks);
    }
    return OMPI_SUCCESS;
}

/* opm_enable (op_base_op_select.c:142-150): the slots this module takes
 * hold the handler the lower-priority components left there; that handler
 * (and its module, retained for as long as the library may call it) is
 * what host buffers go to.
 *
 * Reference counts: the copy loop that follows enable retains this module
 * once per slot it takes, but its 3-buffer branch releases the slot's
 * 2-BUFFER module (op_base_op_select.c:163-164) — this module itself when
 * it took both slots of the type, as it just stored itself there.  The op
 * destructor later releases both arrays (op.c:500-507), so without help
 * this module would end with half the references its slots hold and be
 * released past zero at MPI_Finalize.  One extra retain per type whose
 * 2- and 3-buffer slots it takes balances that (a framework with the
 * release fixed would leak the module instead of freeing it twice). */
static int rocm_module_enable(struct ompi_op_base_module_1_0_0_t *module, struct ompi_op_t *op)
{
    int i;
    for (i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        ompi_op_base_module_t *m2, *m3;
        if (NULL == module->opm_fns[i] && NULL == module->opm_3buff_fns[i]) continue;
        if (NULL != module->opm_fns[i] && NULL != module->opm_3buff_fns[i]) OBJ_RETAIN(module);
        m2 = op->o_func.intrinsic.modules[i];
        m3 = op->o_3buff_intrinsic.modules[i];
        if (NULL != m2) OBJ_RETAIN(m2);
        if (NULL != m3) OBJ_RETAIN(m3);
        (void) ompi_amd_op_set_fallback(op->o_f_to_c_index, i,
                                        (ompi_amd_op_handler_fn_t) op->o_func.intrinsic.fns[i],
                                        (struct ompi_op_base_module_1_0_0_t *) m2,
                                        (ompi_amd_op_3buff_handler_fn_t) op->o_3buff_intrinsic.fns[i],
                                        (struct ompi_op_base_module_1_0_0_t *) m3);
    }
    return OMPI_SUCCESS;
}

static struct ompi_op_base_module_1_0_0_t *
rocm_component_op_query(struct ompi_op_t *op, int *priority)
{
    const ompi_amd_op_handler_fn_t *row2;
    const ompi_amd_op_3buff_handler_fn_t *row3;
    ompi_op_base_module_t *module;
    int i, used = 0;

    if (0 == (OMPI_OP_FLAGS_INTRINSIC & op->o_flags)) {
        return NULL;
    }
    row2 = ompi_amd_op_handler_row(op->o_f_to_c_index);
    row3 = ompi_amd_op_3buff_handler_row(op->o_f_to_c_index);
    if (NULL == row2 || NULL == row3) {
        return NULL;
    }
    module = OBJ_NEW(ompi_op_base_module_t);
    if (NULL == module) {
        return NULL;
    }
    for (i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        ompi_op_base_handler_fn_t base2 = op->o_func.intrinsic.fns[i];
        ompi_op_base_3buff_handler_fn_t base3 = op->o_3buff_intrinsic.fns[i];
        if (NULL != base2 && NULL != row2[i]) {
            module->opm_fns[i] = (ompi_op_base_handler_fn_t) row2[i];
            ++used;
        }
        if (NULL != base3 && NULL != row3[i]) {
            module->opm_3buff_fns[i] = (ompi_op_base_3buff_handler_fn_t) row3[i];
            ++used;
        }
    }
    module->opm_enable = rocm_module_enable;
    if (0 == used) {
        OBJ_RELEASE(module);
        return NULL;
    }
    *priority = mca_op_rocm_component.priority;
    return module;
}
