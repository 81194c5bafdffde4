/*
 * osc/rocm: one-sided communication on device windows, backed by
 * libompi_amd.so (include/ompi_amd_osc.h).  Copy to ompi/mca/osc/rocm/.
 *
 * Selected by the osc framework (ompi_osc_base_select) for MPI_Win_create
 * over device memory and MPI_Win_allocate with info "ompi_amd_device" =
 * true, on node-local intra-communicators, at priority osc_rocm_priority
 * (default 101: above osc/sm's 100, osc_sm_component.c:183).  Each window
 * owns a libompi_amd communicator (as osc/sm dups the communicator).
 */
#ifndef MCA_OSC_ROCM_H
#define MCA_OSC_ROCM_H

#include "ompi_config.h"

#include "mpi.h"
#include "ompi/mca/osc/osc.h"
#include "ompi/request/request.h"

#include "ompi_amd_coll.h"
#include "ompi_amd_osc.h"

BEGIN_C_DECLS

typedef struct ompi_osc_rocm_module_t {
    ompi_osc_base_module_t super;        /* first: win->w_osc_module points here */
    ompi_amd_comm_t *dev_comm;
    ompi_amd_win_t *dev_win;
    struct ompi_communicator_t *comm;
    int size;
} ompi_osc_rocm_module_t;

/* the MPI request of MPI_Rput / _Rget / _Raccumulate / _Rget_accumulate
 * over the library's (completed from opal_progress) */
typedef struct ompi_osc_rocm_request_t {
    ompi_request_t super;
    ompi_amd_rma_request_t *rma;
    struct ompi_osc_rocm_request_t *next_active;
} ompi_osc_rocm_request_t;
OBJ_CLASS_DECLARATION(ompi_osc_rocm_request_t);

typedef struct ompi_osc_rocm_component_t {
    ompi_osc_base_component_t super;
    int priority;    /* osc_rocm_priority */
    int timeout_ms;  /* osc_rocm_timeout_ms */
    int separate_model; /* osc_rocm_separate_model: MPI_Win_create memory peers cannot map gets a
                         * public copy (MPI_WIN_SEPARATE); 0 refuses such a window on every rank */
    int own_stream;     /* osc_rocm_own_stream: a window's epochs on a hardware queue of their own */
    unsigned windows;  /* windows created so far (names the device communicator) */
} ompi_osc_rocm_component_t;

OMPI_MODULE_DECLSPEC extern ompi_osc_rocm_component_t mca_osc_rocm_component;

END_C_DECLS

#endif /* MCA_OSC_ROCM_H */
