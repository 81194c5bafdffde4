/*
 * pml/rocm — device-buffer point-to-point for Open MPI's PML framework
 * (ompi/mca/pml/pml.h:233-506) through libompi_amd.so (include/ompi_amd_p2p.h).
 *
 * Interposition, not selection: like pml/v (pml_v_component.c:123-160) the
 * component is never selected (pmlm_init returns NULL); its close, which the
 * PML base runs after it picked the real PML (ob1), saves that PML's module
 * table and installs pml/rocm's functions into mca_pml, delegating what they
 * do not take.  Drop-in: copy this directory to ompi/mca/pml/rocm/
 * (INTEGRATION.md §4).
 *
 * What goes through the library: user-tag traffic (tag >= 0, and
 * MPI_ANY_TAG receives / probes) on a node-local intra-communicator of 2..16
 * ranks for which pml_add_comm created a library communicator.  By default
 * the rule depends on the communicator and the tag only — never on buffer
 * residency, which MPI lets differ between sender and receiver — so both
 * ends of every message meet in one matching engine.  The library takes
 * host buffers itself (pooled device stages, no allocation or export per
 * message); non-contiguous datatypes are packed on the host first.
 * pml_rocm_host_path = 1 sends every host-buffer operation to the saved PML
 * instead (zero library calls for host traffic) for applications whose
 * senders and receivers always agree on residency: a host-buffer send
 * matched by a device-buffer receive would then never meet it.  Negative
 * (system) tags, used by the collectives' own messages, and MPI_PROC_NULL
 * stay on the saved PML.  Matched probes (improbe / mprobe / imrecv / mrecv)
 * of library traffic are refused (OMPI_ERR_NOT_SUPPORTED).  Blocking calls
 * never time out (they drive opal_progress while they wait, as ob1 does).
 */
#ifndef MCA_PML_ROCM_H
#define MCA_PML_ROCM_H

#include "ompi_config.h"

#include "mpi.h"
#include "ompi/communicator/communicator.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/mca/pml/pml.h"
#include "ompi/request/request.h"

#include "ompi_amd_p2p.h"

BEGIN_C_DECLS

typedef struct mca_pml_rocm_component_t {
    mca_pml_base_component_2_0_0_t super;
    int enable;          /* pml_rocm_enable (1): interpose at close */
    int timeout_ms;      /* pml_rocm_timeout_ms: host wait limit (0, the default: none) */
    int own_stream;      /* pml_rocm_own_stream: a communicator's transfers on a hardware queue of their own */
    int host_path;       /* pml_rocm_host_path: 1 = host buffers to the saved PML */
} mca_pml_rocm_component_t;

OMPI_MODULE_DECLSPEC extern mca_pml_rocm_component_t mca_pml_rocm_component;

/* the saved (host) PML and whether pml/rocm is installed */
extern mca_pml_base_module_t mca_pml_rocm_host;
extern int mca_pml_rocm_installed;

/* A point-to-point request of library traffic: a library request behind an
 * ompi_request_t, plus the staging of a host / non-contiguous buffer and,
 * for persistent requests, the arguments of the next start. */
typedef struct mca_pml_rocm_request_t {
    ompi_request_t super;
    ompi_amd_p2p_request_t *lib;
    int is_send;
    /* the operation (persistent: replayed by every start) */
    void *buf;
    size_t count;
    struct ompi_datatype_t *dtype;
    int peer, tag, mode;
    struct ompi_communicator_t *comm;
    /* packing of a non-contiguous datatype (NULL: the user buffer itself
     * goes to the library, host or device): a device buffer from the
     * component's pool, packed / unpacked by one kernel (stage_dev), or
     * host memory packed on the host */
    void *stage;
    int stage_dev;
    size_t bytes;
    /* a device buffer on the saved PML: its request, and the host copy of
     * the buffer's typed span it runs on (hspan - hgap = the typed base) */
    ompi_request_t *inner;
    char *hspan;
    ptrdiff_t hgap;
    size_t hbytes;
    struct mca_pml_rocm_request_t *next_active;
} mca_pml_rocm_request_t;

OBJ_CLASS_DECLARATION(mca_pml_rocm_request_t);

/* library communicator of `comm`, or NULL when pml/rocm does not take it */
ompi_amd_comm_t *mca_pml_rocm_comm_of(struct ompi_communicator_t *comm);
/* requests on the active list (started, not yet completed; diagnostics) */
int mca_pml_rocm_active_count(void);

END_C_DECLS

#endif /* MCA_PML_ROCM_H */
