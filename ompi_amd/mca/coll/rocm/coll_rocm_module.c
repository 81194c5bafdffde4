/*
 * coll/rocm component + module.
 *
 * Selection: comm_query accepts node-local intra-communicators of at most
 * OMPI_AMD_MAX_RANKS ranks when a HIP device is visible; enable saves the
 * previously selected allreduce / reduce / reduce_scatter /
 * reduce_scatter_block / scan / exscan / allgather / bcast (coll/tuned, coll/basic for scan and exscan;
 * coll_base_comm_select.c:158-232 enables in ascending priority) and creates
 * the libompi_amd communicator.
 *
 * Per call every rank decides locally whether the device path applies
 * (predefined datatype, intrinsic op with a device kernel, device buffers),
 * then the ranks agree (ompi_amd_comm_agree) so that all of them take the
 * same path — MPI lets buffer residency differ between ranks.  The device
 * path is blocking like every MPI collective: ompi_amd_comm_sync waits for
 * the stream and surfaces a device-side timeout as an MPI error.
 *
 * Persistent allreduce (MPI_Allreduce_init) builds a library plan (the
 * peers' buffer mappings are swapped and pinned once, at init) behind an
 * ompi_request_t: req_start enqueues the plan's kernels with no host
 * rendezvous and puts the request on the active list.  Nonblocking
 * allreduce (MPI_Iallreduce) posts a library request (it never waits for a
 * peer) and goes on the same list.  The progress callback (registered with
 * opal_progress, as coll/libnbc does, coll_libnbc_component.c:430-475)
 * completes a request when the library reports its device work finished
 * (and, for iallreduce, launches deferred work whose handle swap is
 * complete), carrying a device-side failure into req_status.
 */
#include "ompi_config.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpi.h"
#include "ompi/constants.h"
#include "ompi/communicator/communicator.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/mca/coll/base/base.h"
#include "ompi/mca/coll/coll.h"
#include "ompi/op/op.h"
#include "ompi/runtime/ompi_rte.h"
#include "opal/mca/base/mca_base_var.h"
#include "opal/mca/threads/mutex.h"
#include "opal/runtime/opal_progress.h"

#include "coll_rocm.h"
#include "ompi_amd.h"

/* ------------------------------------------------------------- component */

static int rocm_register(void);

mca_coll_rocm_component_t mca_coll_rocm_component = {
    .super = {
        .collm_version = {
            MCA_COLL_BASE_VERSION_2_0_0,
            .mca_component_name = "rocm",
            MCA_BASE_MAKE_VERSION(component, OMPI_MAJOR_VERSION, OMPI_MINOR_VERSION,
                                  OMPI_RELEASE_VERSION),
            .mca_register_component_params = rocm_register,
        },
        .collm_data = { MCA_BASE_METADATA_PARAM_CHECKPOINT },
        .collm_init_query = mca_coll_rocm_init_query,
        .collm_comm_query = mca_coll_rocm_comm_query,
    },
    .priority = 80,
    .small_bytes = 1 << 20,
    .zero_copy = 1,
    .timeout_ms = 30000,
    .algorithm = 2,
    .user_ipc = 0,
    .autotune = 1,
    .land_blocking = 0,
    .copy_nt = -1,
    .residency = ROCM_RES_AUTO,
    .residency_lock = 8,
    .residency_recheck = 256,
    .max_device_mib = 1024,
    .own_stream = 1,
};

static int rocm_register(void)
{
    mca_base_component_t *c = &mca_coll_rocm_component.super.collm_version;
    (void) mca_base_component_var_register(c, "priority", "Priority of coll/rocm",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.priority);
    (void) mca_base_component_var_register(c, "small_bytes",
                                           "Messages up to this size are staged through the IPC scratch",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.small_bytes);
    (void) mca_base_component_var_register(c, "zero_copy",
                                           "Large messages peer to peer (through shadows, or the caller's buffers with user_ipc)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.zero_copy);
    (void) mca_base_component_var_register(c, "timeout_ms",
                                           "Device barrier spin limit before the collective fails",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.timeout_ms);
    (void) mca_base_component_var_register(c, "allreduce_algorithm",
                                           "Large-message allreduce data movement: 0 pull, 1 pull+push, 2 push (default; push-gather "
                                           "through the landing buffers when user_ipc is 0), 3 push-land "
                                           "(results stored into every rank's landing buffer, then a local "
                                           "copy; push when user_ipc is 1)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.algorithm);
    (void) mca_base_component_var_register(c, "user_ipc",
                                           "Let peers map the caller's buffers (zero-copy); 0 stages every "
                                           "large call through the communicator's exported shadow arena",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.user_ipc);
    (void) mca_base_component_var_register(c, "autotune",
                                           "Large staged allreduces pick their scheme (push-gather or "
                                           "push-land or pull) and grid by measurement: the first eighteen calls "
                                           "of a size bucket try each of nine candidates twice, all ranks then "
                                           "take the fastest; 0 keeps "
                                           "coll_rocm_allreduce_algorithm",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.autotune);
    (void) mca_base_component_var_register(c, "land_blocking",
                                           "1: blocking allgather / bcast of zero-copy sizes store into the "
                                           "peers' landing buffers (as the nonblocking and persistent forms "
                                           "always do) instead of pulling from the peers' shadows",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.land_blocking);
    (void) mca_base_component_var_register(c, "copy_nt",
                                           "1: the collectives' copy and fold kernels store "
                                           "non-temporally (streaming cache policy); 0: plain stores; "
                                           "-1 (default): non-temporal, and the large-allreduce "
                                           "autotune measures both kinds",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.copy_nt);
    (void) mca_base_component_var_register(c, "residency",
                                           "Where blocking collectives run: 0 vote per call until the ranks "
                                           "agree coll_rocm_residency_lock times in a row, 1 device (host "
                                           "operands are staged), 2 host (the saved functions; device "
                                           "operands are staged)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.residency);
    (void) mca_base_component_var_register(c, "residency_lock",
                                           "Unanimous residency votes in a row before the vote stops (0: never)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.residency_lock);
    (void) mca_base_component_var_register(c, "residency_recheck",
                                           "Locked calls between two votes on whether any rank staged (0: never)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.residency_recheck);
    (void) mca_base_component_var_register(c, "max_device_mib",
                                           "Largest vector (reductions) or per-rank block (allgather, "
                                           "bcast) the device path takes, in MiB; larger calls go to "
                                           "the saved functions",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.max_device_mib);
    (void) mca_base_component_var_register(c, "own_stream",
                                           "1: each communicator's collectives run on a stream with a "
                                           "hardware queue of its own (MPI lets ranks order different "
                                           "communicators' calls differently; device waits of one "
                                           "must not queue in front of another's)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.own_stream);
    return OMPI_SUCCESS;
}

/* ------------------------------------------------------------- coll/tuned */

/* An int (or bool) variable of coll/tuned through the MCA variable system —
 * whatever set it: the environment, an mca-params.conf file, the command
 * line or MPI_T — or dflt when tuned is not built or the variable is not
 * registered. */
static int tuned_var_int(const char *name, int dflt, int is_bool)
{
    const int idx = mca_base_var_find("ompi", "coll", "tuned", name);
    const void *v = NULL;
    if (idx < 0 || OPAL_SUCCESS != mca_base_var_get_value(idx, &v, NULL, NULL) || NULL == v) return dflt;
    return is_bool ? (int) *(const bool *) v : *(const int *) v;
}

static int tuned_var_set_string(const char *name)
{
    const int idx = mca_base_var_find("ompi", "coll", "tuned", name);
    const void *v = NULL;
    if (idx < 0 || OPAL_SUCCESS != mca_base_var_get_value(idx, &v, NULL, NULL) || NULL == v) return 0;
    const char *str = *(char *const *) v;
    return NULL != str && '\0' != str[0];
}

/*
 * coll/tuned's own forcing, as its module reads it at communicator creation
 * (coll_tuned_module.c:211-231, coll_tuned_component.c:170-192): only with
 * coll_tuned_use_dynamic_rules, a forced algorithm per collective
 * (coll_tuned_<coll>_algorithm) and a rules file
 * (coll_tuned_dynamic_rules_filename, read per communicator and message size
 * by coll_tuned_dynamic_file.c:57).  The device path must fold in the order
 * coll/tuned would, so each forced algorithm it implements goes to the
 * library; a blocking reduction whose tuned algorithm it does not implement
 * — or any of them under a rules file, whose per-size choices the library
 * does not replay — is declined here and runs in the saved function (on host
 * copies of device operands, as every declined call does).  Nonblocking and
 * persistent reductions are libnbc's in the reference, which these variables
 * do not steer.
 */
static void rocm_tuned_config(mca_coll_rocm_module_t *m)
{
    const int dyn = tuned_var_int("use_dynamic_rules", 0, 1);
    int ar = 0, red = 0, rs = 0, rsb = 0, red_ok;
    m->tuned_decline = 0;
    if (dyn && tuned_var_set_string("dynamic_rules_filename"))
        m->tuned_decline = ROCM_TUNED_ALLREDUCE | ROCM_TUNED_REDUCE | ROCM_TUNED_RS | ROCM_TUNED_RSB;
    if (dyn) {  /* without dynamic rules tuned ignores its forcing variables */
        ar = tuned_var_int("allreduce_algorithm", 0, 0);
        red = tuned_var_int("reduce_algorithm", 0, 0);
        rs = tuned_var_int("reduce_scatter_algorithm", 0, 0);
        rsb = tuned_var_int("reduce_scatter_block_algorithm", 0, 0);
    }
    red_ok = OMPI_AMD_SUCCESS == ompi_amd_comm_set_param(m->dev_comm, "tuned_reduce_algorithm", red);
    if (!red_ok) m->tuned_decline |= ROCM_TUNED_REDUCE;
    /* allreduce 2 (nonoverlapping) reduces through coll/tuned's reduce */
    if (OMPI_AMD_SUCCESS != ompi_amd_comm_set_param(m->dev_comm, "tuned_allreduce_algorithm", ar) ||
        (2 == ar && !red_ok))
        m->tuned_decline |= ROCM_TUNED_ALLREDUCE;
    /* reduce_scatter 1 (non-overlapping) reduces through it too */
    if (OMPI_AMD_SUCCESS != ompi_amd_comm_set_param(m->dev_comm, "tuned_reduce_scatter_algorithm", rs) ||
        (1 == rs && !red_ok))
        m->tuned_decline |= ROCM_TUNED_RS;
    /* reduce_scatter_block: basic_linear (the fixed choice, 1) reduces through it */
    if (OMPI_AMD_SUCCESS != ompi_amd_comm_set_param(m->dev_comm, "tuned_reduce_scatter_block_algorithm",
                                                    rsb) || !red_ok)
        m->tuned_decline |= ROCM_TUNED_RSB;
}

/* ------------------------------------------------------------- module */

static void rocm_module_construct(mca_coll_rocm_module_t *m)
{
    memset(&m->c_coll, 0, sizeof(m->c_coll));
    m->dev_comm = NULL;
    m->mode = ROCM_RES_AUTO;
    m->forced = 0;
    m->streak_dev = m->streak_host = 0;
    m->since_check = m->mismatched = 0;
    m->tuned_decline = 0;
    for (int k = 0; k < 2; ++k) {
        m->dstage[k] = m->hstage[k] = NULL;
        m->dstage_bytes[k] = m->hstage_bytes[k] = 0;
    }
}

static void rocm_module_destruct(mca_coll_rocm_module_t *m)
{
    if (NULL != m->c_coll.coll_allreduce_module) OBJ_RELEASE(m->c_coll.coll_allreduce_module);
    if (NULL != m->c_coll.coll_reduce_module) OBJ_RELEASE(m->c_coll.coll_reduce_module);
    if (NULL != m->c_coll.coll_reduce_scatter_module)
        OBJ_RELEASE(m->c_coll.coll_reduce_scatter_module);
    if (NULL != m->c_coll.coll_scan_module) OBJ_RELEASE(m->c_coll.coll_scan_module);
    if (NULL != m->c_coll.coll_exscan_module) OBJ_RELEASE(m->c_coll.coll_exscan_module);
    if (NULL != m->c_coll.coll_reduce_scatter_block_module)
        OBJ_RELEASE(m->c_coll.coll_reduce_scatter_block_module);
    if (NULL != m->c_coll.coll_allgather_module) OBJ_RELEASE(m->c_coll.coll_allgather_module);
    if (NULL != m->c_coll.coll_bcast_module) OBJ_RELEASE(m->c_coll.coll_bcast_module);
    if (NULL != m->c_coll.coll_allreduce_init_module)
        OBJ_RELEASE(m->c_coll.coll_allreduce_init_module);
    if (NULL != m->c_coll.coll_iallreduce_module) OBJ_RELEASE(m->c_coll.coll_iallreduce_module);
    if (NULL != m->c_coll.coll_iallgather_module) OBJ_RELEASE(m->c_coll.coll_iallgather_module);
    if (NULL != m->c_coll.coll_ibcast_module) OBJ_RELEASE(m->c_coll.coll_ibcast_module);
    if (NULL != m->c_coll.coll_ireduce_scatter_block_module)
        OBJ_RELEASE(m->c_coll.coll_ireduce_scatter_block_module);
    if (NULL != m->c_coll.coll_ireduce_module) OBJ_RELEASE(m->c_coll.coll_ireduce_module);
    if (NULL != m->c_coll.coll_iscan_module) OBJ_RELEASE(m->c_coll.coll_iscan_module);
    if (NULL != m->c_coll.coll_iexscan_module) OBJ_RELEASE(m->c_coll.coll_iexscan_module);
    if (NULL != m->c_coll.coll_ireduce_scatter_module)
        OBJ_RELEASE(m->c_coll.coll_ireduce_scatter_module);
    if (NULL != m->c_coll.coll_reduce_scatter_block_init_module)
        OBJ_RELEASE(m->c_coll.coll_reduce_scatter_block_init_module);
    if (NULL != m->c_coll.coll_allgather_init_module)
        OBJ_RELEASE(m->c_coll.coll_allgather_init_module);
    if (NULL != m->c_coll.coll_bcast_init_module) OBJ_RELEASE(m->c_coll.coll_bcast_init_module);
    if (NULL != m->c_coll.coll_reduce_init_module) OBJ_RELEASE(m->c_coll.coll_reduce_init_module);
    if (NULL != m->c_coll.coll_reduce_scatter_init_module)
        OBJ_RELEASE(m->c_coll.coll_reduce_scatter_init_module);
    if (NULL != m->c_coll.coll_scan_init_module) OBJ_RELEASE(m->c_coll.coll_scan_init_module);
    if (NULL != m->c_coll.coll_exscan_init_module) OBJ_RELEASE(m->c_coll.coll_exscan_init_module);
    if (NULL != m->dev_comm) (void) ompi_amd_comm_destroy(m->dev_comm);
    for (int k = 0; k < 2; ++k) {
        (void) ompi_amd_device_free(m->dstage[k]);
        free(m->hstage[k]);
    }
}

OBJ_CLASS_INSTANCE(mca_coll_rocm_module_t, mca_coll_base_module_t, rocm_module_construct,
                   rocm_module_destruct);

int mca_coll_rocm_init_query(bool enable_progress_threads, bool enable_mpi_threads)
{
    return ompi_amd_device_count() > 0 ? OMPI_SUCCESS : OMPI_ERR_NOT_AVAILABLE;
}

mca_coll_base_module_t *mca_coll_rocm_comm_query(struct ompi_communicator_t *comm,
                                                 int *priority)
{
    mca_coll_rocm_module_t *m;
    if (OMPI_COMM_IS_INTER(comm) || ompi_comm_size(comm) < 2 ||
        ompi_comm_size(comm) > OMPI_AMD_MAX_RANKS ||
        ompi_group_have_remote_peers(comm->c_local_group)) {
        return NULL;  /* one node, one process per GPU */
    }
    m = OBJ_NEW(mca_coll_rocm_module_t);
    if (NULL == m) return NULL;
    *priority = mca_coll_rocm_component.priority;
    m->super.coll_module_enable = mca_coll_rocm_module_enable;
    m->super.coll_allreduce = mca_coll_rocm_allreduce;
    m->super.coll_reduce = mca_coll_rocm_reduce;
    m->super.coll_reduce_scatter = mca_coll_rocm_reduce_scatter;
    m->super.coll_scan = mca_coll_rocm_scan;
    m->super.coll_exscan = mca_coll_rocm_exscan;
    m->super.coll_reduce_scatter_block = mca_coll_rocm_reduce_scatter_block;
    m->super.coll_allgather = mca_coll_rocm_allgather;
    m->super.coll_bcast = mca_coll_rocm_bcast;
    m->super.coll_iallreduce = mca_coll_rocm_iallreduce;
    m->super.coll_iallgather = mca_coll_rocm_iallgather;
    m->super.coll_ibcast = mca_coll_rocm_ibcast;
    m->super.coll_ireduce_scatter_block = mca_coll_rocm_ireduce_scatter_block;
    m->super.coll_allreduce_init = mca_coll_rocm_allreduce_init;
    m->super.coll_ireduce = mca_coll_rocm_ireduce;
    m->super.coll_iscan = mca_coll_rocm_iscan;
    m->super.coll_iexscan = mca_coll_rocm_iexscan;
    m->super.coll_ireduce_scatter = mca_coll_rocm_ireduce_scatter;
    m->super.coll_reduce_scatter_block_init = mca_coll_rocm_reduce_scatter_block_init;
    m->super.coll_allgather_init = mca_coll_rocm_allgather_init;
    m->super.coll_bcast_init = mca_coll_rocm_bcast_init;
    m->super.coll_reduce_init = mca_coll_rocm_reduce_init;
    m->super.coll_reduce_scatter_init = mca_coll_rocm_reduce_scatter_init;
    m->super.coll_scan_init = mca_coll_rocm_scan_init;
    m->super.coll_exscan_init = mca_coll_rocm_exscan_init;
    return &m->super;
}

int mca_coll_rocm_module_enable(mca_coll_base_module_t *module, struct ompi_communicator_t *comm)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    char name[128];
    int rc;

#define SAVE(fn)                                                            \
    do {                                                                    \
        if (NULL == comm->c_coll->coll_##fn##_module) return OMPI_ERR_NOT_FOUND; \
        m->c_coll.coll_##fn = comm->c_coll->coll_##fn;                     \
        m->c_coll.coll_##fn##_module = comm->c_coll->coll_##fn##_module;   \
        OBJ_RETAIN(m->c_coll.coll_##fn##_module);                          \
    } while (0)
    SAVE(allreduce);
    SAVE(reduce);
    SAVE(reduce_scatter);
    SAVE(scan);
    SAVE(exscan);
    SAVE(reduce_scatter_block);
    SAVE(allgather);
    SAVE(bcast);
    SAVE(iallreduce);
    SAVE(iallgather);
    SAVE(ibcast);
    SAVE(ireduce_scatter_block);
    SAVE(allreduce_init);
    SAVE(ireduce);
    SAVE(iscan);
    SAVE(iexscan);
    SAVE(ireduce_scatter);
    SAVE(reduce_scatter_block_init);
    SAVE(allgather_init);
    SAVE(bcast_init);
    SAVE(reduce_init);
    SAVE(reduce_scatter_init);
    SAVE(scan_init);
    SAVE(exscan_init);
#undef SAVE

    /* node-unique segment name: job id + communicator id */
    snprintf(name, sizeof(name), "%u.%u", (unsigned) OMPI_PROC_MY_NAME->jobid,
             (unsigned) ompi_comm_get_cid(comm));
    rc = ompi_amd_comm_create(name, ompi_comm_rank(comm), ompi_comm_size(comm), -1, &m->dev_comm);
    if (OMPI_AMD_SUCCESS != rc) return OMPI_ERR_NOT_AVAILABLE;
    (void) ompi_amd_comm_set_param(m->dev_comm, "small_bytes", mca_coll_rocm_component.small_bytes);
    (void) ompi_amd_comm_set_param(m->dev_comm, "zero_copy", mca_coll_rocm_component.zero_copy);
    (void) ompi_amd_comm_set_param(m->dev_comm, "timeout_ms", mca_coll_rocm_component.timeout_ms);
    (void) ompi_amd_comm_set_param(m->dev_comm, "algorithm", mca_coll_rocm_component.algorithm);
    (void) ompi_amd_comm_set_param(m->dev_comm, "user_ipc", mca_coll_rocm_component.user_ipc);
    (void) ompi_amd_comm_set_param(m->dev_comm, "land_blocking", mca_coll_rocm_component.land_blocking);
    (void) ompi_amd_comm_set_param(m->dev_comm, "copy_nt", mca_coll_rocm_component.copy_nt);
    (void) ompi_amd_comm_set_param(m->dev_comm, "own_stream", mca_coll_rocm_component.own_stream);
    rocm_tuned_config(m);
    /* last: setting the scheme turns autotuning off */
    (void) ompi_amd_comm_set_param(m->dev_comm, "autotune", mca_coll_rocm_component.autotune);
    if (ROCM_RES_DEVICE == mca_coll_rocm_component.residency ||
        ROCM_RES_HOST == mca_coll_rocm_component.residency) {
        m->mode = mca_coll_rocm_component.residency;
        m->forced = 1;
    }
    return OMPI_SUCCESS;
}

/* ------------------------------------------------------------- helpers */

static int to_ompi_err(int rc)
{
    switch (rc) {
    case OMPI_AMD_SUCCESS: return OMPI_SUCCESS;
    case OMPI_AMD_ERR_BAD_PARAM: return OMPI_ERR_BAD_PARAM;
    case OMPI_AMD_ERR_UNSUPPORTED: return OMPI_ERR_NOT_SUPPORTED;
    case OMPI_AMD_ERR_TIMEOUT: return OMPI_ERR_TIMEOUT;
    default: return OMPI_ERROR;
    }
}

/* op/type code of a predefined datatype, or -1 */
static int type_code(struct ompi_datatype_t *dtype)
{
    if (!ompi_datatype_is_predefined(dtype)) return -1;
    return ompi_op_ddt_map[dtype->id];
}

static int dev(const void *p)
{
    return MPI_IN_PLACE == p || ompi_amd_is_device_pointer(p);
}

/* every rank must answer the same way (buffer residency may differ): the
 * per-call vote the nonblocking and persistent entry points keep */
static bool take_device_path(mca_coll_rocm_module_t *m, int local_ok)
{
    int all_ok = 0;
    if (OMPI_AMD_SUCCESS != ompi_amd_comm_agree(m->dev_comm, local_ok, &all_ok)) return false;
    return all_ok != 0;
}

/* ------------------------------------------------------------- residency */

enum { ROCM_SAVED = 0, ROCM_DEVICE = 1, ROCM_SAVED_HOST = 2 };

/*
 * The path of one blocking call, the same on every rank without a message
 * once the module is locked.
 *
 * uniform_ok is what every rank computes alike: a reduction's count,
 * datatype and op are the same on all ranks (MPI-4.1 §6.9.1), so "predefined
 * type, intrinsic op with a device kernel" needs no agreement.  local_dev is
 * this rank's operand residency, which MPI lets differ.
 *
 * AUTO votes on local_dev (one shared-memory rendezvous, as every call did
 * before): all device -> the device path, otherwise the saved function with
 * the operands as they are.  After residency_lock unanimous votes in a row
 * the module locks to DEVICE or HOST and stops voting.  Locked, a rank whose
 * operands are not where the locked path runs stages them (rocm_stage):
 * host operands into device memory for the device path, device operands
 * into host memory for the saved host path (coll/cuda's approach,
 * coll_cuda_allreduce.c:42-72).  Every residency_recheck locked calls one
 * vote asks whether any rank staged since the last one; if so the module
 * returns to AUTO.  Calls are counted per module in call order, which every
 * rank shares, so every rank votes at the same calls.
 */
static int rocm_path(mca_coll_rocm_module_t *m, int uniform_ok, int local_dev)
{
    const int size = ompi_amd_comm_size(m->dev_comm);
    const int lock = mca_coll_rocm_component.residency_lock;
    const int recheck = mca_coll_rocm_component.residency_recheck;
    int n_yes = 0;
    if (!uniform_ok) return ROCM_SAVED;
    if (ROCM_RES_AUTO != m->mode) {
        const int device = ROCM_RES_DEVICE == m->mode;
        if (!local_dev != !device) m->mismatched++;
        if (!m->forced && recheck > 0 && ++m->since_check >= recheck) {
            if (OMPI_AMD_SUCCESS == ompi_amd_comm_vote(m->dev_comm, m->mismatched > 0, &n_yes) &&
                n_yes > 0) {
                m->mode = ROCM_RES_AUTO;
                m->streak_dev = m->streak_host = 0;
            }
            m->since_check = m->mismatched = 0;
        }
        return device ? ROCM_DEVICE : ROCM_SAVED_HOST;
    }
    if (OMPI_AMD_SUCCESS != ompi_amd_comm_vote(m->dev_comm, local_dev, &n_yes)) return ROCM_SAVED;
    if (n_yes == size) {
        m->streak_dev++;
        m->streak_host = 0;
    } else if (0 == n_yes) {
        m->streak_host++;
        m->streak_dev = 0;
    } else {
        m->streak_dev = m->streak_host = 0;
    }
    if (lock > 0 && (m->streak_dev >= lock || m->streak_host >= lock)) {
        m->mode = m->streak_dev >= lock ? ROCM_RES_DEVICE : ROCM_RES_HOST;
        m->since_check = m->mismatched = 0;
    }
    return n_yes == size ? ROCM_DEVICE : ROCM_SAVED;
}

/* One operand of a collective: the caller's buffer (NULL or MPI_IN_PLACE:
 * nothing to stage), count elements of dtype, and whether the collective
 * reads / writes it.  rocm_stage fills in what the collective gets. */
typedef struct {
    void *user;
    size_t count;
    struct ompi_datatype_t *dtype;
    int in, out;
    void *use;
    int how;        /* 0 as is, 1 byte copy of the typed span, 2 packed */
    ptrdiff_t gap;  /* true lower bound of the span */
    size_t bytes;
    char *hbuf;     /* packed: the host side of the pack / unpack */
    int contig;
} rocm_operand_t;

/* Staging memory of one operand slot: the module's grow-only buffers for
 * blocking calls, a nonblocking request's own for its lifetime. */
typedef char *(*rocm_buf_fn)(void *ctx, int slot, int on_dev, size_t bytes);

/* a nonblocking call's staged operands (rocm_nb_begin), copied back and
 * freed when its request completes */
struct rocm_nb_stage {
    rocm_operand_t o[2];
    int n;
    void *dev[2], *host[2];
};
static void nb_stage_free(struct rocm_nb_stage *st);

/* grow-only staging memory of one operand slot */
static char *stage_buf(void *ctx, int slot, int on_dev, size_t bytes)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) ctx;
    void **p = on_dev ? &m->dstage[slot] : &m->hstage[slot];
    size_t *have = on_dev ? &m->dstage_bytes[slot] : &m->hstage_bytes[slot];
    if (m->fail_stage) {  /* test hook (coll harness): as if the allocation failed */
        m->fail_stage = 0;
        return NULL;
    }
    if (bytes > *have) {
        const size_t want = bytes > 2 * *have ? bytes : 2 * *have;
        if (on_dev) {
            (void) ompi_amd_device_free(*p);
            *p = NULL;
            if (OMPI_AMD_SUCCESS != ompi_amd_device_alloc(p, want)) *p = NULL;
        } else {
            free(*p);
            *p = malloc(want);
        }
        *have = NULL == *p ? 0 : want;
    }
    return (char *) *p;
}

/* Put every operand where the chosen path runs: device memory (packed when
 * its layout is not contiguous, since the device path moves bytes) or host
 * memory (the typed span as it is, for the saved function). */
/* the caller's input into a staged operand (again at every persistent start) */
static int stage_copy_in(const rocm_operand_t *x)
{
    if (2 == x->how) {
        if (x->in && (MPI_SUCCESS != ompi_datatype_sndrcv(x->user, (int) x->count, x->dtype,
                                                          x->hbuf, (int) x->bytes, MPI_BYTE) ||
                      OMPI_AMD_SUCCESS != ompi_amd_memcpy(x->use, x->hbuf, x->bytes))) {
            return OMPI_ERROR;
        }
    } else if (1 == x->how && (x->in || (x->out && !x->contig))) {
        /* an output's gaps must survive the copy back */
        if (OMPI_AMD_SUCCESS != ompi_amd_memcpy((char *) x->use + x->gap,
                                                (char *) x->user + x->gap, x->bytes)) {
            return OMPI_ERROR;
        }
    }
    return OMPI_SUCCESS;
}

static int rocm_stage_with(rocm_buf_fn get, void *ctx, rocm_operand_t *o, int n, int to_dev)
{
    for (int i = 0; i < n; ++i) {
        rocm_operand_t *x = &o[i];
        int is_dev, contig;
        x->use = x->user;
        x->how = 0;
        x->hbuf = NULL;
        if (NULL == x->user || MPI_IN_PLACE == x->user || 0 == x->count) continue;
        is_dev = ompi_amd_is_device_pointer(x->user);
        contig = ompi_datatype_is_contiguous_memory_layout(x->dtype, (int) x->count);
        if (to_dev ? (is_dev && contig) : !is_dev) continue;
        x->contig = contig;
        if (to_dev && !contig) {
            size_t size = 0;
            (void) ompi_datatype_type_size(x->dtype, &size);
            x->bytes = size * x->count;
            x->hbuf = get(ctx, i, 0, x->bytes);
            x->use = get(ctx, i, 1, x->bytes);
            if (NULL == x->hbuf || NULL == x->use) return OMPI_ERR_OUT_OF_RESOURCE;
            x->how = 2;
        } else {
            ptrdiff_t lb, ext, tlb, text;
            char *b;
            (void) ompi_datatype_get_extent(x->dtype, &lb, &ext);
            (void) ompi_datatype_get_true_extent(x->dtype, &tlb, &text);
            x->bytes = (x->count - 1) * (size_t) ext + (size_t) text;
            x->gap = tlb;
            b = get(ctx, i, to_dev, x->bytes);
            if (NULL == b) return OMPI_ERR_OUT_OF_RESOURCE;
            x->use = b - tlb;
            x->how = 1;
        }
        if (OMPI_SUCCESS != stage_copy_in(x)) return OMPI_ERROR;
    }
    return OMPI_SUCCESS;
}

static int rocm_stage(mca_coll_rocm_module_t *m, rocm_operand_t *o, int n, int to_dev)
{
    return rocm_stage_with(stage_buf, m, o, n, to_dev);
}

/* copy staged outputs back to the caller's buffers */
static int rocm_unstage_ops(const rocm_operand_t *o, int n, int rc)
{
    for (int i = 0; OMPI_SUCCESS == rc && i < n; ++i) {
        const rocm_operand_t *x = &o[i];
        if (!x->out || 0 == x->how) continue;
        if (1 == x->how) {
            if (OMPI_AMD_SUCCESS != ompi_amd_memcpy((char *) x->user + x->gap,
                                                    (char *) x->use + x->gap, x->bytes)) {
                rc = OMPI_ERROR;
            }
        } else if (OMPI_AMD_SUCCESS != ompi_amd_memcpy(x->hbuf, x->use, x->bytes) ||
                   MPI_SUCCESS != ompi_datatype_sndrcv(x->hbuf, (int) x->bytes, MPI_BYTE,
                                                       x->user, (int) x->count, x->dtype)) {
            rc = OMPI_ERROR;
        }
    }
    return rc;
}

static int rocm_unstage(mca_coll_rocm_module_t *m, const rocm_operand_t *o, int n, int rc)
{
    (void) m;
    return rocm_unstage_ops(o, n, rc);
}

/* Decide, and stage for the decision: *path is ROCM_DEVICE or a saved path.
 * The saved functions (coll/tuned, coll/basic) run on the host: whatever
 * the reason the device path is not taken — a user op, a derived datatype,
 * a slot without a device kernel, a vector past max_device_mib, or peers
 * whose operands are host memory — this rank's device operands are copied
 * to host memory first and its outputs back after, as coll/cuda does for
 * every call it wraps (coll_cuda_allreduce.c:42-72).  Host operands go as
 * they are. */
/* A staging failure after the device path was agreed (locked DEVICE: no
 * message at all) would leave the peers in the collective's first barrier
 * until timeout_ms: this rank raises the communicator's abort word instead,
 * so every rank's call fails within about 1 ms.  (On the saved host path
 * the peers are inside coll/tuned's messages, as with any rank that fails
 * a host collective: MPI_ERRORS_ARE_FATAL ends the job.) */
static int rocm_staging_failed(mca_coll_rocm_module_t *m, int path, int rc)
{
    if (OMPI_SUCCESS != rc && ROCM_DEVICE == path)
        (void) ompi_amd_comm_abort(m->dev_comm, OMPI_ERR_OUT_OF_RESOURCE == rc ? OMPI_AMD_ERR_HIP
                                                                               : OMPI_AMD_ERR_BAD_PARAM);
    return rc;
}

static int rocm_begin(mca_coll_rocm_module_t *m, int uniform_ok, int local_dev,
                      rocm_operand_t *o, int n, int *path)
{
    *path = rocm_path(m, uniform_ok, local_dev);
    for (int i = 0; i < n; ++i) {
        o[i].use = o[i].user;
        o[i].how = 0;
        o[i].hbuf = NULL;
    }
    return rocm_staging_failed(m, *path, rocm_stage(m, o, n, ROCM_DEVICE == *path));
}

static int rocm_dev_finish(mca_coll_rocm_module_t *m, const rocm_operand_t *o, int n, int rc)
{
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return rocm_unstage(m, o, n, to_ompi_err(rc));
}

/* ------------------------------------------------------------- collectives */

/* The device path moves at most coll_rocm_max_device_mib (1 GiB) of vector
 * per call: every peer-visible region is one IPC allocation, capped below
 * 2 GiB on ROCm 7.2, the push schemes need (N + 1) / N of
 * the vector in one landing buffer, and allgather / bcast stage a rank's
 * block (the root's whole buffer) in one shadow.  Larger calls go to the
 * saved functions.  The sizes tested are ones every rank computes alike
 * (a reduction's count, datatype and op; allgather's and bcast's type
 * signatures must match, MPI-4.1 §6.4), so every rank decides alike. */
static int bytes_ok(size_t bytes)
{
    return bytes <= ((size_t) mca_coll_rocm_component.max_device_mib << 20);
}

static int reduction_ok_n(struct ompi_datatype_t *dtype, struct ompi_op_t *op, size_t elems)
{
    const int t = type_code(dtype);
    return t >= 0 && ompi_op_is_intrinsic(op) && ompi_amd_op_supported(op->o_f_to_c_index, t) &&
           bytes_ok(elems * ompi_amd_type_extent(t));
}


int mca_coll_rocm_allreduce(const void *sbuf, void *rbuf, int count,
                            struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                            struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int inplace = MPI_IN_PLACE == sbuf;
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {rbuf, (size_t) count, dtype, inplace, 1}};
    int path, rc;
    rc = rocm_begin(m, reduction_ok_n(dtype, op, (size_t) count) && !(m->tuned_decline & ROCM_TUNED_ALLREDUCE),
                    dev(sbuf) && dev(rbuf), o, 2, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_allreduce(o[0].use, o[1].use, count, dtype, op, comm,
                                      m->c_coll.coll_allreduce_module);
        return rocm_unstage(m, o, 2, rc);
    }
    /* the call and its wait in one: a fused small allreduce stores its own
     * completion mark, so the wait launches nothing behind it */
    rc = ompi_amd_allreduce_wait(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use, (size_t) count,
                                 type_code(dtype), op->o_f_to_c_index);
    return rocm_unstage(m, o, 2, to_ompi_err(rc));
}

/* MPI_Reduce: rbuf is significant at the root only (MPI-3.1 §5.9.1), so
 * only the root's rbuf residency enters the local decision. */
int mca_coll_rocm_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                         struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                         mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int is_root = ompi_comm_rank(comm) == root;
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {is_root ? rbuf : NULL, (size_t) count, dtype, MPI_IN_PLACE == sbuf, 1}};
    int path, rc;
    rc = rocm_begin(m, reduction_ok_n(dtype, op, (size_t) count) && !(m->tuned_decline & ROCM_TUNED_REDUCE),
                    is_root ? dev(rbuf) && dev(sbuf) : ompi_amd_is_device_pointer(sbuf), o, 2, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_reduce(o[0].use, is_root ? o[1].use : rbuf, count, dtype, op, root, comm,
                                   m->c_coll.coll_reduce_module);
        return rocm_unstage(m, o, 2, rc);
    }
    rc = ompi_amd_reduce(m->dev_comm, o[0].use, is_root ? o[1].use : NULL, (size_t) count,
                         type_code(dtype), op->o_f_to_c_index, root, NULL);
    return rocm_dev_finish(m, o, 2, rc);
}

static int rocm_scan_common(const void *sbuf, void *rbuf, int count,
                            struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                            struct ompi_communicator_t *comm, mca_coll_rocm_module_t *m,
                            int exclusive)
{
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {rbuf, (size_t) count, dtype, MPI_IN_PLACE == sbuf, 1}};
    int path, rc;
    rc = rocm_begin(m, reduction_ok_n(dtype, op, (size_t) count), dev(sbuf) && dev(rbuf), o, 2, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = exclusive ? m->c_coll.coll_exscan(o[0].use, o[1].use, count, dtype, op, comm,
                                               m->c_coll.coll_exscan_module)
                       : m->c_coll.coll_scan(o[0].use, o[1].use, count, dtype, op, comm,
                                             m->c_coll.coll_scan_module);
        return rocm_unstage(m, o, 2, rc);
    }
    rc = (exclusive ? ompi_amd_exscan : ompi_amd_scan)(m->dev_comm, o[0].use, o[1].use,
                                                       (size_t) count, type_code(dtype),
                                                       op->o_f_to_c_index, NULL);
    return rocm_dev_finish(m, o, 2, rc);
}

int mca_coll_rocm_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                       struct ompi_op_t *op, struct ompi_communicator_t *comm,
                       mca_coll_base_module_t *module)
{
    return rocm_scan_common(sbuf, rbuf, count, dtype, op, comm, (mca_coll_rocm_module_t *) module, 0);
}

int mca_coll_rocm_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                         struct ompi_op_t *op, struct ompi_communicator_t *comm,
                         mca_coll_base_module_t *module)
{
    return rocm_scan_common(sbuf, rbuf, count, dtype, op, comm, (mca_coll_rocm_module_t *) module, 1);
}

int mca_coll_rocm_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts,
                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                 struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int n = ompi_comm_size(comm), inplace = MPI_IN_PLACE == sbuf;
    size_t counts[OMPI_AMD_MAX_RANKS], total = 0;
    int path, rc, i;
    for (i = 0; i < n; ++i) total += (size_t) rcounts[i];
    {
        rocm_operand_t o[2] = {{(void *) sbuf, total, dtype, 1, 0},
                               {rbuf, inplace ? total : (size_t) rcounts[ompi_comm_rank(comm)],
                                dtype, inplace, 1}};
        rc = rocm_begin(m, reduction_ok_n(dtype, op, total) && !(m->tuned_decline & ROCM_TUNED_RS),
                        dev(sbuf) && dev(rbuf), o, 2, &path);
        if (OMPI_SUCCESS != rc) return rc;
        if (ROCM_DEVICE != path) {
            rc = m->c_coll.coll_reduce_scatter(o[0].use, o[1].use, rcounts, dtype, op, comm,
                                               m->c_coll.coll_reduce_scatter_module);
            return rocm_unstage(m, o, 2, rc);
        }
        for (i = 0; i < n; ++i) counts[i] = (size_t) rcounts[i];
        rc = ompi_amd_reduce_scatter(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use, counts,
                                     type_code(dtype), op->o_f_to_c_index, NULL);
        return rocm_dev_finish(m, o, 2, rc);
    }
}

int mca_coll_rocm_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount,
                                       struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                       struct ompi_communicator_t *comm,
                                       mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const size_t all = (size_t) rcount * (size_t) ompi_comm_size(comm);
    const int inplace = MPI_IN_PLACE == sbuf;
    rocm_operand_t o[2] = {{(void *) sbuf, all, dtype, 1, 0},
                           {rbuf, inplace ? all : (size_t) rcount, dtype, inplace, 1}};
    int path, rc;
    rc = rocm_begin(m, reduction_ok_n(dtype, op, all) && !(m->tuned_decline & ROCM_TUNED_RSB),
                    dev(sbuf) && dev(rbuf), o, 2, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_reduce_scatter_block(o[0].use, o[1].use, rcount, dtype, op, comm,
                                                 m->c_coll.coll_reduce_scatter_block_module);
        return rocm_unstage(m, o, 2, rc);
    }
    rc = ompi_amd_reduce_scatter_block(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use,
                                       (size_t) rcount, type_code(dtype), op->o_f_to_c_index, NULL);
    return rocm_dev_finish(m, o, 2, rc);
}

/* allgather / bcast move bytes: any datatype qualifies (a rank whose layout
 * is not contiguous packs when the device path runs), so the uniform part
 * is always true and the vote covers residency and layout. */
int mca_coll_rocm_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                            void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                            struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int inplace = MPI_IN_PLACE == sbuf;
    const size_t all = (size_t) rcount * (size_t) ompi_comm_size(comm);
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) scount, sdtype, 1, 0},
                           {rbuf, all, rdtype, inplace, 1}};
    size_t rsize = 0;
    int path, rc, ok;
    (void) ompi_datatype_type_size(rdtype, &rsize);
    ok = ompi_datatype_is_contiguous_memory_layout(rdtype, (int) all) && dev(rbuf) && dev(sbuf) &&
         (inplace || ompi_datatype_is_contiguous_memory_layout(sdtype, scount));
    rc = rocm_begin(m, bytes_ok(rsize * (size_t) rcount), ok, o, 2, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_allgather(o[0].use, scount, sdtype, o[1].use, rcount, rdtype, comm,
                                      m->c_coll.coll_allgather_module);
        return rocm_unstage(m, o, 2, rc);
    }
    rc = ompi_amd_allgather(m->dev_comm, inplace ? (const void *) 1 : o[0].use, o[1].use,
                            rsize * (size_t) rcount, NULL);
    return rocm_dev_finish(m, o, 2, rc);
}

int mca_coll_rocm_bcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                        struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int is_root = ompi_comm_rank(comm) == root;
    rocm_operand_t o[1] = {{buf, (size_t) count, dtype, is_root, !is_root}};
    size_t size = 0;
    int path, rc;
    (void) ompi_datatype_type_size(dtype, &size);
    rc = rocm_begin(m, bytes_ok(size * (size_t) count),
                    ompi_datatype_is_contiguous_memory_layout(dtype, count) && dev(buf), o, 1, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_bcast(o[0].use, count, dtype, root, comm, m->c_coll.coll_bcast_module);
        return rocm_unstage(m, o, 1, rc);
    }
    rc = ompi_amd_bcast(m->dev_comm, o[0].use, size * (size_t) count, root, NULL);
    return rocm_dev_finish(m, o, 1, rc);
}

/* ------------------------------------------------------------- persistent */

static opal_mutex_t rocm_active_lock = OPAL_MUTEX_STATIC_INIT;
static mca_coll_rocm_request_t *rocm_active; /* started requests, not yet complete */
static int rocm_progress_registered;

/* opal_progress callback: complete the started requests whose device work
 * has finished (ompi_amd_plan_test queries the plan's completion event). */
static int rocm_progress(void)
{
    mca_coll_rocm_request_t **pp, *done = NULL;
    int completed = 0;
    if (NULL == rocm_active) return 0;
    OPAL_THREAD_LOCK(&rocm_active_lock);
    pp = &rocm_active;
    while (NULL != *pp) {
        mca_coll_rocm_request_t *r = *pp;
        int fin = 0, rc = OMPI_AMD_SUCCESS;
        if (NULL != r->inner) {  /* the saved function's request (host copies) */
            fin = REQUEST_COMPLETE(r->inner);
        } else {
            rc = NULL != r->plan ? ompi_amd_plan_test(r->plan, &fin)
                                 : ompi_amd_request_test(r->nbreq, &fin);
        }
        if (OMPI_AMD_SUCCESS != rc || fin) {
            r->super.req_status.MPI_ERROR = NULL != r->inner ? r->inner->req_status.MPI_ERROR
                                                             : to_ompi_err(rc);
            *pp = r->next_active;
            r->next_active = done;
            done = r;
        } else {
            pp = &r->next_active;
        }
    }
    OPAL_THREAD_UNLOCK(&rocm_active_lock);
    while (NULL != done) {
        mca_coll_rocm_request_t *r = done;
        done = r->next_active;
        r->next_active = NULL;
        if (NULL != r->inner) {
            if (r->super.req_persistent) {
                r->inner->req_state = OMPI_REQUEST_INACTIVE;  /* as MPI_Wait leaves it */
            } else {
                (void) ompi_request_free(&r->inner);
                r->inner = NULL;
            }
        }
        if (NULL != r->stage) {  /* staged outputs back to the caller's buffers */
            r->super.req_status.MPI_ERROR =
                rocm_unstage_ops(r->stage->o, r->stage->n, r->super.req_status.MPI_ERROR);
            if (!r->super.req_persistent) {  /* a persistent request keeps it for its starts */
                nb_stage_free(r->stage);
                r->stage = NULL;
            }
        }
        ompi_request_complete(&r->super, true);
        ++completed;
    }
    return completed;
}

static void rocm_link_active(mca_coll_rocm_request_t *r)
{
    OPAL_THREAD_LOCK(&rocm_active_lock);
    r->next_active = rocm_active;
    rocm_active = r;
    if (!rocm_progress_registered) {
        rocm_progress_registered = 1;
        (void) opal_progress_register(rocm_progress);
    }
    OPAL_THREAD_UNLOCK(&rocm_active_lock);
}

static void rocm_unlink_active(mca_coll_rocm_request_t *r)
{
    mca_coll_rocm_request_t **pp;
    OPAL_THREAD_LOCK(&rocm_active_lock);
    for (pp = &rocm_active; NULL != *pp; pp = &(*pp)->next_active) {
        if (*pp == r) {
            *pp = r->next_active;
            break;
        }
    }
    OPAL_THREAD_UNLOCK(&rocm_active_lock);
    r->next_active = NULL;
}

/* MPI_Start / MPI_Startall (ompi/request/request.h:60-77) */
static int rocm_request_start(size_t count, ompi_request_t **requests)
{
    size_t i;
    for (i = 0; i < count; ++i) {
        mca_coll_rocm_request_t *r = (mca_coll_rocm_request_t *) requests[i];
        int rc;
        if (NULL == r) continue;
        if (OMPI_REQUEST_ACTIVE == r->super.req_state && !REQUEST_COMPLETE(&r->super)) {
            return OMPI_ERR_REQUEST; /* started twice without a completion */
        }
        r->super.req_complete = REQUEST_PENDING;
        r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
        r->super.req_state = OMPI_REQUEST_ACTIVE;
        rc = OMPI_SUCCESS;
        for (int k = 0; NULL != r->stage && k < r->stage->n; ++k) {  /* this start's inputs */
            if (OMPI_SUCCESS != stage_copy_in(&r->stage->o[k])) rc = OMPI_ERROR;
        }
        if (OMPI_SUCCESS == rc) {
            rc = NULL != r->inner ? r->inner->req_start(1, &r->inner)
                                  : to_ompi_err(ompi_amd_plan_start(r->plan, NULL));
        }
        if (OMPI_SUCCESS != rc) {
            r->super.req_status.MPI_ERROR = rc;
            ompi_request_complete(&r->super, true);
            return rc;
        }
        rocm_link_active(r);
    }
    return OMPI_SUCCESS;
}

/* MPI_Request_free: an active request's device work is waited for first —
 * peers may still read this rank's buffers through it. */
static int rocm_request_free(ompi_request_t **rptr)
{
    mca_coll_rocm_request_t *r = (mca_coll_rocm_request_t *) *rptr;
    int rc = OMPI_AMD_SUCCESS;
    /* always: the oldest active request is the list's tail (next_active
     * NULL) and must leave the list too (a no-op when it is not on it) */
    rocm_unlink_active(r);
    if (NULL != r->plan) {
        rc = ompi_amd_plan_wait(r->plan);
        (void) ompi_amd_plan_free(r->plan);
        r->plan = NULL;
    }
    if (NULL != r->nbreq) {
        rc = ompi_amd_request_free(r->nbreq);  /* waits for the device work */
        r->nbreq = NULL;
    }
    rc = to_ompi_err(rc);
    if (NULL != r->inner) {  /* the host copies must outlive the saved call */
        while (OMPI_REQUEST_ACTIVE == r->inner->req_state && !REQUEST_COMPLETE(r->inner)) {
            opal_progress();
        }
        if (OMPI_SUCCESS == rc) rc = ompi_request_free(&r->inner);
        else (void) ompi_request_free(&r->inner);
        r->inner = NULL;
    }
    nb_stage_free(r->stage);  /* freed before completion: outputs are undefined */
    r->stage = NULL;
    OMPI_REQUEST_FINI(&r->super);
    OBJ_RELEASE(r);
    *rptr = MPI_REQUEST_NULL;
    return rc;
}

static void rocm_request_construct(mca_coll_rocm_request_t *r)
{
    r->super.req_type = OMPI_REQUEST_COLL;
    r->super.req_status._cancelled = 0;
    r->super.req_start = rocm_request_start;
    r->super.req_free = rocm_request_free;
    r->super.req_cancel = NULL;
    r->plan = NULL;
    r->nbreq = NULL;
    r->inner = NULL;
    r->stage = NULL;
    r->next_active = NULL;
}

OBJ_CLASS_INSTANCE(mca_coll_rocm_request_t, ompi_request_t, rocm_request_construct, NULL);

/* ------------------------------------------------------------ nonblocking */

/* a nonblocking request's own staging memory, exact size, freed with it */
static char *nb_buf(void *ctx, int slot, int on_dev, size_t bytes)
{
    struct rocm_nb_stage *st = (struct rocm_nb_stage *) ctx;
    void **p = on_dev ? &st->dev[slot] : &st->host[slot];
    if (NULL == *p) {
        if (!on_dev) {
            *p = malloc(bytes ? bytes : 1);
        } else if (OMPI_AMD_SUCCESS != ompi_amd_device_alloc(p, bytes ? bytes : 1)) {
            *p = NULL;
        }
    }
    return (char *) *p;
}

static void nb_stage_free(struct rocm_nb_stage *st)
{
    if (NULL == st) return;
    for (int k = 0; k < 2; ++k) {
        (void) ompi_amd_device_free(st->dev[k]);
        free(st->host[k]);
    }
    free(st);
}

/* does any of this rank's operands live in device memory? */
static int any_device(const rocm_operand_t *o, int n)
{
    for (int i = 0; i < n; ++i) {
        if (NULL != o[i].user && MPI_IN_PLACE != o[i].user && 0 != o[i].count &&
            ompi_amd_is_device_pointer(o[i].user)) {
            return 1;
        }
    }
    return 0;
}

/* The path of one nonblocking or persistent call.  What every rank computes
 * alike comes first (no rendezvous when it fails).  A module locked to
 * DEVICE (§3.2 of DESIGN.md: every rank locks at the same blocking call)
 * takes the device path with no vote at all; a rank whose operands are not
 * device-contiguous stages them into memory of the request — inputs now
 * (and at every persistent start), outputs back when the request completes
 * (rocm_progress) — and counts the mismatch for the next recheck vote.
 * Otherwise the per-call vote.  When the saved (libnbc) function runs
 * instead, this rank's device operands go to it as host copies owned by a
 * request that wraps the saved one (rocm_saved_post), the blocking calls'
 * coll/cuda pattern (coll_cuda_allreduce.c:42-72) stretched over the
 * request's life. */
static int rocm_nb_begin(mca_coll_rocm_module_t *m, int uniform_ok, int local_ok,
                         rocm_operand_t *o, int n, struct rocm_nb_stage **stage, int *path)
{
    struct rocm_nb_stage *st;
    int rc;
    *stage = NULL;
    for (int i = 0; i < n; ++i) {
        o[i].use = o[i].user;
        o[i].how = 0;
        o[i].hbuf = NULL;
    }
    *path = ROCM_SAVED;
    if (uniform_ok) {
        *path = ROCM_RES_DEVICE == m->mode || take_device_path(m, local_ok) ? ROCM_DEVICE
                                                                            : ROCM_SAVED;
    }
    if (ROCM_DEVICE == *path) {
        if (local_ok) return OMPI_SUCCESS;
        m->mismatched++;  /* locked to DEVICE: this rank's operands go to the device */
    } else if (!any_device(o, n)) {
        return OMPI_SUCCESS;  /* the saved function takes host operands as they are */
    }
    st = calloc(1, sizeof(*st));
    if (NULL == st) return rocm_staging_failed(m, *path, OMPI_ERR_OUT_OF_RESOURCE);
    rc = rocm_stage_with(nb_buf, st, o, n, ROCM_DEVICE == *path);
    if (OMPI_SUCCESS != rc) {
        nb_stage_free(st);
        return rocm_staging_failed(m, *path, rc);
    }
    memcpy(st->o, o, (size_t) n * sizeof(*o));
    st->n = n;
    *stage = st;
    return OMPI_SUCCESS;
}

/* a library request (and the call's staged operands) behind an MPI
 * request, completed by rocm_progress */
static int rocm_wrap_nb(ompi_amd_request_t *nb, struct rocm_nb_stage *stage,
                        struct ompi_communicator_t *comm, ompi_request_t **request)
{
    mca_coll_rocm_request_t *r = OBJ_NEW(mca_coll_rocm_request_t);
    if (NULL == r) {
        (void) ompi_amd_request_free(nb);
        nb_stage_free(stage);
        return OMPI_ERROR;
    }
    OMPI_REQUEST_INIT(&r->super, false);
    r->super.req_state = OMPI_REQUEST_ACTIVE;
    r->super.req_mpi_object.comm = comm;
    r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
    r->nbreq = nb;
    r->stage = stage;
    rocm_link_active(r);
    *request = &r->super;
    return OMPI_SUCCESS;
}

/* the library's answer to a nonblocking post: a request, or the error (the
 * staged operands go with it) */
static int rocm_nb_post(int rc, ompi_amd_request_t *nb, struct rocm_nb_stage *stage,
                        struct ompi_communicator_t *comm, ompi_request_t **request)
{
    if (OMPI_AMD_SUCCESS != rc) {
        if (NULL != nb) (void) ompi_amd_request_free(nb);
        nb_stage_free(stage);
        return to_ompi_err(rc);
    }
    return rocm_wrap_nb(nb, stage, comm, request);
}

/* The saved function's answer: with nothing staged its request is the
 * caller's; otherwise a request of ours wraps it, completes when it does
 * (rocm_progress copies the staged outputs back first) and, persistent,
 * refills the staged inputs before every start of it. */
static int rocm_saved_post(int rc, ompi_request_t *inner, struct rocm_nb_stage *stage,
                           struct ompi_communicator_t *comm, ompi_request_t **request)
{
    mca_coll_rocm_request_t *r = NULL;
    if (NULL == stage) {
        *request = inner;
        return rc;
    }
    if (OMPI_SUCCESS == rc) r = OBJ_NEW(mca_coll_rocm_request_t);
    if (NULL == r) {
        if (OMPI_SUCCESS == rc && NULL != inner) (void) ompi_request_free(&inner);
        nb_stage_free(stage);
        return OMPI_SUCCESS != rc ? rc : OMPI_ERROR;
    }
    OMPI_REQUEST_INIT(&r->super, inner->req_persistent);
    r->super.req_mpi_object.comm = comm;
    r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
    r->inner = inner;
    r->stage = stage;
    *request = &r->super;
    if (!inner->req_persistent) {
        r->super.req_state = OMPI_REQUEST_ACTIVE;
        rocm_link_active(r);
    }
    return OMPI_SUCCESS;
}

/* MPI_Iallreduce (coll.h:271-274) */
int mca_coll_rocm_iallreduce(const void *sbuf, void *rbuf, int count,
                             struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                             struct ompi_communicator_t *comm, ompi_request_t **request,
                             mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int inplace = MPI_IN_PLACE == sbuf;
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {rbuf, (size_t) count, dtype, inplace, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_request_t *nb = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, (size_t) count), dev(sbuf) && dev(rbuf), o, 2,
                       &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_iallreduce(o[0].use, o[1].use, count, dtype, op, comm, &inner,
                                       m->c_coll.coll_iallreduce_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_iallreduce(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use,
                             (size_t) count, type_code(dtype), op->o_f_to_c_index, NULL, &nb);
    return rocm_nb_post(rc, nb, st, comm, request);
}

/* MPI_Ireduce_scatter_block / MPI_Iallgather / MPI_Ibcast (coll.h:261-265,
 * 293-296, 319-322): as MPI_Iallreduce. */
int mca_coll_rocm_ireduce_scatter_block(const void *sbuf, void *rbuf, int rcount,
                                        struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                        struct ompi_communicator_t *comm, ompi_request_t **request,
                                        mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const size_t all = (size_t) rcount * (size_t) ompi_comm_size(comm);
    const int inplace = MPI_IN_PLACE == sbuf;
    rocm_operand_t o[2] = {{(void *) sbuf, all, dtype, 1, 0},
                           {rbuf, inplace ? all : (size_t) rcount, dtype, inplace, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_request_t *nb = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, all), dev(sbuf) && dev(rbuf), o, 2, &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_ireduce_scatter_block(o[0].use, o[1].use, rcount, dtype, op, comm, &inner,
                                                  m->c_coll.coll_ireduce_scatter_block_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_ireduce_scatter_block(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use,
                                        (size_t) rcount, type_code(dtype), op->o_f_to_c_index, NULL,
                                        &nb);
    return rocm_nb_post(rc, nb, st, comm, request);
}

int mca_coll_rocm_iallgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                             void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                             struct ompi_communicator_t *comm, ompi_request_t **request,
                             mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int inplace = MPI_IN_PLACE == sbuf;
    const size_t all = (size_t) rcount * (size_t) ompi_comm_size(comm);
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) scount, sdtype, 1, 0},
                           {rbuf, all, rdtype, inplace, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_request_t *nb = NULL;
    ompi_request_t *inner = NULL;
    size_t rsize = 0;
    int path, rc, ok;
    (void) ompi_datatype_type_size(rdtype, &rsize);
    ok = ompi_datatype_is_contiguous_memory_layout(rdtype, (int) all) && dev(rbuf) && dev(sbuf) &&
         (inplace || ompi_datatype_is_contiguous_memory_layout(sdtype, scount));
    rc = rocm_nb_begin(m, bytes_ok(rsize * (size_t) rcount), ok, o, 2, &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_iallgather(o[0].use, scount, sdtype, o[1].use, rcount, rdtype, comm, &inner,
                                       m->c_coll.coll_iallgather_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_iallgather(m->dev_comm, inplace ? (const void *) 1 : o[0].use, o[1].use,
                             rsize * (size_t) rcount, NULL, &nb);
    return rocm_nb_post(rc, nb, st, comm, request);
}

int mca_coll_rocm_ibcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                         struct ompi_communicator_t *comm, ompi_request_t **request,
                         mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int is_root = ompi_comm_rank(comm) == root;
    rocm_operand_t o[1] = {{buf, (size_t) count, dtype, is_root, !is_root}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_request_t *nb = NULL;
    ompi_request_t *inner = NULL;
    size_t size = 0;
    int path, rc;
    (void) ompi_datatype_type_size(dtype, &size);
    rc = rocm_nb_begin(m, bytes_ok(size * (size_t) count),
                       ompi_datatype_is_contiguous_memory_layout(dtype, count) && dev(buf), o, 1, &st,
                       &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_ibcast(o[0].use, count, dtype, root, comm, &inner,
                                   m->c_coll.coll_ibcast_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_ibcast(m->dev_comm, o[0].use, size * (size_t) count, root, NULL, &nb);
    return rocm_nb_post(rc, nb, st, comm, request);
}

static int rocm_wrap_plan(int rc, ompi_amd_plan_t *plan, struct rocm_nb_stage *stage,
                          struct ompi_communicator_t *comm, ompi_request_t **request);

/* MPI_Allreduce_init (coll.h:349-352).  Collective: the path decision is
 * rocm_nb_begin's (no vote under the DEVICE lock; a rank with host operands
 * gets staging memory owned by the request, refilled at every start and
 * copied back at every completion), and on the device path the plan's
 * init swaps the buffer handles (it synchronises the ranks once). */
int mca_coll_rocm_allreduce_init(const void *sbuf, void *rbuf, int count,
                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                 struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                 ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int inplace = MPI_IN_PLACE == sbuf;
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {rbuf, (size_t) count, dtype, inplace, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_plan_t *plan = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, (size_t) count), dev(sbuf) && dev(rbuf), o, 2,
                       &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_allreduce_init(o[0].use, o[1].use, count, dtype, op, comm, info, &inner,
                                           m->c_coll.coll_allreduce_init_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_allreduce_init(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use,
                                 (size_t) count, type_code(dtype), op->o_f_to_c_index, &plan);
    return rocm_wrap_plan(rc, plan, st, comm, request);
}

/* MPI_Ireduce / MPI_Iscan / MPI_Iexscan / MPI_Ireduce_scatter (coll.h:
 * 297-326): rocm_nb_begin, then the library posts the call (no handle
 * swap; ompi_amd_ireduce posts the root's in-place choice); otherwise the
 * saved (libnbc) functions.  MPI_Ireduce's rbuf matters at the root only. */
int mca_coll_rocm_ireduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                          ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int is_root = ompi_comm_rank(comm) == root;
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {is_root ? rbuf : NULL, (size_t) count, dtype, MPI_IN_PLACE == sbuf, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_request_t *nb = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, (size_t) count),
                       is_root ? dev(rbuf) && dev(sbuf) : ompi_amd_is_device_pointer(sbuf), o, 2,
                       &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_ireduce(o[0].use, is_root ? o[1].use : rbuf, count, dtype, op, root, comm,
                                    &inner, m->c_coll.coll_ireduce_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_ireduce(m->dev_comm, o[0].use, is_root ? o[1].use : NULL, (size_t) count,
                          type_code(dtype), op->o_f_to_c_index, root, NULL, &nb);
    return rocm_nb_post(rc, nb, st, comm, request);
}

static int rocm_iscan_common(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                             struct ompi_op_t *op, struct ompi_communicator_t *comm,
                             ompi_request_t **request, mca_coll_rocm_module_t *m, int exclusive)
{
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {rbuf, (size_t) count, dtype, MPI_IN_PLACE == sbuf, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_request_t *nb = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, (size_t) count), dev(sbuf) && dev(rbuf), o, 2,
                       &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = exclusive ? m->c_coll.coll_iexscan(o[0].use, o[1].use, count, dtype, op, comm, &inner,
                                                m->c_coll.coll_iexscan_module)
                       : m->c_coll.coll_iscan(o[0].use, o[1].use, count, dtype, op, comm, &inner,
                                              m->c_coll.coll_iscan_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = (exclusive ? ompi_amd_iexscan : ompi_amd_iscan)(m->dev_comm, o[0].use, o[1].use,
                                                         (size_t) count, type_code(dtype),
                                                         op->o_f_to_c_index, NULL, &nb);
    return rocm_nb_post(rc, nb, st, comm, request);
}

int mca_coll_rocm_iscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                        struct ompi_op_t *op, struct ompi_communicator_t *comm,
                        ompi_request_t **request, mca_coll_base_module_t *module)
{
    return rocm_iscan_common(sbuf, rbuf, count, dtype, op, comm, request,
                             (mca_coll_rocm_module_t *) module, 0);
}

int mca_coll_rocm_iexscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, struct ompi_communicator_t *comm,
                          ompi_request_t **request, mca_coll_base_module_t *module)
{
    return rocm_iscan_common(sbuf, rbuf, count, dtype, op, comm, request,
                             (mca_coll_rocm_module_t *) module, 1);
}

int mca_coll_rocm_ireduce_scatter(const void *sbuf, void *rbuf, const int *rcounts,
                                  struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                  struct ompi_communicator_t *comm, ompi_request_t **request,
                                  mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int n = ompi_comm_size(comm), inplace = MPI_IN_PLACE == sbuf;
    size_t counts[OMPI_AMD_MAX_RANKS], total = 0;
    struct rocm_nb_stage *st = NULL;
    ompi_amd_request_t *nb = NULL;
    ompi_request_t *inner = NULL;
    int path, rc, i;
    for (i = 0; i < n; ++i) total += (size_t) rcounts[i];
    {
        rocm_operand_t o[2] = {{(void *) sbuf, total, dtype, 1, 0},
                               {rbuf, inplace ? total : (size_t) rcounts[ompi_comm_rank(comm)],
                                dtype, inplace, 1}};
        rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, total), dev(sbuf) && dev(rbuf), o, 2, &st,
                           &path);
        if (OMPI_SUCCESS != rc) return rc;
        if (ROCM_DEVICE != path) {
            rc = m->c_coll.coll_ireduce_scatter(o[0].use, o[1].use, rcounts, dtype, op, comm, &inner,
                                                m->c_coll.coll_ireduce_scatter_module);
            return rocm_saved_post(rc, inner, st, comm, request);
        }
        for (i = 0; i < n; ++i) counts[i] = (size_t) rcounts[i];
        rc = ompi_amd_ireduce_scatter(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use, counts,
                                      type_code(dtype), op->o_f_to_c_index, NULL, &nb);
        return rocm_nb_post(rc, nb, st, comm, request);
    }
}

/* MPI_Reduce_scatter_block_init / MPI_Allgather_init / MPI_Bcast_init
 * (coll.h:339-400): the same decision as MPI_Allreduce_init; on the device
 * path a library plan behind a persistent request (its start posts the
 * nonblocking call, completion through the progress callback), otherwise
 * the saved (libnbc) functions build the request. */
static int rocm_wrap_plan(int rc, ompi_amd_plan_t *plan, struct rocm_nb_stage *stage,
                          struct ompi_communicator_t *comm, ompi_request_t **request)
{
    mca_coll_rocm_request_t *r = NULL;
    if (OMPI_AMD_SUCCESS == rc) r = OBJ_NEW(mca_coll_rocm_request_t);
    if (NULL == r) {
        if (NULL != plan) (void) ompi_amd_plan_free(plan);
        nb_stage_free(stage);
        return OMPI_AMD_SUCCESS != rc ? to_ompi_err(rc) : OMPI_ERROR;
    }
    OMPI_REQUEST_INIT(&r->super, true);
    r->super.req_mpi_object.comm = comm;
    r->plan = plan;
    r->stage = stage;
    *request = &r->super;
    return OMPI_SUCCESS;
}

int mca_coll_rocm_reduce_scatter_block_init(const void *sbuf, void *rbuf, int rcount,
                                            struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                            struct ompi_communicator_t *comm,
                                            struct ompi_info_t *info, ompi_request_t **request,
                                            mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const size_t all = (size_t) rcount * (size_t) ompi_comm_size(comm);
    const int inplace = MPI_IN_PLACE == sbuf;
    rocm_operand_t o[2] = {{(void *) sbuf, all, dtype, 1, 0},
                           {rbuf, inplace ? all : (size_t) rcount, dtype, inplace, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_plan_t *plan = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, all), dev(sbuf) && dev(rbuf), o, 2, &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_reduce_scatter_block_init(o[0].use, o[1].use, rcount, dtype, op, comm, info,
                                                      &inner,
                                                      m->c_coll.coll_reduce_scatter_block_init_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_reduce_scatter_block_init(m->dev_comm, inplace ? MPI_IN_PLACE : o[0].use,
                                            o[1].use, (size_t) rcount, type_code(dtype),
                                            op->o_f_to_c_index, &plan);
    return rocm_wrap_plan(rc, plan, st, comm, request);
}

int mca_coll_rocm_allgather_init(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                                 void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                                 struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                 ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int inplace = MPI_IN_PLACE == sbuf;
    const size_t all = (size_t) rcount * (size_t) ompi_comm_size(comm);
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) scount, sdtype, 1, 0},
                           {rbuf, all, rdtype, inplace, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_plan_t *plan = NULL;
    ompi_request_t *inner = NULL;
    size_t rsize = 0;
    int path, rc, ok;
    (void) ompi_datatype_type_size(rdtype, &rsize);
    ok = ompi_datatype_is_contiguous_memory_layout(rdtype, (int) all) && dev(rbuf) && dev(sbuf) &&
         (inplace || ompi_datatype_is_contiguous_memory_layout(sdtype, scount));
    rc = rocm_nb_begin(m, bytes_ok(rsize * (size_t) rcount), ok, o, 2, &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_allgather_init(o[0].use, scount, sdtype, o[1].use, rcount, rdtype, comm,
                                           info, &inner, m->c_coll.coll_allgather_init_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_allgather_init(m->dev_comm, inplace ? (const void *) 1 : o[0].use, o[1].use,
                                 rsize * (size_t) rcount, &plan);
    return rocm_wrap_plan(rc, plan, st, comm, request);
}

int mca_coll_rocm_bcast_init(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                             struct ompi_communicator_t *comm, struct ompi_info_t *info,
                             ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int is_root = ompi_comm_rank(comm) == root;
    rocm_operand_t o[1] = {{buf, (size_t) count, dtype, is_root, !is_root}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_plan_t *plan = NULL;
    ompi_request_t *inner = NULL;
    size_t size = 0;
    int path, rc;
    (void) ompi_datatype_type_size(dtype, &size);
    rc = rocm_nb_begin(m, bytes_ok(size * (size_t) count),
                       ompi_datatype_is_contiguous_memory_layout(dtype, count) && dev(buf), o, 1, &st,
                       &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_bcast_init(o[0].use, count, dtype, root, comm, info, &inner,
                                       m->c_coll.coll_bcast_init_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_bcast_init(m->dev_comm, o[0].use, size * (size_t) count, root, &plan);
    return rocm_wrap_plan(rc, plan, st, comm, request);
}

/* MPI_Reduce_init / MPI_Reduce_scatter_init / MPI_Scan_init / MPI_Exscan_init
 * (coll.h:555-567 coll_reduce_init, coll_reduce_scatter_init,
 * coll_scan_init, coll_exscan_init; libnbc's in the reference): the same
 * decision as MPI_Allreduce_init; on the device path a library plan whose
 * every start posts the nonblocking call with the init's arguments.
 * MPI_Reduce_init's rbuf matters at the root only. */
int mca_coll_rocm_reduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                              struct ompi_info_t *info, ompi_request_t **request,
                              mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int is_root = ompi_comm_rank(comm) == root;
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {is_root ? rbuf : NULL, (size_t) count, dtype, MPI_IN_PLACE == sbuf, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_plan_t *plan = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, (size_t) count),
                       is_root ? dev(rbuf) && dev(sbuf) : ompi_amd_is_device_pointer(sbuf), o, 2,
                       &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = m->c_coll.coll_reduce_init(o[0].use, is_root ? o[1].use : rbuf, count, dtype, op, root,
                                        comm, info, &inner, m->c_coll.coll_reduce_init_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = ompi_amd_reduce_init(m->dev_comm, o[0].use, is_root ? o[1].use : NULL, (size_t) count,
                              type_code(dtype), op->o_f_to_c_index, root, &plan);
    return rocm_wrap_plan(rc, plan, st, comm, request);
}

int mca_coll_rocm_reduce_scatter_init(const void *sbuf, void *rbuf, const int *rcounts,
                                      struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                      struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                      ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int n = ompi_comm_size(comm), inplace = MPI_IN_PLACE == sbuf;
    size_t counts[OMPI_AMD_MAX_RANKS], total = 0;
    struct rocm_nb_stage *st = NULL;
    ompi_amd_plan_t *plan = NULL;
    ompi_request_t *inner = NULL;
    int path, rc, i;
    for (i = 0; i < n; ++i) total += (size_t) rcounts[i];
    {
        rocm_operand_t o[2] = {{(void *) sbuf, total, dtype, 1, 0},
                               {rbuf, inplace ? total : (size_t) rcounts[ompi_comm_rank(comm)],
                                dtype, inplace, 1}};
        rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, total), dev(sbuf) && dev(rbuf), o, 2, &st,
                           &path);
        if (OMPI_SUCCESS != rc) return rc;
        if (ROCM_DEVICE != path) {
            rc = m->c_coll.coll_reduce_scatter_init(o[0].use, o[1].use, rcounts, dtype, op, comm, info,
                                                    &inner, m->c_coll.coll_reduce_scatter_init_module);
            return rocm_saved_post(rc, inner, st, comm, request);
        }
        for (i = 0; i < n; ++i) counts[i] = (size_t) rcounts[i];
        rc = ompi_amd_reduce_scatter_init(m->dev_comm, inplace ? o[1].use : o[0].use, o[1].use,
                                          counts, type_code(dtype), op->o_f_to_c_index, &plan);
        return rocm_wrap_plan(rc, plan, st, comm, request);
    }
}

static int rocm_scan_init_common(const void *sbuf, void *rbuf, int count,
                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                 struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                 ompi_request_t **request, mca_coll_rocm_module_t *m, int exclusive)
{
    rocm_operand_t o[2] = {{(void *) sbuf, (size_t) count, dtype, 1, 0},
                           {rbuf, (size_t) count, dtype, MPI_IN_PLACE == sbuf, 1}};
    struct rocm_nb_stage *st = NULL;
    ompi_amd_plan_t *plan = NULL;
    ompi_request_t *inner = NULL;
    int path, rc;
    rc = rocm_nb_begin(m, reduction_ok_n(dtype, op, (size_t) count), dev(sbuf) && dev(rbuf), o, 2,
                       &st, &path);
    if (OMPI_SUCCESS != rc) return rc;
    if (ROCM_DEVICE != path) {
        rc = exclusive ? m->c_coll.coll_exscan_init(o[0].use, o[1].use, count, dtype, op, comm, info,
                                                    &inner, m->c_coll.coll_exscan_init_module)
                       : m->c_coll.coll_scan_init(o[0].use, o[1].use, count, dtype, op, comm, info,
                                                  &inner, m->c_coll.coll_scan_init_module);
        return rocm_saved_post(rc, inner, st, comm, request);
    }
    rc = (exclusive ? ompi_amd_exscan_init : ompi_amd_scan_init)(m->dev_comm, o[0].use, o[1].use,
                                                                 (size_t) count, type_code(dtype),
                                                                 op->o_f_to_c_index, &plan);
    return rocm_wrap_plan(rc, plan, st, comm, request);
}

int mca_coll_rocm_scan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                            struct ompi_op_t *op, struct ompi_communicator_t *comm,
                            struct ompi_info_t *info, ompi_request_t **request,
                            mca_coll_base_module_t *module)
{
    return rocm_scan_init_common(sbuf, rbuf, count, dtype, op, comm, info, request,
                                 (mca_coll_rocm_module_t *) module, 0);
}

int mca_coll_rocm_exscan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, struct ompi_communicator_t *comm,
                              struct ompi_info_t *info, ompi_request_t **request,
                              mca_coll_base_module_t *module)
{
    return rocm_scan_init_common(sbuf, rbuf, count, dtype, op, comm, info, request,
                                 (mca_coll_rocm_module_t *) module, 1);
}
