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
    .algorithm = 0,
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
                                           "Read peers' user buffers directly for large messages",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.zero_copy);
    (void) mca_base_component_var_register(c, "timeout_ms",
                                           "Device barrier spin limit before the collective fails",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.timeout_ms);
    (void) mca_base_component_var_register(c, "allreduce_algorithm",
                                           "Large-message allreduce data movement: 0 pull, 1 pull+push, 2 push",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_coll_rocm_component.algorithm);
    return OMPI_SUCCESS;
}

/* ------------------------------------------------------------- module */

static void rocm_module_construct(mca_coll_rocm_module_t *m)
{
    memset(&m->c_coll, 0, sizeof(m->c_coll));
    m->dev_comm = NULL;
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
    if (NULL != m->dev_comm) (void) ompi_amd_comm_destroy(m->dev_comm);
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
    m->super.coll_allreduce_init = mca_coll_rocm_allreduce_init;
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
    SAVE(allreduce_init);
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

/* every rank must answer the same way (buffer residency may differ) */
static bool take_device_path(mca_coll_rocm_module_t *m, int local_ok)
{
    int all_ok = 0;
    if (OMPI_AMD_SUCCESS != ompi_amd_comm_agree(m->dev_comm, local_ok, &all_ok)) return false;
    return all_ok != 0;
}

/* ------------------------------------------------------------- collectives */

int mca_coll_rocm_allreduce(const void *sbuf, void *rbuf, int count,
                            struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                            struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int t = type_code(dtype);
    const int ok = t >= 0 && ompi_op_is_intrinsic(op) &&
                   ompi_amd_op_supported(op->o_f_to_c_index, t) && dev(sbuf) && dev(rbuf);
    int rc;
    if (!take_device_path(m, ok)) {
        return m->c_coll.coll_allreduce(sbuf, rbuf, count, dtype, op, comm,
                                        m->c_coll.coll_allreduce_module);
    }
    rc = ompi_amd_allreduce(m->dev_comm, MPI_IN_PLACE == sbuf ? rbuf : sbuf, rbuf,
                            (size_t) count, t, op->o_f_to_c_index, NULL);
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return to_ompi_err(rc);
}

/* MPI_Reduce: rbuf is significant at the root only (MPI-3.1 §5.9.1), so
 * only the root's rbuf residency enters the local decision. */
int mca_coll_rocm_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                         struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                         mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int t = type_code(dtype);
    const int is_root = ompi_comm_rank(comm) == root;
    const int ok = t >= 0 && ompi_op_is_intrinsic(op) &&
                   ompi_amd_op_supported(op->o_f_to_c_index, t) &&
                   (is_root ? dev(rbuf) && dev(sbuf) : ompi_amd_is_device_pointer(sbuf));
    int rc;
    if (!take_device_path(m, ok)) {
        return m->c_coll.coll_reduce(sbuf, rbuf, count, dtype, op, root, comm,
                                     m->c_coll.coll_reduce_module);
    }
    rc = ompi_amd_reduce(m->dev_comm, sbuf, is_root ? rbuf : NULL, (size_t) count, t,
                         op->o_f_to_c_index, root, NULL);
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return to_ompi_err(rc);
}

static int rocm_scan_common(const void *sbuf, void *rbuf, int count,
                            struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                            struct ompi_communicator_t *comm, mca_coll_rocm_module_t *m,
                            int exclusive)
{
    const int t = type_code(dtype);
    const int ok = t >= 0 && ompi_op_is_intrinsic(op) &&
                   ompi_amd_op_supported(op->o_f_to_c_index, t) && dev(sbuf) && dev(rbuf);
    int rc;
    if (!take_device_path(m, ok)) {
        return exclusive ? m->c_coll.coll_exscan(sbuf, rbuf, count, dtype, op, comm,
                                                 m->c_coll.coll_exscan_module)
                         : m->c_coll.coll_scan(sbuf, rbuf, count, dtype, op, comm,
                                               m->c_coll.coll_scan_module);
    }
    rc = (exclusive ? ompi_amd_exscan : ompi_amd_scan)(m->dev_comm, sbuf, rbuf, (size_t) count, t,
                                                       op->o_f_to_c_index, NULL);
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return to_ompi_err(rc);
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
    const int t = type_code(dtype);
    const int n = ompi_comm_size(comm);
    const int ok = t >= 0 && ompi_op_is_intrinsic(op) &&
                   ompi_amd_op_supported(op->o_f_to_c_index, t) && dev(sbuf) && dev(rbuf);
    size_t counts[OMPI_AMD_MAX_RANKS];
    int rc, i;
    if (!take_device_path(m, ok)) {
        return m->c_coll.coll_reduce_scatter(sbuf, rbuf, rcounts, dtype, op, comm,
                                             m->c_coll.coll_reduce_scatter_module);
    }
    for (i = 0; i < n; ++i) counts[i] = (size_t) rcounts[i];
    rc = ompi_amd_reduce_scatter(m->dev_comm, MPI_IN_PLACE == sbuf ? rbuf : sbuf, rbuf, counts, t,
                                 op->o_f_to_c_index, NULL);
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return to_ompi_err(rc);
}

int mca_coll_rocm_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount,
                                       struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                       struct ompi_communicator_t *comm,
                                       mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int t = type_code(dtype);
    const int ok = t >= 0 && ompi_op_is_intrinsic(op) &&
                   ompi_amd_op_supported(op->o_f_to_c_index, t) && dev(sbuf) && dev(rbuf);
    int rc;
    if (!take_device_path(m, ok)) {
        return m->c_coll.coll_reduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm,
                                                   m->c_coll.coll_reduce_scatter_block_module);
    }
    rc = ompi_amd_reduce_scatter_block(m->dev_comm, MPI_IN_PLACE == sbuf ? rbuf : sbuf, rbuf,
                                       (size_t) rcount, t, op->o_f_to_c_index, NULL);
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return to_ompi_err(rc);
}

int mca_coll_rocm_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                            void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                            struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    size_t rsize = 0;
    int rc, ok;
    (void) ompi_datatype_type_size(rdtype, &rsize);
    /* contiguous, gap-free receive type: the gather is a byte copy */
    ok = ompi_datatype_is_contiguous_memory_layout(rdtype, rcount) && dev(rbuf) && dev(sbuf) &&
         (MPI_IN_PLACE == sbuf || ompi_datatype_is_contiguous_memory_layout(sdtype, scount));
    if (!take_device_path(m, ok)) {
        return m->c_coll.coll_allgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm,
                                        m->c_coll.coll_allgather_module);
    }
    rc = ompi_amd_allgather(m->dev_comm, MPI_IN_PLACE == sbuf ? (const void *) 1 : sbuf, rbuf,
                            rsize * (size_t) rcount, NULL);
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return to_ompi_err(rc);
}

int mca_coll_rocm_bcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                        struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    size_t size = 0;
    int rc;
    (void) ompi_datatype_type_size(dtype, &size);
    if (!take_device_path(m, ompi_datatype_is_contiguous_memory_layout(dtype, count) && dev(buf))) {
        return m->c_coll.coll_bcast(buf, count, dtype, root, comm, m->c_coll.coll_bcast_module);
    }
    rc = ompi_amd_bcast(m->dev_comm, buf, size * (size_t) count, root, NULL);
    if (OMPI_AMD_SUCCESS == rc) rc = ompi_amd_comm_sync(m->dev_comm, NULL);
    return to_ompi_err(rc);
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
        int fin = 0;
        const int rc = NULL != r->plan ? ompi_amd_plan_test(r->plan, &fin)
                                       : ompi_amd_request_test(r->nbreq, &fin);
        if (OMPI_AMD_SUCCESS != rc || fin) {
            r->super.req_status.MPI_ERROR = to_ompi_err(rc);
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
        rc = ompi_amd_plan_start(r->plan, NULL);
        if (OMPI_AMD_SUCCESS != rc) {
            r->super.req_status.MPI_ERROR = to_ompi_err(rc);
            ompi_request_complete(&r->super, true);
            return to_ompi_err(rc);
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
    if (NULL != r->next_active) rocm_unlink_active(r);
    if (NULL != r->plan) {
        rc = ompi_amd_plan_wait(r->plan);
        (void) ompi_amd_plan_free(r->plan);
        r->plan = NULL;
    }
    if (NULL != r->nbreq) {
        rc = ompi_amd_request_free(r->nbreq);
        r->nbreq = NULL;
    }
    OMPI_REQUEST_FINI(&r->super);
    OBJ_RELEASE(r);
    *rptr = MPI_REQUEST_NULL;
    return to_ompi_err(rc);
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
    r->next_active = NULL;
}

OBJ_CLASS_INSTANCE(mca_coll_rocm_request_t, ompi_request_t, rocm_request_construct, NULL);

/* MPI_Iallreduce (coll.h:271-274).  The path agreement is the one host
 * rendezvous that precedes the call's own (nonblocking) post: every rank
 * reaches it at the same collective, as for the blocking allreduce. */
int mca_coll_rocm_iallreduce(const void *sbuf, void *rbuf, int count,
                             struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                             struct ompi_communicator_t *comm, ompi_request_t **request,
                             mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int t = type_code(dtype);
    const int ok = t >= 0 && ompi_op_is_intrinsic(op) &&
                   ompi_amd_op_supported(op->o_f_to_c_index, t) && dev(sbuf) && dev(rbuf);
    mca_coll_rocm_request_t *r;
    ompi_amd_request_t *nb = NULL;
    int rc;
    if (!take_device_path(m, ok)) {
        return m->c_coll.coll_iallreduce(sbuf, rbuf, count, dtype, op, comm, request,
                                         m->c_coll.coll_iallreduce_module);
    }
    r = OBJ_NEW(mca_coll_rocm_request_t);
    if (NULL == r) return OMPI_ERROR;
    rc = ompi_amd_iallreduce(m->dev_comm, MPI_IN_PLACE == sbuf ? rbuf : sbuf, rbuf,
                             (size_t) count, t, op->o_f_to_c_index, NULL, &nb);
    if (OMPI_AMD_SUCCESS != rc) {
        if (NULL != nb) (void) ompi_amd_request_free(nb);
        OBJ_RELEASE(r);
        return to_ompi_err(rc);
    }
    OMPI_REQUEST_INIT(&r->super, false);
    r->super.req_state = OMPI_REQUEST_ACTIVE;
    r->super.req_mpi_object.comm = comm;
    r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
    r->nbreq = nb;
    rocm_link_active(r);
    *request = &r->super;
    return OMPI_SUCCESS;
}

/* MPI_Allreduce_init (coll.h:349-352).  Collective: the path decision is
 * agreed like the blocking allreduce's, and on the device path the plan's
 * init swaps the buffer handles (it synchronises the ranks once). */
int mca_coll_rocm_allreduce_init(const void *sbuf, void *rbuf, int count,
                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                 struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                 ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_rocm_module_t *m = (mca_coll_rocm_module_t *) module;
    const int t = type_code(dtype);
    const int ok = t >= 0 && ompi_op_is_intrinsic(op) &&
                   ompi_amd_op_supported(op->o_f_to_c_index, t) && dev(sbuf) && dev(rbuf);
    mca_coll_rocm_request_t *r;
    ompi_amd_plan_t *plan = NULL;
    int rc;
    if (!take_device_path(m, ok)) {
        return m->c_coll.coll_allreduce_init(sbuf, rbuf, count, dtype, op, comm, info, request,
                                             m->c_coll.coll_allreduce_init_module);
    }
    rc = ompi_amd_allreduce_init(m->dev_comm, MPI_IN_PLACE == sbuf ? rbuf : sbuf, rbuf,
                                 (size_t) count, t, op->o_f_to_c_index, &plan);
    if (OMPI_AMD_SUCCESS != rc) return to_ompi_err(rc);
    r = OBJ_NEW(mca_coll_rocm_request_t);
    if (NULL == r) {
        (void) ompi_amd_plan_free(plan);
        return OMPI_ERROR;
    }
    OMPI_REQUEST_INIT(&r->super, true);
    r->super.req_mpi_object.comm = comm;
    r->plan = plan;
    *request = &r->super;
    return OMPI_SUCCESS;
}
