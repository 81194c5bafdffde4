/*
 * osc/rocm component: device windows through libompi_amd.so.
 *
 * Mirrors osc/sm's module functions (ompi/mca/osc/sm/osc_sm_comm.c,
 * osc_sm_active_target.c, osc_sm_passive_target.c) one call each; the
 * data moves by kernels on the origin's GPU over the peers' IPC mappings
 * (include/ompi_amd_osc.h).  Predefined datatypes with equal origin and
 * target signatures; everything else returns OMPI_ERR_NOT_SUPPORTED, as
 * osc/sm rejects what it cannot do.  Blocking MPI semantics come from the
 * stream synchronisation in fence / unlock / flush (ompi_amd_comm_sync,
 * which also turns a peer that never released a lock into
 * OMPI_ERR_TIMEOUT).
 */
#include "ompi_config.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpi.h"
#include "ompi/constants.h"
#include "ompi/communicator/communicator.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/mca/osc/osc.h"
#include "ompi/op/op.h"
#include "ompi/runtime/ompi_rte.h"
#include "ompi/win/win.h"
#include "opal/mca/base/mca_base_var.h"
#include "opal/util/info.h"

#include "ompi_amd.h"
#include "osc_rocm.h"

static int rocm_register(void);
static int rocm_init(bool progress_threads, bool mpi_threads);
static int rocm_finalize(void);
static int rocm_query(struct ompi_win_t *win, void **base, size_t size, int disp_unit,
                      struct ompi_communicator_t *comm, struct opal_info_t *info, int flavor);
static int rocm_select(struct ompi_win_t *win, void **base, size_t size, int disp_unit,
                       struct ompi_communicator_t *comm, struct opal_info_t *info, int flavor,
                       int *model);

ompi_osc_rocm_component_t mca_osc_rocm_component = {
    .super = {
        .osc_version = {
            OMPI_OSC_BASE_VERSION_3_0_0,
            .mca_component_name = "rocm",
            MCA_BASE_MAKE_VERSION(component, OMPI_MAJOR_VERSION, OMPI_MINOR_VERSION,
                                  OMPI_RELEASE_VERSION),
            .mca_register_component_params = rocm_register,
        },
        .osc_data = { MCA_BASE_METADATA_PARAM_CHECKPOINT },
        .osc_init = rocm_init,
        .osc_query = rocm_query,
        .osc_select = rocm_select,
        .osc_finalize = rocm_finalize,
    },
    .priority = 101,
    .timeout_ms = 30000,
    .windows = 0,
};

static int rocm_register(void)
{
    const mca_base_component_t *c = &mca_osc_rocm_component.super.osc_version;
    (void) mca_base_component_var_register(c, "priority", "Priority of osc/rocm for device windows",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_9,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_osc_rocm_component.priority);
    (void) mca_base_component_var_register(c, "timeout_ms",
                                           "Bound on waiting for a peer's lock or fence (ms)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_9,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_osc_rocm_component.timeout_ms);
    return OMPI_SUCCESS;
}

static int rocm_init(bool progress_threads, bool mpi_threads)
{
    return ompi_amd_device_count() > 0 ? OMPI_SUCCESS : OMPI_ERR_NOT_AVAILABLE;
}

static int rocm_finalize(void) { return OMPI_SUCCESS; }

static int to_ompi_err(int rc)
{
    switch (rc) {
    case OMPI_AMD_SUCCESS: return OMPI_SUCCESS;
    case OMPI_AMD_ERR_UNSUPPORTED: return OMPI_ERR_NOT_SUPPORTED;
    case OMPI_AMD_ERR_BAD_PARAM: return OMPI_ERR_BAD_PARAM;
    case OMPI_AMD_ERR_TIMEOUT: return OMPI_ERR_TIMEOUT;
    default: return OMPI_ERROR;
    }
}

static ompi_osc_rocm_module_t *mod(struct ompi_win_t *win)
{
    return (ompi_osc_rocm_module_t *) win->w_osc_module;
}

/* op/base type code of a predefined datatype (ompi_op_ddt_map, op.c:102), or -1 */
static int type_code(struct ompi_datatype_t *dt)
{
    if (!ompi_datatype_is_predefined(dt)) return -1;
    return ompi_op_ddt_map[dt->id];
}

/* bytes of `count` elements of a contiguous predefined type, or 0 if unsupported */
static size_t span(struct ompi_datatype_t *dt, int count)
{
    size_t size = 0;
    const int t = type_code(dt);
    if (!ompi_datatype_is_predefined(dt) || !ompi_datatype_is_contiguous_memory_layout(dt, count))
        return 0;
    (void) ompi_datatype_type_size(dt, &size);
    if (t >= 0 && ompi_amd_type_extent(t) > 0) size = ompi_amd_type_extent(t);  /* pair types */
    return size * (size_t) count;
}

/* the MPI_Win_fence / unlock completion: device work done, sticky error checked */
static int complete(ompi_osc_rocm_module_t *m, int rc)
{
    if (OMPI_AMD_SUCCESS != rc) return to_ompi_err(rc);
    return to_ompi_err(ompi_amd_comm_sync(m->dev_comm, NULL));
}

/* ------------------------------------------------------------ communication */

static int rocm_put(const void *origin, int ocount, struct ompi_datatype_t *odt, int target,
                    ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt, struct ompi_win_t *win)
{
    const size_t bytes = span(odt, ocount);
    if (0 == ocount) return OMPI_SUCCESS;
    if (0 == bytes || bytes != span(tdt, tcount) || disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_put(mod(win)->dev_win, origin, bytes, target, (size_t) disp, NULL));
}

static int rocm_get(void *origin, int ocount, struct ompi_datatype_t *odt, int target,
                    ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt, struct ompi_win_t *win)
{
    const size_t bytes = span(odt, ocount);
    if (0 == ocount) return OMPI_SUCCESS;
    if (0 == bytes || bytes != span(tdt, tcount) || disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_get(mod(win)->dev_win, origin, bytes, target, (size_t) disp, NULL));
}

/* same predefined type on both sides, same count (osc_sm_comm.c:289-303 reduces
 * origin into target with ompi_op_reduce, which needs exactly this) */
static int acc_ok(struct ompi_datatype_t *odt, int ocount, struct ompi_datatype_t *tdt,
                  int tcount, struct ompi_op_t *op)
{
    const int t = type_code(tdt);
    if (t < 0 || odt->id != tdt->id || ocount != tcount || !ompi_op_is_intrinsic(op)) return 0;
    if (OMPI_AMD_OP_REPLACE == op->o_f_to_c_index || OMPI_AMD_OP_NO_OP == op->o_f_to_c_index)
        return 1;
    return ompi_amd_op_supported(op->o_f_to_c_index, t) == 1;
}

static int rocm_accumulate(const void *origin, int ocount, struct ompi_datatype_t *odt,
                           int target, ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                           struct ompi_op_t *op, struct ompi_win_t *win)
{
    if (0 == ocount) return OMPI_SUCCESS;
    if (!acc_ok(odt, ocount, tdt, tcount, op) || disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_accumulate(mod(win)->dev_win, origin, (size_t) ocount,
                                           type_code(tdt), target, (size_t) disp,
                                           op->o_f_to_c_index, NULL));
}

static int rocm_get_accumulate(const void *origin, int ocount, struct ompi_datatype_t *odt,
                               void *result, int rcount, struct ompi_datatype_t *rdt, int target,
                               ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                               struct ompi_op_t *op, struct ompi_win_t *win)
{
    const int no_op = ompi_op_is_intrinsic(op) && OMPI_AMD_OP_NO_OP == op->o_f_to_c_index;
    if (0 == tcount) return OMPI_SUCCESS;
    if (rdt->id != tdt->id || rcount != tcount || disp < 0 ||
        !acc_ok(no_op ? tdt : odt, no_op ? tcount : ocount, tdt, tcount, op))
        return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_get_accumulate(mod(win)->dev_win, no_op ? NULL : origin, result,
                                               (size_t) tcount, type_code(tdt), target,
                                               (size_t) disp, op->o_f_to_c_index, NULL));
}

static int rocm_fetch_and_op(const void *origin, void *result, struct ompi_datatype_t *dt,
                             int target, ptrdiff_t disp, struct ompi_op_t *op,
                             struct ompi_win_t *win)
{
    if (!acc_ok(dt, 1, dt, 1, op) || disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_fetch_and_op(mod(win)->dev_win, origin, result, type_code(dt),
                                             target, (size_t) disp, op->o_f_to_c_index, NULL));
}

static int rocm_compare_and_swap(const void *origin, const void *compare, void *result,
                                 struct ompi_datatype_t *dt, int target, ptrdiff_t disp,
                                 struct ompi_win_t *win)
{
    if (type_code(dt) < 0 || disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_compare_and_swap(mod(win)->dev_win, origin, compare, result,
                                                 type_code(dt), target, (size_t) disp, NULL));
}

/* ------------------------------------------------------------ synchronisation */

static int rocm_fence(int assert_, struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    return complete(m, ompi_amd_win_fence(m->dev_win, assert_, NULL));
}

static int rocm_lock(int lock_type, int target, int assert_, struct ompi_win_t *win)
{
    return to_ompi_err(ompi_amd_win_lock(mod(win)->dev_win, lock_type, target, assert_, NULL));
}

static int rocm_unlock(int target, struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    return complete(m, ompi_amd_win_unlock(m->dev_win, target, NULL));
}

static int rocm_lock_all(int assert_, struct ompi_win_t *win)
{
    return to_ompi_err(ompi_amd_win_lock_all(mod(win)->dev_win, assert_, NULL));
}

static int rocm_unlock_all(struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    return complete(m, ompi_amd_win_unlock_all(m->dev_win, NULL));
}

static int rocm_flush(int target, struct ompi_win_t *win)
{
    return to_ompi_err(ompi_amd_win_flush(mod(win)->dev_win, target, NULL));
}

static int rocm_flush_all(struct ompi_win_t *win) { return rocm_flush(0, win); }

static int rocm_sync(struct ompi_win_t *win) { return complete(mod(win), OMPI_AMD_SUCCESS); }

static int rocm_free(struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    int rc = ompi_amd_win_free(m->dev_win);
    const int crc = ompi_amd_comm_destroy(m->dev_comm);
    if (OMPI_AMD_SUCCESS == rc) rc = crc;
    win->w_osc_module = NULL;
    free(m);
    return to_ompi_err(rc);
}

/* PSCW, dynamic / shared windows and request-based RMA: not provided (the
 * framework reports MPI_ERR_UNSUPPORTED_OPERATION) */
static int ns_shared_query(struct ompi_win_t *w, int r, size_t *s, int *d, void *b)
{ return OMPI_ERR_NOT_SUPPORTED; }
static int ns_attach(struct ompi_win_t *w, void *b, size_t s) { return OMPI_ERR_NOT_SUPPORTED; }
static int ns_detach(struct ompi_win_t *w, const void *b) { return OMPI_ERR_NOT_SUPPORTED; }
static int ns_group(struct ompi_group_t *g, int a, struct ompi_win_t *w) { return OMPI_ERR_NOT_SUPPORTED; }
static int ns_win(struct ompi_win_t *w) { return OMPI_ERR_NOT_SUPPORTED; }
static int ns_test(struct ompi_win_t *w, int *f) { return OMPI_ERR_NOT_SUPPORTED; }
static int ns_rput(const void *o, int oc, struct ompi_datatype_t *od, int t, ptrdiff_t d, int tc,
                   struct ompi_datatype_t *td, struct ompi_win_t *w, ompi_request_t **r)
{ return OMPI_ERR_NOT_SUPPORTED; }
static int ns_rget(void *o, int oc, struct ompi_datatype_t *od, int t, ptrdiff_t d, int tc,
                   struct ompi_datatype_t *td, struct ompi_win_t *w, ompi_request_t **r)
{ return OMPI_ERR_NOT_SUPPORTED; }
static int ns_racc(const void *o, int oc, struct ompi_datatype_t *od, int t, ptrdiff_t d, int tc,
                   struct ompi_datatype_t *td, struct ompi_op_t *op, struct ompi_win_t *w,
                   ompi_request_t **r)
{ return OMPI_ERR_NOT_SUPPORTED; }
static int ns_rgacc(const void *o, int oc, struct ompi_datatype_t *od, void *res, int rc,
                    struct ompi_datatype_t *rd, int t, ptrdiff_t d, int tc,
                    struct ompi_datatype_t *td, struct ompi_op_t *op, struct ompi_win_t *w,
                    ompi_request_t **r)
{ return OMPI_ERR_NOT_SUPPORTED; }

static const ompi_osc_base_module_t rocm_module_template = {
    .osc_win_shared_query = ns_shared_query,
    .osc_win_attach = ns_attach,
    .osc_win_detach = ns_detach,
    .osc_free = rocm_free,
    .osc_put = rocm_put,
    .osc_get = rocm_get,
    .osc_accumulate = rocm_accumulate,
    .osc_compare_and_swap = rocm_compare_and_swap,
    .osc_fetch_and_op = rocm_fetch_and_op,
    .osc_get_accumulate = rocm_get_accumulate,
    .osc_rput = ns_rput,
    .osc_rget = ns_rget,
    .osc_raccumulate = ns_racc,
    .osc_rget_accumulate = ns_rgacc,
    .osc_fence = rocm_fence,
    .osc_start = ns_group,
    .osc_complete = ns_win,
    .osc_post = ns_group,
    .osc_wait = ns_win,
    .osc_test = ns_test,
    .osc_lock = rocm_lock,
    .osc_unlock = rocm_unlock,
    .osc_lock_all = rocm_lock_all,
    .osc_unlock_all = rocm_unlock_all,
    .osc_sync = rocm_sync,
    .osc_flush = rocm_flush,
    .osc_flush_all = rocm_flush_all,
    .osc_flush_local = rocm_flush,
    .osc_flush_local_all = rocm_flush_all,
};

/* ------------------------------------------------------------ selection */

static int rocm_query(struct ompi_win_t *win, void **base, size_t size, int disp_unit,
                      struct ompi_communicator_t *comm, struct opal_info_t *info, int flavor)
{
    bool dev = false;
    int flag = 0;
    if (ompi_amd_device_count() <= 0 || OMPI_COMM_IS_INTER(comm) ||
        ompi_group_have_remote_peers(comm->c_local_group) ||
        ompi_comm_size(comm) > OMPI_AMD_MAX_RANKS)
        return -1;
    if (MPI_WIN_FLAVOR_CREATE == flavor)
        return (0 == size || 1 == ompi_amd_is_device_pointer(*base)) ? mca_osc_rocm_component.priority
                                                                      : -1;
    if (MPI_WIN_FLAVOR_ALLOCATE == flavor) {
        (void) opal_info_get_bool(info, "ompi_amd_device", &dev, &flag);
        return (flag && dev) ? mca_osc_rocm_component.priority : -1;
    }
    return -1;  /* dynamic / shared windows stay with osc/sm, osc/rdma */
}

static int rocm_select(struct ompi_win_t *win, void **base, size_t size, int disp_unit,
                       struct ompi_communicator_t *comm, struct opal_info_t *info, int flavor,
                       int *model)
{
    char name[128];
    int rc, all_ok = 0, local_ok;
    ompi_osc_rocm_module_t *m = calloc(1, sizeof(*m));
    if (NULL == m) return OMPI_ERR_NOT_AVAILABLE;
    m->super = rocm_module_template;
    m->comm = comm;
    m->size = ompi_comm_size(comm);
    /* node-unique name: job id + communicator id + window serial (windows are
     * created collectively, so every rank draws the same serial) */
    snprintf(name, sizeof(name), "%u.%u.w%u", (unsigned) OMPI_PROC_MY_NAME->jobid,
             (unsigned) ompi_comm_get_cid(comm), ++mca_osc_rocm_component.windows);
    rc = ompi_amd_comm_create(name, ompi_comm_rank(comm), m->size, -1, &m->dev_comm);
    if (OMPI_AMD_SUCCESS != rc) {
        free(m);
        return to_ompi_err(rc);
    }
    (void) ompi_amd_comm_set_param(m->dev_comm, "timeout_ms", mca_osc_rocm_component.timeout_ms);
    /* residency may differ between ranks (query is local): decide together */
    local_ok = MPI_WIN_FLAVOR_ALLOCATE == flavor || 0 == size ||
               1 == ompi_amd_is_device_pointer(*base);
    rc = ompi_amd_comm_agree(m->dev_comm, local_ok, &all_ok);
    if (OMPI_AMD_SUCCESS == rc && !all_ok) rc = OMPI_AMD_ERR_UNSUPPORTED;
    if (OMPI_AMD_SUCCESS == rc) {
        rc = MPI_WIN_FLAVOR_ALLOCATE == flavor
                 ? ompi_amd_win_allocate(m->dev_comm, size, disp_unit, base, &m->dev_win)
                 : ompi_amd_win_create(m->dev_comm, *base, size, disp_unit, &m->dev_win);
    }
    if (OMPI_AMD_SUCCESS != rc) {
        (void) ompi_amd_comm_destroy(m->dev_comm);
        free(m);
        return to_ompi_err(rc);
    }
    win->w_osc_module = &m->super;
    *model = MPI_WIN_UNIFIED;
    return OMPI_SUCCESS;
}
