/*
 * osc/rocm component: device windows through libompi_amd.so.
 *
 * Mirrors osc/sm's module functions (ompi/mca/osc/sm/osc_sm_comm.c,
 * osc_sm_active_target.c, osc_sm_passive_target.c) one call each; the
 * data moves by kernels on the origin's GPU over the peers' IPC mappings
 * (include/ompi_amd_osc.h).  General active target synchronisation
 * (post / start / complete / wait / test) runs on the device too: start and
 * wait are kernels that wait for the peers' counters, so MPI's blocking
 * calls return once the stream got there (complete and wait synchronise).
 * Request-based RMA completes its request from the opal_progress callback
 * once the call's kernels have run.  MPI_Win_allocate_shared windows keep
 * every rank's segment in one device allocation that all ranks map
 * (MPI_Win_shared_query hands out the addresses).  Put and get take any
 * datatype pair the convertor has device programs for; accumulates any
 * pair built from one predefined type; everything else returns
 * OMPI_ERR_NOT_SUPPORTED.  Blocking MPI semantics come from the
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
#include "ompi/group/group.h"
#include "ompi/mca/osc/osc.h"
#include "ompi/op/op.h"
#include "ompi/request/request.h"
#include "ompi/runtime/ompi_rte.h"
#include "ompi/win/win.h"
#include "opal/mca/base/mca_base_var.h"
#include "opal/mca/threads/mutex.h"
#include "opal/runtime/opal_progress.h"
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
    .separate_model = 1,
    .own_stream = 1,
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
    (void) mca_base_component_var_register(c, "separate_model",
                                           "1: an MPI_Win_create window over memory its peers cannot "
                                           "map as it is (not an IPC-safe size, or allocated before an "
                                           "IPC close of the process) runs in MPI's separate memory "
                                           "model through a public copy (MPI_WIN_MODEL then reports "
                                           "MPI_WIN_SEPARATE); 0: such a window fails on every rank",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_9,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_osc_rocm_component.separate_model);
    (void) mca_base_component_var_register(c, "own_stream",
                                           "1: a window's epochs and RMA run on a stream with a "
                                           "hardware queue of its own (a lock or PSCW wait on the "
                                           "device never queues in front of other communicators' "
                                           "kernels)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_9,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_osc_rocm_component.own_stream);
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
    case OMPI_AMD_ERR_RMA_SYNC: return OMPI_ERR_RMA_SYNC;
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

/* One side of MPI_Put / MPI_Get with any datatype (osc_sm_comm.c:24-100,
 * 209-270 move it with ompi_datatype_sndrcv): a contiguous predefined type
 * as bytes (program NULL), any other datatype through the device program
 * common/rocm's cache built for the convertor. */
struct opal_datatype_t;
const ompi_amd_ddt_t *opal_rocm_device_ddt(const struct opal_datatype_t *dt);

static int rma_side(struct ompi_datatype_t *dt, int count, const ompi_amd_ddt_t **prog, size_t *n)
{
    const size_t bytes = span(dt, count);
    if (0 != bytes) {
        *prog = NULL;
        *n = bytes;
        return 1;
    }
    /* an ompi_datatype_t begins with its opal_datatype_t (ompi_datatype.h:70-71) */
    *prog = opal_rocm_device_ddt((const struct opal_datatype_t *) dt);
    *n = (size_t) count;
    return NULL != *prog;
}

static int rocm_put(const void *origin, int ocount, struct ompi_datatype_t *odt, int target,
                    ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt, struct ompi_win_t *win)
{
    const ompi_amd_ddt_t *op = NULL, *tp = NULL;
    size_t on = 0, tn = 0;
    const size_t bytes = span(odt, ocount);
    if (0 == ocount) return OMPI_SUCCESS;
    if (disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (0 != bytes && bytes == span(tdt, tcount))
        return to_ompi_err(ompi_amd_put(mod(win)->dev_win, origin, bytes, target, (size_t) disp, NULL));
    if (!rma_side(odt, ocount, &op, &on) || !rma_side(tdt, tcount, &tp, &tn)) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_put_ddt(mod(win)->dev_win, origin, on, op, target, (size_t) disp, tn, tp,
                                        NULL));
}

static int rocm_get(void *origin, int ocount, struct ompi_datatype_t *odt, int target,
                    ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt, struct ompi_win_t *win)
{
    const ompi_amd_ddt_t *op = NULL, *tp = NULL;
    size_t on = 0, tn = 0;
    const size_t bytes = span(odt, ocount);
    if (0 == ocount) return OMPI_SUCCESS;
    if (disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (0 != bytes && bytes == span(tdt, tcount))
        return to_ompi_err(ompi_amd_get(mod(win)->dev_win, origin, bytes, target, (size_t) disp, NULL));
    if (!rma_side(odt, ocount, &op, &on) || !rma_side(tdt, tcount, &tp, &tn)) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_get_ddt(mod(win)->dev_win, origin, on, op, target, (size_t) disp, tn, tp,
                                        NULL));
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

/* Derived datatypes (osc_sm_comm.c:301, 350 -> ompi_osc_base_sndrcv_op):
 * every side built from one predefined type op/base provides the op on
 * (REPLACE / NO_OP on any); each side either that type contiguous (program
 * NULL, count in elements) or a datatype with a device program
 * (common/rocm's cache of the convertor's programs). */
typedef struct {
    int type;                    /* op/base type code of the primitive */
    const ompi_amd_ddt_t *prog;  /* NULL: `type` contiguous */
    size_t count;
} ddt_side;

static int ddt_side_of(struct ompi_datatype_t *dt, int count, int prim_id, ddt_side *out)
{
    struct ompi_datatype_t *p = ompi_datatype_get_single_predefined_type_from_args(dt);
    if (NULL == p || (prim_id >= 0 && p->id != prim_id) || type_code(p) < 0) return 0;
    out->type = type_code(p);
    if (ompi_datatype_is_predefined(dt) && ompi_datatype_is_contiguous_memory_layout(dt, count)) {
        out->prog = NULL;
        out->count = (size_t) count;
        return 1;
    }
    /* an ompi_datatype_t begins with its opal_datatype_t (ompi_datatype.h:70-71) */
    out->prog = opal_rocm_device_ddt((const struct opal_datatype_t *) dt);
    out->count = (size_t) count;
    return NULL != out->prog;
}

static int acc_ddt_ok(struct ompi_datatype_t *odt, int ocount, struct ompi_datatype_t *tdt,
                      int tcount, struct ompi_op_t *op, ddt_side *o, ddt_side *t)
{
    const int idx = op->o_f_to_c_index;
    if (!ompi_op_is_intrinsic(op) || !ddt_side_of(tdt, tcount, -1, t)) return 0;
    struct ompi_datatype_t *prim = ompi_datatype_get_single_predefined_type_from_args(tdt);
    if (OMPI_AMD_OP_NO_OP != idx && !ddt_side_of(odt, ocount, prim->id, o)) return 0;
    if (OMPI_AMD_OP_REPLACE == idx || OMPI_AMD_OP_NO_OP == idx) return 1;
    return ompi_amd_op_supported(idx, t->type) == 1;
}

static int rocm_accumulate(const void *origin, int ocount, struct ompi_datatype_t *odt,
                           int target, ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                           struct ompi_op_t *op, struct ompi_win_t *win)
{
    ddt_side o, t;
    if (0 == ocount) return OMPI_SUCCESS;
    if (disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (acc_ok(odt, ocount, tdt, tcount, op))
        return to_ompi_err(ompi_amd_accumulate(mod(win)->dev_win, origin, (size_t) ocount,
                                               type_code(tdt), target, (size_t) disp,
                                               op->o_f_to_c_index, NULL));
    if (!acc_ddt_ok(odt, ocount, tdt, tcount, op, &o, &t)) return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_accumulate_ddt(mod(win)->dev_win, origin, o.count, o.prog, target,
                                               (size_t) disp, t.count, t.prog, t.type,
                                               op->o_f_to_c_index, NULL));
}

static int rocm_get_accumulate(const void *origin, int ocount, struct ompi_datatype_t *odt,
                               void *result, int rcount, struct ompi_datatype_t *rdt, int target,
                               ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                               struct ompi_op_t *op, struct ompi_win_t *win)
{
    const int no_op = ompi_op_is_intrinsic(op) && OMPI_AMD_OP_NO_OP == op->o_f_to_c_index;
    ddt_side o = {0, NULL, 0}, t, r;
    if (0 == tcount) return OMPI_SUCCESS;
    if (disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (rdt->id == tdt->id && rcount == tcount &&
        acc_ok(no_op ? tdt : odt, no_op ? tcount : ocount, tdt, tcount, op))
        return to_ompi_err(ompi_amd_get_accumulate(mod(win)->dev_win, no_op ? NULL : origin,
                                                   result, (size_t) tcount, type_code(tdt),
                                                   target, (size_t) disp, op->o_f_to_c_index,
                                                   NULL));
    if (!acc_ddt_ok(odt, ocount, tdt, tcount, op, &o, &t) ||
        !ddt_side_of(rdt, rcount, ompi_datatype_get_single_predefined_type_from_args(tdt)->id, &r))
        return OMPI_ERR_NOT_SUPPORTED;
    return to_ompi_err(ompi_amd_get_accumulate_ddt(mod(win)->dev_win, no_op ? NULL : origin,
                                                   o.count, o.prog, result, r.count, r.prog,
                                                   target, (size_t) disp, t.count, t.prog, t.type,
                                                   op->o_f_to_c_index, NULL));
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

/* MPI_Win_sync: the window's copies merged when it runs in the separate
 * model (ompi_amd_win_model), else only the caller's work completed */
static int rocm_sync(struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    return complete(m, ompi_amd_win_sync(m->dev_win, NULL));
}

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

/* ------------------------------------------------- general active target */

/* the members of `group` as ranks of the window's communicator
 * (osc_sm_active_target.c:63-90); NULL when one is not a member */
static int *group_ranks(ompi_osc_rocm_module_t *m, ompi_group_t *group, int *n)
{
    int i, *r1, *r2;
    *n = ompi_group_size(group);
    r1 = malloc(sizeof(int) * (size_t) (*n + 1));
    r2 = malloc(sizeof(int) * (size_t) (*n + 1));
    if (NULL == r1 || NULL == r2) goto fail;
    for (i = 0; i < *n; ++i) r1[i] = i;
    if (OMPI_SUCCESS != ompi_group_translate_ranks(group, *n, r1, m->comm->c_local_group, r2))
        goto fail;
    for (i = 0; i < *n; ++i)
        if (r2[i] < 0 || r2[i] >= m->size) goto fail;
    free(r1);
    return r2;
fail:
    free(r1);
    free(r2);
    return NULL;
}

static int rocm_start(struct ompi_group_t *group, int assert_, struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    int n, rc, *ranks = group_ranks(m, group, &n);
    if (NULL == ranks) return OMPI_ERR_OUT_OF_RESOURCE;
    rc = ompi_amd_win_start(m->dev_win, ranks, n, assert_, NULL);
    free(ranks);
    return to_ompi_err(rc);
}

static int rocm_post(struct ompi_group_t *group, int assert_, struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    int n, rc, *ranks = group_ranks(m, group, &n);
    if (NULL == ranks) return OMPI_ERR_OUT_OF_RESOURCE;
    rc = ompi_amd_win_post(m->dev_win, ranks, n, assert_, NULL);
    free(ranks);
    return to_ompi_err(rc);
}

/* MPI_Win_complete returns when the access epoch's RMA is done everywhere
 * it goes (osc_sm_active_target.c:180-213): the stream is synchronised */
static int rocm_complete(struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    return complete(m, ompi_amd_win_complete(m->dev_win, NULL));
}

static int rocm_wait(struct ompi_win_t *win)
{
    ompi_osc_rocm_module_t *m = mod(win);
    return complete(m, ompi_amd_win_wait(m->dev_win, NULL));
}

static int rocm_test(struct ompi_win_t *win, int *flag)
{
    ompi_osc_rocm_module_t *m = mod(win);
    const int rc = ompi_amd_win_test(m->dev_win, flag);
    if (OMPI_AMD_SUCCESS != rc || !*flag) return to_ompi_err(rc);
    return complete(m, rc);  /* the acquire the library queued has run */
}

/* ------------------------------------------------------ request-based RMA */

static opal_mutex_t rma_active_lock = OPAL_MUTEX_STATIC_INIT;
static ompi_osc_rocm_request_t *rma_active;
static int rma_progress_registered;

/* opal_progress callback: complete the requests whose kernels finished */
static int rma_progress(void)
{
    ompi_osc_rocm_request_t **pp, *done = NULL;
    int completed = 0;
    if (NULL == rma_active) return 0;
    OPAL_THREAD_LOCK(&rma_active_lock);
    pp = &rma_active;
    while (NULL != *pp) {
        ompi_osc_rocm_request_t *r = *pp;
        int fin = 0;
        const int rc = ompi_amd_rma_test(r->rma, &fin);
        if (OMPI_AMD_SUCCESS != rc || fin) {
            r->super.req_status.MPI_ERROR = to_ompi_err(rc);
            *pp = r->next_active;
            r->next_active = done;
            done = r;
        } else {
            pp = &r->next_active;
        }
    }
    OPAL_THREAD_UNLOCK(&rma_active_lock);
    while (NULL != done) {
        ompi_osc_rocm_request_t *r = done;
        done = r->next_active;
        r->next_active = NULL;
        ompi_request_complete(&r->super, true);
        ++completed;
    }
    return completed;
}

static int rma_request_free(ompi_request_t **rptr)
{
    ompi_osc_rocm_request_t *r = (ompi_osc_rocm_request_t *) *rptr, **pp;
    int rc;
    OPAL_THREAD_LOCK(&rma_active_lock);
    for (pp = &rma_active; NULL != *pp; pp = &(*pp)->next_active) {
        if (*pp == r) {
            *pp = r->next_active;
            break;
        }
    }
    OPAL_THREAD_UNLOCK(&rma_active_lock);
    rc = ompi_amd_rma_free(r->rma);  /* waits for the kernels first */
    OMPI_REQUEST_FINI(&r->super);
    OBJ_RELEASE(r);
    *rptr = MPI_REQUEST_NULL;
    return to_ompi_err(rc);
}

static void rma_request_construct(ompi_osc_rocm_request_t *r)
{
    r->super.req_type = OMPI_REQUEST_WIN;
    r->super.req_status._cancelled = 0;
    r->super.req_free = rma_request_free;
    r->super.req_cancel = NULL;
    r->rma = NULL;
    r->next_active = NULL;
}

OBJ_CLASS_INSTANCE(ompi_osc_rocm_request_t, ompi_request_t, rma_request_construct, NULL);

/* an MPI request over the library request of a call that returned rc */
static int rma_wrap(int rc, ompi_amd_rma_request_t *const *rmap, struct ompi_win_t *win,
                    ompi_request_t **request)
{
    ompi_amd_rma_request_t *rma = *rmap;  /* read after the call that set it */
    ompi_osc_rocm_request_t *r;
    if (OMPI_AMD_SUCCESS != rc) return to_ompi_err(rc);
    r = OBJ_NEW(ompi_osc_rocm_request_t);
    if (NULL == r) {
        (void) ompi_amd_rma_free(rma);
        return OMPI_ERR_OUT_OF_RESOURCE;
    }
    OMPI_REQUEST_INIT(&r->super, false);
    r->super.req_state = OMPI_REQUEST_ACTIVE;
    r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
    r->rma = rma;
    OPAL_THREAD_LOCK(&rma_active_lock);
    r->next_active = rma_active;
    rma_active = r;
    if (!rma_progress_registered) {
        rma_progress_registered = 1;
        (void) opal_progress_register(rma_progress);
    }
    OPAL_THREAD_UNLOCK(&rma_active_lock);
    *request = &r->super;
    return OMPI_SUCCESS;
}

/* a zero-count call completes at once (osc_sm_comm.c:54-57 hands back
 * ompi_request_empty); here a library request over no kernels does */
static int rocm_rput(const void *origin, int ocount, struct ompi_datatype_t *odt, int target,
                     ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                     struct ompi_win_t *win, ompi_request_t **request)
{
    ompi_amd_rma_request_t *rma = NULL;
    const ompi_amd_ddt_t *op = NULL, *tp = NULL;
    size_t on = 0, tn = 0;
    const size_t bytes = span(odt, ocount);
    if (disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (0 == ocount || (0 != bytes && bytes == span(tdt, tcount)))
        return rma_wrap(ompi_amd_rput(mod(win)->dev_win, origin, 0 == ocount ? 0 : bytes, target,
                                      (size_t) disp, NULL, &rma), &rma, win, request);
    if (!rma_side(odt, ocount, &op, &on) || !rma_side(tdt, tcount, &tp, &tn)) return OMPI_ERR_NOT_SUPPORTED;
    return rma_wrap(ompi_amd_rput_ddt(mod(win)->dev_win, origin, on, op, target, (size_t) disp, tn, tp,
                                      NULL, &rma), &rma, win, request);
}

static int rocm_rget(void *origin, int ocount, struct ompi_datatype_t *odt, int target,
                     ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                     struct ompi_win_t *win, ompi_request_t **request)
{
    ompi_amd_rma_request_t *rma = NULL;
    const ompi_amd_ddt_t *op = NULL, *tp = NULL;
    size_t on = 0, tn = 0;
    const size_t bytes = span(odt, ocount);
    if (disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (0 == ocount || (0 != bytes && bytes == span(tdt, tcount)))
        return rma_wrap(ompi_amd_rget(mod(win)->dev_win, origin, 0 == ocount ? 0 : bytes, target,
                                      (size_t) disp, NULL, &rma), &rma, win, request);
    if (!rma_side(odt, ocount, &op, &on) || !rma_side(tdt, tcount, &tp, &tn)) return OMPI_ERR_NOT_SUPPORTED;
    return rma_wrap(ompi_amd_rget_ddt(mod(win)->dev_win, origin, on, op, target, (size_t) disp, tn, tp,
                                      NULL, &rma), &rma, win, request);
}

static int rocm_raccumulate(const void *origin, int ocount, struct ompi_datatype_t *odt,
                            int target, ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                            struct ompi_op_t *op, struct ompi_win_t *win, ompi_request_t **request)
{
    ompi_amd_rma_request_t *rma = NULL;
    ddt_side o, t;
    if (0 != ocount && disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (0 == ocount || acc_ok(odt, ocount, tdt, tcount, op))
        return rma_wrap(ompi_amd_raccumulate(mod(win)->dev_win, origin, (size_t) ocount,
                                             0 != ocount ? type_code(tdt) : 0, target,
                                             (size_t) disp, op->o_f_to_c_index, NULL, &rma),
                        &rma, win, request);
    if (!acc_ddt_ok(odt, ocount, tdt, tcount, op, &o, &t)) return OMPI_ERR_NOT_SUPPORTED;
    return rma_wrap(ompi_amd_raccumulate_ddt(mod(win)->dev_win, origin, o.count, o.prog, target,
                                             (size_t) disp, t.count, t.prog, t.type,
                                             op->o_f_to_c_index, NULL, &rma), &rma, win, request);
}

static int rocm_rget_accumulate(const void *origin, int ocount, struct ompi_datatype_t *odt,
                                void *result, int rcount, struct ompi_datatype_t *rdt, int target,
                                ptrdiff_t disp, int tcount, struct ompi_datatype_t *tdt,
                                struct ompi_op_t *op, struct ompi_win_t *win,
                                ompi_request_t **request)
{
    ompi_amd_rma_request_t *rma = NULL;
    const int no_op = ompi_op_is_intrinsic(op) && OMPI_AMD_OP_NO_OP == op->o_f_to_c_index;
    ddt_side o = {0, NULL, 0}, t, r;
    if (0 != tcount && disp < 0) return OMPI_ERR_NOT_SUPPORTED;
    if (0 == tcount || (rdt->id == tdt->id && rcount == tcount &&
                        acc_ok(no_op ? tdt : odt, no_op ? tcount : ocount, tdt, tcount, op)))
        return rma_wrap(ompi_amd_rget_accumulate(mod(win)->dev_win, no_op ? NULL : origin, result,
                                                 (size_t) tcount, 0 != tcount ? type_code(tdt) : 0,
                                                 target, (size_t) disp, op->o_f_to_c_index, NULL,
                                                 &rma), &rma, win, request);
    if (!acc_ddt_ok(odt, ocount, tdt, tcount, op, &o, &t) ||
        !ddt_side_of(rdt, rcount, ompi_datatype_get_single_predefined_type_from_args(tdt)->id, &r))
        return OMPI_ERR_NOT_SUPPORTED;
    return rma_wrap(ompi_amd_rget_accumulate_ddt(mod(win)->dev_win, no_op ? NULL : origin,
                                                 o.count, o.prog, result, r.count, r.prog, target,
                                                 (size_t) disp, t.count, t.prog, t.type,
                                                 op->o_f_to_c_index, NULL, &rma),
                    &rma, win, request);
}

/* MPI_Win_shared_query (osc_sm_component.c:455-485): baseptr points to a
 * void *; MPI_PROC_NULL asks for the first segment of nonzero size */
static int rocm_shared_query(struct ompi_win_t *win, int rank, size_t *size, int *disp_unit,
                             void *baseptr)
{
    const int rc = ompi_amd_win_shared_query(mod(win)->dev_win, MPI_PROC_NULL == rank ? -1 : rank,
                                             size, disp_unit, (void **) baseptr);
    return OMPI_AMD_ERR_UNSUPPORTED == rc ? MPI_ERR_WIN : to_ompi_err(rc);
}

/* MPI_Win_attach / MPI_Win_detach (osc_rdma_dynamic.c:162-300 for the
 * host flavor): device memory peers can map into a dynamic window made with
 * the ompi_amd_device info key.  Host memory, device memory peers cannot
 * map as it is, or a window of another flavor (as osc/sm,
 * osc_sm_component.c:488-511): MPI_ERR_RMA_ATTACH; detaching what was not
 * attached: MPI_ERR_RMA_RANGE. */
static int rocm_attach(struct ompi_win_t *w, void *b, size_t s)
{
    const int rc = ompi_amd_win_attach(mod(w)->dev_win, b, s);
    return OMPI_AMD_SUCCESS == rc ? OMPI_SUCCESS : MPI_ERR_RMA_ATTACH;
}
static int rocm_detach(struct ompi_win_t *w, const void *b)
{
    const int rc = ompi_amd_win_detach(mod(w)->dev_win, b);
    return OMPI_AMD_SUCCESS == rc ? OMPI_SUCCESS
         : OMPI_AMD_ERR_UNSUPPORTED == rc ? MPI_ERR_RMA_ATTACH : MPI_ERR_RMA_RANGE;
}

static const ompi_osc_base_module_t rocm_module_template = {
    .osc_win_shared_query = rocm_shared_query,
    .osc_win_attach = rocm_attach,
    .osc_win_detach = rocm_detach,
    .osc_free = rocm_free,
    .osc_put = rocm_put,
    .osc_get = rocm_get,
    .osc_accumulate = rocm_accumulate,
    .osc_compare_and_swap = rocm_compare_and_swap,
    .osc_fetch_and_op = rocm_fetch_and_op,
    .osc_get_accumulate = rocm_get_accumulate,
    .osc_rput = rocm_rput,
    .osc_rget = rocm_rget,
    .osc_raccumulate = rocm_raccumulate,
    .osc_rget_accumulate = rocm_rget_accumulate,
    .osc_fence = rocm_fence,
    .osc_start = rocm_start,
    .osc_complete = rocm_complete,
    .osc_post = rocm_post,
    .osc_wait = rocm_wait,
    .osc_test = rocm_test,
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

/* A window whose ranks disagree about device memory (see rocm_query),
 * refused by the rocm_select that follows the query on this thread. */
static _Thread_local struct ompi_win_t *mixed_win;

/* The osc framework selects per rank (ompi_osc_base_select,
 * osc_base_init.c:33-80: the highest-priority query wins, locally), but
 * whether a window is a device window may differ between ranks: MPI lets
 * MPI_Win_create bases live in device memory on some ranks and host memory
 * on others, and the info key of the allocating flavors is per rank too.
 * Every rank of the communicator runs this query at the same point of its
 * collective ompi_osc_base_select, so the decision is agreed here, over the
 * communicator's own allreduce (as osc/rdma agrees on its setup,
 * osc_rdma_component.c:533): no rank holds device memory -> -1 on every
 * rank (the host components take the window alike); device memory only ->
 * this component everywhere; both -> this component everywhere, and
 * rocm_select refuses the window on every rank with the same error (peers
 * cannot map a host base; no component serves the mix). */
static int rocm_query(struct ompi_win_t *win, void **base, size_t size, int disp_unit,
                      struct ompi_communicator_t *comm, struct opal_info_t *info, int flavor)
{
    bool dev = false;
    int flag = 0, v[2] = {0, 0};  /* some rank has device memory / host memory */
    /* a refusal is for the select that follows this query: a query whose
     * select never ran (another component won) leaves nothing behind */
    mixed_win = NULL;
    if (ompi_amd_device_count() <= 0 || OMPI_COMM_IS_INTER(comm) ||
        ompi_group_have_remote_peers(comm->c_local_group) ||
        ompi_comm_size(comm) > OMPI_AMD_MAX_RANKS)
        return -1;
    if (MPI_WIN_FLAVOR_CREATE == flavor) {
        if (0 != size) {
            dev = 1 == ompi_amd_is_device_pointer(*base);
            v[0] = dev;
            v[1] = !dev;
        }
    } else if (MPI_WIN_FLAVOR_ALLOCATE == flavor || MPI_WIN_FLAVOR_SHARED == flavor ||
               MPI_WIN_FLAVOR_DYNAMIC == flavor) {
        /* a dynamic window holds device memory only when the application
         * says so at creation (what it attaches comes later): with the info
         * key this component takes it and refuses host attaches; without
         * it osc/rdma keeps dynamic windows, for host memory */
        (void) opal_info_get_bool(info, "ompi_amd_device", &dev, &flag);
        v[0] = flag && dev;
        v[1] = !v[0];
    } else {
        return -1;
    }
    if (OMPI_SUCCESS != comm->c_coll->coll_allreduce(MPI_IN_PLACE, v, 2, MPI_INT, MPI_MAX, comm,
                                                     comm->c_coll->coll_allreduce_module))
        return -1;
    if (!v[0]) return -1;
    mixed_win = v[1] ? win : NULL;
    return mca_osc_rocm_component.priority;
}

static int rocm_select(struct ompi_win_t *win, void **base, size_t size, int disp_unit,
                       struct ompi_communicator_t *comm, struct opal_info_t *info, int flavor,
                       int *model)
{
    char name[128];
    int rc, all_ok = 0, local_ok;
    ompi_osc_rocm_module_t *m;
    if (mixed_win == win) {  /* agreed in rocm_query: every rank refuses alike */
        mixed_win = NULL;
        return OMPI_ERR_NOT_SUPPORTED;
    }
    m = calloc(1, sizeof(*m));
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
    (void) ompi_amd_comm_set_param(m->dev_comm, "osc_win_separate", mca_osc_rocm_component.separate_model);
    (void) ompi_amd_comm_set_param(m->dev_comm, "own_stream", mca_osc_rocm_component.own_stream);
    /* agreed in rocm_query already; the library confirms it on its own
     * rendezvous (a failure here fails every rank alike) */
    local_ok = MPI_WIN_FLAVOR_CREATE != flavor || 0 == size ||
               1 == ompi_amd_is_device_pointer(*base);
    rc = ompi_amd_comm_agree(m->dev_comm, local_ok, &all_ok);
    if (OMPI_AMD_SUCCESS == rc && !all_ok) rc = OMPI_AMD_ERR_UNSUPPORTED;
    if (OMPI_AMD_SUCCESS == rc && MPI_WIN_FLAVOR_DYNAMIC == flavor) {
        rc = ompi_amd_win_create_dynamic(m->dev_comm, &m->dev_win);
    } else if (OMPI_AMD_SUCCESS == rc && MPI_WIN_FLAVOR_SHARED == flavor) {
        /* one allocation, segments back to back unless alloc_shared_noncontig
         * (osc_sm_component.c:259-268) */
        bool noncontig = false;
        int nflag = 0;
        (void) opal_info_get_bool(info, "alloc_shared_noncontig", &noncontig, &nflag);
        rc = ompi_amd_win_allocate_shared(m->dev_comm, size, disp_unit, nflag && noncontig, base,
                                          &m->dev_win);
    } else if (OMPI_AMD_SUCCESS == rc) {
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
    /* MPI_WIN_SEPARATE when some rank's MPI_Win_create memory is reached
     * through a public copy (include/ompi_amd_osc.h); every rank agrees */
    *model = OMPI_AMD_WIN_SEPARATE == ompi_amd_win_model(m->dev_win) ? MPI_WIN_SEPARATE
                                                                      : MPI_WIN_UNIFIED;
    return OMPI_SUCCESS;
}
