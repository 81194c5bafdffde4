/*
 * pml/rocm component: interposition on the selected PML (see pml_rocm.h).
 *
 * Component protocol (pml_base_select.c): every PML component is opened,
 * the selected one's pmlm_init provides mca_pml, the others are closed.
 * pml/rocm's pmlm_init returns NULL, so it is always closed; its close
 * saves mca_pml (the selected PML's table) and installs the functions below
 * — pml/v's parasite pattern (pml_v_component.c:123-160).
 *
 * Requests: library transfers complete on the device; a progress callback
 * registered with opal_progress (as coll/rocm and coll/libnbc do) tests the
 * active requests with ompi_amd_p2p_test, copies staged receives back, fills
 * the status and completes them, so MPI_Wait / MPI_Test work unchanged.
 */
#include "ompi_config.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mpi.h"
#include "ompi/constants.h"
#include "ompi/runtime/ompi_rte.h"
#include "opal/mca/base/mca_base_var.h"
#include "opal/mca/threads/mutex.h"
#include "opal/runtime/opal_progress.h"

#include "ompi_amd.h"
#include "pml_rocm.h"

static int rocm_register(void);
static int rocm_open(void);
static int rocm_close(void);
static mca_pml_base_module_t *rocm_init(int *priority, bool progress_threads, bool mpi_threads);
static int rocm_finalize(void);

mca_pml_rocm_component_t mca_pml_rocm_component = {
    .super = {
        .pmlm_version = {
            MCA_PML_BASE_VERSION_2_0_0,
            .mca_component_name = "rocm",
            MCA_BASE_MAKE_VERSION(component, OMPI_MAJOR_VERSION, OMPI_MINOR_VERSION,
                                  OMPI_RELEASE_VERSION),
            .mca_open_component = rocm_open,
            .mca_close_component = rocm_close,
            .mca_register_component_params = rocm_register,
        },
        .pmlm_data = { MCA_BASE_METADATA_PARAM_CHECKPOINT },
        .pmlm_init = rocm_init,
        .pmlm_finalize = rocm_finalize,
    },
    .enable = 1,
    .timeout_ms = 0,
    .own_stream = 1,
    .host_path = 0,
};

mca_pml_base_module_t mca_pml_rocm_host;
int mca_pml_rocm_installed;

static int rocm_register(void)
{
    mca_base_component_t *c = &mca_pml_rocm_component.super.pmlm_version;
    (void) mca_base_component_var_register(c, "enable",
                                           "Route user-tag messages of node-local communicators "
                                           "through the device library",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_pml_rocm_component.enable);
    (void) mca_base_component_var_register(c, "own_stream",
                                           "1: a communicator's device transfers run on a stream with "
                                           "a hardware queue of its own (a receive's copy waiting on "
                                           "the device for its sender never queues in front of "
                                           "another communicator's kernels)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_pml_rocm_component.own_stream);
    (void) mca_base_component_var_register(c, "timeout_ms",
                                           "Host wait limit of a library transfer (0: none, MPI "
                                           "semantics)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_pml_rocm_component.timeout_ms);
    (void) mca_base_component_var_register(c, "host_path",
                                           "1: host-buffer operations go to the saved PML (the "
                                           "application never mixes host and device buffers in "
                                           "one message)",
                                           MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                           MCA_BASE_VAR_SCOPE_READONLY,
                                           &mca_pml_rocm_component.host_path);
    return OMPI_SUCCESS;
}

static int rocm_open(void) { return OMPI_SUCCESS; }

/* never selected: the interposition happens at close */
static mca_pml_base_module_t *rocm_init(int *priority, bool progress_threads, bool mpi_threads)
{
    *priority = -1;
    return NULL;
}

static int rocm_finalize(void) { return OMPI_SUCCESS; }

/* ------------------------------------------------------------- communicators */

struct rocm_comm {
    struct ompi_communicator_t *comm;
    ompi_amd_comm_t *dev;
    struct rocm_comm *next;
};
static struct rocm_comm *rocm_comms;
static opal_mutex_t rocm_lock = OPAL_MUTEX_STATIC_INIT;

ompi_amd_comm_t *mca_pml_rocm_comm_of(struct ompi_communicator_t *comm)
{
    struct rocm_comm *e;
    for (e = rocm_comms; NULL != e; e = e->next)
        if (e->comm == comm) return e->dev;
    return NULL;
}

/* pml_add_comm (pml.h:175): the saved PML first, then — collectively, every
 * rank of the new communicator runs it — a library communicator for a
 * node-local intra-communicator of 2..16 ranks. */
static int rocm_add_comm(struct ompi_communicator_t *comm)
{
    char name[128];
    ompi_amd_comm_t *dev = NULL;
    struct rocm_comm *e;
    int rc = mca_pml_rocm_host.pml_add_comm(comm);
    if (OMPI_SUCCESS != rc) return rc;
    if (OMPI_COMM_IS_INTER(comm) || ompi_comm_size(comm) < 2 ||
        ompi_comm_size(comm) > OMPI_AMD_MAX_RANKS ||
        ompi_group_have_remote_peers(comm->c_local_group) || ompi_amd_device_count() < 1) {
        return OMPI_SUCCESS;
    }
    snprintf(name, sizeof(name), "%u.%u.p", (unsigned) OMPI_PROC_MY_NAME->jobid,
             (unsigned) ompi_comm_get_cid(comm));
    if (OMPI_AMD_SUCCESS != ompi_amd_comm_create(name, ompi_comm_rank(comm), ompi_comm_size(comm),
                                                 -1, &dev)) {
        return OMPI_SUCCESS; /* every rank fails alike (the creation is collective) */
    }
    /* host waits follow MPI: no limit unless the parameter sets one */
    (void) ompi_amd_comm_set_param(dev, "p2p_timeout_ms", mca_pml_rocm_component.timeout_ms);
    (void) ompi_amd_comm_set_param(dev, "own_stream", mca_pml_rocm_component.own_stream);
    e = (struct rocm_comm *) calloc(1, sizeof(*e));
    if (NULL == e) {
        (void) ompi_amd_comm_destroy(dev);
        return OMPI_ERR_OUT_OF_RESOURCE;
    }
    e->comm = comm;
    e->dev = dev;
    OPAL_THREAD_LOCK(&rocm_lock);
    e->next = rocm_comms;
    rocm_comms = e;
    OPAL_THREAD_UNLOCK(&rocm_lock);
    return OMPI_SUCCESS;
}

static int rocm_del_comm(struct ompi_communicator_t *comm)
{
    struct rocm_comm **pp, *e = NULL;
    OPAL_THREAD_LOCK(&rocm_lock);
    for (pp = &rocm_comms; NULL != *pp; pp = &(*pp)->next) {
        if ((*pp)->comm == comm) {
            e = *pp;
            *pp = e->next;
            break;
        }
    }
    OPAL_THREAD_UNLOCK(&rocm_lock);
    if (NULL != e) {
        (void) ompi_amd_comm_destroy(e->dev); /* collective, like del_comm */
        free(e);
    }
    return mca_pml_rocm_host.pml_del_comm(comm);
}

/* ------------------------------------------------------------- helpers */

static int rocm_err(int rc)
{
    switch (rc) {
    case OMPI_AMD_SUCCESS: return OMPI_SUCCESS;
    case OMPI_AMD_ERR_TRUNCATE: return MPI_ERR_TRUNCATE;
    case OMPI_AMD_ERR_BAD_PARAM: return OMPI_ERR_BAD_PARAM;
    case OMPI_AMD_ERR_TIMEOUT: return OMPI_ERR_TIMEOUT;
    default: return OMPI_ERROR;
    }
}

/* library traffic: a library communicator and a user tag (ANY_TAG included) */
static ompi_amd_comm_t *takes(struct ompi_communicator_t *comm, int tag, int peer)
{
    if (peer == MPI_PROC_NULL || (tag < 0 && tag != MPI_ANY_TAG)) return NULL;
    return mca_pml_rocm_comm_of(comm);
}

/* takes(), and with pml_rocm_host_path the buffer is device memory (a
 * zero-byte operation counts as host: nothing to move) */
static ompi_amd_comm_t *takes_buf(struct ompi_communicator_t *comm, int tag, int peer,
                                  const void *buf, size_t count)
{
    ompi_amd_comm_t *dev = takes(comm, tag, peer);
    if (NULL != dev && mca_pml_rocm_component.host_path &&
        (0 == count || !ompi_amd_is_device_pointer(buf))) {
        return NULL;
    }
    return dev;
}

static size_t type_bytes(struct ompi_datatype_t *dtype, size_t count)
{
    size_t size = 0;
    (void) ompi_datatype_type_size(dtype, &size);
    return size * count;
}

/* common/rocm (opal_datatype_rocm.h): a device typed buffer packed into /
 * unpacked from a packed device buffer by one kernel; 1 when the datatype
 * has no device program.  An ompi_datatype_t begins with its
 * opal_datatype_t (ompi/datatype/ompi_datatype.h:70-71). */
struct opal_datatype_t;
int opal_rocm_pack_device(const struct opal_datatype_t *dt, size_t count, const void *src,
                          void *packed, void *stream);
int opal_rocm_unpack_device(const struct opal_datatype_t *dt, size_t count, const void *packed,
                            void *dst, void *stream);
int opal_rocm_device_program(const struct opal_datatype_t *dt);
#define OPAL_DT(d) ((const struct opal_datatype_t *) (d))

/* Device packing buffers, reused (a hipMalloc per message would cost more
 * than the pack): the smallest free one that fits, else a new one; at most
 * DEV_POOL kept. */
#define DEV_POOL 8
static struct { void *p; size_t cap; } dev_pool[DEV_POOL];
static int dev_pool_n;
static opal_mutex_t dev_pool_lock = OPAL_MUTEX_STATIC_INIT;

static void *dev_stage_take(size_t bytes)
{
    void *p = NULL;
    int best = -1;
    OPAL_THREAD_LOCK(&dev_pool_lock);
    for (int i = 0; i < dev_pool_n; ++i)
        if (dev_pool[i].cap >= bytes && (best < 0 || dev_pool[i].cap < dev_pool[best].cap)) best = i;
    if (best >= 0) {
        p = dev_pool[best].p;
        dev_pool[best] = dev_pool[--dev_pool_n];
    }
    OPAL_THREAD_UNLOCK(&dev_pool_lock);
    if (NULL == p && OMPI_AMD_SUCCESS != ompi_amd_device_alloc(&p, bytes)) p = NULL;
    return p;
}

/* back to the pool; `bytes` (what the request needed) is a lower bound of
 * the buffer's capacity */
static void dev_stage_put(void *p, size_t bytes)
{
    if (NULL == p) return;
    OPAL_THREAD_LOCK(&dev_pool_lock);
    if (dev_pool_n < DEV_POOL) {
        dev_pool[dev_pool_n].p = p;
        dev_pool[dev_pool_n++].cap = bytes;
        p = NULL;
    }
    OPAL_THREAD_UNLOCK(&dev_pool_lock);
    (void) ompi_amd_device_free(p);
}

static void stage_free(mca_pml_rocm_request_t *r)
{
    if (r->stage_dev) dev_stage_put(r->stage, r->bytes);
    else free(r->stage);
    r->stage = NULL;
    r->stage_dev = 0;
}

/* what the library gets for the user's buffer: the buffer itself when its
 * layout is contiguous (host or device: the library stages host memory in
 * its own pooled device buffers); a device buffer of a non-contiguous type
 * is packed on the device into a pooled device buffer (one kernel: no host
 * round trip — the reference packs device data through the convertor in
 * the send path, pml_ob1_cuda.c:56-101); a host one is packed on the host */
static int stage_for(mca_pml_rocm_request_t *r, int fill)
{
    r->bytes = type_bytes(r->dtype, r->count);
    r->stage = NULL;
    r->stage_dev = 0;
    if (0 == r->bytes || ompi_datatype_is_contiguous_memory_layout(r->dtype, (int) r->count))
        return OMPI_SUCCESS;
    if (ompi_amd_is_device_pointer(r->buf) && opal_rocm_device_program(OPAL_DT(r->dtype))) {
        void *d = dev_stage_take(r->bytes);
        const int rc = NULL == d ? 1 : fill ? opal_rocm_pack_device(OPAL_DT(r->dtype), r->count,
                                                                   r->buf, d, NULL) : 0;
        if (0 == rc) {
            r->stage = d;
            r->stage_dev = 1;
            return OMPI_SUCCESS;
        }
        dev_stage_put(d, r->bytes);
        if (rc < 0) return OMPI_ERROR;
    }
    r->stage = malloc(r->bytes);
    if (NULL == r->stage) return OMPI_ERR_OUT_OF_RESOURCE;
    if (fill && MPI_SUCCESS != ompi_datatype_sndrcv(r->buf, (int) r->count, r->dtype, r->stage,
                                                    (int) r->bytes, MPI_BYTE)) {
        free(r->stage);
        r->stage = NULL;
        return OMPI_ERROR;
    }
    return OMPI_SUCCESS;
}

/* a packed receive's `got` bytes back into the user's layout (whole
 * elements: a short message fills a prefix of them) */
static int unstage_recv(mca_pml_rocm_request_t *r, size_t got)
{
    size_t size = 0;
    if (NULL == r->stage || 0 == got) return OMPI_SUCCESS;
    (void) ompi_datatype_type_size(r->dtype, &size);
    if (r->stage_dev)
        return 0 == opal_rocm_unpack_device(OPAL_DT(r->dtype), size ? got / size : 0, r->stage,
                                            r->buf, NULL)
                   ? OMPI_SUCCESS
                   : OMPI_ERROR;
    return MPI_SUCCESS == ompi_datatype_sndrcv(r->stage, (int) got, MPI_BYTE, r->buf,
                                               (int) (size ? got / size : 0), r->dtype)
               ? OMPI_SUCCESS
               : OMPI_ERROR;
}

static void *lib_buf(mca_pml_rocm_request_t *r) { return NULL != r->stage ? r->stage : r->buf; }

/* ------------------------------------------- the saved PML, device buffers */

/* The saved PML (ob1) moves host memory only.  What pml/rocm leaves to it —
 * system tags: the collectives' own messages (coll/base algorithms, libnbc
 * schedules, every collective coll/rocm does not offload) — can still name
 * device buffers; such a message runs on a host copy of its typed span: a
 * send copies the span out before the saved PML sees it, a receive gets a
 * host span (pre-filled, so the type's gaps keep their bytes) and copies it
 * back when it completes — coll/cuda's staging (coll_cuda_allreduce.c:
 * 42-72) per message; the reference's ob1 moves device memory itself
 * (pml_ob1_cuda.c:56-101). */
static int on_device(const void *buf, size_t count, struct ompi_datatype_t *dtype)
{
    ptrdiff_t tlb = 0, text = 0;
    if (0 == count || NULL == buf) return 0;
    (void) ompi_datatype_get_true_extent(dtype, &tlb, &text);
    return ompi_amd_is_device_pointer((const char *) buf + tlb);
}

/* A received span goes back to the device whole (pre-filled, so the type's
 * gaps carry the device's own bytes) only for a non-contiguous type the
 * convertor has no device program for; every other receive writes back
 * exactly the bytes the message delivered (host_span_back). */
static int recv_whole_span(const mca_pml_rocm_request_t *r)
{
    return !ompi_datatype_is_contiguous_memory_layout(r->dtype, (int) r->count) &&
           !opal_rocm_device_program(OPAL_DT(r->dtype));
}

/* r->hspan: host memory for r->buf's typed span; a send's is filled from
 * the device (the payload), a receive's only when it goes back whole */
static int host_span(mca_pml_rocm_request_t *r)
{
    ptrdiff_t lb, ext, tlb, text;
    (void) ompi_datatype_get_extent(r->dtype, &lb, &ext);
    (void) ompi_datatype_get_true_extent(r->dtype, &tlb, &text);
    r->hbytes = (r->count - 1) * (size_t) ext + (size_t) text;
    r->hgap = tlb;
    if (NULL == r->hspan && NULL == (r->hspan = malloc(r->hbytes ? r->hbytes : 1)))
        return OMPI_ERR_OUT_OF_RESOURCE;
    if (!r->is_send && !recv_whole_span(r)) return OMPI_SUCCESS;
    return OMPI_AMD_SUCCESS == ompi_amd_memcpy(r->hspan, (char *) r->buf + tlb, r->hbytes) ? OMPI_SUCCESS
                                                                                       : OMPI_ERROR;
}

static void *host_base(const mca_pml_rocm_request_t *r) { return r->hspan - r->hgap; }

/* A received host span back into the device buffer: the `got` bytes the
 * message delivered and nothing else, as ob1 writes exactly the typed bytes
 * through the convertor.  Several receives can be in flight into one device
 * buffer with interleaved typed spans (coll/base's linear gather into a
 * resized column type, an alltoall of vectors): copying a whole span back
 * would overwrite the other receives' elements with this one's stale
 * gaps.  Contiguous layout: the received prefix.  Otherwise the received
 * elements are packed on the host, copied into a pooled device stage and
 * scattered by the type's device program (one kernel, typed bytes only). */
static int host_span_back(const mca_pml_rocm_request_t *r, size_t got)
{
    size_t size = 0, elems, bytes;
    char *packed;
    void *d;
    int rc;
    if (0 == got || 0 == r->count) return OMPI_SUCCESS;
    if (ompi_datatype_is_contiguous_memory_layout(r->dtype, (int) r->count)) {
        bytes = got < r->hbytes ? got : r->hbytes;
        return OMPI_AMD_SUCCESS == ompi_amd_memcpy((char *) r->buf + r->hgap, r->hspan, bytes)
                   ? OMPI_SUCCESS
                   : OMPI_ERROR;
    }
    if (recv_whole_span(r))
        return OMPI_AMD_SUCCESS == ompi_amd_memcpy((char *) r->buf + r->hgap, r->hspan, r->hbytes)
                   ? OMPI_SUCCESS
                   : OMPI_ERROR;
    (void) ompi_datatype_type_size(r->dtype, &size);
    elems = size ? got / size : 0;
    if (elems > r->count) elems = r->count;
    bytes = elems * size;
    if (0 == bytes) return OMPI_SUCCESS;
    if (NULL == (packed = malloc(bytes))) return OMPI_ERR_OUT_OF_RESOURCE;
    rc = MPI_SUCCESS == ompi_datatype_sndrcv(host_base(r), (int) elems, r->dtype, packed, (int) bytes,
                                             MPI_BYTE)
             ? OMPI_SUCCESS
             : OMPI_ERROR;
    d = OMPI_SUCCESS == rc ? dev_stage_take(bytes) : NULL;
    if (OMPI_SUCCESS == rc && NULL == d) rc = OMPI_ERR_OUT_OF_RESOURCE;
    if (OMPI_SUCCESS == rc && OMPI_AMD_SUCCESS != ompi_amd_memcpy(d, packed, bytes)) rc = OMPI_ERROR;
    if (OMPI_SUCCESS == rc && 0 != opal_rocm_unpack_device(OPAL_DT(r->dtype), elems, d, r->buf, NULL))
        rc = OMPI_ERROR;
    dev_stage_put(d, bytes);
    free(packed);
    return rc;
}

/* Wait for a library request without a time limit, driving opal_progress
 * (other PML traffic, e.g. the system-tag messages of a collective the peer
 * is inside, must keep moving: ob1's blocking calls do the same). */
/* Wait for a library request while driving opal_progress.  No limit by
 * default (MPI semantics); pml_rocm_timeout_ms > 0 bounds it (diagnostics:
 * a lost message becomes OMPI_ERR_TIMEOUT instead of a hang). */
static int wait_lib(ompi_amd_p2p_request_t *lib, ompi_amd_status_t *s)
{
    const int limit_ms = mca_pml_rocm_component.timeout_ms;
    struct timespec t0, t;
    (void) clock_gettime(CLOCK_MONOTONIC, &t0);
    for (unsigned k = 0;; ++k) {
        int fin = 0;
        const int rc = ompi_amd_p2p_test(lib, &fin, s);
        if (OMPI_AMD_SUCCESS != rc || fin) return rc;
        opal_progress();
        if (limit_ms > 0 && 0 == (k & 1023)) {
            (void) clock_gettime(CLOCK_MONOTONIC, &t);
            if ((t.tv_sec - t0.tv_sec) * 1000 + (t.tv_nsec - t0.tv_nsec) / 1000000 > limit_ms)
                return OMPI_AMD_ERR_TIMEOUT;
        }
    }
}

static void fill_status(ompi_status_public_t *st, const ompi_amd_status_t *s, int err)
{
    if (NULL == st) return;
    st->MPI_SOURCE = s->source;
    st->MPI_TAG = s->tag;
    st->MPI_ERROR = err;
    st->_cancelled = 0;
    st->_ucount = s->bytes;
}

/* ------------------------------------------------------------- requests */

static opal_mutex_t active_lock = OPAL_MUTEX_STATIC_INIT;
static mca_pml_rocm_request_t *active;
static int progress_registered;

/* finish a library request that completed: unstage, status, error */
static int finish(mca_pml_rocm_request_t *r, int rc, const ompi_amd_status_t *s)
{
    int err = rocm_err(rc);
    if (OMPI_SUCCESS == err && !r->is_send) err = unstage_recv(r, s->bytes);
    if (!r->is_send) fill_status(&r->super.req_status, s, err);
    else r->super.req_status.MPI_ERROR = err;
    (void) ompi_amd_p2p_free(r->lib);
    r->lib = NULL;
    stage_free(r);
    return err;
}

/* the saved PML completed a request of a device buffer: its status, the
 * received span back to the device; a persistent one keeps both for the
 * next start */
static void finish_inner(mca_pml_rocm_request_t *r)
{
    int err = r->inner->req_status.MPI_ERROR;
    if (OMPI_SUCCESS == err && !r->is_send) err = host_span_back(r, r->inner->req_status._ucount);
    r->super.req_status = r->inner->req_status;
    r->super.req_status.MPI_ERROR = err;
    if (r->super.req_persistent) {
        r->inner->req_state = OMPI_REQUEST_INACTIVE;
    } else {
        (void) ompi_request_free(&r->inner);
        r->inner = NULL;
        free(r->hspan);
        r->hspan = NULL;
    }
}

static int rocm_progress(void)
{
    mca_pml_rocm_request_t **pp, *done = NULL;
    int completed = 0;
    if (NULL == active) return 0;
    OPAL_THREAD_LOCK(&active_lock);
    pp = &active;
    while (NULL != *pp) {
        mca_pml_rocm_request_t *r = *pp;
        ompi_amd_status_t s = {0, 0, 0, 0};
        int fin = 0;
        if (NULL != r->inner) {  /* a device buffer on the saved PML */
            if (REQUEST_COMPLETE(r->inner)) {
                finish_inner(r);
                *pp = r->next_active;
                r->next_active = done;
                done = r;
            } else {
                pp = &r->next_active;
            }
            continue;
        }
        const int rc = ompi_amd_p2p_test(r->lib, &fin, &s);
        if (OMPI_AMD_SUCCESS != rc || fin) {
            (void) finish(r, rc, &s);
            *pp = r->next_active;
            r->next_active = done;
            done = r;
        } else {
            pp = &r->next_active;
        }
    }
    OPAL_THREAD_UNLOCK(&active_lock);
    while (NULL != done) {
        mca_pml_rocm_request_t *r = done;
        done = r->next_active;
        r->next_active = NULL;
        ompi_request_complete(&r->super, true);
        ++completed;
    }
    return completed;
}

int mca_pml_rocm_active_count(void)
{
    int n = 0;
    OPAL_THREAD_LOCK(&active_lock);
    for (mca_pml_rocm_request_t *r = active; NULL != r; r = r->next_active) ++n;
    OPAL_THREAD_UNLOCK(&active_lock);
    return n;
}

static void link_active(mca_pml_rocm_request_t *r)
{
    OPAL_THREAD_LOCK(&active_lock);
    r->next_active = active;
    active = r;
    if (!progress_registered) {
        progress_registered = 1;
        (void) opal_progress_register(rocm_progress);
    }
    OPAL_THREAD_UNLOCK(&active_lock);
}

static void unlink_active(mca_pml_rocm_request_t *r)
{
    mca_pml_rocm_request_t **pp;
    OPAL_THREAD_LOCK(&active_lock);
    for (pp = &active; NULL != *pp; pp = &(*pp)->next_active) {
        if (*pp == r) {
            *pp = r->next_active;
            break;
        }
    }
    OPAL_THREAD_UNLOCK(&active_lock);
    r->next_active = NULL;
}

/* post the request's operation on the library */
static int post(mca_pml_rocm_request_t *r)
{
    ompi_amd_comm_t *dev = mca_pml_rocm_comm_of(r->comm);
    int rc;
    if (NULL == dev) return OMPI_ERR_BAD_PARAM;
    rc = stage_for(r, r->is_send);
    if (OMPI_SUCCESS != rc) return rc;
    if (r->is_send) {
        rc = ompi_amd_isend(dev, lib_buf(r), r->bytes, r->peer, r->tag, r->mode, NULL, &r->lib);
    } else {
        rc = ompi_amd_irecv(dev, lib_buf(r), r->bytes,
                            MPI_ANY_SOURCE == r->peer ? OMPI_AMD_ANY_SOURCE : r->peer,
                            MPI_ANY_TAG == r->tag ? OMPI_AMD_ANY_TAG : r->tag, NULL, &r->lib);
    }
    if (OMPI_AMD_SUCCESS != rc) {
        stage_free(r);
        return rocm_err(rc);
    }
    r->super.req_complete = REQUEST_PENDING;
    r->super.req_state = OMPI_REQUEST_ACTIVE;
    r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
    link_active(r);
    return OMPI_SUCCESS;
}

/* MPI_Start / MPI_Startall of persistent requests (request.h:60-77) */
static int rocm_start_req(size_t count, ompi_request_t **requests)
{
    size_t i;
    for (i = 0; i < count; ++i) {
        mca_pml_rocm_request_t *r = (mca_pml_rocm_request_t *) requests[i];
        int rc;
        if (NULL == r) continue;
        if (OMPI_REQUEST_ACTIVE == r->super.req_state && !REQUEST_COMPLETE(&r->super))
            return OMPI_ERR_REQUEST;
        if (NULL != r->inner) {  /* the saved PML's request on the host span */
            rc = host_span(r);  /* this start's payload (a receive: its gap bytes, if whole) */
            if (OMPI_SUCCESS == rc) rc = r->inner->req_start(1, &r->inner);
            if (OMPI_SUCCESS != rc) return rc;
            r->super.req_complete = REQUEST_PENDING;
            r->super.req_state = OMPI_REQUEST_ACTIVE;
            r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
            link_active(r);
            continue;
        }
        rc = post(r);
        if (OMPI_SUCCESS != rc) return rc;
    }
    return OMPI_SUCCESS;
}

/* MPI_Request_free: an active transfer is waited for first (no time limit) */
static int rocm_free_req(ompi_request_t **rptr)
{
    mca_pml_rocm_request_t *r = (mca_pml_rocm_request_t *) *rptr;
    int rc = OMPI_SUCCESS;
    /* always: the oldest active request is the list's tail (next_active
     * NULL) and must leave the list before it is released */
    unlink_active(r);
    if (NULL != r->lib) {
        ompi_amd_status_t s = {0, 0, 0, 0};
        rc = finish(r, wait_lib(r->lib, &s), &s);
    }
    if (NULL != r->inner) {  /* the host span must outlive the saved PML's transfer */
        while (OMPI_REQUEST_ACTIVE == r->inner->req_state && !REQUEST_COMPLETE(r->inner)) opal_progress();
        (void) ompi_request_free(&r->inner);
        r->inner = NULL;
    }
    free(r->hspan);
    r->hspan = NULL;
    OMPI_REQUEST_FINI(&r->super);
    OBJ_RELEASE(r);
    *rptr = MPI_REQUEST_NULL;
    return rc;
}

static void rocm_request_construct(mca_pml_rocm_request_t *r)
{
    r->super.req_type = OMPI_REQUEST_PML;
    r->super.req_status._cancelled = 0;
    r->super.req_free = rocm_free_req;
    r->super.req_start = rocm_start_req;
    r->super.req_cancel = NULL;
    r->lib = NULL;
    r->stage = NULL;
    r->inner = NULL;
    r->hspan = NULL;
    r->next_active = NULL;
}

OBJ_CLASS_INSTANCE(mca_pml_rocm_request_t, ompi_request_t, rocm_request_construct, NULL);

static mca_pml_rocm_request_t *new_req(int is_send, void *buf, size_t count,
                                       struct ompi_datatype_t *dtype, int peer, int tag, int mode,
                                       struct ompi_communicator_t *comm, bool persistent)
{
    mca_pml_rocm_request_t *r = OBJ_NEW(mca_pml_rocm_request_t);
    if (NULL == r) return NULL;
    OMPI_REQUEST_INIT(&r->super, persistent);
    r->super.req_mpi_object.comm = comm;
    r->is_send = is_send;
    r->buf = buf;
    r->count = count;
    r->dtype = dtype;
    r->peer = peer;
    r->tag = tag;
    r->mode = mode;
    r->comm = comm;
    return r;
}

/* A device-buffer operation on the saved PML through the host span: an
 * active request of ours around the saved PML's (nonblocking), or a
 * persistent one whose starts refill the span and start it. */
static int saved_device_op(int is_send, void *buf, size_t count, struct ompi_datatype_t *dtype,
                           int peer, int tag, int mode, struct ompi_communicator_t *comm,
                           bool persistent, struct ompi_request_t **request)
{
    mca_pml_rocm_request_t *r = new_req(is_send, buf, count, dtype, peer, tag, mode, comm, persistent);
    int rc;
    if (NULL == r) return OMPI_ERR_OUT_OF_RESOURCE;
    rc = host_span(r);
    if (OMPI_SUCCESS == rc) {
        void *h = host_base(r);
        if (is_send)
            rc = persistent ? mca_pml_rocm_host.pml_isend_init(h, count, dtype, peer, tag,
                                                              (mca_pml_base_send_mode_t) mode, comm,
                                                              &r->inner)
                            : mca_pml_rocm_host.pml_isend(h, count, dtype, peer, tag,
                                                         (mca_pml_base_send_mode_t) mode, comm, &r->inner);
        else
            rc = persistent ? mca_pml_rocm_host.pml_irecv_init(h, count, dtype, peer, tag, comm, &r->inner)
                            : mca_pml_rocm_host.pml_irecv(h, count, dtype, peer, tag, comm, &r->inner);
    }
    if (OMPI_SUCCESS != rc) {  /* the saved PML refused: nothing of it to free */
        r->inner = NULL;
        free(r->hspan);
        r->hspan = NULL;
        OBJ_RELEASE(r);
        return rc;
    }
    if (!persistent) {
        r->super.req_complete = REQUEST_PENDING;
        r->super.req_state = OMPI_REQUEST_ACTIVE;
        r->super.req_status.MPI_ERROR = OMPI_SUCCESS;
        link_active(r);
    }
    *request = &r->super;
    return OMPI_SUCCESS;
}

/* ------------------------------------------------------------- pml entry points */

static int rocm_isend(const void *buf, size_t count, struct ompi_datatype_t *dtype, int dst, int tag,
                      mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm,
                      struct ompi_request_t **request)
{
    mca_pml_rocm_request_t *r;
    int rc;
    if (NULL == takes_buf(comm, tag, dst, buf, count)) {
        if (on_device(buf, count, dtype))
            return saved_device_op(1, (void *) buf, count, dtype, dst, tag, (int) mode, comm, false,
                                   request);
        return mca_pml_rocm_host.pml_isend(buf, count, dtype, dst, tag, mode, comm, request);
    }
    r = new_req(1, (void *) buf, count, dtype, dst, tag, (int) mode, comm, false);
    if (NULL == r) return OMPI_ERR_OUT_OF_RESOURCE;
    rc = post(r);
    if (OMPI_SUCCESS != rc) {
        OBJ_RELEASE(r);
        return rc;
    }
    *request = &r->super;
    return OMPI_SUCCESS;
}

static int rocm_irecv(void *buf, size_t count, struct ompi_datatype_t *dtype, int src, int tag,
                      struct ompi_communicator_t *comm, struct ompi_request_t **request)
{
    mca_pml_rocm_request_t *r;
    int rc;
    if (NULL == takes_buf(comm, tag, src, buf, count)) {
        if (on_device(buf, count, dtype))
            return saved_device_op(0, buf, count, dtype, src, tag, 0, comm, false, request);
        return mca_pml_rocm_host.pml_irecv(buf, count, dtype, src, tag, comm, request);
    }
    r = new_req(0, buf, count, dtype, src, tag, 0, comm, false);
    if (NULL == r) return OMPI_ERR_OUT_OF_RESOURCE;
    rc = post(r);
    if (OMPI_SUCCESS != rc) {
        OBJ_RELEASE(r);
        return rc;
    }
    *request = &r->super;
    return OMPI_SUCCESS;
}

static int rocm_isend_init(const void *buf, size_t count, struct ompi_datatype_t *dtype, int dst,
                           int tag, mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm,
                           struct ompi_request_t **request)
{
    mca_pml_rocm_request_t *r;
    if (NULL == takes_buf(comm, tag, dst, buf, count)) {
        if (on_device(buf, count, dtype))
            return saved_device_op(1, (void *) buf, count, dtype, dst, tag, (int) mode, comm, true,
                                   request);
        return mca_pml_rocm_host.pml_isend_init(buf, count, dtype, dst, tag, mode, comm, request);
    }
    r = new_req(1, (void *) buf, count, dtype, dst, tag, (int) mode, comm, true);
    if (NULL == r) return OMPI_ERR_OUT_OF_RESOURCE;
    *request = &r->super;
    return OMPI_SUCCESS;
}

static int rocm_irecv_init(void *buf, size_t count, struct ompi_datatype_t *dtype, int src, int tag,
                           struct ompi_communicator_t *comm, struct ompi_request_t **request)
{
    mca_pml_rocm_request_t *r;
    if (NULL == takes_buf(comm, tag, src, buf, count)) {
        if (on_device(buf, count, dtype))
            return saved_device_op(0, buf, count, dtype, src, tag, 0, comm, true, request);
        return mca_pml_rocm_host.pml_irecv_init(buf, count, dtype, src, tag, comm, request);
    }
    r = new_req(0, buf, count, dtype, src, tag, 0, comm, true);
    if (NULL == r) return OMPI_ERR_OUT_OF_RESOURCE;
    *request = &r->super;
    return OMPI_SUCCESS;
}

/* pml_start: requests of this component start themselves; others go to the
 * saved PML (a mixed array is split in order) */
static int rocm_start(size_t count, ompi_request_t **requests)
{
    size_t i;
    for (i = 0; i < count; ++i) {
        ompi_request_t *q = requests[i];
        int rc;
        if (NULL == q) continue;
        rc = q->req_start == rocm_start_req ? rocm_start_req(1, &requests[i])
                                           : mca_pml_rocm_host.pml_start(1, &requests[i]);
        if (OMPI_SUCCESS != rc) return rc;
    }
    return OMPI_SUCCESS;
}

static int rocm_send(const void *buf, size_t count, struct ompi_datatype_t *dtype, int dst, int tag,
                     mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm)
{
    mca_pml_rocm_request_t r;
    ompi_amd_comm_t *dev = takes_buf(comm, tag, dst, buf, count);
    ompi_amd_p2p_request_t *lib = NULL;
    ompi_amd_status_t s = {0, 0, 0, 0};
    int rc;
    if (NULL == dev && on_device(buf, count, dtype)) {  /* the saved PML on a host copy */
        memset(&r, 0, sizeof(r));
        r.is_send = 1;
        r.buf = (void *) buf;
        r.count = count;
        r.dtype = dtype;
        rc = host_span(&r);
        if (OMPI_SUCCESS == rc)
            rc = mca_pml_rocm_host.pml_send(host_base(&r), count, dtype, dst, tag, mode, comm);
        free(r.hspan);
        return rc;
    }
    if (NULL == dev) return mca_pml_rocm_host.pml_send(buf, count, dtype, dst, tag, mode, comm);
    memset(&r, 0, sizeof(r));
    r.buf = (void *) buf;
    r.count = count;
    r.dtype = dtype;
    rc = stage_for(&r, 1);
    if (OMPI_SUCCESS != rc) return rc;
    rc = rocm_err(ompi_amd_isend(dev, lib_buf(&r), r.bytes, dst, tag, (int) mode, NULL, &lib));
    if (OMPI_SUCCESS == rc) {
        rc = rocm_err(wait_lib(lib, &s));
        (void) ompi_amd_p2p_free(lib);
    }
    stage_free(&r);
    return rc;
}

static int rocm_recv(void *buf, size_t count, struct ompi_datatype_t *dtype, int src, int tag,
                     struct ompi_communicator_t *comm, ompi_status_public_t *status)
{
    mca_pml_rocm_request_t r;
    ompi_amd_status_t s = {0, 0, 0, 0};
    ompi_amd_comm_t *dev = takes_buf(comm, tag, src, buf, count);
    ompi_amd_p2p_request_t *lib = NULL;
    int rc;
    if (NULL == dev && on_device(buf, count, dtype)) {  /* the saved PML on a host copy */
        memset(&r, 0, sizeof(r));
        r.buf = buf;
        r.count = count;
        r.dtype = dtype;
        ompi_status_public_t own, *st = NULL != status ? status : &own;  /* MPI_STATUS_IGNORE */
        rc = host_span(&r);
        if (OMPI_SUCCESS == rc)
            rc = mca_pml_rocm_host.pml_recv(host_base(&r), count, dtype, src, tag, comm, st);
        if (OMPI_SUCCESS == rc) rc = host_span_back(&r, st->_ucount);
        free(r.hspan);
        return rc;
    }
    if (NULL == dev) return mca_pml_rocm_host.pml_recv(buf, count, dtype, src, tag, comm, status);
    memset(&r, 0, sizeof(r));
    r.buf = buf;
    r.count = count;
    r.dtype = dtype;
    rc = stage_for(&r, 0);
    if (OMPI_SUCCESS != rc) return rc;
    rc = rocm_err(ompi_amd_irecv(dev, lib_buf(&r), r.bytes,
                                 MPI_ANY_SOURCE == src ? OMPI_AMD_ANY_SOURCE : src,
                                 MPI_ANY_TAG == tag ? OMPI_AMD_ANY_TAG : tag, NULL, &lib));
    if (OMPI_SUCCESS == rc) {
        rc = rocm_err(wait_lib(lib, &s));
        (void) ompi_amd_p2p_free(lib);
    }
    if (OMPI_SUCCESS == rc) rc = unstage_recv(&r, s.bytes);
    stage_free(&r);
    fill_status(status, &s, rc);
    return rc;
}

/* With pml_rocm_host_path a message may arrive on either engine: a probe
 * asks the library first, then the saved PML. */
static int rocm_iprobe(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                       ompi_status_public_t *status)
{
    ompi_amd_status_t s = {0, 0, 0, 0};
    ompi_amd_comm_t *dev = takes(comm, tag, src);
    int rc;
    if (NULL == dev) return mca_pml_rocm_host.pml_iprobe(src, tag, comm, matched, status);
    rc = rocm_err(ompi_amd_iprobe(dev, MPI_ANY_SOURCE == src ? OMPI_AMD_ANY_SOURCE : src,
                                  MPI_ANY_TAG == tag ? OMPI_AMD_ANY_TAG : tag, matched, &s));
    if (OMPI_SUCCESS == rc && *matched) fill_status(status, &s, OMPI_SUCCESS);
    if (OMPI_SUCCESS == rc && !*matched && mca_pml_rocm_component.host_path)
        return mca_pml_rocm_host.pml_iprobe(src, tag, comm, matched, status);
    return rc;
}

/* no time limit: iprobe + opal_progress until a message is there */
static int rocm_probe(int src, int tag, struct ompi_communicator_t *comm, ompi_status_public_t *status)
{
    if (NULL == takes(comm, tag, src)) return mca_pml_rocm_host.pml_probe(src, tag, comm, status);
    for (;;) {
        int matched = 0;
        const int rc = rocm_iprobe(src, tag, comm, &matched, status);
        if (OMPI_SUCCESS != rc || matched) return rc;
        opal_progress();
    }
}

/* matched probes of library traffic are not provided */
static int rocm_improbe(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                        struct ompi_message_t **message, ompi_status_public_t *status)
{
    if (NULL != takes(comm, tag, src) && !mca_pml_rocm_component.host_path)
        return OMPI_ERR_NOT_SUPPORTED;
    return mca_pml_rocm_host.pml_improbe(src, tag, comm, matched, message, status);
}

static int rocm_mprobe(int src, int tag, struct ompi_communicator_t *comm,
                       struct ompi_message_t **message, ompi_status_public_t *status)
{
    if (NULL != takes(comm, tag, src) && !mca_pml_rocm_component.host_path)
        return OMPI_ERR_NOT_SUPPORTED;
    return mca_pml_rocm_host.pml_mprobe(src, tag, comm, message, status);
}

/* close: after the PML base selected the real PML — save it, interpose */
static int rocm_close(void)
{
    if (!mca_pml_rocm_component.enable || mca_pml_rocm_installed || NULL == mca_pml.pml_isend)
        return OMPI_SUCCESS;
    mca_pml_rocm_host = mca_pml;
    mca_pml.pml_add_comm = rocm_add_comm;
    mca_pml.pml_del_comm = rocm_del_comm;
    mca_pml.pml_isend = rocm_isend;
    mca_pml.pml_send = rocm_send;
    mca_pml.pml_irecv = rocm_irecv;
    mca_pml.pml_recv = rocm_recv;
    mca_pml.pml_isend_init = rocm_isend_init;
    mca_pml.pml_irecv_init = rocm_irecv_init;
    mca_pml.pml_start = rocm_start;
    mca_pml.pml_iprobe = rocm_iprobe;
    mca_pml.pml_probe = rocm_probe;
    mca_pml.pml_improbe = rocm_improbe;
    mca_pml.pml_mprobe = rocm_mprobe;
    mca_pml_rocm_installed = 1;
    return OMPI_SUCCESS;
}
