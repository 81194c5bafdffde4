/*
 * TEST HARNESS ONLY.  The previously selected coll functions ("tuned",
 * libnbc) that coll/rocm saves at enable time and delegates to, played by
 * stand-ins that really run the collective on the host: each rank packs its
 * contribution into a POSIX-shm exchange (one slot per rank, a
 * process-shared barrier), every rank combines what it needs from the slots
 * and writes its result into its own buffers — read and written by the
 * CPU, as coll/tuned + op/base do.  Every stand-in first checks that none
 * of its buffers is device memory: a device pointer reaching a saved
 * function fails the run (coll/tuned would walk it from the host).
 *
 * The reduction is a fixed linear fold in rank order through the oracle's
 * op/base restatement (orc_op_2buff; long double by hand — op/base's
 * loop, which no device kernel replaces).  harness_expect_* give the test
 * the same host computation to compare the glue's results with.
 *
 * Nonblocking stand-ins run at the call and hand back a request that
 * completes after two opal_progress polls, so a glue that copies staged
 * outputs back before completion would be caught; persistent stand-ins keep
 * their arguments and run at every start.
 */
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include "mpi.h"
#include "ompi/communicator/communicator.h"
#include "ompi/constants.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/op/op.h"
#include "opal/runtime/opal_progress.h"
#include "../../oracle/oracle.h"
#include "coll_saved.h"
#include "ompi_amd.h"
#include "ompi_amd_coll.h"

int tuned_calls;
int t_sdev = -1, t_rdev = -1;

#define HX_SLOT ((size_t) 8 << 20)

struct hx_hdr {
    volatile int arrive;
    volatile int gen;
    char pad[56];
};
static struct hx_hdr *hx;
static char *hx_slots;
static int hx_rank, hx_size;
static char hx_name[96];

static void die(const char *what)
{
    fprintf(stderr, "FAIL rank %d saved stand-in: %s\n", hx_rank, what);
    exit(1);
}

void harness_saved_init(const char *segment, int rank, int size)
{
    const size_t bytes = sizeof(struct hx_hdr) + HX_SLOT * (size_t) size;
    int fd;
    void *p;
    hx_rank = rank;
    hx_size = size;
    snprintf(hx_name, sizeof(hx_name), "/coll_saved_%s", segment);
    fd = shm_open(hx_name, O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t) bytes) != 0) die("shm_open");
    p = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (MAP_FAILED == p) die("mmap");
    hx = (struct hx_hdr *) p;
    hx_slots = (char *) p + sizeof(struct hx_hdr);
}

/* sense-reversing barrier over the segment's header */
static void hx_barrier(void)
{
    const int gen = __atomic_load_n(&hx->gen, __ATOMIC_ACQUIRE);
    if (__atomic_add_fetch(&hx->arrive, 1, __ATOMIC_ACQ_REL) == hx_size) {
        __atomic_store_n(&hx->arrive, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&hx->gen, gen + 1, __ATOMIC_RELEASE);
    } else {
        while (__atomic_load_n(&hx->gen, __ATOMIC_ACQUIRE) == gen) sched_yield();
    }
}

void harness_saved_fini(void)
{
    hx_barrier();
    if (0 == hx_rank) shm_unlink(hx_name);
}

static const char *slot(int r) { return hx_slots + HX_SLOT * (size_t) r; }

/* this rank's contribution into its slot; after the call every slot holds
 * its rank's bytes until hx_done() */
static void hx_put(const void *mine, size_t bytes)
{
    if (bytes > HX_SLOT) die("exchange slot too small");
    hx_barrier();  /* the previous exchange's readers are done */
    if (bytes) memcpy(hx_slots + HX_SLOT * (size_t) hx_rank, mine, bytes);
    hx_barrier();
}

/* ------------------------------------------------------------ datatypes */

size_t harness_esize(const ompi_datatype_t *d) { return d->size; }

/* byte offset of element i in a buffer of the stand-in layout */
static size_t eoff(const ompi_datatype_t *d, size_t i) { return i * (d->contiguous ? 1 : 2) * d->size; }

static void pack(const ompi_datatype_t *d, const void *buf, size_t first, size_t count, char *out)
{
    for (size_t i = 0; i < count; ++i)
        memcpy(out + i * d->size, (const char *) buf + eoff(d, first + i), d->size);
}

static void unpack(const ompi_datatype_t *d, const char *in, size_t first, size_t count, void *buf)
{
    for (size_t i = 0; i < count; ++i)
        memcpy((char *) buf + eoff(d, first + i), in + i * d->size, d->size);
}

static void host_only(const void *p)
{
    if (NULL == p || MPI_IN_PLACE == p) return;
    if (ompi_amd_is_device_pointer(p)) die("a saved function was handed device memory");
}

/* inout = inout (op) in, count elements of the element type */
void harness_fold(int op, int type, const void *in, void *inout, size_t count)
{
    if (HARNESS_T_LONG_DOUBLE == type) {
        const long double *a = (const long double *) in;
        long double *b = (long double *) inout;
        for (size_t i = 0; i < count; ++i) {
            switch (op) {
            case ORC_OP_SUM: b[i] += a[i]; break;
            case ORC_OP_PROD: b[i] *= a[i]; break;
            case ORC_OP_MAX: b[i] = a[i] > b[i] ? a[i] : b[i]; break;
            case ORC_OP_MIN: b[i] = a[i] < b[i] ? a[i] : b[i]; break;
            default: die("long double op");
            }
        }
        return;
    }
    if (orc_op_2buff(op, type, in, inout, count) != 0) die("oracle op");
}

/* out = x[first] (op) ... (op) x[last - 1] in rank order, count packed
 * elements starting at element `at` of each packed input */
static void combine(int op, const ompi_datatype_t *d, const char *const *x, int first, int last,
                    size_t at, size_t count, char *out)
{
    const size_t es = d->size;
    memcpy(out, x[first] + at * es, count * es);
    for (int r = first + 1; r < last; ++r) harness_fold(op, d->id, x[r] + at * es, out, count);
}

static const char *const *slots_of(void)
{
    static const char *s[OMPI_AMD_MAX_RANKS];
    for (int r = 0; r < hx_size; ++r) s[r] = slot(r);
    return s;
}

/* ------------------------------------------------ the host collectives */

static int h_allreduce(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o)
{
    const size_t n = (size_t) c, es = d->size;
    char *mine = malloc(n * es + 1), *res = malloc(n * es + 1);
    pack(d, MPI_IN_PLACE == s ? r : s, 0, n, mine);
    hx_put(mine, n * es);
    combine(o->o_f_to_c_index, d, slots_of(), 0, hx_size, 0, n, res);
    unpack(d, res, 0, n, r);
    free(mine);
    free(res);
    return OMPI_SUCCESS;
}

static int h_reduce(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o, int root)
{
    const size_t n = (size_t) c, es = d->size;
    char *mine = malloc(n * es + 1), *res = malloc(n * es + 1);
    pack(d, MPI_IN_PLACE == s ? r : s, 0, n, mine);
    hx_put(mine, n * es);
    if (hx_rank == root) {
        combine(o->o_f_to_c_index, d, slots_of(), 0, hx_size, 0, n, res);
        unpack(d, res, 0, n, r);
    }
    free(mine);
    free(res);
    return OMPI_SUCCESS;
}

static int h_scan(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o, int exclusive)
{
    const size_t n = (size_t) c, es = d->size;
    char *mine = malloc(n * es + 1), *res = malloc(n * es + 1);
    pack(d, MPI_IN_PLACE == s ? r : s, 0, n, mine);
    hx_put(mine, n * es);
    if (!(exclusive && 0 == hx_rank)) {
        combine(o->o_f_to_c_index, d, slots_of(), 0, exclusive ? hx_rank : hx_rank + 1, 0, n, res);
        unpack(d, res, 0, n, r);
    }
    free(mine);
    free(res);
    return OMPI_SUCCESS;
}

/* reduce_scatter with per-rank counts; rsb passes equal ones */
static int h_rs(const void *s, void *r, const int *rc, ompi_datatype_t *d, ompi_op_t *o)
{
    size_t total = 0, at = 0;
    const size_t es = d->size;
    char *mine, *res;
    for (int k = 0; k < hx_size; ++k) total += (size_t) rc[k];
    for (int k = 0; k < hx_rank; ++k) at += (size_t) rc[k];
    mine = malloc(total * es + 1);
    res = malloc((size_t) rc[hx_rank] * es + 1);
    pack(d, MPI_IN_PLACE == s ? r : s, 0, total, mine);
    hx_put(mine, total * es);
    combine(o->o_f_to_c_index, d, slots_of(), 0, hx_size, at, (size_t) rc[hx_rank], res);
    unpack(d, res, 0, (size_t) rc[hx_rank], r);
    free(mine);
    free(res);
    return OMPI_SUCCESS;
}

static int h_rsb(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o)
{
    int rc[OMPI_AMD_MAX_RANKS];
    for (int k = 0; k < hx_size; ++k) rc[k] = c;
    return h_rs(s, r, rc, d, o);
}

static int h_allgather(const void *s, int sc, ompi_datatype_t *sd, void *r, int rcount,
                       ompi_datatype_t *rd)
{
    const size_t bytes = (size_t) rcount * rd->size;
    char *mine = malloc(bytes + 1);
    if (MPI_IN_PLACE == s) pack(rd, r, (size_t) rcount * (size_t) hx_rank, (size_t) rcount, mine);
    else if ((size_t) sc * sd->size != bytes) die("allgather signature");
    else pack(sd, s, 0, (size_t) sc, mine);
    hx_put(mine, bytes);
    for (int k = 0; k < hx_size; ++k) unpack(rd, slot(k), (size_t) rcount * (size_t) k, (size_t) rcount, r);
    free(mine);
    return OMPI_SUCCESS;
}

static int h_bcast(void *b, int c, ompi_datatype_t *d, int root)
{
    const size_t bytes = (size_t) c * d->size;
    char *mine = calloc(bytes + 1, 1);
    if (hx_rank == root) pack(d, b, 0, (size_t) c, mine);
    hx_put(mine, hx_rank == root ? bytes : 0);
    if (hx_rank != root) unpack(d, slot(root), 0, (size_t) c, b);
    free(mine);
    return OMPI_SUCCESS;
}

/* --------------------------------------------------------- requests */

enum { K_ALLREDUCE, K_REDUCE, K_SCAN, K_EXSCAN, K_RS, K_RSB, K_ALLGATHER, K_BCAST };

typedef struct h_req {
    ompi_request_t super;
    int kind;
    const void *s;
    void *r;
    int c, sc, root;
    const int *rcounts;
    int rc_copy[OMPI_AMD_MAX_RANKS];
    ompi_datatype_t *d, *sd;
    ompi_op_t *o;
    int polls;
    struct h_req *next;
} h_req;

static h_req *h_active;
int harness_saved_live;  /* stand-in requests not yet freed */

static int h_run(h_req *q)
{
    switch (q->kind) {
    case K_ALLREDUCE: return h_allreduce(q->s, q->r, q->c, q->d, q->o);
    case K_REDUCE: return h_reduce(q->s, q->r, q->c, q->d, q->o, q->root);
    case K_SCAN: return h_scan(q->s, q->r, q->c, q->d, q->o, 0);
    case K_EXSCAN: return h_scan(q->s, q->r, q->c, q->d, q->o, 1);
    case K_RS: return h_rs(q->s, q->r, q->rc_copy, q->d, q->o);
    case K_RSB: return h_rsb(q->s, q->r, q->c, q->d, q->o);
    case K_ALLGATHER: return h_allgather(q->s, q->sc, q->sd, q->r, q->c, q->d);
    case K_BCAST: return h_bcast(q->r, q->c, q->d, q->root);
    }
    return OMPI_ERROR;
}

/* opal_progress: a running stand-in request completes at its second poll */
static int h_progress(void)
{
    int n = 0;
    for (h_req **pp = &h_active; NULL != *pp;) {
        h_req *q = *pp;
        if (--q->polls <= 0) {
            *pp = q->next;
            ompi_request_complete(&q->super, true);
            ++n;
        } else {
            pp = &q->next;
        }
    }
    return n;
}

static void h_launch(h_req *q)
{
    q->super.req_status.MPI_ERROR = h_run(q);
    q->super.req_complete = REQUEST_PENDING;
    q->super.req_state = OMPI_REQUEST_ACTIVE;
    q->polls = 2;
    q->next = h_active;
    h_active = q;
    (void) opal_progress_register(h_progress);
}

static int h_start(size_t count, ompi_request_t **reqs)
{
    for (size_t i = 0; i < count; ++i) h_launch((h_req *) reqs[i]);
    return OMPI_SUCCESS;
}

static int h_free(ompi_request_t **rq)
{
    h_req *q = (h_req *) *rq;
    if (!REQUEST_COMPLETE(&q->super)) die("stand-in request freed before it completed");
    --harness_saved_live;
    free(q);
    *rq = MPI_REQUEST_NULL;
    return OMPI_SUCCESS;
}

static h_req *h_new(int kind, int persistent)
{
    h_req *q = calloc(1, sizeof(*q));
    OMPI_REQUEST_INIT(&q->super, persistent);
    q->super.req_type = OMPI_REQUEST_COLL;
    q->super.req_start = h_start;
    q->super.req_free = h_free;
    q->kind = kind;
    ++harness_saved_live;
    return q;
}

int harness_is_saved_request(const ompi_request_t *r)
{
    return NULL != r && h_free == r->req_free;
}

/* a nonblocking stand-in: run now, complete from progress */
static int h_post(h_req *q, ompi_request_t **req)
{
    h_launch(q);
    *req = &q->super;
    return OMPI_SUCCESS;
}

/* ------------------------------------------- the stand-ins ("tuned") */

#define HOST2(a, b) do { tuned_calls++; host_only(a); host_only(b); } while (0)

static int t_allreduce(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                       ompi_communicator_t *cm, mca_coll_base_module_t *m)
{
    HOST2(s, r);
    t_sdev = MPI_IN_PLACE == s ? -1 : ompi_amd_is_device_pointer(s);
    t_rdev = ompi_amd_is_device_pointer(r);
    return h_allreduce(s, r, c, d, o);
}
static int t_reduce(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o, int root,
                    ompi_communicator_t *cm, mca_coll_base_module_t *m)
{ HOST2(s, cm->rank == root ? r : NULL); return h_reduce(s, r, c, d, o, root); }
/* a reduce_scatter rbuf with no elements for this rank is never touched */
#define RS_RBUF(s, r, c, cm) (MPI_IN_PLACE == (s) || (c)[(cm)->rank] > 0 ? (r) : NULL)
static int t_rs(const void *s, void *r, const int *c, ompi_datatype_t *d, ompi_op_t *o,
                ompi_communicator_t *cm, mca_coll_base_module_t *m)
{ HOST2(s, RS_RBUF(s, r, c, cm)); return h_rs(s, r, c, d, o); }
static int t_rsb(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                 ompi_communicator_t *cm, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_rsb(s, r, c, d, o); }
static int t_scan(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                  ompi_communicator_t *cm, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_scan(s, r, c, d, o, 0); }
static int t_exscan(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                    ompi_communicator_t *cm, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_scan(s, r, c, d, o, 1); }
static int t_allgather(const void *s, int sc, ompi_datatype_t *sd, void *r, int rc,
                       ompi_datatype_t *rd, ompi_communicator_t *cm, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_allgather(s, sc, sd, r, rc, rd); }
static int t_bcast(void *b, int c, ompi_datatype_t *d, int root, ompi_communicator_t *cm,
                   mca_coll_base_module_t *m)
{ HOST2(b, NULL); return h_bcast(b, c, d, root); }

/* request-building stand-ins: fill an h_req with the call's arguments */
static h_req *h_args(int kind, int persistent, const void *s, void *r, int c, ompi_datatype_t *d,
                     ompi_op_t *o, int root)
{
    h_req *q = h_new(kind, persistent);
    q->s = s;
    q->r = r;
    q->c = c;
    q->d = d;
    q->o = o;
    q->root = root;
    return q;
}

static int t_iallreduce(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                        ompi_communicator_t *cm, ompi_request_t **req, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_post(h_args(K_ALLREDUCE, 0, s, r, c, d, o, 0), req); }
static int t_ireduce(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o, int root,
                     ompi_communicator_t *cm, ompi_request_t **req, mca_coll_base_module_t *m)
{ HOST2(s, cm->rank == root ? r : NULL); return h_post(h_args(K_REDUCE, 0, s, r, c, d, o, root), req); }
static int t_iscan(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                   ompi_communicator_t *cm, ompi_request_t **req, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_post(h_args(K_SCAN, 0, s, r, c, d, o, 0), req); }
static int t_iexscan(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                     ompi_communicator_t *cm, ompi_request_t **req, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_post(h_args(K_EXSCAN, 0, s, r, c, d, o, 0), req); }
static int t_irsb(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                  ompi_communicator_t *cm, ompi_request_t **req, mca_coll_base_module_t *m)
{ HOST2(s, r); return h_post(h_args(K_RSB, 0, s, r, c, d, o, 0), req); }
static int t_irs(const void *s, void *r, const int *c, ompi_datatype_t *d, ompi_op_t *o,
                 ompi_communicator_t *cm, ompi_request_t **req, mca_coll_base_module_t *m)
{
    h_req *q;
    HOST2(s, RS_RBUF(s, r, c, cm));
    q = h_args(K_RS, 0, s, r, 0, d, o, 0);
    memcpy(q->rc_copy, c, sizeof(int) * (size_t) cm->size);
    return h_post(q, req);
}
static int t_iallgather(const void *s, int sc, ompi_datatype_t *sd, void *r, int rc,
                        ompi_datatype_t *rd, ompi_communicator_t *cm, ompi_request_t **req,
                        mca_coll_base_module_t *m)
{
    h_req *q;
    HOST2(s, r);
    q = h_args(K_ALLGATHER, 0, s, r, rc, rd, NULL, 0);
    q->sc = sc;
    q->sd = sd;
    return h_post(q, req);
}
static int t_ibcast(void *b, int c, ompi_datatype_t *d, int root, ompi_communicator_t *cm,
                    ompi_request_t **req, mca_coll_base_module_t *m)
{ HOST2(b, NULL); return h_post(h_args(K_BCAST, 0, NULL, b, c, d, NULL, root), req); }

/* persistent: nothing runs at init; every start runs the collective */
static int h_init(h_req *q, ompi_request_t **req)
{
    *req = &q->super;
    return OMPI_SUCCESS;
}
static int t_ar_init(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                     ompi_communicator_t *cm, struct ompi_info_t *info, ompi_request_t **req,
                     mca_coll_base_module_t *m)
{ HOST2(s, r); return h_init(h_args(K_ALLREDUCE, 1, s, r, c, d, o, 0), req); }
static int t_red_init(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o, int root,
                      ompi_communicator_t *cm, struct ompi_info_t *info, ompi_request_t **req,
                      mca_coll_base_module_t *m)
{ HOST2(s, cm->rank == root ? r : NULL); return h_init(h_args(K_REDUCE, 1, s, r, c, d, o, root), req); }
static int t_scan_init(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                       ompi_communicator_t *cm, struct ompi_info_t *info, ompi_request_t **req,
                       mca_coll_base_module_t *m)
{ HOST2(s, r); return h_init(h_args(K_SCAN, 1, s, r, c, d, o, 0), req); }
static int t_exscan_init(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                         ompi_communicator_t *cm, struct ompi_info_t *info, ompi_request_t **req,
                         mca_coll_base_module_t *m)
{ HOST2(s, r); return h_init(h_args(K_EXSCAN, 1, s, r, c, d, o, 0), req); }
static int t_rsb_init(const void *s, void *r, int c, ompi_datatype_t *d, ompi_op_t *o,
                      ompi_communicator_t *cm, struct ompi_info_t *info, ompi_request_t **req,
                      mca_coll_base_module_t *m)
{ HOST2(s, r); return h_init(h_args(K_RSB, 1, s, r, c, d, o, 0), req); }
static int t_rs_init(const void *s, void *r, const int *c, ompi_datatype_t *d, ompi_op_t *o,
                     ompi_communicator_t *cm, struct ompi_info_t *info, ompi_request_t **req,
                     mca_coll_base_module_t *m)
{
    h_req *q;
    HOST2(s, RS_RBUF(s, r, c, cm));
    q = h_args(K_RS, 1, s, r, 0, d, o, 0);
    memcpy(q->rc_copy, c, sizeof(int) * (size_t) cm->size);
    return h_init(q, req);
}
static int t_ag_init(const void *s, int sc, ompi_datatype_t *sd, void *r, int rc,
                     ompi_datatype_t *rd, ompi_communicator_t *cm, struct ompi_info_t *info,
                     ompi_request_t **req, mca_coll_base_module_t *m)
{
    h_req *q;
    HOST2(s, r);
    q = h_args(K_ALLGATHER, 1, s, r, rc, rd, NULL, 0);
    q->sc = sc;
    q->sd = sd;
    return h_init(q, req);
}
static int t_bc_init(void *b, int c, ompi_datatype_t *d, int root, ompi_communicator_t *cm,
                     struct ompi_info_t *info, ompi_request_t **req, mca_coll_base_module_t *m)
{ HOST2(b, NULL); return h_init(h_args(K_BCAST, 1, NULL, b, c, d, NULL, root), req); }

void harness_fill_tuned(mca_coll_base_comm_coll_t *t, mca_coll_base_module_t *tm)
{
    memset(t, 0, sizeof(*t));
#define SET(fn, f) do { t->coll_##fn = f; t->coll_##fn##_module = tm; OBJ_RETAIN(tm); } while (0)
    SET(allreduce, t_allreduce);
    SET(reduce, t_reduce);
    SET(reduce_scatter, t_rs);
    SET(reduce_scatter_block, t_rsb);
    SET(scan, t_scan);
    SET(exscan, t_exscan);
    SET(allgather, t_allgather);
    SET(bcast, t_bcast);
    SET(iallreduce, t_iallreduce);
    SET(allreduce_init, t_ar_init);
    SET(iallgather, t_iallgather);
    SET(ibcast, t_ibcast);
    SET(ireduce_scatter_block, t_irsb);
    SET(ireduce, t_ireduce);
    SET(iscan, t_iscan);
    SET(iexscan, t_iexscan);
    SET(ireduce_scatter, t_irs);
    SET(reduce_scatter_block_init, t_rsb_init);
    SET(allgather_init, t_ag_init);
    SET(bcast_init, t_bc_init);
    SET(reduce_init, t_red_init);
    SET(reduce_scatter_init, t_rs_init);
    SET(scan_init, t_scan_init);
    SET(exscan_init, t_exscan_init);
#undef SET
}

/* --------------------------------------------- expectations for tests */

/* the host result the stand-ins give rank `me`, from every rank's packed
 * input x[r] (count elements): allreduce / reduce (root) / scan / exscan */
void harness_expect_reduction(int kind, int op, const ompi_datatype_t *d, const char *const *x,
                              int n, int me, size_t count, char *out)
{
    switch (kind) {
    case HARNESS_ALLREDUCE: combine(op, d, x, 0, n, 0, count, out); break;
    case HARNESS_SCAN: combine(op, d, x, 0, me + 1, 0, count, out); break;
    case HARNESS_EXSCAN: if (me > 0) combine(op, d, x, 0, me, 0, count, out); break;
    }
}

/* reduce_scatter: rank me's block (rcounts) of the combined vector */
void harness_expect_rs(int op, const ompi_datatype_t *d, const char *const *x, int n, int me,
                       const int *rcounts, char *out)
{
    size_t at = 0;
    for (int k = 0; k < me; ++k) at += (size_t) rcounts[k];
    combine(op, d, x, 0, n, at, (size_t) rcounts[me], out);
}
