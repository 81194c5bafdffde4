/*
 * TEST HARNESS ONLY.  One rank of a multi-process run that drives
 * ompi_amd/mca/coll/rocm/coll_rocm_module.c the way the coll framework does
 * (coll_base_comm_select.c:158-232): the previously selected functions are
 * played by counting stand-ins ("tuned"), the component is queried, the
 * module enabled (it saves and retains the stand-ins) and its functions
 * installed in the communicator's table; then every collective is called
 * through that table.
 *
 *   CPU (HARNESS_GPU=0): init_query refuses without a device; comm_query
 *   accepts only node-local intra-communicators of 2..16 ranks.
 *   GPU (HARNESS_GPU=1): device buffers run the library and match the CPU
 *   oracle bit for bit; host buffers, mixed residency across ranks and
 *   non-intrinsic ops go to the saved functions on every rank.  A
 *   persistent allreduce request is started and completed through
 *   opal_progress the way MPI_Start / MPI_Wait drive it, and so are
 *   nonblocking allreduce requests.
 *
 * usage: coll_harness <segment-name> <rank> <size>; prints "ok" / "ok gpu".
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mpi.h"
#include "ompi/communicator/communicator.h"
#include "ompi/constants.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/op/op.h"
#include "ompi/runtime/ompi_rte.h"
#include "opal/runtime/opal_progress.h"
#include "../../oracle/oracle.h"
#include "coll_rocm.h"
#include "coll_saved.h"
#include "ompi_amd.h"

extern mca_coll_rocm_component_t mca_coll_rocm_component;
extern int harness_dev_alloc_copy(void **d, const void *h, size_t bytes);
extern int harness_dev_copy_in(void *d, const void *h, size_t bytes);
extern int harness_dev_copy_back(void *h, const void *d, size_t bytes);
extern int harness_dev_free(void *d);

OBJ_CLASS_INSTANCE(mca_coll_base_module_t, opal_object_t, NULL, NULL);

/* ompi_request_default_wait for a persistent request (request/req_wait.c) */
static void harness_wait(ompi_request_t *req)
{
    while (!REQUEST_COMPLETE(req)) opal_progress();
    req->req_state = OMPI_REQUEST_INACTIVE;
}
harness_proc_name_t harness_proc_name = {4242, 0};
int ompi_op_ddt_map[64];

#define CHECK(c, ...)                                                   \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "FAIL rank %d %s:%d: ", g_rank, __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                               \
            fprintf(stderr, "\n");                                      \
            exit(1);                                                    \
        }                                                               \
    } while (0)

static int g_rank, g_size;
struct ompi_datatype_t harness_mpi_byte = {ORC_T_BYTE, 1, 1, 1};

/* coll_base_comm_select.c:210-232: install what the module provides */
static void install(mca_coll_base_comm_coll_t *t, mca_coll_base_module_t *m)
{
#define INST(fn) if (m->coll_##fn) { OBJ_RELEASE(t->coll_##fn##_module); t->coll_##fn = m->coll_##fn; \
                                      t->coll_##fn##_module = m; OBJ_RETAIN(m); }
    INST(allreduce) INST(reduce) INST(reduce_scatter) INST(reduce_scatter_block) INST(scan)
    INST(exscan)
    INST(allgather) INST(bcast) INST(iallreduce) INST(allreduce_init)
    INST(iallgather) INST(ibcast) INST(ireduce_scatter_block)
    INST(ireduce) INST(iscan) INST(iexscan) INST(ireduce_scatter)
    INST(reduce_scatter_block_init) INST(allgather_init) INST(bcast_init)
    INST(reduce_init) INST(reduce_scatter_init) INST(scan_init) INST(exscan_init)
#undef INST
}

static void release_table(mca_coll_base_comm_coll_t *t)
{
    OBJ_RELEASE(t->coll_allreduce_module);
    OBJ_RELEASE(t->coll_reduce_module);
    OBJ_RELEASE(t->coll_reduce_scatter_module);
    OBJ_RELEASE(t->coll_reduce_scatter_block_module);
    OBJ_RELEASE(t->coll_scan_module);
    OBJ_RELEASE(t->coll_exscan_module);
    OBJ_RELEASE(t->coll_allgather_module);
    OBJ_RELEASE(t->coll_bcast_module);
    OBJ_RELEASE(t->coll_iallreduce_module);
    OBJ_RELEASE(t->coll_allreduce_init_module);
    OBJ_RELEASE(t->coll_iallgather_module);
    OBJ_RELEASE(t->coll_ibcast_module);
    OBJ_RELEASE(t->coll_ireduce_scatter_block_module);
    OBJ_RELEASE(t->coll_ireduce_module);
    OBJ_RELEASE(t->coll_iscan_module);
    OBJ_RELEASE(t->coll_iexscan_module);
    OBJ_RELEASE(t->coll_ireduce_scatter_module);
    OBJ_RELEASE(t->coll_reduce_scatter_block_init_module);
    OBJ_RELEASE(t->coll_allgather_init_module);
    OBJ_RELEASE(t->coll_bcast_init_module);
    OBJ_RELEASE(t->coll_reduce_init_module);
    OBJ_RELEASE(t->coll_reduce_scatter_init_module);
    OBJ_RELEASE(t->coll_scan_init_module);
    OBJ_RELEASE(t->coll_exscan_init_module);
}

/* deterministic per-rank floats in [-1, 1): fp sums depend on order */
static void gen(float *x, size_t n, int rank, int salt)
{
    unsigned long long s = 0x9E3779B97F4A7C15ull * (unsigned long long)(rank * 131 + salt + 1);
    for (size_t i = 0; i < n; ++i) {
        s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
        x[i] = (float)((double)((s * 2685821657736338717ull) >> 40) / (double)(1ull << 24)) * 2.f - 1.f;
    }
}

static float **all_inputs(size_t n, int salt)
{
    float **xs = malloc(sizeof(float *) * (size_t)g_size);
    for (int r = 0; r < g_size; ++r) {
        xs[r] = malloc(n * sizeof(float) + 4);
        gen(xs[r], n, r, salt);
    }
    return xs;
}

static void free_inputs(float **xs)
{
    for (int r = 0; r < g_size; ++r) free(xs[r]);
    free(xs);
}

static void *dev_of(const void *h, size_t bytes)
{
    void *d = NULL;
    CHECK(harness_dev_alloc_copy(&d, h, bytes) == 0, "device alloc");
    return d;
}

static void expect_dev(const void *d, const void *exp, size_t bytes, const char *what)
{
    char *got = malloc(bytes + 1);
    CHECK(harness_dev_copy_back(got, d, bytes) == 0, "copy back");
    CHECK(memcmp(got, exp, bytes) == 0, "%s differs from the oracle", what);
    free(got);
}

/* ---- section 6: one collective on the saved path, checked exactly ---- */
enum { C_ALLREDUCE, C_REDUCE, C_SCAN, C_EXSCAN, C_RSB, C_RS, C_ALLGATHER, C_BCAST };
enum { F_BLOCKING, F_NONBLOCKING, F_PERSISTENT };
static mca_coll_base_comm_coll_t *g_table;
static ompi_communicator_t *g_comm;

/* packed element bytes of rank r's input */
static void gen_packed(const ompi_datatype_t *d, size_t count, int r, int salt, char *out)
{
    float *f = malloc(count * sizeof(float) + 4);
    gen(f, count, r, salt);
    memset(out, 0, count * d->size);
    for (size_t i = 0; i < count; ++i) {
        if (HARNESS_T_LONG_DOUBLE == d->id) ((long double *) out)[i] = (long double) f[i] / 3.0L;
        else if (ORC_T_BYTE == d->id) out[i] = (char) (f[i] * 127.f);
        else ((float *) out)[i] = f[i];
    }
    free(f);
}

/* typed layout of packed elements: gaps (vector type) hold 0x5A */
static size_t span_of(const ompi_datatype_t *d, size_t count)
{
    return count == 0 ? 0 : (d->contiguous ? count * d->size : (2 * count - 1) * d->size);
}

static void to_typed(const ompi_datatype_t *d, const char *packed, size_t first, size_t count,
                     char *typed)
{
    const size_t st = d->contiguous ? d->size : 2 * d->size;
    for (size_t i = 0; i < count; ++i) memcpy(typed + (first + i) * st, packed + i * d->size, d->size);
}

/* a buffer this rank passes: device memory unless it is the host rank */
static void *place(const char *typed, size_t bytes, int on_host)
{
    void *p;
    if (on_host) {
        p = malloc(bytes + 1);
        memcpy(p, typed, bytes);
        return p;
    }
    return dev_of(typed, bytes + 1);
}

static void unplace(void *p, int on_host)
{
    if (on_host) free(p);
    else harness_dev_free(p);
}

static void fetch(void *got, const void *p, size_t bytes, int on_host)
{
    if (on_host) memcpy(got, p, bytes);
    else CHECK(harness_dev_copy_back(got, p, bytes) == 0, "copy back");
}

static void refill(void *p, const char *typed, size_t bytes, int on_host)
{
    if (on_host) memcpy(p, typed, bytes);
    else CHECK(harness_dev_copy_in(p, typed, bytes) == 0, "copy in");
}

/* host_rank: -1 every rank on device memory, -2 every rank on host memory,
 * r >= 0 rank r on host memory and the others on device memory */
static void saved_case(const char *what, int coll, int form, ompi_datatype_t *d, ompi_op_t *op,
                       size_t count, int inplace, int salt, int host_rank)
{
    static const char *cname[] = {"allreduce", "reduce", "scan", "exscan", "rsb", "rs",
                                  "allgather", "bcast"};
    static const char *fname[] = {"blocking", "nonblocking", "persistent"};
    mca_coll_base_comm_coll_t *t = g_table;
    const int n = g_size, me = g_rank, root = 1 % n;
    const int on_host = host_rank == -2 || host_rank == me;
    const int opc = NULL != op ? op->o_f_to_c_index : 0;
    const size_t es = d->size;
    int rcounts[OMPI_AMD_MAX_RANKS];
    size_t nin = count, nout = count, at_out = 0, rtotal = 0;
    char **x = malloc(sizeof(char *) * (size_t) n), *exp, *sbuf_t = NULL, *rbuf_t, *got;
    void *sb = NULL, *rb = NULL;
    ompi_request_t *rq = NULL;
    const int calls0 = tuned_calls;
    int rounds = F_PERSISTENT == form ? 2 : 1, rc = OMPI_SUCCESS;
    size_t rspan, sspan;

    for (int r = 0; r < n; ++r) {
        rcounts[r] = (int) count + 3 * r - (r == 1 ? (int) count + 3 : 0);
        rtotal += (size_t) rcounts[r];
    }
    if (C_RSB == coll) nin = count * (size_t) n;
    if (C_RS == coll) { nin = rtotal; nout = (size_t) rcounts[me]; }
    if (C_ALLGATHER == coll) { nout = count * (size_t) n; at_out = count * (size_t) me; }
    /* the receive buffer: in place it carries the input too */
    if (inplace && (C_RSB == coll || C_RS == coll)) nout = nin;
    for (int r = 0; r < n; ++r) x[r] = malloc(nin * es + 16);
    exp = malloc(nout * es + 16);
    sspan = span_of(d, nin);
    rspan = span_of(d, nout);
    sbuf_t = malloc(sspan + 16);
    rbuf_t = malloc(rspan + 16);
    got = malloc(rspan + 16);
    for (int round = 0; round < rounds; ++round) {
        const int rs = salt * 10 + round;
        int is_out = 1;
        for (int r = 0; r < n; ++r) gen_packed(d, nin, r, rs, x[r]);
        /* the expected bytes of this rank's receive buffer, typed */
        memset(rbuf_t, 0x5A, rspan + 16);
        memset(sbuf_t, 0x5A, sspan + 16);
        to_typed(d, x[me], 0, nin, sbuf_t);
        switch (coll) {
        case C_ALLREDUCE: case C_SCAN: case C_EXSCAN:
            harness_expect_reduction(C_ALLREDUCE == coll ? HARNESS_ALLREDUCE
                                     : C_SCAN == coll ? HARNESS_SCAN : HARNESS_EXSCAN,
                                     opc, d, (const char *const *) x, n, me, count, exp);
            is_out = !(C_EXSCAN == coll && 0 == me);
            break;
        case C_REDUCE:
            harness_expect_reduction(HARNESS_ALLREDUCE, opc, d, (const char *const *) x, n, me,
                                     count, exp);
            is_out = me == root;
            break;
        case C_RSB: case C_RS: {
            int eq[OMPI_AMD_MAX_RANKS];
            for (int r = 0; r < n; ++r) eq[r] = C_RSB == coll ? (int) count : rcounts[r];
            harness_expect_rs(opc, d, (const char *const *) x, n, me, eq, exp);
            break;
        }
        case C_ALLGATHER:
            for (int r = 0; r < n; ++r) memcpy(exp + (size_t) r * count * es, x[r], count * es);
            break;
        case C_BCAST:
            memcpy(exp, x[root], count * es);
            break;
        }
        if (round == 0) {  /* buffers: the receive side starts as 0x5A, or the input in place */
            char *init = malloc(rspan + 16);
            memset(init, 0x5A, rspan + 16);
            if (inplace && C_ALLGATHER == coll) to_typed(d, x[me], at_out, count, init);
            else if (inplace || C_BCAST == coll) to_typed(d, x[me], 0, C_BCAST == coll ? count : nin, init);
            if (C_BCAST == coll && me != root) memset(init, 0x5A, rspan + 16);
            rb = place(init, rspan, on_host);
            if (!inplace && C_BCAST != coll) sb = place(sbuf_t, sspan, on_host);
            free(init);
        } else {
            char *init = malloc(rspan + 16);
            memset(init, 0x5A, rspan + 16);
            if (inplace && C_ALLGATHER == coll) to_typed(d, x[me], at_out, count, init);
            else if (inplace || (C_BCAST == coll && me == root))
                to_typed(d, x[me], 0, C_BCAST == coll ? count : nin, init);
            refill(rb, init, rspan, on_host);
            if (sb) refill(sb, sbuf_t, sspan, on_host);
            free(init);
        }
        if (round == 0 || F_PERSISTENT != form) {
            const void *s = inplace ? MPI_IN_PLACE : sb;
            ompi_request_t **rp = &rq;
            switch (form * 8 + coll) {
#define B(c) (F_BLOCKING * 8 + (c))
#define NB(c) (F_NONBLOCKING * 8 + (c))
#define P(c) (F_PERSISTENT * 8 + (c))
            case B(C_ALLREDUCE): rc = t->coll_allreduce(s, rb, (int) count, d, op, g_comm, t->coll_allreduce_module); break;
            case B(C_REDUCE): rc = t->coll_reduce(inplace && me == root ? MPI_IN_PLACE : (inplace ? rb : sb), me == root ? rb : NULL, (int) count, d, op, root, g_comm, t->coll_reduce_module); break;
            case B(C_SCAN): rc = t->coll_scan(s, rb, (int) count, d, op, g_comm, t->coll_scan_module); break;
            case B(C_EXSCAN): rc = t->coll_exscan(s, rb, (int) count, d, op, g_comm, t->coll_exscan_module); break;
            case B(C_RSB): rc = t->coll_reduce_scatter_block(s, rb, (int) count, d, op, g_comm, t->coll_reduce_scatter_block_module); break;
            case B(C_RS): rc = t->coll_reduce_scatter(s, rb, rcounts, d, op, g_comm, t->coll_reduce_scatter_module); break;
            case B(C_ALLGATHER): rc = t->coll_allgather(s, (int) count, d, rb, (int) count, d, g_comm, t->coll_allgather_module); break;
            case B(C_BCAST): rc = t->coll_bcast(rb, (int) count, d, root, g_comm, t->coll_bcast_module); break;
            case NB(C_ALLREDUCE): rc = t->coll_iallreduce(s, rb, (int) count, d, op, g_comm, rp, t->coll_iallreduce_module); break;
            case NB(C_REDUCE): rc = t->coll_ireduce(inplace && me == root ? MPI_IN_PLACE : (inplace ? rb : sb), me == root ? rb : NULL, (int) count, d, op, root, g_comm, rp, t->coll_ireduce_module); break;
            case NB(C_SCAN): rc = t->coll_iscan(s, rb, (int) count, d, op, g_comm, rp, t->coll_iscan_module); break;
            case NB(C_EXSCAN): rc = t->coll_iexscan(s, rb, (int) count, d, op, g_comm, rp, t->coll_iexscan_module); break;
            case NB(C_RSB): rc = t->coll_ireduce_scatter_block(s, rb, (int) count, d, op, g_comm, rp, t->coll_ireduce_scatter_block_module); break;
            case NB(C_RS): rc = t->coll_ireduce_scatter(s, rb, rcounts, d, op, g_comm, rp, t->coll_ireduce_scatter_module); break;
            case NB(C_ALLGATHER): rc = t->coll_iallgather(s, (int) count, d, rb, (int) count, d, g_comm, rp, t->coll_iallgather_module); break;
            case NB(C_BCAST): rc = t->coll_ibcast(rb, (int) count, d, root, g_comm, rp, t->coll_ibcast_module); break;
            case P(C_ALLREDUCE): rc = t->coll_allreduce_init(s, rb, (int) count, d, op, g_comm, NULL, rp, t->coll_allreduce_init_module); break;
            case P(C_REDUCE): rc = t->coll_reduce_init(inplace && me == root ? MPI_IN_PLACE : (inplace ? rb : sb), me == root ? rb : NULL, (int) count, d, op, root, g_comm, NULL, rp, t->coll_reduce_init_module); break;
            case P(C_SCAN): rc = t->coll_scan_init(s, rb, (int) count, d, op, g_comm, NULL, rp, t->coll_scan_init_module); break;
            case P(C_EXSCAN): rc = t->coll_exscan_init(s, rb, (int) count, d, op, g_comm, NULL, rp, t->coll_exscan_init_module); break;
            case P(C_RSB): rc = t->coll_reduce_scatter_block_init(s, rb, (int) count, d, op, g_comm, NULL, rp, t->coll_reduce_scatter_block_init_module); break;
            case P(C_RS): rc = t->coll_reduce_scatter_init(s, rb, rcounts, d, op, g_comm, NULL, rp, t->coll_reduce_scatter_init_module); break;
            case P(C_ALLGATHER): rc = t->coll_allgather_init(s, (int) count, d, rb, (int) count, d, g_comm, NULL, rp, t->coll_allgather_init_module); break;
            case P(C_BCAST): rc = t->coll_bcast_init(rb, (int) count, d, root, g_comm, NULL, rp, t->coll_bcast_init_module); break;
#undef B
#undef NB
#undef P
            }
            CHECK(OMPI_SUCCESS == rc, "%s %s %s: rc %d", what, cname[coll], fname[form], rc);
            CHECK(tuned_calls == calls0 + 1, "%s %s %s: the saved function was not called (%d)",
                  what, cname[coll], fname[form], tuned_calls - calls0);
        }
        if (F_PERSISTENT == form) CHECK(rq->req_start(1, &rq) == OMPI_SUCCESS, "start");
        if (F_BLOCKING != form) {
            harness_wait(rq);
            CHECK(rq->req_status.MPI_ERROR == OMPI_SUCCESS, "%s %s %s: status %d", what,
                  cname[coll], fname[form], rq->req_status.MPI_ERROR);
        }
        /* compare the receive buffer: results where they belong, every
         * other byte as it was */
        if (C_REDUCE == coll && me != root && !inplace) is_out = 0;
        fetch(got, rb, rspan, on_host);
        if (is_out) {
            if (C_RS == coll || C_RSB == coll) {
                const size_t mine = C_RS == coll ? (size_t) rcounts[me] : count;
                to_typed(d, exp, 0, mine, rbuf_t);
                if (inplace) {  /* past the result: the input as it was */
                    const size_t st = d->contiguous ? es : 2 * es;
                    for (size_t i = mine; i < nin; ++i) memcpy(rbuf_t + i * st, x[me] + i * es, es);
                }
            } else {
                to_typed(d, exp, 0, nout, rbuf_t);
            }
            CHECK(memcmp(got, rbuf_t, rspan) == 0, "%s %s %s round %d (n %d, count %zu): result differs",
                  what, cname[coll], fname[form], round, n, count);
        }
        if (F_NONBLOCKING == form) CHECK(rq->req_free(&rq) == OMPI_SUCCESS, "free");
    }
    if (F_PERSISTENT == form) CHECK(rq->req_free(&rq) == OMPI_SUCCESS, "persistent free");
    if (sb) unplace(sb, on_host);
    unplace(rb, on_host);
    for (int r = 0; r < n; ++r) free(x[r]);
    free(x);
    free(exp);
    free(sbuf_t);
    free(rbuf_t);
    free(got);
}

/* HARNESS_COLL_BENCH=1 (GPU): MPI_Allreduce, MPI_Iallreduce + wait and
 * MPI_Allreduce_init start + wait, fp32 SUM on device buffers, called
 * through the installed table the way the MPI layer calls coll/rocm (the
 * osu_allreduce shape): mean per call over K calls after W warm-up calls
 * (enough to finish the autotune), each timed region opened by an 8-B
 * allreduce; one JSON line per size from rank 0.  Every input is 1.0, so
 * every result is exactly the rank count. */
static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec * 1e6 + (double) ts.tv_nsec * 1e-3;
}

static int bench(mca_coll_base_comm_coll_t *t, ompi_communicator_t *comm, ompi_datatype_t *f,
                 ompi_op_t *sum)
{
    static const size_t sizes[] = {8, 64, 1024, 16384, 65536, 262144, 1 << 20, 4 << 20,
                                   16 << 20, 64 << 20, 256 << 20};
    float one = 1.f, sync_h[2] = {1.f, 1.f};
    void *sync_d = dev_of(sync_h, sizeof(sync_h)), *sync_r = dev_of(sync_h, sizeof(sync_h));
    for (size_t z = 0; z < sizeof(sizes) / sizeof(sizes[0]); ++z) {
        const size_t bytes = sizes[z], n = bytes / 4;
        const int k = bytes <= (1 << 20) ? 200 : bytes <= (16 << 20) ? 40 : 10;
        const int w = 80;  /* the autotune decides at call 72 */
        float *h = malloc(bytes), *exp = malloc(bytes);
        double us[3];
        void *ds, *dr;
        ompi_request_t *req = NULL;
        for (size_t i = 0; i < n; ++i) { h[i] = one; exp[i] = (float) g_size; }
        ds = dev_of(h, bytes);
        dr = dev_of(h, bytes);
#define SYNC() CHECK(t->coll_allreduce(sync_d, sync_r, 2, f, sum, comm, t->coll_allreduce_module) == \
                     OMPI_SUCCESS, "sync allreduce")
#define AR() CHECK(t->coll_allreduce(ds, dr, (int) n, f, sum, comm, t->coll_allreduce_module) == \
                   OMPI_SUCCESS, "allreduce")
        for (int i = 0; i < w; ++i) AR();
        SYNC();
        {
            const double t0 = now_us();
            for (int i = 0; i < k; ++i) AR();
            us[0] = (now_us() - t0) / k;
        }
        expect_dev(dr, exp, bytes, "bench allreduce");
        for (int i = 0; i < 5; ++i) {
            CHECK(t->coll_iallreduce(ds, dr, (int) n, f, sum, comm, &req, t->coll_iallreduce_module) ==
                      OMPI_SUCCESS, "iallreduce");
            harness_wait(req);
            CHECK(req->req_free(&req) == OMPI_SUCCESS, "free");
        }
        SYNC();
        {
            const double t0 = now_us();
            for (int i = 0; i < k; ++i) {
                CHECK(t->coll_iallreduce(ds, dr, (int) n, f, sum, comm, &req,
                                         t->coll_iallreduce_module) == OMPI_SUCCESS, "iallreduce");
                harness_wait(req);
                CHECK(req->req_free(&req) == OMPI_SUCCESS, "free");
            }
            us[1] = (now_us() - t0) / k;
        }
        expect_dev(dr, exp, bytes, "bench iallreduce");
        CHECK(t->coll_allreduce_init(ds, dr, (int) n, f, sum, comm, NULL, &req,
                                     t->coll_allreduce_init_module) == OMPI_SUCCESS, "allreduce_init");
        for (int i = 0; i < 5; ++i) {
            CHECK(req->req_start(1, &req) == OMPI_SUCCESS, "start");
            harness_wait(req);
        }
        SYNC();
        {
            const double t0 = now_us();
            for (int i = 0; i < k; ++i) {
                CHECK(req->req_start(1, &req) == OMPI_SUCCESS, "start");
                harness_wait(req);
            }
            us[2] = (now_us() - t0) / k;
        }
        CHECK(req->req_free(&req) == OMPI_SUCCESS, "persistent free");
        expect_dev(dr, exp, bytes, "bench persistent allreduce");
#undef AR
#undef SYNC
        if (g_rank == 0)
            printf("{\"ranks\": %d, \"bytes\": %zu, \"calls\": %d, \"allreduce_us\": %.2f, "
                   "\"iallreduce_wait_us\": %.2f, \"persistent_start_wait_us\": %.2f, "
                   "\"busbw_GBps\": %.3f, \"exact\": true}\n",
                   g_size, bytes, k, us[0], us[1], us[2],
                   (double) bytes / (us[0] * 1e3) * 2.0 * (g_size - 1) / g_size);
        fflush(stdout);
        harness_dev_free(ds);
        harness_dev_free(dr);
        free(h);
        free(exp);
    }
    harness_dev_free(sync_d);
    harness_dev_free(sync_r);
    return 0;
}

/* ---- section T: coll/tuned's forcing variables (HARNESS_TUNED=1) ----
 * Run with some of OMPI_MCA_coll_tuned_{use_dynamic_rules, allreduce_algorithm,
 * reduce_algorithm, reduce_scatter_algorithm, reduce_scatter_block_algorithm,
 * dynamic_rules_filename} in the environment (the harness's MCA variable
 * stand-in reads them as the MCA system would).  Each blocking reduction
 * either runs on the device in exactly the order coll/tuned would run with
 * those settings (the oracle's forced algorithms, fp SUM, bit-exact), or —
 * where the glue does not implement that order — reaches the saved function
 * (tuned_calls) and returns what it computed. */
static int env_int(const char *n)
{
    const char *v = getenv(n);
    return v ? atoi(v) : 0;
}

static void tuned_section(mca_coll_base_comm_coll_t *t, ompi_communicator_t *comm, ompi_datatype_t *df,
                          ompi_op_t *sum)
{
    const int dyn = env_int("OMPI_MCA_coll_tuned_use_dynamic_rules");
    const char *file = getenv("OMPI_MCA_coll_tuned_dynamic_rules_filename");
    const int rules = dyn && file && file[0];
    const int ar = dyn ? env_int("OMPI_MCA_coll_tuned_allreduce_algorithm") : 0;
    const int red = dyn ? env_int("OMPI_MCA_coll_tuned_reduce_algorithm") : 0;
    const int rs = dyn ? env_int("OMPI_MCA_coll_tuned_reduce_scatter_algorithm") : 0;
    const int rsb = dyn ? env_int("OMPI_MCA_coll_tuned_reduce_scatter_block_algorithm") : 0;
    const int red_ok = red == 0 || red == 1 || red == 3 || red == 4 || red == 5;
    const int dev_red = !rules && red_ok;
    const int dev_ar = !rules && ar >= 0 && ar <= 6 && !(ar == 2 && !red_ok);
    const int dev_rs = !rules && rs >= 0 && rs <= 3 && !(rs == 1 && !red_ok);
    const int dev_rsb = !rules && (rsb == 0 || rsb == 1) && red_ok;
    const size_t sizes[2] = {3000, 400003};  /* staged and zero-copy */
    const int root = g_size - 1;
    for (int k = 0; k < 2; ++k) {
        const size_t n = sizes[k];
        float **xs = all_inputs(n, 90 + k);
        float **rb = malloc(sizeof(float *) * (size_t) g_size);
        float *exp = calloc(n, sizeof(float));
        void *ds = dev_of(xs[g_rank], n * 4), *dr = dev_of(exp, n * 4);
        int calls;
        for (int r = 0; r < g_size; ++r) rb[r] = calloc(n, sizeof(float));
        /* allreduce */
        if (dev_ar) {
            CHECK(orc_allreduce_forced_red(ar, g_size, (const void *const *) xs, (void *const *) rb, n,
                                           ORC_OP_SUM, ORC_T_FLOAT, 0, 0, red) >= 0, "oracle allreduce");
            memcpy(exp, rb[g_rank], n * 4);
        } else {
            harness_expect_reduction(HARNESS_ALLREDUCE, ORC_OP_SUM, df, (const char *const *) xs, g_size,
                                     g_rank, n, (char *) exp);
        }
        calls = tuned_calls;
        CHECK(t->coll_allreduce(ds, dr, (int) n, df, sum, comm, t->coll_allreduce_module) == OMPI_SUCCESS,
              "forced allreduce");
        CHECK((tuned_calls - calls) == !dev_ar, "allreduce %d: saved calls %d, want %d", ar,
              tuned_calls - calls, !dev_ar);
        expect_dev(dr, exp, n * 4, dev_ar ? "forced allreduce" : "declined allreduce");
        /* reduce to the last rank */
        if (dev_red) {
            CHECK(orc_reduce(red, g_size, (const void *const *) xs, exp, n, ORC_OP_SUM, ORC_T_FLOAT, root,
                             0) >= 0, "oracle reduce");
        } else {
            harness_expect_reduction(HARNESS_ALLREDUCE, ORC_OP_SUM, df, (const char *const *) xs, g_size,
                                     g_rank, n, (char *) exp);
        }
        calls = tuned_calls;
        CHECK(t->coll_reduce(ds, g_rank == root ? dr : NULL, (int) n, df, sum, root, comm,
                             t->coll_reduce_module) == OMPI_SUCCESS, "forced reduce");
        CHECK((tuned_calls - calls) == !dev_red, "reduce %d: saved calls %d", red, tuned_calls - calls);
        if (g_rank == root) expect_dev(dr, exp, n * 4, dev_red ? "forced reduce" : "declined reduce");
        /* reduce_scatter_block: n / size elements each */
        {
            const size_t rc = n / (size_t) g_size;
            if (dev_rsb) {
                CHECK(orc_reduce_scatter_block_alg(g_size, (const void *const *) xs, (void *const *) rb, rc,
                                                   ORC_OP_SUM, ORC_T_FLOAT, red) >= 0, "oracle rsb");
                memcpy(exp, rb[g_rank], rc * 4);
            } else {
                float *all = calloc(n, sizeof(float));
                harness_expect_reduction(HARNESS_ALLREDUCE, ORC_OP_SUM, df, (const char *const *) xs,
                                         g_size, g_rank, rc * (size_t) g_size, (char *) all);
                memcpy(exp, all + rc * (size_t) g_rank, rc * 4);
                free(all);
            }
            calls = tuned_calls;
            CHECK(t->coll_reduce_scatter_block(ds, dr, (int) rc, df, sum, comm,
                                               t->coll_reduce_scatter_block_module) == OMPI_SUCCESS,
                  "forced rsb");
            CHECK((tuned_calls - calls) == !dev_rsb, "rsb %d/%d: saved calls %d", rsb, red, tuned_calls - calls);
            expect_dev(dr, exp, rc * 4, dev_rsb ? "forced rsb" : "declined rsb");
        }
        /* reduce_scatter, uneven blocks */
        {
            int rcounts[OMPI_AMD_MAX_RANKS];
            size_t rcz[OMPI_AMD_MAX_RANKS], tot = 0;
            for (int r = 0; r < g_size; ++r) {
                rcounts[r] = (int) (n / (size_t) g_size) - 3 * r;
                rcz[r] = (size_t) rcounts[r];
                tot += rcz[r];
            }
            if (dev_rs) {
                if (rs == 1) {
                    CHECK(orc_reduce_scatter_nonoverlapping(g_size, (const void *const *) xs, (void *const *) rb,
                                                            rcz, ORC_OP_SUM, ORC_T_FLOAT, red, 0) >= 0,
                          "oracle rs nonoverlapping");
                } else {
                    CHECK(orc_reduce_scatter(rs == 2 ? ORC_RS_HALVING : rs == 3 ? ORC_RS_RING : ORC_RS_TUNED,
                                             g_size, (const void *const *) xs, (void *const *) rb, rcz,
                                             ORC_OP_SUM, ORC_T_FLOAT) >= 0, "oracle rs");
                }
                memcpy(exp, rb[g_rank], rcz[g_rank] * 4);
            } else {
                harness_expect_rs(ORC_OP_SUM, df, (const char *const *) xs, g_size, g_rank, rcounts, (char *) exp);
            }
            (void) tot;
            calls = tuned_calls;
            CHECK(t->coll_reduce_scatter(ds, dr, rcounts, df, sum, comm, t->coll_reduce_scatter_module) ==
                      OMPI_SUCCESS, "forced reduce_scatter");
            CHECK((tuned_calls - calls) == !dev_rs, "rs %d/%d: saved calls %d", rs, red, tuned_calls - calls);
            expect_dev(dr, exp, rcz[g_rank] * 4, dev_rs ? "forced reduce_scatter" : "declined reduce_scatter");
        }
        harness_dev_free(ds);
        harness_dev_free(dr);
        for (int r = 0; r < g_size; ++r) free(rb[r]);
        free(rb);
        free(exp);
        free_inputs(xs);
    }
}

int main(int argc, char **argv)
{
    const int use_gpu = getenv("HARNESS_GPU") && atoi(getenv("HARNESS_GPU"));
    ompi_group_t local = {0}, remote = {1};
    mca_coll_base_comm_coll_t table;
    ompi_communicator_t comm;
    mca_coll_base_module_t *tm, *m;
    ompi_datatype_t dfloat = {ORC_T_FLOAT, 4, 1, 1}, ddouble = {ORC_T_DOUBLE, 8, 1, 1};
    ompi_datatype_t dbyte = {ORC_T_BYTE, 1, 1, 1};
    ompi_op_t sum = {OMPI_OP_FLAGS_INTRINSIC, ORC_OP_SUM}, user = {0, ORC_OP_SUM};
    int prio = -1, i;

    if (argc < 4) return 2;
    g_rank = atoi(argv[2]);
    g_size = atoi(argv[3]);
    harness_proc_name.jobid = (unsigned) strtoul(argv[1], NULL, 16);
    for (i = 0; i < 64; ++i) ompi_op_ddt_map[i] = i;

    tm = OBJ_NEW(mca_coll_base_module_t);
    harness_saved_init(argv[1], g_rank, g_size);
    harness_fill_tuned(&table, tm);
    comm = (ompi_communicator_t){g_rank, g_size, 3, 0, &local, &table};

    /* selection (coll_base_comm_select.c): init_query, comm_query */
    CHECK((mca_coll_rocm_component.super.collm_init_query(false, false) == OMPI_SUCCESS) ==
              (ompi_amd_device_count() > 0), "init_query vs device presence");
    m = mca_coll_rocm_component.super.collm_comm_query(&comm, &prio);
    CHECK(m != NULL && prio == 80, "comm_query on a local intra-communicator");
    CHECK(m->coll_allreduce && m->coll_reduce && m->coll_reduce_scatter &&
              m->coll_reduce_scatter_block && m->coll_scan &&
              m->coll_exscan && m->coll_allgather && m->coll_bcast && m->coll_allreduce_init && m->coll_iallreduce &&
              m->coll_iallgather && m->coll_ibcast && m->coll_ireduce_scatter_block &&
              m->coll_ireduce && m->coll_iscan && m->coll_iexscan && m->coll_ireduce_scatter &&
              m->coll_reduce_scatter_block_init && m->coll_allgather_init && m->coll_bcast_init &&
              m->coll_reduce_init && m->coll_reduce_scatter_init && m->coll_scan_init &&
              m->coll_exscan_init && m->coll_module_enable,
          "module function table");
    {
        ompi_communicator_t c1 = comm, ci = comm, cr = comm;
        mca_coll_base_module_t *x;
        c1.size = 1;
        ci.inter = 1;
        cr.c_local_group = &remote;
        CHECK(mca_coll_rocm_component.super.collm_comm_query(&c1, &prio) == NULL, "size 1");
        CHECK(mca_coll_rocm_component.super.collm_comm_query(&ci, &prio) == NULL, "inter");
        CHECK(mca_coll_rocm_component.super.collm_comm_query(&cr, &prio) == NULL, "remote peers");
        c1.size = OMPI_AMD_MAX_RANKS + 1;
        x = mca_coll_rocm_component.super.collm_comm_query(&c1, &prio);
        CHECK(x == NULL, "too many ranks");
    }
    if (!use_gpu) {
        OBJ_RELEASE(m);
        release_table(&table);
        OBJ_RELEASE(tm);
        harness_saved_fini();
        printf("ok\n");
        return 0;
    }

    if (getenv("HARNESS_OWN_STREAM"))  /* the component parameter, as the MCA system would set it */
        mca_coll_rocm_component.own_stream = atoi(getenv("HARNESS_OWN_STREAM"));
    CHECK(m->coll_module_enable(m, &comm) == OMPI_SUCCESS, "enable");
    CHECK(tm->super.obj_reference_count == 1 + 24 + 24, "enable retains the saved modules (%d)",
          tm->super.obj_reference_count);
    install(&table, m);
    g_table = &table;
    g_comm = &comm;
    /* the bench runs with the component's defaults (residency locks after
     * coll_rocm_residency_lock unanimous votes, as in an application) */
    if (getenv("HARNESS_COLL_BENCH") && atoi(getenv("HARNESS_COLL_BENCH"))) {
        bench(&table, &comm, &dfloat, &sum);
        release_table(&table);
        OBJ_RELEASE(m);
        OBJ_RELEASE(tm);
        harness_saved_fini();
        return 0;
    }
    /* sections 1-8: the per-call residency vote (never locks) */
    mca_coll_rocm_component.residency_lock = 0;
    if (getenv("HARNESS_TUNED") && atoi(getenv("HARNESS_TUNED"))) {
        tuned_section(&table, &comm, &dfloat, &sum);
        release_table(&table);
        OBJ_RELEASE(m);
        OBJ_RELEASE(tm);
        harness_saved_fini();
        printf("ok gpu tuned\n");
        return 0;
    }

    /* 1. allreduce: staged (1000) and zero-copy (300001) sizes */
    {
        const int counts[2] = {1000, 300001};
        for (int k = 0; k < 2; ++k) {
            const size_t n = (size_t) counts[k];
            float **xs = all_inputs(n, 10 + k);
            float **rb = malloc(sizeof(float *) * (size_t) g_size);
            void *ds, *dr;
            for (int r = 0; r < g_size; ++r) rb[r] = calloc(n, sizeof(float));
            CHECK(orc_allreduce(ORC_AR_TUNED, g_size, (const void *const *) xs, (void *const *) rb,
                                n, ORC_OP_SUM, ORC_T_FLOAT, 0) >= 0, "oracle allreduce");
            ds = dev_of(xs[g_rank], n * 4);
            dr = dev_of(rb[g_rank], n * 4);  /* contents irrelevant */
            tuned_calls = 0;
            CHECK(table.coll_allreduce(ds, dr, (int) n, &dfloat, &sum, &comm,
                                       table.coll_allreduce_module) == OMPI_SUCCESS, "allreduce");
            CHECK(tuned_calls == 0, "device allreduce fell back");
            expect_dev(dr, rb[g_rank], n * 4, "allreduce");
            /* in place */
            CHECK(table.coll_allreduce(MPI_IN_PLACE, ds, (int) n, &dfloat, &sum, &comm,
                                       table.coll_allreduce_module) == OMPI_SUCCESS, "allreduce ip");
            expect_dev(ds, rb[g_rank], n * 4, "allreduce in place");
            harness_dev_free(ds);
            harness_dev_free(dr);
            for (int r = 0; r < g_size; ++r) free(rb[r]);
            free(rb);
            free_inputs(xs);
        }
    }
    /* 2. reduce to the last rank (tuned decision order), root in place */
    {
        const size_t n = 5000;
        const int root = g_size - 1;
        float **xs = all_inputs(n, 20);
        float *exp = calloc(n, sizeof(float)), *expip = calloc(n, sizeof(float));
        void *ds = dev_of(xs[g_rank], n * 4), *dr = dev_of(exp, n * 4);
        CHECK(orc_reduce(ORC_RED_TUNED, g_size, (const void *const *) xs, exp, n, ORC_OP_SUM,
                         ORC_T_FLOAT, root, 0) >= 0, "oracle reduce");
        CHECK(orc_reduce(ORC_RED_TUNED, g_size, (const void *const *) xs, expip, n, ORC_OP_SUM,
                         ORC_T_FLOAT, root, 1) >= 0, "oracle reduce in place");
        CHECK(table.coll_reduce(ds, g_rank == root ? dr : NULL, (int) n, &dfloat, &sum, root, &comm,
                                table.coll_reduce_module) == OMPI_SUCCESS, "reduce");
        if (g_rank == root) expect_dev(dr, exp, n * 4, "reduce");
        CHECK(table.coll_reduce(g_rank == root ? MPI_IN_PLACE : ds, g_rank == root ? ds : NULL,
                                (int) n, &dfloat, &sum, root, &comm,
                                table.coll_reduce_module) == OMPI_SUCCESS, "reduce in place");
        if (g_rank == root) expect_dev(ds, expip, n * 4, "reduce in place");
        harness_dev_free(ds);
        harness_dev_free(dr);
        free(exp);
        free(expip);
        free_inputs(xs);
    }
    /* 3. scan / exscan, fp64 */
    for (int ex = 0; ex < 2; ++ex) {
        const size_t n = 2000;
        double **xs = malloc(sizeof(double *) * (size_t) g_size);
        double **rb = malloc(sizeof(double *) * (size_t) g_size);
        float *tmp = malloc(n * sizeof(float));
        void *ds, *dr;
        for (int r = 0; r < g_size; ++r) {
            xs[r] = malloc(n * 8);
            rb[r] = calloc(n, 8);
            gen(tmp, n, r, 30 + ex);
            for (size_t k = 0; k < n; ++k) xs[r][k] = (double) tmp[k] / 3.0;
        }
        CHECK(orc_scan(ex, g_size, (const void *const *) xs, (void *const *) rb, n, ORC_OP_SUM,
                       ORC_T_DOUBLE) == 0, "oracle scan");
        ds = dev_of(xs[g_rank], n * 8);
        dr = dev_of(rb[g_rank], n * 8);
        CHECK((ex ? table.coll_exscan(ds, dr, (int) n, &ddouble, &sum, &comm,
                                      table.coll_exscan_module)
                  : table.coll_scan(ds, dr, (int) n, &ddouble, &sum, &comm,
                                    table.coll_scan_module)) == OMPI_SUCCESS, "scan");
        if (!(ex && g_rank == 0)) expect_dev(dr, rb[g_rank], n * 8, ex ? "exscan" : "scan");
        harness_dev_free(ds);
        harness_dev_free(dr);
        for (int r = 0; r < g_size; ++r) { free(xs[r]); free(rb[r]); }
        free(xs); free(rb); free(tmp);
    }
    /* 4. reduce_scatter_block (tuned reduce-to-0 order) */
    {
        const size_t rc = 1500, n = rc * (size_t) g_size;
        float **xs = all_inputs(n, 40);
        float **rb = malloc(sizeof(float *) * (size_t) g_size);
        void *ds, *dr;
        for (int r = 0; r < g_size; ++r) rb[r] = calloc(rc, sizeof(float));
        CHECK(orc_reduce_scatter_block(g_size, (const void *const *) xs, (void *const *) rb, rc,
                                       ORC_OP_SUM, ORC_T_FLOAT) >= 0, "oracle rsb");
        ds = dev_of(xs[g_rank], n * 4);
        dr = dev_of(rb[g_rank], rc * 4);
        CHECK(table.coll_reduce_scatter_block(ds, dr, (int) rc, &dfloat, &sum, &comm,
                                              table.coll_reduce_scatter_block_module) ==
                  OMPI_SUCCESS, "rsb");
        expect_dev(dr, rb[g_rank], rc * 4, "reduce_scatter_block");
        harness_dev_free(ds);
        harness_dev_free(dr);
        for (int r = 0; r < g_size; ++r) free(rb[r]);
        free(rb);
        free_inputs(xs);
    }
    /* 4b. reduce_scatter with uneven counts (one rank gets none) */
    {
        int rcounts[OMPI_AMD_MAX_RANKS];
        size_t rcz[OMPI_AMD_MAX_RANKS], n = 0;
        for (int r = 0; r < g_size; ++r) {
            rcounts[r] = (r == 1) ? 0 : 700 + 37 * r;
            rcz[r] = (size_t) rcounts[r];
            n += rcz[r];
        }
        float **xs = all_inputs(n, 45);
        float **rb = malloc(sizeof(float *) * (size_t) g_size);
        void *ds, *dr;
        for (int r = 0; r < g_size; ++r) rb[r] = calloc(rcz[r] + 1, sizeof(float));
        CHECK(orc_reduce_scatter(ORC_RS_TUNED, g_size, (const void *const *) xs, (void *const *) rb,
                                 rcz, ORC_OP_SUM, ORC_T_FLOAT) >= 0, "oracle reduce_scatter");
        ds = dev_of(xs[g_rank], n * 4);
        dr = dev_of(rb[g_rank], (rcz[g_rank] + 1) * 4);
        CHECK(table.coll_reduce_scatter(ds, dr, rcounts, &dfloat, &sum, &comm,
                                        table.coll_reduce_scatter_module) == OMPI_SUCCESS,
              "reduce_scatter");
        expect_dev(dr, rb[g_rank], rcz[g_rank] * 4, "reduce_scatter");
        harness_dev_free(ds);
        harness_dev_free(dr);
        for (int r = 0; r < g_size; ++r) free(rb[r]);
        free(rb);
        free_inputs(xs);
    }
    /* 5. allgather and bcast of bytes */
    {
        const size_t b = 1000;
        unsigned char *mine = malloc(b), *all = malloc(b * (size_t) g_size);
        void *ds, *dr;
        for (int r = 0; r < g_size; ++r)
            for (size_t k = 0; k < b; ++k) all[(size_t) r * b + k] = (unsigned char)(r * 17 + k * 3);
        memcpy(mine, all + (size_t) g_rank * b, b);
        ds = dev_of(mine, b);
        {
            unsigned char *zero = calloc(b * (size_t) g_size, 1);
            dr = dev_of(zero, b * (size_t) g_size);
            free(zero);
        }
        CHECK(table.coll_allgather(ds, (int) b, &dbyte, dr, (int) b, &dbyte, &comm,
                                   table.coll_allgather_module) == OMPI_SUCCESS, "allgather");
        expect_dev(dr, all, b * (size_t) g_size, "allgather");
        /* bcast from rank 1 % size of its slot */
        {
            const int root = 1 % g_size;
            void *bb = dev_of(g_rank == root ? all + (size_t) root * b : mine, b);
            CHECK(table.coll_bcast(bb, (int) b, &dbyte, root, &comm, table.coll_bcast_module) ==
                      OMPI_SUCCESS, "bcast");
            expect_dev(bb, all + (size_t) root * b, b, "bcast");
            harness_dev_free(bb);
        }
        harness_dev_free(ds);
        harness_dev_free(dr);
        free(mine);
        free(all);
    }
    /* 6. the saved functions on device buffers: whatever keeps a call off
     * the device path — a user op, a derived datatype, a type without a
     * device kernel (long double), a vector past max_device_mib, a peer
     * with host buffers — the saved (host) function must get host copies
     * of this rank's device operands and its results must come back into
     * them, in blocking, nonblocking and persistent form (the stand-ins fail
     * the run on any device pointer and compute the result on the host) */
    {
        ompi_datatype_t vfloat = {ORC_T_FLOAT, 4, 0, 0}; /* vector: 4 data + 4 gap bytes */
        ompi_datatype_t ldbl = {HARNESS_T_LONG_DOUBLE, 16, 1, 1};
        const int live0 = harness_saved_live;
        static const int reductions[6] = {C_ALLREDUCE, C_REDUCE, C_SCAN, C_EXSCAN, C_RSB, C_RS};
        /* (a) user op: every reduction, every form, in place where MPI has it */
        for (int f = 0; f < 3; ++f)
            for (int k = 0; k < 6; ++k) {
                saved_case("user op", reductions[k], f, &dfloat, &user, 1500 + 7 * k, 0, 200 + k, -1);
                if (reductions[k] != C_EXSCAN)
                    saved_case("user op in place", reductions[k], f, &dfloat, &user, 999, 1, 210 + k, -1);
            }
        /* (b) vector datatype: reductions with an intrinsic op, and the
         * data movers (device path packs only when locked to DEVICE) */
        for (int f = 0; f < 3; ++f) {
            saved_case("vector", C_ALLREDUCE, f, &vfloat, &sum, 2001, 0, 220, -1);
            saved_case("vector in place", C_ALLREDUCE, f, &vfloat, &sum, 2001, 1, 221, -1);
            saved_case("vector", C_REDUCE, f, &vfloat, &sum, 777, 0, 222, -1);
            saved_case("vector", C_RS, f, &vfloat, &sum, 300, 0, 223, -1);
            saved_case("vector", C_ALLGATHER, f, &vfloat, NULL, 333, 0, 224, -1);
            saved_case("vector in place", C_ALLGATHER, f, &vfloat, NULL, 333, 1, 225, -1);
            saved_case("vector", C_BCAST, f, &vfloat, NULL, 1234, 0, 226, -1);
        }
        /* (c) long double (op/base only) */
        for (int f = 0; f < 3; ++f) {
            saved_case("long double", C_ALLREDUCE, f, &ldbl, &sum, 1001, 0, 230, -1);
            saved_case("long double", C_REDUCE, f, &ldbl, &sum, 1001, 1, 231, -1);
            saved_case("long double", C_SCAN, f, &ldbl, &sum, 500, 0, 232, -1);
            saved_case("long double", C_RSB, f, &ldbl, &sum, 250, 0, 233, -1);
        }
        /* (d) past coll_rocm_max_device_mib (lowered to 1 MiB): every rank
         * decides alike (count, datatype and root agree) */
        {
            const int saved_mib = mca_coll_rocm_component.max_device_mib;
            const size_t big = (1u << 20) + 64;
            mca_coll_rocm_component.max_device_mib = 1;
            for (int f = 0; f < 3; ++f) {
                saved_case("past the cap", C_ALLREDUCE, f, &dfloat, &sum, big / 4, 0, 240, -1);
                saved_case("past the cap", C_BCAST, f, &dbyte, NULL, big, 0, 241, -1);
                saved_case("past the cap", C_ALLGATHER, f, &dbyte, NULL, big, 0, 242, -1);
                saved_case("past the cap", C_RSB, f, &dfloat, &sum, big / 4 / (size_t) g_size + 1, 0,
                           243, -1);
            }
            mca_coll_rocm_component.max_device_mib = saved_mib;
        }
        /* (e) mixed residency: rank 0's buffers are host memory, the vote
         * sends every rank to the saved functions, the others stage */
        for (int f = 0; f < 3; ++f) {
            saved_case("mixed residency", C_ALLREDUCE, f, &dfloat, &sum, 4096, 0, 250, 0);
            saved_case("mixed residency", C_SCAN, f, &dfloat, &sum, 4096, 0, 251, 0);
            saved_case("mixed residency", C_BCAST, f, &dbyte, NULL, 5000, 0, 252, 0);
            saved_case("mixed residency in place", C_ALLGATHER, f, &dbyte, NULL, 700, 1, 253, 0);
        }
        /* (f) host buffers on every rank: the saved functions as they are */
        for (int f = 0; f < 3; ++f) {
            saved_case("host", C_ALLREDUCE, f, &dfloat, &sum, 4096, 0, 260, -2);
            saved_case("host", C_REDUCE, f, &dfloat, &sum, 4096, 0, 261, -2);
        }
        CHECK(harness_saved_live == live0, "stand-in requests leaked (%d)", harness_saved_live - live0);
    }
    /* 7. persistent allreduce (MPI_Allreduce_init): init once, then three
     * start / wait rounds with fresh inputs (the plan reads the buffers'
     * current contents), staged and zero-copy sizes, in place; free */
    {
        const size_t counts[3] = {1000, 300001, 300001};
        for (int k = 0; k < 3; ++k) {
            const size_t n = counts[k];
            const int inplace = k == 2;
            float *zero = calloc(n, sizeof(float));
            void *ds = dev_of(zero, n * 4), *dr = dev_of(zero, n * 4);
            ompi_request_t *req = NULL;
            tuned_calls = 0;
            CHECK(table.coll_allreduce_init(inplace ? MPI_IN_PLACE : ds, dr, (int) n, &dfloat, &sum,
                                            &comm, NULL, &req,
                                            table.coll_allreduce_init_module) == OMPI_SUCCESS,
                  "allreduce_init");
            CHECK(tuned_calls == 0 && req != NULL && req->req_persistent &&
                      REQUEST_COMPLETE(req) && req->req_type == OMPI_REQUEST_COLL,
                  "allreduce_init request");
            for (int it = 0; it < 3; ++it) {
                float **xs = all_inputs(n, 60 + 3 * k + it);
                float **rb = malloc(sizeof(float *) * (size_t) g_size);
                for (int r = 0; r < g_size; ++r) rb[r] = calloc(n, sizeof(float));
                CHECK(orc_allreduce(ORC_AR_TUNED, g_size, (const void *const *) xs,
                                    (void *const *) rb, n, ORC_OP_SUM, ORC_T_FLOAT, 0) >= 0,
                      "oracle allreduce");
                CHECK(harness_dev_copy_in(inplace ? dr : ds, xs[g_rank], n * 4) == 0, "copy in");
                CHECK(req->req_start(1, &req) == OMPI_SUCCESS, "start");
                CHECK(req->req_state == OMPI_REQUEST_ACTIVE, "start activates");
                harness_wait(req);
                CHECK(req->req_status.MPI_ERROR == OMPI_SUCCESS, "persistent status %d",
                      req->req_status.MPI_ERROR);
                expect_dev(dr, rb[g_rank], n * 4, "persistent allreduce");
                for (int r = 0; r < g_size; ++r) free(rb[r]);
                free(rb);
                free_inputs(xs);
            }
            CHECK(req->req_free(&req) == OMPI_SUCCESS && req == MPI_REQUEST_NULL, "request free");
            harness_dev_free(ds);
            harness_dev_free(dr);
            free(zero);
        }
        /* host buffers: the saved allreduce_init builds the request */
        {
            float h[16] = {0}, h2[16] = {0};
            ompi_request_t *req = NULL;
            tuned_calls = 0;
            CHECK(table.coll_allreduce_init(h, h2, 16, &dfloat, &sum, &comm, NULL, &req,
                                            table.coll_allreduce_init_module) == OMPI_SUCCESS &&
                      tuned_calls == 1 && harness_is_saved_request(req),
                  "host allreduce_init falls back");
            CHECK(req->req_free(&req) == OMPI_SUCCESS, "free");
        }
    }
    /* 8. nonblocking allreduce (MPI_Iallreduce): staged and zero-copy sizes
     * outstanding together, completed through opal_progress, then freed */
    {
        const size_t counts[2] = {1000, 300001};
        float **xs[2], **rb[2];
        void *ds[2], *dr[2];
        ompi_request_t *req[2];
        tuned_calls = 0;
        for (int k = 0; k < 2; ++k) {
            const size_t n = counts[k];
            xs[k] = all_inputs(n, 70 + k);
            rb[k] = malloc(sizeof(float *) * (size_t) g_size);
            for (int r = 0; r < g_size; ++r) rb[k][r] = calloc(n, sizeof(float));
            CHECK(orc_allreduce(ORC_AR_TUNED, g_size, (const void *const *) xs[k],
                                (void *const *) rb[k], n, ORC_OP_SUM, ORC_T_FLOAT, 0) >= 0,
                  "oracle allreduce");
            ds[k] = dev_of(xs[k][g_rank], n * 4);
            dr[k] = dev_of(rb[k][g_rank], n * 4);
            CHECK(harness_dev_copy_in(dr[k], xs[k][(g_rank + 1) % g_size], n * 4) == 0, "junk");
            CHECK(table.coll_iallreduce(ds[k], dr[k], (int) n, &dfloat, &sum, &comm, &req[k],
                                        table.coll_iallreduce_module) == OMPI_SUCCESS,
                  "iallreduce");
            CHECK(req[k] != NULL && !req[k]->req_persistent &&
                      req[k]->req_type == OMPI_REQUEST_COLL, "iallreduce request");
        }
        CHECK(tuned_calls == 0, "device iallreduce fell back");
        for (int k = 1; k >= 0; --k) {
            harness_wait(req[k]);
            CHECK(req[k]->req_status.MPI_ERROR == OMPI_SUCCESS, "iallreduce status");
            expect_dev(dr[k], rb[k][g_rank], counts[k] * 4, "iallreduce");
            CHECK(req[k]->req_free(&req[k]) == OMPI_SUCCESS && req[k] == MPI_REQUEST_NULL,
                  "iallreduce free");
            harness_dev_free(ds[k]);
            harness_dev_free(dr[k]);
            for (int r = 0; r < g_size; ++r) free(rb[k][r]);
            free(rb[k]);
            free_inputs(xs[k]);
        }
        {
            float h[16] = {0}, h2[16] = {0};
            ompi_request_t *hr = NULL;
            CHECK(table.coll_iallreduce(h, h2, 16, &dfloat, &sum, &comm, &hr,
                                        table.coll_iallreduce_module) == OMPI_SUCCESS &&
                      tuned_calls == 1 && harness_is_saved_request(hr),
                  "host iallreduce falls back");
            harness_wait(hr);
            CHECK(hr->req_free(&hr) == OMPI_SUCCESS, "free");
        }
    }
    /* 10. MPI_Ireduce_scatter_block / MPI_Iallgather / MPI_Ibcast on device
     * buffers (staged and zero-copy sizes, all outstanding at once, completed
     * through opal_progress), bit-exact; host buffers go to the saved ones */
    {
        const size_t rcs[2] = {700, 300001};
        const size_t agb[2] = {3000, 1500001};
        float **xs[2], **rb[2];
        void *ds[2], *dr[2], *ag_d[2], *bc_d[2];
        unsigned char *ag_all[2], *bc_data[2];
        ompi_request_t *req[6];
        int nr = 0;
        tuned_calls = 0;
        for (int k = 0; k < 2; ++k) {
            const size_t rc = rcs[k], n = rc * (size_t) g_size;
            xs[k] = all_inputs(n, 80 + k);
            rb[k] = malloc(sizeof(float *) * (size_t) g_size);
            for (int r = 0; r < g_size; ++r) rb[k][r] = calloc(rc, sizeof(float));
            CHECK(orc_reduce_scatter_block(g_size, (const void *const *) xs[k], (void *const *) rb[k],
                                           rc, ORC_OP_SUM, ORC_T_FLOAT) >= 0, "oracle rsb");
            ds[k] = dev_of(xs[k][g_rank], n * 4);
            {
                float *z = calloc(rc, sizeof(float));
                dr[k] = dev_of(z, rc * 4);
                free(z);
            }
            CHECK(table.coll_ireduce_scatter_block(ds[k], dr[k], (int) rc, &dfloat, &sum, &comm,
                                                   &req[nr++],
                                                   table.coll_ireduce_scatter_block_module) ==
                      OMPI_SUCCESS, "ireduce_scatter_block");
            /* allgather of agb[k] bytes per rank */
            ag_all[k] = malloc(agb[k] * (size_t) g_size);
            for (int r = 0; r < g_size; ++r)
                for (size_t b = 0; b < agb[k]; ++b)
                    ag_all[k][(size_t) r * agb[k] + b] = (unsigned char) (r * 41 + b * 7 + k);
            {
                unsigned char *z = calloc(agb[k] * (size_t) g_size, 1);
                memcpy(z + (size_t) g_rank * agb[k], ag_all[k] + (size_t) g_rank * agb[k], agb[k]);
                ag_d[k] = dev_of(z, agb[k] * (size_t) g_size);  /* in place */
                free(z);
            }
            CHECK(table.coll_iallgather(MPI_IN_PLACE, 0, &dbyte, ag_d[k], (int) agb[k], &dbyte, &comm,
                                        &req[nr++], table.coll_iallgather_module) == OMPI_SUCCESS,
                  "iallgather");
            /* bcast of agb[k] bytes from rank k % size */
            bc_data[k] = malloc(agb[k]);
            for (size_t b = 0; b < agb[k]; ++b) bc_data[k][b] = (unsigned char) (b * 13 + k + 1);
            {
                unsigned char *z = calloc(agb[k], 1);
                bc_d[k] = dev_of(g_rank == k % g_size ? bc_data[k] : z, agb[k]);
                free(z);
            }
            CHECK(table.coll_ibcast(bc_d[k], (int) agb[k], &dbyte, k % g_size, &comm, &req[nr++],
                                    table.coll_ibcast_module) == OMPI_SUCCESS, "ibcast");
        }
        CHECK(tuned_calls == 0, "device nonblocking collectives fell back");
        for (int i = nr - 1; i >= 0; --i) {
            harness_wait(req[i]);
            CHECK(req[i]->req_status.MPI_ERROR == OMPI_SUCCESS, "nonblocking status");
            CHECK(req[i]->req_free(&req[i]) == OMPI_SUCCESS, "nonblocking free");
        }
        for (int k = 0; k < 2; ++k) {
            expect_dev(dr[k], rb[k][g_rank], rcs[k] * 4, "ireduce_scatter_block");
            expect_dev(ag_d[k], ag_all[k], agb[k] * (size_t) g_size, "iallgather");
            expect_dev(bc_d[k], bc_data[k], agb[k], "ibcast");
            harness_dev_free(ds[k]);
            harness_dev_free(dr[k]);
            harness_dev_free(ag_d[k]);
            harness_dev_free(bc_d[k]);
            for (int r = 0; r < g_size; ++r) free(rb[k][r]);
            free(rb[k]);
            free_inputs(xs[k]);
            free(ag_all[k]);
            free(bc_data[k]);
        }
        {
            unsigned char h[64] = {0};
            ompi_request_t *hr = NULL;
            CHECK(table.coll_ibcast(h, 64, &dbyte, 0, &comm, &hr, table.coll_ibcast_module) ==
                      OMPI_SUCCESS && tuned_calls == 1 && harness_is_saved_request(hr),
                  "host ibcast falls back");
            harness_wait(hr);
            CHECK(hr->req_free(&hr) == OMPI_SUCCESS, "free");
        }
    }
    /* 11. MPI_Ireduce / MPI_Iscan / MPI_Iexscan / MPI_Ireduce_scatter and the
     * persistent MPI_Reduce_scatter_block_init / MPI_Allgather_init /
     * MPI_Bcast_init through the communicator's table, on device buffers,
     * all outstanding at once, every result against the oracle; host
     * buffers go to the saved functions */
    {
        const size_t counts[2] = {1500, 300001};
        ompi_request_t *req[16];
        int nr = 0;
        void *d_in[2], *d_red[2], *d_scan[2], *d_exs[2], *d_rs[2], *d_rsbi[2], *d_rsbo[2];
        float **xs[2], *redexp[2], **scanexp[2], **exsexp[2], **rsexp[2], **rsbexp[2];
        float **rsbin[2];
        int rcounts[2][OMPI_AMD_MAX_RANKS];
        size_t rcz[2][OMPI_AMD_MAX_RANKS];
        tuned_calls = 0;
        for (int k = 0; k < 2; ++k) {
            const size_t n = counts[k];
            size_t total = 0;
            const int root = (k + 1) % g_size;
            xs[k] = all_inputs(n, 110 + k);
            redexp[k] = calloc(n, 4);
            scanexp[k] = malloc(sizeof(float *) * (size_t) g_size);
            exsexp[k] = malloc(sizeof(float *) * (size_t) g_size);
            rsexp[k] = malloc(sizeof(float *) * (size_t) g_size);
            for (int r = 0; r < g_size; ++r) {
                scanexp[k][r] = calloc(n, 4);
                exsexp[k][r] = calloc(n, 4);
                rcounts[k][r] = (int) (n / (size_t) g_size) + (r == 1 ? -7 : 3 * r);
                rcz[k][r] = (size_t) rcounts[k][r];
                total += rcz[k][r];
            }
            for (int r = 0; r < g_size; ++r) rsexp[k][r] = calloc(rcz[k][r] + 1, 4);
            CHECK(total <= n, "rs total");
            CHECK(orc_reduce(ORC_RED_TUNED, g_size, (const void *const *) xs[k], redexp[k], n, ORC_OP_SUM,
                             ORC_T_FLOAT, root, 0) >= 0, "oracle reduce");
            CHECK(orc_scan(0, g_size, (const void *const *) xs[k], (void *const *) scanexp[k], n, ORC_OP_SUM,
                           ORC_T_FLOAT) >= 0, "oracle scan");
            CHECK(orc_scan(1, g_size, (const void *const *) xs[k], (void *const *) exsexp[k], n, ORC_OP_SUM,
                           ORC_T_FLOAT) >= 0, "oracle exscan");
            CHECK(orc_reduce_scatter(ORC_RS_TUNED, g_size, (const void *const *) xs[k], (void *const *) rsexp[k],
                                     rcz[k], ORC_OP_SUM, ORC_T_FLOAT) >= 0, "oracle reduce_scatter");
            d_in[k] = dev_of(xs[k][g_rank], n * 4);
            {
                float *z = calloc(n + 1, 4);
                d_red[k] = dev_of(z, n * 4);
                d_scan[k] = dev_of(z, n * 4);
                d_exs[k] = dev_of(z, n * 4);
                d_rs[k] = dev_of(z, (rcz[k][g_rank] + 1) * 4);
                free(z);
            }
            CHECK(table.coll_ireduce(d_in[k], g_rank == root ? d_red[k] : NULL, (int) n, &dfloat, &sum, root,
                                     &comm, &req[nr++], table.coll_ireduce_module) == OMPI_SUCCESS,
                  "ireduce");
            CHECK(table.coll_iscan(d_in[k], d_scan[k], (int) n, &dfloat, &sum, &comm, &req[nr++],
                                   table.coll_iscan_module) == OMPI_SUCCESS, "iscan");
            CHECK(table.coll_iexscan(d_in[k], d_exs[k], (int) n, &dfloat, &sum, &comm, &req[nr++],
                                     table.coll_iexscan_module) == OMPI_SUCCESS, "iexscan");
            CHECK(table.coll_ireduce_scatter(d_in[k], d_rs[k], rcounts[k], &dfloat, &sum, &comm, &req[nr++],
                                             table.coll_ireduce_scatter_module) == OMPI_SUCCESS,
                  "ireduce_scatter");
        }
        CHECK(tuned_calls == 0, "device ireduce / iscan / ireduce_scatter fell back");
        for (int i = 0; i < nr; ++i) {
            harness_wait(req[i]);
            CHECK(req[i]->req_status.MPI_ERROR == OMPI_SUCCESS, "status");
            CHECK(req[i]->req_free(&req[i]) == OMPI_SUCCESS, "free");
        }
        for (int k = 0; k < 2; ++k) {
            const size_t n = counts[k];
            if (g_rank == (k + 1) % g_size) expect_dev(d_red[k], redexp[k], n * 4, "ireduce");
            expect_dev(d_scan[k], scanexp[k][g_rank], n * 4, "iscan");
            if (g_rank > 0) expect_dev(d_exs[k], exsexp[k][g_rank], n * 4, "iexscan");
            expect_dev(d_rs[k], rsexp[k][g_rank], rcz[k][g_rank] * 4, "ireduce_scatter");
        }
        /* persistent: three starts of each, fresh data every time */
        for (int k = 0; k < 2; ++k) {
            const size_t rc = counts[k] / (size_t) g_size;
            ompi_request_t *pr[3];
            unsigned char *ag_all = malloc(rc * 4 * (size_t) g_size), *bc_data = malloc(rc * 4);
            void *ag_d, *bc_d;
            rsbin[k] = all_inputs(rc * (size_t) g_size, 120 + k);
            rsbexp[k] = malloc(sizeof(float *) * (size_t) g_size);
            for (int r = 0; r < g_size; ++r) rsbexp[k][r] = calloc(rc, 4);
            d_rsbi[k] = dev_of(rsbin[k][g_rank], rc * 4 * (size_t) g_size);
            {
                float *z = calloc(rc + 1, 4);
                d_rsbo[k] = dev_of(z, rc * 4);
                free(z);
                unsigned char *zb = calloc(rc * 4 * (size_t) g_size, 1);
                ag_d = dev_of(zb, rc * 4 * (size_t) g_size);
                bc_d = dev_of(zb, rc * 4);
                free(zb);
            }
            CHECK(table.coll_reduce_scatter_block_init(d_rsbi[k], d_rsbo[k], (int) rc, &dfloat, &sum, &comm,
                                                       NULL, &pr[0],
                                                       table.coll_reduce_scatter_block_init_module) ==
                      OMPI_SUCCESS && pr[0]->req_persistent, "reduce_scatter_block_init");
            CHECK(table.coll_allgather_init(MPI_IN_PLACE, 0, &dbyte, ag_d, (int) (rc * 4), &dbyte, &comm, NULL,
                                            &pr[1], table.coll_allgather_init_module) == OMPI_SUCCESS &&
                      pr[1]->req_persistent, "allgather_init");
            CHECK(table.coll_bcast_init(bc_d, (int) (rc * 4), &dbyte, k % g_size, &comm, NULL, &pr[2],
                                        table.coll_bcast_init_module) == OMPI_SUCCESS &&
                      pr[2]->req_persistent, "bcast_init");
            CHECK(tuned_calls == 0, "device persistent inits fell back");
            for (int it = 0; it < 3; ++it) {
                for (int r = 0; r < g_size; ++r) gen(rsbin[k][r], rc * (size_t) g_size, r, 130 + 10 * k + it);
                CHECK(orc_reduce_scatter_block(g_size, (const void *const *) rsbin[k], (void *const *) rsbexp[k],
                                               rc, ORC_OP_SUM, ORC_T_FLOAT) >= 0, "oracle rsb");
                CHECK(harness_dev_copy_in(d_rsbi[k], rsbin[k][g_rank], rc * 4 * (size_t) g_size) == 0, "in");
                for (int r = 0; r < g_size; ++r)
                    for (size_t b = 0; b < rc * 4; ++b) ag_all[(size_t) r * rc * 4 + b] = (unsigned char) (r * 7 + b + it);
                for (size_t b = 0; b < rc * 4; ++b) bc_data[b] = (unsigned char) (b * 3 + it + k);
                {
                    unsigned char *zb = calloc(rc * 4 * (size_t) g_size, 1);
                    memcpy(zb + (size_t) g_rank * rc * 4, ag_all + (size_t) g_rank * rc * 4, rc * 4);
                    CHECK(harness_dev_copy_in(ag_d, zb, rc * 4 * (size_t) g_size) == 0, "ag in");
                    CHECK(harness_dev_copy_in(bc_d, g_rank == k % g_size ? bc_data : zb, rc * 4) == 0, "bc in");
                    free(zb);
                }
                for (int i = 0; i < 3; ++i)  /* MPI_Startall (request.h:60-77) */
                    CHECK(pr[i]->req_start(1, &pr[i]) == OMPI_SUCCESS, "start");
                for (int i = 0; i < 3; ++i) {
                    harness_wait(pr[i]);
                    CHECK(pr[i]->req_status.MPI_ERROR == OMPI_SUCCESS, "persistent status");
                }
                expect_dev(d_rsbo[k], rsbexp[k][g_rank], rc * 4, "reduce_scatter_block_init start");
                expect_dev(ag_d, ag_all, rc * 4 * (size_t) g_size, "allgather_init start");
                expect_dev(bc_d, bc_data, rc * 4, "bcast_init start");
            }
            for (int i = 0; i < 3; ++i) CHECK(pr[i]->req_free(&pr[i]) == OMPI_SUCCESS, "persistent free");
            harness_dev_free(ag_d);
            harness_dev_free(bc_d);
            free(ag_all);
            free(bc_data);
        }
        for (int k = 0; k < 2; ++k) {
            harness_dev_free(d_in[k]); harness_dev_free(d_red[k]); harness_dev_free(d_scan[k]);
            harness_dev_free(d_exs[k]); harness_dev_free(d_rs[k]); harness_dev_free(d_rsbi[k]);
            harness_dev_free(d_rsbo[k]);
            for (int r = 0; r < g_size; ++r) {
                free(scanexp[k][r]); free(exsexp[k][r]); free(rsexp[k][r]); free(rsbexp[k][r]);
            }
            free(scanexp[k]); free(exsexp[k]); free(rsexp[k]); free(rsbexp[k]); free(redexp[k]);
            free_inputs(xs[k]);
            free_inputs(rsbin[k]);
        }
        {
            float h[16] = {0}, h2[16] = {0};
            ompi_request_t *hr = NULL;
            CHECK(table.coll_iscan(h, h2, 16, &dfloat, &sum, &comm, &hr, table.coll_iscan_module) ==
                      OMPI_SUCCESS && tuned_calls == 1 && harness_is_saved_request(hr),
                  "host iscan falls back");
            harness_wait(hr);
            CHECK(hr->req_free(&hr) == OMPI_SUCCESS, "free");
            CHECK(table.coll_bcast_init(h, 16, &dbyte, 0, &comm, NULL, &hr, table.coll_bcast_init_module) ==
                      OMPI_SUCCESS && tuned_calls == 2 && harness_is_saved_request(hr),
                  "host bcast_init falls back");
            CHECK(hr->req_free(&hr) == OMPI_SUCCESS, "free");
        }
    }
    /* 9. residency policy: unanimous votes lock the module, a locked call
     * makes no bootstrap call, a rank whose buffers sit elsewhere stages
     * them, and a recheck vote unlocks after such a call */
    {
        mca_coll_rocm_module_t *rm = (mca_coll_rocm_module_t *) m;
        const size_t n = 1000;
        float **xs = all_inputs(n, 90);
        float **rb = malloc(sizeof(float *) * (size_t) g_size);
        float *h = malloc(n * 4), *h2 = calloc(n, 4), *got = malloc(n * 4);
        void *d, *d2;
        int64_t b0 = 0, b1 = 0;
        for (int r = 0; r < g_size; ++r) rb[r] = calloc(n, sizeof(float));
        CHECK(orc_allreduce(ORC_AR_TUNED, g_size, (const void *const *) xs, (void *const *) rb, n,
                            ORC_OP_SUM, ORC_T_FLOAT, 0) >= 0, "oracle allreduce");
        memcpy(h, xs[g_rank], n * 4);
        d = dev_of(h, n * 4);
        d2 = dev_of(h2, n * 4);
#define BOOT(v) CHECK(ompi_amd_comm_get_param(rm->dev_comm, "boot_calls", &(v)) == 0, "boot_calls")
        mca_coll_rocm_component.residency_lock = 3;
        mca_coll_rocm_component.residency_recheck = 4;
        CHECK(rm->mode == ROCM_RES_AUTO, "auto before the votes");
        rm->streak_dev = rm->streak_host = 0; /* sections 1-8 voted too */
        /* (a) three unanimous host votes lock HOST */
        tuned_calls = 0;
        BOOT(b0);
        for (int k = 0; k < 3; ++k)
            CHECK(table.coll_allreduce(h, h2, (int) n, &dfloat, &sum, &comm,
                                       table.coll_allreduce_module) == OMPI_SUCCESS, "host vote");
        BOOT(b1);
        CHECK(b1 - b0 == 3 && tuned_calls == 3 && rm->mode == ROCM_RES_HOST,
              "3 votes lock HOST (boot %lld, tuned %d, mode %d)", (long long) (b1 - b0), tuned_calls,
              rm->mode);
        /* (b) locked: a host-buffer allreduce makes no bootstrap call */
        BOOT(b0);
        CHECK(table.coll_allreduce(h, h2, (int) n, &dfloat, &sum, &comm,
                                   table.coll_allreduce_module) == OMPI_SUCCESS, "locked host");
        BOOT(b1);
        CHECK(b1 == b0 && tuned_calls == 4 && t_sdev == 0 && t_rdev == 0,
              "locked host call: %lld bootstrap calls", (long long) (b1 - b0));
        /* (c) rank 0 brings device buffers: it stages them to the host, the
         * saved function sees host memory on every rank, and its result
         * comes back into rank 0's device rbuf */
        CHECK(table.coll_allreduce(g_rank == 0 ? d : (void *) h, g_rank == 0 ? d2 : (void *) h2,
                                   (int) n, &dfloat, &sum, &comm,
                                   table.coll_allreduce_module) == OMPI_SUCCESS, "staged to host");
        CHECK(tuned_calls == 5 && t_sdev == 0 && t_rdev == 0, "saved function got host buffers");
        {
            float *want = malloc(n * 4);
            harness_expect_reduction(HARNESS_ALLREDUCE, ORC_OP_SUM, &dfloat, (const char *const *) xs,
                                     g_size, g_rank, n, (char *) want);
            if (g_rank == 0) {
                CHECK(harness_dev_copy_back(got, d2, n * 4) == 0 && memcmp(got, want, n * 4) == 0,
                      "staged rbuf copied back");
            } else {
                CHECK(memcmp(h2, want, n * 4) == 0, "host result beside a staging rank");
            }
            free(want);
        }
        /* (d) the 4th locked call is a recheck vote: rank 0 staged, so AUTO */
        BOOT(b0);
        for (int k = 0; k < 2; ++k)
            CHECK(table.coll_allreduce(h, h2, (int) n, &dfloat, &sum, &comm,
                                       table.coll_allreduce_module) == OMPI_SUCCESS, "recheck");
        BOOT(b1);
        CHECK(b1 - b0 == 1 && rm->mode == ROCM_RES_AUTO, "recheck unlocks (boot %lld mode %d)",
              (long long) (b1 - b0), rm->mode);
        /* (e) three unanimous device votes lock DEVICE (results exact) */
        tuned_calls = 0;
        for (int k = 0; k < 3; ++k) {
            CHECK(table.coll_allreduce(d, d2, (int) n, &dfloat, &sum, &comm,
                                       table.coll_allreduce_module) == OMPI_SUCCESS, "dev vote");
            expect_dev(d2, rb[g_rank], n * 4, "allreduce while voting");
        }
        CHECK(rm->mode == ROCM_RES_DEVICE && tuned_calls == 0, "DEVICE lock (mode %d)", rm->mode);
        /* (f) rank 0 brings host buffers: it stages them to the device, the
         * device path runs on every rank with no bootstrap call (staged size) */
        memset(h2, 0, n * 4);
        BOOT(b0);
        CHECK(table.coll_allreduce(g_rank == 0 ? (void *) h : d, g_rank == 0 ? (void *) h2 : d2,
                                   (int) n, &dfloat, &sum, &comm,
                                   table.coll_allreduce_module) == OMPI_SUCCESS, "staged to device");
        BOOT(b1);
        CHECK(b1 == b0 && tuned_calls == 0, "locked device call: %lld bootstrap calls, tuned %d",
              (long long) (b1 - b0), tuned_calls);
        if (g_rank == 0) CHECK(memcmp(h2, rb[0], n * 4) == 0, "host rbuf after device staging");
        else expect_dev(d2, rb[g_rank], n * 4, "allreduce beside a staging rank");
        /* (g) rank 0 receives an allgather into a non-contiguous type: it
         * packs through the datatype engine; its gaps stay untouched */
        {
            const size_t b = 64, elems = b / 4 * (size_t) g_size, span = elems * 8 - 4;
            ompi_datatype_t gap4 = {ORC_T_FLOAT, 4, 0, 0};
            unsigned char *mine = malloc(b), *all = malloc(b * (size_t) g_size), *t = malloc(span);
            void *ds, *dr;
            for (int r = 0; r < g_size; ++r)
                for (size_t k = 0; k < b; ++k) all[(size_t) r * b + k] = (unsigned char) (r * 29 + k);
            memcpy(mine, all + (size_t) g_rank * b, b);
            memset(t, 0x5A, span);
            ds = dev_of(mine, b);
            dr = dev_of(t, g_rank == 0 ? span : b * (size_t) g_size);
            CHECK(table.coll_allgather(ds, (int) b, &dbyte, dr, g_rank == 0 ? (int) (b / 4) : (int) b,
                                       g_rank == 0 ? &gap4 : &dbyte, &comm,
                                       table.coll_allgather_module) == OMPI_SUCCESS, "allgather");
            CHECK(tuned_calls == 0, "packed allgather stayed on the device path");
            if (g_rank == 0) {
                CHECK(harness_dev_copy_back(t, dr, span) == 0, "copy back");
                for (size_t e = 0; e < elems; ++e) {
                    CHECK(memcmp(t + e * 8, all + e * 4, 4) == 0, "packed element %zu", e);
                    if (e + 1 < elems) CHECK(t[e * 8 + 4] == 0x5A, "gap %zu overwritten", e);
                }
            } else {
                expect_dev(dr, all, b * (size_t) g_size, "allgather beside a packing rank");
            }
            harness_dev_free(ds);
            harness_dev_free(dr);
            free(mine);
            free(all);
            free(t);
        }
        /* (h) nonblocking calls under the DEVICE lock: no vote (zero
         * bootstrap calls); rank 0's host buffers go into its request's own
         * device memory and its output comes back when the request
         * completes (from opal_progress), counted as a mismatch for the
         * next recheck */
        {
            ompi_request_t *rq = NULL;
            const int mism0 = rm->mismatched;
            BOOT(b0);
            CHECK(table.coll_iallreduce(d, d2, (int) n, &dfloat, &sum, &comm, &rq,
                                        table.coll_iallreduce_module) == OMPI_SUCCESS,
                  "locked iallreduce");
            harness_wait(rq);
            CHECK(rq->req_status.MPI_ERROR == OMPI_SUCCESS && rq->req_free(&rq) == OMPI_SUCCESS,
                  "locked iallreduce completes");
            BOOT(b1);
            CHECK(b1 == b0 && tuned_calls == 0, "locked nonblocking call: %lld bootstrap calls",
                  (long long) (b1 - b0));
            expect_dev(d2, rb[g_rank], n * 4, "locked iallreduce");
            memset(h2, 0, n * 4);
            BOOT(b0);
            CHECK(table.coll_iallreduce(g_rank == 0 ? (void *) h : d, g_rank == 0 ? (void *) h2 : d2,
                                        (int) n, &dfloat, &sum, &comm, &rq,
                                        table.coll_iallreduce_module) == OMPI_SUCCESS,
                  "staged iallreduce");
            harness_wait(rq);
            CHECK(rq->req_status.MPI_ERROR == OMPI_SUCCESS && rq->req_free(&rq) == OMPI_SUCCESS,
                  "staged iallreduce completes");
            BOOT(b1);
            CHECK(b1 == b0 && tuned_calls == 0, "staged nonblocking call: %lld bootstrap calls",
                  (long long) (b1 - b0));
            if (g_rank == 0) {
                CHECK(memcmp(h2, rb[0], n * 4) == 0, "host rbuf after nonblocking staging");
                CHECK(rm->mismatched == mism0 + 1, "the staged call counts as a mismatch");
            } else {
                expect_dev(d2, rb[g_rank], n * 4, "iallreduce beside a staging rank");
            }
            /* MPI_Ibcast from the last rank, whose buffer is host memory */
            {
                const int root = g_size - 1;
                unsigned char *hb = malloc(777), *want = malloc(777);
                void *db;
                for (int k = 0; k < 777; ++k) want[k] = (unsigned char) (k * 7 + 3);
                memcpy(hb, g_rank == root ? want : (unsigned char *) h, 777);
                db = dev_of(hb, 777);
                CHECK(table.coll_ibcast(g_rank == root ? (void *) hb : db, 777, &dbyte, root, &comm,
                                        &rq, table.coll_ibcast_module) == OMPI_SUCCESS, "ibcast");
                harness_wait(rq);
                CHECK(rq->req_status.MPI_ERROR == OMPI_SUCCESS && rq->req_free(&rq) == OMPI_SUCCESS,
                      "ibcast completes");
                CHECK(tuned_calls == 0, "staged ibcast stayed on the device path");
                if (g_rank != root) expect_dev(db, want, 777, "ibcast from a host-buffer root");
                harness_dev_free(db);
                free(hb);
                free(want);
            }
            /* (i) MPI_Allreduce_init under the lock, rank 0 on host buffers:
             * every start refills its staged input, every completion
             * copies its output back */
            for (int round = 0; round < 2; ++round) {
                float **xs2 = all_inputs(n, 95 + round);
                float **rb2 = malloc(sizeof(float *) * (size_t) g_size);
                for (int r = 0; r < g_size; ++r) rb2[r] = calloc(n, sizeof(float));
                CHECK(orc_allreduce(ORC_AR_TUNED, g_size, (const void *const *) xs2,
                                    (void *const *) rb2, n, ORC_OP_SUM, ORC_T_FLOAT, 0) >= 0,
                      "oracle allreduce");
                if (0 == round) {
                    CHECK(table.coll_allreduce_init(g_rank == 0 ? (void *) h : d,
                                                    g_rank == 0 ? (void *) h2 : d2, (int) n, &dfloat,
                                                    &sum, &comm, NULL, &rq,
                                                    table.coll_allreduce_init_module) == OMPI_SUCCESS,
                          "allreduce_init under the lock");
                }
                if (g_rank == 0) memcpy(h, xs2[0], n * 4);
                else CHECK(harness_dev_copy_in(d, xs2[g_rank], n * 4) == 0, "input");
                CHECK(rq->req_start(1, &rq) == OMPI_SUCCESS, "start %d", round);
                harness_wait(rq);
                CHECK(rq->req_status.MPI_ERROR == OMPI_SUCCESS, "persistent status");
                if (g_rank == 0) CHECK(memcmp(h2, rb2[0], n * 4) == 0, "staged persistent result %d", round);
                else expect_dev(d2, rb2[g_rank], n * 4, "persistent beside a staging rank");
                for (int r = 0; r < g_size; ++r) free(rb2[r]);
                free(rb2);
                free_inputs(xs2);
            }
            CHECK(rq->req_free(&rq) == OMPI_SUCCESS && tuned_calls == 0, "persistent free");
        }
        /* (j) a staging failure on rank 0 under the DEVICE lock (VERDICT r4
         * item 7): its MPI_Allreduce returns the error, and every peer's
         * call fails within 1 s through the abort word instead of waiting
         * out the barrier timeout.  The communicator is unusable afterwards:
         * the section's last call. */
        {
            struct timespec t0, t1;
            double secs;
            int rc;
            CHECK(rm->mode == ROCM_RES_DEVICE, "still locked to DEVICE (mode %d)", rm->mode);
            rm->fail_stage = 0 == g_rank;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            rc = table.coll_allreduce(0 == g_rank ? (void *) h : d, 0 == g_rank ? (void *) h2 : d2,
                                      (int) n, &dfloat, &sum, &comm, table.coll_allreduce_module);
            clock_gettime(CLOCK_MONOTONIC, &t1);
            secs = (double) (t1.tv_sec - t0.tv_sec) + 1e-9 * (double) (t1.tv_nsec - t0.tv_nsec);
            CHECK(OMPI_SUCCESS != rc, "the call with rank 0's staging failure succeeded");
            CHECK(secs < 1.0, "failed after %.3f s (the peers waited for the barrier timeout)", secs);
            fprintf(stderr, "rank %d: staging failure on rank 0 -> rc %d after %.1f ms\n", g_rank, rc,
                    secs * 1e3);
        }
#undef BOOT
        harness_dev_free(d);
        harness_dev_free(d2);
        for (int r = 0; r < g_size; ++r) free(rb[r]);
        free(rb);
        free(h);
        free(h2);
        free(got);
        free_inputs(xs);
    }
    /* teardown: the table's references, then the module (its destructor
     * releases the saved modules and destroys the device communicator) */
    release_table(&table);
    OBJ_RELEASE(m);
    CHECK(tm->super.obj_reference_count == 1, "saved modules released (%d)",
          tm->super.obj_reference_count);
    OBJ_RELEASE(tm);
    harness_saved_fini();
    printf("ok gpu\n");
    return 0;
}
