/*
 * TEST HARNESS ONLY: drives ompi_amd/mca/osc/rocm through the osc
 * framework's selection protocol (ompi_osc_base_select: osc_init,
 * osc_query per flavor, osc_select) and the module table, one process per
 * rank (argv: name rank size).  HARNESS_GPU=0: selection checks only (no
 * device).  HARNESS_GPU=1: windows over device memory; every accumulate is
 * checked against the oracle's op/base restatement.  Prints "ok" / "ok gpu".
 */
#include <stdint.h>
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
#include "ompi/request/request.h"
#include "ompi/win/win.h"
#include "opal/runtime/opal_progress.h"
#include "opal/util/info.h"
#include "../../oracle/oracle.h"
#include "osc_rocm.h"
#include "ompi_amd.h"
#include "coll_saved.h"

extern int harness_dev_alloc_copy(void **d, const void *h, size_t bytes);
extern int harness_dev_copy_in(void *d, const void *h, size_t bytes);
extern int harness_dev_copy_back(void *h, const void *d, size_t bytes);
extern int harness_dev_free(void *d);

harness_proc_name_t harness_proc_name = {4242, 0};
int ompi_op_ddt_map[64];
OBJ_CLASS_INSTANCE(mca_coll_base_module_t, opal_object_t, NULL, NULL);
ompi_datatype_t harness_mpi_int = {ORC_T_INT32, 4, 1, 1};
ompi_op_t harness_mpi_max = {OMPI_OP_FLAGS_INTRINSIC, ORC_OP_MAX};

#define CHECK(c, ...)                                                   \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "rank %d: FAILED %s: ", g_rank, #c);         \
            fprintf(stderr, __VA_ARGS__);                               \
            fprintf(stderr, " (%s)\n", ompi_amd_last_error());          \
            exit(1);                                                    \
        }                                                               \
    } while (0)

static int g_rank, g_size;

/* exact data: k * 2^-8, k in [-1024, 1024] from a per-(rank, salt) LCG */
static void fill_exact(float *a, size_t n, int rank, int salt)
{
    uint64_t x = 0x9E3779B97F4A7C15ull ^ ((uint64_t)(rank + 1) << 20) ^ (uint64_t)salt;
    for (size_t i = 0; i < n; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        a[i] = (float)((int64_t)((x >> 33) % 2049) - 1024) * (1.0f / 256.0f);
    }
}

int main(int argc, char **argv)
{
    const int use_gpu = getenv("HARNESS_GPU") && atoi(getenv("HARNESS_GPU"));
    ompi_group_t local = {0}, remote = {1};
    ompi_communicator_t comm;
    ompi_datatype_t dfloat = {ORC_T_FLOAT, 4, 1, 1}, dint64 = {ORC_T_INT64, 8, 1, 1};
    ompi_op_t sum = {OMPI_OP_FLAGS_INTRINSIC, ORC_OP_SUM}, user = {0, ORC_OP_SUM};
    opal_info_t dev_info = {"ompi_amd_device", "true", NULL};
    ompi_osc_base_component_t *c = &mca_osc_rocm_component.super;
    mca_coll_base_comm_coll_t table;
    mca_coll_base_module_t *tm;
    int i;

    if (argc < 4) return 2;
    harness_proc_name.jobid = (unsigned) strtoul(argv[1], NULL, 16);
    g_rank = atoi(argv[2]);
    g_size = atoi(argv[3]);
    for (i = 0; i < 64; ++i) ompi_op_ddt_map[i] = i;
    local.grp_proc_count = g_size;
    /* the communicator's collectives (the query's agreement): host stand-ins */
    tm = OBJ_NEW(mca_coll_base_module_t);
    harness_saved_init(argv[1], g_rank, g_size);
    harness_fill_tuned(&table, tm);
    comm = (ompi_communicator_t){g_rank, g_size, 5, 0, &local, &table};
    if (c->osc_version.mca_register_component_params)
        c->osc_version.mca_register_component_params();

    /* selection (ompi_osc_base_select): init, then query per flavor */
    CHECK((c->osc_init(false, false) == OMPI_SUCCESS) == (ompi_amd_device_count() > 0),
          "osc_init vs device presence");
    {
        ompi_win_t w = {0};
        float host[4];
        void *hb = host;
        ompi_communicator_t ci = comm, cr = comm;
        ci.inter = 1;
        cr.c_local_group = &remote;
        CHECK(c->osc_query(&w, &hb, sizeof(host), 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE) < 0,
              "host memory is not a device window");
        CHECK(c->osc_query(&w, &hb, 0, 4, &comm, NULL, MPI_WIN_FLAVOR_ALLOCATE) < 0,
              "allocate without the device info key");
        CHECK(c->osc_query(&w, &hb, 0, 4, &ci, &dev_info, MPI_WIN_FLAVOR_ALLOCATE) < 0, "inter");
        CHECK(c->osc_query(&w, &hb, 0, 4, &cr, &dev_info, MPI_WIN_FLAVOR_ALLOCATE) < 0,
              "remote peers");
        CHECK(c->osc_query(&w, &hb, 0, 4, &comm, NULL, MPI_WIN_FLAVOR_DYNAMIC) < 0,
              "dynamic windows without the device info key (osc/rdma keeps them)");
        CHECK(c->osc_query(&w, &hb, 0, 4, &comm, NULL, MPI_WIN_FLAVOR_SHARED) < 0,
              "shared without the device info key");
    }
    if (!use_gpu) {
        harness_saved_fini();
        printf("ok\n");
        return 0;
    }

    const size_t n = 100003;
    const int nxt = (g_rank + 1) % g_size, prv = (g_rank + g_size - 1) % g_size;
    float *init = malloc(n * 4), *org = malloc(n * 4), *exp = malloc(n * 4), *got = malloc(n * 4);
    float *init_nxt = malloc(n * 4), *org_rank = malloc(n * 4);
    void *dbase = NULL, *dorg = NULL, *dgot = NULL, *abase = NULL;
    ompi_win_t win = {0}, awin = {0};
    int model = -1, prio;

    fill_exact(init, n, g_rank, 1);
    fill_exact(org, n, g_rank, 2);
    CHECK(harness_dev_alloc_copy(&dbase, init, n * 4) == 0, "device window");
    CHECK(harness_dev_alloc_copy(&dorg, org, n * 4) == 0, "device origin");
    CHECK(harness_dev_alloc_copy(&dgot, init, n * 4) == 0, "device result");

    /* residency differs between ranks: the framework
     * selects per rank, so the query agrees over the communicator.  Host
     * memory everywhere: no rank takes osc/rocm.  Rank 0 on host memory,
     * the others on device memory: every rank takes osc/rocm and every
     * rank's select refuses the window with the same error at once (no
     * rank waits for a peer).  Rank 0 with an empty window on a host
     * pointer: a device window. */
    {
        ompi_win_t mw = {0};
        float hostbuf[64];
        void *hb = hostbuf, *mb = 0 == g_rank ? (void *) hostbuf : dbase;
        struct timespec t0, t1;
        double secs;
        int rc;
        CHECK(c->osc_query(&mw, &hb, sizeof(hostbuf), 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE) < 0,
              "host windows on every rank stay with the host components");
        prio = c->osc_query(&mw, &mb, 64 * 4, 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE);
        CHECK(prio == 101, "mixed residency: every rank takes osc/rocm (%d)", prio);
        clock_gettime(CLOCK_MONOTONIC, &t0);
        rc = c->osc_select(&mw, &mb, 64 * 4, 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE, &model);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        secs = (double) (t1.tv_sec - t0.tv_sec) + 1e-9 * (double) (t1.tv_nsec - t0.tv_nsec);
        CHECK(rc == OMPI_ERR_NOT_SUPPORTED && NULL == mw.w_osc_module,
              "mixed residency refused alike (rc %d)", rc);
        CHECK(secs < 1.0, "mixed residency refused in %.3f s", secs);
        /* an empty host-pointer window beside device windows is a device window */
        mb = 0 == g_rank ? (void *) hostbuf : dbase;
        CHECK(c->osc_query(&mw, &mb, 0 == g_rank ? 0 : 64 * 4, 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE) == 101,
              "empty window on a host pointer");
        CHECK(c->osc_select(&mw, &mb, 0 == g_rank ? 0 : 64 * 4, 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE,
                            &model) == OMPI_SUCCESS && mw.w_osc_module, "select with an empty rank");
        CHECK(((ompi_osc_base_module_t *) mw.w_osc_module)->osc_free(&mw) == OMPI_SUCCESS, "free");
        /* the allocating flavor's info key on some ranks only: refused alike */
        CHECK(c->osc_query(&mw, &hb, 64, 8, &comm, 0 == g_rank ? NULL : &dev_info,
                           MPI_WIN_FLAVOR_ALLOCATE) == 101, "info key on some ranks");
        CHECK(c->osc_select(&mw, &hb, 64, 8, &comm, 0 == g_rank ? NULL : &dev_info,
                            MPI_WIN_FLAVOR_ALLOCATE, &model) == OMPI_ERR_NOT_SUPPORTED,
              "allocate with the info key on some ranks refused alike");
    }

    prio = c->osc_query(&win, &dbase, n * 4, 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE);
    CHECK(prio == 101, "query on device memory: %d", prio);
    CHECK(c->osc_query(&awin, &abase, 64, 8, &comm, &dev_info, MPI_WIN_FLAVOR_ALLOCATE) == 101,
          "query allocate with the device info key");
    CHECK(c->osc_select(&win, &dbase, n * 4, 4, &comm, NULL, MPI_WIN_FLAVOR_CREATE, &model) ==
              OMPI_SUCCESS && win.w_osc_module,
          "select create");
    /* a 400,012-byte hipMalloc is no IPC-safe size: peers reach a public
     * copy, the separate model (include/ompi_amd_osc.h); every fence, wait
     * and MPI_Win_sync below merges it with dbase */
    CHECK(model == MPI_WIN_SEPARATE, "model %d for a window over an IPC-unsafe allocation", model);
    ompi_osc_base_module_t *m = win.w_osc_module;

    /* active target: accumulate SUM into the next rank, bit-exact vs op/base */
    CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence 1");
    CHECK(m->osc_accumulate(dorg, (int) n, &dfloat, nxt, 0, (int) n, &dfloat, &sum, &win) ==
              OMPI_SUCCESS, "accumulate");
    CHECK(m->osc_accumulate(dorg, 3, &dfloat, nxt, 0, 3, &dfloat, &user, &win) ==
              OMPI_ERR_NOT_SUPPORTED, "user op refused");
    CHECK(m->osc_accumulate(dorg, 3, &dfloat, nxt, 0, 3, &dint64, &sum, &win) ==
              OMPI_ERR_NOT_SUPPORTED, "mismatched datatypes refused");
    CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence 2");
    CHECK(harness_dev_copy_back(got, dbase, n * 4) == 0, "copy back");
    {
        float *oprv = malloc(n * 4);
        fill_exact(oprv, n, prv, 2);
        memcpy(exp, init, n * 4);
        orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, oprv, exp, n);
        CHECK(0 == memcmp(got, exp, n * 4), "accumulated window");
        free(oprv);
    }
    /* get the next rank's window: its init + my origin */
    CHECK(m->osc_get(dgot, (int) n, &dfloat, nxt, 0, (int) n, &dfloat, &win) == OMPI_SUCCESS, "get");
    CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence 3");
    CHECK(harness_dev_copy_back(got, dgot, n * 4) == 0, "copy back get");
    fill_exact(init_nxt, n, nxt, 1);
    memcpy(org_rank, org, n * 4);
    orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, org_rank, init_nxt, n);
    CHECK(0 == memcmp(got, init_nxt, n * 4), "get of the next window");

    /* derived datatypes (osc_sm_comm.c:301, 350 -> ompi_osc_base_sndrcv_op):
     * a gapped stand-in float type (4 data bytes every 8) at the target and
     * result; expected values from op/base slot by slot in type-map order */
    {
        ompi_datatype_t dgap = {ORC_T_FLOAT, 4, 0, 0};
        ompi_op_t max = {OMPI_OP_FLAGS_INTRINSIC, ORC_OP_MAX};
        const size_t k = 4001;
        float *slots = malloc(k * 4), *oprv = malloc(n * 4), *mine = malloc(n * 4);
        float *nxtw = malloc(n * 4), *fetched = malloc(2 * k * 4), *pattern = malloc(2 * k * 4);
        size_t j;
        extern int harness_device_ddts;
        fill_exact(oprv, n, prv, 2);
        memcpy(mine, init, n * 4);  /* my window now: init + prv's origin */
        orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, oprv, mine, n);
        memcpy(nxtw, init_nxt, n * 4);  /* the next window now */
        CHECK(m->osc_accumulate(dorg, (int) k, &dfloat, nxt, 0, (int) k, &dgap, &max, &win) ==
                  OMPI_SUCCESS, "derived-target accumulate");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence derived 1");
        for (j = 0; j < k; ++j) slots[j] = mine[2 * j];
        orc_op_2buff(ORC_OP_MAX, ORC_T_FLOAT, oprv, slots, k);
        for (j = 0; j < k; ++j) mine[2 * j] = slots[j];
        for (j = 0; j < k; ++j) slots[j] = nxtw[2 * j];
        orc_op_2buff(ORC_OP_MAX, ORC_T_FLOAT, org, slots, k);
        for (j = 0; j < k; ++j) nxtw[2 * j] = slots[j];
        CHECK(harness_dev_copy_back(got, dbase, n * 4) == 0, "copy back derived 1");
        CHECK(0 == memcmp(got, mine, n * 4), "derived MAX accumulated into every other float");
        /* get_accumulate SUM: the old slots into a gapped result */
        fill_exact(pattern, 2 * k, g_rank, 77);
        CHECK(harness_dev_copy_in(dgot, pattern, 2 * k * 4) == 0, "result pattern");
        CHECK(m->osc_get_accumulate(dorg, (int) k, &dfloat, dgot, (int) k, &dgap, nxt, 0, (int) k,
                                    &dgap, &sum, &win) == OMPI_SUCCESS, "derived get_accumulate");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence derived 2");
        CHECK(harness_dev_copy_back(fetched, dgot, 2 * k * 4) == 0, "copy back fetched");
        for (j = 0; j < k; ++j) {
            CHECK(0 == memcmp(&fetched[2 * j], &nxtw[2 * j], 4), "fetched slot %zu", j);
            CHECK(0 == memcmp(&fetched[2 * j + 1], &pattern[2 * j + 1], 4), "result gap %zu", j);
        }
        for (j = 0; j < k; ++j) slots[j] = mine[2 * j];
        orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, oprv, slots, k);
        for (j = 0; j < k; ++j) mine[2 * j] = slots[j];
        CHECK(harness_dev_copy_back(got, dbase, n * 4) == 0, "copy back derived 2");
        CHECK(0 == memcmp(got, mine, n * 4), "derived get_accumulate summed");
        CHECK(harness_device_ddts > 0, "the device programs were used");
        CHECK(m->osc_accumulate(dorg, 3, &dfloat, nxt, 0, 3, &dgap, &user, &win) ==
                  OMPI_ERR_NOT_SUPPORTED, "user op on a derived type refused");
        /* the window as the next sections expect it: init + prv's origin */
        memcpy(mine, init, n * 4);
        orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, oprv, mine, n);
        CHECK(harness_dev_copy_in(dbase, mine, n * 4) == 0, "restore window");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence derived 3");
        /* derived put / get (osc_sm_comm.c:24-100, 209-270): my origin's
         * first k floats into every other float of the next window (its
         * gaps untouched), then those slots of the next window back into
         * a gapped origin layout whose gaps survive */
        {
            const size_t kk = 3001;
            float *expw = malloc(n * 4), *pat = malloc(2 * kk * 4), *back = malloc(2 * kk * 4);
            const int ddts0 = harness_device_ddts;
            CHECK(m->osc_put(dorg, (int) kk, &dfloat, nxt, 0, (int) kk, &dgap, &win) == OMPI_SUCCESS,
                  "derived-target put");
            CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence derived put");
            memcpy(expw, mine, n * 4);
            for (j = 0; j < kk; ++j) expw[2 * j] = oprv[j];
            CHECK(harness_dev_copy_back(got, dbase, n * 4) == 0, "copy back derived put");
            CHECK(0 == memcmp(got, expw, n * 4), "derived put: every other float, gaps untouched");
            fill_exact(pat, 2 * kk, g_rank, 78);
            CHECK(harness_dev_copy_in(dgot, pat, 2 * kk * 4) == 0, "get pattern");
            CHECK(m->osc_get(dgot, (int) kk, &dgap, nxt, 0, (int) kk, &dgap, &win) == OMPI_SUCCESS,
                  "derived get into a gapped origin");
            CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence derived get");
            CHECK(harness_dev_copy_back(back, dgot, 2 * kk * 4) == 0, "copy back derived get");
            {  /* which slots, and what they hold (pattern: never written; origin: the put) */
                size_t bad = 0, first = kk, last = 0, as_pat = 0;
                for (j = 0; j < kk; ++j)
                    if (0 != memcmp(&back[2 * j], &org[j], 4)) {
                        ++bad;
                        if (first == kk) first = j;
                        last = j;
                        as_pat += 0 == memcmp(&back[2 * j], &pat[2 * j], 4);
                    }
                if (bad)
                    fprintf(stderr, "rank %d: derived get: %zu of %zu slots wrong [%zu, %zu], %zu still "
                            "the pattern; slot %zu holds %g, expected %g\n", g_rank, bad, kk, first,
                            last, as_pat, first, back[2 * first], org[first]);
            }
            for (j = 0; j < kk; ++j) {
                CHECK(0 == memcmp(&back[2 * j], &org[j], 4), "derived get slot %zu", j);
                CHECK(0 == memcmp(&back[2 * j + 1], &pat[2 * j + 1], 4), "derived get gap %zu", j);
            }
            CHECK(harness_device_ddts >= ddts0, "device programs");
            CHECK(harness_dev_copy_in(dbase, mine, n * 4) == 0, "restore window after put");
            CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence derived 4");
            free(expw), free(pat), free(back);
        }
        free(slots), free(oprv), free(mine), free(nxtw), free(fetched), free(pattern);
    }

    /* passive target: each rank puts its rank id at displacement `rank` of
     * rank 0's window under an exclusive lock */
    {
        float me = (float) g_rank;
        CHECK(harness_dev_copy_in(dorg, &me, 4) == 0, "origin");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence 4");
        CHECK(m->osc_lock(MPI_LOCK_EXCLUSIVE, 0, 0, &win) == OMPI_SUCCESS, "lock");
        CHECK(m->osc_put(dorg, 1, &dfloat, 0, g_rank, 1, &dfloat, &win) == OMPI_SUCCESS, "put");
        CHECK(m->osc_unlock(0, &win) == OMPI_SUCCESS, "unlock");
        /* every origin unlocked (a host barrier): rank 0's MPI_Win_sync
         * brings the puts into its own memory, no fence needed */
        {
            int one = 1;
            CHECK(comm.c_coll->coll_allreduce(MPI_IN_PLACE, &one, 1, &harness_mpi_int, &harness_mpi_max,
                                              &comm, comm.c_coll->coll_allreduce_module) == OMPI_SUCCESS,
                  "host barrier");
        }
        if (0 == g_rank) {
            CHECK(m->osc_sync(&win) == OMPI_SUCCESS, "win_sync");
            CHECK(harness_dev_copy_back(got, dbase, 4 * (size_t) g_size) == 0, "copy back");
            for (i = 0; i < g_size; ++i) CHECK(got[i] == (float) i, "slot %d holds %g", i, got[i]);
        }
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence 5");
    }

    /* general active target (osc_sm_active_target.c:126-335): expose to the
     * previous rank, access the next; two epochs closed by wait, one by test */
    {
        const int wprv = prv, wnxt = nxt;
        ompi_group_t gprv = {0, 1, &wprv}, gnxt = {0, 1, &wnxt}, gnone = {0, 0, NULL};
        const int k = 4099;
        int flag = 0, e;
        CHECK(m->osc_complete(&win) == OMPI_ERR_RMA_SYNC, "complete without start");
        CHECK(m->osc_wait(&win) == OMPI_ERR_RMA_SYNC, "wait without post");
        CHECK(m->osc_test(&win, &flag) == OMPI_ERR_RMA_SYNC, "test without post");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence before pscw");
        for (e = 0; e < 3; ++e) {
            float *mine = malloc(k * 4), *theirs = malloc(k * 4);
            long spins = 0;
            fill_exact(mine, k, g_rank, 10 + e);
            fill_exact(theirs, k, prv, 10 + e);
            CHECK(harness_dev_copy_in(dorg, mine, k * 4) == 0, "origin");
            CHECK(m->osc_post(&gprv, 0, &win) == OMPI_SUCCESS, "post %d", e);
            CHECK(m->osc_post(&gprv, 0, &win) == OMPI_ERR_RMA_SYNC, "second post");
            CHECK(m->osc_start(&gnxt, 0, &win) == OMPI_SUCCESS, "start %d", e);
            CHECK(m->osc_start(&gnxt, 0, &win) == OMPI_ERR_RMA_SYNC, "second start");
            CHECK(m->osc_put(dorg, k, &dfloat, nxt, 0, k, &dfloat, &win) == OMPI_SUCCESS, "pscw put");
            CHECK(m->osc_complete(&win) == OMPI_SUCCESS, "complete %d", e);
            if (e < 2) {
                CHECK(m->osc_wait(&win) == OMPI_SUCCESS, "wait %d", e);
            } else {
                do {
                    CHECK(m->osc_test(&win, &flag) == OMPI_SUCCESS, "test");
                } while (!flag && ++spins < 2000000L);
                CHECK(flag, "MPI_Win_test never completed");
            }
            CHECK(harness_dev_copy_back(got, dbase, k * 4) == 0, "copy back");
            CHECK(0 == memcmp(got, theirs, k * 4), "pscw epoch %d window", e);
            /* everyone checked before the next epoch overwrites: an empty
             * epoch of a fence does it */
            CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence after epoch");
            free(mine);
            free(theirs);
        }
        /* the empty group and MPI_MODE_NOCHECK pass through */
        CHECK(m->osc_post(&gnone, MPI_MODE_NOCHECK, &win) == OMPI_SUCCESS &&
                  m->osc_start(&gnone, MPI_MODE_NOCHECK, &win) == OMPI_SUCCESS &&
                  m->osc_complete(&win) == OMPI_SUCCESS && m->osc_wait(&win) == OMPI_SUCCESS,
              "empty epoch");
    }

    /* request-based RMA under lock_all: MPI_Wait = opal_progress until the
     * request completes; then the window holds the put and the sum */
    {
        const int k = 5003;
        float *mine = malloc(k * 4), *theirs = malloc(k * 4), *fetched = malloc(k * 4);
        ompi_request_t *r1 = NULL, *r2 = NULL, *r3 = NULL;
        fill_exact(mine, k, g_rank, 20);
        fill_exact(theirs, k, prv, 20);
        CHECK(harness_dev_copy_in(dorg, mine, k * 4) == 0, "origin");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence before requests");
        CHECK(harness_dev_copy_back(exp, dbase, n * 4) == 0, "window before");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence before requests 2");
        CHECK(m->osc_lock_all(0, &win) == OMPI_SUCCESS, "lock_all");
        CHECK(m->osc_rput(dorg, k, &dfloat, nxt, 0, k, &dfloat, &win, &r1) == OMPI_SUCCESS && r1,
              "rput");
        CHECK(m->osc_raccumulate(dorg, k, &dfloat, nxt, 2 * k, k, &dfloat, &sum, &win, &r2) ==
                  OMPI_SUCCESS && r2, "raccumulate");
        CHECK(m->osc_rget(dgot, k, &dfloat, nxt, 4 * k, k, &dfloat, &win, &r3) == OMPI_SUCCESS && r3,
              "rget");
        CHECK(m->osc_raccumulate(dorg, 3, &dfloat, nxt, 0, 3, &dfloat, &user, &win, &r3) ==
                  OMPI_ERR_NOT_SUPPORTED, "user op refused (request)");
        while (!REQUEST_COMPLETE(r1) || !REQUEST_COMPLETE(r2)) opal_progress();
        CHECK(r1->req_status.MPI_ERROR == OMPI_SUCCESS && r2->req_status.MPI_ERROR == OMPI_SUCCESS,
              "request status");
        CHECK(r1->req_free(&r1) == OMPI_SUCCESS && r1 == MPI_REQUEST_NULL, "free r1");
        CHECK(r2->req_free(&r2) == OMPI_SUCCESS, "free r2");
        CHECK(r3->req_free(&r3) == OMPI_SUCCESS, "free r3 (waits)");
        CHECK(m->osc_unlock_all(&win) == OMPI_SUCCESS, "unlock_all");
        CHECK(m->osc_fence(0, &win) == OMPI_SUCCESS, "fence after requests");
        CHECK(harness_dev_copy_back(got, dbase, n * 4) == 0, "window after");
        CHECK(0 == memcmp(got, theirs, k * 4), "rput landed");
        memcpy(init_nxt, exp + 2 * k, k * 4);
        orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, theirs, init_nxt, k);
        CHECK(0 == memcmp(got + 2 * k, init_nxt, k * 4), "raccumulate landed");
        /* rget read [4k, 5k) of the next window: its init + my first accumulate */
        fill_exact(init_nxt, n, nxt, 1);
        memcpy(org_rank, org, n * 4);
        orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, org_rank, init_nxt, n);
        CHECK(harness_dev_copy_back(fetched, dgot, k * 4) == 0, "rget back");
        CHECK(0 == memcmp(fetched, init_nxt + 4 * k, k * 4), "rget fetched");
        free(mine);
        free(theirs);
        free(fetched);
    }

    /* MPI_Win_allocate_shared: segments of (rank + 1) * 1000 floats back to
     * back in one device allocation; each rank fills its own, reads every
     * peer's through MPI_Win_shared_query's address */
    {
        opal_info_t contig = {"alloc_shared_noncontig", "false", NULL};
        opal_info_t sinfo = {"ompi_amd_device", "true", &contig};
        ompi_win_t swin = {0};
        void *sbase = NULL, *qbase = NULL, *prev_end = NULL;
        const size_t mine_n = 1000 * (size_t)(g_rank + 1);
        float *buf = malloc(1000 * (size_t) g_size * 4), *ref = malloc(1000 * (size_t) g_size * 4);
        size_t qsize = 0;
        int qdu = 0, p;
        CHECK(c->osc_query(&swin, &sbase, mine_n * 4, 4, &comm, &sinfo, MPI_WIN_FLAVOR_SHARED) ==
                  101, "query shared with the device info key");
        CHECK(c->osc_select(&swin, &sbase, mine_n * 4, 4, &comm, &sinfo, MPI_WIN_FLAVOR_SHARED,
                            &model) == OMPI_SUCCESS && swin.w_osc_module && sbase,
              "select shared");
        ompi_osc_base_module_t *sm = swin.w_osc_module;
        fill_exact(buf, mine_n, g_rank, 30);
        CHECK(harness_dev_copy_in(sbase, buf, mine_n * 4) == 0, "own segment");
        CHECK(sm->osc_fence(0, &swin) == OMPI_SUCCESS, "shared fence");
        for (p = 0; p < g_size; ++p) {
            CHECK(sm->osc_win_shared_query(&swin, p, &qsize, &qdu, &qbase) == OMPI_SUCCESS,
                  "shared_query %d", p);
            CHECK(qsize == 1000 * (size_t)(p + 1) * 4 && qdu == 4, "segment %d size %zu", p, qsize);
            CHECK(p != g_rank || qbase == sbase, "own segment address");
            CHECK(p == 0 || qbase == prev_end, "segment %d not contiguous", p);
            prev_end = (char *) qbase + qsize;
            CHECK(harness_dev_copy_back(buf, qbase, qsize) == 0, "read segment %d", p);
            fill_exact(ref, qsize / 4, p, 30);
            CHECK(0 == memcmp(buf, ref, qsize), "segment %d bytes", p);
        }
        CHECK(sm->osc_win_shared_query(&swin, MPI_PROC_NULL, &qsize, &qdu, &qbase) == OMPI_SUCCESS &&
                  qsize == 4000 && qdu == 4, "MPI_PROC_NULL query");
        CHECK(m->osc_win_shared_query(&win, 0, &qsize, &qdu, &qbase) == MPI_ERR_WIN,
              "shared_query on an MPI_Win_create window");
        CHECK(m->osc_win_attach(&win, dorg, 64) == MPI_ERR_RMA_ATTACH &&
                  m->osc_win_detach(&win, dorg) == MPI_ERR_RMA_ATTACH, "attach / detach refused");
        CHECK(sm->osc_fence(0, &swin) == OMPI_SUCCESS, "shared fence 2");
        CHECK(sm->osc_free(&swin) == OMPI_SUCCESS, "free shared");
        free(buf);
        free(ref);
    }

    /* MPI_Win_create_dynamic with the device info key:
     * a 4 MiB device region attached on every rank, its address shared,
     * MPI_Put of 1000 floats into the next rank's region at an absolute
     * displacement under fences, bit-exact; host memory refused at attach
     * (MPI_ERR_RMA_ATTACH), a second detach refused (MPI_ERR_RMA_RANGE) */
    {
        ompi_win_t dw = {0};
        void *nb = NULL, *reg = NULL, *zero = calloc(1, 4 << 20), *hostbuf = calloc(1, 4096);
        int addr[4 * OMPI_AMD_MAX_RANKS] = {0};
        const size_t k = 1000;
        CHECK(c->osc_query(&dw, &nb, 0, 1, &comm, &dev_info, MPI_WIN_FLAVOR_DYNAMIC) == 101,
              "query dynamic with the device info key");
        CHECK(c->osc_select(&dw, &nb, 0, 1, &comm, &dev_info, MPI_WIN_FLAVOR_DYNAMIC, &model) ==
                  OMPI_SUCCESS && dw.w_osc_module, "select dynamic");
        ompi_osc_base_module_t *dm = dw.w_osc_module;
        CHECK(harness_dev_alloc_copy(&reg, zero, 4 << 20) == 0, "dynamic region");
        CHECK(dm->osc_win_attach(&dw, reg, 4 << 20) == OMPI_SUCCESS, "attach a device region");
        CHECK(dm->osc_win_attach(&dw, hostbuf, 4096) == MPI_ERR_RMA_ATTACH, "host attach refused");
        for (int q = 0; q < 4; ++q)  /* the address in 16-bit pieces: MAX over ints gathers them */
            addr[4 * g_rank + q] = (int) (((uint64_t) (uintptr_t) reg >> (16 * q)) & 0xffff);
        CHECK(comm.c_coll->coll_allreduce(MPI_IN_PLACE, addr, 4 * g_size, &harness_mpi_int, &harness_mpi_max,
                                          &comm, comm.c_coll->coll_allreduce_module) == OMPI_SUCCESS,
              "address exchange");
        uint64_t an = 0;
        for (int q = 0; q < 4; ++q) an |= (uint64_t) (unsigned) addr[4 * nxt + q] << (16 * q);
        CHECK(harness_dev_copy_in(dorg, org, k * 4) == 0, "origin");  /* earlier sections reused it */
        CHECK(dm->osc_fence(0, &dw) == OMPI_SUCCESS, "dynamic fence 1");
        CHECK(dm->osc_put(dorg, (int) k, &dfloat, nxt, (ptrdiff_t) (an + 256), (int) k, &dfloat, &dw) ==
                  OMPI_SUCCESS, "dynamic put");
        CHECK(dm->osc_fence(0, &dw) == OMPI_SUCCESS, "dynamic fence 2");
        {
            float *gotd = malloc(k * 4), *want = malloc(n * 4);
            fill_exact(want, n, prv, 2);  /* the previous rank's origin */
            CHECK(harness_dev_copy_back(gotd, (char *) reg + 256, k * 4) == 0, "dynamic copy back");
            CHECK(0 == memcmp(gotd, want, k * 4),
                  "dynamic put landed in the attached region (got %g %g, want %g %g; region %p, next's %llx)",
                  gotd[0], gotd[1], want[0], want[1], reg, (unsigned long long) an);
            free(gotd);
            free(want);
        }
        CHECK(dm->osc_win_detach(&dw, reg) == OMPI_SUCCESS, "detach");
        CHECK(dm->osc_win_detach(&dw, reg) == MPI_ERR_RMA_RANGE, "second detach refused");
        CHECK(dm->osc_free(&dw) == OMPI_SUCCESS, "free dynamic");
        harness_dev_free(reg);
        free(zero);
        free(hostbuf);
    }

    /* MPI_Win_allocate: a shared counter, fetch_and_op from every rank */
    CHECK(c->osc_select(&awin, &abase, 0 == g_rank ? 64 : 0, 8, &comm, &dev_info,
                        MPI_WIN_FLAVOR_ALLOCATE, &model) == OMPI_SUCCESS && awin.w_osc_module,
          "select allocate");
    {
        ompi_osc_base_module_t *a = awin.w_osc_module;
        int64_t one = 1, seen = -1, total = -1;
        void *done = NULL, *dres = NULL;
        const int k = 10;
        CHECK(harness_dev_alloc_copy(&done, &one, 8) == 0 && harness_dev_alloc_copy(&dres, &one, 8) == 0,
              "counter buffers");
        CHECK(a->osc_fence(0, &awin) == OMPI_SUCCESS, "afence 1");
        for (i = 0; i < k; ++i)
            CHECK(a->osc_fetch_and_op(done, dres, &dint64, 0, 0, &sum, &awin) == OMPI_SUCCESS,
                  "fetch_and_op");
        CHECK(a->osc_fence(0, &awin) == OMPI_SUCCESS, "afence 2");
        CHECK(harness_dev_copy_back(&seen, dres, 8) == 0, "last fetched");
        CHECK(seen >= k - 1 && seen < (int64_t) k * g_size, "last fetched value %lld", (long long) seen);
        if (0 == g_rank) {
            CHECK(harness_dev_copy_back(&total, abase, 8) == 0, "counter");
            CHECK(total == (int64_t) k * g_size, "counter %lld", (long long) total);
        }
        CHECK(a->osc_free(&awin) == OMPI_SUCCESS && NULL == awin.w_osc_module, "free allocate");
        harness_dev_free(done);
        harness_dev_free(dres);
    }
    CHECK(m->osc_free(&win) == OMPI_SUCCESS, "free create");
    harness_dev_free(dbase);
    harness_dev_free(dorg);
    harness_dev_free(dgot);
    harness_saved_fini();
    printf("ok gpu\n");
    return 0;
}
