/*
 * TEST HARNESS ONLY.  One rank of a multi-process run that drives
 * ompi_amd/mca/pml/rocm/pml_rocm.c the way the PML base does
 * (pml_base_select.c, pml_v_component.c:123-160): a stand-in "ob1" module is
 * the selected PML (its functions count and complete at once), pml/rocm's
 * init declines, its close interposes on mca_pml, pml_add_comm creates the
 * library communicator; then MPI-level traffic goes through mca_pml.
 *
 *   CPU (HARNESS_GPU=0): init declines, close installs the functions and
 *   saves ob1's; a communicator gets no library state without a device and
 *   every call reaches ob1.
 *   GPU (HARNESS_GPU=1): a ring of isend/irecv on device buffers (0 B,
 *   eager, rendezvous, 8 MiB), byte-exact; blocking send/recv from host
 *   memory (the library's pooled stages: no allocation per message); a
 *   non-contiguous receive type (packed, gaps kept); ANY_SOURCE / ANY_TAG
 *   status; iprobe / probe; persistent send/recv started three times;
 *   truncation; negative (system) tags and PROC_NULL reach ob1; matched
 *   probes of library traffic are refused; MPI_Request_free of an in-flight
 *   Ssend and irecv leaves no request on the active list; a sender that
 *   frees and reallocates its device buffer between messages (staged
 *   default and p2p_user_ipc = 1) stays byte-exact; pml_rocm_host_path = 1
 *   sends host-buffer traffic to ob1 with zero library calls.
 *
 * usage: pml_harness <segment-name-hex> <rank> <size>; prints "ok" / "ok gpu".
 */
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include "mpi.h"
#include "ompi/communicator/communicator.h"
#include "ompi/constants.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/mca/pml/pml.h"
#include "ompi/runtime/ompi_rte.h"
#include "opal/runtime/opal_progress.h"
#include "pml_rocm.h"
#include "pml_saved.h"
#include "ompi_amd.h"

extern int harness_dev_alloc_copy(void **d, const void *h, size_t bytes);
extern int harness_dev_copy_back(void *h, const void *d, size_t bytes);
extern int harness_dev_copy_in(void *d, const void *h, size_t bytes);
extern int harness_dev_free(void *d);

harness_proc_name_t harness_proc_name = {4343, 0};
struct ompi_datatype_t harness_mpi_byte = {0, 1, 1, 1};
mca_pml_base_module_t mca_pml;

static int g_rank, g_size;
/* where a rank is (stderr, shown when the test fails or hangs) */
#define SECTION(k) (fprintf(stderr, "rank %d: section %d\n", g_rank, (k)), fflush(stderr))
#define CHECK(c, ...)                                                             \
    do {                                                                          \
        if (!(c)) {                                                               \
            fprintf(stderr, "FAIL rank %d %s:%d: ", g_rank, __FILE__, __LINE__);  \
            fprintf(stderr, __VA_ARGS__);                                         \
            fprintf(stderr, " (library: %s)\n", ompi_amd_last_error());          \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

/* ---- the selected PML ("ob1"): count, complete at once ---- */
static int ob1_calls;
static ompi_request_t ob1_req;
static int o_add_comm(struct ompi_communicator_t *c) { return OMPI_SUCCESS; }
static int o_del_comm(struct ompi_communicator_t *c) { return OMPI_SUCCESS; }
/* tags at or below HARNESS_SYS_TAG: a real host transport (pml_saved.c);
 * HARNESS_PML_BENCH=1: every tag (the host_path A/B: ob1's place taken by
 * a one-copy-in, one-copy-out shared-memory transport, as btl/sm) */
static int g_ob1_all;
#define REAL(tag) ((tag) <= HARNESS_SYS_TAG || g_ob1_all)
static int o_isend(const void *b, size_t n, struct ompi_datatype_t *d, int dst, int tag,
                   mca_pml_base_send_mode_t m, struct ompi_communicator_t *c, ompi_request_t **r)
{
    ob1_calls++;
    *r = REAL(tag) ? harness_pml_saved_request(1, (void *) b, n, d, dst, tag, 0) : &ob1_req;
    return OMPI_SUCCESS;
}
static int o_send(const void *b, size_t n, struct ompi_datatype_t *d, int dst, int tag,
                  mca_pml_base_send_mode_t m, struct ompi_communicator_t *c)
{
    ob1_calls++;
    if (REAL(tag)) harness_pml_saved_send(b, n, d, dst, tag);
    return OMPI_SUCCESS;
}
static int o_irecv(void *b, size_t n, struct ompi_datatype_t *d, int src, int tag,
                   struct ompi_communicator_t *c, ompi_request_t **r)
{
    ob1_calls++;
    *r = REAL(tag) ? harness_pml_saved_request(0, b, n, d, src, tag, 0) : &ob1_req;
    return OMPI_SUCCESS;
}
static int o_recv(void *b, size_t n, struct ompi_datatype_t *d, int src, int tag,
                  struct ompi_communicator_t *c, ompi_status_public_t *s)
{
    ob1_calls++;
    if (REAL(tag))
        while (!harness_pml_saved_try_recv(b, n, d, src, tag, s)) opal_progress();
    return OMPI_SUCCESS;
}
static int o_isend_init(const void *b, size_t n, struct ompi_datatype_t *d, int dst, int tag,
                        mca_pml_base_send_mode_t m, struct ompi_communicator_t *c, ompi_request_t **r)
{
    ob1_calls++;
    *r = REAL(tag) ? harness_pml_saved_request(1, (void *) b, n, d, dst, tag, 1) : &ob1_req;
    return OMPI_SUCCESS;
}
static int o_irecv_init(void *b, size_t n, struct ompi_datatype_t *d, int src, int tag,
                        struct ompi_communicator_t *c, ompi_request_t **r)
{
    ob1_calls++;
    *r = REAL(tag) ? harness_pml_saved_request(0, b, n, d, src, tag, 1) : &ob1_req;
    return OMPI_SUCCESS;
}
static int o_start(size_t n, ompi_request_t **r) { ob1_calls++; return OMPI_SUCCESS; }
static int o_iprobe(int s, int t, struct ompi_communicator_t *c, int *m, ompi_status_public_t *st)
{ ob1_calls++; *m = 0; return OMPI_SUCCESS; }
static int o_probe(int s, int t, struct ompi_communicator_t *c, ompi_status_public_t *st)
{ ob1_calls++; return OMPI_SUCCESS; }
static int o_improbe(int s, int t, struct ompi_communicator_t *c, int *m, struct ompi_message_t **msg,
                     ompi_status_public_t *st)
{ ob1_calls++; *m = 0; return OMPI_SUCCESS; }
static int o_mprobe(int s, int t, struct ompi_communicator_t *c, struct ompi_message_t **msg,
                    ompi_status_public_t *st)
{ ob1_calls++; return OMPI_SUCCESS; }

static void wait_req(ompi_request_t *r)
{
    while (!REQUEST_COMPLETE(r)) opal_progress();
}

static unsigned char pat(int src, size_t i, int salt) { return (unsigned char)(src * 37 + i * 11 + salt); }

int main(int argc, char **argv)
{
    const int use_gpu = getenv("HARNESS_GPU") && atoi(getenv("HARNESS_GPU"));
    ompi_group_t local = {0};
    ompi_communicator_t comm;
    ompi_datatype_t dbyte = {0, 1, 1, 1}, dint = {6, 4, 1, 1}, gap4 = {6, 4, 0, 0};
    mca_pml_base_module_t ob1;
    int prio = 7;
    if (argc < 4) return 2;
    g_rank = atoi(argv[2]);
    g_size = atoi(argv[3]);
    harness_proc_name.jobid = (unsigned) strtoul(argv[1], NULL, 16);
    comm = (ompi_communicator_t){g_rank, g_size, 5, 0, &local, NULL};
    harness_pml_saved_init(argv[1], g_rank, g_size);

    /* the base selected "ob1" */
    memset(&ob1, 0, sizeof(ob1));
    ob1.pml_add_comm = o_add_comm;
    ob1.pml_del_comm = o_del_comm;
    ob1.pml_isend = o_isend;
    ob1.pml_send = o_send;
    ob1.pml_irecv = o_irecv;
    ob1.pml_recv = o_recv;
    ob1.pml_isend_init = o_isend_init;
    ob1.pml_irecv_init = o_irecv_init;
    ob1.pml_start = o_start;
    ob1.pml_iprobe = o_iprobe;
    ob1.pml_probe = o_probe;
    ob1.pml_improbe = o_improbe;
    ob1.pml_mprobe = o_mprobe;
    ob1.pml_max_tag = 0x7fffffff;
    mca_pml = ob1;

    /* selection: pml/rocm's init declines; its close interposes */
    CHECK(mca_pml_rocm_component.super.pmlm_version.mca_open_component() == OMPI_SUCCESS, "open");
    CHECK(mca_pml_rocm_component.super.pmlm_init(&prio, false, false) == NULL && prio < 0,
          "pml/rocm must never be selected");
    CHECK(mca_pml_rocm_component.super.pmlm_version.mca_close_component() == OMPI_SUCCESS, "close");
    CHECK(mca_pml_rocm_installed && mca_pml.pml_isend != o_isend && mca_pml_rocm_host.pml_isend == o_isend &&
              mca_pml.pml_max_tag == ob1.pml_max_tag,
          "close saves ob1 and installs pml/rocm");
    /* a lost message ends the run with a CHECK message instead of a hang */
    if (use_gpu) mca_pml_rocm_component.timeout_ms = 60000;
    CHECK(mca_pml.pml_add_comm(&comm) == OMPI_SUCCESS, "add_comm");
    if (!use_gpu) {
        int m = -1;
        ompi_request_t *r = NULL;
        CHECK(mca_pml_rocm_comm_of(&comm) == NULL, "no library communicator without a device");
        CHECK(mca_pml.pml_isend("x", 1, &dbyte, (g_rank + 1) % g_size, 3, MCA_PML_BASE_SEND_STANDARD,
                                &comm, &r) == OMPI_SUCCESS && r == &ob1_req && ob1_calls == 1,
              "isend reaches ob1");
        CHECK(mca_pml.pml_iprobe(MPI_ANY_SOURCE, MPI_ANY_TAG, &comm, &m, NULL) == OMPI_SUCCESS &&
                  ob1_calls == 2, "iprobe reaches ob1");
        CHECK(mca_pml.pml_del_comm(&comm) == OMPI_SUCCESS, "del_comm");
        harness_pml_saved_fini();
        printf("ok\n");
        return 0;
    }
    CHECK(mca_pml_rocm_comm_of(&comm) != NULL, "library communicator created");
    const int right = (g_rank + 1) % g_size, left = (g_rank + g_size - 1) % g_size;

    if (getenv("HARNESS_PML_BENCH") && atoi(getenv("HARNESS_PML_BENCH")) && g_size == 2) {
        /* host-buffer ping-pong through pml/rocm with
         * pml_rocm_host_path = 0 (the library's staged path) and 1 (the
         * saved PML, here the shared-memory transport above) */
        const size_t sizes[6] = {8, 1024, 16384, 65536, 131072, 262144};
        g_ob1_all = 1;
        for (int hp = 0; hp < 2; ++hp) {
            mca_pml_rocm_component.host_path = hp;
            for (int k = 0; k < 6; ++k) {
                const size_t n = sizes[k];
                const int iters = n <= 16384 ? 500 : 100;
                unsigned char *b = malloc(n);
                memset(b, g_rank, n);
                for (int it = -10; it < iters; ++it) {  /* 10 warm-up round trips */
                    static struct timespec t0;
                    if (it == 0) clock_gettime(CLOCK_MONOTONIC, &t0);
                    if (g_rank == 0) {
                        CHECK(mca_pml.pml_send(b, n, &dbyte, 1, 90, MCA_PML_BASE_SEND_STANDARD, &comm) ==
                                  OMPI_SUCCESS, "bench send");
                        CHECK(mca_pml.pml_recv(b, n, &dbyte, 1, 90, &comm, NULL) == OMPI_SUCCESS, "bench recv");
                    } else {
                        CHECK(mca_pml.pml_recv(b, n, &dbyte, 0, 90, &comm, NULL) == OMPI_SUCCESS, "bench recv");
                        CHECK(mca_pml.pml_send(b, n, &dbyte, 0, 90, MCA_PML_BASE_SEND_STANDARD, &comm) ==
                                  OMPI_SUCCESS, "bench send");
                    }
                    if (it == iters - 1 && g_rank == 0) {
                        struct timespec t1;
                        clock_gettime(CLOCK_MONOTONIC, &t1);
                        const double us = ((t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec)) /
                                          1e3 / iters / 2;  /* one way */
                        printf("{\"host_path\": %d, \"bytes\": %zu, \"one_way_us\": %.2f, \"GBps\": %.3f, "
                               "\"iters\": %d, \"path\": \"%s\"}\n", hp, n, us, n / us / 1e3, iters,
                               hp ? "saved PML (shm one-copy transport, ob1 + btl/sm stand-in)"
                                  : "library (pinned stage + device IPC)");
                        fflush(stdout);
                    }
                }
                free(b);
            }
        }
        CHECK(mca_pml.pml_del_comm(&comm) == OMPI_SUCCESS, "del_comm");
        harness_pml_saved_fini();
        return 0;
    }

    SECTION(1);
    /* 1. ring isend / irecv on device buffers */
    {
        const size_t sizes[5] = {0, 777, 4096, 300001, 8u << 20};
        for (int k = 0; k < 5; ++k) {
            const size_t n = sizes[k];
            unsigned char *h = malloc(n + 1), *exp = malloc(n + 1), *got = malloc(n + 1);
            void *ds, *dr;
            ompi_request_t *rs = NULL, *rr = NULL;
            for (size_t i = 0; i < n; ++i) {
                h[i] = pat(g_rank, i, k);
                exp[i] = pat(left, i, k);
            }
            memset(got, 0, n + 1);
            CHECK(harness_dev_alloc_copy(&ds, h, n + 1) == 0 && harness_dev_alloc_copy(&dr, got, n + 1) == 0,
                  "device buffers");
            ob1_calls = 0;
            CHECK(mca_pml.pml_irecv(dr, n, &dbyte, left, 10 + k, &comm, &rr) == OMPI_SUCCESS, "irecv");
            CHECK(mca_pml.pml_isend(ds, n, &dbyte, right, 10 + k, MCA_PML_BASE_SEND_STANDARD, &comm,
                                    &rs) == OMPI_SUCCESS, "isend");
            CHECK(ob1_calls == 0 && rr != &ob1_req && rs != &ob1_req, "user tags go to the library");
            wait_req(rr);
            wait_req(rs);
            CHECK(rr->req_status.MPI_ERROR == OMPI_SUCCESS && rr->req_status.MPI_SOURCE == left &&
                      rr->req_status.MPI_TAG == 10 + k && rr->req_status._ucount == n,
                  "recv status (err %d src %d tag %d count %zu)", rr->req_status.MPI_ERROR,
                  rr->req_status.MPI_SOURCE, rr->req_status.MPI_TAG, rr->req_status._ucount);
            CHECK(harness_dev_copy_back(got, dr, n + 1) == 0 && memcmp(got, exp, n) == 0,
                  "ring payload of %zu bytes", n);
            CHECK(rr->req_free(&rr) == OMPI_SUCCESS && rs->req_free(&rs) == OMPI_SUCCESS, "free");
            harness_dev_free(ds);
            harness_dev_free(dr);
            free(h);
            free(exp);
            free(got);
        }
    }
    SECTION(2);
    /* 2. blocking send / recv from host memory (staged through the device),
     * ANY_SOURCE / ANY_TAG on the receive */
    {
        const size_t n = 100003;
        int *h = malloc(n * 4), *got = calloc(n, 4);
        ompi_status_public_t st;
        for (size_t i = 0; i < n; ++i) h[i] = g_rank * 1000003 + (int) i;
        if (g_rank % 2 == 0) {
            CHECK(mca_pml.pml_send(h, n, &dint, right, 7, MCA_PML_BASE_SEND_STANDARD, &comm) ==
                      OMPI_SUCCESS, "send");
            CHECK(mca_pml.pml_recv(got, n, &dint, MPI_ANY_SOURCE, MPI_ANY_TAG, &comm, &st) == OMPI_SUCCESS,
                  "recv");
        } else {
            CHECK(mca_pml.pml_recv(got, n, &dint, MPI_ANY_SOURCE, MPI_ANY_TAG, &comm, &st) == OMPI_SUCCESS,
                  "recv");
            CHECK(mca_pml.pml_send(h, n, &dint, right, 7, MCA_PML_BASE_SEND_STANDARD, &comm) ==
                      OMPI_SUCCESS, "send");
        }
        CHECK(st.MPI_SOURCE == left && st.MPI_TAG == 7 && st._ucount == n * 4, "wildcard status");
        for (size_t i = 0; i < n; ++i) CHECK(got[i] == left * 1000003 + (int) i, "host payload %zu", i);
        free(h);
        free(got);
    }
    SECTION(3);
    /* 3. non-contiguous receive type: 4-byte elements with 4-byte gaps */
    {
        const size_t n = 5000;
        int *h = malloc(n * 4), *t = malloc(n * 8);
        void *ds;
        ompi_request_t *rs = NULL, *rr = NULL;
        for (size_t i = 0; i < n; ++i) h[i] = g_rank * 7919 + (int) i;
        for (size_t i = 0; i < 2 * n; ++i) t[i] = -1;
        CHECK(harness_dev_alloc_copy(&ds, h, n * 4) == 0, "device send buffer");
        CHECK(mca_pml.pml_irecv(t, n, &gap4, left, 9, &comm, &rr) == OMPI_SUCCESS, "irecv gap type");
        CHECK(mca_pml.pml_isend(ds, n, &dint, right, 9, MCA_PML_BASE_SEND_STANDARD, &comm, &rs) ==
                  OMPI_SUCCESS, "isend");
        wait_req(rr);
        wait_req(rs);
        for (size_t i = 0; i < n; ++i) {
            CHECK(t[2 * i] == left * 7919 + (int) i, "packed element %zu", i);
            CHECK(t[2 * i + 1] == -1, "gap %zu overwritten", i);
        }
        CHECK(rr->req_free(&rr) == OMPI_SUCCESS && rs->req_free(&rs) == OMPI_SUCCESS, "free");
        harness_dev_free(ds);
        free(h);
        free(t);
    }
    /* 3b. non-contiguous device buffers on both sides: packed and unpacked
     * on the device (common/rocm), no host copy of the payload; the
     * receive buffer's gaps survive */
    {
        extern int harness_device_packs;
        const size_t n = 70001;
        int *h = malloc(n * 8), *t = malloc(n * 8);
        void *ds, *dr;
        ompi_request_t *rs = NULL, *rr = NULL;
        const int packs0 = harness_device_packs;
        for (size_t i = 0; i < n; ++i) {
            h[2 * i] = g_rank * 104729 + (int) i;
            h[2 * i + 1] = -7;
        }
        for (size_t i = 0; i < 2 * n; ++i) t[i] = -1;
        CHECK(harness_dev_alloc_copy(&ds, h, n * 8) == 0 && harness_dev_alloc_copy(&dr, t, n * 8) == 0,
              "device gap buffers");
        CHECK(mca_pml.pml_irecv(dr, n, &gap4, left, 10, &comm, &rr) == OMPI_SUCCESS, "irecv device gap type");
        CHECK(mca_pml.pml_isend(ds, n, &gap4, right, 10, MCA_PML_BASE_SEND_STANDARD, &comm, &rs) ==
                  OMPI_SUCCESS, "isend device gap type");
        wait_req(rr);
        wait_req(rs);
        CHECK(harness_dev_copy_back(t, dr, n * 8) == 0, "copy back");
        for (size_t i = 0; i < n; ++i) {
            CHECK(t[2 * i] == left * 104729 + (int) i, "device packed element %zu", i);
            CHECK(t[2 * i + 1] == -1, "device gap %zu overwritten", i);
        }
        CHECK(harness_device_packs - packs0 == 2, "device pack + unpack (%d)", harness_device_packs - packs0);
        CHECK(rr->req_free(&rr) == OMPI_SUCCESS && rs->req_free(&rs) == OMPI_SUCCESS, "free");
        harness_dev_free(ds);
        harness_dev_free(dr);
        free(h);
        free(t);
    }
    SECTION(4);
    /* 4. iprobe / probe, then the receive */
    {
        unsigned char v = (unsigned char) g_rank, w = 0;
        void *dv, *dw;
        ompi_request_t *rs = NULL;
        ompi_status_public_t st;
        int m = 0;
        CHECK(harness_dev_alloc_copy(&dv, &v, 1) == 0 && harness_dev_alloc_copy(&dw, &w, 1) == 0, "dev");
        CHECK(mca_pml.pml_isend(dv, 1, &dbyte, right, 21, MCA_PML_BASE_SEND_STANDARD, &comm, &rs) ==
                  OMPI_SUCCESS, "isend");
        CHECK(mca_pml.pml_probe(left, MPI_ANY_TAG, &comm, &st) == OMPI_SUCCESS && st.MPI_TAG == 21 &&
                  st.MPI_SOURCE == left && st._ucount == 1, "probe");
        CHECK(mca_pml.pml_iprobe(MPI_ANY_SOURCE, 21, &comm, &m, &st) == OMPI_SUCCESS && m == 1, "iprobe");
        CHECK(mca_pml.pml_recv(dw, 1, &dbyte, left, 21, &comm, &st) == OMPI_SUCCESS, "recv");
        CHECK(harness_dev_copy_back(&w, dw, 1) == 0 && w == (unsigned char) left, "probed payload");
        wait_req(rs);
        CHECK(rs->req_free(&rs) == OMPI_SUCCESS, "free");
        harness_dev_free(dv);
        harness_dev_free(dw);
    }
    SECTION(5);
    /* 5. persistent send / recv, three starts with fresh data */
    {
        const size_t n = 65537;
        unsigned char *h = malloc(n), *got = malloc(n);
        void *ds, *dr;
        ompi_request_t *rs = NULL, *rr = NULL;
        memset(h, 0, n);
        CHECK(harness_dev_alloc_copy(&ds, h, n) == 0 && harness_dev_alloc_copy(&dr, h, n) == 0, "dev");
        CHECK(mca_pml.pml_isend_init(ds, n, &dbyte, right, 33, MCA_PML_BASE_SEND_STANDARD, &comm, &rs) ==
                  OMPI_SUCCESS && mca_pml.pml_irecv_init(dr, n, &dbyte, left, 33, &comm, &rr) ==
                  OMPI_SUCCESS, "persistent init");
        CHECK(rs->req_persistent && rr->req_persistent, "persistent requests");
        for (int it = 0; it < 3; ++it) {
            /* fresh data in the same buffer; the peer must see this start's */
            for (size_t i = 0; i < n; ++i) h[i] = pat(g_rank, i, 50 + it);
            CHECK(harness_dev_copy_in(ds, h, n) == 0, "fresh send data");
            CHECK(mca_pml.pml_start(1, &rr) == OMPI_SUCCESS, "start recv");
            CHECK(mca_pml.pml_start(1, &rs) == OMPI_SUCCESS, "start send");
            wait_req(rr);
            wait_req(rs);
            CHECK(rr->req_status.MPI_ERROR == OMPI_SUCCESS && rr->req_status._ucount == n, "status");
            CHECK(harness_dev_copy_back(got, dr, n) == 0, "copy back");
            for (size_t i = 0; i < n; ++i) CHECK(got[i] == pat(left, i, 50 + it), "start %d byte %zu", it, i);
        }
        CHECK(rr->req_free(&rr) == OMPI_SUCCESS && rs->req_free(&rs) == OMPI_SUCCESS, "free");
        harness_dev_free(ds);
        harness_dev_free(dr);
        free(h);
        free(got);
    }
    SECTION(6);
    /* 6. truncation: 1000 bytes into a 999-byte receive */
    {
        unsigned char h[1000] = {0};
        void *ds, *dr;
        ompi_request_t *rs = NULL, *rr = NULL;
        CHECK(harness_dev_alloc_copy(&ds, h, 1000) == 0 && harness_dev_alloc_copy(&dr, h, 1000) == 0, "dev");
        CHECK(mca_pml.pml_irecv(dr, 999, &dbyte, left, 44, &comm, &rr) == OMPI_SUCCESS, "irecv");
        CHECK(mca_pml.pml_isend(ds, 1000, &dbyte, right, 44, MCA_PML_BASE_SEND_STANDARD, &comm, &rs) ==
                  OMPI_SUCCESS, "isend");
        wait_req(rr);
        wait_req(rs);
        CHECK(rr->req_status.MPI_ERROR == MPI_ERR_TRUNCATE, "truncation reported (%d)",
              rr->req_status.MPI_ERROR);
        (void) rr->req_free(&rr);
        (void) rs->req_free(&rs);
        harness_dev_free(ds);
        harness_dev_free(dr);
    }
    SECTION(7);
    /* 7. system tags, PROC_NULL and matched probes */
    {
        ompi_request_t *r = NULL;
        int m = 0;
        struct ompi_message_t *msg = NULL;
        ob1_calls = 0;
        CHECK(mca_pml.pml_isend("x", 1, &dbyte, right, -17, MCA_PML_BASE_SEND_STANDARD, &comm, &r) ==
                  OMPI_SUCCESS && r == &ob1_req && ob1_calls == 1, "system tag reaches ob1");
        CHECK(mca_pml.pml_recv(NULL, 0, &dbyte, MPI_PROC_NULL, 3, &comm, NULL) == OMPI_SUCCESS &&
                  ob1_calls == 2, "PROC_NULL reaches ob1");
        CHECK(mca_pml.pml_improbe(left, 3, &comm, &m, &msg, NULL) == OMPI_ERR_NOT_SUPPORTED,
              "matched probe of library traffic refused");
        CHECK(mca_pml.pml_improbe(left, -20, &comm, &m, &msg, NULL) == OMPI_SUCCESS && ob1_calls == 3,
              "matched probe of a system tag reaches ob1");
    }
    SECTION(8);
    /* 8. MPI_Request_free of active requests (the oldest active request is
     * the list's tail): an in-flight Ssend and irecv, freed, leave the list */
    {
        const size_t n = 65536;
        unsigned char *h = malloc(n), *got = malloc(n);
        void *ds, *dr;
        ompi_request_t *rs = NULL, *rr = NULL;
        for (size_t i = 0; i < n; ++i) h[i] = pat(g_rank, i, 60);
        memset(got, 0, n);
        CHECK(harness_dev_alloc_copy(&ds, h, n) == 0 && harness_dev_alloc_copy(&dr, got, n) == 0, "dev");
        CHECK(mca_pml.pml_irecv(dr, n, &dbyte, left, 60, &comm, &rr) == OMPI_SUCCESS, "irecv");
        CHECK(mca_pml.pml_isend(ds, n, &dbyte, right, 60, MCA_PML_BASE_SEND_SYNCHRONOUS, &comm, &rs) ==
                  OMPI_SUCCESS, "issend");
        CHECK(mca_pml_rocm_active_count() == 2, "two active requests (%d)", mca_pml_rocm_active_count());
        CHECK(rr->req_free(&rr) == OMPI_SUCCESS, "free active irecv");
        CHECK(rs->req_free(&rs) == OMPI_SUCCESS, "free active issend");
        CHECK(mca_pml_rocm_active_count() == 0, "freed requests left on the active list (%d)",
              mca_pml_rocm_active_count());
        opal_progress();
        CHECK(harness_dev_copy_back(got, dr, n) == 0, "copy back");
        for (size_t i = 0; i < n; ++i) CHECK(got[i] == pat(left, i, 60), "freed irecv byte %zu", i);
        harness_dev_free(ds);
        harness_dev_free(dr);
        free(h);
        free(got);
    }
    SECTION(9);
    /* 9. the sender frees and reallocates its device buffer between
     * messages: staged (default: the receiver reads library memory) and
     * p2p_user_ipc = 1 (the receiver maps the send buffer; the IPC registry
     * retires the freed allocation's mapping) */
    {
        ompi_amd_comm_t *dev = mca_pml_rocm_comm_of(&comm);
        const size_t n = 8u << 20;
        unsigned char *h = malloc(n), *got = malloc(n);
        int64_t staged0 = 0, staged1 = 0, aged0 = 0, aged1 = 0, direct0 = 0, direct1 = 0;
        for (int mode = 0; mode < 2; ++mode) {
            CHECK(ompi_amd_comm_set_param(dev, "p2p_user_ipc", mode) == OMPI_AMD_SUCCESS, "p2p_user_ipc");
            (void) ompi_amd_comm_get_param(dev, "p2p_staged_sends", &staged0);
            (void) ompi_amd_comm_get_param(dev, "p2p_unsafe_sends", &aged0);
            (void) ompi_amd_comm_get_param(dev, "p2p_direct_sends", &direct0);
            for (int it = 0; it < 3; ++it) {
                void *ds, *dr;
                ompi_status_public_t st;
                for (size_t i = 0; i < n; i += 4099) h[i] = pat(g_rank, i, 70 + it + 3 * mode);
                memset(got, 0, n);
                CHECK(harness_dev_alloc_copy(&ds, h, n) == 0 && harness_dev_alloc_copy(&dr, got, n) == 0,
                      "dev");
                if (g_rank % 2 == 0) {
                    CHECK(mca_pml.pml_send(ds, n, &dbyte, right, 70, MCA_PML_BASE_SEND_STANDARD, &comm) ==
                              OMPI_SUCCESS, "send");
                    CHECK(mca_pml.pml_recv(dr, n, &dbyte, left, 70, &comm, &st) == OMPI_SUCCESS, "recv");
                } else {
                    CHECK(mca_pml.pml_recv(dr, n, &dbyte, left, 70, &comm, &st) == OMPI_SUCCESS, "recv");
                    CHECK(mca_pml.pml_send(ds, n, &dbyte, right, 70, MCA_PML_BASE_SEND_STANDARD, &comm) ==
                              OMPI_SUCCESS, "send");
                }
                CHECK(harness_dev_copy_back(got, dr, n) == 0, "copy back");
                for (size_t i = 0; i < n; i += 4099)
                    CHECK(got[i] == pat(left, i, 70 + it + 3 * mode), "mode %d round %d byte %zu", mode, it, i);
                harness_dev_free(ds);  /* freed while the peer may still hold a mapping of it */
                harness_dev_free(dr);
            }
            (void) ompi_amd_comm_get_param(dev, "p2p_staged_sends", &staged1);
            (void) ompi_amd_comm_get_param(dev, "p2p_unsafe_sends", &aged1);
            (void) ompi_amd_comm_get_param(dev, "p2p_direct_sends", &direct1);
            /* mode 0: every send staged.  mode 1: from the buffer itself,
             * except a buffer allocated before this rank closed an IPC
             * mapping (its receive retired the peer's freed buffer): ROCm
             * 7.2 may refuse to export that one, so it is
             * staged without being offered — no runtime refusal reaches the
             * send (the round-4 intermittent failure of this section) */
            CHECK(mode == 0 ? staged1 - staged0 == 3
                            : staged1 - staged0 == aged1 - aged0 && (staged1 - staged0) + (direct1 - direct0) == 3,
                  "mode %d: %lld staged sends, %lld aged, %lld direct", mode, (long long) (staged1 - staged0),
                  (long long) (aged1 - aged0), (long long) (direct1 - direct0));
            if (mode == 1)
                fprintf(stderr, "rank %d: user_ipc sends: %lld direct, %lld staged (older than an IPC close)\n",
                        g_rank, (long long) (direct1 - direct0), (long long) (aged1 - aged0));
        }
        (void) ompi_amd_comm_set_param(dev, "p2p_user_ipc", 0);
        free(h);
        free(got);
    }
    SECTION(10);
    /* 10. pml_rocm_host_path = 1: host-buffer operations reach ob1 and make
     * no library call; device buffers still go to the library */
    {
        ompi_amd_comm_t *dev = mca_pml_rocm_comm_of(&comm);
        int64_t hs0 = 0, hs1 = 0, hr0 = 0, hr1 = 0;
        int x = g_rank, y = -1, m = 0;
        ompi_request_t *r = NULL;
        mca_pml_rocm_component.host_path = 1;
        (void) ompi_amd_comm_get_param(dev, "p2p_host_sends", &hs0);
        (void) ompi_amd_comm_get_param(dev, "p2p_host_recvs", &hr0);
        ob1_calls = 0;
        CHECK(mca_pml.pml_send(&x, 1, &dint, right, 80, MCA_PML_BASE_SEND_STANDARD, &comm) == OMPI_SUCCESS,
              "host send");
        CHECK(mca_pml.pml_recv(&y, 1, &dint, left, 80, &comm, NULL) == OMPI_SUCCESS, "host recv");
        CHECK(mca_pml.pml_isend(&x, 1, &dint, right, 81, MCA_PML_BASE_SEND_STANDARD, &comm, &r) ==
                  OMPI_SUCCESS && r == &ob1_req, "host isend");
        CHECK(ob1_calls == 3, "host traffic reaches ob1 (%d calls)", ob1_calls);
        (void) ompi_amd_comm_get_param(dev, "p2p_host_sends", &hs1);
        (void) ompi_amd_comm_get_param(dev, "p2p_host_recvs", &hr1);
        CHECK(hs1 == hs0 && hr1 == hr0, "library calls for host traffic");
        CHECK(mca_pml.pml_iprobe(left, 99, &comm, &m, NULL) == OMPI_SUCCESS && m == 0 && ob1_calls == 4,
              "probe asks both engines");
        {
            void *dv, *dw;
            unsigned char v = (unsigned char) (g_rank + 1), w = 0;
            CHECK(harness_dev_alloc_copy(&dv, &v, 1) == 0 && harness_dev_alloc_copy(&dw, &w, 1) == 0, "dev");
            ob1_calls = 0;
            int src_rc = OMPI_SUCCESS, rcv_rc = OMPI_SUCCESS;
            if (g_rank % 2 == 0) {
                src_rc = mca_pml.pml_send(dv, 1, &dbyte, right, 82, MCA_PML_BASE_SEND_STANDARD, &comm);
                CHECK(src_rc == OMPI_SUCCESS, "device send: %d (%s)", src_rc, ompi_amd_last_error());
                rcv_rc = mca_pml.pml_recv(dw, 1, &dbyte, left, 82, &comm, NULL);
                CHECK(rcv_rc == OMPI_SUCCESS, "device recv: %d (%s)", rcv_rc, ompi_amd_last_error());
            } else {
                rcv_rc = mca_pml.pml_recv(dw, 1, &dbyte, left, 82, &comm, NULL);
                CHECK(rcv_rc == OMPI_SUCCESS, "device recv: %d (%s)", rcv_rc, ompi_amd_last_error());
                src_rc = mca_pml.pml_send(dv, 1, &dbyte, right, 82, MCA_PML_BASE_SEND_STANDARD, &comm);
                CHECK(src_rc == OMPI_SUCCESS, "device send: %d (%s)", src_rc, ompi_amd_last_error());
            }
            CHECK(ob1_calls == 0, "device traffic stays on the library under host_path");
            CHECK(harness_dev_copy_back(&w, dw, 1) == 0 && w == (unsigned char) (left + 1), "device payload");
            harness_dev_free(dv);
            harness_dev_free(dw);
        }
        mca_pml_rocm_component.host_path = 0;
    }
    SECTION(11);
    /* 11. system-tag traffic on device buffers (the collectives' own
     * messages: coll/base, libnbc): it stays on ob1, which moves host
     * memory only, through host copies of the typed spans — the transport
     * behind ob1 fails the run on any device pointer.  Nonblocking,
     * blocking, persistent (two starts), a gapped type whose receive gaps
     * must survive. */
    {
        const size_t n = 20000;
        const int tag = HARNESS_SYS_TAG - 5;
        int *h = malloc(n * 8), *t = malloc(n * 8);
        void *ds, *dr;
        ompi_request_t *rs = NULL, *rr = NULL;
        const int msgs0 = harness_saved_pml_msgs;
        for (int form = 0; form < 3; ++form) {
            for (int gap = 0; gap < 2; ++gap) {
                ompi_datatype_t *d = gap ? &gap4 : &dint;
                const int starts = form == 2 ? 2 : 1;
                for (size_t i = 0; i < 2 * n; ++i) h[i] = (int) (g_rank * 7001 + i * 3 + form * 11 + gap);
                for (size_t i = 0; i < 2 * n; ++i) t[i] = -1;
                CHECK(harness_dev_alloc_copy(&ds, h, n * 8) == 0 && harness_dev_alloc_copy(&dr, t, n * 8) == 0,
                      "device buffers");
                if (form == 2) {
                    CHECK(mca_pml.pml_irecv_init(dr, n, d, left, tag, &comm, &rr) == OMPI_SUCCESS &&
                              mca_pml.pml_isend_init(ds, n, d, right, tag, MCA_PML_BASE_SEND_STANDARD, &comm,
                                                     &rs) == OMPI_SUCCESS,
                          "persistent system-tag requests");
                }
                for (int st = 0; st < starts; ++st) {
                    if (st > 0) {  /* fresh data for the second start */
                        for (size_t i = 0; i < 2 * n; ++i) h[i] += 1000;
                        CHECK(harness_dev_copy_in(ds, h, n * 8) == 0, "refill");
                    }
                    if (form == 0) {
                        CHECK(mca_pml.pml_irecv(dr, n, d, left, tag, &comm, &rr) == OMPI_SUCCESS &&
                                  mca_pml.pml_isend(ds, n, d, right, tag, MCA_PML_BASE_SEND_STANDARD, &comm,
                                                    &rs) == OMPI_SUCCESS,
                              "nonblocking system-tag calls");
                    } else if (form == 2) {
                        CHECK(mca_pml.pml_start(1, &rr) == OMPI_SUCCESS &&
                                  mca_pml.pml_start(1, &rs) == OMPI_SUCCESS, "starts");
                    }
                    if (form == 1) {
                        CHECK(mca_pml.pml_send(ds, n, d, right, tag, MCA_PML_BASE_SEND_STANDARD, &comm) ==
                                  OMPI_SUCCESS, "blocking system-tag send");
                        CHECK(mca_pml.pml_recv(dr, n, d, left, tag, &comm, NULL) == OMPI_SUCCESS,
                              "blocking system-tag recv");
                    } else {
                        wait_req(rr);
                        wait_req(rs);
                        CHECK(rr->req_status.MPI_ERROR == OMPI_SUCCESS && rr->req_status._ucount == n * 4,
                              "system-tag receive status");
                    }
                    CHECK(harness_dev_copy_back(t, dr, n * 8) == 0, "copy back");
                    for (size_t i = 0; i < n; ++i) {
                        const size_t at = gap ? 2 * i : i;
                        const int want = (int) (left * 7001 + at * 3 + form * 11 + gap) + 1000 * st;
                        CHECK(t[at] == want, "form %d gap %d start %d element %zu: %d, want %d", form, gap, st,
                              i, t[at], want);
                        if (gap) CHECK(t[2 * i + 1] == -1, "gap %zu overwritten", i);
                    }
                }
                if (form != 1) {
                    CHECK(rr->req_free(&rr) == OMPI_SUCCESS && rs->req_free(&rs) == OMPI_SUCCESS, "free");
                }
                harness_dev_free(ds);
                harness_dev_free(dr);
            }
        }
        /* 2 messages per call pair, 4 one-start forms + 2 two-start ones */
        CHECK(harness_saved_pml_msgs - msgs0 == 2 * (2 + 2 + 4), "system-tag messages moved by the host "
              "transport: %d", harness_saved_pml_msgs - msgs0);
        free(h);
        free(t);
    }
    SECTION(12);
    /* 12. two system-tag receives in flight into ONE device buffer whose
     * typed spans interleave (the gapped type at offsets 0 and 4: each
     * one's elements sit in the other's gaps, as a linear gather into a
     * resized column type lays them out).  Each receive must write back
     * only the bytes it received: a whole-span copy of the second to
     * complete would put its stale pre-fill over the first one's data
     * (ADVICE r4, high). */
    {
        const size_t n = 12345;
        const int tag = HARNESS_SYS_TAG - 21;  /* tag and tag + 1: no other section uses them */
        int *h = malloc(n * 8), *t = malloc(n * 8);
        void *ds, *dr;
        ompi_request_t *ra = NULL, *rb = NULL;
        for (size_t i = 0; i < 2 * n; ++i) h[i] = (int) (g_rank * 9001 + i * 5 + 3);
        for (size_t i = 0; i < 2 * n; ++i) t[i] = -7;
        CHECK(harness_dev_alloc_copy(&ds, h, n * 8) == 0 && harness_dev_alloc_copy(&dr, t, n * 8) == 0,
              "device buffers");
        CHECK(mca_pml.pml_irecv(dr, n, &gap4, left, tag, &comm, &ra) == OMPI_SUCCESS &&
                  mca_pml.pml_irecv((char *) dr + 4, n, &gap4, left, tag + 1, &comm, &rb) == OMPI_SUCCESS,
              "two interleaved receives");
        /* the even elements of ds into the first, the odd ones into the second */
        CHECK(mca_pml.pml_send(ds, n, &gap4, right, tag, MCA_PML_BASE_SEND_STANDARD, &comm) == OMPI_SUCCESS &&
                  mca_pml.pml_send((char *) ds + 4, n, &gap4, right, tag + 1, MCA_PML_BASE_SEND_STANDARD,
                                   &comm) == OMPI_SUCCESS,
              "two sends");
        wait_req(ra);
        wait_req(rb);
        CHECK(ra->req_status.MPI_ERROR == OMPI_SUCCESS && rb->req_status.MPI_ERROR == OMPI_SUCCESS,
              "interleaved receive status");
        CHECK(harness_dev_copy_back(t, dr, n * 8) == 0, "copy back");
        for (size_t i = 0; i < 2 * n; ++i)
            CHECK(t[i] == (int) (left * 9001 + i * 5 + 3), "interleaved receives, int %zu: %d", i, t[i]);
        CHECK(ra->req_free(&ra) == OMPI_SUCCESS && rb->req_free(&rb) == OMPI_SUCCESS, "free");
        harness_dev_free(ds);
        harness_dev_free(dr);
        free(h);
        free(t);
    }
    CHECK(mca_pml.pml_del_comm(&comm) == OMPI_SUCCESS && mca_pml_rocm_comm_of(&comm) == NULL, "del_comm");
    harness_pml_saved_fini();
    printf("ok gpu\n");
    return 0;
}
