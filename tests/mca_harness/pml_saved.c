/*
 * TEST HARNESS ONLY.  A real host transport behind the stand-in "ob1" for
 * system tags at or below HARNESS_SYS_TAG (section 11 of pml_harness.c):
 * every message is packed through its datatype into a POSIX-shm mailbox of
 * the (source, destination) pair and unpacked into the receive buffer by
 * the receiver — read and written by the CPU, as ob1 over btl/sm does.  A
 * device pointer reaching it fails the run.  Sends are eager (complete at
 * once); receives match in posting order from opal_progress.
 */
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include "mpi.h"
#include "ompi/constants.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/request/request.h"
#include "opal/runtime/opal_progress.h"
#include "ompi_amd.h"
#include "pml_saved.h"

#define SLOTS 8
#define SLOT_BYTES ((size_t) 256 << 10)

struct slot {
    volatile int full;
    int tag;
    size_t bytes;
    char data[SLOT_BYTES];
};
struct pair {
    struct slot s[SLOTS];
    volatile unsigned long posted, taken;
};

static struct pair *g_box;
static int g_me, g_n;
static char g_name[96];
int harness_saved_pml_msgs;

static void die(const char *what)
{
    fprintf(stderr, "FAIL rank %d saved PML stand-in: %s\n", g_me, what);
    exit(1);
}

void harness_pml_saved_init(const char *segment, int rank, int size)
{
    const size_t bytes = sizeof(struct pair) * (size_t) size * (size_t) size;
    int fd;
    g_me = rank;
    g_n = size;
    snprintf(g_name, sizeof(g_name), "/pml_saved_%s", segment);
    fd = shm_open(g_name, O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t) bytes) != 0) die("shm_open");
    g_box = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (MAP_FAILED == (void *) g_box) die("mmap");
}

void harness_pml_saved_fini(void)
{
    if (0 == g_me) shm_unlink(g_name);
}

static struct pair *pair_of(int src, int dst) { return &g_box[src * g_n + dst]; }

static void host_only(const void *p, size_t count)
{
    if (count && NULL != p && ompi_amd_is_device_pointer(p)) die("device memory reached the saved PML");
}

static size_t stride_of(const ompi_datatype_t *d) { return d->contiguous ? d->size : 2 * d->size; }

void harness_pml_saved_send(const void *buf, size_t count, const ompi_datatype_t *d, int dst, int tag)
{
    struct pair *p = pair_of(g_me, dst);
    const size_t bytes = count * d->size;
    host_only(buf, count);
    if (bytes > SLOT_BYTES) die("message larger than a mailbox slot");
    while (p->posted - __atomic_load_n(&p->taken, __ATOMIC_ACQUIRE) >= SLOTS) sched_yield();
    struct slot *s = &p->s[p->posted % SLOTS];
    if (d->contiguous) memcpy(s->data, buf, bytes);
    else
        for (size_t i = 0; i < count; ++i)
            memcpy(s->data + i * d->size, (const char *) buf + i * stride_of(d), d->size);
    s->tag = tag;
    s->bytes = bytes;
    __atomic_store_n(&s->full, 1, __ATOMIC_RELEASE);
    __atomic_add_fetch(&p->posted, 1, __ATOMIC_RELEASE);
    ++harness_saved_pml_msgs;
}

/* the oldest message of src with tag, unpacked into buf; 0: none yet */
int harness_pml_saved_try_recv(void *buf, size_t count, const ompi_datatype_t *d, int src, int tag,
                               ompi_status_public_t *st)
{
    struct pair *p = pair_of(src, g_me);
    host_only(buf, count);
    if (__atomic_load_n(&p->posted, __ATOMIC_ACQUIRE) == p->taken) return 0;
    struct slot *s = &p->s[p->taken % SLOTS];
    if (!__atomic_load_n(&s->full, __ATOMIC_ACQUIRE)) return 0;
    if (s->tag != tag) {
        fprintf(stderr, "saved PML stand-in: receive (src %d, tag %d) found tag %d at the head\n", src, tag,
                s->tag);
        die("message order: another tag at the head of the mailbox");
    }
    if (s->bytes > count * d->size) die("truncation");
    if (d->contiguous) memcpy(buf, s->data, s->bytes);
    else
        for (size_t i = 0; i < s->bytes / d->size; ++i)
            memcpy((char *) buf + i * stride_of(d), s->data + i * d->size, d->size);
    if (st) {
        st->MPI_SOURCE = src;
        st->MPI_TAG = tag;
        st->MPI_ERROR = OMPI_SUCCESS;
        st->_ucount = s->bytes;
    }
    __atomic_store_n(&s->full, 0, __ATOMIC_RELEASE);
    __atomic_add_fetch(&p->taken, 1, __ATOMIC_RELEASE);
    ++harness_saved_pml_msgs;
    return 1;
}

/* ---- requests: receives complete from opal_progress, sends at once ---- */
typedef struct sreq {
    ompi_request_t super;
    int is_send;
    void *buf;
    size_t count;
    const ompi_datatype_t *d;
    int peer, tag;
    struct sreq *next;
} sreq;

static sreq *g_pending;

/* Receives match in posting order per source: once one pending receive of
 * a source finds nothing, the later ones of that source wait too (the
 * message at the head may be the earlier receive's, still being posted) —
 * so a head whose tag differs from the first pending receive's is an order
 * error. */
static int s_progress(void)
{
    int n = 0;
    unsigned long long blocked = 0;  /* sources (< 64) with an unmatched earlier receive */
    for (sreq **pp = &g_pending; *pp;) {
        sreq *q = *pp;
        const unsigned long long bit = 1ull << (q->peer & 63);
        if (blocked & bit) {
            pp = &q->next;
            continue;
        }
        if (harness_pml_saved_try_recv(q->buf, q->count, q->d, q->peer, q->tag, &q->super.req_status)) {
            *pp = q->next;
            ompi_request_complete(&q->super, true);
            ++n;
        } else {
            blocked |= bit;
            pp = &q->next;
        }
    }
    return n;
}

static void s_launch(sreq *q)
{
    q->super.req_state = OMPI_REQUEST_ACTIVE;
    q->super.req_status.MPI_ERROR = OMPI_SUCCESS;
    if (q->is_send) {
        harness_pml_saved_send(q->buf, q->count, q->d, q->peer, q->tag);
        ompi_request_complete(&q->super, true);
        return;
    }
    q->super.req_complete = REQUEST_PENDING;
    q->next = NULL;  /* posting order: receives match in the order they were posted (MPI) */
    {
        sreq **pp = &g_pending;
        while (*pp) pp = &(*pp)->next;
        *pp = q;
    }
    (void) opal_progress_register(s_progress);
}

static int s_start(size_t count, ompi_request_t **reqs)
{
    for (size_t i = 0; i < count; ++i) s_launch((sreq *) reqs[i]);
    return OMPI_SUCCESS;
}

static int s_free(ompi_request_t **rq)
{
    if (!REQUEST_COMPLETE(*rq)) die("request freed before it completed");
    free(*rq);
    *rq = MPI_REQUEST_NULL;
    return OMPI_SUCCESS;
}

ompi_request_t *harness_pml_saved_request(int is_send, void *buf, size_t count, const ompi_datatype_t *d,
                                          int peer, int tag, int persistent)
{
    sreq *q = calloc(1, sizeof(*q));
    host_only(buf, count);
    OMPI_REQUEST_INIT(&q->super, persistent);
    q->super.req_type = OMPI_REQUEST_PML;
    q->super.req_start = s_start;
    q->super.req_free = s_free;
    q->is_send = is_send;
    q->buf = buf;
    q->count = count;
    q->d = d;
    q->peer = peer;
    q->tag = tag;
    if (!persistent) s_launch(q);
    return &q->super;
}
