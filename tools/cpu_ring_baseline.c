/*
 * CPU baseline for BASELINE configs[0] (MPI_Allreduce SUM FLOAT, N host
 * processes): a restatement of coll/tuned's ring_segmented allreduce
 * (coll_base_allreduce.c:618-856, 1 MiB segments) over POSIX shared memory,
 * with op/base's loop (the oracle's orc_op_2buff) as the reduction.  It
 * stands in for `mpirun -np N --mca btl self,vader` because no Open MPI
 * install exists on the box and the reference cannot be built
 * (BASELINE.md §5 "Otherwise").  Reported as a baseline, never the target.
 *
 * Transport: rank r writes each message into its right neighbour's mailbox
 * (two 1 MiB slots, like the reference's inbuf[2]); the receiver reduces
 * straight out of the mailbox — one copy per byte, the cost of btl/sm's
 * single-copy path.
 *
 * usage: cpu_ring_baseline <nranks> <bytes> <warmup> <iters> [<in> <out>]
 * prints one JSON line (rank 0): median seconds, GB/s, busBW.  With <in> and
 * <out>, rank r reads its input from the raw float32 file <in>.<r> instead of
 * generating dataset E and writes its result to <out>.<r>: the CPU test
 * (tests/test_coll_cpu.py) feeds dataset R this way and compares every
 * element bit-exactly with the oracle's ring_segmented.
 */
#define _GNU_SOURCE
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "../oracle/oracle.h"

#define SEGSIZE (1u << 20) /* coll_tuned_allreduce_algorithm_segmentsize */

typedef struct {
    _Atomic uint64_t full[2];   /* sequence number of the message in slot */
    _Atomic uint64_t freed[2];  /* sequence number the receiver released */
    char pad[32];
} mailbox_t;

typedef struct {
    _Atomic uint64_t barrier_count;
    _Atomic uint64_t barrier_gen;
    char pad[48];
} ctl_t;

static mailbox_t *boxes;
static char *slots;     /* [N][2][slot_bytes]: mailbox r's two message slots */
static size_t slot_bytes;
static ctl_t *ctl;
static int N;

static char *slot_data(int box, int slot)
{
    return slots + ((size_t) box * 2 + (size_t) slot) * slot_bytes;
}

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void barrier(void)
{
    uint64_t gen = atomic_load(&ctl->barrier_gen);
    if (atomic_fetch_add(&ctl->barrier_count, 1) == (uint64_t) N - 1) {
        atomic_store(&ctl->barrier_count, 0);
        atomic_fetch_add(&ctl->barrier_gen, 1);
    } else {
        while (atomic_load(&ctl->barrier_gen) == gen) sched_yield();
    }
}

/* per-direction message counters (sender side and receiver side) */
static uint64_t sent_seq, recv_seq;

static void send_to(int dst, const void *buf, size_t bytes)
{
    mailbox_t *b = &boxes[dst];
    uint64_t s = ++sent_seq;
    int slot = (int) (s & 1);
    /* wait until the receiver released the message two sends ago */
    while (s > 2 && atomic_load_explicit(&b->freed[slot], memory_order_acquire) < s - 2)
        sched_yield();
    memcpy(slot_data(dst, slot), buf, bytes);
    atomic_store_explicit(&b->full[slot], s, memory_order_release);
}

static const void *recv_wait(int me)
{
    mailbox_t *b = &boxes[me];
    uint64_t s = ++recv_seq;
    int slot = (int) (s & 1);
    while (atomic_load_explicit(&b->full[slot], memory_order_acquire) < s) sched_yield();
    return slot_data(me, slot);
}

static void recv_done(int me)
{
    mailbox_t *b = &boxes[me];
    atomic_store_explicit(&b->freed[recv_seq & 1], recv_seq, memory_order_release);
}

static void blockcount(size_t count, size_t n, size_t *split, size_t *early, size_t *late)
{
    *early = *late = count / n;
    *split = count % n;
    if (*split) *early += 1;
}

/* The phase count of ring_segmented (coll_base_allreduce.c:661-665); below
   N segments the reference runs the plain ring (:655-659), i.e. one phase. */
static size_t phases(size_t count)
{
    const size_t seg = SEGSIZE / sizeof(float);
    size_t nph = count / ((size_t) N * seg);
    if ((count % ((size_t) N * seg) >= (size_t) N) &&
        (count % ((size_t) N * seg) > ((size_t) N * seg) / 2))
        nph++;
    return nph ? nph : 1;
}

/* The largest message: a phase segment of an early block (the reference's
   max_segcount, :674-678), which exceeds the segment size by up to half of
   it; the allgather's fragments are at most one segment. */
static size_t max_message(size_t count)
{
    size_t split, early, late, sp, e, l;
    blockcount(count, (size_t) N, &split, &early, &late);
    blockcount(early, phases(count), &sp, &e, &l);
    return (e > SEGSIZE / sizeof(float) ? e : SEGSIZE / sizeof(float)) * sizeof(float);
}

/* ring_segmented, float SUM: the reference's phase / block / segment plan */
static void allreduce(int r, const float *sbuf, float *rbuf, size_t count)
{
    const size_t seg = SEGSIZE / sizeof(float);
    size_t split, early, late, nph = phases(count), ph;
    int k;
    memcpy(rbuf, sbuf, count * sizeof(float));
    blockcount(count, (size_t) N, &split, &early, &late);
    for (ph = 0; ph < nph; ph++) {
#define RANGE(b, off, cnt)                                                        \
    do {                                                                          \
        size_t bc_ = ((size_t) (b) < split) ? early : late;                       \
        size_t bo_ = ((size_t) (b) < split) ? (size_t) (b) * early                 \
                                            : (size_t) (b) * late + split;         \
        size_t sp_, e_, l_;                                                       \
        blockcount(bc_, nph, &sp_, &e_, &l_);                                     \
        cnt = (ph < sp_) ? e_ : l_;                                               \
        off = bo_ + ((ph < sp_) ? ph * e_ : ph * l_ + sp_);                       \
    } while (0)
        size_t off, cnt;
        RANGE(r, off, cnt);
        send_to((r + 1) % N, rbuf + off, cnt * sizeof(float));
        for (k = 2; k < N; k++) {
            int prev = (r + N - k + 1) % N;
            const void *in = recv_wait(r);
            RANGE(prev, off, cnt);
            orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, in, rbuf + off, cnt);
            recv_done(r);
            send_to((r + 1) % N, rbuf + off, cnt * sizeof(float));
        }
        {
            const void *in = recv_wait(r);
            RANGE((r + 1) % N, off, cnt);
            orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, in, rbuf + off, cnt);
            recv_done(r);
        }
#undef RANGE
    }
    /* ring allgather of whole blocks, in mailbox-sized fragments */
    for (k = 0; k < N - 1; k++) {
        size_t sb = (size_t) ((r + 1 + N - k) % N), rb = (size_t) ((r + N - k) % N);
        size_t soff = sb < split ? sb * early : sb * late + split;
        size_t scnt = sb < split ? early : late;
        size_t roff = rb < split ? rb * early : rb * late + split;
        size_t rcnt = rb < split ? early : late;
        size_t done_s = 0, done_r = 0;
        while (done_s < scnt || done_r < rcnt) {
            if (done_s < scnt) {
                size_t c = scnt - done_s < seg ? scnt - done_s : seg;
                send_to((r + 1) % N, rbuf + soff + done_s, c * sizeof(float));
                done_s += c;
            }
            if (done_r < rcnt) {
                size_t c = rcnt - done_r < seg ? rcnt - done_r : seg;
                const void *in = recv_wait(r);
                memcpy(rbuf + roff + done_r, in, c * sizeof(float));
                recv_done(r);
                done_r += c;
            }
        }
    }
}

static int cmp(const void *a, const void *b)
{
    double x = *(const double *) a, y = *(const double *) b;
    return (x > y) - (x < y);
}

int main(int argc, char **argv)
{
    size_t bytes, count;
    int warm, iters, r;
    double *times;
    const char *in_prefix = NULL, *out_prefix = NULL;
    if (argc != 5 && argc != 7) {
        fprintf(stderr, "usage: %s nranks bytes warmup iters [in-prefix out-prefix]\n", argv[0]);
        return 2;
    }
    if (argc == 7) {
        in_prefix = argv[5];
        out_prefix = argv[6];
    }
    N = atoi(argv[1]);
    bytes = strtoull(argv[2], NULL, 10);
    warm = atoi(argv[3]);
    iters = atoi(argv[4]);
    count = bytes / sizeof(float);
    boxes = mmap(NULL, sizeof(mailbox_t) * (size_t) N, PROT_READ | PROT_WRITE,
                 MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    slot_bytes = (max_message(count) + 63) & ~(size_t) 63;
    slots = mmap(NULL, slot_bytes * 2 * (size_t) N, PROT_READ | PROT_WRITE,
                 MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (boxes == MAP_FAILED || slots == MAP_FAILED) {
        perror("mmap");
        return 1;
    }
    ctl = mmap(NULL, sizeof(ctl_t), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    times = mmap(NULL, sizeof(double) * (size_t) iters * (size_t) N, PROT_READ | PROT_WRITE,
                 MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    memset(boxes, 0, sizeof(mailbox_t) * (size_t) N);
    memset(ctl, 0, sizeof(ctl_t));
    for (r = 0; r < N; r++) {
        if (fork() == 0) {
            float *s = malloc(bytes), *o = malloc(bytes);
            size_t i;
            int it;
            cpu_set_t set;
            CPU_ZERO(&set);
            CPU_SET(r % (int) sysconf(_SC_NPROCESSORS_ONLN), &set);
            sched_setaffinity(0, sizeof(set), &set);  /* --bind-to core */
            if (in_prefix) {  /* the caller's input (dataset R in the CPU test) */
                char path[4096];
                FILE *f;
                snprintf(path, sizeof(path), "%s.%d", in_prefix, r);
                f = fopen(path, "rb");
                if (!f || fread(s, 1, bytes, f) != bytes) {
                    fprintf(stderr, "rank %d: cannot read %s\n", r, path);
                    _exit(1);
                }
                fclose(f);
            } else {
                for (i = 0; i < count; i++)  /* dataset E: k * 2^-8 */
                    s[i] = (float) ((int) ((i * 2654435761u + (unsigned) r * 97u) % 2049u) - 1024) / 256.0f;
            }
            for (it = 0; it < warm + iters; it++) {
                double t0;
                barrier();
                t0 = now();
                allreduce(r, s, o, count);
                barrier();
                if (it >= warm) times[(size_t) (it - warm) * N + r] = now() - t0;
            }
            if (out_prefix) {  /* the result, for the caller's comparison */
                char path[4096];
                FILE *f;
                snprintf(path, sizeof(path), "%s.%d", out_prefix, r);
                f = fopen(path, "wb");
                if (!f || fwrite(o, 1, bytes, f) != bytes) {
                    fprintf(stderr, "rank %d: cannot write %s\n", r, path);
                    _exit(1);
                }
                fclose(f);
                _exit(0);
            }
            /* dataset E sums exactly in any order: check every element */
            for (i = 0; i < count; i++) {
                float e = 0.0f;
                int q;
                for (q = 0; q < N; q++)
                    e += (float) ((int) ((i * 2654435761u + (unsigned) q * 97u) % 2049u) - 1024) / 256.0f;
                if (e != o[i]) {
                    fprintf(stderr, "rank %d: wrong result at %zu\n", r, i);
                    _exit(1);
                }
            }
            _exit(0);
        }
    }
    for (r = 0; r < N; r++) {
        int st = 0;
        wait(&st);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
            fprintf(stderr, "a rank failed\n");
            return 1;
        }
    }
    {
        double *mx = malloc(sizeof(double) * (size_t) iters), med, gbs;
        int it;
        for (it = 0; it < iters; it++) {
            mx[it] = 0;
            for (r = 0; r < N; r++)
                if (times[(size_t) it * N + r] > mx[it]) mx[it] = times[(size_t) it * N + r];
        }
        qsort(mx, (size_t) iters, sizeof(double), cmp);
        med = mx[iters / 2];
        gbs = (double) bytes / med / 1e9;
        printf("{\"baseline\": \"cpu ring_segmented restatement over POSIX shm (oracle op/base loop)\", "
               "\"nranks\": %d, \"bytes\": %zu, \"median_s\": %.6f, \"algbw_GBps\": %.3f, "
               "\"busbw_GBps\": %.3f, \"cores\": %d, \"warmup\": %d, \"iters\": %d}\n",
               N, bytes, med, gbs, gbs * 2.0 * (N - 1) / N, N, warm, iters);
    }
    return 0;
}
