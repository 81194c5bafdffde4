/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Message-flow simulation of coll/base's allreduce algorithms over N
 * in-memory ranks.  Every reduction goes through orc_op_2buff with the same
 * (source, target) roles as the reference's ompi_op_reduce(op, source,
 * target) calls, so the per-element operand order — and therefore fp bits,
 * NaN and signed-zero results — is the reference's.
 *
 *   decision          coll_tuned_decision_fixed.c:45-89
 *   recursive doubl.  coll_base_allreduce.c:130-274
 *   ring              coll_base_allreduce.c:341-536
 *   ring segmented    coll_base_allreduce.c:618-856
 *   basic linear      coll_base_allreduce.c:881-912 (linear reduce to 0 + bcast)
 *   nonoverlapping    coll_base_allreduce.c:54-86 (tuned reduce to 0 + bcast)
 *   redscat_allgather coll_base_allreduce.c:970-1243 (Rabenseifner)
 *   forced selection  coll_tuned_allreduce_decision.c:130-150
 *   block partition   coll_base_functions.h:425-431 (COMPUTE_BLOCKCOUNT)
 *   segment count     coll_base_functions.h:407-416 (COMPUTED_SEGCOUNT)
 *
 * Closed forms these reduce to (verified against the reference in
 * SURVEY.md §8c): ring block b = x[b-1] (+) (x[b-2] (+) (... (x[b+1] (+) x[b])))
 * with out=left, in=right; recursive doubling (pof2) = pairwise tree.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

void orc_blockcount(size_t count, int nblocks, size_t *split, size_t *early,
                    size_t *late)
{
    *early = *late = count / (size_t)nblocks;
    *split = count % (size_t)nblocks;
    if (*split != 0) *early += 1;
}

static size_t block_offset(size_t b, size_t split, size_t early, size_t late)
{
    return (b < split) ? b * early : b * late + split;
}

static size_t block_count(size_t b, size_t split, size_t early, size_t late)
{
    return (b < split) ? early : late;
}

/* ---------------- recursive doubling ---------------- */
static int ar_recursive_doubling(int n, const void *const *sb, void *const *rb,
                                 size_t count, int op, int type)
{
    const size_t ext = orc_type_extent(type), bytes = count * ext;
    char **tmp = calloc((size_t)n, sizeof(char *));
    char **snd = calloc((size_t)n, sizeof(char *)), **rcv = calloc((size_t)n, sizeof(char *));
    char **msg = calloc((size_t)n, sizeof(char *));
    int *newrank = calloc((size_t)n, sizeof(int));
    int r, adjsize = 1, extra, distance;

    for (r = 0; r < n; r++) {
        tmp[r] = malloc(bytes ? bytes : 1);
        msg[r] = malloc(bytes ? bytes : 1);
        memcpy(tmp[r], sb[r], bytes);       /* inplacebuf <- sbuf (:165-168) */
        snd[r] = tmp[r];                    /* tmpsend = inplacebuf (:171) */
        rcv[r] = (char *)rb[r];             /* tmprecv = rbuf (:172) */
    }
    while (adjsize <= n) adjsize <<= 1;     /* opal_next_poweroftwo(size) >> 1 */
    adjsize >>= 1;
    extra = n - adjsize;

    /* non-pof2 fold (:184-203) */
    for (r = 0; r < n; r++) memcpy(msg[r], snd[r], bytes);
    for (r = 0; r < n; r++) {
        if (r < 2 * extra) {
            if (r % 2 == 0) {
                newrank[r] = -1;
            } else {
                memcpy(rcv[r], msg[r - 1], bytes);
                orc_op_2buff(op, type, rcv[r], snd[r], count); /* tmpsend = tmprecv op tmpsend */
                newrank[r] = r >> 1;
            }
        } else {
            newrank[r] = r - extra;
        }
    }
    /* exchange loop (:210-236) */
    for (distance = 1; distance < adjsize; distance <<= 1) {
        for (r = 0; r < n; r++) memcpy(msg[r], snd[r], bytes);
        for (r = 0; r < n; r++) {
            int newremote, remote;
            if (newrank[r] < 0) continue;
            newremote = newrank[r] ^ distance;
            remote = (newremote < extra) ? (newremote * 2 + 1) : (newremote + extra);
            memcpy(rcv[r], msg[remote], bytes);
            if (r < remote) {
                char *sw;
                orc_op_2buff(op, type, snd[r], rcv[r], count); /* tmprecv = tmpsend op tmprecv */
                sw = rcv[r]; rcv[r] = snd[r]; snd[r] = sw;
            } else {
                orc_op_2buff(op, type, rcv[r], snd[r], count); /* tmpsend = tmprecv op tmpsend */
            }
        }
    }
    /* unfold (:243-258) + final copy (:261-264) */
    for (r = 0; r < n; r++) memcpy(msg[r], snd[r], bytes);
    for (r = 0; r < n; r++) {
        if (r < 2 * extra && r % 2 == 0) {
            memcpy(rb[r], msg[r + 1], bytes);
        } else if (snd[r] != (char *)rb[r]) {
            memmove(rb[r], snd[r], bytes);
        }
    }
    for (r = 0; r < n; r++) { free(tmp[r]); free(msg[r]); }
    free(tmp); free(snd); free(rcv); free(msg); free(newrank);
    return ORC_AR_RECURSIVE_DOUBLING;
}

/* ---------------- ring (one pass over sub-ranges) ----------------
 * Runs the reduce-scatter half of the ring on, for every block b, the
 * element range [block_offset(b) + sub_off(b), +sub_cnt(b)).  With
 * sub = whole block this is the plain ring (:423-500); with sub = phase
 * segment it is one phase of ring_segmented (:700-812). */
typedef struct {
    size_t split, early, late;       /* block partition */
    int nphases;                     /* 1 = plain ring */
    int phase;
} ring_part_t;

static void phase_range(const ring_part_t *p, size_t b, size_t *off, size_t *cnt)
{
    size_t bc = block_count(b, p->split, p->early, p->late);
    size_t bo = block_offset(b, p->split, p->early, p->late);
    size_t sp, e, l;
    if (p->nphases == 1) { *off = bo; *cnt = bc; return; }
    orc_blockcount(bc, p->nphases, &sp, &e, &l);
    *cnt = ((size_t)p->phase < sp) ? e : l;
    *off = bo + (((size_t)p->phase < sp) ? (size_t)p->phase * e
                                        : (size_t)p->phase * l + sp);
}

static void ring_reduce_pass(int n, void *const *rb, const ring_part_t *part,
                             int op, int type, char **msg, char **nmsg)
{
    const size_t ext = orc_type_extent(type);
    size_t *mcnt = calloc((size_t)n, sizeof(size_t)), *ncnt = calloc((size_t)n, sizeof(size_t));
    int r, k;
    /* first send: my block (:437-446) */
    for (r = 0; r < n; r++) {
        size_t off, cnt;
        phase_range(part, (size_t)r, &off, &cnt);
        memcpy(msg[r], (char *)rb[r] + off * ext, cnt * ext);
        mcnt[r] = cnt;
    }
    for (k = 2; k < n; k++) {                   /* :448-472 */
        for (r = 0; r < n; r++) {
            int from = (r + n - 1) % n, prevblock = (r + n - k + 1) % n;
            size_t off, cnt;
            phase_range(part, (size_t)prevblock, &off, &cnt);
            orc_op_2buff(op, type, msg[from], (char *)rb[r] + off * ext, cnt);
            memcpy(nmsg[r], (char *)rb[r] + off * ext, cnt * ext);
            ncnt[r] = cnt;
        }
        for (r = 0; r < n; r++) {
            char *t = msg[r]; msg[r] = nmsg[r]; nmsg[r] = t;
            mcnt[r] = ncnt[r];
        }
    }
    for (r = 0; r < n; r++) {                   /* last block (:478-492) */
        int from = (r + n - 1) % n, b = (r + 1) % n;
        size_t off, cnt;
        phase_range(part, (size_t)b, &off, &cnt);
        orc_op_2buff(op, type, msg[from], (char *)rb[r] + off * ext, cnt);
    }
    free(mcnt); free(ncnt);
}

static void ring_allgather(int n, void *const *rb, const ring_part_t *part,
                           int type, char **msg)
{
    const size_t ext = orc_type_extent(type);
    int r, k;
    for (k = 0; k < n - 1; k++) {               /* :495-519 / :817-841 */
        for (r = 0; r < n; r++) {
            size_t b = (size_t)((r + 1 + n - k) % n);
            size_t off = block_offset(b, part->split, part->early, part->late);
            size_t cnt = block_count(b, part->split, part->early, part->late);
            memcpy(msg[r], (char *)rb[r] + off * ext, cnt * ext);
        }
        for (r = 0; r < n; r++) {
            int from = (r + n - 1) % n;
            size_t b = (size_t)((r + n - k) % n);
            size_t off = block_offset(b, part->split, part->early, part->late);
            size_t cnt = block_count(b, part->split, part->early, part->late);
            memcpy((char *)rb[r] + off * ext, msg[from], cnt * ext);
        }
    }
}

static int ar_ring_common(int n, const void *const *sb, void *const *rb,
                          size_t count, int op, int type, int nphases)
{
    const size_t ext = orc_type_extent(type);
    ring_part_t part;
    char **msg = calloc((size_t)n, sizeof(char *)), **nmsg = calloc((size_t)n, sizeof(char *));
    size_t maxb;
    int r;
    orc_blockcount(count, n, &part.split, &part.early, &part.late);
    maxb = part.early * ext + 1;
    for (r = 0; r < n; r++) {
        msg[r] = malloc(maxb);
        nmsg[r] = malloc(maxb);
        if (sb[r] != rb[r]) memcpy(rb[r], sb[r], count * ext);
    }
    part.nphases = nphases;
    for (part.phase = 0; part.phase < nphases; part.phase++)
        ring_reduce_pass(n, rb, &part, op, type, msg, nmsg);
    ring_allgather(n, rb, &part, type, msg);
    for (r = 0; r < n; r++) { free(msg[r]); free(nmsg[r]); }
    free(msg); free(nmsg);
    return ORC_AR_RING;
}

static int ar_ring(int n, const void *const *sb, void *const *rb, size_t count,
                   int op, int type)
{
    if (count < (size_t)n)                     /* :371-377 */
        return ar_recursive_doubling(n, sb, rb, count, op, type);
    return ar_ring_common(n, sb, rb, count, op, type, 1);
}

static int ar_ring_segmented(int n, const void *const *sb, void *const *rb,
                             size_t count, int op, int type, size_t segsize)
{
    const size_t typelng = orc_type_extent(type);  /* == size for non-gapped types */
    size_t segcount = count, nphases;
    if (segsize >= typelng && segsize < typelng * segcount) {   /* COMPUTED_SEGCOUNT */
        size_t residual;
        segcount = segsize / typelng;
        residual = segsize - segcount * typelng;
        if (residual > (typelng >> 1)) segcount++;
    }
    if (count < (size_t)n * segcount)           /* :652-656 */
        return ar_ring(n, sb, rb, count, op, type);
    nphases = count / ((size_t)n * segcount);   /* :663-667 */
    if ((count % ((size_t)n * segcount) >= (size_t)n) &&
        (count % ((size_t)n * segcount) > (((size_t)n * segcount) / 2)))
        nphases++;
    ar_ring_common(n, sb, rb, count, op, type, (int)nphases);
    return ORC_AR_RING_SEGMENTED;
}

/* ---------------- reduce to 0 + bcast ---------------- */
static int ar_reduce_bcast(int n, const void *const *sb, void *const *rb, size_t count, int op,
                           int type, int red_alg, int root0_inplace, int ret)
{
    const size_t bytes = count * orc_type_extent(type);
    char *acc = malloc(bytes ? bytes : 1);
    int r;
    if (orc_reduce(red_alg, n, sb, acc, count, op, type, 0, root0_inplace) < 0) {
        free(acc);
        return -1;
    }
    for (r = 0; r < n; r++) memcpy(rb[r], acc, bytes);   /* bcast from 0 */
    free(acc);
    return ret;
}

/* ---------------- Rabenseifner (redscat_allgather) ---------------- */
static int ar_redscat_allgather(int n, const void *const *sb, void *const *rb, size_t count,
                                int op, int type)
{
    const size_t ext = orc_type_extent(type), bytes = count * ext;
    int nsteps = 0, p2 = 1, rem, r, step, mask;
    size_t lh, rh;
    char **tmp, **msg;
    int *vrank;
    size_t *rindex, *sindex, *rcount, *scount, *wsize;
    while (p2 * 2 <= n) { p2 *= 2; nsteps++; }
    if (count < (size_t)p2)                                   /* :988-995 */
        return ar_reduce_bcast(n, sb, rb, count, op, type, ORC_RED_LINEAR, 0,
                               ORC_AR_BASIC_LINEAR);
    rem = n - p2;
    tmp = calloc((size_t)n, sizeof(char *));
    msg = calloc((size_t)n, sizeof(char *));
    vrank = calloc((size_t)n, sizeof(int));
    rindex = calloc((size_t)n * (size_t)(nsteps + 1), sizeof(size_t));
    sindex = calloc((size_t)n * (size_t)(nsteps + 1), sizeof(size_t));
    rcount = calloc((size_t)n * (size_t)(nsteps + 1), sizeof(size_t));
    scount = calloc((size_t)n * (size_t)(nsteps + 1), sizeof(size_t));
    wsize = calloc((size_t)n, sizeof(size_t));
    for (r = 0; r < n; r++) {
        tmp[r] = malloc(bytes ? bytes : 1);
        msg[r] = malloc(bytes ? bytes : 1);
        if (sb[r] != rb[r]) memcpy(rb[r], sb[r], bytes);      /* :1006-1010 */
    }
    /* step 1 (:1031-1086): even/odd pairs of the 2*rem lowest ranks */
    lh = count / 2;
    rh = count - lh;
    for (r = 0; r < n; r++) memcpy(msg[r], rb[r], bytes);   /* sendrecv: values before the step */
    for (r = 0; r < 2 * rem; r++) {
        if (r % 2) {   /* odd: recv the right half from r-1, reduce it */
            memcpy(tmp[r] + lh * ext, msg[r - 1] + lh * ext, rh * ext);
            orc_op_2buff(op, type, tmp[r] + lh * ext, (char *)rb[r] + lh * ext, rh);
        } else {       /* even: recv the left half from r+1, reduce it */
            memcpy(tmp[r], msg[r + 1], lh * ext);
            orc_op_2buff(op, type, tmp[r], rb[r], lh);
        }
    }
    for (r = 0; r < 2 * rem; r += 2)  /* the odd rank sends its right half back */
        memcpy((char *)rb[r] + lh * ext, (char *)rb[r + 1] + lh * ext, rh * ext);
    for (r = 0; r < n; r++)
        vrank[r] = r < 2 * rem ? (r % 2 ? -1 : r / 2) : r - rem;
    /* step 2 (:1104-1171): recursive vector halving, distance doubling */
    for (r = 0; r < n; r++) wsize[r] = count;
    for (step = 0, mask = 1; mask < p2; mask <<= 1, step++) {
        for (r = 0; r < n; r++) memcpy(msg[r], rb[r], bytes);
        for (r = 0; r < n; r++) {
            size_t *ri = rindex + (size_t)r * (nsteps + 1), *si = sindex + (size_t)r * (nsteps + 1);
            size_t *rc = rcount + (size_t)r * (nsteps + 1), *sc = scount + (size_t)r * (nsteps + 1);
            int vdest, dest;
            if (vrank[r] < 0) continue;
            vdest = vrank[r] ^ mask;
            dest = vdest < rem ? vdest * 2 : vdest + rem;
            if (r < dest) {
                rc[step] = wsize[r] / 2;
                sc[step] = wsize[r] - rc[step];
                si[step] = ri[step] + rc[step];
            } else {
                sc[step] = wsize[r] / 2;
                rc[step] = wsize[r] - sc[step];
                ri[step] = si[step] + sc[step];
            }
            /* dest sends rbuf[its sindex ..], which is our [rindex ..] */
            memcpy(tmp[r] + ri[step] * ext, msg[dest] + ri[step] * ext, rc[step] * ext);
            orc_op_2buff(op, type, tmp[r] + ri[step] * ext, (char *)rb[r] + ri[step] * ext, rc[step]);
            if (step + 1 < nsteps) {
                ri[step + 1] = ri[step];
                si[step + 1] = ri[step];
                wsize[r] = rc[step];
            }
        }
    }
    /* step 3 (:1183-1206): allgather, reverse order */
    for (step = nsteps - 1, mask = p2 >> 1; mask > 0; mask >>= 1, step--) {
        for (r = 0; r < n; r++) memcpy(msg[r], rb[r], bytes);
        for (r = 0; r < n; r++) {
            size_t *si = sindex + (size_t)r * (nsteps + 1), *sc = scount + (size_t)r * (nsteps + 1);
            int vdest, dest;
            if (vrank[r] < 0) continue;
            vdest = vrank[r] ^ mask;
            dest = vdest < rem ? vdest * 2 : vdest + rem;
            memcpy((char *)rb[r] + si[step] * ext, msg[dest] + si[step] * ext, sc[step] * ext);
        }
    }
    /* step 4 (:1212-1228): the excluded odd ranks get the result */
    for (r = 1; r < 2 * rem; r += 2) memcpy(rb[r], rb[r - 1], bytes);
    for (r = 0; r < n; r++) { free(tmp[r]); free(msg[r]); }
    free(tmp); free(msg); free(vrank); free(rindex); free(sindex); free(rcount); free(scount);
    free(wsize);
    return ORC_AR_REDSCAT_ALLGATHER;
}

int orc_allreduce(int algorithm, int n, const void *const *sb, void *const *rb,
                  size_t count, int op, int type, size_t segsize)
{
    return orc_allreduce_forced(algorithm, n, sb, rb, count, op, type, segsize, 0);
}

int orc_allreduce_forced(int algorithm, int n, const void *const *sb, void *const *rb,
                         size_t count, int op, int type, size_t segsize, int root0_inplace)
{
    return orc_allreduce_forced_red(algorithm, n, sb, rb, count, op, type, segsize, root0_inplace,
                                    ORC_RED_TUNED);
}

/* red_alg: the algorithm of coll/tuned's reduce that nonoverlapping calls
 * through comm->c_coll->coll_reduce (its own forced reduce algorithm when
 * dynamic rules are on; ORC_RED_TUNED = the fixed decision). */
int orc_allreduce_forced_red(int algorithm, int n, const void *const *sb, void *const *rb,
                             size_t count, int op, int type, size_t segsize, int root0_inplace,
                             int red_alg)
{
    const size_t ext = orc_type_extent(type);
    if (n < 1 || ext == 0 || !orc_op_defined(op, type)) return -1;
    if (count == 0) return algorithm;
    if (n == 1) {
        if (sb[0] != rb[0]) memcpy(rb[0], sb[0], count * ext);
        return algorithm;
    }
    if (algorithm == ORC_AR_TUNED) {
        /* the size used by the decision is the type SIZE (12 for DOUBLE_INT),
         * not the extent (coll_tuned_decision_fixed.c:63-64) */
        size_t tsize = ext;
        size_t block_dsize;
        if (type == ORC_T_DOUBLE_INT || type == ORC_T_LONG_INT) tsize = 12;
        if (type == ORC_T_SHORT_INT) tsize = 6;
        block_dsize = tsize * count;
        if (block_dsize < 10000) return ar_recursive_doubling(n, sb, rb, count, op, type);
        if (count > (size_t)n) {
            if ((size_t)n * (1u << 20) >= block_dsize) return ar_ring(n, sb, rb, count, op, type);
            return ar_ring_segmented(n, sb, rb, count, op, type, 1u << 20);
        }
        return -2; /* nonoverlapping: not restated */
    }
    switch (algorithm) {
    case ORC_AR_BASIC_LINEAR:
        return ar_reduce_bcast(n, sb, rb, count, op, type, ORC_RED_LINEAR, 0, ORC_AR_BASIC_LINEAR);
    case ORC_AR_NONOVERLAPPING:
        return ar_reduce_bcast(n, sb, rb, count, op, type, red_alg, root0_inplace,
                               ORC_AR_NONOVERLAPPING);
    case ORC_AR_RECURSIVE_DOUBLING: return ar_recursive_doubling(n, sb, rb, count, op, type);
    case ORC_AR_RING: return ar_ring(n, sb, rb, count, op, type);
    case ORC_AR_RING_SEGMENTED:
        return ar_ring_segmented(n, sb, rb, count, op, type, segsize ? segsize : (1u << 20));
    case ORC_AR_REDSCAT_ALLGATHER: return ar_redscat_allgather(n, sb, rb, count, op, type);
    default: return -2;
    }
}

/* reduce_scatter_block, reduce, scan, exscan: coll_reduce_oracle.c */

int orc_allgather(int n, const void *const *sb, void *const *rb, size_t bytes)
{
    int r, p;
    for (r = 0; r < n; r++)
        for (p = 0; p < n; p++) memcpy((char *)rb[r] + (size_t)p * bytes, sb[p], bytes);
    return 0;
}

int orc_bcast(int n, int root, void *const *bufs, size_t bytes)
{
    int r;
    for (r = 0; r < n; r++)
        if (r != root) memcpy(bufs[r], bufs[root], bytes);
    return 0;
}
