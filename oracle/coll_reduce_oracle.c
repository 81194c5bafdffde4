/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Message-flow restatement of coll/tuned's reduce (the fixed decision and
 * the four algorithms it picks for commutative ops), of reduce_scatter_block
 * (reduce to rank 0 through that decision, then scatter) and of the linear
 * scan / exscan that coll/basic provides when tuned has no scan.
 *
 *   decision            coll_tuned_decision_fixed.c:354-428
 *   generic tree reduce coll_base_reduce.c:62-370  (operand roles below)
 *   basic_linear        coll_base_reduce.c:627-735
 *   binomial            coll_base_reduce.c:471-500 + topo in_order_bmtree (coll_base_topo.c:402-458)
 *   pipeline            coll_base_reduce.c:409-438 + topo chain fanout 1 (coll_base_topo.c:530-600)
 *   binary              coll_base_reduce.c:440-469 + topo build_tree(2)  (coll_base_topo.c:77-175)
 *   rsb basic_linear    coll_base_reduce_scatter_block.c:54-110 (comm->c_coll->coll_reduce = tuned)
 *   scan linear         coll_base_scan.c:35-122
 *   exscan linear       coll_base_exscan.c:35-107
 *
 * Operand roles of ompi_coll_base_reduce_generic for a commutative op at a
 * node with children c0..c(k-1) (the segment loop does not change any
 * element's order, so whole buffers are reduced at once here):
 *   c0's data is received straight into the accumulator (:170-173), then
 *   acc = acc (op) own   i.e. ompi_op_reduce(op, in = own, inout = acc)
 *                        (:196-205 for k >= 2, :206-215 for k == 1)
 *   acc = acc (op) c_i   for i = 1..k-1 (:203-205, last child :214)
 * At the root under MPI_IN_PLACE the receive goes to a scratch buffer and
 * the accumulator starts as the root's own data (:170-171, :197-198):
 *   acc = own; acc = acc (op) c0; acc = acc (op) c_i ...
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define ORC_MAXFAN 32

typedef struct {
    int prev;
    int nnext;
    int next[ORC_MAXFAN];
} orc_tree_t;

/* coll_base_topo.c:34-63 */
static int pown(int fanout, int num)
{
    int j, p = 1;
    if (num < 0) return 0;
    if (1 == num) return fanout;
    if (2 == fanout) return p << num;
    for (j = 0; j < num; j++) p *= fanout;
    return p;
}

static int calculate_level(int fanout, int rank)
{
    int level, num;
    if (rank < 0) return -1;
    for (level = 0, num = 0; num <= rank; level++) num += pown(fanout, level);
    return level - 1;
}

/* build_tree(fanout) restated (coll_base_topo.c:77-175): children of the
 * shifted rank s are s + delta*(i+1), delta = fanout^level(s). */
static void build_tree(int fanout, int n, int root, int rank, orc_tree_t *t)
{
    int s = rank - root, level, delta, i;
    if (s < 0) s += n;
    t->prev = -1;
    t->nnext = 0;
    if (n < 2) return;
    level = calculate_level(fanout, s);
    delta = pown(fanout, level);
    for (i = 0; i < fanout; i++) {
        int schild = s + delta * (i + 1);
        if (schild >= n) break;
        t->next[t->nnext++] = (schild + root) % n;
    }
}

/* in-order binomial tree (coll_base_topo.c:402-458): children of vrank v
 * are v ^ mask for ascending masks while the bit is clear. */
static void build_in_order_bmtree(int n, int root, int rank, orc_tree_t *t)
{
    int v = (rank - root + n) % n, mask = 1;
    t->prev = root;
    t->nnext = 0;
    while (mask < n) {
        int remote = v ^ mask;
        if (remote < v) {
            t->prev = (remote + root) % n;
            break;
        } else if (remote < n) {
            t->next[t->nnext++] = (remote + root) % n;
        }
        mask <<= 1;
    }
}

/* chain with fanout 1 (coll_base_topo.c:588-600) */
static void build_pipeline(int n, int root, int rank, orc_tree_t *t)
{
    int s = (rank - root + n) % n;
    t->prev = (s == 0) ? -1 : (s - 1 + root) % n;
    t->nnext = 0;
    if (s + 1 < n) t->next[t->nnext++] = (s + 1 + root) % n;
}

/* Data a node hands to its parent (or the result at the root). */
static void node_value(const orc_tree_t *trees, int r, int root, int root_inplace,
                       const void *const *sb, size_t count, int op, int type, char *out)
{
    const size_t bytes = count * orc_type_extent(type);
    const orc_tree_t *t = &trees[r];
    char *child;
    int i;
    if (t->nnext == 0) {
        memcpy(out, sb[r], bytes);
        return;
    }
    child = malloc(bytes ? bytes : 1);
    node_value(trees, t->next[0], root, root_inplace, sb, count, op, type, child);
    if (r == root && root_inplace) {
        memcpy(out, sb[r], bytes);               /* accumbuf = recvbuf (own data) */
        orc_op_2buff(op, type, child, out, count);
    } else {
        memcpy(out, child, bytes);               /* c0 received into accumbuf */
        orc_op_2buff(op, type, sb[r], out, count);
    }
    for (i = 1; i < t->nnext; i++) {
        node_value(trees, t->next[i], root, root_inplace, sb, count, op, type, child);
        orc_op_2buff(op, type, child, out, count);
    }
    free(child);
}

static void reduce_tree(int alg, int n, const void *const *sb, void *out, size_t count,
                        int op, int type, int root, int root_inplace)
{
    orc_tree_t *trees = calloc((size_t)n, sizeof(orc_tree_t));
    int r;
    for (r = 0; r < n; r++) {
        if (alg == ORC_RED_BINOMIAL) build_in_order_bmtree(n, root, r, &trees[r]);
        else if (alg == ORC_RED_PIPELINE) build_pipeline(n, root, r, &trees[r]);
        else build_tree(2, n, root, r, &trees[r]);
    }
    node_value(trees, root, root, root_inplace, sb, count, op, type, (char *)out);
    free(trees);
}

/* basic_linear (coll_base_reduce.c:667-722): rbuf = x[n-1]; then
 * ompi_op_reduce(op, x[i], rbuf) for i = n-2 .. 0. */
static void reduce_linear(int n, const void *const *sb, void *out, size_t count, int op,
                          int type)
{
    int i;
    memcpy(out, sb[n - 1], count * orc_type_extent(type));
    for (i = n - 2; i >= 0; --i) orc_op_2buff(op, type, sb[i], out, count);
}

/* coll_tuned_decision_fixed.c:354-428, commutative branch.  msg = type
 * SIZE * count (:376-377). */
int orc_reduce_decision(int n, size_t msg, size_t count)
{
    const double a1 = 0.6016 / 1024.0, b1 = 1.3496;
    const double a2 = 0.0410 / 1024.0, b2 = 9.7128;
    const double a3 = 0.0422 / 1024.0, b3 = 1.1614;
    if (n < 8 && msg < 512) return ORC_RED_LINEAR;
    if ((n < 8 && msg < 20480) || msg < 2048 || count <= 1) return ORC_RED_BINOMIAL;
    if (n > a1 * (double)msg + b1) return ORC_RED_BINOMIAL;
    if (n > a2 * (double)msg + b2) return ORC_RED_PIPELINE;
    if (n > a3 * (double)msg + b3) return ORC_RED_BINARY;
    return ORC_RED_PIPELINE;
}

static size_t type_size(int type)
{
    if (type == ORC_T_DOUBLE_INT || type == ORC_T_LONG_INT) return 12;
    if (type == ORC_T_SHORT_INT) return 6;
    return orc_type_extent(type);
}

int orc_reduce(int algorithm, int n, const void *const *sb, void *rbuf_root, size_t count,
               int op, int type, int root, int root_inplace)
{
    if (n < 1 || root < 0 || root >= n || orc_type_extent(type) == 0 || !orc_op_defined(op, type))
        return -1;
    if (count == 0) return algorithm;
    if (n == 1) {
        memmove(rbuf_root, sb[0], count * orc_type_extent(type));
        return algorithm;
    }
    if (algorithm == ORC_RED_TUNED) algorithm = orc_reduce_decision(n, type_size(type) * count, count);
    if (algorithm == ORC_RED_LINEAR) reduce_linear(n, sb, rbuf_root, count, op, type);
    else if (algorithm == ORC_RED_BINOMIAL || algorithm == ORC_RED_PIPELINE ||
             algorithm == ORC_RED_BINARY)
        reduce_tree(algorithm, n, sb, rbuf_root, count, op, type, root, root_inplace);
    else return -2;
    return algorithm;
}

/* rsb basic_linear (coll_base_reduce_scatter_block.c:54-111): a reduce of
 * n*rcount elements to rank 0 through comm->c_coll->coll_reduce — coll/tuned's,
 * so its forced algorithm (red_alg, ORC_RED_*; 0 = the fixed decision) when
 * dynamic rules are on — never in place at the reduce level (sbuf = rbuf is
 * passed as sbuf), then scatter. */
int orc_reduce_scatter_block_alg(int n, const void *const *sb, void *const *rb,
                                 size_t rcount, int op, int type, int red_alg)
{
    const size_t ext = orc_type_extent(type), total = rcount * (size_t)n;
    char *acc;
    int r, alg;
    if (ext == 0 || !orc_op_defined(op, type)) return -1;
    acc = malloc(total * ext + 1);
    alg = orc_reduce(red_alg, n, sb, acc, total, op, type, 0, 0);
    if (alg < 0) { free(acc); return alg; }
    for (r = 0; r < n; r++) memcpy(rb[r], acc + (size_t)r * rcount * ext, rcount * ext);
    free(acc);
    return alg;
}

int orc_reduce_scatter_block(int n, const void *const *sb, void *const *rb,
                             size_t rcount, int op, int type)
{
    const size_t ext = orc_type_extent(type), total = rcount * (size_t)n;
    char *acc;
    int r, alg;
    if (ext == 0 || !orc_op_defined(op, type)) return -1;
    acc = malloc(total * ext + 1);
    alg = orc_reduce(ORC_RED_TUNED, n, sb, acc, total, op, type, 0, 0);
    if (alg < 0) { free(acc); return alg; }
    for (r = 0; r < n; r++) memcpy(rb[r], acc + (size_t)r * rcount * ext, rcount * ext);
    free(acc);
    return alg;
}

/* linear scan: P_0 = x_0, P_r = ompi_op_reduce(op, in = P_(r-1), inout = x_r);
 * scan writes P_r to rank r, exscan writes P_(r-1) (rank 0 untouched). */
int orc_scan(int exclusive, int n, const void *const *sb, void *const *rb, size_t count,
             int op, int type)
{
    const size_t bytes = count * orc_type_extent(type);
    char *prev, *cur;
    int r;
    if (n < 1 || orc_type_extent(type) == 0 || !orc_op_defined(op, type)) return -1;
    prev = malloc(bytes + 1);
    cur = malloc(bytes + 1);
    memcpy(prev, sb[0], bytes);
    if (!exclusive) memcpy(rb[0], prev, bytes);
    for (r = 1; r < n; r++) {
        memcpy(cur, sb[r], bytes);
        orc_op_2buff(op, type, prev, cur, count);
        memcpy(rb[r], exclusive ? prev : cur, bytes);
        memcpy(prev, cur, bytes);
    }
    free(prev);
    free(cur);
    return 0;
}

/* ---------------- reduce_scatter (vector counts) ----------------
 *   decision            coll_tuned_decision_fixed.c:466-512
 *   recursive halving   coll_base_reduce_scatter.c:132-391
 *   ring                coll_base_reduce_scatter.c:456-623 */
int orc_reduce_scatter_decision(int n, size_t total_bytes)
{
    int pow2 = 1;
    while (pow2 < n) pow2 <<= 1;                      /* next_poweroftwo_inclusive */
    if (total_bytes <= 12 * 1024 || (total_bytes <= 256 * 1024 && pow2 == n) ||
        (double)n >= 0.0012 * (double)total_bytes + 8.0)
        return ORC_RS_HALVING;
    return ORC_RS_RING;
}

static void rs_halving(int n, const void *const *sb, void *const *rb, const size_t *rcounts,
                       int op, int type)
{
    const size_t ext = orc_type_extent(type);
    size_t *disps = calloc((size_t)n, sizeof(size_t)), count;
    char **res = calloc((size_t)n, sizeof(char *)), **msg = calloc((size_t)n, sizeof(char *));
    int *trank = calloc((size_t)n, sizeof(int));
    int r, i, tmp_size = 1, remain, mask;
    for (r = 1; r < n; r++) disps[r] = disps[r - 1] + rcounts[r - 1];
    count = disps[n - 1] + rcounts[n - 1];
    for (r = 0; r < n; r++) {
        res[r] = malloc(count * ext + 1);
        msg[r] = malloc(count * ext + 1);
        memcpy(res[r], sb[r], count * ext);            /* result_buf <- sbuf (:190) */
    }
    while (tmp_size <= n) tmp_size <<= 1;              /* opal_next_poweroftwo(size) >> 1 */
    tmp_size >>= 1;
    remain = n - tmp_size;
    /* non-pof2 fold (:203-228): odd r < 2*remain: res = res (op) even's res */
    for (r = 0; r < n; r++) {
        if (r < 2 * remain) {
            if ((r & 1) == 0) trank[r] = -1;
            else {
                orc_op_2buff(op, type, res[r - 1], res[r], count);
                trank[r] = r / 2;
            }
        } else {
            trank[r] = r - remain;
        }
    }
    {
        size_t *trc = calloc((size_t)tmp_size, sizeof(size_t));
        size_t *tds = calloc((size_t)tmp_size, sizeof(size_t));
        int *sidx = calloc((size_t)n, sizeof(int)), *ridx = calloc((size_t)n, sizeof(int));
        int *lidx = calloc((size_t)n, sizeof(int));
        for (i = 0; i < tmp_size; i++)
            trc[i] = (i < remain) ? rcounts[i * 2 + 1] + rcounts[i * 2] : rcounts[i + remain];
        for (i = 0; i + 1 < tmp_size; i++) tds[i + 1] = tds[i] + trc[i];
        for (r = 0; r < n; r++) { sidx[r] = ridx[r] = 0; lidx[r] = tmp_size; }
        for (mask = tmp_size >> 1; mask > 0; mask >>= 1) {
            /* every participant sends the half it gives away (:276-323) */
            int *snd = calloc((size_t)n, sizeof(int)), *rcv = calloc((size_t)n, sizeof(int));
            for (r = 0; r < n; r++) {
                int tp;
                if (trank[r] < 0) continue;
                tp = trank[r] ^ mask;
                if (trank[r] < tp) { snd[r] = ridx[r] + mask; rcv[r] = ridx[r]; }
                else { rcv[r] = sidx[r] + mask; snd[r] = sidx[r]; }
                memcpy(msg[r], res[r], count * ext);   /* snapshot = what r sends */
            }
            for (r = 0; r < n; r++) {
                int tp, peer, hi_end;
                size_t rc = 0;
                if (trank[r] < 0) continue;
                tp = trank[r] ^ mask;
                peer = (tp < remain) ? tp * 2 + 1 : tp + remain;
                hi_end = (trank[r] < tp) ? snd[r] : lidx[r];
                for (i = rcv[r]; i < hi_end; i++) rc += trc[i];
                if (rc > 0)   /* :335-338: res[recv] = res[recv] (op) peer's */
                    orc_op_2buff(op, type, msg[peer] + tds[rcv[r]] * ext, res[r] + tds[rcv[r]] * ext, rc);
            }
            for (r = 0; r < n; r++) {                  /* :342-344 */
                if (trank[r] < 0) continue;
                sidx[r] = rcv[r];
                ridx[r] = rcv[r];
                lidx[r] = rcv[r] + mask;
            }
            free(snd);
            free(rcv);
        }
        free(trc); free(tds); free(sidx); free(ridx); free(lidx);
    }
    /* results: participants copy their block (:348-357); odd ranks below
     * 2*remain also hand the even neighbour its block (:365-383) */
    for (r = 0; r < n; r++) {
        if (trank[r] < 0) continue;
        memcpy(rb[r], res[r] + disps[r] * ext, rcounts[r] * ext);
        if (r < 2 * remain) memcpy(rb[r - 1], res[r] + disps[r - 1] * ext, rcounts[r - 1] * ext);
    }
    for (r = 0; r < n; r++) { free(res[r]); free(msg[r]); }
    free(res); free(msg); free(disps); free(trank);
}

static void rs_ring(int n, const void *const *sb, void *const *rb, const size_t *rcounts, int op,
                    int type)
{
    const size_t ext = orc_type_extent(type);
    size_t *disps = calloc((size_t)n, sizeof(size_t)), total, maxb = 0;
    char **acc = calloc((size_t)n, sizeof(char *)), **msg = calloc((size_t)n, sizeof(char *));
    char **nmsg = calloc((size_t)n, sizeof(char *));
    int r, k;
    for (r = 1; r < n; r++) disps[r] = disps[r - 1] + rcounts[r - 1];
    total = disps[n - 1] + rcounts[n - 1];
    for (r = 0; r < n; r++) if (rcounts[r] > maxb) maxb = rcounts[r];
    for (r = 0; r < n; r++) {
        acc[r] = malloc(total * ext + 1);
        msg[r] = malloc(maxb * ext + 1);
        nmsg[r] = malloc(maxb * ext + 1);
        memcpy(acc[r], sb[r], total * ext);           /* accumbuf <- sbuf (:530) */
    }
    for (r = 0; r < n; r++) {                          /* first send: block r-1 (:560) */
        int b = (r + n - 1) % n;
        memcpy(msg[r], acc[r] + disps[b] * ext, rcounts[b] * ext);
    }
    for (k = 2; k < n; k++) {                          /* :566-592 */
        for (r = 0; r < n; r++) {
            int from = (r + n - 1) % n, pb = (r + n - k) % n;
            orc_op_2buff(op, type, msg[from], acc[r] + disps[pb] * ext, rcounts[pb]);
            memcpy(nmsg[r], acc[r] + disps[pb] * ext, rcounts[pb] * ext);
        }
        for (r = 0; r < n; r++) { char *t = msg[r]; msg[r] = nmsg[r]; nmsg[r] = t; }
    }
    for (r = 0; r < n; r++) {                          /* my block (:598-605) */
        int from = (r + n - 1) % n;
        orc_op_2buff(op, type, msg[from], acc[r] + disps[r] * ext, rcounts[r]);
        memcpy(rb[r], acc[r] + disps[r] * ext, rcounts[r] * ext);
    }
    for (r = 0; r < n; r++) { free(acc[r]); free(msg[r]); free(nmsg[r]); }
    free(acc); free(msg); free(nmsg); free(disps);
}

/* reduce_scatter non-overlapping (coll_base_reduce_scatter.c:42-92): a
 * reduce of the whole vector to rank 0 through comm->c_coll->coll_reduce
 * (coll/tuned's: red_alg as above), rank 0 in place when it passed
 * MPI_IN_PLACE (:62-68), then scatterv of the blocks. */
int orc_reduce_scatter_nonoverlapping(int n, const void *const *sb, void *const *rb,
                                      const size_t *rcounts, int op, int type, int red_alg,
                                      int inplace)
{
    const size_t ext = orc_type_extent(type);
    size_t total = 0, off = 0;
    char *acc;
    int r, alg;
    if (n < 1 || ext == 0 || !orc_op_defined(op, type)) return -1;
    for (r = 0; r < n; r++) total += rcounts[r];
    if (total == 0) return 0;
    acc = malloc(total * ext + 1);
    alg = orc_reduce(red_alg, n, sb, acc, total, op, type, 0, inplace);
    if (alg < 0) { free(acc); return alg; }
    for (r = 0; r < n; r++) {
        memcpy(rb[r], acc + off * ext, rcounts[r] * ext);
        off += rcounts[r];
    }
    free(acc);
    return alg;
}

int orc_reduce_scatter(int algorithm, int n, const void *const *sb, void *const *rb,
                       const size_t *rcounts, int op, int type)
{
    size_t total = 0;
    int r;
    if (n < 1 || orc_type_extent(type) == 0 || !orc_op_defined(op, type)) return -1;
    for (r = 0; r < n; r++) total += rcounts[r];
    if (total == 0) return algorithm;
    if (n == 1) {
        memmove(rb[0], sb[0], rcounts[0] * orc_type_extent(type));
        return algorithm;
    }
    if (algorithm == ORC_RS_TUNED) algorithm = orc_reduce_scatter_decision(n, total * type_size(type));
    if (algorithm == ORC_RS_HALVING) rs_halving(n, sb, rb, rcounts, op, type);
    else if (algorithm == ORC_RS_RING) rs_ring(n, sb, rb, rcounts, op, type);
    else return -2;
    return algorithm;
}
