/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's reduction-collective hot path, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * CHECKER.  Nothing in ompi_amd/ (the product) links, loads or calls this.
 *
 * Pinned against: the reference's own known-answer tests
 * (test/datatype/reduce_local.c, test/datatype/check_op.sh,
 * test/datatype/ddt_test.c, test/datatype/opal_datatype_test.c) restated as
 * fixtures in tests/golden/, and the reference executions recorded in
 * SURVEY.md §8(c) (op/base NaN / ±0 / MAXLOC tie behaviour, ring and
 * recursive-doubling summation orders).  See DESIGN.md "Oracle".
 *
 * Codes follow the reference enums so fixtures can be read against it:
 *   op   = OMPI_OP_BASE_FORTRAN_*  (ompi/mca/op/op.h:203-237)
 *   type = OMPI_OP_BASE_TYPE_*     (ompi/mca/op/op.h:104-190)
 */
#ifndef OMPI_AMD_ORACLE_H
#define OMPI_AMD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* op codes (Fortran index, ompi/mca/op/op.h:203-237) */
enum {
    ORC_OP_NULL = 0, ORC_OP_MAX, ORC_OP_MIN, ORC_OP_SUM, ORC_OP_PROD,
    ORC_OP_LAND, ORC_OP_BAND, ORC_OP_LOR, ORC_OP_BOR, ORC_OP_LXOR,
    ORC_OP_BXOR, ORC_OP_MAXLOC, ORC_OP_MINLOC, ORC_OP_REPLACE, ORC_OP_NO_OP,
    ORC_OP_COUNT
};

/* type codes (ompi/mca/op/op.h:104-190); only the predefined C types this
 * oracle restates are named. */
enum {
    ORC_T_INT8 = 0, ORC_T_UINT8 = 1, ORC_T_INT16 = 2, ORC_T_UINT16 = 3,
    ORC_T_INT32 = 4, ORC_T_UINT32 = 5, ORC_T_INT64 = 6, ORC_T_UINT64 = 7,
    ORC_T_SHORT_FLOAT = 14,
    ORC_T_FLOAT = 15, ORC_T_DOUBLE = 16, ORC_T_BOOL = 25,
    ORC_T_C_SHORT_FLOAT_COMPLEX = 26, ORC_T_C_FLOAT_COMPLEX = 27, ORC_T_C_DOUBLE_COMPLEX = 28, ORC_T_BYTE = 30,
    ORC_T_FLOAT_INT = 34, ORC_T_DOUBLE_INT = 35, ORC_T_LONG_INT = 36,
    ORC_T_2INT = 37, ORC_T_SHORT_INT = 38,
    ORC_T_COUNT = 41
};

/* ---- op/base restatement (ompi/mca/op/base/op_base_functions.c) ---- */
/* 1 if the reference's op/base table has a handler for (op,type) AND this
 * oracle restates it. */
int    orc_op_defined(int op, int type);
/* bytes between consecutive elements (the datatype extent) */
size_t orc_type_extent(int type);
/* 2-buffer: inout[i] = inout[i] (op) in[i]   (OP_FUNC/FUNC_FUNC/LOC_FUNC) */
int    orc_op_2buff(int op, int type, const void *in, void *inout, size_t count);
/* 3-buffer: out[i] = in1[i] (op) in2[i]      (*_3BUF macros) */
int    orc_op_3buff(int op, int type, const void *in1, const void *in2,
                    void *out, size_t count);
/* IEEE binary16 <-> binary32 (round to nearest even), the conversions an
 * x86-64 build of op/base performs around its float evaluation of
 * opal_short_float_t (_Float16) expressions */
float    orc_h2f(uint16_t h);
uint16_t orc_f2h(float f);

/* ---- coll/base allreduce restatement (coll_base_allreduce.c) ---- */
enum {
    ORC_AR_TUNED = 0,              /* coll_tuned_decision_fixed.c:45-89 */
    ORC_AR_BASIC_LINEAR = 1,       /* coll_base_allreduce.c:881-912 */
    ORC_AR_NONOVERLAPPING = 2,     /* coll_base_allreduce.c:54-86 */
    ORC_AR_RECURSIVE_DOUBLING = 3, /* coll_base_allreduce.c:130-274 */
    ORC_AR_RING = 4,               /* coll_base_allreduce.c:341-536 */
    ORC_AR_RING_SEGMENTED = 5,     /* coll_base_allreduce.c:618-856 */
    ORC_AR_REDSCAT_ALLGATHER = 6   /* coll_base_allreduce.c:970-1243 */
};
/* Simulates the algorithm's message flow over `nranks` in-memory ranks.
 * sbufs[r] is rank r's send buffer, rbufs[r] its receive buffer (both
 * count*extent bytes).  Returns the algorithm actually run (tuned resolves
 * to 3/4/5), or <0 on error. */
int orc_allreduce(int algorithm, int nranks, const void *const *sbufs,
                  void *const *rbufs, size_t count, int op, int type,
                  size_t segsize);

/* The algorithm a user forced (coll_tuned_use_dynamic_rules +
 * coll_tuned_allreduce_algorithm, coll_tuned_allreduce_decision.c:130-150,
 * numbering as above), with each algorithm's fallbacks; root0_inplace: rank
 * 0 passed MPI_IN_PLACE (changes nonoverlapping's reduce). */
int orc_allreduce_forced(int algorithm, int nranks, const void *const *sbufs,
                         void *const *rbufs, size_t count, int op, int type,
                         size_t segsize, int root0_inplace);
int orc_allreduce_forced_red(int algorithm, int nranks, const void *const *sbufs,
                             void *const *rbufs, size_t count, int op, int type, size_t segsize,
                             int root0_inplace, int red_alg);

/* Block partition COLL_BASE_COMPUTE_BLOCKCOUNT (coll_base_functions.h:425-431) */
void orc_blockcount(size_t count, int nblocks, size_t *split,
                    size_t *early, size_t *late);

/* ---- coll/tuned reduce restatement (coll_reduce_oracle.c) ---- */
enum {
    ORC_RED_TUNED = 0,     /* coll_tuned_decision_fixed.c:354-428 */
    ORC_RED_LINEAR = 1,    /* basic_linear, coll_base_reduce.c:627-735 */
    ORC_RED_PIPELINE = 3,  /* chain fanout 1, coll_base_reduce.c:409-438 */
    ORC_RED_BINARY = 4,    /* coll_base_reduce.c:440-469 */
    ORC_RED_BINOMIAL = 5   /* in-order binomial, coll_base_reduce.c:471-500 */
};
/* The algorithm the fixed decision picks for a commutative op; msg = type
 * size * count. */
int orc_reduce_decision(int nranks, size_t msg, size_t count);
/* Reduce of sbufs[0..n) to `root` into rbuf_root; root_inplace = the root
 * passed MPI_IN_PLACE (its sbufs[root] is its recvbuf).  Returns the
 * algorithm run (tuned resolves to 1/3/4/5), <0 on error. */
int orc_reduce(int algorithm, int nranks, const void *const *sbufs, void *rbuf_root,
               size_t count, int op, int type, int root, int root_inplace);
/* reduce_scatter_block = tuned reduce of n*rcount elements to rank 0 +
 * scatter (coll_base_reduce_scatter_block.c:54-110).  Returns the reduce
 * algorithm run. */
int orc_reduce_scatter_block(int nranks, const void *const *sbufs,
                             void *const *rbufs, size_t rcount, int op, int type);
/* reduce_scatter with per-rank counts (coll_tuned_decision_fixed.c:466-512,
 * coll_base_reduce_scatter.c:132-623).  rbufs[r] receives rcounts[r]
 * elements.  Returns the algorithm run. */
int orc_reduce_scatter_block_alg(int nranks, const void *const *sbufs, void *const *rbufs,
                                 size_t rcount, int op, int type, int red_alg);
int orc_reduce_scatter_nonoverlapping(int nranks, const void *const *sbufs, void *const *rbufs,
                                      const size_t *rcounts, int op, int type, int red_alg,
                                      int inplace);
enum { ORC_RS_TUNED = 0, ORC_RS_HALVING = 1, ORC_RS_RING = 2 };
int orc_reduce_scatter_decision(int nranks, size_t total_bytes);
int orc_reduce_scatter(int algorithm, int nranks, const void *const *sbufs,
                       void *const *rbufs, const size_t *rcounts, int op, int type);
/* linear scan (exclusive = 0) / exscan (exclusive = 1); exscan leaves
 * rbufs[0] untouched. */
int orc_scan(int exclusive, int nranks, const void *const *sbufs, void *const *rbufs,
             size_t count, int op, int type);

/* allgather / bcast reference results (data movement only). */
int orc_allgather(int nranks, const void *const *sbufs, void *const *rbufs,
                  size_t bytes_per_rank);
int orc_bcast(int nranks, int root, void *const *bufs, size_t bytes);

/* ---- opal_datatype convertor restatement (opal/datatype/) ---- */
/* A committed datatype flattened to its typemap: nblocks contiguous byte
 * runs {disp, len} in typemap order, repeated every `extent` bytes. */
typedef struct {
    int64_t disp;
    int64_t len;
} orc_block_t;

/* pack bytes [offset, offset+bytes) of the packed stream of `count`
 * elements at `src` into `dst` (opal_generic_simple_pack semantics for a
 * homogeneous convertor; stream position == bConverted). Returns bytes
 * packed (truncated at the stream end). */
size_t orc_pack(const orc_block_t *blocks, int nblocks, int64_t extent,
                size_t count, const void *src, void *dst, size_t offset,
                size_t bytes);
/* inverse of orc_pack (opal_generic_simple_unpack) */
size_t orc_unpack(const orc_block_t *blocks, int nblocks, int64_t extent,
                  size_t count, const void *src, void *dst, size_t offset,
                  size_t bytes);

/* ---- CPU baseline helper: op loop timing (bench.py cpu_baseline) ---- */
double orc_time_op_3buff(int op, int type, const void *in1, const void *in2,
                         void *out, size_t count, int iters);

#ifdef __cplusplus
}
#endif
#endif
