/*
 * TEST HARNESS ONLY.  Drives ompi_amd/mca/op/rocm/op_rocm_component.c the
 * way the op framework does (op_base_op_select.c:90-211): install op/base's
 * handlers, query the component, copy every non-NULL slot of its module over
 * them, run the NULL-pattern sanity check, then reduce through the
 * resulting op->o_func table like ompi_op_reduce (op.h:585-587).
 *
 * op/base is played by the CPU oracle (oracle/liboracle.so, the C
 * restatement of op_base_functions.c).  Host buffers must come back through
 * the registered fallback; with HARNESS_GPU=1 device buffers must run the
 * HIP handler.  Results are compared with the oracle.  Prints "ok".
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ompi/op/op.h"
#include "../../oracle/oracle.h"
#include "ompi_amd.h"

extern ompi_op_base_component_1_0_0_t mca_op_rocm_component;

#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);               \
            fprintf(stderr, "\n");                      \
            exit(1);                                    \
        }                                               \
    } while (0)

/* op/base stand-ins: the oracle, one wrapper per (op, type) used below */
#define BASE2(OPC, T, NAME)                                                       \
    static void NAME(const void *in, void *inout, int *n, struct ompi_datatype_t **d, \
                     ompi_op_base_module_t *m)                                    \
    {                                                                             \
        (void) d; (void) m;                                                       \
        base_calls++;                                                             \
        orc_op_2buff(OPC, T, in, inout, (size_t) *n);                             \
    }
#define BASE3(OPC, T, NAME)                                                       \
    static void NAME(const void *a, const void *b, void *o, int *n,               \
                     struct ompi_datatype_t **d, ompi_op_base_module_t *m)        \
    {                                                                             \
        (void) d; (void) m;                                                       \
        base_calls++;                                                             \
        orc_op_3buff(OPC, T, a, b, o, (size_t) *n);                               \
    }
static int base_calls = 0;
BASE2(ORC_OP_SUM, ORC_T_FLOAT, base_sum_float)
BASE3(ORC_OP_SUM, ORC_T_FLOAT, base3_sum_float)
BASE2(ORC_OP_MAXLOC, ORC_T_DOUBLE_INT, base_maxloc_double_int)
BASE3(ORC_OP_MAXLOC, ORC_T_DOUBLE_INT, base3_maxloc_double_int)

/* present in op/base but never expected to be called here */
static void base_other(const void *a, void *b, int *n, struct ompi_datatype_t **d,
                       ompi_op_base_module_t *m)
{
    (void) a; (void) b; (void) n; (void) d; (void) m;
    fprintf(stderr, "unexpected op/base call\n");
    exit(2);
}
static void base3_other(const void *a, const void *b, void *o, int *n,
                        struct ompi_datatype_t **d, ompi_op_base_module_t *m)
{
    (void) a; (void) b; (void) o; (void) n; (void) d; (void) m;
    fprintf(stderr, "unexpected op/base 3buff call\n");
    exit(2);
}

/* op/base's slot pattern for the types the reference builds here: the
 * oracle's predefined C types plus Fortran INTEGER/REAL/DOUBLE PRECISION and
 * long double, which this library leaves to op/base. */
static int base_has(int op, int t)
{
    if (orc_op_defined(op, t)) return 1;
    if (op >= ORC_OP_MAX && op <= ORC_OP_PROD) return t == 8 || t == 17 || t == 22 || t == 23;
    return 0;
}

static void select_op(ompi_op_t *op, int opidx, ompi_op_base_module_t *base)
{
    int i, prio = -1;
    ompi_op_base_module_t *m;
    memset(op, 0, sizeof(*op));
    op->o_flags = OMPI_OP_FLAGS_INTRINSIC;
    op->o_f_to_c_index = opidx;
    for (i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        if (!base_has(opidx, i)) continue;
        op->o_func.intrinsic.fns[i] = base_other;
        op->o_3buff_intrinsic.fns[i] = base3_other;
        op->o_func.intrinsic.modules[i] = base;
        op->o_3buff_intrinsic.modules[i] = base;
    }
    if (opidx == ORC_OP_SUM) {
        op->o_func.intrinsic.fns[ORC_T_FLOAT] = base_sum_float;
        op->o_3buff_intrinsic.fns[ORC_T_FLOAT] = base3_sum_float;
    }
    if (opidx == ORC_OP_MAXLOC) {
        op->o_func.intrinsic.fns[ORC_T_DOUBLE_INT] = base_maxloc_double_int;
        op->o_3buff_intrinsic.fns[ORC_T_DOUBLE_INT] = base3_maxloc_double_int;
    }
    m = mca_op_rocm_component.opc_op_query(op, &prio);
    CHECK(m != NULL && prio == 60, "query op %d", opidx);
    /* op_base_op_select.c:137-178: copy non-NULL slots */
    for (i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        if (m->opm_fns[i]) {
            op->o_func.intrinsic.fns[i] = m->opm_fns[i];
            op->o_func.intrinsic.modules[i] = m;
        }
        if (m->opm_3buff_fns[i]) {
            op->o_3buff_intrinsic.fns[i] = m->opm_3buff_fns[i];
            op->o_3buff_intrinsic.modules[i] = m;
        }
    }
    /* op_base_op_select.c:182-204: NULL pattern must stay op/base's */
    for (i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        CHECK((op->o_func.intrinsic.fns[i] != NULL) == (base_has(opidx, i) != 0),
              "NULL pattern op %d type %d", opidx, i);
        /* the library takes exactly the slots it has kernels for */
        CHECK((op->o_func.intrinsic.fns[i] != base_other &&
               op->o_func.intrinsic.fns[i] != NULL &&
               op->o_func.intrinsic.fns[i] != base_sum_float &&
               op->o_func.intrinsic.fns[i] != base_maxloc_double_int) ==
                  (base_has(opidx, i) && ompi_amd_op_supported(opidx, i)),
              "slot ownership op %d type %d", opidx, i);
    }
}

int main(void)
{
    const int use_gpu = getenv("HARNESS_GPU") && atoi(getenv("HARNESS_GPU"));
    ompi_op_base_module_t *base = OBJ_NEW(ompi_op_base_module_t);
    ompi_op_t sum, maxloc, band;
    int n = 1000, i, cnt;
    float *a, *b, *e;

    select_op(&sum, ORC_OP_SUM, base);
    select_op(&maxloc, ORC_OP_MAXLOC, base);
    select_op(&band, ORC_OP_BAND, base);

    /* host buffers: ompi_op_reduce -> rocm handler -> op/base fallback */
    a = malloc(n * sizeof(float));
    b = malloc(n * sizeof(float));
    e = malloc(n * sizeof(float));
    for (i = 0; i < n; ++i) {
        a[i] = (float) i * 0.5f;
        b[i] = e[i] = 3.0f - (float) i;
    }
    orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, a, e, (size_t) n);
    cnt = n;
    base_calls = 0;
    sum.o_func.intrinsic.fns[ORC_T_FLOAT](a, b, &cnt, NULL, sum.o_func.intrinsic.modules[ORC_T_FLOAT]);
    CHECK(base_calls == 1, "host SUM did not fall back (%d)", base_calls);
    CHECK(memcmp(b, e, n * sizeof(float)) == 0, "host SUM result");

    if (use_gpu) {
        void *da, *db;
        float *got = malloc(n * sizeof(float));
        for (i = 0; i < n; ++i) b[i] = e[i] = 3.0f - (float) i;
        orc_op_2buff(ORC_OP_SUM, ORC_T_FLOAT, a, e, (size_t) n);
        extern int harness_dev_alloc_copy(void **d, const void *h, size_t bytes);
        extern int harness_dev_copy_back(void *h, const void *d, size_t bytes);
        CHECK(harness_dev_alloc_copy(&da, a, n * sizeof(float)) == 0, "alloc");
        CHECK(harness_dev_alloc_copy(&db, b, n * sizeof(float)) == 0, "alloc");
        base_calls = 0;
        sum.o_func.intrinsic.fns[ORC_T_FLOAT](da, db, &cnt, NULL, NULL);
        CHECK(base_calls == 0, "device SUM fell back to the host");
        CHECK(harness_dev_copy_back(got, db, n * sizeof(float)) == 0, "copy back");
        CHECK(memcmp(got, e, n * sizeof(float)) == 0, "device SUM result");
        free(got);
    }
    printf("ok%s\n", use_gpu ? " gpu" : "");
    return 0;
}
