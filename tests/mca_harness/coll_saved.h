/* TEST HARNESS ONLY: the host "saved" coll functions (coll_saved.c). */
#ifndef HARNESS_COLL_SAVED_H
#define HARNESS_COLL_SAVED_H
#include <stddef.h>
#include "ompi/mca/coll/coll.h"
#include "ompi/datatype/ompi_datatype.h"

/* OMPI_OP_BASE_TYPE_LONG_DOUBLE (ompi/mca/op/op.h:104-199): op/base has it,
 * no device kernel does */
#define HARNESS_T_LONG_DOUBLE 23

enum { HARNESS_ALLREDUCE = 0, HARNESS_SCAN = 2, HARNESS_EXSCAN = 3 };

extern int tuned_calls;        /* calls that reached a saved function */
extern int t_sdev, t_rdev;     /* residency of the last saved allreduce's buffers */
extern int harness_saved_live; /* stand-in requests not yet freed */

void harness_saved_init(const char *segment, int rank, int size);
void harness_saved_fini(void);
void harness_fill_tuned(mca_coll_base_comm_coll_t *t, mca_coll_base_module_t *tm);
int harness_is_saved_request(const ompi_request_t *r);
size_t harness_esize(const ompi_datatype_t *d);
void harness_fold(int op, int type, const void *in, void *inout, size_t count);
void harness_expect_reduction(int kind, int op, const ompi_datatype_t *d, const char *const *x,
                              int n, int me, size_t count, char *out);
void harness_expect_rs(int op, const ompi_datatype_t *d, const char *const *x, int n, int me,
                       const int *rcounts, char *out);
#endif
