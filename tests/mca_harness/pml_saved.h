/* TEST HARNESS ONLY: the real host transport behind the stand-in ob1 for
 * system tags at or below HARNESS_SYS_TAG (pml_saved.c). */
#ifndef HARNESS_PML_SAVED_H
#define HARNESS_PML_SAVED_H
#include <stddef.h>
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/request/request.h"

#define HARNESS_SYS_TAG (-1000)

extern int harness_saved_pml_msgs;  /* messages the transport moved */
void harness_pml_saved_init(const char *segment, int rank, int size);
void harness_pml_saved_fini(void);
void harness_pml_saved_send(const void *buf, size_t count, const ompi_datatype_t *d, int dst, int tag);
int harness_pml_saved_try_recv(void *buf, size_t count, const ompi_datatype_t *d, int src, int tag,
                               ompi_status_public_t *st);
ompi_request_t *harness_pml_saved_request(int is_send, void *buf, size_t count, const ompi_datatype_t *d,
                                          int peer, int tag, int persistent);
#endif
