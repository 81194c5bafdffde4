/* TEST HARNESS ONLY: the ompi_request_t subset a persistent collective
 * uses (ompi/request/request.h:74-82, 120-200, 436-460). */
#ifndef HARNESS_REQUEST_H
#define HARNESS_REQUEST_H
#include <stdbool.h>
#include <stddef.h>
#include "opal/class/opal_object.h"
struct ompi_request_t;
struct ompi_communicator_t;
typedef int (*ompi_request_start_fn_t)(size_t count, struct ompi_request_t **requests);
typedef int (*ompi_request_free_fn_t)(struct ompi_request_t **rptr);
typedef int (*ompi_request_cancel_fn_t)(struct ompi_request_t *request, int flag);
typedef int (*ompi_request_complete_fn_t)(struct ompi_request_t *request);
typedef enum { OMPI_REQUEST_PML, OMPI_REQUEST_IO, OMPI_REQUEST_GEN, OMPI_REQUEST_WIN,
               OMPI_REQUEST_COLL, OMPI_REQUEST_NULL, OMPI_REQUEST_NOOP, OMPI_REQUEST_PART,
               OMPI_REQUEST_MAX } ompi_request_type_t;
typedef enum { OMPI_REQUEST_INVALID, OMPI_REQUEST_INACTIVE, OMPI_REQUEST_ACTIVE,
               OMPI_REQUEST_CANCELLED } ompi_request_state_t;
typedef struct ompi_status_public_t {
    int MPI_SOURCE, MPI_TAG, MPI_ERROR, _cancelled;
    size_t _ucount;
} ompi_status_public_t;
typedef union ompi_mpi_object_t { struct ompi_communicator_t *comm; } ompi_mpi_object_t;
typedef struct ompi_request_t {
    opal_object_t super;
    ompi_request_type_t req_type;
    ompi_status_public_t req_status;
    volatile void *req_complete;
    volatile ompi_request_state_t req_state;
    bool req_persistent;
    int req_f_to_c_index;
    ompi_request_start_fn_t req_start;
    ompi_request_free_fn_t req_free;
    ompi_request_cancel_fn_t req_cancel;
    ompi_request_complete_fn_t req_complete_cb;
    void *req_complete_cb_data;
    ompi_mpi_object_t req_mpi_object;
} ompi_request_t;
OBJ_CLASS_DECLARATION(ompi_request_t);
#define REQUEST_PENDING (void *) 0L
#define REQUEST_COMPLETED (void *) 1L
#define REQUEST_COMPLETE(req) (REQUEST_COMPLETED == (req)->req_complete)
#define OMPI_REQUEST_INIT(request, persistent)                               \
    do {                                                                     \
        (request)->req_complete = (persistent) ? REQUEST_COMPLETED : REQUEST_PENDING; \
        (request)->req_state = OMPI_REQUEST_INACTIVE;                        \
        (request)->req_persistent = (persistent);                            \
        (request)->req_complete_cb = NULL;                                   \
        (request)->req_complete_cb_data = NULL;                              \
    } while (0);
#define OMPI_REQUEST_FINI(request)                                           \
    do {                                                                     \
        (request)->req_state = OMPI_REQUEST_INVALID;                         \
    } while (0);
static inline int ompi_request_complete(ompi_request_t *request, bool with_signal)
{
    (void) with_signal;
    request->req_complete = REQUEST_COMPLETED;
    return 0;
}
/* request.h:381-384 */
static inline int ompi_request_free(ompi_request_t **request)
{
    return (*request)->req_free(request);
}
extern ompi_request_t harness_request_null;
#define MPI_REQUEST_NULL (&harness_request_null)
#endif
