/*
 * TEST HARNESS ONLY: the request class, MPI_REQUEST_NULL and opal_progress
 * (opal/runtime/opal_progress.c: registered callbacks polled by every
 * progress call) shared by the coll, pml and osc harnesses.
 */
#include "opal/runtime/opal_progress.h"
#include "ompi/request/request.h"

OBJ_CLASS_INSTANCE(ompi_request_t, opal_object_t, NULL, NULL);
ompi_request_t harness_request_null;

static opal_progress_callback_t progress_cbs[8];
static int n_progress_cbs;

int opal_progress_register(opal_progress_callback_t cb)
{
    for (int i = 0; i < n_progress_cbs; ++i)
        if (progress_cbs[i] == cb) return 0;
    if (n_progress_cbs == (int) (sizeof(progress_cbs) / sizeof(progress_cbs[0]))) return -1;
    progress_cbs[n_progress_cbs++] = cb;
    return 0;
}

int opal_progress_unregister(opal_progress_callback_t cb)
{
    for (int i = 0; i < n_progress_cbs; ++i)
        if (progress_cbs[i] == cb) progress_cbs[i] = progress_cbs[--n_progress_cbs];
    return 0;
}

void opal_progress(void)
{
    for (int i = 0; i < n_progress_cbs; ++i) progress_cbs[i]();
}
