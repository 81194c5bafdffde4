/* TEST HARNESS ONLY: the mpi.h constants the osc glue uses
 * (ompi/include/mpi.h.in:542-557, 640, 656). */
#ifndef HARNESS_MPI_H
#define HARNESS_MPI_H
#define MPI_IN_PLACE ((void *) 1)
#define MPI_SUCCESS 0
#define MPI_MODE_NOCHECK 1
#define MPI_LOCK_EXCLUSIVE 1
#define MPI_LOCK_SHARED 2
#define MPI_WIN_FLAVOR_CREATE 1
#define MPI_WIN_FLAVOR_ALLOCATE 2
#define MPI_WIN_FLAVOR_DYNAMIC 3
#define MPI_WIN_FLAVOR_SHARED 4
#define MPI_WIN_UNIFIED 0
#define MPI_WIN_SEPARATE 1
#define MPI_PROC_NULL (-2)
#define MPI_ERR_WIN 53
#define MPI_ERR_RMA_RANGE 68
#define MPI_ERR_RMA_ATTACH 69
/* the predefined handles the glue's agreement uses (ompi/include/mpi.h.in:
 * OMPI_PREDEFINED_GLOBAL): harness objects, defined by osc_harness.c */
struct ompi_datatype_t;
struct ompi_op_t;
extern struct ompi_datatype_t harness_mpi_int;
extern struct ompi_op_t harness_mpi_max;
#define MPI_INT (&harness_mpi_int)
#define MPI_MAX (&harness_mpi_max)
#endif
