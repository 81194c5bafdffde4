/* TEST HARNESS ONLY */
#ifndef HARNESS_MPI_H
#define HARNESS_MPI_H
#define MPI_IN_PLACE ((void *) 1)
#define MPI_SUCCESS 0
#define MPI_ANY_SOURCE (-1)
#define MPI_ANY_TAG (-1)
#define MPI_PROC_NULL (-2)
#define MPI_ERR_TRUNCATE 15
struct ompi_datatype_t;
extern struct ompi_datatype_t harness_mpi_byte;
#define MPI_BYTE (&harness_mpi_byte)
#endif
