/* TEST HARNESS ONLY: the communicator fields and accessors the glue uses. */
#ifndef HARNESS_COMMUNICATOR_H
#define HARNESS_COMMUNICATOR_H
#include "ompi/mca/coll/coll.h"
#include "ompi/group/group.h"
typedef struct ompi_communicator_t {
    int rank, size, cid, inter;
    ompi_group_t *c_local_group;
    mca_coll_base_comm_coll_t *c_coll;
} ompi_communicator_t;
#define OMPI_COMM_IS_INTER(c) ((c)->inter)
static inline int ompi_comm_rank(const ompi_communicator_t *c) { return c->rank; }
static inline int ompi_comm_size(const ompi_communicator_t *c) { return c->size; }
static inline int ompi_comm_get_cid(const ompi_communicator_t *c) { return c->cid; }
#endif
