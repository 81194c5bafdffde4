/*
 * coll/rocm — MI355X coll component for Open MPI's coll framework.
 *
 * Drop-in: copy this directory to ompi/mca/coll/rocm/ (INTEGRATION.md §2).
 * The module provides coll_allreduce, coll_reduce, coll_reduce_scatter,
 * coll_reduce_scatter_block,
 * coll_scan, coll_exscan, coll_allgather, coll_bcast
 * (ompi/mca/coll/coll.h:200-250), the nonblocking coll_iallreduce
 * (coll.h:271-274), coll_ireduce_scatter_block / coll_iallgather /
 * coll_ibcast, coll_ireduce, coll_iscan, coll_iexscan, coll_ireduce_scatter
 * (coll.h:261-326) and the persistent coll_allreduce_init,
 * coll_reduce_scatter_block_init, coll_allgather_init and coll_bcast_init
 * (coll.h:339-400)
 * for device buffers through libompi_amd.so,
 * and interposes on the previously selected functions (coll/tuned, coll/basic
 * for scan/exscan) for everything else, exactly like coll/cuda does
 * (ompi/mca/coll/cuda/coll_cuda_module.c:120-155).
 */
#ifndef MCA_COLL_ROCM_EXPORT_H
#define MCA_COLL_ROCM_EXPORT_H

#include "ompi_config.h"

#include "mpi.h"
#include "ompi/communicator/communicator.h"
#include "ompi/mca/coll/base/coll_base_functions.h"
#include "ompi/mca/coll/coll.h"
#include "ompi/request/request.h"
#include "opal/class/opal_object.h"

#include "ompi_amd_coll.h"

BEGIN_C_DECLS

typedef struct mca_coll_rocm_module_t {
    mca_coll_base_module_t super;
    /* the functions this module replaces, saved at enable time */
    mca_coll_base_comm_coll_t c_coll;
    /* libompi_amd communicator (IPC mappings, flags, epoch) */
    ompi_amd_comm_t *dev_comm;
    /* residency policy (coll_rocm_residency): which path a blocking call
     * takes.  AUTO votes per call; after coll_rocm_residency_lock unanimous
     * votes in a row the module locks to DEVICE or HOST and stops voting
     * (a rank whose operands sit elsewhere stages them); every
     * coll_rocm_residency_recheck locked calls one vote asks whether any
     * rank staged, and unlocks if so. */
    int mode;
    int forced;                  /* mode set by the parameter: never unlocks */
    int streak_dev, streak_host; /* consecutive unanimous votes (AUTO) */
    int since_check, mismatched; /* locked: calls since the last recheck, own stagings */
    void *dstage[2], *hstage[2]; /* grow-only staging per operand slot */
    size_t dstage_bytes[2], hstage_bytes[2];
    int fail_stage;              /* test hook: the next staging allocation fails */
    /* coll/tuned's forcing state read at enable (rocm_tuned_config): the
     * blocking reductions whose tuned algorithm the device path does not
     * run (ROCM_TUNED_* bits) stay with the saved functions */
    int tuned_decline;
} mca_coll_rocm_module_t;

enum { ROCM_TUNED_ALLREDUCE = 1, ROCM_TUNED_REDUCE = 2, ROCM_TUNED_RS = 4, ROCM_TUNED_RSB = 8 };

enum { ROCM_RES_AUTO = 0, ROCM_RES_DEVICE = 1, ROCM_RES_HOST = 2 };

OBJ_CLASS_DECLARATION(mca_coll_rocm_module_t);

typedef struct mca_coll_rocm_component_t {
    mca_coll_base_component_2_0_0_t super;
    int priority;        /* coll_rocm_priority (default 80: above coll/cuda's 78) */
    int small_bytes;     /* coll_rocm_small_bytes */
    int zero_copy;       /* coll_rocm_zero_copy */
    int timeout_ms;      /* coll_rocm_timeout_ms */
    int algorithm;       /* coll_rocm_allreduce_algorithm (0 pull, 1 pull+push, 2 push) */
    int user_ipc;        /* coll_rocm_user_ipc: peers map the caller's buffers (else staged) */
    int autotune;        /* coll_rocm_autotune: measure the large-allreduce scheme and grid */
    int land_blocking;   /* coll_rocm_land_blocking: blocking allgather / bcast by landing stores */
    int copy_nt;         /* coll_rocm_copy_nt: non-temporal stores in the copy kernels (-1 autotuned) */
    int residency;       /* coll_rocm_residency: 0 auto, 1 device, 2 host */
    int residency_lock;  /* coll_rocm_residency_lock: unanimous votes before locking (0 never) */
    int residency_recheck; /* coll_rocm_residency_recheck: locked calls per recheck vote (0 never) */
    int max_device_mib;  /* coll_rocm_max_device_mib: larger calls go to the saved functions */
    int own_stream;      /* coll_rocm_own_stream: each communicator's calls on a hardware queue of its own */
} mca_coll_rocm_component_t;

OMPI_MODULE_DECLSPEC extern mca_coll_rocm_component_t mca_coll_rocm_component;

/* A device collective's MPI request: persistent (MPI_Allreduce_init: a
 * library plan, started by req_start) or nonblocking (MPI_Iallreduce: a
 * library request).  The component's progress callback completes it once
 * the library reports its device work finished. */
typedef struct mca_coll_rocm_request_t {
    ompi_request_t super;
    ompi_amd_plan_t *plan;       /* persistent */
    ompi_amd_request_t *nbreq;   /* nonblocking */
    /* the saved (libnbc) function's request when it runs on host copies of
     * this rank's device operands (nonblocking or persistent) */
    ompi_request_t *inner;
    struct rocm_nb_stage *stage; /* this rank's staged operands */
    struct mca_coll_rocm_request_t *next_active; /* started, not yet complete */
} mca_coll_rocm_request_t;

OBJ_CLASS_DECLARATION(mca_coll_rocm_request_t);

int mca_coll_rocm_init_query(bool enable_progress_threads, bool enable_mpi_threads);
mca_coll_base_module_t *mca_coll_rocm_comm_query(struct ompi_communicator_t *comm,
                                                 int *priority);
int mca_coll_rocm_module_enable(mca_coll_base_module_t *module,
                                struct ompi_communicator_t *comm);

int mca_coll_rocm_allreduce(const void *sbuf, void *rbuf, int count,
                            struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                            struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
int mca_coll_rocm_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                         struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                         mca_coll_base_module_t *module);
int mca_coll_rocm_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                       struct ompi_op_t *op, struct ompi_communicator_t *comm,
                       mca_coll_base_module_t *module);
int mca_coll_rocm_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                         struct ompi_op_t *op, struct ompi_communicator_t *comm,
                         mca_coll_base_module_t *module);
int mca_coll_rocm_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts,
                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                 struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
int mca_coll_rocm_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount,
                                       struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                       struct ompi_communicator_t *comm,
                                       mca_coll_base_module_t *module);
int mca_coll_rocm_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                            void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                            struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
int mca_coll_rocm_iallreduce(const void *sbuf, void *rbuf, int count,
                             struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                             struct ompi_communicator_t *comm, ompi_request_t **request,
                             mca_coll_base_module_t *module);
int mca_coll_rocm_ireduce_scatter_block(const void *sbuf, void *rbuf, int rcount,
                                        struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                        struct ompi_communicator_t *comm, ompi_request_t **request,
                                        mca_coll_base_module_t *module);
int mca_coll_rocm_iallgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                             void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                             struct ompi_communicator_t *comm, ompi_request_t **request,
                             mca_coll_base_module_t *module);
int mca_coll_rocm_ibcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                         struct ompi_communicator_t *comm, ompi_request_t **request,
                         mca_coll_base_module_t *module);
int mca_coll_rocm_allreduce_init(const void *sbuf, void *rbuf, int count,
                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                 struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                 ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_rocm_bcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                        struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
int mca_coll_rocm_ireduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                          ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_rocm_iscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                        struct ompi_op_t *op, struct ompi_communicator_t *comm,
                        ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_rocm_iexscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, struct ompi_communicator_t *comm,
                          ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_rocm_ireduce_scatter(const void *sbuf, void *rbuf, const int *rcounts,
                                  struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                  struct ompi_communicator_t *comm, ompi_request_t **request,
                                  mca_coll_base_module_t *module);
int mca_coll_rocm_reduce_scatter_block_init(const void *sbuf, void *rbuf, int rcount,
                                            struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                            struct ompi_communicator_t *comm,
                                            struct ompi_info_t *info, ompi_request_t **request,
                                            mca_coll_base_module_t *module);
int mca_coll_rocm_allgather_init(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                                 void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                                 struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                 ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_rocm_bcast_init(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                             struct ompi_communicator_t *comm, struct ompi_info_t *info,
                             ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_rocm_reduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                              struct ompi_info_t *info, ompi_request_t **request,
                              mca_coll_base_module_t *module);
int mca_coll_rocm_reduce_scatter_init(const void *sbuf, void *rbuf, const int *rcounts,
                                      struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                      struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                      ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_rocm_scan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                            struct ompi_op_t *op, struct ompi_communicator_t *comm,
                            struct ompi_info_t *info, ompi_request_t **request,
                            mca_coll_base_module_t *module);
int mca_coll_rocm_exscan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, struct ompi_communicator_t *comm,
                              struct ompi_info_t *info, ompi_request_t **request,
                              mca_coll_base_module_t *module);

END_C_DECLS

#endif /* MCA_COLL_ROCM_EXPORT_H */
