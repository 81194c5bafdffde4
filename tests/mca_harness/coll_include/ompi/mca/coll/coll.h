/* TEST HARNESS ONLY: the coll framework types the glue uses, with the
 * reference's function signatures (ompi/mca/coll/coll.h:141-143, 200-250,
 * 261-274, 293-300, 311-326, 339-343, 349-352, 371-374, 381-400, 471-603). */
#ifndef HARNESS_COLL_H
#define HARNESS_COLL_H
#include <stdbool.h>
#include "ompi/mca/mca.h"
#include "opal/class/opal_object.h"
#include "ompi/request/request.h"
struct ompi_communicator_t;
struct ompi_info_t;
struct ompi_datatype_t;
struct ompi_op_t;
struct mca_coll_base_module_2_3_0_t;
#define HMOD struct mca_coll_base_module_2_3_0_t *
typedef int (*mca_coll_base_module_allgather_fn_t)(const void *, int, struct ompi_datatype_t *,
                                                   void *, int, struct ompi_datatype_t *,
                                                   struct ompi_communicator_t *, HMOD);
typedef int (*mca_coll_base_module_allreduce_fn_t)(const void *, void *, int, struct ompi_datatype_t *,
                                                   struct ompi_op_t *, struct ompi_communicator_t *,
                                                   HMOD);
typedef int (*mca_coll_base_module_bcast_fn_t)(void *, int, struct ompi_datatype_t *, int,
                                               struct ompi_communicator_t *, HMOD);
typedef int (*mca_coll_base_module_exscan_fn_t)(const void *, void *, int, struct ompi_datatype_t *,
                                                struct ompi_op_t *, struct ompi_communicator_t *, HMOD);
typedef int (*mca_coll_base_module_reduce_fn_t)(const void *, void *, int, struct ompi_datatype_t *,
                                                struct ompi_op_t *, int, struct ompi_communicator_t *,
                                                HMOD);
typedef int (*mca_coll_base_module_reduce_scatter_fn_t)(const void *, void *, const int *,
                                                        struct ompi_datatype_t *,
                                                        struct ompi_op_t *,
                                                        struct ompi_communicator_t *, HMOD);
typedef int (*mca_coll_base_module_reduce_scatter_block_fn_t)(const void *, void *, int,
                                                              struct ompi_datatype_t *,
                                                              struct ompi_op_t *,
                                                              struct ompi_communicator_t *, HMOD);
typedef int (*mca_coll_base_module_scan_fn_t)(const void *, void *, int, struct ompi_datatype_t *,
                                              struct ompi_op_t *, struct ompi_communicator_t *, HMOD);
typedef int (*mca_coll_base_module_iallreduce_fn_t)(const void *, void *, int,
                                                    struct ompi_datatype_t *, struct ompi_op_t *,
                                                    struct ompi_communicator_t *,
                                                    ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_iallgather_fn_t)(const void *, int, struct ompi_datatype_t *,
                                                    void *, int, struct ompi_datatype_t *,
                                                    struct ompi_communicator_t *, ompi_request_t **,
                                                    HMOD);
typedef int (*mca_coll_base_module_ibcast_fn_t)(void *, int, struct ompi_datatype_t *, int,
                                                struct ompi_communicator_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_ireduce_scatter_block_fn_t)(const void *, void *, int,
                                                               struct ompi_datatype_t *,
                                                               struct ompi_op_t *,
                                                               struct ompi_communicator_t *,
                                                               ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_allreduce_init_fn_t)(const void *, void *, int,
                                                        struct ompi_datatype_t *, struct ompi_op_t *,
                                                        struct ompi_communicator_t *,
                                                        struct ompi_info_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_iexscan_fn_t)(const void *, void *, int, struct ompi_datatype_t *,
                                                 struct ompi_op_t *, struct ompi_communicator_t *,
                                                 ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_ireduce_fn_t)(const void *, void *, int, struct ompi_datatype_t *,
                                                 struct ompi_op_t *, int, struct ompi_communicator_t *,
                                                 ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_ireduce_scatter_fn_t)(const void *, void *, const int *,
                                                         struct ompi_datatype_t *, struct ompi_op_t *,
                                                         struct ompi_communicator_t *,
                                                         ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_iscan_fn_t)(const void *, void *, int, struct ompi_datatype_t *,
                                               struct ompi_op_t *, struct ompi_communicator_t *,
                                               ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_allgather_init_fn_t)(const void *, int, struct ompi_datatype_t *,
                                                        void *, int, struct ompi_datatype_t *,
                                                        struct ompi_communicator_t *,
                                                        struct ompi_info_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_bcast_init_fn_t)(void *, int, struct ompi_datatype_t *, int,
                                                    struct ompi_communicator_t *, struct ompi_info_t *,
                                                    ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_reduce_scatter_block_init_fn_t)(
    const void *, void *, int, struct ompi_datatype_t *, struct ompi_op_t *,
    struct ompi_communicator_t *, struct ompi_info_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_exscan_init_fn_t)(const void *, void *, int,
                                                     struct ompi_datatype_t *, struct ompi_op_t *,
                                                     struct ompi_communicator_t *,
                                                     struct ompi_info_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_reduce_init_fn_t)(const void *, void *, int,
                                                     struct ompi_datatype_t *, struct ompi_op_t *, int,
                                                     struct ompi_communicator_t *,
                                                     struct ompi_info_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_reduce_scatter_init_fn_t)(
    const void *, void *, const int *, struct ompi_datatype_t *, struct ompi_op_t *,
    struct ompi_communicator_t *, struct ompi_info_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_scan_init_fn_t)(const void *, void *, int,
                                                   struct ompi_datatype_t *, struct ompi_op_t *,
                                                   struct ompi_communicator_t *,
                                                   struct ompi_info_t *, ompi_request_t **, HMOD);
typedef int (*mca_coll_base_module_enable_1_1_0_fn_t)(HMOD, struct ompi_communicator_t *);
#undef HMOD
typedef struct mca_coll_base_module_2_3_0_t {
    opal_object_t super;
    mca_coll_base_module_enable_1_1_0_fn_t coll_module_enable;
    mca_coll_base_module_allgather_fn_t coll_allgather;
    mca_coll_base_module_allreduce_fn_t coll_allreduce;
    mca_coll_base_module_bcast_fn_t coll_bcast;
    mca_coll_base_module_exscan_fn_t coll_exscan;
    mca_coll_base_module_reduce_fn_t coll_reduce;
    mca_coll_base_module_reduce_scatter_fn_t coll_reduce_scatter;
    mca_coll_base_module_reduce_scatter_block_fn_t coll_reduce_scatter_block;
    mca_coll_base_module_scan_fn_t coll_scan;
    mca_coll_base_module_iallgather_fn_t coll_iallgather;
    mca_coll_base_module_iallreduce_fn_t coll_iallreduce;
    mca_coll_base_module_ibcast_fn_t coll_ibcast;
    mca_coll_base_module_ireduce_scatter_block_fn_t coll_ireduce_scatter_block;
    mca_coll_base_module_iexscan_fn_t coll_iexscan;
    mca_coll_base_module_ireduce_fn_t coll_ireduce;
    mca_coll_base_module_ireduce_scatter_fn_t coll_ireduce_scatter;
    mca_coll_base_module_iscan_fn_t coll_iscan;
    mca_coll_base_module_allgather_init_fn_t coll_allgather_init;
    mca_coll_base_module_allreduce_init_fn_t coll_allreduce_init;
    mca_coll_base_module_bcast_init_fn_t coll_bcast_init;
    mca_coll_base_module_reduce_scatter_block_init_fn_t coll_reduce_scatter_block_init;
    mca_coll_base_module_exscan_init_fn_t coll_exscan_init;
    mca_coll_base_module_reduce_init_fn_t coll_reduce_init;
    mca_coll_base_module_reduce_scatter_init_fn_t coll_reduce_scatter_init;
    mca_coll_base_module_scan_init_fn_t coll_scan_init;
    void *base_data;
} mca_coll_base_module_2_3_0_t;
typedef mca_coll_base_module_2_3_0_t mca_coll_base_module_t;
OBJ_CLASS_DECLARATION(mca_coll_base_module_t);
typedef int (*mca_coll_base_component_init_query_fn_t)(bool, bool);
typedef mca_coll_base_module_t *(*mca_coll_base_component_comm_query_2_0_0_fn_t)(
    struct ompi_communicator_t *, int *);
typedef struct mca_coll_base_component_2_0_0_t {
    mca_base_component_t collm_version;
    mca_base_component_data_t collm_data;
    mca_coll_base_component_init_query_fn_t collm_init_query;
    mca_coll_base_component_comm_query_2_0_0_fn_t collm_comm_query;
} mca_coll_base_component_2_0_0_t;
/* per-communicator function table (coll.h:608-666 shape) */
#define HFN(name) mca_coll_base_module_##name##_fn_t coll_##name; mca_coll_base_module_t *coll_##name##_module;
typedef struct mca_coll_base_comm_coll_t {
    HFN(allgather) HFN(allreduce) HFN(bcast) HFN(exscan) HFN(reduce) HFN(reduce_scatter)
    HFN(reduce_scatter_block)
    HFN(scan) HFN(iallgather) HFN(iallreduce) HFN(ibcast) HFN(ireduce_scatter_block)
    HFN(iexscan) HFN(ireduce) HFN(ireduce_scatter) HFN(iscan)
    HFN(allgather_init) HFN(allreduce_init) HFN(bcast_init) HFN(reduce_scatter_block_init)
    HFN(exscan_init) HFN(reduce_init) HFN(reduce_scatter_init) HFN(scan_init)
} mca_coll_base_comm_coll_t;
#undef HFN
#define MCA_COLL_BASE_VERSION_2_0_0 OMPI_MCA_BASE_VERSION_2_1_0("coll", 2, 0, 0)
#endif
