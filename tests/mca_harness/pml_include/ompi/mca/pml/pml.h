/* TEST HARNESS ONLY: the PML framework types pml/rocm uses, with the
 * reference's signatures and slot order (ompi/mca/pml/pml.h:97-112,
 * 134-478, 492-527; pml_constants.h:30-37). */
#ifndef HARNESS_PML_H
#define HARNESS_PML_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include "ompi/mca/mca.h"
#include "ompi/request/request.h"
struct ompi_communicator_t;
struct ompi_datatype_t;
struct ompi_proc_t;
struct ompi_message_t;
typedef enum {
    MCA_PML_BASE_SEND_SYNCHRONOUS,
    MCA_PML_BASE_SEND_COMPLETE,
    MCA_PML_BASE_SEND_BUFFERED,
    MCA_PML_BASE_SEND_READY,
    MCA_PML_BASE_SEND_STANDARD,
    MCA_PML_BASE_SEND_SIZE
} mca_pml_base_send_mode_t;
typedef struct mca_pml_base_module_1_0_1_t *(*mca_pml_base_component_init_fn_t)(
    int *priority, bool enable_progress_threads, bool enable_mpi_threads);
typedef int (*mca_pml_base_component_finalize_fn_t)(void);
typedef struct mca_pml_base_component_2_0_0_t {
    mca_base_component_t pmlm_version;
    mca_base_component_data_t pmlm_data;
    mca_pml_base_component_init_fn_t pmlm_init;
    mca_pml_base_component_finalize_fn_t pmlm_finalize;
} mca_pml_base_component_2_0_0_t;
typedef int (*mca_pml_base_module_add_procs_fn_t)(struct ompi_proc_t **procs, size_t nprocs);
typedef int (*mca_pml_base_module_del_procs_fn_t)(struct ompi_proc_t **procs, size_t nprocs);
typedef int (*mca_pml_base_module_enable_fn_t)(bool enable);
typedef int (*mca_pml_base_module_progress_fn_t)(void);
typedef int (*mca_pml_base_module_add_comm_fn_t)(struct ompi_communicator_t *comm);
typedef int (*mca_pml_base_module_del_comm_fn_t)(struct ompi_communicator_t *comm);
typedef int (*mca_pml_base_module_irecv_init_fn_t)(void *buf, size_t count,
                                                   struct ompi_datatype_t *datatype, int src,
                                                   int tag, struct ompi_communicator_t *comm,
                                                   struct ompi_request_t **request);
typedef int (*mca_pml_base_module_irecv_fn_t)(void *buf, size_t count,
                                              struct ompi_datatype_t *datatype, int src, int tag,
                                              struct ompi_communicator_t *comm,
                                              struct ompi_request_t **request);
typedef int (*mca_pml_base_module_recv_fn_t)(void *buf, size_t count,
                                             struct ompi_datatype_t *datatype, int src, int tag,
                                             struct ompi_communicator_t *comm,
                                             ompi_status_public_t *status);
typedef int (*mca_pml_base_module_isend_init_fn_t)(const void *buf, size_t count,
                                                   struct ompi_datatype_t *datatype, int dst,
                                                   int tag, mca_pml_base_send_mode_t mode,
                                                   struct ompi_communicator_t *comm,
                                                   struct ompi_request_t **request);
typedef int (*mca_pml_base_module_isend_fn_t)(const void *buf, size_t count,
                                              struct ompi_datatype_t *datatype, int dst, int tag,
                                              mca_pml_base_send_mode_t mode,
                                              struct ompi_communicator_t *comm,
                                              struct ompi_request_t **request);
typedef int (*mca_pml_base_module_send_fn_t)(const void *buf, size_t count,
                                             struct ompi_datatype_t *datatype, int dst, int tag,
                                             mca_pml_base_send_mode_t mode,
                                             struct ompi_communicator_t *comm);
typedef ompi_request_start_fn_t mca_pml_base_module_start_fn_t;
typedef int (*mca_pml_base_module_iprobe_fn_t)(int src, int tag, struct ompi_communicator_t *comm,
                                               int *matched, ompi_status_public_t *status);
typedef int (*mca_pml_base_module_improbe_fn_t)(int src, int tag, struct ompi_communicator_t *comm,
                                                int *matched, struct ompi_message_t **message,
                                                ompi_status_public_t *status);
typedef int (*mca_pml_base_module_probe_fn_t)(int src, int tag, struct ompi_communicator_t *comm,
                                              ompi_status_public_t *status);
typedef int (*mca_pml_base_module_mprobe_fn_t)(int src, int tag, struct ompi_communicator_t *comm,
                                               struct ompi_message_t **message,
                                               ompi_status_public_t *status);
typedef int (*mca_pml_base_module_imrecv_fn_t)(void *buf, size_t count,
                                               struct ompi_datatype_t *datatype,
                                               struct ompi_message_t **message,
                                               struct ompi_request_t **request);
typedef int (*mca_pml_base_module_mrecv_fn_t)(void *buf, size_t count,
                                              struct ompi_datatype_t *datatype,
                                              struct ompi_message_t **message,
                                              ompi_status_public_t *status);
typedef int (*mca_pml_base_module_dump_fn_t)(struct ompi_communicator_t *comm, int verbose);
typedef int (*mca_pml_base_module_ft_event_fn_t)(int status);
typedef struct mca_pml_base_module_1_0_1_t {
    mca_pml_base_module_add_procs_fn_t pml_add_procs;
    mca_pml_base_module_del_procs_fn_t pml_del_procs;
    mca_pml_base_module_enable_fn_t pml_enable;
    mca_pml_base_module_progress_fn_t pml_progress;
    mca_pml_base_module_add_comm_fn_t pml_add_comm;
    mca_pml_base_module_del_comm_fn_t pml_del_comm;
    mca_pml_base_module_irecv_init_fn_t pml_irecv_init;
    mca_pml_base_module_irecv_fn_t pml_irecv;
    mca_pml_base_module_recv_fn_t pml_recv;
    mca_pml_base_module_isend_init_fn_t pml_isend_init;
    mca_pml_base_module_isend_fn_t pml_isend;
    mca_pml_base_module_send_fn_t pml_send;
    mca_pml_base_module_iprobe_fn_t pml_iprobe;
    mca_pml_base_module_probe_fn_t pml_probe;
    mca_pml_base_module_start_fn_t pml_start;
    mca_pml_base_module_improbe_fn_t pml_improbe;
    mca_pml_base_module_mprobe_fn_t pml_mprobe;
    mca_pml_base_module_imrecv_fn_t pml_imrecv;
    mca_pml_base_module_mrecv_fn_t pml_mrecv;
    mca_pml_base_module_dump_fn_t pml_dump;
    mca_pml_base_module_ft_event_fn_t pml_ft_event;
    uint32_t pml_max_contextid;
    int pml_max_tag;
    int pml_flags;
} mca_pml_base_module_1_0_1_t;
typedef mca_pml_base_module_1_0_1_t mca_pml_base_module_t;
#define MCA_PML_BASE_VERSION_2_0_0 OMPI_MCA_BASE_VERSION_2_1_0("pml", 2, 0, 0)
extern mca_pml_base_module_t mca_pml;
#endif
