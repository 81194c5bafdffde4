/*
 * ompi_amd — point-to-point messages between device buffers of the ranks of
 * one node.  Replaces, for device memory, the PML
 * entry points (ompi/mca/pml/pml.h):
 *
 *   pml_isend  pml.h:317-326   pml_send   pml.h:341-349
 *   pml_irecv  pml.h:233-241   pml_recv   pml.h:262-270
 *   pml_iprobe pml.h:371-377   pml_probe  pml.h:398-403
 *
 * and the CUDA path underneath them: ob1's RDMA rendezvous for device
 * buffers (pml_ob1_cuda.c:56-101) over btl/smcuda, whose get copies from
 * the sender's buffer mapped with a CUDA IPC handle (btl_smcuda.c:1077-1250,
 * common_cuda.c:1008-1320).  Here the same receiver-driven "get" runs as
 * one copy kernel on the receiver's GPU that loads the sender's buffer
 * through its hipIpcOpenMemHandle mapping over xGMI; matching happens on
 * host in a POSIX shared-memory mailbox per (source, destination) pair
 * (created with the communicator), in MPI order: messages from one source
 * are matched in the order they were sent, receives in the order they were
 * posted, MPI_ANY_SOURCE / MPI_ANY_TAG as wildcards.
 *
 * Completion semantics.  A send's data is read in `stream` order (after
 * the work already queued on it).  Messages of at most 4 KiB (btl/smcuda's
 * eager limit) are copied into the sender's device eager area (ob1's eager
 * protocol): from a device buffer by a kernel on `stream` that publishes
 * the cell itself — the message is posted at once, the receiver's copy
 * waits for the cell on the device, and the send completes when that
 * kernel has run; from a host buffer before the call returns.  Larger ones
 * (after a synchronisation of `stream`) are copied into a library-owned
 * send stage (a pool of exported device buffers that live as long as the
 * communicator) and the send completes once staged — the receiver pulls
 * from the stage, so no peer ever maps an application buffer; MPI_Ssend
 * completes at the receiver's FIN.  Past the pool's cap (param
 * "p2p_stage_mib", default 1024) or with param "p2p_user_ipc" = 1 the
 * receiver maps the send buffer itself (rendezvous).  Host (pageable or
 * pinned) buffers are accepted on both sides: a host send always goes
 * through a stage, a host receive lands in a device receive stage and is
 * copied out before it completes.  MPI_Bsend is not provided.  A receive
 * completes when its data is in its buffer.  Host-side waits (a full
 * 64-slot ring, wait, probe) are bounded by param "p2p_timeout_ms" (-1: the
 * communicator's timeout_ms, the default; 0: no limit — the PML glue's
 * setting, MPI semantics).  The byte count is the message size; the MCA
 * glue packs non-contiguous datatypes first.
  */
#ifndef OMPI_AMD_P2P_H
#define OMPI_AMD_P2P_H

#include <stddef.h>
#include <stdint.h>

#include "ompi_amd_coll.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OMPI_AMD_ANY_SOURCE (-1)     /* MPI_ANY_SOURCE */
#define OMPI_AMD_ANY_TAG    (-1)     /* MPI_ANY_TAG */
#define OMPI_AMD_ERR_TRUNCATE (-7)   /* message longer than the receive buffer */

/* mca_pml_base_send_mode_t, same values (pml_constants.h:30-37) */
#define OMPI_AMD_SEND_SYNCHRONOUS 0
#define OMPI_AMD_SEND_COMPLETE    1
#define OMPI_AMD_SEND_BUFFERED    2
#define OMPI_AMD_SEND_READY       3
#define OMPI_AMD_SEND_STANDARD    4

typedef struct ompi_amd_p2p_request ompi_amd_p2p_request_t;

/* ompi_status_public_t's fields (MPI_SOURCE, MPI_TAG, MPI_ERROR, count). */
typedef struct {
    int source;
    int tag;
    int error;
    size_t bytes;
} ompi_amd_status_t;

/* Nonblocking send of `bytes` from `buf` (device or host memory) to rank
 * `dst`.  tag >= 0.  Up to 64 sends to one destination may be unmatched at
 * a time; the 65th waits (bounded by p2p_timeout_ms) for one to
 * complete. */
int ompi_amd_isend(ompi_amd_comm_t *comm, const void *buf, size_t bytes, int dst, int tag,
                   int mode, void *stream, ompi_amd_p2p_request_t **request);
/* Nonblocking receive into `buf` (device or host) of capacity `bytes` from
 * `src` (or OMPI_AMD_ANY_SOURCE) with `tag` (or OMPI_AMD_ANY_TAG).  The
 * copy runs on `stream` once the message is matched. */
int ompi_amd_irecv(ompi_amd_comm_t *comm, void *buf, size_t bytes, int src, int tag,
                   void *stream, ompi_amd_p2p_request_t **request);
/* Blocking forms: isend/irecv + wait + free. */
int ompi_amd_send(ompi_amd_comm_t *comm, const void *buf, size_t bytes, int dst, int tag,
                  int mode, void *stream);
int ompi_amd_recv(ompi_amd_comm_t *comm, void *buf, size_t bytes, int src, int tag,
                  void *stream, ompi_amd_status_t *status);
/* MPI_Sendrecv: both posted before either is waited on. */
int ompi_amd_sendrecv(ompi_amd_comm_t *comm, const void *sbuf, size_t sbytes, int dst, int stag,
                      void *rbuf, size_t rbytes, int src, int rtag, void *stream,
                      ompi_amd_status_t *status);
/* *done = 1 when complete (status filled for receives; status may be NULL).
 * Every test / wait also matches pending receives of the communicator. */
int ompi_amd_p2p_test(ompi_amd_p2p_request_t *request, int *done, ompi_amd_status_t *status);
int ompi_amd_p2p_wait(ompi_amd_p2p_request_t *request, ompi_amd_status_t *status);
/* Waits for completion, then releases the request. */
int ompi_amd_p2p_free(ompi_amd_p2p_request_t *request);
/* MPI_Iprobe / MPI_Probe: a message that a receive with (src, tag) would
 * match, without receiving it. */
int ompi_amd_iprobe(ompi_amd_comm_t *comm, int src, int tag, int *flag, ompi_amd_status_t *status);
int ompi_amd_probe(ompi_amd_comm_t *comm, int src, int tag, ompi_amd_status_t *status);

#ifdef __cplusplus
}
#endif

#endif /* OMPI_AMD_P2P_H */
