/*
 * ompi_amd — one-sided communication on device windows of the ranks of one
 * node.  Replaces, for device memory, osc/sm's module
 * functions (ompi/mca/osc/sm/osc_sm_comm.c, osc_sm_active_target.c,
 * osc_sm_passive_target.c) behind the osc framework's module table
 * (ompi/mca/osc/osc.h):
 *
 *   osc_put / osc_get              osc_sm_comm.c:209-268
 *   osc_accumulate                 osc_sm_comm.c:271-309
 *   osc_get_accumulate             osc_sm_comm.c:312-360
 *   osc_compare_and_swap           osc_sm_comm.c:363-400
 *   osc_fetch_and_op               osc_sm_comm.c:403-441
 *   osc_fence                      osc_sm_active_target.c:95-115 (a barrier)
 *   osc_lock / unlock / flush      osc_sm_passive_target.c:57-270 (ticket lock)
 *
 * osc/sm computes with ompi_op_reduce on the target's shared segment under
 * the target's accumulate spinlock (osc_sm_comm.c:130-139, :296-305).  Here
 * every window is device memory mapped into each peer with
 * hipIpcOpenMemHandle; the origin rank's GPU runs the operation as kernels
 * on its stream that load and store the target's memory over xGMI:
 *   lock kernel   one lane takes the target's accumulate lock (system-scope
 *                 CAS on a word in the target's fine-grained control page);
 *   op kernel     target[i] = f(target[i], origin[i]) with op/base's element
 *                 rule (f(out, in), op_base_functions.c:40-104), preceded by
 *                 a copy target -> result for the fetching forms;
 *   unlock kernel release, then stores 0.
 * All stream-ordered: a call returns after enqueueing; the stream carries
 * the ordering (MPI's default accumulate_ordering rar,raw,war,waw between
 * one origin's calls to one target holds).  Results are bit-identical to
 * osc/sm's for every order of the targets' locks, since each element of the
 * target is combined by one origin's call at a time with op/base's rule.
 *
 * Displacements are in the TARGET's disp_unit (osc_sm_comm.c:289); counts
 * in elements of `type` (its extent, as op/base: DOUBLE_INT 16 B).  op is an
 * OMPI_AMD_OP_* code incl. OMPI_AMD_OP_REPLACE and OMPI_AMD_OP_NO_OP.
 */
#ifndef OMPI_AMD_OSC_H
#define OMPI_AMD_OSC_H

#include <stddef.h>
#include <stdint.h>

#include "ompi_amd_coll.h"
#include "ompi_amd_ddt.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OMPI_AMD_LOCK_EXCLUSIVE 1     /* MPI_LOCK_EXCLUSIVE (mpi.h.in:548) */
#define OMPI_AMD_LOCK_SHARED    2     /* MPI_LOCK_SHARED (mpi.h.in:549) */
#define OMPI_AMD_MODE_NOCHECK   1     /* MPI_MODE_NOCHECK (mpi.h.in:542): lock takes no lock */

typedef struct ompi_amd_win ompi_amd_win_t;
typedef struct ompi_amd_rma_request ompi_amd_rma_request_t;

/* MPI_Win_create over device memory [base, base + bytes) (collective).
 * bytes may be 0 (base ignored). */
int ompi_amd_win_create(ompi_amd_comm_t *comm, void *base, size_t bytes, int disp_unit,
                        ompi_amd_win_t **win);
/* MPI_Win_allocate: the window's memory is allocated here (zeroed). */
int ompi_amd_win_allocate(ompi_amd_comm_t *comm, size_t bytes, int disp_unit, void **base,
                          ompi_amd_win_t **win);
/* MPI_Win_create_dynamic (collective; osc/rdma's flavor, osc_rdma_dynamic.c):
 * a window with no memory; displacements are the target's absolute
 * addresses (disp_unit 1) inside regions the target attached.
 * MPI_Win_attach (local): device memory peers can map as it is (an
 * IPC-safe allocation no IPC close of this process predates) — host memory
 * returns OMPI_AMD_ERR_NOT_DEVICE, other device memory
 * OMPI_AMD_ERR_UNSUPPORTED (MPI_ERR_RMA_ATTACH), at most 64 regions per
 * rank, none overlapping.  MPI_Win_detach (local): base as attached.  An
 * origin finds the target's region at each access; accessing memory the
 * target has not attached is OMPI_AMD_ERR_BAD_PARAM (MPI_ERR_RMA_RANGE). */
int ompi_amd_win_create_dynamic(ompi_amd_comm_t *comm, ompi_amd_win_t **win);
int ompi_amd_win_attach(ompi_amd_win_t *win, void *base, size_t size);
int ompi_amd_win_detach(ompi_amd_win_t *win, const void *base);
/* MPI_Win_free (collective; waits for every rank's outstanding work). */
int ompi_amd_win_free(ompi_amd_win_t *win);
/* MPI_Win_fence: a device barrier on `stream` over the window's ranks.
 * Every RMA call each rank enqueued before its fence (on the same stream)
 * is complete at every target when the fence completes. */
int ompi_amd_win_fence(ompi_amd_win_t *win, int assert_, void *stream);
/* MPI_Win_lock / _unlock (passive target; lock_type as above): the lock
 * kernel on `stream` waits for the target's ticket lock (FIFO; shared
 * holders run together).  Unlock releases it after every RMA call the
 * caller enqueued on `stream` in between. */
int ompi_amd_win_lock(ompi_amd_win_t *win, int lock_type, int target, int assert_, void *stream);
int ompi_amd_win_unlock(ompi_amd_win_t *win, int target, void *stream);
/* MPI_Win_lock_all / unlock_all: shared locks on every rank. */
int ompi_amd_win_lock_all(ompi_amd_win_t *win, int assert_, void *stream);
int ompi_amd_win_unlock_all(ompi_amd_win_t *win, void *stream);
/* MPI_Win_flush: the calls enqueued so far on `stream` are complete at the
 * target when the host returns (synchronises the stream). */
int ompi_amd_win_flush(ompi_amd_win_t *win, int target, void *stream);
/* MPI_Win_sync (osc.h osc_sync): the window's public and private copies
 * merged (separate model, below); nothing to do otherwise. */
int ompi_amd_win_sync(ompi_amd_win_t *win, void *stream);
/* The window's memory model (MPI_WIN_MODEL): UNIFIED, or SEPARATE when some
 * rank's MPI_Win_create memory cannot be mapped by its peers as it is (not
 * an IPC-safe size, or older than an IPC close of that process): that rank's
 * RMA target is a public copy in library memory, merged with the caller's
 * memory (the private copy) at every fence, post / wait, lock / unlock of
 * its own window and MPI_Win_sync; every rank of the window then reports
 * SEPARATE and takes part in the fence's merge step. */
#define OMPI_AMD_WIN_UNIFIED 0
#define OMPI_AMD_WIN_SEPARATE 1
int ompi_amd_win_model(const ompi_amd_win_t *win);
/* Diagnostics (no MPI counterpart): this rank's private copy (the window
 * memory), its public copy and the last merge's snapshot; *pub and *snap
 * are NULL where the window is unified on this rank. */
int ompi_amd_win_copies(const ompi_amd_win_t *win, void **priv, void **pub, void **snap);
/* Diagnostics: rank `peer`'s window memory as this process reaches it (the
 * address RMA toward `peer` targets: its public copy, mapped). */
int ompi_amd_win_peer_base(const ompi_amd_win_t *win, int peer, void **base);

int ompi_amd_put(ompi_amd_win_t *win, const void *origin, size_t bytes, int target, size_t disp,
                 void *stream);
int ompi_amd_get(ompi_amd_win_t *win, void *origin, size_t bytes, int target, size_t disp,
                 void *stream);
/* target = op(target, origin) element-wise, under the target's lock. */
int ompi_amd_accumulate(ompi_amd_win_t *win, const void *origin, size_t count, int type,
                        int target, size_t disp, int op, void *stream);
/* result = target, then target = op(target, origin), as one step. */
int ompi_amd_get_accumulate(ompi_amd_win_t *win, const void *origin, void *result, size_t count,
                            int type, int target, size_t disp, int op, void *stream);
/* MPI_Accumulate / MPI_Get_accumulate with derived datatypes
 * (osc_sm_comm.c:301, 350 -> ompi_osc_base_sndrcv_op,
 * osc_base_obj_convert.c:160-245): the origin's ocount x odt elements, as a
 * packed stream of `type` elements, are combined in order into the element
 * slots of tcount x tdt at the target (get_accumulate: the old elements are
 * returned into rcount x rdt at result first).  odt / rdt / tdt NULL: `type`
 * contiguous.  The three type signatures must hold the same number of
 * `type` elements; pair types (MAXLOC / MINLOC operands) only contiguous. */
int ompi_amd_accumulate_ddt(ompi_amd_win_t *win, const void *origin, size_t ocount,
                            const ompi_amd_ddt_t *odt, int target, size_t disp, size_t tcount,
                            const ompi_amd_ddt_t *tdt, int type, int op, void *stream);
int ompi_amd_get_accumulate_ddt(ompi_amd_win_t *win, const void *origin, size_t ocount,
                                const ompi_amd_ddt_t *odt, void *result, size_t rcount,
                                const ompi_amd_ddt_t *rdt, int target, size_t disp, size_t tcount,
                                const ompi_amd_ddt_t *tdt, int type, int op, void *stream);
/* MPI_Put / MPI_Get with derived datatypes (osc_sm_comm.c:24-100,
 * 209-270: ompi_datatype_sndrcv of any datatype pair): the origin's ocount x
 * odt bytes, in type-map order, into (put) or out of (get) the tcount x tdt
 * layout at the target; only the target type's bytes are written, its gaps
 * keep theirs.  odt / tdt NULL: `ocount` / `tcount` contiguous bytes.  Both
 * sides must move the same number of bytes.  No accumulate lock (put and
 * get are not atomic); inside a passive epoch the epoch's lock gates it. */
int ompi_amd_put_ddt(ompi_amd_win_t *win, const void *origin, size_t ocount,
                     const ompi_amd_ddt_t *odt, int target, size_t disp, size_t tcount,
                     const ompi_amd_ddt_t *tdt, void *stream);
int ompi_amd_get_ddt(ompi_amd_win_t *win, void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                     int target, size_t disp, size_t tcount, const ompi_amd_ddt_t *tdt,
                     void *stream);
/* get_accumulate of one element. */
int ompi_amd_fetch_and_op(ompi_amd_win_t *win, const void *origin, void *result, int type,
                          int target, size_t disp, int op, void *stream);
/* result = target; if target's bytes equal compare's, target = origin. */
int ompi_amd_compare_and_swap(ompi_amd_win_t *win, const void *origin, const void *compare,
                              void *result, int type, int target, size_t disp, void *stream);

/* MPI_Win_allocate_shared (osc_sm_component.c:244-360): rank 0 allocates
 * one exportable device allocation holding every rank's segment back to
 * back (each `bytes`, or rounded up to 4 KiB with noncontig =
 * alloc_shared_noncontig), every other rank maps it once, so the segments
 * are contiguous in every process and kernels may load / store any of them
 * directly.  *base = this rank's segment.  Zero-filled.  Collective. */
int ompi_amd_win_allocate_shared(ompi_amd_comm_t *comm, size_t bytes, int disp_unit, int noncontig,
                                 void **base, ompi_amd_win_t **win);
/* MPI_Win_shared_query (osc_sm_component.c:455-485): size, disp_unit and
 * this process's address of `rank`'s segment; rank < 0 (MPI_PROC_NULL) =
 * the first segment of nonzero size.  Windows not made by
 * ompi_amd_win_allocate_shared: OMPI_AMD_ERR_UNSUPPORTED (osc/sm's
 * MPI_ERR_WIN). */
int ompi_amd_win_shared_query(ompi_amd_win_t *win, int rank, size_t *size, int *disp_unit,
                              void **baseptr);

/* General active target synchronisation (MPI_Win_post / _start /
 * _complete / _wait / _test; osc.h:366-372, osc/sm's
 * osc_sm_active_target.c:126-330).  ranks: the group's members as ranks of
 * the window's communicator.  Stream-ordered like fence: post releases this
 * rank's window and tells each origin; start waits (on the device) until
 * every target of its group posted this epoch; complete releases the
 * epoch's RMA and tells each target; wait waits (on the device) until every
 * origin of the post group completed.  test is host-side and never blocks
 * (*flag = 1 ends the exposure epoch).  The glue syncs the stream where MPI
 * blocks (wait, complete). */
int ompi_amd_win_post(ompi_amd_win_t *win, const int *ranks, int n, int assert_, void *stream);
int ompi_amd_win_start(ompi_amd_win_t *win, const int *ranks, int n, int assert_, void *stream);
int ompi_amd_win_complete(ompi_amd_win_t *win, void *stream);
int ompi_amd_win_wait(ompi_amd_win_t *win, void *stream);
int ompi_amd_win_test(ompi_amd_win_t *win, int *flag);

/* Request-based RMA (MPI_Rput / _Rget / _Raccumulate / _Rget_accumulate,
 * osc.h:384-393): the call as above plus a request that completes when its
 * kernels have finished on `stream` (local and remote completion at once). */
int ompi_amd_rput(ompi_amd_win_t *win, const void *origin, size_t bytes, int target, size_t disp,
                  void *stream, ompi_amd_rma_request_t **request);
int ompi_amd_rget(ompi_amd_win_t *win, void *origin, size_t bytes, int target, size_t disp,
                  void *stream, ompi_amd_rma_request_t **request);
int ompi_amd_raccumulate(ompi_amd_win_t *win, const void *origin, size_t count, int type,
                         int target, size_t disp, int op, void *stream,
                         ompi_amd_rma_request_t **request);
int ompi_amd_rget_accumulate(ompi_amd_win_t *win, const void *origin, void *result, size_t count,
                             int type, int target, size_t disp, int op, void *stream,
                             ompi_amd_rma_request_t **request);
/* request-based forms of the derived-datatype calls above */
int ompi_amd_rput_ddt(ompi_amd_win_t *win, const void *origin, size_t ocount,
                      const ompi_amd_ddt_t *odt, int target, size_t disp, size_t tcount,
                      const ompi_amd_ddt_t *tdt, void *stream, ompi_amd_rma_request_t **req);
int ompi_amd_rget_ddt(ompi_amd_win_t *win, void *origin, size_t ocount, const ompi_amd_ddt_t *odt,
                      int target, size_t disp, size_t tcount, const ompi_amd_ddt_t *tdt, void *stream,
                      ompi_amd_rma_request_t **req);
int ompi_amd_raccumulate_ddt(ompi_amd_win_t *win, const void *origin, size_t ocount,
                             const ompi_amd_ddt_t *odt, int target, size_t disp, size_t tcount,
                             const ompi_amd_ddt_t *tdt, int type, int op, void *stream,
                             ompi_amd_rma_request_t **req);
int ompi_amd_rget_accumulate_ddt(ompi_amd_win_t *win, const void *origin, size_t ocount,
                                 const ompi_amd_ddt_t *odt, void *result, size_t rcount,
                                 const ompi_amd_ddt_t *rdt, int target, size_t disp,
                                 size_t tcount, const ompi_amd_ddt_t *tdt, int type, int op,
                                 void *stream, ompi_amd_rma_request_t **req);
int ompi_amd_rma_test(ompi_amd_rma_request_t *request, int *done);
int ompi_amd_rma_wait(ompi_amd_rma_request_t *request);
int ompi_amd_rma_free(ompi_amd_rma_request_t *request);

#ifdef __cplusplus
}
#endif

#endif /* OMPI_AMD_OSC_H */
