/*
 * ompi_amd — device-buffer collectives over xGMI (one process per GPU, one
 * node).  Replaces coll/tuned's (and coll/basic's) functions for device
 * buffers behind the coll framework's module table
 * (ompi/mca/coll/coll.h:200-247):
 *
 *   coll_allreduce            coll.h:208-210  (tuned: coll_tuned_decision_fixed.c:45-89)
 *   coll_reduce               coll.h:239-241  (tuned: :354-428)
 *   coll_reduce_scatter_block coll.h:245-247  (tuned: :522-532)
 *   coll_reduce_scatter       coll.h:242-244  (tuned: :466-512)
 *   coll_scan / coll_exscan   coll.h:248-250, 228-230 (basic: coll_base_scan.c:35-122,
 *                                                      coll_base_exscan.c:35-107)
 *   coll_allgather            coll.h:200-203  (tuned: :543-600)
 *   coll_bcast                coll.h:225-227  (tuned: :234-300)
 *
 * Data moves by kernels that load peer memory mapped with
 * hipIpcOpenMemHandle (replacing the PML/BTL path and the CUDA IPC
 * handshake of btl/smcuda, btl_smcuda.c:1077-1250), with the reduction
 * fused into the load.  Peers synchronise through device-scope flags in
 * IPC-mapped memory; the only host rendezvous is a POSIX shared-memory
 * segment used to swap IPC handles (bootstrap, and per call for
 * zero-copy user buffers).
 *
 * Results: ring / ring_segmented summation order for >= 10000-byte
 * allreduces and the recursive-doubling tree below; for reduce and
 * reduce_scatter_block the operand order of the algorithm coll/tuned's
 * fixed decision picks (basic_linear, in-order binomial, pipeline chain or
 * binary tree); the linear order for scan/exscan — so fp results are
 * bit-identical to coll/tuned (+ coll/basic) + op/base.
 */
#ifndef OMPI_AMD_COLL_H
#define OMPI_AMD_COLL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMPI_AMD_MAX_RANKS 16

typedef struct ompi_amd_comm ompi_amd_comm_t;
typedef struct ompi_amd_plan ompi_amd_plan_t;
typedef struct ompi_amd_request ompi_amd_request_t;

/* Collective over the `size` ranks of one node.  `name` identifies the
 * communicator node-wide and must be unique per job (e.g. "<jobid>.<cid>");
 * it names the POSIX shared-memory rendezvous segment.  `device` is this
 * rank's HIP device (-1: the calling thread's current device).  Every rank
 * calls it with the same name and size. */
int ompi_amd_comm_create(const char *name, int rank, int size, int device,
                         ompi_amd_comm_t **comm);
/* Collective: every rank must call it. */
int ompi_amd_comm_destroy(ompi_amd_comm_t *comm);
int ompi_amd_comm_rank(const ompi_amd_comm_t *comm);
int ompi_amd_comm_size(const ompi_amd_comm_t *comm);

/* MCA-parameter surface (coll_rocm_*):
 *   "small_bytes"   messages up to this size go through the staged path
 *                   (copy into the IPC scratch, no host rendezvous);
 *                   default 1 MiB, capped at the scratch size
 *   "zero_copy"     1 (default): large messages move peer to peer (through
 *                   shadows, or the caller's buffers with user_ipc);
 *                   0: always stage through the scratch
 *   "user_ipc"      0 (default): every large call stages what peers read
 *                   into the communicator's shadow arena (exported once,
 *                   freed only with the communicator); 1: peers map the
 *                   caller's buffers directly (env OMPI_AMD_USER_IPC) —
 *                   only for buffers that are not freed and reallocated
 *                   while the communicator lives
 *   "timeout_ms"    device spin limit per barrier (default 30000)
 *   "blocks"        grid cap of the transfer kernels (default 1024)
 *   "algorithm"     data movement of zero-copy allreduces (all ranks alike):
 *                   0 pull (reduce own block from peers' inputs, then pull
 *                   the other blocks), 1 pull+push (reduce own block and
 *                   store it into every rbuf in the same pass), 2 push
 *                   (default: scatter blocks into the owners' landing
 *                   buffers, owners reduce locally; with user_ipc 0 the
 *                   results are gathered from the owners' landing result
 *                   slots — no staging copy, nothing of the caller's
 *                   exported — with user_ipc 1 stored into every rbuf).
 *                   Env OMPI_AMD_COLL_ALGORITHM sets the default.
 *   "profile"       1: bracket the allreduce's fold, gather and scatter
 *                   kernels with HIP events (read with ompi_amd_comm_phase_ms)
 *   "force_shadow"  1: zero-copy calls treat every user buffer as one the
 *                   runtime refused to export and run through the export
 *                   fallback (a shadow copy of the communicator's own);
 *                   for tests */
int ompi_amd_comm_set_param(ompi_amd_comm_t *comm, const char *key, int64_t value);
/* Read a parameter above, or a state counter: "landing_bytes" (current
 * landing-buffer capacity), "landing_deferred_growths" (growths nonblocking
 * calls queued and progress completed), "landing_retired" (landing buffers
 * any growth replaced, kept until the communicator is destroyed), "imports" (this communicator's references to
 * peer mappings), "shadowed" (zero-copy calls that ran through the export
 * fallback), and the process-wide IPC registry's counters (mappings are
 * shared by every communicator, window and message of the process and
 * closed with their last reference): "ipc_opens" / "ipc_closes" (runtime
 * open / close calls made), "ipc_shared" (maps answered from a mapping the
 * process already held), "ipc_retired" (mappings closed because the
 * exporter freed the allocation), "ipc_live", "ipc_refs"; "ipc_mode_legacy"
 * (HSA_ENABLE_IPC_MODE_LEGACY in effect, -1 unset) and
 * "ipc_mode_legacy_env" (its value when the library was loaded, -1 unset:
 * the library then defaulted it to 0). */
int ompi_amd_comm_get_param(const ompi_amd_comm_t *comm, const char *key, int64_t *value);

/* Sticky error of the device side (a barrier that timed out, ...).
 * 0 = none, else an OMPI_AMD_ERR_* code.  Reading it does not sync. */
int ompi_amd_comm_error(const ompi_amd_comm_t *comm);

/* Host-side agreement across the communicator (shared-memory rendezvous,
 * no GPU work): *all_ok = 1 iff every rank passed local_ok != 0.  The MCA
 * glue uses it so that all ranks take the device path or all fall back to
 * the saved tuned functions (buffer residency may differ across ranks). */
int ompi_amd_comm_agree(ompi_amd_comm_t *comm, int local_ok, int *all_ok);
/* The same rendezvous, counting: *n_yes = number of ranks that passed
 * local_yes != 0 (all ranks get the same count).  coll/rocm's residency
 * vote: size = all device, 0 = all host, else mixed.  Each call (agree,
 * vote, and every host-side handle swap) adds one to get_param
 * "boot_calls". */
int ompi_amd_comm_vote(ompi_amd_comm_t *comm, int local_yes, int *n_yes);

/* MPI_Allreduce's blocking form: ompi_amd_allreduce on the per-thread
 * stream, then the wait ompi_amd_comm_sync would do.  A fused small
 * allreduce (<= fused_bytes) stores its own host-observed completion from
 * its last workgroup, so the wait needs no mark kernel behind it (coll/rocm's
 * blocking allreduce; OMPI_AMD_FUSED_MARK=0 turns the embedded mark off). */
int ompi_amd_allreduce_wait(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count,
                            int type, int op);

/* This rank cannot take part in a collective its peers will run on the
 * device (e.g. staging its operands failed after the path was agreed):
 * make `rc` (an OMPI_AMD_ERR_* code) this communicator's sticky error and
 * raise every peer's abort word, so the peers' barrier waits give up within
 * about 1 ms and their calls fail with OMPI_AMD_ERR_TIMEOUT instead of
 * waiting out timeout_ms.  The communicator is unusable afterwards (MPI:
 * an error in a collective leaves it undefined). */
int ompi_amd_comm_abort(ompi_amd_comm_t *comm, int rc);

/* Wait for `stream` (NULL = per-thread) and report a sticky device error:
 * the blocking completion the MPI entry points need. */
int ompi_amd_comm_sync(ompi_amd_comm_t *comm, void *stream);

/* Kernel time of the profiled allreduce phases since the last read:
 * phase 0 = the reduction (fold), 1 = the peer gather of finished blocks,
 * 2 = the scatter of input blocks into the owners' landing slots (push
 * schemes).  Waits for the recorded events. */
int ompi_amd_comm_phase_ms(ompi_amd_comm_t *comm, int phase, double *total_ms, int *calls);

/* The ring block partition and ownership the allreduce uses (host-only,
 * no GPU needed): block b covers elements [off, off+cnt) of the vector
 * (COLL_BASE_COMPUTE_BLOCKCOUNT, coll_base_functions.h:425-431) and is
 * produced by rank (b - 1) mod size — where the reference's ring finishes
 * it (coll_base_allreduce.c:478-492). */
int ompi_amd_coll_block(size_t count, int size, int block, size_t *off, size_t *cnt);
int ompi_amd_coll_owner(int size, int block);
/* The operand order coll/tuned's fixed reduce decision gives a commutative
 * op (coll_tuned_decision_fixed.c:354-428; msg_bytes = type size * count):
 * *order 2 = chain (basic_linear when *first == 0 and no root in-place
 * swap, else pipeline rooted at *first), 3 = in-order binomial, 4 = binary
 * tree, rooted at *first.  Host-only. */
int ompi_amd_coll_reduce_order(int size, size_t msg_bytes, size_t count, int root,
                               int root_inplace, int *order, int *first);
/* The same under coll_tuned_use_dynamic_rules with coll_tuned_reduce_algorithm
 * = forced (coll_tuned_reduce_decision.c:146-179): 1 basic_linear, 3 pipeline,
 * 4 binary, 5 binomial (0: the fixed decision above).  The others (2 chain
 * with fan-out, 6 in-order binary, 7 Rabenseifner) return
 * OMPI_AMD_ERR_UNSUPPORTED: the device path does not run them and coll/rocm
 * leaves those reductions to coll/tuned.  Host-only. */
int ompi_amd_coll_reduce_order_forced(int size, size_t msg_bytes, size_t count, int root,
                                      int root_inplace, int forced, int *order, int *first);

/* MPI_IN_PLACE is spelled sbuf == rbuf or sbuf == (void *)1.
 * Stream-ordered: results are valid when `stream` reaches this point; the
 * caller keeps every rank's buffers alive until then.  All ranks must call
 * with matching arguments, in the same order. */
int ompi_amd_allreduce(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                       size_t count, int type, int op, void *stream);
/* Persistent allreduce (MPI_Allreduce_init, coll.h:349-352; libnbc's
 * ompi_coll_libnbc_allreduce_init in the reference).  Collective and
 * blocking: fixes sbuf/rbuf/count/type/op, picks the path, swaps and pins
 * the peers' buffer mappings (and sizes the landing buffer for the push
 * scheme).  ompi_amd_plan_start enqueues one allreduce on `stream` with no
 * host rendezvous — a truly nonblocking start; every rank must start its
 * plans in the same order relative to its other collectives.
 * ompi_amd_plan_free is local; free plans before the communicator. */
int ompi_amd_allreduce_init(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                            size_t count, int type, int op, ompi_amd_plan_t **plan);
int ompi_amd_plan_start(ompi_amd_plan_t *plan, void *stream);
/* Completion of the last start (the request's MPI_Test / MPI_Wait):
 * *done = 1 once the device work finished (or nothing was started); a
 * device-side failure (barrier timeout) is returned as its error code.
 * The completion point is marked on the start's stream at the first test /
 * wait after the start (keeping the start itself to kernel launches), so
 * work queued on that stream in between also has to finish first. */
int ompi_amd_plan_test(ompi_amd_plan_t *plan, int *done);
int ompi_amd_plan_wait(ompi_amd_plan_t *plan);
int ompi_amd_plan_free(ompi_amd_plan_t *plan);
/* Persistent reduce_scatter_block / allgather / bcast (MPI-4
 * MPI_Reduce_scatter_block_init / MPI_Allgather_init / MPI_Bcast_init;
 * coll.h:545-566 coll_*_init).  Local (nothing is exchanged at init); every
 * ompi_amd_plan_start posts the nonblocking call with the init's arguments
 * on `stream` (it never waits for a peer) and ompi_amd_plan_test / _wait /
 * _free follow that call's request; a start waits for the previous one to
 * have completed (MPI requires it anyway).  Same argument rules as the
 * blocking calls (rbuf / buf, MPI_IN_PLACE = (void *)1). */
int ompi_amd_reduce_scatter_block_init(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                                       size_t rcount, int type, int op, ompi_amd_plan_t **plan);
int ompi_amd_allgather_init(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes,
                            ompi_amd_plan_t **plan);
int ompi_amd_bcast_init(ompi_amd_comm_t *comm, void *buf, size_t bytes, int root,
                        ompi_amd_plan_t **plan);
/* Persistent reduce / reduce_scatter / scan / exscan (MPI-4 MPI_Reduce_init,
 * MPI_Reduce_scatter_init, MPI_Scan_init, MPI_Exscan_init; coll.h:561-567
 * coll_reduce_init / coll_reduce_scatter_init / coll_scan_init /
 * coll_exscan_init).  Plans of kind 4, as above: local at init, every start
 * posts ompi_amd_ireduce / _ireduce_scatter / _iscan / _iexscan with the
 * init's arguments (rcounts is copied at init).  Results exactly those of
 * the blocking calls. */
int ompi_amd_reduce_init(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count,
                         int type, int op, int root, ompi_amd_plan_t **plan);
int ompi_amd_reduce_scatter_init(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                                 const size_t *rcounts, int type, int op, ompi_amd_plan_t **plan);
int ompi_amd_scan_init(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count,
                       int type, int op, ompi_amd_plan_t **plan);
int ompi_amd_exscan_init(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count,
                         int type, int op, ompi_amd_plan_t **plan);
/* Which path a plan's starts take (diagnostics / tests): 0 = the plain call
 * re-run (fused / staged sizes, and the default push-gather scheme at any
 * size: no handle swap), 1 pull, 2 pull+push, 3 push with the caller's
 * buffers mapped (user_ipc), 4 a persistent reduce_scatter_block /
 * allgather / bcast / reduce / reduce_scatter / scan / exscan; -1 for NULL. */
int ompi_amd_plan_kind(const ompi_amd_plan_t *plan);
/* Nonblocking allreduce (MPI_Iallreduce, coll.h:271-274; libnbc's
 * ompi_coll_libnbc_iallreduce in the reference).  Returns without waiting
 * for any peer: sizes without a handle swap (fused / staged paths) are
 * enqueued on `stream` at once; zero-copy sizes post this rank's half of the
 * handle swap and are launched by the first ompi_amd_request_test / _wait
 * (or the next collective call on `comm`) that finds every peer's half.
 * Deferred calls launch in posting order, and every other collective entry
 * point launches them first, so device work enters every rank's stream in
 * the same order.  Up to 7 calls with a handle swap may be outstanding; the
 * 8th waits for the peers to post the 1st.  Results and errors as
 * ompi_amd_allreduce once the request completes. */
int ompi_amd_iallreduce(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count,
                        int type, int op, void *stream, ompi_amd_request_t **request);
/* Nonblocking forms of the other hot-path collectives
 * (coll_ireduce_scatter_block / coll_iallgather / coll_ibcast, coll.h:261-410;
 * libnbc's ompi_coll_libnbc_ireduce_scatter_block / _iallgather / _ibcast in
 * the reference), on the same post / progress machinery and request type as
 * ompi_amd_iallreduce: sizes at most small_bytes are enqueued at once;
 * zero-copy sizes post this rank's descriptor of what its peers read and
 * launch once every peer posted.  Results exactly those of the blocking
 * calls.  An in-place ireduce_scatter_block at a zero-copy size reads this
 * rank's input from a shadow copy (its rbuf is written while peers read). */
int ompi_amd_ireduce_scatter_block(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                                   size_t rcount, int type, int op, void *stream,
                                   ompi_amd_request_t **request);
int ompi_amd_iallgather(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes,
                        void *stream, ompi_amd_request_t **request);
int ompi_amd_ibcast(ompi_amd_comm_t *comm, void *buf, size_t bytes, int root, void *stream,
                    ompi_amd_request_t **request);
/* Nonblocking reduce / scan / exscan / reduce_scatter (coll_ireduce,
 * coll_iscan, coll_iexscan, coll_ireduce_scatter: coll.h:276-300; libnbc's
 * in the reference).  Results exactly those of the blocking calls (the same
 * operand orders).  They post no buffer descriptors: every size launches on
 * the staged or landing paths, in posting order, with no handle swap (a
 * zero-copy size grows the landing buffer at post time if it must —
 * collective, as for ompi_amd_iallreduce).  ompi_amd_ireduce posts one
 * ticket carrying the root's MPI_IN_PLACE choice and launches once every
 * peer posted it. */
int ompi_amd_ireduce(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type,
                     int op, int root, void *stream, ompi_amd_request_t **request);
int ompi_amd_iscan(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type,
                   int op, void *stream, ompi_amd_request_t **request);
int ompi_amd_iexscan(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type,
                     int op, void *stream, ompi_amd_request_t **request);
int ompi_amd_ireduce_scatter(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                             const size_t *rcounts, int type, int op, void *stream,
                             ompi_amd_request_t **request);
/* *done = 1 once the collective's device work finished; launches deferred
 * calls whose swap completed (never waits for a peer).  As for plans, the
 * completion point is marked at the first test / wait after the launch. */
int ompi_amd_request_test(ompi_amd_request_t *request, int *done);
/* Waits for the peers' swap halves (if needed) and for the device work. */
int ompi_amd_request_wait(ompi_amd_request_t *request);
/* Completes (waits) and releases the request. */
int ompi_amd_request_free(ompi_amd_request_t *request);
/* MPI_Reduce to `root` (coll.h:239-241).  rbuf matters at the root only;
 * the root may pass sbuf = MPI_IN_PLACE.  Every rank folds one block of the
 * vector from every rank's sbuf and stores it into the root's rbuf. */
int ompi_amd_reduce(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                    size_t count, int type, int op, int root, void *stream);
/* rbuf receives block `rank` (rcount elements) of the element-wise
 * reduction of the size*rcount element sbufs. */
int ompi_amd_reduce_scatter_block(ompi_amd_comm_t *comm, const void *sbuf,
                                  void *rbuf, size_t rcount, int type, int op,
                                  void *stream);
/* MPI_Reduce_scatter (coll.h:242-244): rbuf receives rcounts[rank]
 * elements — this rank's block, at offset sum(rcounts[0..rank)) of the
 * element-wise reduction of the sum(rcounts)-element sbufs — in the operand
 * order of coll/tuned's decision (recursive halving or ring,
 * coll_base_reduce_scatter.c:132-623).  rcounts has `size` entries. */
int ompi_amd_reduce_scatter(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                            const size_t *rcounts, int type, int op, void *stream);
/* MPI_Scan / MPI_Exscan (coll.h:248-250, 228-230): rank r receives the
 * reduction of ranks 0..r (exscan: 0..r-1; rank 0's rbuf is untouched). */
int ompi_amd_scan(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                  size_t count, int type, int op, void *stream);
int ompi_amd_exscan(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                    size_t count, int type, int op, void *stream);
int ompi_amd_allgather(ompi_amd_comm_t *comm, const void *sbuf, void *rbuf,
                       size_t bytes_per_rank, void *stream);
int ompi_amd_bcast(ompi_amd_comm_t *comm, void *buf, size_t bytes, int root,
                   void *stream);

#ifdef __cplusplus
}
#endif
#endif /* OMPI_AMD_COLL_H */
