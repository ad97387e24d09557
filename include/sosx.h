/*
 * sosx.h -- the thin C ABI between the host side of the SOS reduction path and the
 * hand-written gfx950 (MI355X) HIP kernels in libsos_amd.so.
 *
 * Plain C types only: pointers, sizes, ints.  `stream` is a hipStream_t passed as
 * void* (NULL = the library's own per-PE stream).  Every entry point returns an int
 * status (SOSX_OK or a negative SOSX_ERR_*); the shmem.h API layer turns non-zero
 * statuses into an abort, as SOS's RAISE_ERROR_MSG does (src/shmem_internal.h:124-128).
 *
 * Enum values are SOS's own, so an SOS maintainer can pass them through unchanged:
 *   op     : shm_internal_op_t        (src/transport_none.h:25-33)
 *   dtype  : shm_internal_datatype_t  (src/transport.h:19-49)
 */
#ifndef SOSX_H
#define SOSX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------- */
#define SOSX_OK                0
#define SOSX_ERR_DTYPE        (-1)  /* "invalid data type" (src/shmem_internal_op.h:335) */
#define SOSX_ERR_OP           (-2)  /* "unsupported reduction on <type>" (:245,:260,:285) */
#define SOSX_ERR_ARG          (-3)  /* bad pointer/count/team argument */
#define SOSX_ERR_HIP          (-4)  /* a HIP runtime call failed */
#define SOSX_ERR_RCCL         (-5)  /* an RCCL call failed */
#define SOSX_ERR_UNSUPPORTED  (-6)  /* valid in SOS, not available on this device path */
#define SOSX_ERR_STATE        (-7)  /* library not initialised / already initialised */

/* ---- shm_internal_op_t (src/transport_none.h:25-33) ----------------------- */
#define SOSX_OP_BAND 0
#define SOSX_OP_BOR  1
#define SOSX_OP_BXOR 2
#define SOSX_OP_MIN  3
#define SOSX_OP_MAX  4
#define SOSX_OP_SUM  5
#define SOSX_OP_PROD 6

/* ---- shm_internal_datatype_t (src/transport.h:19-49) ---------------------- */
#define SOSX_DT_SIGNED_BYTE     0
#define SOSX_DT_CHAR            1
#define SOSX_DT_SCHAR           2
#define SOSX_DT_SHORT           3
#define SOSX_DT_INT             4
#define SOSX_DT_LONG            5
#define SOSX_DT_LONG_LONG       6
#define SOSX_DT_FORTRAN_INTEGER 7
#define SOSX_DT_INT8            8
#define SOSX_DT_INT16           9
#define SOSX_DT_INT32          10
#define SOSX_DT_INT64          11
#define SOSX_DT_PTRDIFF_T      12
#define SOSX_DT_UCHAR          13
#define SOSX_DT_USHORT         14
#define SOSX_DT_UINT           15
#define SOSX_DT_ULONG          16
#define SOSX_DT_ULONG_LONG     17
#define SOSX_DT_UINT8          18
#define SOSX_DT_UINT16         19
#define SOSX_DT_UINT32         20
#define SOSX_DT_UINT64         21
#define SOSX_DT_SIZE_T         22
#define SOSX_DT_FLOAT          23
#define SOSX_DT_DOUBLE         24
#define SOSX_DT_LONG_DOUBLE    25
#define SOSX_DT_FLOAT_COMPLEX  26
#define SOSX_DT_DOUBLE_COMPLEX 27
#define SOSX_DT_COUNT          28

/* ---- fold orders (how a P-input element is combined) ----------------------- */
#define SOSX_ORDER_LINEAR 0  /* acc = in[0]; acc = acc OP in[k], k = 1..P-1 (ring fold) */
#define SOSX_ORDER_TREE   1  /* recdbl_sw butterfly tree (src/collectives.c:905-963)   */

/* ---- reduction algorithms (SHMEM_REDUCE_ALGORITHM, src/collectives.c:195-210) */
#define SOSX_ALG_AUTO       0  /* SOS AUTO without NIC atomics (src/shmem_collectives.h:180-199) */
#define SOSX_ALG_RECDBL     1  /* butterfly, full vector per step (src/collectives.c:850-984)    */
#define SOSX_ALG_RING       2  /* ring fold order (src/collectives.c:647-764), direct exchange  */
#define SOSX_ALG_RECHALVING 3  /* recursive halving + doubling, recdbl_sw tree, pairwise xGMI  */
#define SOSX_ALG_RECDBL_DIRECT 4 /* recdbl_sw tree evaluated by the owner after a direct exchange */
#define SOSX_ALG_RECDBL_GATHER 5 /* recdbl_sw, every PE's own tree, after ONE all-gather round */

/* ---- synthetic input distributions ------------------------ */
#define SOSX_DIST_UNIFORM 0  /* fp: uniform [-1,1); ints: full-range random bits      */
#define SOSX_DIST_PROD    1  /* fp: [0.5,2) (complex: +-[0.5,1) parts); ints: [-3,3]   */

/* Size in bytes of the C type behind `dtype` on x86-64/LP64, 0 if not reducible. */
size_t sosx_dtype_size(int dtype);

/* 0 if (op, dtype) is a valid reduce_local combination, else SOSX_ERR_DTYPE/OP. */
int sosx_check_op(int op, int dtype);

/*
 * inout[i] = inout[i] OP in[i], i < count, on device memory, async on `stream`.
 * Device replacement for shmem_internal_reduce_local (src/shmem_internal_op.h:305-339):
 * same op/dtype enums, same operand order (left = inout), same per-type semantics.
 * Unlike the reference, `count` is size_t (the reference's int truncates at 2^31).
 */
int sosx_combine(int op, int dtype, void *inout, const void *in, size_t count, void *stream);

/* The same combine on HOST-resident operands (SOS's symmetric heap is host memory),
 * pipelined H2D || combine || D2H in chunks of `chunk_bytes` (0 = 16 MiB pinned,
 * 64 MiB pageable) over three streams; pinned memory overlaps fully.  Synchronous.
 * The pipeline keeps 6 chunk-sized HBM slots between calls. */
int sosx_combine_host(int op, int dtype, void *inout, const void *in, size_t count,
                      size_t chunk_bytes);

/* Frees the host pipeline's HBM slots and streams (shmem_finalize calls it). */
void sosx_combine_host_release(void);

/* out[i] = a[i] OP b[i]; `out` may alias `a` (then this is sosx_combine). */
int sosx_combine3(int op, int dtype, void *out, const void *a, const void *b, size_t count,
                  void *stream);

/*
 * out[i] = fold_{k<nin}(ins[k][i]) in the given SOSX_ORDER_*; `out` may alias ins[0].
 * nin <= SOSX_MAX_FOLD.  This is the fused P-way combine used by the team schedules.
 */
#define SOSX_MAX_FOLD 64

/* Plan ids of the non-reduction team collectives (scans, broadcast) that share the
 * reduction's plan executors (sosx_loopback_allreduce, sosx_plan_encode). */
#define SOSX_PLAN_INSCAN 16
#define SOSX_PLAN_EXSCAN 17
#define SOSX_PLAN_BCAST(root, copy_root) (32 + 2 * (root) + ((copy_root) ? 1 : 0))
int sosx_fold(int op, int dtype, int order, void *out, const void *const *ins, int nin,
              size_t count, void *stream);

/*
 * Fused prefix: outs[k][i] = ins[0][i] OP ins[1][i] OP ... OP ins[k][i] (the running
 * prefix is the left operand), k < np <= 64 -- the local step of the team scans.
 * `own` (or -1) is the one input allowed to alias an output for np > 8; for np <= 8 any
 * input may alias any output.
 */
int sosx_prefix(int op, int dtype, void *const *outs, const void *const *ins, int np, int own,
                size_t count, void *stream);

/*
 * One PE's recdbl_sw value in one launch (the small host-resident path): leaf y
 * (y < p2, p2 a power of two <= SOSX_MAX_FOLD) is leaves[y][i], folded first with
 * extras[y][i] (leaves[y] the left operand) when extras/extras[y] is not null; the
 * leaves are then reduced by the recdbl_sw tree (SOSX_ORDER_TREE).  Completion is
 * signalled in memory, not by the stream: workgroup b (b < *nblocks) stores `seq` into
 * flags[b] (pinned host memory) after its results are visible system-wide; flags must
 * hold count / 256 + 8 words.  count <= SOSX_SMALL_FOLD_MAX.
 */
#define SOSX_SMALL_FOLD_MAX (1 << 20)
int sosx_small_fold(int op, int dtype, void *out, const void *const *leaves,
                    const void *const *extras, int p2, size_t count, uint32_t *flags,
                    uint32_t seq, int *nblocks, void *stream);

/*
 * Every element's SOS ring value in one launch (the small host-resident path above the
 * crossover): element i of ring chunk c (src/collectives.c:697-709) is the LINEAR fold
 * ((ins[c] OP ins[c+1]) OP ...) OP ins[c-1] of the np (2..8) team operands, the value
 * SOS's ring reduce-scatter + allgather leaves in every PE's target.  Completion words
 * as sosx_small_fold; *nblocks receives how many workgroups store one (<= count / 256
 * + np).  count <= SOSX_SMALL_FOLD_MAX.
 */
int sosx_small_ring(int op, int dtype, void *out, const void *const *ins, int np, size_t count,
                    uint32_t *flags, uint32_t seq, int *nblocks, void *stream);

/* The LINEAR fold ((ins[0] OP ins[1]) OP ...) OP ins[np-1] of np = 1..8 operands in one
 * launch: one PE's team scan value (inscan: the team's sources 0..me, exscan 0..me-1,
 * src/collectives.c:1111-1209) on the small host-resident path.  Completion words as
 * sosx_small_fold.  acquire != 0: the operands are peers' slots, and every workgroup runs
 * a system-scope acquire before its first load (as sosx_small_fold and sosx_small_ring
 * always do); 0 for local operands. */
int sosx_small_linear(int op, int dtype, void *out, const void *const *ins, int np, size_t count,
                      uint32_t *flags, uint32_t seq, int *nblocks, int acquire, void *stream);

/* Fill `count` elements of device buffer dst with the synthetic input of PE `pe`,
 * element indices [index0, index0 + count).  Bit-identical to the CPU generator
 * (tests/ and bench.py use oracle/sos_oracle.c's oracle_fill). */
int sosx_fill(int dtype, int dist, uint64_t seed, int pe, void *dst, size_t count,
              size_t index0, void *stream);

/* Bitwise comparison of two device buffers; *mismatches receives the number of
 * differing elements (elements of `elem_size` bytes).  Synchronous. */
int sosx_count_mismatch(const void *a, const void *b, size_t count, size_t elem_size,
                        unsigned long long *mismatches, void *stream);

/* Synchronous copy between any host/device addresses (hipMemcpyDefault semantics). */
int sosx_memcpy(void *dst, const void *src, size_t bytes, void *stream);

/* Multi-segment copy in one launch (peer-to-peer transport gathers). */
int sosx_gather(int nseg, const void *const *srcs, void *const *dsts, const size_t *bytes,
                void *stream);

/* p2p transport signalling (internal): store wval[i] to waddr[i] (i < nw) in stream
 * order, then wait until *qaddr[i] >= qval[i] (i < nq); a wait longer than limit_ticks
 * of the device wall clock sets *err and gives up.  Addresses are device views of
 * host-registered memory. */
int sosx_p2p_signal(int nw, uint64_t *const *waddr, const uint64_t *wval, int nq,
                    const uint64_t *const *qaddr, const uint64_t *qval, uint64_t *err,
                    long long limit_ticks, void *stream);

/* sosx_gather preceded by such a signalling step (at most 16 stores and 16 waits); a
 * small grid carries the step inside the copy launch. */
int sosx_gather_signalled(int nseg, const void *const *srcs, void *const *dsts,
                          const size_t *bytes, int nw, uint64_t *const *waddr,
                          const uint64_t *wval, int nq, const uint64_t *const *qaddr,
                          const uint64_t *qval, uint64_t *err, long long limit_ticks, void *stream);

/* The p2p transport's signalling mode: 1 = stream-ordered device signals, 0 = host
 * synchronisation every round (SHMEMX_P2P_SIGNAL=host), -1 = no p2p transport. */
int sosx_p2p_signal_mode(void);
/* Switch it between calls (1 stream, 0 host; collective: every PE at the same point of
 * its call sequence).  Returns the previous mode, or -1 when unavailable. */
int sosx_set_p2p_signal_mode(int mode);

/* RCCL executor: equal-chunk allgather rounds of world-team plans as one ncclAllGather
 * (1) or as grouped send/receive pairs (0, default; SHMEMX_RCCL_ALLGATHER sets the
 * start value).  Collective switch; returns the previous setting. */
int sosx_set_rccl_allgather(int on);

/* RCCL executor: reductions over a world-shaped team as one ncclAllReduce where RCCL has
 * the type and op.  0 = off (default; every call runs its SOS schedule), 1 = integer
 * sum/prod/min/max of 8/32/64-bit types (two's-complement results are the same in any
 * order, so bit-exact), 2 = also float/double sum/prod (RCCL's order: within the fp
 * tolerance, not bit-exact with SOS's ring).  SHMEMX_RCCL_ALLREDUCE sets the start
 * value.  Collective switch; returns the previous mode, -1 if out of range. */
int sosx_set_rccl_allreduce(int mode);

/* The rank count of the job's RCCL communicator (ncclCommCount), or -1 when the job has
 * none (p2p transport only, or a single PE).  Introspection for benchmarks. */
int sosx_rccl_comm_count(void);

/* Free this PE's private device workspaces (exchange scratch and the staging buffer of
 * host operands) once the library stream has drained; the next call that needs one
 * allocates it again.  Local (not collective).  Returns the bytes released. */
size_t sosx_release_workspaces(void);

/* System-scope completion markers issued so far: every call that returns data (and every
 * p2p post) first records an event with hipEventReleaseToSystem on the library stream, so
 * its device stores are in HBM -- visible to DMA reads, the host and peer GPUs -- when the
 * call returns.  Introspection for tests. */
long sosx_sys_releases(void);

/* The consumer half of the memory-visibility rule: a launch that
 * reads bytes a peer published (the p2p transport's gathers and in-place folds of peer
 * memory, the small path's slot reads) follows, in stream order, a system-scope acquire
 * issued after the wait for the peer's post.  *acquires: acquires issued (acquire
 * kernels, and launches that carry their own per-workgroup acquire); *peer_reads:
 * consuming launches; *unacquired: consuming launches with a peer wait since the last
 * acquire (0 unless the protocol is broken); *xcc_mask: the XCDs the acquire kernels ran
 * on (synchronises the library stream).  Any pointer may be null.  Introspection for
 * tests. */
void sosx_acquire_stats(long *acquires, long *peer_reads, long *unacquired, unsigned *xcc_mask);

/* Of those acquires, the stream-wide acquire kernels the p2p transport enqueued (the rest
 * ran in the workgroups of the small consuming launches themselves).  For tests. */
long sosx_acquire_kernels(void);

/* One acquire kernel on `stream`: 64 workgroups, each running a system-scope acquire
 * (buffer_inv sc0 sc1: this CU's L1 and its XCD's L2 drop lines other agents may have
 * rewritten) and OR-ing its XCD id into *xcc_mask (device memory, or null). */
int sosx_acquire_system(unsigned *xcc_mask, void *stream);

/* The executable's data segment [__data_start, _end) as shmem_init registered it with
 * HIP (SOS registers it with every transport, src/init.c:341-346): its page-rounded base
 * in *base (may be null) and its size; 0 when it is not registered
 * (SHMEMX_REGISTER_DATA=0, or HIP refused the range). */
size_t sosx_data_segment(void **base);

/* The p2p transport's mapping flags (introspection for tests): the hipHostRegister
 * flags of the shared pair-counter segment and the hipIpcOpenMemHandle flags of a peer's
 * device heap. */
void sosx_p2p_flags(unsigned *host_register, unsigned *ipc_open);

/* Team collectives (reductions, scans, broadcasts) that took the small path through
 * node shared memory (operands copied into shared slots, one kernel per PE reading every
 * PE's slot in place), and how many of them had a device-resident
 * operand (SHMEMX_SMALL_DEVICE).  Introspection for tests and benchmarks. */
/* The small path's staging of a device-resident operand: one workgroup copies `bytes`
 * from src (device) to dst (a node-shared slot, device view), fences at system scope and
 * then stores vals[k] into *words[k], k < nwords (release, system scope: the slot's
 * posts).  bytes <= SOSX_SMALL_FOLD_MAX, 1 <= nwords <= SOSX_MAX_FOLD. */
int sosx_small_stage(void *dst, const void *src, size_t bytes, uint64_t *const *words,
                     const uint64_t *vals, int nwords, void *stream);

long sosx_small_path_calls(void);
long sosx_small_path_device_calls(void);
/* Limit for device-resident operands on that path: a call takes it when team size *
 * operand bytes <= team_bytes (0: never; default SHMEMX_SMALL_DEVICE, 128 KiB).  Returns
 * the previous limit.  Collective in effect: every PE of a team must hold the same limit
 * when it calls, as the path choice is made on each PE. */
size_t sosx_set_small_device_bytes(size_t team_bytes);

/* Library / build identification. */
const char *sosx_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* SOSX_H */
