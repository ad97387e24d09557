/*
 * shmemx.h -- extensions of the MI355X SOS reduction path.
 *
 *   shmemx_heap_create      SOS's external-heap hook (src/symmetric_heap_c.c:439-464,
 *                           mpp/shmemx-def.h:25-26) with a HIP device type, so a
 *                           device (HBM) region is symmetric memory the reductions
 *                           can run on without host staging.
 *   shmemx_malloc_device    collective symmetric allocation in HBM.
 *   shmemx_reduce_local     the local combine (shmem_internal_reduce_local,
 *                           src/shmem_internal_op.h:305-339) on HBM or host operands.
 *   shmemx_init_attr /      bootstrap with an RCCL unique id obtained out of band
 *   shmemx_get_unique_id    (e.g. broadcast by torch.distributed), instead of the
 *                           built-in TCP bootstrap of shmem_init().
 *   shmemx_set_stream       run the collectives on the caller's HIP stream.
 */
#ifndef SHMEMX_H
#define SHMEMX_H

#include <stddef.h>

#include "shmem.h"
#include "sosx.h"

#define SHMEMX_EXTERNAL_HEAP_ZE   0
#define SHMEMX_EXTERNAL_HEAP_CUDA 1
#define SHMEMX_EXTERNAL_HEAP_HIP  2   /* this build: HBM of the PE's MI355X */

#define SHMEMX_UNIQUE_ID_BYTES 128    /* NCCL_UNIQUE_ID_BYTES */

#ifdef __cplusplus
extern "C" {
#endif

/* the PEs of this node (src/shmem_team.c:101-164); one node per job in this build */
extern shmem_team_t SHMEMX_TEAM_NODE;

SHMEM_FUNCTION_ATTRIBUTES void shmemx_heap_create(void *base, size_t size, int device_type,
                                                  int device_index);
SHMEM_FUNCTION_ATTRIBUTES void *shmemx_malloc_device(size_t size);
SHMEM_FUNCTION_ATTRIBUTES void shmemx_free_device(void *ptr);

SHMEM_FUNCTION_ATTRIBUTES int shmemx_get_unique_id(void *uid, size_t len);
SHMEM_FUNCTION_ATTRIBUTES int shmemx_init_attr(int my_pe, int n_pes, const void *uid, size_t len);

SHMEM_FUNCTION_ATTRIBUTES void shmemx_set_stream(void *hip_stream);
SHMEM_FUNCTION_ATTRIBUTES void *shmemx_get_stream(void);
SHMEM_FUNCTION_ATTRIBUTES int shmemx_get_device(void);

/* inout[i] = inout[i] OP in[i]; op/datatype are SOS's internal enums (SOSX_OP_*,
 * SOSX_DT_*).  Either operand may be in HBM or host memory (pageable or pinned):
 * both in HBM -> one kernel; both on the host -> the H2D || combine || D2H chunk
 * pipeline; mixed -> the host operand is staged through HBM (the kernel never
 * dereferences host memory).  Completion: every path returns after the result is
 * in `inout`, as SOS's CPU loop does.  Returns SOSX_OK or a negative SOSX_ERR_*. */
SHMEM_FUNCTION_ATTRIBUTES int shmemx_reduce_local(int op, int datatype, size_t count,
                                                  const void *in, void *inout);

/* Inter-PE transport of the team reductions (SHMEMX_TRANSPORT=rccl|p2p|both at init):
 * SOSX_TRANSPORT_RCCL = ncclSend/ncclRecv over xGMI (any device buffer);
 * SOSX_TRANSPORT_P2P  = kernels read peers' HBM through the IPC-mapped device heap.
 * Returns the previous transport, or -1 if the requested one was not set up. */
#define SOSX_TRANSPORT_RCCL 0
#define SOSX_TRANSPORT_P2P  1
SHMEM_FUNCTION_ATTRIBUTES int shmemx_set_transport(int transport);

/* Reduction algorithm control, as SHMEM_REDUCE_ALGORITHM (src/collectives.c:195-210):
 * SOSX_ALG_AUTO / _RECDBL / _RING / _RECHALVING / _RECDBL_DIRECT. */
SHMEM_FUNCTION_ATTRIBUTES int shmemx_set_reduce_algorithm(int alg);

/* Single-GPU loopback team (tests/validation): run the SOS team reduction of P
 * simulated PEs whose source/target buffers all live on this device, with the same
 * per-PE plans the RCCL executor runs and device-to-device copies as the transport.
 * `alg` may also be SOSX_PLAN_INSCAN / SOSX_PLAN_EXSCAN (the team scans) or
 * SOSX_PLAN_BCAST(root, copy_root) (broadcast; op ignored, datatype sets the element
 * size). */
SHMEM_FUNCTION_ATTRIBUTES int sosx_loopback_allreduce(int alg, int P, int op, int datatype,
                                                      void *const *srcs, void *const *dsts,
                                                      size_t count, void *stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

/* ---- team prefix sums (generated: sos_amd/csrc/gen_bindings.py) ------------- */
#include "shmemx_scans.h"

#endif /* SHMEMX_H */
