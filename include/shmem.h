/*
 * shmem.h -- OpenSHMEM 1.5 API subset of the MI355X SOS reduction path.
 *
 * A drop-in for Sandia OpenSHMEM's team-reduction family
 * (shmem_<TYPE>_{and,or,xor,min,max,sum,prod}_{reduce,to_all}, mpp/shmem_c_func.h4:413-438,
 * :688-702) plus the runtime calls a program needs around it (init/finalize, PE
 * queries, symmetric allocation, barrier, teams).  Names, signatures, constants and
 * error behaviour (abort on invalid arguments) are SOS's; the implementation is
 * HIP kernels on gfx950 and RCCL over xGMI (libsos_amd.so).
 */
#ifndef SHMEM_H
#define SHMEM_H

#include <stddef.h>
#include <stdint.h>
#if !defined(__cplusplus)
#include <complex.h>
#endif

#define SHMEM_FUNCTION_ATTRIBUTES __attribute__((visibility("default")))

/* version (configure.ac:16, mpp/shmem-def.h.in:55-62) */
#define SHMEM_MAJOR_VERSION 1
#define _SHMEM_MAJOR_VERSION SHMEM_MAJOR_VERSION
#define SHMEM_MINOR_VERSION 5
#define _SHMEM_MINOR_VERSION SHMEM_MINOR_VERSION
#define SHMEM_MAX_NAME_LEN 256
#define _SHMEM_MAX_NAME_LEN SHMEM_MAX_NAME_LEN
#define SHMEM_VENDOR_STRING "Sandia OpenSHMEM (MI355X reduction path)"
#define _SHMEM_VENDOR_STRING SHMEM_VENDOR_STRING

/* work-array sizes (configure.ac:653-694 with C_LOG_MAXPES = 32, LP64) */
#define SHMEM_BCAST_SYNC_SIZE 1
#define _SHMEM_BCAST_SYNC_SIZE SHMEM_BCAST_SYNC_SIZE
#define SHMEM_REDUCE_SYNC_SIZE 35
#define _SHMEM_REDUCE_SYNC_SIZE SHMEM_REDUCE_SYNC_SIZE
#define SHMEM_BARRIER_SYNC_SIZE 16
#define _SHMEM_BARRIER_SYNC_SIZE SHMEM_BARRIER_SYNC_SIZE
#define SHMEM_COLLECT_SYNC_SIZE 18
#define _SHMEM_COLLECT_SYNC_SIZE SHMEM_COLLECT_SYNC_SIZE
#define SHMEM_ALLTOALL_SYNC_SIZE 16
#define SHMEM_ALLTOALLS_SYNC_SIZE 16
#define SHMEM_SYNC_SIZE 35
#define SHMEM_REDUCE_MIN_WRKDATA_SIZE 1
#define _SHMEM_REDUCE_MIN_WRKDATA_SIZE SHMEM_REDUCE_MIN_WRKDATA_SIZE
#define SHMEM_SYNC_VALUE 0
#define _SHMEM_SYNC_VALUE SHMEM_SYNC_VALUE

/* threading (mpp/shmem-def.h.in) */
#define SHMEM_THREAD_SINGLE     0
#define SHMEM_THREAD_FUNNELED   1
#define SHMEM_THREAD_SERIALIZED 2
#define SHMEM_THREAD_MULTIPLE   3

/* teams (mpp/shmem-def.h.in:94-96, :110): the same opaque handle type as SOS, so C++
 * code that overloads or mangles on shmem_team_t links the same way */
typedef struct shmem_impl_team_t {
    int dummy;
} * shmem_team_t;
typedef struct {
    int num_contexts;
} shmem_team_config_t;
#define SHMEM_TEAM_NUM_CONTEXTS (1L << 0)

#ifdef __cplusplus
extern "C" {
#endif

extern shmem_team_t SHMEM_TEAM_WORLD;
extern shmem_team_t SHMEM_TEAM_SHARED;
#define SHMEM_TEAM_INVALID NULL

/* ---- library setup, exit and query (src/init_c.c, src/query_c.c) ---------- */
SHMEM_FUNCTION_ATTRIBUTES void shmem_init(void);
SHMEM_FUNCTION_ATTRIBUTES int shmem_init_thread(int requested, int *provided);
SHMEM_FUNCTION_ATTRIBUTES void shmem_query_thread(int *provided);
SHMEM_FUNCTION_ATTRIBUTES void shmem_finalize(void);
SHMEM_FUNCTION_ATTRIBUTES void shmem_global_exit(int status);
SHMEM_FUNCTION_ATTRIBUTES int shmem_my_pe(void);
SHMEM_FUNCTION_ATTRIBUTES int shmem_n_pes(void);
SHMEM_FUNCTION_ATTRIBUTES int shmem_pe_accessible(int pe);
SHMEM_FUNCTION_ATTRIBUTES int shmem_addr_accessible(const void *addr, int pe);
SHMEM_FUNCTION_ATTRIBUTES void shmem_info_get_version(int *major, int *minor);
SHMEM_FUNCTION_ATTRIBUTES void shmem_info_get_name(char *name);

/* ---- symmetric memory (src/symmetric_heap_c.c) ---------------------------- */
SHMEM_FUNCTION_ATTRIBUTES void *shmem_malloc(size_t size);
SHMEM_FUNCTION_ATTRIBUTES void *shmem_calloc(size_t count, size_t size);
SHMEM_FUNCTION_ATTRIBUTES void *shmem_align(size_t alignment, size_t size);
SHMEM_FUNCTION_ATTRIBUTES void *shmem_realloc(void *ptr, size_t size);
SHMEM_FUNCTION_ATTRIBUTES void shmem_free(void *ptr);

/* ---- synchronisation ------------------------------------------------------ */
SHMEM_FUNCTION_ATTRIBUTES void shmem_barrier_all(void);
SHMEM_FUNCTION_ATTRIBUTES void shmem_sync_all(void);
SHMEM_FUNCTION_ATTRIBUTES void shmem_quiet(void);
SHMEM_FUNCTION_ATTRIBUTES void shmem_fence(void);

/* ---- teams (src/teams_c.c4) ----------------------------------------------- */
SHMEM_FUNCTION_ATTRIBUTES int shmem_team_my_pe(shmem_team_t team);
SHMEM_FUNCTION_ATTRIBUTES int shmem_team_n_pes(shmem_team_t team);
SHMEM_FUNCTION_ATTRIBUTES int shmem_team_get_config(shmem_team_t team, long config_mask,
                                                    shmem_team_config_t *config);
SHMEM_FUNCTION_ATTRIBUTES int shmem_team_translate_pe(shmem_team_t src_team, int src_pe,
                                                      shmem_team_t dest_team);
SHMEM_FUNCTION_ATTRIBUTES int shmem_team_split_strided(shmem_team_t parent_team, int PE_start,
                                                       int PE_stride, int PE_size,
                                                       const shmem_team_config_t *config,
                                                       long config_mask, shmem_team_t *new_team);
SHMEM_FUNCTION_ATTRIBUTES int shmem_team_split_2d(shmem_team_t parent_team, int xrange,
                                                  const shmem_team_config_t *xaxis_config,
                                                  long xaxis_mask, shmem_team_t *xaxis_team,
                                                  const shmem_team_config_t *yaxis_config,
                                                  long yaxis_mask, shmem_team_t *yaxis_team);
SHMEM_FUNCTION_ATTRIBUTES void shmem_team_destroy(shmem_team_t team);
SHMEM_FUNCTION_ATTRIBUTES int shmem_team_sync(shmem_team_t team);
SHMEM_FUNCTION_ATTRIBUTES void shmem_sync(int PE_start, int logPE_stride, int PE_size,
                                          long *pSync);
SHMEM_FUNCTION_ATTRIBUTES void shmem_barrier(int PE_start, int logPE_stride, int PE_size,
                                             long *pSync);

/* broadcast (src/collectives_c.c4:342-400): the active-set forms leave the root's
 * target untouched; the team form also copies source to dest on the root */
SHMEM_FUNCTION_ATTRIBUTES void shmem_broadcast32(void *target, const void *source, size_t nlong,
                                                 int PE_root, int PE_start, int logPE_stride,
                                                 int PE_size, long *pSync);
SHMEM_FUNCTION_ATTRIBUTES void shmem_broadcast64(void *target, const void *source, size_t nlong,
                                                 int PE_root, int PE_start, int logPE_stride,
                                                 int PE_size, long *pSync);
SHMEM_FUNCTION_ATTRIBUTES int shmem_broadcastmem(shmem_team_t team, void *dest, const void *source,
                                                 size_t nelems, int PE_root);
void pshmem_broadcast32(void *target, const void *source, size_t nlong, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync);
void pshmem_broadcast64(void *target, const void *source, size_t nlong, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync);
int pshmem_broadcastmem(shmem_team_t team, void *dest, const void *source, size_t nelems,
                        int PE_root);

#ifdef __cplusplus
}  /* extern "C" */
#endif

/* ---- the reduction family + typed broadcasts (generated: gen_bindings.py) --- */
#include "shmem_reductions.h"

#endif /* SHMEM_H */
