// api_internal.h -- the generic entry points behind the typed reductions, team
// broadcasts and scans (reductions_gen.cpp).
#pragma once
#include <stddef.h>

#include "shmem.h"

#ifdef __cplusplus
extern "C" {
#endif

// SHMEM_DEF_TO_ALL (src/collectives_c.c4:221-246)
void sos_api_to_all(void *target, const void *source, int nreduce, size_t type_size,
                    int PE_start, int logPE_stride, int PE_size, void *pWrk, long *pSync, int op,
                    int datatype, const char *fn);

// SHMEM_DEF_REDUCE (src/collectives_c.c4:248-269)
int sos_api_reduce(shmem_team_t team, void *dest, const void *source, size_t nreduce,
                   size_t type_size, int op, int datatype, const char *fn);

// SHMEM_DEF_BCAST (src/collectives_c.c4:402-429): team broadcast, root copies too
int sos_api_broadcast(shmem_team_t team, void *dest, const void *source, size_t nelems,
                      size_t type_size, int PE_root, const char *fn);

// SHMEM_DEF_INSCAN / SHMEM_DEF_EXSCAN (src/collectives_c.c4:294-340)
int sos_api_scan(shmem_team_t team, void *dest, const void *source, size_t nelems,
                 size_t type_size, int op, int datatype, int exclusive, const char *fn);

#ifdef __cplusplus
}
#endif
