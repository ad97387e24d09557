// bootstrap.h -- rank discovery + one-shot TCP exchange used by shmem_init().
#pragma once
#include <stddef.h>

namespace sosboot {

// Rank and size of this PE from the launcher environment; false = singleton.
bool discover(int *rank, int *size);

// Local (per-node) rank, for the GPU choice.
int local_rank(int rank);

// PE 0 broadcasts root_blob and all PEs all-gather rec_len-byte records.
int exchange(int rank, int size, const void *root_blob, size_t root_len, void *out_blob,
             const void *my_rec, size_t rec_len, void *all_recs, char *err, size_t errlen);

}  // namespace sosboot
