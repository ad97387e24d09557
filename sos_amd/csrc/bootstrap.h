// bootstrap.h -- rank discovery, a persistent TCP hub, and a shared-memory barrier.
//
// SOS bootstraps through PMI (src/runtime-pmi.c:53-288: rank/size, KVS exchange,
// barrier).  Here: rank/size from the launcher environment, a star of TCP connections
// to PE 0 (kept open for later all-gathers such as the device heap's IPC handles), and
// a POSIX shared-memory segment for fast host barriers between PEs of one node.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace sosboot {

// Rank and size of this PE from the launcher environment; false = singleton.
bool discover(int *rank, int *size);

// Local (per-node) rank, for the GPU choice.
int local_rank(int rank);

struct Hub {
    int rank = 0, size = 1;
    bool up = false;
    std::vector<int> fds;  // PE 0: fd per PE (fds[0] unused); others: fds[0] = link to PE 0
};

// Connect every PE to PE 0 (SHMEM_BOOTSTRAP_ADDR/PORT, else MASTER_ADDR/MASTER_PORT+1).
int hub_connect(Hub *h, int rank, int size, char *err, size_t errlen);
// PE 0's `buf` (len bytes) to everyone.
int hub_bcast(Hub *h, void *buf, size_t len);
// Every PE's `rec` (len bytes) to everyone, in rank order, into `all` (size*len).
int hub_allgather(Hub *h, const void *rec, size_t len, void *all);
void hub_close(Hub *h);

// One-shot compatibility wrapper used by the probe test: connect, bcast, allgather, close.
int exchange(int rank, int size, const void *root_blob, size_t root_len, void *out_blob,
             const void *my_rec, size_t rec_len, void *all_recs, char *err, size_t errlen);

// Shared-memory barrier over any subset of the node's PEs.  Each distinct member set
// (team key) gets its own monotonically increasing arrival counters.
struct ShmBarrier {
    void *base = nullptr;
    size_t bytes = 0;
    int rank = 0;
    std::vector<std::pair<uint64_t, uint64_t>> seq;  // (key, last sequence) per team key
    void *extra = nullptr;                            // caller's region after the slots
    bool attach(const char *name, bool create, int rank, size_t extra_bytes = 0);
    void detach();
    // members: world ranks start + i*stride, i < size; returns false on timeout
    bool wait(int start, int stride, int size, double timeout_s);
};

}  // namespace sosboot
