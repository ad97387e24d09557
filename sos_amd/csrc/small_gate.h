// small_gate.h -- the device-side wait of a small-path call whose own operand is staged
// from HBM by a kernel (smallpath.cpp): instead of the host waiting for the peers' posts
// and only then launching the fold, the fold is queued right behind the staging kernel
// and its workgroups wait for the posts themselves, then read which of the peer's two
// slots each post names.  Host-visible layout; the kernels are in small.hip.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace sos {

constexpr int kGateMax = 8;  // peers whose posts one gate awaits (teams of up to 9 PEs)

struct SmallGate {
    const uint64_t *posted[kGateMax];  // device view of a peer's post count for this PE
    uint64_t want[kGateMax];           // the count this call waits for
    const uint32_t *ring[kGateMax];    // device view of the slot id that post names
    const char *base[kGateMax];        // device view of that peer's slot 0
    uint64_t slot;                     // bytes from a PE's slot 0 to its slot 1
    uint64_t *err;                     // set (system scope) when a wait expires
    long long limit;                   // device wall-clock ticks of SHMEMX_P2P_TIMEOUT
    int n;                             // entries; 0: no wait, the operands are final
    signed char op_of[16];             // kernel operand -> entry, or -1 (fold: leaves 0..7,
                                       // extras 8..15; ring / linear: inputs 0..7)
};

// sosx_small_fold / _ring / _linear (sosx.h) with a gate (null: none).  A gated call
// needs p2 <= 8 (fold) / np <= 8.
int small_fold_gated(int op, int dtype, void *out, const void *const *leaves, const void *const *extras,
                     int p2, size_t count, uint32_t *flags, uint32_t seq, int *nblocks, const SmallGate *gate,
                     void *stream);
int small_ring_gated(int op, int dtype, void *out, const void *const *ins, int np, size_t count,
                     uint32_t *flags, uint32_t seq, int *nblocks, const SmallGate *gate, void *stream);
int small_linear_gated(int op, int dtype, void *out, const void *const *ins, int np, size_t count,
                       uint32_t *flags, uint32_t seq, int *nblocks, int acquire, const SmallGate *gate,
                       void *stream);

}  // namespace sos
