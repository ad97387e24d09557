// carry.h -- the consumer-side acquire carried from the p2p transport into the launches
// that read peers' bytes.  Host code; the kernels' side is
// elementwise.h wg_acquire, the launchers' side carry_acquire (copy.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace sos {

// The acquire handed from the p2p transport's backend (p2p.cpp HipBackend) to the
// launches that read a peer's bytes.  `want`: a wait saw peers' posts and no stream-wide
// acquire has run since; `peer`: the launches being made read a peer's heap.  Host code,
// one per thread (the transport runs on the PE's calling thread).
struct AcquireCarry {
    bool want = false;
    bool peer = false;
    long carried = 0;                            // launches that acquired in each workgroup
    int (*stream_wide)(hipStream_t) = nullptr;   // the acquire kernel with the runtime's
                                                 // bookkeeping (null: the bare kernel)
};
AcquireCarry &acquire_carry();  // copy.hip

// Grids up to this many workgroups carry the acquire themselves: at most one workgroup
// per CU, so each invalidate is paid once, beside the launch it saves.
constexpr unsigned kCarryMaxGrid = 256;

// A launcher calls this right before a launch that may read a peer's bytes (under
// `want && peer`): 1 = the kernel (of `grid` workgroups) must wg_acquire; 0 = nothing is
// owed, or the grid is too large (or `can` is false: a copy-engine or library copy) and
// the acquire kernel was just enqueued, which settles `want`; -1 = that launch failed.
int carry_acquire(hipStream_t st, unsigned grid, bool can = true);

}  // namespace sos
