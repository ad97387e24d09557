// copy.hip -- multi-segment gather copy for the peer-to-peer transport.
//
// An allgather round pulls P-1 chunks, one from each peer's HBM over its own xGMI
// link.  One launch copies all segments at once (workgroups dealt across segments in
// proportion to their size), so the links work concurrently; serial per-peer copies
// would use one link at a time.  16-B nontemporal loads/stores on the 16-B congruent
// body of each segment, bytes for the ragged ends.
#include "elementwise.h"

namespace sos {

constexpr int kMaxSeg = 16;

struct GatherArgs {
    const char *src[kMaxSeg];
    char *dst[kMaxSeg];
    uint64_t head[kMaxSeg];    // bytes before the 16-B aligned body
    uint64_t nvec[kMaxSeg];    // 16-B vectors in the body
    uint64_t bytes[kMaxSeg];
    uint64_t vstart[kMaxSeg + 1];  // prefix sums of nvec
    int nseg;
};

__global__ __launch_bounds__(kThreads) void k_gather(GatherArgs g)
{
    const uint64_t total = g.vstart[g.nseg];
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    int s = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * kThreads + threadIdx.x; v < total; v += stride) {
        while (v >= g.vstart[s + 1]) ++s;
        const uint64_t j = v - g.vstart[s];
        const u32x4 *src = reinterpret_cast<const u32x4 *>(g.src[s] + g.head[s]);
        u32x4 *dst = reinterpret_cast<u32x4 *>(g.dst[s] + g.head[s]);
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + j), dst + j);
    }
    // ragged ends: the last workgroup copies them byte by byte
    if (blockIdx.x == gridDim.x - 1) {
        for (int t = 0; t < g.nseg; ++t) {
            for (uint64_t b = threadIdx.x; b < g.head[t]; b += kThreads) g.dst[t][b] = g.src[t][b];
            const uint64_t tail0 = g.head[t] + g.nvec[t] * 16;
            for (uint64_t b = tail0 + threadIdx.x; b < g.bytes[t]; b += kThreads)
                g.dst[t][b] = g.src[t][b];
        }
    }
}

}  // namespace sos

using namespace sos;

extern "C" {

// Copy nseg (src, dst, bytes) segments in one launch (<= 16 per launch; more are
// split into several launches).  src may be peer memory mapped by IPC.
int sosx_gather(int nseg, const void *const *srcs, void *const *dsts, const size_t *bytes,
                void *stream)
{
    hipStream_t st = as_stream(stream);
    for (int base = 0; base < nseg; base += kMaxSeg) {
        GatherArgs g;
        memset(&g, 0, sizeof(g));
        int n = 0;
        uint64_t tot = 0;
        for (int i = base; i < nseg && n < kMaxSeg; ++i) {
            if (!bytes[i]) continue;
            const uintptr_t s = (uintptr_t)srcs[i], d = (uintptr_t)dsts[i];
            g.src[n] = (const char *)srcs[i];
            g.dst[n] = (char *)dsts[i];
            g.bytes[n] = bytes[i];
            if (((s ^ d) & 15) == 0) {
                uint64_t h = (16 - (d & 15)) & 15;
                if (h > bytes[i]) h = bytes[i];
                g.head[n] = h;
                g.nvec[n] = (bytes[i] - h) / 16;
            } else {
                g.head[n] = bytes[i];  // incongruent: all bytes by the byte loop
                g.nvec[n] = 0;
            }
            g.vstart[n] = tot;
            tot += g.nvec[n];
            ++n;
        }
        if (!n) continue;
        g.nseg = n;
        g.vstart[n] = tot;
        uint64_t blocks = (tot + kThreads * 4 - 1) / (kThreads * 4);
        if (blocks < 1) blocks = 1;
        if (blocks > 16384) blocks = 16384;
        hipLaunchKernelGGL(k_gather, dim3((unsigned)blocks), dim3(kThreads), 0, st, g);
        if (hipGetLastError() != hipSuccess) return SOSX_ERR_HIP;
    }
    return SOSX_OK;
}

}  // extern "C"
