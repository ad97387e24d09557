// copy.hip -- multi-segment gather copy and stream-ordered signalling for the
// peer-to-peer transport.
//
// An allgather round pulls P-1 chunks, one from each peer's HBM over its own xGMI
// link.  One launch copies all segments at once (workgroups dealt across segments in
// proportion to their size), so the links work concurrently; serial per-peer copies
// would use one link at a time.  16-B nontemporal loads/stores on the 16-B congruent
// body of each segment, bytes for the ragged ends.
#include "elementwise.h"

#ifndef GATHER_U
#define GATHER_U 4
#endif

namespace sos {

constexpr int kMaxSeg = 16;

// ---------------------------------------------------------------------------------
// Stream-ordered signalling of the peer-to-peer transport (p2p.cpp): one lane per
// counter.  Lanes first store their new counter values (monotonic transfer counters in
// node shared memory, registered with HIP so the GPU reaches them), then every lane
// waits until its counter reaches its wanted value.  Because the launch sits in stream
// order, the stores happen after the kernels that produced the sent bytes and the
// waits hold back the kernels that read a peer's bytes.  Every wait is bounded by
// `limit` wall-clock ticks: on expiry the lane sets *err and returns, so the grid
// always drains (the host turns *err into an error after the stream synchronises).
// ---------------------------------------------------------------------------------
constexpr int kMaxSig = 64;

// Lane i < nw stores its counter, then lane i < nq waits for its counter (bounded).
template <int N> struct Sig {
    uint64_t *waddr[N];
    uint64_t wval[N];
    const uint64_t *qaddr[N];
    uint64_t qval[N];
    uint64_t *err;
    long long limit;
    int nw, nq;
};

// A call whose earlier step already timed out (*err set) does not wait again: each later
// step of the same call gives up at once, so a peer that died mid-call ends the call
// after ONE timeout, not one per remaining step.  The error word is re-read inside the
// spin too (another lane or workgroup of this step may have expired first).
template <int N> __device__ __forceinline__ void sig_step(const Sig<N> &a, int i)
{
    if (i < a.nw) __hip_atomic_store(a.waddr[i], a.wval[i], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (i < a.nq && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
        const long long t0 = wall_clock64();
        while (__hip_atomic_load(a.qaddr[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.qval[i]) {
            if (wall_clock64() - t0 > a.limit) {
                __hip_atomic_store(a.err, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

using SigArgs = Sig<kMaxSig>;

__global__ __launch_bounds__(kMaxSig) void k_p2p_signal(SigArgs a) { sig_step(a, threadIdx.x); }

// ---------------------------------------------------------------------------------
// The consumer half of the memory-visibility rule.  A peer's
// bytes are read after a wait that saw its post; this GPU's L2s may still hold lines of
// the same addresses from an earlier call, and a kernel dispatch does not promise to drop
// them (tools/acquire_probe.hip: a kernel queued behind a device-side wait read a whole
// rewritten buffer stale).  A system-scope acquire does (elementwise.h wg_acquire).  Small
// consuming grids carry it in each workgroup (carry_acquire below); a streaming grid
// cannot (a 1 GiB copy 6.6 -> 1.1 TB/s, profiles/r6_acquire_probe.txt), so THIS kernel
// runs once before it: 64 one-wave workgroups, dealt round-robin over the 8 XCDs, each
// fencing and recording its XCD id (the mask tests read).  The next launch on the stream
// starts after it completes.
// ---------------------------------------------------------------------------------
constexpr unsigned kAcquireBlocks = 64;

__global__ __launch_bounds__(64) void k_acquire_system(unsigned *xcc_mask)
{
    if (threadIdx.x == 0) {
        acquire_system_lane();
        if (xcc_mask) {
            unsigned id;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
            atomicOr(xcc_mask, 1u << (id & 31u));
        }
    }
}

struct GatherArgs {
    const char *src[kMaxSeg];
    char *dst[kMaxSeg];
    uint64_t head[kMaxSeg];    // bytes before the 16-B aligned body (of dst)
    unsigned sd[kMaxSeg];      // src's offset within its aligned vectors there (0: congruent)
    uint64_t nvec[kMaxSeg];    // 16-B vectors in the body
    uint64_t bytes[kMaxSeg];
    uint64_t tstart[kMaxSeg + 1];  // prefix sums of each segment's tiles
    int nseg;
    int acquire;               // each workgroup acquires before its loads (carry_acquire)
    int ul;                    // incongruent sources at 4-B offsets: unaligned loads
};

// A gather whose launch also carries the preceding p2p signalling step: every workgroup
// stores the counters (idempotent) and waits for its own view of the awaited ones
// before copying, so no workgroup depends on another being resident.  Only for grids
// of at most 16 workgroups (<= 256 KiB): waiting workgroups hold their CUs, and with
// several PEs on one GPU 256-workgroup gates starved the peers' kernels (a 4 MiB ring
// call at P = 2 took 67 us instead of 30, profiles/r2_p2p_signal_latency.txt).
constexpr int kMaxGate = 16;
constexpr unsigned kGateMaxBlocks = 16;

// One tile of kGatherU 16-B vectors per lane, one tile per workgroup (the combine's
// shape: every load of the tile issued before the first store, no grid-stride loop);
// a tile lies in one segment, so the segment lookup is uniform per workgroup.
constexpr int kGatherU = GATHER_U;
constexpr uint64_t kTileVec = (uint64_t)kThreads * kGatherU;

template <bool GATED>
__global__ __launch_bounds__(kThreads) void k_gather(GatherArgs g, Sig<kMaxGate> gate)
{
    bool acq = g.acquire != 0;
    if constexpr (GATED) {
        sig_step(gate, threadIdx.x);
        // the awaited posts published peers' bytes: this workgroup's own acquire before
        // its loads (at most kGateMaxBlocks workgroups, so the price is one invalidate each)
        acq |= gate.nq > 0;
    }
    if (acq) wg_acquire();
    const uint64_t t = blockIdx.x;
    if (t < g.tstart[g.nseg]) {
        int s = 0;
        while (t >= g.tstart[s + 1]) ++s;
        const unsigned sd = g.sd[s];
        const u32x4 *src = reinterpret_cast<const u32x4 *>(g.src[s] + g.head[s] - sd);
        u32x4 *dst = reinterpret_cast<u32x4 *>(g.dst[s] + g.head[s]);
        const uint64_t j0 = (t - g.tstart[s]) * kTileVec + threadIdx.x;
        const uint64_t nv = g.nvec[s];
        u32x4 v[kGatherU];
        if (sd == 0) {
#pragma unroll
            for (int u = 0; u < kGatherU; ++u) {
                const uint64_t j = j0 + (uint64_t)u * kThreads;
                if (j < nv) v[u] = __builtin_nontemporal_load(src + j);
            }
        } else if (g.ul && (sd & 3) == 0) {  // one unaligned 16-B load per vector
#pragma unroll
            for (int u = 0; u < kGatherU; ++u) {
                const uint64_t j = j0 + (uint64_t)u * kThreads;
                if (j < nv) v[u] = ldv_unaligned(reinterpret_cast<const char *>(src + j) + sd);
            }
        } else {  // src at another 16-B offset: aligned vectors j and j + 1, funnel-shifted
            // vector j + 1 is the next lane's vector j: taken by DPP (next_lane16), loaded
            // only by the wave's last lane -- a second nt load in every lane re-fetched the
            // lines (the fold's case, profiles/r6_realign_pmc.txt).  Lanes load vector j up
            // to j == nv: the straddled vector after the body holds bytes of the segment.
            const bool last_lane = (threadIdx.x & 63) == 63;
            u32x4 lo[kGatherU], hi[kGatherU];
#pragma unroll
            for (int u = 0; u < kGatherU; ++u) {
                const uint64_t j = j0 + (uint64_t)u * kThreads;
                if (j <= nv) lo[u] = __builtin_nontemporal_load(src + j);
            }
            if (last_lane) {
#pragma unroll
                for (int u = 0; u < kGatherU; ++u) {
                    const uint64_t j = j0 + (uint64_t)u * kThreads;
                    if (j < nv) hi[u] = __builtin_nontemporal_load(src + j + 1);
                }
            }
#pragma unroll
            for (int u = 0; u < kGatherU; ++u) {
                const uint64_t j = j0 + (uint64_t)u * kThreads;
                const u32x4 nx = next_lane16(lo[u]);
                if (!last_lane) hi[u] = nx;
                if (j < nv) v[u] = realign16(lo[u], hi[u], sd);
            }
        }
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const uint64_t j = j0 + (uint64_t)u * kThreads;
            if (j < nv) __builtin_nontemporal_store(v[u], dst + j);
        }
    }
    // ragged ends: the last workgroup copies them byte by byte
    if (blockIdx.x == gridDim.x - 1) {
        for (int t2 = 0; t2 < g.nseg; ++t2) {
            for (uint64_t b = threadIdx.x; b < g.head[t2]; b += kThreads) g.dst[t2][b] = g.src[t2][b];
            const uint64_t tail0 = g.head[t2] + g.nvec[t2] * 16;
            for (uint64_t b = tail0 + threadIdx.x; b < g.bytes[t2]; b += kThreads)
                g.dst[t2][b] = g.src[t2][b];
        }
    }
}

}  // namespace sos

using namespace sos;

namespace {

// An incongruent source at a 4-B multiple offset: one unaligned 16-B load per vector
// (2, the default), 6.20-6.24 TB/s against 6.08-6.11 for the DPP shape and 6.28 congruent
// (7 x 64 MiB, profiles/r6_gather_realign_ab.txt); other offsets keep DPP.  Bench switch
// SOSX_GATHER_REALIGN=0: DPP for every offset.
inline int gather_realign_mode()
{
    static const int m = [] {
        const char *e = getenv("SOSX_GATHER_REALIGN");
        return e && *e ? atoi(e) : 2;
    }();
    return m;
}

// A gate's signalling step as its own one-workgroup launch.
int launch_step(const Sig<kMaxGate> &gate, hipStream_t st)
{
    SigArgs a;
    memset(&a, 0, sizeof(a));
    for (int i = 0; i < gate.nw; ++i) {
        a.waddr[i] = gate.waddr[i];
        a.wval[i] = gate.wval[i];
    }
    for (int i = 0; i < gate.nq; ++i) {
        a.qaddr[i] = gate.qaddr[i];
        a.qval[i] = gate.qval[i];
    }
    a.nw = gate.nw;
    a.nq = gate.nq;
    a.err = gate.err;
    a.limit = gate.limit;
    hipLaunchKernelGGL(k_p2p_signal, dim3(1), dim3(kMaxSig), 0, st, a);
    return hip_ok(hipGetLastError());
}

// Copy nseg (src, dst, bytes) segments, <= 16 per launch.  `gate` (or null): a
// signalling step that must precede the copies.  It rides in the copy launch when the
// whole gather is ONE launch of at most kGateMaxBlocks tiles (each workgroup acquires
// after its own wait); otherwise it runs as its own k_p2p_signal launch and -- when it
// awaits posts -- the copies owe the acquire (carry_acquire: in their workgroups, or the
// acquire kernel first), so every copy launch reads the peers' bytes behind a
// system-scope acquire.  The copies' sources are peer memory
// whenever the transport asked for an acquire.
int gather_impl(int nseg, const void *const *srcs, void *const *dsts, const size_t *bytes,
                const Sig<kMaxGate> *gate, hipStream_t st)
{
    AcquireCarry &c = acquire_carry();
    const bool peer_was = c.peer;
    struct Restore {
        AcquireCarry &c;
        bool peer;
        ~Restore() { c.peer = peer; }
    } restore{c, peer_was};
    bool gate_pending = gate != nullptr;
    int live = 0;
    for (int i = 0; i < nseg; ++i) live += bytes[i] != 0;
    const bool one_launch = live <= kMaxSeg;
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
            // the body on dst's 16-B grid; an incongruent src is realigned in registers
            // (every load is a 16-B-aligned block holding at least one byte of the
            // segment, so none crosses a page the segment does not touch)
            uint64_t h = (16 - (d & 15)) & 15;
            if (h > bytes[i]) h = bytes[i];
            g.head[n] = h;
            g.nvec[n] = (bytes[i] - h) / 16;
            g.sd[n] = (unsigned)((s + h) & 15);
            g.tstart[n] = tot;
            tot += (g.nvec[n] + kTileVec - 1) / kTileVec;
            ++n;
        }
        if (!n) continue;
        g.nseg = n;
        g.tstart[n] = tot;
        g.ul = gather_realign_mode() == 2;
        const uint64_t blocks = tot ? tot : 1;  // one tile per workgroup (+ the ragged ends)
        if (blocks > 0xffffffffull) return SOSX_ERR_ARG;
        Sig<kMaxGate> none;
        memset(&none, 0, sizeof(none));
        if (gate_pending && one_launch && blocks <= kGateMaxBlocks) {
            g.acquire = carry_acquire(st, (unsigned)blocks);
            if (g.acquire < 0) return SOSX_ERR_HIP;
            hipLaunchKernelGGL(k_gather<true>, dim3((unsigned)blocks), dim3(kThreads), 0, st, g, *gate);
            if (gate->nq > 0 && !g.acquire) ++c.carried;  // acquired after the step's own wait
            gate_pending = false;
        } else {
            if (gate_pending) {  // large or several grids: the step as its own launch
                if (launch_step(*gate, st) != SOSX_OK) return SOSX_ERR_HIP;
                if (gate->nq > 0) {  // it awaited posts: the copies owe the acquire
                    c.want = true;
                    c.peer = true;
                }
                gate_pending = false;
            }
            g.acquire = carry_acquire(st, (unsigned)blocks);
            if (g.acquire < 0) return SOSX_ERR_HIP;
            hipLaunchKernelGGL(k_gather<false>, dim3((unsigned)blocks), dim3(kThreads), 0, st, g, none);
        }
        if (hipGetLastError() != hipSuccess) return SOSX_ERR_HIP;
    }
    if (gate_pending && launch_step(*gate, st) != SOSX_OK) return SOSX_ERR_HIP;  // nothing copied
    return SOSX_OK;
}

}  // namespace

namespace sos {

AcquireCarry &acquire_carry()
{
    static thread_local AcquireCarry c;
    return c;
}

int carry_acquire(hipStream_t st, unsigned grid, bool can)
{
    AcquireCarry &c = acquire_carry();
    if (!c.want || !c.peer) return 0;
    if (can && grid <= kCarryMaxGrid) {
        ++c.carried;
        return 1;
    }
    c.want = false;
    const int rc = c.stream_wide ? c.stream_wide(st) : sosx_acquire_system(nullptr, st);
    return rc == 0 ? 0 : -1;
}

}  // namespace sos

extern "C" {

// Copy nseg (src, dst, bytes) segments in one launch (<= 16 per launch; more are
// split into several launches).  src may be peer memory mapped by IPC.
int sosx_gather(int nseg, const void *const *srcs, void *const *dsts, const size_t *bytes,
                void *stream)
{
    return gather_impl(nseg, srcs, dsts, bytes, nullptr, as_stream(stream));
}

// sosx_gather preceded by a p2p signalling step (the arguments of sosx_p2p_signal, at
// most 16 stores and 16 waits): small grids carry the step in the copy launch itself.
int sosx_gather_signalled(int nseg, const void *const *srcs, void *const *dsts,
                          const size_t *bytes, int nw, uint64_t *const *waddr,
                          const uint64_t *wval, int nq, const uint64_t *const *qaddr,
                          const uint64_t *qval, uint64_t *err, long long limit_ticks, void *stream)
{
    if (nw < 0 || nq < 0 || nw > kMaxGate || nq > kMaxGate || (nq && !err)) return SOSX_ERR_ARG;
    Sig<kMaxGate> gate;
    memset(&gate, 0, sizeof(gate));
    for (int i = 0; i < nw; ++i) {
        gate.waddr[i] = waddr[i];
        gate.wval[i] = wval[i];
    }
    for (int i = 0; i < nq; ++i) {
        gate.qaddr[i] = qaddr[i];
        gate.qval[i] = qval[i];
    }
    gate.nw = nw;
    gate.nq = nq;
    gate.err = err;
    gate.limit = limit_ticks;
    return gather_impl(nseg, srcs, dsts, bytes, &gate, as_stream(stream));
}

// A system-scope acquire in stream order (k_acquire_system above); xcc_mask: a device word
// that collects the XCD ids it ran on, or null.
int sosx_acquire_system(unsigned *xcc_mask, void *stream)
{
    hipLaunchKernelGGL(k_acquire_system, dim3(kAcquireBlocks), dim3(64), 0, as_stream(stream), xcc_mask);
    return hip_ok(hipGetLastError());
}

// One signalling step of the p2p transport on `stream`: store vals[i] to waddr[i]
// (i < nw), then wait until *qaddr[i] >= qval[i] (i < nq), each wait bounded by
// `limit_ticks` of the device wall clock (expiry sets *err).  All addresses are device
// views of host-registered memory.  More than 64 entries run as several launches,
// every store launch before the first wait launch.
int sosx_p2p_signal(int nw, uint64_t *const *waddr, const uint64_t *wval, int nq,
                    const uint64_t *const *qaddr, const uint64_t *qval, uint64_t *err,
                    long long limit_ticks, void *stream)
{
    if (nw < 0 || nq < 0 || (nq && !err)) return SOSX_ERR_ARG;
    hipStream_t st = as_stream(stream);
    int w = 0, q = 0;
    while (w < nw || q < nq) {
        SigArgs a;
        memset(&a, 0, sizeof(a));
        a.err = err;
        a.limit = limit_ticks;
        while (w < nw && a.nw < kMaxSig) {
            a.waddr[a.nw] = waddr[w];
            a.wval[a.nw++] = wval[w++];
        }
        if (w == nw)  // waits only once every store has been issued
            while (q < nq && a.nq < kMaxSig) {
                a.qaddr[a.nq] = qaddr[q];
                a.qval[a.nq++] = qval[q++];
            }
        hipLaunchKernelGGL(k_p2p_signal, dim3(1), dim3(kMaxSig), 0, st, a);
        if (hipGetLastError() != hipSuccess) return SOSX_ERR_HIP;
    }
    return SOSX_OK;
}

}  // extern "C"
