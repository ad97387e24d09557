// collectives.cpp -- the SOS team reduction on MI355X: argument checks, algorithm
// dispatch, and the executors that run a per-PE plan (plan.h).
//
// shmem_internal_op_to_all (src/shmem_collectives.h:169-239) picks linear/tree
// (NIC atomics), recdbl_sw or ring.  Here there are no NIC atomics, so AUTO is SOS's
// non-atomic branch: recdbl below SHMEM_COLL_SIZE_CROSSOVER bytes, ring above; the
// GPU ring is bit-exact with SOS's (same chunks, same fold order) but moves bytes by a
// direct exchange over all xGMI links at once.
//
// Executors:
//   * RCCL: each round's transfers are ncclSend/ncclRecv (byte views) inside one
//     ncclGroupStart/End on the PE's stream, followed by the round's fused folds
//     (sosx_fold) on the same stream -- no host round trip until the call returns.
//   * loopback (sosx_loopback_allreduce): P PEs' buffers on one GPU, transfers as
//     device-to-device copies matched in the same FIFO-per-peer order RCCL uses.
// Host-resident source/target are staged through device memory (H2D, device
// reduction, D2H), as the north star's host-symmetric-heap path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <map>
#include <tuple>
#include <vector>

#include "api_internal.h"
#include "dtypes.h"
#include "plan.h"
#include "runtime.h"
#include "shmemx.h"
#include "sosx.h"

using namespace sosrt;
using sosplan::Plan;

namespace {

// ---------------------------------------------------------------------------------
// optional per-phase timing (sosx_prof_*), HIP events on the PE stream
// ---------------------------------------------------------------------------------
struct Prof {
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> fold_ev, xfer_ev;
    size_t nf = 0, nx = 0;
    double fold_ms = 0, xfer_ms = 0, call_ms = 0;
    long nfold = 0, nxfer = 0, ncall = 0;
    hipEvent_t get(std::vector<std::pair<hipEvent_t, hipEvent_t>> &v, size_t &n, bool second)
    {
        if (!second) {
            if (n == v.size()) {
                hipEvent_t a, b;
                (void)hipEventCreate(&a);
                (void)hipEventCreate(&b);
                v.push_back({a, b});
            }
            return v[n].first;
        }
        return v[n++].second;
    }
    void collect()
    {
        (void)hipStreamSynchronize(sosrt::st().stream);  // every event of the call complete
        for (size_t i = 0; i < nf; ++i) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, fold_ev[i].first, fold_ev[i].second) == hipSuccess) fold_ms += ms;
        }
        for (size_t i = 0; i < nx; ++i) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, xfer_ev[i].first, xfer_ev[i].second) == hipSuccess) xfer_ms += ms;
        }
        nfold += (long)nf;
        nxfer += (long)nx;
        nf = nx = 0;
    }
};
Prof g_prof;

}  // namespace

namespace sosrt {
// phase-timing hooks shared with the peer-to-peer executor (p2p.cpp)
void prof_mark(int which, bool end, hipStream_t s)
{
    if (!g_prof.on) return;
    auto &v = which == 0 ? g_prof.fold_ev : g_prof.xfer_ev;
    auto &n = which == 0 ? g_prof.nf : g_prof.nx;
    (void)hipEventRecord(g_prof.get(v, n, end), s);
}
}  // namespace sosrt

namespace {

struct Bufs {
    const char *src;
    char *dst;
    char *scr;
    const char *at(int b, uint64_t off) const
    {
        return (b == sosplan::SRC ? src : b == sosplan::DST ? (const char *)dst : (const char *)scr) + off;
    }
    char *wat(int b, uint64_t off) const { return (char *)at(b, off); }
};

// Run one round's local operations.
int run_locals(const sosplan::Round &r, const Bufs &b, int op, int dt, hipStream_t stream)
{
    for (const auto &l : r.ops) {
        if (l.kind == sosplan::COPY) {
            if (b.at(l.in_buf[0], l.in_off[0]) == b.at(l.out_buf, l.out_off)) continue;
            hipError_t e = hipMemcpyAsync(b.wat(l.out_buf, l.out_off), b.at(l.in_buf[0], l.in_off[0]),
                                          l.count, hipMemcpyDefault, stream);
            if (e != hipSuccess) return SOSX_ERR_HIP;
            continue;
        }
        if (l.kind == sosplan::ZERO) {
            if (hipMemsetAsync(b.wat(l.out_buf, l.out_off), 0, l.count, stream) != hipSuccess)
                return SOSX_ERR_HIP;
            continue;
        }
        const void *ins[sosplan::PLAN_MAX_PE];
        for (int k = 0; k < l.nin; ++k) ins[k] = b.at(l.in_buf[k], l.in_off[k]);
        if (g_prof.on) (void)hipEventRecord(g_prof.get(g_prof.fold_ev, g_prof.nf, false), stream);
        int rc;
        if (l.kind == sosplan::PREFIX) {
            void *outs[sosplan::PLAN_MAX_PE];
            for (int k = 0; k < l.nout; ++k) outs[k] = b.wat(l.outs_buf[k], l.outs_off[k]);
            rc = sosx_prefix(op, dt, outs, ins, l.nin, l.own, l.count, stream);
        } else {
            rc = sosx_fold(op, dt, l.order, b.wat(l.out_buf, l.out_off), ins, l.nin, l.count, stream);
        }
        if (g_prof.on) (void)hipEventRecord(g_prof.get(g_prof.fold_ev, g_prof.nf, true), stream);
        if (rc) return rc;
    }
    return SOSX_OK;
}

// Is round r, for this PE of the WORLD team, a pure allgather of equal chunks inside
// DST: one send of this PE's chunk (bytes B at off0 + me*B) to every other PE and one
// receive of PE q's chunk at off0 + q*B from every PE q, no local ops?  (The ring and
// recdbl_direct plans' second round when P divides nreduce.)  Then RCCL's own
// allgather moves exactly the bytes the send/receive pairs would.
bool allgather_round(const sosplan::Round &r, const Team &t, uint64_t *off0, uint64_t *B)
{
    const State &s = st();
    const int P = t.size, me = t.my_idx;
    if (P < 2 || t.start != 0 || t.stride != 1 || P != s.n_pes || !r.ops.empty() ||
        r.xfers.size() != 2 * (size_t)(P - 1))
        return false;
    uint64_t bytes = 0, base = 0;
    bool have = false;
    std::vector<char> sent((size_t)P, 0), got((size_t)P, 0);
    for (const auto &x : r.xfers) {
        if (x.buf != sosplan::DST || x.peer == me || x.peer < 0 || x.peer >= P) return false;
        const int owner = x.send ? me : x.peer;
        if (!have) {
            bytes = x.bytes;
            if (!bytes || x.off < (uint64_t)owner * bytes) return false;
            base = x.off - (uint64_t)owner * bytes;
            have = true;
        }
        if (x.bytes != bytes || x.off != base + (uint64_t)owner * bytes) return false;
        char &seen = (x.send ? sent : got)[(size_t)x.peer];
        if (seen) return false;
        seen = 1;
    }
    *off0 = base;
    *B = bytes;
    return true;
}

// RCCL executor: one ncclGroup per round, folds after it, all on `stream`.
int exec_rccl(const Plan &p, const Team &t, const Bufs &b, int op, int dt, hipStream_t stream)
{
    State &s = st();
    for (const auto &r : p.rounds) {
        uint64_t off0 = 0, B = 0;
        if (s.rccl_allgather && allgather_round(r, t, &off0, &B)) {
            if (g_prof.on) (void)hipEventRecord(g_prof.get(g_prof.xfer_ev, g_prof.nx, false), stream);
            char *base = b.wat(sosplan::DST, off0);
            if (ncclAllGather(base + (size_t)t.my_idx * B, base, B, ncclUint8, s.comm, stream) != ncclSuccess)
                return SOSX_ERR_RCCL;
            if (g_prof.on) (void)hipEventRecord(g_prof.get(g_prof.xfer_ev, g_prof.nx, true), stream);
            continue;
        }
        if (!r.xfers.empty()) {
            if (g_prof.on) (void)hipEventRecord(g_prof.get(g_prof.xfer_ev, g_prof.nx, false), stream);
            if (ncclGroupStart() != ncclSuccess) return SOSX_ERR_RCCL;
            for (const auto &x : r.xfers) {
                const int peer = t.world_rank(x.peer);
                ncclResult_t rc = x.send
                    ? ncclSend(b.at(x.buf, x.off), x.bytes, ncclUint8, peer, s.comm, stream)
                    : ncclRecv(b.wat(x.buf, x.off), x.bytes, ncclUint8, peer, s.comm, stream);
                if (rc != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return SOSX_ERR_RCCL;
                }
            }
            if (ncclGroupEnd() != ncclSuccess) return SOSX_ERR_RCCL;
            if (g_prof.on) (void)hipEventRecord(g_prof.get(g_prof.xfer_ev, g_prof.nx, true), stream);
        }
        int rc = run_locals(r, b, op, dt, stream);
        if (rc) return rc;
    }
    return SOSX_OK;
}

// SHMEMX_RCCL_ALLREDUCE (sosx_set_rccl_allreduce): may this reduction run as one
// ncclAllReduce?  Only over a world-shaped team (the communicator is the world's) and
// only where RCCL's type and op give the combine's own element semantics: integer
// sum/prod/min/max of 8/32/64-bit kinds (dtypes.h: char, ptrdiff_t and the unsigned
// types included) are the same in any order -- two's-complement wrap, min/max with the
// kind's signedness -- so mode 1 stays bit-exact; mode 2 adds fp32/fp64 sum/prod, whose
// bits follow RCCL's order instead of SOS's (DESIGN.md section 5 tolerance).  No RCCL
// type for 16-bit integers, no bitwise ops, no complex or long double: those keep their
// SOS schedule.
bool rccl_allreduce_type(const Team &t, int op, int dt, ncclDataType_t *ty, ncclRedOp_t *ro)
{
    const State &s = st();
    if (!s.rccl_allreduce || !s.comm || s.transport != TRANSPORT_RCCL || t.start != 0 ||
        t.stride != 1 || t.size != s.n_pes)
        return false;
    switch (op) {
        case SOSX_OP_SUM: *ro = ncclSum; break;
        case SOSX_OP_PROD: *ro = ncclProd; break;
        case SOSX_OP_MIN: *ro = ncclMin; break;
        case SOSX_OP_MAX: *ro = ncclMax; break;
        default: return false;
    }
    const bool fp_ok = s.rccl_allreduce >= 2 && (op == SOSX_OP_SUM || op == SOSX_OP_PROD);
    switch (sos_dtype_info(dt).kind) {
        case K_S8: *ty = ncclInt8; return true;
        case K_U8: *ty = ncclUint8; return true;
        case K_S32: *ty = ncclInt32; return true;
        case K_U32: *ty = ncclUint32; return true;
        case K_S64: *ty = ncclInt64; return true;
        case K_U64: *ty = ncclUint64; return true;
        case K_F32: *ty = ncclFloat32; return fp_ok;
        case K_F64: *ty = ncclFloat64; return fp_ok;
        default: return false;
    }
}

// Plan cache: the same call shape every step reuses its plan.
const Plan &cached_plan(int alg, int P, int me, uint64_t count, uint64_t ts, unsigned smis,
                        unsigned dmis)
{
    static std::map<std::tuple<int, int, int, uint64_t, uint64_t, unsigned, unsigned>, Plan> cache;
    auto key = std::make_tuple(alg, P, me, count, ts, smis, dmis);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    if (cache.size() > 64) cache.clear();
    Plan p;
    if (sosplan::build(alg, P, me, count, ts, smis, dmis, &p) != SOSX_OK)
        raise_error("internal: cannot build reduction plan (alg %d, P %d)", alg, P);
    return cache.emplace(key, std::move(p)).first->second;
}

const char *status_text(int rc)
{
    switch (rc) {
        case SOSX_ERR_DTYPE: return "invalid data type";
        case SOSX_ERR_OP: return "unsupported reduction for this data type";
        case SOSX_ERR_UNSUPPORTED: return "long double reductions are not supported on the gfx950 device path";
        case SOSX_ERR_HIP: return "HIP runtime failure";
        case SOSX_ERR_RCCL: return "RCCL failure";
        default: return "invalid argument";
    }
}

// The peer-to-peer leg of execute(): operands in the IPC-mapped heap run in place,
// others are staged through the stage region; scan scratch follows the staged operand.
void execute_p2p(const Plan &p, const Team &t, int alg, size_t count, size_t ts, const void *source,
                 void *target, const char *dsrc, char *ddst, bool direct, size_t base, int op,
                 int dt, const char *fn)
{
    State &s = st();
    const size_t bytes = count * ts;
    const char *hb = s.sym_stage;
    if (!direct && p.reads_src)
        hip_check(hipMemcpyAsync(s.sym_stage, source, bytes, hipMemcpyDefault, s.stream), "stage in");
    char *scr = nullptr;
    size_t scr_off = 0;
    if (p.scratch_bytes && p.scr_sent) {
        scr = s.sym_stage + base;
        scr_off = base;
    } else if (p.scratch_bytes) {
        scr = (char *)scratch(p.scratch_bytes);
    }
    const unsigned smis = (unsigned)((uintptr_t)dsrc & 15), dmis = (unsigned)((uintptr_t)ddst & 15);
    P2PBufs pb{dsrc, ddst, scr, (size_t)(dsrc - hb), (size_t)(ddst - hb), scr_off, smis, dmis};
    if (g_prof.on) g_prof.ncall++;
    int rc = p2p_exec(p, t, alg, count, ts, pb, op, dt, s.stream);
    if (rc) raise_error("%s: %s", fn, status_text(rc));
    // p2p_exec returned with the stream drained; a staged result still has to come out
    // (its target may be pageable memory: a full stream synchronisation)
    if (!direct && p.writes_dst) {
        hip_check(hipMemcpyAsync(target, s.sym_stage, bytes, hipMemcpyDefault, s.stream), "stage out");
        hip_check(sync_system(s.stream), fn);
    }
    if (g_prof.on) g_prof.collect();
}

// Host-resident ring reductions, pipelined in stripes.
//
// SOS's operands live in the host symmetric heap.  Staged whole, a call costs
// H2D(n*s) + exchange + D2H(n*s) in sequence.  The ring's element order depends only on
// which ring chunk an element is in (chunk c is folded starting at PE c,
// src/collectives.c:693-727), so the vector is cut into stripes that take the k-th
// slice of EVERY ring chunk: stripe k = concat over c of chunk c's elements
// [k*L, k*L + L_k).  Run as an ordinary ring over its P*L_k elements, the stripe's chunk c
// is exactly that slice of the full chunk c, owned and folded by PE c in the same order,
// so the result is bit-identical to the ring over the whole vector (tests/test_stripes.py
// checks this with the oracle).  The r = n mod P last elements of chunks c < r form a
// final stripe of r elements (one per chunk: again the ring's own split).  Stripes flow
// through three device slots:
//   H2D(k+2) on a copy stream || exchange(k) on the library stream || D2H(k-1),
// so a call approaches max(H2D, D2H) on a full-duplex PCIe link instead of their sum.
// Returns false (nothing done) when the call does not qualify.
bool striped_host_ring(int alg, void *target, const void *source, size_t count, size_t ts,
                       const Team &t, int op, int dt, const char *fn)
{
    State &s = st();
    const int P = t.size;
    if (alg != SOSX_ALG_RING || P < 2 || P > SOSX_MAX_FOLD || s.host_stripe_bytes == 0) return false;
    const size_t q = count / (size_t)P, r = count % (size_t)P;
    // Stripe shape, from measurements of this copy pattern on MI355X with HIP 7.0
    // (tools/diag/stripe_copy_probe.py, profiles/r2_stripe_probe.txt): with 2-D copies a
    // 512 MiB pass takes 0.62x the serial time at 8-16 stripes, a 64 MiB pass 0.72x even
    // with 0.5 MiB slices.  So: slices of >= SHMEMX_HOST_STRIPE_BYTES (default 256 KiB),
    // at most 16 stripes.  The p2p executor synchronises the host every round, which
    // leaves the copy streams little to overlap: it stripes only when
    // SHMEMX_HOST_STRIPE_BYTES is set explicitly (the tests use tiny stripes to exercise
    // the decomposition).
    const bool p2p = s.transport == TRANSPORT_P2P;
    if (p2p && !s.host_stripe_explicit) return false;
    size_t L = (s.host_stripe_bytes + ts - 1) / ts;
    if (!s.host_stripe_explicit) L = std::max(L, (q + 15) / 16);
    if (p2p) {  // three slots in the IPC-mapped stage region
        const size_t lim = s.sym_stage_bytes / 3 / ((size_t)P * ts);
        if (lim < L) L = lim;
    }
    if (L == 0 || q < 2 * L) return false;
    // only now the (costlier) residency queries: both operands must be host memory
    if (is_device_ptr(source) || is_device_ptr(target)) return false;
    const size_t slot_bytes = ((size_t)P * L * ts + 255) / 256 * 256;
    char *slots;
    if (p2p) {
        slots = s.sym_stage;
    } else {
        if (s.stripes_bytes < 3 * slot_bytes) {
            if (s.stripes) {
                hip_check(hipStreamSynchronize(s.stream), "hipStreamSynchronize");
                hip_check(hipFree(s.stripes), "hipFree(stripes)");
                s.stripes = nullptr;
            }
            hip_check(hipMalloc(&s.stripes, 3 * slot_bytes), "hipMalloc(stripes)");
            s.stripes_bytes = 3 * slot_bytes;
        }
        slots = (char *)s.stripes;
    }
    if (!s.pipe_h2d) {
        hip_check(hipStreamCreateWithFlags(&s.pipe_h2d, hipStreamNonBlocking), "hipStreamCreate");
        hip_check(hipStreamCreateWithFlags(&s.pipe_d2h, hipStreamNonBlocking), "hipStreamCreate");
        for (auto &slot : s.pipe_ev)
            for (hipEvent_t &e : slot)
                hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToSystem), "hipEventCreate");
    }
    enum { H2D = 0, XCH = 1, D2H = 2 };
    const size_t nfull = (q + L - 1) / L;
    const size_t nstripes = nfull + (r ? 1 : 0);
    debug_msg("%s: host-resident ring in %zu stripes of %zu x %zu elements", fn, nstripes,
              (size_t)P, L);
    auto disp = [&](size_t c) { return c * q + (c < r ? c : r); };
    // stripe k: slice length per chunk, first element of the slice within each chunk,
    // and the number of chunks it takes a slice of
    auto geom = [&](size_t k, size_t *len, size_t *first, size_t *npieces) {
        if (k < nfull) {
            *first = k * L;
            *len = q - k * L < L ? q - k * L : L;
            *npieces = (size_t)P;
        } else {
            *first = q;
            *len = 1;
            *npieces = r;
        }
    };
    const char *src = (const char *)source;
    char *dst = (char *)target;
    // The np slices of a stripe, packed in the slot at len-element spacing, sit in the
    // host vector at ring-chunk spacing: (q+1) elements for chunks c < r, q after.  So a
    // stripe moves as at most two 2-D copies (hipMemcpy2DAsync), not np 1-D ones: the
    // runtime pipelines a few large rectangular copies well and many small 1-D copies
    // badly (profiles/r2_stripe_probe.txt).
    auto copy_slices = [&](char *slot, char *host, size_t first, size_t len, size_t np,
                           bool to_dev, hipStream_t strm) {
        const size_t lo = np < r ? np : r;  // slices of the longer chunks, then the others
        const size_t groups[2][2] = {{0, lo}, {lo, np}};
        for (const auto &g : groups) {
            const size_t c0 = g[0], rows = g[1] - g[0];
            if (!rows) continue;
            const size_t hpitch = (c0 < r ? q + 1 : q) * ts;
            char *h = host + (disp(c0) + first) * ts;
            char *d = slot + c0 * len * ts;
            const hipError_t e =
                to_dev ? hipMemcpy2DAsync(d, len * ts, h, hpitch, len * ts, rows,
                                          hipMemcpyHostToDevice, strm)
                       : hipMemcpy2DAsync(h, hpitch, d, len * ts, len * ts, rows,
                                          hipMemcpyDeviceToHost, strm);
            hip_check(e, to_dev ? "stripe H2D" : "stripe D2H");
        }
    };
    auto h2d = [&](size_t k) {
        const int sl = (int)(k % 3);
        size_t len, first, np;
        geom(k, &len, &first, &np);
        char *slot = slots + (size_t)sl * slot_bytes;
        hip_check(hipStreamWaitEvent(s.pipe_h2d, s.pipe_ev[sl][D2H], 0), "stripe wait");
        copy_slices(slot, (char *)src, first, len, np, true, s.pipe_h2d);
        hip_check(hipEventRecord(s.pipe_ev[sl][H2D], s.pipe_h2d), "stripe event");
    };
    // every slot starts free: its "D2H done" event is recorded on the idle copy stream
    for (auto &slot : s.pipe_ev) hip_check(hipEventRecord(slot[D2H], s.pipe_d2h), "stripe event");
    h2d(0);
    if (nstripes > 1) h2d(1);
    if (g_prof.on) g_prof.ncall++;
    for (size_t k = 0; k < nstripes; ++k) {
        if (k + 2 < nstripes) h2d(k + 2);
        const int sl = (int)(k % 3);
        size_t len, first, np;
        geom(k, &len, &first, &np);
        const size_t m = len * np;  // elements of this stripe's ring
        char *slot = slots + (size_t)sl * slot_bytes;
        hip_check(hipStreamWaitEvent(s.stream, s.pipe_ev[sl][H2D], 0), "stripe wait");
        const unsigned mis = (unsigned)((uintptr_t)slot & 15);
        const Plan &p = cached_plan(SOSX_ALG_RING, P, t.my_idx, m, ts, mis, mis);
        char *scr = p.scratch_bytes ? (char *)scratch(p.scratch_bytes) : nullptr;
        int rc;
        if (p2p) {
            const size_t off = (size_t)(slot - s.sym_stage);
            P2PBufs pb{slot, slot, scr, off, off, 0, mis, mis};
            rc = p2p_exec(p, t, SOSX_ALG_RING, m, ts, pb, op, dt, s.stream);
        } else {
            Bufs b{slot, slot, scr};
            rc = exec_rccl(p, t, b, op, dt, s.stream);
        }
        if (rc) raise_error("%s: %s", fn, status_text(rc));
        hip_check(hipEventRecord(s.pipe_ev[sl][XCH], s.stream), "stripe event");
        hip_check(hipStreamWaitEvent(s.pipe_d2h, s.pipe_ev[sl][XCH], 0), "stripe wait");
        copy_slices(slot, dst, first, len, np, false, s.pipe_d2h);
        hip_check(hipEventRecord(s.pipe_ev[sl][D2H], s.pipe_d2h), "stripe event");
    }
    hip_check(sync_system(s.pipe_d2h), fn);
    hip_check(sync_system(s.stream), fn);
    if (g_prof.on) g_prof.collect();
    return true;
}

// Run plan `alg` (a reduction SOSX_ALG_*, a scan or a broadcast, plan.h) for this PE
// over team t, on the library stream; returns when the call is complete.  `reduction`:
// the call may take the ncclAllReduce path (rccl_allreduce_type).
void execute(int alg, void *target, const void *source, size_t count, size_t ts, const Team &t,
             int op, int dt, const char *fn, bool reduction = false)
{
    State &s = st();
    const size_t bytes = count * ts;
    int rc;
    ncclDataType_t ar_ty = ncclUint8;
    ncclRedOp_t ar_op = ncclSum;
    const bool ar = reduction && rccl_allreduce_type(t, op, dt, &ar_ty, &ar_op);
    if (!ar && striped_host_ring(alg, target, source, count, ts, t, op, dt, fn)) return;
    if (s.transport == TRANSPORT_P2P) {
        // buffers must live in the IPC-mapped device heap; anything else is staged
        // through this PE's stage region (in place), whose offset is published
        const char *hb = s.sym_stage;
        auto in_heap = [&](const void *p) {
            return hb && (const char *)p >= hb && (const char *)p + bytes <= hb + s.dev_heap_bytes;
        };
        const bool direct = in_heap(source) && in_heap(target);
        const char *dsrc = direct ? (const char *)source : s.sym_stage;
        char *ddst = direct ? (char *)target : s.sym_stage;
        const unsigned smis = (unsigned)((uintptr_t)dsrc & 15), dmis = (unsigned)((uintptr_t)ddst & 15);
        const Plan &p = cached_plan(alg, t.size, t.my_idx, count, ts, smis, dmis);
        // the staged operand and the scratch the peers read (scan results) must fit the
        // IPC-mapped stage region; the decision depends only on sizes, residency of
        // symmetric addresses and SHMEMX_STAGE_BYTES, so every PE takes the same branch
        const size_t base = direct ? 0 : (bytes + 255) / 256 * 256;
        const size_t need = (p.scratch_bytes && p.scr_sent) ? base + p.scratch_bytes : (direct ? 0 : bytes);
        if (need <= s.sym_stage_bytes) {
            execute_p2p(p, t, alg, count, ts, source, target, dsrc, ddst, direct, base, op, dt, fn);
            return;
        }
        if (!s.comm)
            raise_error("%s: %zu bytes (staged operand + exchange scratch) exceed the p2p stage "
                        "region (SHMEMX_STAGE_BYTES=%zu); allocate operands with "
                        "shmemx_malloc_device or raise SHMEMX_STAGE_BYTES", fn, need,
                        s.sym_stage_bytes);
        // both transports are up: this call runs on RCCL instead
        debug_msg("%s: %zu bytes exceed the p2p stage region, call runs on RCCL", fn, need);
    }

    // residency: device pointers run in place; host memory is staged through HBM
    const bool dev_src = is_device_ptr(source);
    const bool dev_dst = target == source ? dev_src : is_device_ptr(target);
    const char *dsrc = (const char *)source;
    char *ddst = (char *)target;
    char *stg = nullptr;
    const size_t half = (bytes + 255) / 256 * 256;
    if (!dev_src || !dev_dst) {
        stg = (char *)stage(2 * half);
        if (!dev_src) dsrc = stg;
        if (!dev_dst) ddst = target == source ? stg : stg + half;
    }
    if (ar) {
        if (!dev_src) hip_check(hipMemcpyAsync(stg, source, bytes, hipMemcpyHostToDevice, s.stream), "H2D");
        if (g_prof.on) {
            g_prof.ncall++;
            (void)hipEventRecord(g_prof.get(g_prof.xfer_ev, g_prof.nx, false), s.stream);
        }
        if (ncclAllReduce(dsrc, ddst, count, ar_ty, ar_op, s.comm, s.stream) != ncclSuccess)
            raise_error("%s: %s", fn, status_text(SOSX_ERR_RCCL));
        if (g_prof.on) (void)hipEventRecord(g_prof.get(g_prof.xfer_ev, g_prof.nx, true), s.stream);
        if (!dev_dst)
            hip_check(hipMemcpyAsync(target, ddst, bytes, hipMemcpyDeviceToHost, s.stream), "D2H");
        hip_check(sync_system(s.stream), fn);
        if (g_prof.on) g_prof.collect();
        return;
    }
    const Plan &p = cached_plan(alg, t.size, t.my_idx, count, ts, (unsigned)((uintptr_t)dsrc & 15),
                                (unsigned)((uintptr_t)ddst & 15));
    if (!dev_src && p.reads_src)
        hip_check(hipMemcpyAsync(stg, source, bytes, hipMemcpyHostToDevice, s.stream), "H2D");
    Bufs b{dsrc, ddst, p.scratch_bytes ? (char *)scratch(p.scratch_bytes) : nullptr};
    if (g_prof.on) g_prof.ncall++;
    rc = exec_rccl(p, t, b, op, dt, s.stream);
    if (rc) raise_error("%s: %s", fn, status_text(rc));
    if (!dev_dst && p.writes_dst)
        hip_check(hipMemcpyAsync(target, ddst, bytes, hipMemcpyDeviceToHost, s.stream), "D2H");
    hip_check(sync_system(s.stream), fn);
    if (g_prof.on) g_prof.collect();
}

// shmem_internal_op_to_all for this PE over team t.
void op_to_all(void *target, const void *source, size_t count, size_t ts, const Team &t, int op,
               int dt, const char *fn)
{
    State &s = st();
    if (count == 0) return;
    const size_t bytes = count * ts;
    if (t.size == 1) {
        // PE_size 1: copy (src/collectives.c:664-668), no combine, any datatype
        if (target != source)
            hip_check(hipMemcpyAsync(target, source, bytes, hipMemcpyDefault, s.stream), fn);
        hip_check(sync_system(s.stream), fn);
        return;
    }
    int rc = sos_check_op(op, dt);
    if (rc) raise_error("%s: %s (datatype %d, op %d)", fn, status_text(rc), dt, op);

    int alg = sosplan::resolve_alg(s.reduce_alg, bytes, s.coll_size_crossover);
    // the one-kernel forms fold at most SOSX_MAX_FOLD inputs: bigger teams keep the
    // same element order through the pairwise schedules (ring/recdbl_direct: recdbl_sw
    // tree by recursive halving; recdbl_gather: recdbl_sw itself)
    if ((alg == SOSX_ALG_RING || alg == SOSX_ALG_RECDBL_DIRECT) && t.size > SOSX_MAX_FOLD)
        alg = SOSX_ALG_RECHALVING;
    if (alg == SOSX_ALG_RECDBL_GATHER && sosplan::pow2_floor(t.size) > SOSX_MAX_FOLD)
        alg = SOSX_ALG_RECDBL;
    // small operands (recdbl_sw below the crossover, the ring above it; host-resident, or
    // device-resident below SHMEMX_SMALL_DEVICE): through the node shared segment, one
    // kernel reading every PE's operand in place (smallpath.cpp), no DMA copies
    if (small_path_route(alg, target, source, bytes, t, !s.rccl_allreduce, fn)) {
        small_path_reduce(alg, target, source, count, ts, t, op, dt, fn);
        return;
    }
    execute(alg, target, source, count, ts, t, op, dt, fn, true);
}

// SHMEM_ERR_CHECK_OVERLAP (src/shmem_internal.h:319-336), complete overlap allowed
void check_overlap(const void *a, const void *b, size_t bytes, const char *fn)
{
    if (a == b || bytes == 0) return;
    const char *lo = (const char *)(a < b ? a : b), *hi = (const char *)(a < b ? b : a);
    if (lo + bytes > hi)
        raise_error("%s: Argument \"dest\" [%p..%p) overlaps argument (%p)", fn, (const void *)lo,
                    (const void *)(lo + bytes), (const void *)hi);
}

void check_symmetric(const void *p, size_t bytes, const char *what, const char *fn)
{
    if (st().error_checking && bytes && !is_symmetric(p, bytes))
        raise_error("%s: argument \"%s\" (%p, %zu bytes) is not symmetric", fn, what, p, bytes);
}

// SHMEM_ERR_CHECK_ACTIVE_SET (src/shmem_internal.h:214-227) for the deprecated active-set
// forms, whose stride is 1 << logPE_stride (src/collectives_c.c4:226).  SOS shifts
// without a check (undefined for logPE_stride >= 31 or < 0) and tests the last member
// with `> num_pes`; here both are refused: logPE_stride outside [0, 30], and a set whose
// last member is not a PE.  The extent is computed in 64 bits (no int overflow).
int active_set_stride(int PE_start, int logPE_stride, int PE_size, const char *fn)
{
    const State &s = st();
    if (logPE_stride < 0 || logPE_stride > 30)
        raise_error("%s: Invalid active set (PE_start = %d, logPE_stride = %d, PE_size = %d)", fn,
                    PE_start, logPE_stride, PE_size);
    const int stride = 1 << logPE_stride;
    const long long last = (long long)PE_start + (long long)(PE_size - 1) * stride;
    if (PE_start < 0 || PE_size < 0 || last >= s.n_pes)
        raise_error("%s: Invalid active set (PE_start = %d, PE_stride = %d, PE_size = %d)", fn,
                    PE_start, stride, PE_size);
    if (!(s.my_pe >= PE_start && s.my_pe <= last && (s.my_pe - PE_start) % stride == 0))
        raise_error("%s: Calling PE (%d) is not a member of the active set", fn, s.my_pe);
    return stride;
}

// nelems * type_size for the size_t-count team forms: SOS multiplies unchecked; a count
// whose byte size does not fit size_t is refused instead of wrapping.
size_t checked_bytes(size_t nelems, size_t type_size, const char *what, const char *fn)
{
    if (type_size && nelems > SIZE_MAX / type_size)
        raise_error("%s: Argument %s (%zu) times the element size (%zu) overflows size_t", fn, what,
                    nelems, type_size);
    return nelems * type_size;
}

}  // namespace

extern "C" {

void sos_api_to_all(void *target, const void *source, int nreduce, size_t type_size,
                    int PE_start, int logPE_stride, int PE_size, void *pWrk, long *pSync, int op,
                    int datatype, const char *fn)
{
    check_initialized(fn);
    State &s = st();
    const int stride = active_set_stride(PE_start, logPE_stride, PE_size, fn);
    if (nreduce < 0)
        raise_error("%s: Argument nreduce must be greater or equal to zero (%ld)", fn, (long)nreduce);
    const size_t bytes = (size_t)nreduce * type_size;
    check_symmetric(target, bytes, "target", fn);
    check_symmetric(source, bytes, "source", fn);
    const size_t wrk = (size_t)(nreduce / 2 + 1 > SHMEM_REDUCE_MIN_WRKDATA_SIZE
                                    ? nreduce / 2 + 1 : SHMEM_REDUCE_MIN_WRKDATA_SIZE);
    check_symmetric(pWrk, type_size * wrk, "pWrk", fn);
    check_symmetric(pSync, sizeof(long) * SHMEM_REDUCE_SYNC_SIZE, "pSync", fn);
    check_overlap(target, source, bytes, fn);
    // pWrk is never touched by any SOS reduction algorithm; pSync holds
    // SHMEM_SYNC_VALUE on entry and is left so (RCCL does the synchronisation).
    Team t;
    t.start = PE_start;
    t.stride = stride;
    t.size = PE_size;
    t.my_idx = (s.my_pe - PE_start) / stride;
    t.valid = true;
    op_to_all(target, source, (size_t)nreduce, type_size, t, op, datatype, fn);
}

int sos_api_reduce(shmem_team_t team, void *dest, const void *source, size_t nreduce,
                   size_t type_size, int op, int datatype, const char *fn)
{
    check_initialized(fn);
    Team *t = team_from_handle(team);
    if (!t || !t->valid) raise_error("%s: invalid team", fn);
    const size_t bytes = checked_bytes(nreduce, type_size, "nreduce", fn);
    check_symmetric(dest, bytes, "dest", fn);
    check_symmetric(source, bytes, "source", fn);
    check_overlap(dest, source, bytes, fn);
    if (t->my_idx < 0) raise_error("%s: calling PE is not a member of the team", fn);
    op_to_all(dest, source, nreduce, type_size, *t, op, datatype, fn);
    return 0;
}

// Team-relative root check shared by the broadcasts (SHMEM_ERR_CHECK_PE, then the
// root must be a member: src/collectives.c:435 real_root = PE_start + PE_root*stride).
static void check_root(int PE_root, int size, const char *fn)
{
    if (PE_root < 0 || PE_root >= size)
        raise_error("%s: Invalid PE_root %d (team/active set of %d PEs)", fn, PE_root, size);
}

int sos_api_broadcast(shmem_team_t team, void *dest, const void *source, size_t nelems,
                      size_t type_size, int PE_root, const char *fn)
{
    check_initialized(fn);
    Team *t = team_from_handle(team);
    if (!t || !t->valid) raise_error("%s: invalid team", fn);
    const size_t bytes = checked_bytes(nelems, type_size, "nelems", fn);
    check_symmetric(dest, bytes, "dest", fn);
    check_symmetric(source, bytes, "source", fn);
    check_overlap(dest, source, bytes, fn);
    if (t->my_idx < 0) raise_error("%s: calling PE is not a member of the team", fn);
    check_root(PE_root, t->size, fn);
    if (bytes == 0) return 0;
    // the team forms copy source to dest on the root as well (collectives_c.c4:390-397)
    const int plan = sosplan::bcast_alg(PE_root, true);
    if (t->size > 1 && small_path_route(plan, dest, source, bytes, *t, true, fn)) {
        small_path_reduce(plan, dest, source, nelems, type_size, *t, SOSX_OP_SUM, SOSX_DT_UCHAR, fn);
        return 0;
    }
    execute(plan, dest, source, nelems, type_size, *t, SOSX_OP_SUM, SOSX_DT_UCHAR, fn);
    return 0;
}

static void bcast_active_set(void *target, const void *source, size_t nlong, size_t ts,
                             int PE_root, int PE_start, int logPE_stride, int PE_size, long *pSync,
                             const char *fn)
{
    check_initialized(fn);
    State &s = st();
    const int stride = active_set_stride(PE_start, logPE_stride, PE_size, fn);
    check_root(PE_root, PE_size, fn);
    const size_t bytes = checked_bytes(nlong, ts, "nlong", fn);
    check_symmetric(target, bytes, "target", fn);
    check_symmetric(source, bytes, "source", fn);
    check_symmetric(pSync, sizeof(long) * SHMEM_BCAST_SYNC_SIZE, "pSync", fn);
    check_overlap(target, source, bytes, fn);
    if (PE_size == 1 || bytes == 0) return;  // src/collectives.c:441
    Team t;
    t.start = PE_start;
    t.stride = stride;
    t.size = PE_size;
    t.my_idx = (s.my_pe - PE_start) / stride;
    t.valid = true;
    // the root's target is not written (collectives_c.c4:342-378)
    const int plan = sosplan::bcast_alg(PE_root, false);
    if (small_path_route(plan, target, source, bytes, t, true, fn)) {
        small_path_reduce(plan, target, source, nlong, ts, t, SOSX_OP_SUM, SOSX_DT_UCHAR, fn);
        return;
    }
    execute(plan, target, source, nlong, ts, t, SOSX_OP_SUM, SOSX_DT_UCHAR, fn);
}

void pshmem_broadcast32(void *target, const void *source, size_t nlong, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync)
{
    bcast_active_set(target, source, nlong, 4, PE_root, PE_start, logPE_stride, PE_size, pSync,
                     "shmem_broadcast32");
}

void pshmem_broadcast64(void *target, const void *source, size_t nlong, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync)
{
    bcast_active_set(target, source, nlong, 8, PE_root, PE_start, logPE_stride, PE_size, pSync,
                     "shmem_broadcast64");
}

int pshmem_broadcastmem(shmem_team_t team, void *dest, const void *source, size_t nelems,
                        int PE_root)
{
    return sos_api_broadcast(team, dest, source, nelems, 1, PE_root, "shmem_broadcastmem");
}

void shmem_broadcast32(void *, const void *, size_t, int, int, int, int, long *)
    __attribute__((weak, alias("pshmem_broadcast32")));
void shmem_broadcast64(void *, const void *, size_t, int, int, int, int, long *)
    __attribute__((weak, alias("pshmem_broadcast64")));
int shmem_broadcastmem(shmem_team_t, void *, const void *, size_t, int)
    __attribute__((weak, alias("pshmem_broadcastmem")));

int sos_api_scan(shmem_team_t team, void *dest, const void *source, size_t nelems,
                 size_t type_size, int op, int datatype, int exclusive, const char *fn)
{
    check_initialized(fn);
    Team *t = team_from_handle(team);
    if (!t || !t->valid) raise_error("%s: invalid team", fn);
    const size_t bytes = checked_bytes(nelems, type_size, "nelems", fn);
    check_symmetric(dest, bytes, "dest", fn);
    check_symmetric(source, bytes, "source", fn);
    check_overlap(dest, source, bytes, fn);
    if (t->my_idx < 0) raise_error("%s: calling PE is not a member of the team", fn);
    if (nelems == 0) return 0;
    int rc = sos_check_op(op, datatype);
    if (rc) raise_error("%s: %s (datatype %d, op %d)", fn, status_text(rc), datatype, op);
    if (t->size > sosplan::PLAN_MAX_PE)
        raise_error("%s: teams of more than %d PEs are not supported", fn, sosplan::PLAN_MAX_PE);
    const int plan = exclusive ? sosplan::PLAN_EXSCAN : sosplan::PLAN_INSCAN;
    if (t->size > 1 && small_path_route(plan, dest, source, bytes, *t, true, fn)) {
        // small operands: one kernel per PE over node shared memory (smallpath.cpp)
        small_path_reduce(plan, dest, source, nelems, type_size, *t, op, datatype, fn);
        return 0;
    }
    execute(plan, dest, source, nelems, type_size, *t, op, datatype, fn);
    return 0;
}

int shmemx_reduce_local(int op, int datatype, size_t count, const void *in, void *inout)
{
    check_initialized("shmemx_reduce_local");
    // One completion rule for every residency, as SOS's CPU loop: the result is in
    // `inout` when the call returns.
    int rc = sos_check_op(op, datatype);
    if (rc || count == 0) return rc;
    if (!inout || !in) return SOSX_ERR_ARG;
    const bool dev_io = is_device_ptr(inout), dev_in = is_device_ptr(in);
    // small operands, same residency: one launch, completion words (smallpath.cpp)
    if (small_local_combine(op, datatype, inout, in, count, sosx_dtype_size(datatype), dev_io, dev_in))
        return SOSX_OK;
    // both on the host (the SOS heap): H2D || combine || D2H pipeline, synchronous
    if (!dev_io && !dev_in) return sosx_combine_host(op, datatype, inout, in, count, 0);
    State &s = st();
    if (dev_io && dev_in) {
        rc = sosx_combine(op, datatype, inout, in, count, s.stream);
    } else {
        // mixed residency: the kernel never dereferences host memory; the host operand
        // is staged through HBM (and `inout` copied back when it is the host one)
        const size_t bytes = count * sosx_dtype_size(datatype);
        void *d = stage(bytes);
        if (hipMemcpyAsync(d, dev_io ? in : inout, bytes, hipMemcpyHostToDevice, s.stream) !=
            hipSuccess)
            return SOSX_ERR_HIP;
        rc = dev_io ? sosx_combine(op, datatype, inout, d, count, s.stream)
                    : sosx_combine(op, datatype, d, in, count, s.stream);
        if (!rc && !dev_io &&
            hipMemcpyAsync(inout, d, bytes, hipMemcpyDeviceToHost, s.stream) != hipSuccess)
            return SOSX_ERR_HIP;
    }
    if (rc) return rc;
    return sync_system(s.stream) == hipSuccess ? SOSX_OK : SOSX_ERR_HIP;
}

// ---- phase timing -----------------------------------------------------------------
void sosx_prof_enable(int on)
{
    g_prof.on = on != 0;
    g_prof.fold_ms = g_prof.xfer_ms = 0;
    g_prof.nfold = g_prof.nxfer = g_prof.ncall = 0;
}

void sosx_prof_get(double *fold_ms, double *xfer_ms, long *nfold, long *nxfer, long *ncall)
{
    if (fold_ms) *fold_ms = g_prof.fold_ms;
    if (xfer_ms) *xfer_ms = g_prof.xfer_ms;
    if (nfold) *nfold = g_prof.nfold;
    if (nxfer) *nxfer = g_prof.nxfer;
    if (ncall) *ncall = g_prof.ncall;
}

// ---- single-GPU loopback team -------------------------------------------------------
int sosx_loopback_allreduce(int alg, int P, int op, int datatype, void *const *srcs,
                            void *const *dsts, size_t count, void *stream)
{
    if (P < 1 || P > SOSX_MAX_FOLD || !srcs || !dsts) return SOSX_ERR_ARG;
    int rc = sosplan::is_bcast(alg) ? (sos_dtype_info(datatype).size ? SOSX_OK : SOSX_ERR_DTYPE)
                                    : sos_check_op(op, datatype);
    if (rc) return rc;
    if (sosplan::is_bcast(alg) && ((alg - sosplan::PLAN_BCAST) >> 1) >= P) return SOSX_ERR_ARG;
    const size_t ts = sos_dtype_info(datatype).size;
    hipStream_t sm = (hipStream_t)stream;
    const int a = sosplan::resolve_alg(alg, count * ts, 16384);
    std::vector<Plan> plans(P);
    std::vector<void *> scr(P, nullptr);
    for (int p = 0; p < P; ++p) {
        rc = sosplan::build(a, P, p, count, ts, (unsigned)((uintptr_t)srcs[p] & 15),
                            (unsigned)((uintptr_t)dsts[p] & 15), &plans[p]);
        if (rc) return rc;
        if (plans[p].scratch_bytes && hipMalloc(&scr[p], plans[p].scratch_bytes) != hipSuccess)
            return SOSX_ERR_HIP;
    }
    struct Send { const char *ptr; uint64_t bytes; int from; };
    std::map<std::pair<int, int>, std::deque<Send>> q;  // (from, to) FIFO, as RCCL matches
    std::vector<size_t> k(P, 0);
    std::vector<int> posted(P, 0), outstanding(P, 0);
    std::vector<std::vector<char>> recv_done(P);
    auto bufs = [&](int p) { return Bufs{(const char *)srcs[p], (char *)dsts[p], (char *)scr[p]}; };
    for (;;) {
        bool progress = false, all_done = true;
        for (int p = 0; p < P; ++p) {
            if (k[p] >= plans[p].rounds.size()) continue;
            all_done = false;
            const auto &r = plans[p].rounds[k[p]];
            const Bufs b = bufs(p);
            if (!posted[p]) {
                for (const auto &x : r.xfers)
                    if (x.send) {
                        q[{p, x.peer}].push_back(Send{b.at(x.buf, x.off), x.bytes, p});
                        outstanding[p]++;
                    }
                recv_done[p].assign(r.xfers.size(), 0);
                posted[p] = 1;
                progress = true;
            }
            bool recvs_ok = true;
            for (size_t i = 0; i < r.xfers.size(); ++i) {
                const auto &x = r.xfers[i];
                if (x.send || recv_done[p][i]) continue;
                auto &fifo = q[{x.peer, p}];
                // FIFO per (peer, me): only the oldest pending send from that peer matches
                bool earlier_pending = false;
                for (size_t j = 0; j < i; ++j)
                    if (!r.xfers[j].send && r.xfers[j].peer == x.peer && !recv_done[p][j]) earlier_pending = true;
                if (earlier_pending || fifo.empty()) {
                    recvs_ok = false;
                    continue;
                }
                Send snd = fifo.front();
                fifo.pop_front();
                if (snd.bytes != x.bytes) {
                    for (auto v : scr) if (v) (void)hipFree(v);
                    return SOSX_ERR_ARG;  // plan mismatch between PEs
                }
                if (hipMemcpyAsync(b.wat(x.buf, x.off), snd.ptr, x.bytes, hipMemcpyDeviceToDevice, sm) != hipSuccess)
                    return SOSX_ERR_HIP;
                outstanding[snd.from]--;
                recv_done[p][i] = 1;
                progress = true;
            }
            if (recvs_ok && outstanding[p] == 0) {
                rc = run_locals(r, b, op, datatype, sm);
                if (rc) return rc;
                k[p]++;
                posted[p] = 0;
                progress = true;
            }
        }
        if (all_done) break;
        if (!progress) {
            for (auto v : scr) if (v) (void)hipFree(v);
            return SOSX_ERR_ARG;  // deadlock: inconsistent plans
        }
    }
    hipError_t e = sync_system(sm);
    if (g_prof.on) {
        g_prof.ncall++;
        g_prof.collect();
    }
    for (auto v : scr)
        if (v) (void)hipFree(v);
    return e == hipSuccess ? SOSX_OK : SOSX_ERR_HIP;
}

}  // extern "C"
