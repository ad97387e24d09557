// p2p.cpp -- the peer-to-peer transport: a PE's kernels read its peers' HBM directly.
//
// The device symmetric heap of every PE is IPC-mapped into every other PE (runtime.cpp,
// ensure_device_heap), so a transfer of a plan round is a PULL: the receiver reads the
// bytes the sender's plan would send, straight out of the sender's buffer.  Semantics are
// RCCL's (a receive matches the sender's next send to it, FIFO per pair), enforced by two
// monotonic counters per ordered pair in node shared memory:
//   posted[from][to]   the sender's data for its k-th send to `to` is final
//   consumed[from][to] the receiver has finished reading the sender's k-th send
// plus each PE's published heap offsets of its source/target for the current call.
//
// Per round, at PE me:
//   1. stream sync if the round sends (send buffers must hold their final bytes),
//      post every send;
//   2. for every receive: wait for the peer's post, locate the bytes from the peer's
//      own plan (built here: plans are deterministic) and its published offsets;
//   3. folds whose inputs are received chunks read them IN PLACE from peer memory
//      (no staging copy) -- allowed when the round's outputs do not overlap the
//      bytes this PE is sending in the same round; the other receives are copied by
//      one multi-segment gather launch (all peers' links at once);
//   4. stream sync, mark every receive consumed; wait until the peers consumed every
//      send of this round; run the remaining local ops.
// For the SOS ring plan this is: fold chunk `me` straight from the P-1 peers' sources
// over their xGMI links (P+1 HBM/xGMI streams, one launch), then gather the P-1 owned
// chunks -- the RCCL version's scratch round trip disappears.
#include <time.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <map>
#include <tuple>
#include <vector>

#include "plan.h"
#include "runtime.h"
#include "sosx.h"

extern "C" int sosx_prefix(int op, int dtype, void *const *outs, const void *const *ins, int np,
                           int own, size_t count, void *stream);
extern "C" int sosx_gather(int nseg, const void *const *srcs, void *const *dsts,
                           const size_t *bytes, void *stream);

namespace sosrt {

void prof_mark(int which, bool end, hipStream_t s);  // collectives.cpp (0 = fold, 1 = transfer)

namespace {

constexpr int kMaxPE = 64;

struct P2PShared {
    std::atomic<uint64_t> posted[kMaxPE][kMaxPE];
    std::atomic<uint64_t> consumed[kMaxPE][kMaxPE];
    struct Pub {
        std::atomic<uint64_t> src_off, dst_off, scr_off, mis;
    } pub[kMaxPE];
    // team creation agreement (runtime.cpp shmem_team_split_strided): per world PE, the
    // free team-slot bit mask and the creation status, read by the other members
    std::atomic<uint64_t> team_word[2][kMaxPE];
};

// What this PE has seen/done per ordered pair (monotonic across calls).
struct Local {
    uint64_t posted_by_me[kMaxPE] = {0};      // posts I made to each peer
    uint64_t seen_from[kMaxPE] = {0};         // posts from each peer I have consumed
};

Local g_local;

P2PShared *shared()
{
    return (P2PShared *)st().shm.extra;
}

// Wall-clock bound of one wait (SHMEMX_P2P_TIMEOUT seconds, default 300): a peer that
// never posts ends the job with a message instead of hanging it.
double wait_limit_s()
{
    static const double lim = [] {
        const char *e = getenv("SHMEMX_P2P_TIMEOUT");
        const double v = e ? atof(e) : 0.0;
        return v > 0 ? v : 300.0;
    }();
    return lim;
}

double now_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

void spin_until(std::atomic<uint64_t> &a, uint64_t want, const char *what)
{
    unsigned spins = 0;
    double t0 = 0;
    while (a.load(std::memory_order_acquire) < want) {
        if (++spins < 4096) {
            __builtin_ia32_pause();
            continue;
        }
        sched_yield();
        if ((spins & 1023) == 0) {
            const double t = now_s();
            if (t0 == 0) t0 = t;
            else if (t - t0 > wait_limit_s())
                raise_error("p2p transport: timed out after %.0f s waiting for %s", t - t0, what);
        }
    }
}

// SOSX_P2P_TRACE=N (diagnostics): host time per phase of p2p_exec, averaged and printed
// to stderr every N calls.
struct Trace {
    int every = -1;  // -1: not read yet, 0: off
    double t[6] = {0, 0, 0, 0, 0, 0};
    long calls = 0;
};
Trace g_trace;
enum { PH_SYNC_SEND, PH_WAIT_POST, PH_ENQUEUE, PH_SYNC_OPS, PH_WAIT_CONSUMED, PH_SYNC_END };

bool trace_on()
{
    if (g_trace.every < 0) {
        const char *e = getenv("SOSX_P2P_TRACE");
        g_trace.every = e ? atoi(e) : 0;
    }
    return g_trace.every > 0;
}

struct PeerSend {
    int buf;
    uint64_t off, bytes;
};

// The sends peer q's plan makes to `me`, in order (deterministic: rebuild q's plan from
// its published operand misalignment, which places its scratch slots).
const std::vector<PeerSend> &peer_sends(int alg, int P, int q, int me, uint64_t count,
                                        uint64_t ts, uint64_t mis)
{
    static std::map<std::tuple<int, int, int, int, uint64_t, uint64_t, uint64_t>,
                    std::vector<PeerSend>> cache;
    auto key = std::make_tuple(alg, P, q, me, count, ts, mis);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    if (cache.size() > 512) cache.clear();
    sosplan::Plan p;
    if (sosplan::build(alg, P, q, count, ts, (unsigned)(mis & 15), (unsigned)(mis >> 4), &p) != SOSX_OK)
        raise_error("p2p transport: cannot build the plan of PE %d", q);
    std::vector<PeerSend> v;
    for (const auto &r : p.rounds)
        for (const auto &x : r.xfers)
            if (x.send && x.peer == me) v.push_back(PeerSend{x.buf, x.off, x.bytes});
    return cache.emplace(key, std::move(v)).first->second;
}

bool overlaps(const char *a, uint64_t na, const char *b, uint64_t nb)
{
    return a < b + nb && b < a + na;
}

}  // namespace

size_t p2p_shared_bytes() { return sizeof(P2PShared); }

void team_word_put(int which, int world_pe, uint64_t v)
{
    shared()->team_word[which][world_pe].store(v, std::memory_order_release);
}

uint64_t team_word_get(int which, int world_pe)
{
    return shared()->team_word[which][world_pe].load(std::memory_order_acquire);
}

int p2p_exec(const sosplan::Plan &plan, const Team &t, int alg, uint64_t count, uint64_t ts,
             const P2PBufs &b, int op, int dt, hipStream_t stream)
{
    State &s = st();
    P2PShared *sh = shared();
    if (!sh) return SOSX_ERR_STATE;
    const int me = t.my_idx;
    const int my_world = t.world_rank(me);
    sh->pub[my_world].src_off.store(b.src_off, std::memory_order_relaxed);
    sh->pub[my_world].scr_off.store(b.scr_off, std::memory_order_relaxed);
    sh->pub[my_world].mis.store((uint64_t)(b.smis & 15) | (uint64_t)(b.dmis & 15) << 4,
                                std::memory_order_relaxed);
    sh->pub[my_world].dst_off.store(b.dst_off, std::memory_order_release);
    std::vector<int> recv_idx((size_t)t.size, 0);  // k-th receive from each team peer
    const bool tr = trace_on();
    double tp = tr ? now_s() : 0;
    auto phase = [&](int ph) {
        if (!tr) return;
        const double now = now_s();
        g_trace.t[ph] += now - tp;
        tp = now;
    };
    auto local_ptr = [&](int buf, uint64_t off) -> char * {
        return (buf == sosplan::SRC ? (char *)b.src : buf == sosplan::DST ? b.dst : b.scr) + off;
    };
    for (const auto &r : plan.rounds) {
        // 1. post sends
        bool any_send = false;
        for (const auto &x : r.xfers) any_send |= x.send != 0;
        if (any_send) {
            if (hipStreamSynchronize(stream) != hipSuccess) return SOSX_ERR_HIP;
            phase(PH_SYNC_SEND);
            for (const auto &x : r.xfers)
                if (x.send) {
                    const int pw = t.world_rank(x.peer);
                    sh->posted[my_world][pw].fetch_add(1, std::memory_order_release);
                    g_local.posted_by_me[pw]++;
                }
        }
        // 2. locate every receive in the sender's memory
        struct Seg { const char *src; char *dst; uint64_t bytes; int peer_world; bool used; };
        std::vector<Seg> segs;
        for (const auto &x : r.xfers) {
            if (x.send) continue;
            const int pw = t.world_rank(x.peer);
            const uint64_t want = ++g_local.seen_from[pw];
            spin_until(sh->posted[pw][my_world], want, "a peer's data");
            phase(PH_WAIT_POST);
            const uint64_t dst_off = sh->pub[pw].dst_off.load(std::memory_order_acquire);
            const auto &sends = peer_sends(alg, t.size, x.peer, me, count, ts,
                                           sh->pub[pw].mis.load(std::memory_order_relaxed));
            const int k = recv_idx[(size_t)x.peer]++;
            if (k >= (int)sends.size() || sends[(size_t)k].bytes != x.bytes)
                raise_error("p2p transport: plan mismatch with PE %d", pw);
            const PeerSend &ps = sends[(size_t)k];
            const uint64_t boff = ps.buf == sosplan::SRC ? sh->pub[pw].src_off.load(std::memory_order_relaxed)
                                : ps.buf == sosplan::DST ? dst_off
                                                         : sh->pub[pw].scr_off.load(std::memory_order_relaxed);
            const char *remote = s.peer_heap[(size_t)pw] + boff + ps.off;
            segs.push_back(Seg{remote, local_ptr(x.buf, x.off), x.bytes, pw, false});
        }
        // 3. folds/prefixes read received chunks in place when no output overlaps a send
        bool fuse_ok = true;
        for (const auto &l : r.ops) {
            const bool typed = l.kind == sosplan::FOLD || l.kind == sosplan::PREFIX;
            const uint64_t ob = typed ? l.count * ts : l.count;
            const int nout = l.kind == sosplan::PREFIX ? l.nout : 1;
            for (int k = 0; k < nout; ++k) {
                const char *o = l.kind == sosplan::PREFIX ? local_ptr(l.outs_buf[k], l.outs_off[k])
                                                          : local_ptr(l.out_buf, l.out_off);
                for (const auto &x : r.xfers)
                    if (x.send && overlaps(o, ob, local_ptr(x.buf, x.off), x.bytes)) fuse_ok = false;
            }
        }
        std::vector<std::vector<const void *>> fold_ins(r.ops.size());
        for (size_t i = 0; i < r.ops.size(); ++i) {
            const auto &l = r.ops[i];
            for (int k = 0; k < l.nin; ++k) {
                const char *p = local_ptr(l.in_buf[k], l.in_off[k]);
                if (fuse_ok && (l.kind == sosplan::FOLD || l.kind == sosplan::PREFIX))
                    for (auto &sg : segs)
                        if (sg.dst == p && sg.bytes == l.count * ts) {
                            p = sg.src;
                            sg.used = true;
                        }
                fold_ins[i].push_back(p);
            }
        }
        std::vector<const void *> gs;
        std::vector<void *> gd;
        std::vector<size_t> gb;
        for (auto &sg : segs)
            if (!sg.used) {
                gs.push_back(sg.src);
                gd.push_back(sg.dst);
                gb.push_back(sg.bytes);
            }
        if (!gs.empty()) {
            prof_mark(1, false, stream);
            int rc = sosx_gather((int)gs.size(), gs.data(), gd.data(), gb.data(), stream);
            prof_mark(1, true, stream);
            if (rc) return rc;
        }
        auto run_ops = [&]() -> int {
            for (size_t i = 0; i < r.ops.size(); ++i) {
                const auto &l = r.ops[i];
                if (l.kind == sosplan::COPY) {
                    if (fold_ins[i][0] != local_ptr(l.out_buf, l.out_off) &&
                        hipMemcpyAsync(local_ptr(l.out_buf, l.out_off), fold_ins[i][0], l.count,
                                       hipMemcpyDeviceToDevice, stream) != hipSuccess)
                        return SOSX_ERR_HIP;
                    continue;
                }
                if (l.kind == sosplan::ZERO) {
                    if (hipMemsetAsync(local_ptr(l.out_buf, l.out_off), 0, l.count, stream) != hipSuccess)
                        return SOSX_ERR_HIP;
                    continue;
                }
                if (l.kind == sosplan::PREFIX) {
                    void *outs[sosplan::PLAN_MAX_PE];
                    for (int k = 0; k < l.nout; ++k) outs[k] = local_ptr(l.outs_buf[k], l.outs_off[k]);
                    prof_mark(0, false, stream);
                    int rc = sosx_prefix(op, dt, outs, fold_ins[i].data(), l.nin, l.own, l.count, stream);
                    prof_mark(0, true, stream);
                    if (rc) return rc;
                    continue;
                }
                prof_mark(0, false, stream);
                int rc = sosx_fold(op, dt, l.order, local_ptr(l.out_buf, l.out_off),
                                   fold_ins[i].data(), l.nin, l.count, stream);
                prof_mark(0, true, stream);
                if (rc) return rc;
            }
            return SOSX_OK;
        };
        if (fuse_ok) {
            int rc = run_ops();
            if (rc) return rc;
        }
        // 4. receives done -> consumed; wait for my sends to be consumed
        phase(PH_ENQUEUE);
        if (!segs.empty() || fuse_ok) {
            if (hipStreamSynchronize(stream) != hipSuccess) return SOSX_ERR_HIP;
        }
        phase(PH_SYNC_OPS);
        for (auto &sg : segs) sh->consumed[sg.peer_world][my_world].fetch_add(1, std::memory_order_release);
        for (const auto &x : r.xfers)
            if (x.send) {
                const int pw = t.world_rank(x.peer);
                spin_until(sh->consumed[my_world][pw], g_local.posted_by_me[pw], "a peer to read");
            }
        phase(PH_WAIT_CONSUMED);
        if (!fuse_ok) {
            int rc = run_ops();
            if (rc) return rc;
        }
    }
    const hipError_t e = hipStreamSynchronize(stream);
    phase(PH_SYNC_END);
    if (tr && ++g_trace.calls % g_trace.every == 0) {  // window averages, then reset
        const double k = 1e6 / (double)g_trace.every;
        fprintf(stderr, "[%04d] p2p trace (calls %ld-%ld, us/call): sync-send %.1f wait-post %.1f "
                "enqueue %.1f sync-ops %.1f wait-consumed %.1f sync-end %.1f\n", s.my_pe,
                g_trace.calls - g_trace.every + 1, g_trace.calls, g_trace.t[0] * k, g_trace.t[1] * k,
                g_trace.t[2] * k, g_trace.t[3] * k, g_trace.t[4] * k, g_trace.t[5] * k);
        for (double &v : g_trace.t) v = 0;
    }
    return e == hipSuccess ? SOSX_OK : SOSX_ERR_HIP;
}

}  // namespace sosrt
