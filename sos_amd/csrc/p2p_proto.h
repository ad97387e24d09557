// p2p_proto.h -- the peer-to-peer transport's pairing protocol (host- and stream-signalling
// modes), written once over a backend: p2p.cpp instantiates it with the HIP stream (kernels,
// system-scope completion), tests/p2p_proto_harness.cpp with CPU threads and memcpy
// (run under ThreadSanitizer: every byte a PE reads from a peer must be ordered after the
// peer's writes by the protocol's release/acquire counters, and every overwrite after
// the peers' reads).
//
// The host-mode protocol (see p2p.cpp's header; stream mode: exec_stream below): a
// transfer is a PULL.  Per round, at PE me:
//   1. if the round sends: complete the stream (the sent bytes are final and in memory),
//      then post every send (posted[me][to]++ , release);
//   2. for every receive: wait for the peer's post (acquire), locate the bytes from the
//      peer's plan (deterministic) and its published offsets;
//   3. folds/prefixes read received chunks in place when no output of the round
//      overlaps what this PE sends in it; the other receives are gathered by one copy;
//   4. complete the stream, mark every receive consumed (consumed[from][me]++, release),
//      wait until every peer consumed this PE's sends (acquire); then the round's
//      remaining (non-fused) ops.
// The consumer half of the memory-visibility rule: every launch
// that reads a peer's bytes follows, in stream order, a system-scope acquire issued after
// the wait that saw the peer's post (be.acquire(), or the gather that carries its own
// signalling step and acquires in each of its workgroups).  Both backends check it on
// their own: they classify each wait by the counter it reads and each launch by the
// addresses it reads, and count a peer read with a wait since the last acquire as an
// error (AcquireTrack; the HIP backend's counters are sosx_acquire_stats).
// Only headers that need no HIP: plan.h (the plans) and <atomic>.
#pragma once
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <functional>
#include <map>
#include <tuple>
#include <vector>

#include "plan.h"

namespace sosp2p {

constexpr int kMaxPE = 64;
constexpr int kDescRing = 4;

// Per-call buffer offsets of a sender, as the receiver needs them to find its bytes.
struct Desc {
    uint64_t src_off, dst_off, scr_off, mis;
};

// The node-shared segment of the transport (one per job, every PE maps it).
struct Shared {
    std::atomic<uint64_t> posted[kMaxPE][kMaxPE];
    std::atomic<uint64_t> consumed[kMaxPE][kMaxPE];
    // stream mode: counters stored by the GPUs (sosx_p2p_signal), cumulative per pair
    uint64_t dposted[kMaxPE][kMaxPE];
    uint64_t dconsumed[kMaxPE][kMaxPE];
    uint64_t sig_err[kMaxPE];                  // a PE's timed-out device wait
    // stream mode: descriptor ring per ordered pair [from][to]
    Desc desc[kMaxPE][kMaxPE][kDescRing];
    std::atomic<uint64_t> desc_posted[kMaxPE][kMaxPE];
    std::atomic<uint64_t> desc_read[kMaxPE][kMaxPE];
    struct Pub {
        std::atomic<uint64_t> src_off, dst_off, scr_off, mis;
    } pub[kMaxPE];
    // team creation agreement (runtime.cpp shmem_team_split_strided): per world PE, the
    // free team-slot bit mask and the creation status, read by the other members
    std::atomic<uint64_t> team_word[2][kMaxPE];
};

// The consumer-side check, in stream (= enqueue) order: waited() when a wait for a peer's
// post completes (host) or is queued (device step); acquired() for an acquire step;
// read(own) for a launch that reads peer bytes (own: it acquires in every workgroup itself).
struct AcquireTrack {
    bool pending = false;
    long acquires = 0, reads = 0, unacquired = 0;
    void waited() { pending = true; }
    void acquired()
    {
        pending = false;
        ++acquires;
    }
    void read(bool own)
    {
        ++reads;
        if (own) ++acquires;
        else if (pending) ++unacquired;
    }
};

inline bool in_posted(const Shared *sh, const void *p)
{
    const char *a = (const char *)&sh->posted[0][0], *b = (const char *)(&sh->posted[kMaxPE - 1][kMaxPE - 1] + 1);
    return (const char *)p >= a && (const char *)p < b;
}

// dposted as seen through `base` (the host segment, or the device view of it: base is
// where the segment starts in that view)
inline bool in_dposted(const Shared *sh, const char *base, const void *p)
{
    const size_t a = (size_t)((const char *)&sh->dposted[0][0] - (const char *)sh);
    const size_t b = (size_t)((const char *)(&sh->dposted[kMaxPE - 1][kMaxPE - 1] + 1) - (const char *)sh);
    return (const char *)p >= base + a && (const char *)p < base + b;
}

// What one PE has seen/done per ordered pair (monotonic across calls).
struct Local {
    uint64_t posted_by_me[kMaxPE] = {0};      // posts I made to each peer
    uint64_t seen_from[kMaxPE] = {0};         // posts from each peer I have consumed
};

// The same for stream mode (cumulative device counters and descriptor ring indices).
struct StreamLocal {
    uint64_t posted[kMaxPE] = {0};  // my sends to each world PE (cumulative)
    uint64_t seen[kMaxPE] = {0};    // sends from each world PE I have waited for
    uint64_t desc_sent[kMaxPE] = {0}, desc_got[kMaxPE] = {0};
};

// One call's buffers at this PE: addresses, and the heap offsets the peers rebuild them from.
struct Bufs {
    const char *src;
    char *dst;
    char *scr;
    uint64_t src_off, dst_off, scr_off;
    unsigned smis, dmis;      // src/dst address mod 16 the plan was built with
};

struct PeerSend {
    int buf;
    uint64_t off, bytes;
};

// The sends peer q's plan makes to `me`, in order (deterministic: rebuild q's plan from
// its published operand misalignment, which places its scratch slots).  Empty with
// *ok = false when q's plan cannot be built.
inline const std::vector<PeerSend> &peer_sends(int alg, int P, int q, int me, uint64_t count,
                                               uint64_t ts, uint64_t mis, bool *ok)
{
    static thread_local std::map<std::tuple<int, int, int, int, uint64_t, uint64_t, uint64_t>,
                                 std::vector<PeerSend>> cache;
    *ok = true;
    auto key = std::make_tuple(alg, P, q, me, count, ts, mis);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    if (cache.size() > 512) cache.clear();
    sosplan::Plan p;
    std::vector<PeerSend> v;
    if (sosplan::build(alg, P, q, count, ts, (unsigned)(mis & 15), (unsigned)(mis >> 4), &p) != SOSX_OK) {
        *ok = false;
        static thread_local std::vector<PeerSend> none;
        return none;
    }
    for (const auto &r : p.rounds)
        for (const auto &x : r.xfers)
            if (x.send && x.peer == me) v.push_back(PeerSend{x.buf, x.off, x.bytes});
    return cache.emplace(key, std::move(v)).first->second;
}

inline bool overlaps(const char *a, uint64_t na, const char *b, uint64_t nb)
{
    return a < b + nb && b < a + na;
}

using LocalPtr = std::function<char *(int, uint64_t)>;

// Does any output of the round's ops overlap bytes this PE sends in the same round?
// If not, folds/prefixes may read received chunks in place (the peers' memory) before
// the round's sends are consumed.
inline bool round_fusable(const sosplan::Round &r, uint64_t ts, const LocalPtr &local_ptr)
{
    for (const auto &l : r.ops) {
        const bool typed = l.kind == sosplan::FOLD || l.kind == sosplan::PREFIX;
        const uint64_t ob = typed ? l.count * ts : l.count;
        const int nout = l.kind == sosplan::PREFIX ? l.nout : 1;
        for (int k = 0; k < nout; ++k) {
            const char *o = l.kind == sosplan::PREFIX ? local_ptr(l.outs_buf[k], l.outs_off[k])
                                                      : local_ptr(l.out_buf, l.out_off);
            for (const auto &x : r.xfers)
                if (x.send && overlaps(o, ob, local_ptr(x.buf, x.off), x.bytes)) return false;
        }
    }
    return true;
}

// Host-signalled executor of one plan at team index `me` of a team whose team index i is
// world PE world_of(i).  Backend B provides (all on this PE's ordered "stream"):
//   int complete()        drain the stream, stores in memory (system scope); 0 = ok
//   int drain(bool release) drain the stream (this PE's reads are done), with a
//                          system-scope release first when `release` (= complete()); 0 = ok
//   bool merge_syncs()     let a round's drain serve as the next completion point
//   int gather(n, srcs, dsts, bytes)                      one multi-segment copy
//   int run_ops(round, ins, local_ptr)                    the round's local ops
//   int acquire()          a system-scope acquire in stream order (before peer reads)
//   const char *peer_base(world_pe)                       the peer's heap, mapped here
//   void spin(std::atomic<uint64_t> &a, uint64_t want, const char *what)   bounded wait
//   void plan_mismatch(world_pe)                          fatal
//   void phase(int)                                        tracing (may be a no-op)
template <class B, class WorldOf>
int exec_host(const sosplan::Plan &plan, int P, int me, const WorldOf &world_of, int alg,
              uint64_t count, uint64_t ts, const Bufs &b, Shared *sh, Local &loc, B &be)
{
    enum { PH_SYNC_SEND, PH_WAIT_POST, PH_ENQUEUE, PH_SYNC_OPS, PH_WAIT_CONSUMED, PH_SYNC_END };
    const int my_world = world_of(me);
    sh->pub[my_world].src_off.store(b.src_off, std::memory_order_relaxed);
    sh->pub[my_world].scr_off.store(b.scr_off, std::memory_order_relaxed);
    sh->pub[my_world].mis.store((uint64_t)(b.smis & 15) | (uint64_t)(b.dmis & 15) << 4,
                                std::memory_order_relaxed);
    sh->pub[my_world].dst_off.store(b.dst_off, std::memory_order_release);
    std::vector<int> recv_idx((size_t)P, 0);  // k-th receive from each team peer
    LocalPtr local_ptr = [&](int buf, uint64_t off) -> char * {
        return (buf == sosplan::SRC ? (char *)b.src : buf == sosplan::DST ? b.dst : b.scr) + off;
    };
    // `settled`: the stream is idle and its writes released (complete()) with nothing
    // enqueued since, so the next completion point needs no second round trip.  A round
    // whose reads end its stream work completes (release + sync) where it would only
    // drain, which settles the next round's send boundary or the call's exit.
    bool settled = false;
    const bool merge = be.merge_syncs();
    for (const auto &r : plan.rounds) {
        // 1. post sends, once their bytes are final and in memory
        bool any_send = false;
        for (const auto &x : r.xfers) any_send |= x.send != 0;
        if (any_send) {
            if (!settled && be.complete() != 0) return SOSX_ERR_HIP;
            settled = true;
            be.phase(PH_SYNC_SEND);
            for (const auto &x : r.xfers)
                if (x.send) {
                    const int pw = world_of(x.peer);
                    sh->posted[my_world][pw].fetch_add(1, std::memory_order_release);
                    loc.posted_by_me[pw]++;
                }
        }
        // 2. locate every receive in the sender's memory
        struct Seg { const char *src; char *dst; uint64_t bytes; int peer_world; bool used; };
        std::vector<Seg> segs;
        for (const auto &x : r.xfers) {
            if (x.send) continue;
            const int pw = world_of(x.peer);
            const uint64_t want = ++loc.seen_from[pw];
            be.spin(sh->posted[pw][my_world], want, "a peer's data");
            be.phase(PH_WAIT_POST);
            const uint64_t dst_off = sh->pub[pw].dst_off.load(std::memory_order_acquire);
            bool ok;
            const auto &sends = peer_sends(alg, P, x.peer, me, count, ts,
                                           sh->pub[pw].mis.load(std::memory_order_relaxed), &ok);
            const int k = recv_idx[(size_t)x.peer]++;
            if (!ok || k >= (int)sends.size() || sends[(size_t)k].bytes != x.bytes) be.plan_mismatch(pw);
            const PeerSend &ps = sends[(size_t)k];
            const uint64_t boff = ps.buf == sosplan::SRC ? sh->pub[pw].src_off.load(std::memory_order_relaxed)
                                : ps.buf == sosplan::DST ? dst_off
                                                         : sh->pub[pw].scr_off.load(std::memory_order_relaxed);
            segs.push_back(Seg{be.peer_base(pw) + boff + ps.off, local_ptr(x.buf, x.off), x.bytes, pw, false});
        }
        // 3. folds/prefixes read received chunks in place when no output overlaps a send
        const bool fuse_ok = round_fusable(r, ts, local_ptr);
        std::vector<std::vector<const void *>> ins(r.ops.size());
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
                ins[i].push_back(p);
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
        // the peers' posts were seen: acquire before the first launch that reads their bytes
        if (!segs.empty() && be.acquire() != 0) return SOSX_ERR_HIP;
        if (!gs.empty()) {
            const int rc = be.gather((int)gs.size(), gs.data(), gd.data(), gb.data());
            if (rc) return rc;
            settled = false;
        }
        if (fuse_ok) {
            const int rc = be.run_ops(r, ins, local_ptr);
            if (rc) return rc;
            settled = false;
        }
        // 4. receives done -> consumed; wait for my sends to be consumed.  With the
        //    round's ops already queued (fuse_ok) nothing follows on the stream: complete
        //    instead of draining (one round trip serves the next boundary too)
        be.phase(PH_ENQUEUE);
        if ((!segs.empty() || fuse_ok) && !settled) {
            if (be.drain(merge && fuse_ok) != 0) return SOSX_ERR_HIP;
            settled = merge && fuse_ok;
        }
        be.phase(PH_SYNC_OPS);
        for (auto &sg : segs) sh->consumed[sg.peer_world][my_world].fetch_add(1, std::memory_order_release);
        for (const auto &x : r.xfers)
            if (x.send) {
                const int pw = world_of(x.peer);
                be.spin(sh->consumed[my_world][pw], loc.posted_by_me[pw], "a peer to read");
            }
        be.phase(PH_WAIT_CONSUMED);
        if (!fuse_ok) {
            const int rc = be.run_ops(r, ins, local_ptr);
            if (rc) return rc;
            settled = false;
        }
    }
    const int e = settled ? 0 : be.complete();  // the caller's result in memory
    be.phase(PH_SYNC_END);
    return e == 0 ? SOSX_OK : SOSX_ERR_HIP;
}

// Stream-signalled executor (stream mode, p2p.cpp's header): the whole call is enqueued
// at once.  The call's offsets travel ahead through a descriptor ring per ordered pair
// (host handshake, never waiting on a GPU); between rounds the pair counters move in
// stream order (a signal step: stores, then bounded waits), carried by a small gather's
// own launch when it can; the call's exit boundary runs on the host, its entry boundary
// on the host or (host_entry() false) as the first queued step.
// Backend B adds to exec_host's:
//   int release()                     a system-scope release in stream order
//   int signal(nw, waddr, wval, nq, qaddr, qval)              one queued step
//   int gather_signalled(n, srcs, dsts, bytes, nw, waddr, wval, nq, qaddr, qval)
//   uint64_t *dev(uint64_t *), const uint64_t *dev(const uint64_t *)   the step's view
//   void spin_u64(const uint64_t *a, uint64_t want, const char *what)  host wait
//   void entry_hook()                 after the entry boundary (test hook)
//   bool host_entry()                 entry boundary on the host (else queued)
//   bool device_wait_failed()         a queued wait timed out (after complete())
template <class B, class WorldOf>
int exec_stream(const sosplan::Plan &plan, int P, int me, const WorldOf &world_of, int alg,
                uint64_t count, uint64_t ts, const Bufs &b, Shared *sh, StreamLocal &sl, B &be)
{
    enum { PH_WAIT_POST = 1, PH_ENQUEUE = 2, PH_SYNC_END = 5 };
    const int my_world = world_of(me);
    LocalPtr local_ptr = [&](int buf, uint64_t off) -> char * {
        return (buf == sosplan::SRC ? (char *)b.src : buf == sosplan::DST ? b.dst : b.scr) + off;
    };
    // 1. descriptors: publish this call's offsets to every PE this call sends to, then
    //    read those of every PE it receives from
    std::vector<char> sends_to((size_t)P, 0), recvs_from((size_t)P, 0);
    for (const auto &r : plan.rounds)
        for (const auto &x : r.xfers) (x.send ? sends_to : recvs_from)[(size_t)x.peer] = 1;
    const Desc mine{b.src_off, b.dst_off, b.scr_off,
                    (uint64_t)(b.smis & 15) | (uint64_t)(b.dmis & 15) << 4};
    for (int q = 0; q < P; ++q) {
        if (!sends_to[(size_t)q]) continue;
        const int pw = world_of(q);
        const uint64_t idx = sl.desc_sent[pw]++;
        if (idx >= (uint64_t)kDescRing)
            be.spin(sh->desc_read[my_world][pw], idx + 1 - kDescRing, "a peer to take a descriptor");
        sh->desc[my_world][pw][idx % kDescRing] = mine;
        sh->desc_posted[my_world][pw].store(idx + 1, std::memory_order_release);
    }
    std::vector<Desc> peer_desc((size_t)P);
    for (int q = 0; q < P; ++q) {
        if (!recvs_from[(size_t)q]) continue;
        const int pw = world_of(q);
        const uint64_t idx = sl.desc_got[pw]++;
        be.spin(sh->desc_posted[pw][my_world], idx + 1, "a peer's call descriptor");
        peer_desc[(size_t)q] = sh->desc[pw][my_world][idx % kDescRing];
        sh->desc_read[pw][my_world].store(idx + 1, std::memory_order_release);
    }
    be.phase(PH_WAIT_POST);
    // pending signalling step: stores first, then waits (merged across a round boundary
    // when no local op sits between them)
    std::map<uint64_t *, uint64_t> pw_store;
    std::map<const uint64_t *, uint64_t> pw_wait;
    bool data_wait = false;  // pw_wait holds a wait for a peer's post (not only consumed marks)
    auto take = [&](std::vector<uint64_t *> &wa, std::vector<uint64_t> &wv,
                    std::vector<const uint64_t *> &qa, std::vector<uint64_t> &qv) {
        data_wait = false;
        for (auto &kv : pw_store) {
            wa.push_back(be.dev(kv.first));
            wv.push_back(kv.second);
        }
        for (auto &kv : pw_wait) {
            qa.push_back(be.dev(kv.first));
            qv.push_back(kv.second);
        }
        pw_store.clear();
        pw_wait.clear();
    };
    auto flush = [&]() -> int {
        if (pw_store.empty() && pw_wait.empty()) return SOSX_OK;
        // posts make the bytes of this round's sends readable by peers, on other GPUs
        // over xGMI: a system-scope release in stream order first
        if (!pw_store.empty() && be.release() != 0) return SOSX_ERR_HIP;
        const bool acq = data_wait;
        std::vector<uint64_t *> wa;
        std::vector<uint64_t> wv;
        std::vector<const uint64_t *> qa;
        std::vector<uint64_t> qv;
        take(wa, wv, qa, qv);
        const int rc = be.signal((int)wa.size(), wa.data(), wv.data(), (int)qa.size(), qa.data(), qv.data());
        if (rc) return rc;
        // the step awaited peers' posts: the acquire before anything reads their bytes
        return acq && be.acquire() != 0 ? SOSX_ERR_HIP : SOSX_OK;
    };
    // the same step done by the host (the call's first and last boundaries)
    auto host_flush = [&]() {
        for (auto &kv : pw_store) __atomic_store_n(kv.first, kv.second, __ATOMIC_RELEASE);
        for (auto &kv : pw_wait) be.spin_u64(kv.first, kv.second, "a peer (call boundary)");
        pw_store.clear();
        pw_wait.clear();
        data_wait = false;
    };
    std::vector<int> recv_idx((size_t)P, 0);  // k-th receive from each team peer
    bool first_xfer_round = true;
    for (const auto &r : plan.rounds) {
        if (r.xfers.empty()) {
            int rc = flush();
            if (rc) return rc;
            std::vector<std::vector<const void *>> ins(r.ops.size());
            for (size_t i = 0; i < r.ops.size(); ++i)
                for (int k = 0; k < r.ops[i].nin; ++k)
                    ins[i].push_back(local_ptr(r.ops[i].in_buf[k], r.ops[i].in_off[k]));
            rc = be.run_ops(r, ins, local_ptr);
            if (rc) return rc;
            continue;
        }
        // post this round's sends (their bytes are final in stream order), wait for the
        // peers' posts of what this round receives
        for (const auto &x : r.xfers) {
            const int pw = world_of(x.peer);
            if (x.send) {
                pw_store[&sh->dposted[my_world][pw]] = ++sl.posted[pw];
            } else {
                pw_wait[&sh->dposted[pw][my_world]] = ++sl.seen[pw];
                data_wait = true;
            }
        }
        int rc;
        bool step_pending = false;  // the signalling step still to be enqueued
        if (first_xfer_round && !be.host_entry()) {
            // device entry: the first round's posts and waits are a signalling step in
            // stream order like every later round's (a system-scope release ahead of the
            // posts), so the call waits for the GPU once, at its end
            first_xfer_round = false;
            be.entry_hook();
            step_pending = true;
        } else if (first_xfer_round) {
            // host entry: the boundary runs on the host (complete only when this round
            // sends), then the host posts and waits
            first_xfer_round = false;
            bool sends = false;
            for (const auto &x : r.xfers) sends |= x.send != 0;
            if (sends && be.complete() != 0) return SOSX_ERR_HIP;
            const bool acq = data_wait;
            host_flush();
            if (acq && be.acquire() != 0) return SOSX_ERR_HIP;
            be.entry_hook();
        } else {
            step_pending = true;
        }
        struct Seg { const char *src; char *dst; uint64_t bytes; bool used; };
        std::vector<Seg> segs;
        for (const auto &x : r.xfers) {
            if (x.send) continue;
            const int pw = world_of(x.peer);
            const Desc &d = peer_desc[(size_t)x.peer];
            bool ok;
            const auto &sends = peer_sends(alg, P, x.peer, me, count, ts, d.mis, &ok);
            const int k = recv_idx[(size_t)x.peer]++;
            if (!ok || k >= (int)sends.size() || sends[(size_t)k].bytes != x.bytes) be.plan_mismatch(pw);
            const PeerSend &ps = sends[(size_t)k];
            const uint64_t boff = ps.buf == sosplan::SRC ? d.src_off
                                : ps.buf == sosplan::DST ? d.dst_off : d.scr_off;
            segs.push_back(Seg{be.peer_base(pw) + boff + ps.off, local_ptr(x.buf, x.off), x.bytes, false});
        }
        const bool fuse_ok = round_fusable(r, ts, local_ptr);
        std::vector<std::vector<const void *>> ins(r.ops.size());
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
                ins[i].push_back(p);
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
        if (step_pending && !gs.empty() && pw_store.size() <= 16 && pw_wait.size() <= 16) {
            // the step rides in the gather launch (small grids; else its own launch)
            const bool posts = !pw_store.empty();
            std::vector<uint64_t *> wa;
            std::vector<uint64_t> wv;
            std::vector<const uint64_t *> qa;
            std::vector<uint64_t> qv;
            take(wa, wv, qa, qv);
            if (posts && be.release() != 0) return SOSX_ERR_HIP;
            rc = be.gather_signalled((int)gs.size(), gs.data(), gd.data(), gb.data(), (int)wa.size(),
                                     wa.data(), wv.data(), (int)qa.size(), qa.data(), qv.data());
            if (rc) return rc;
            // the gather's workgroups acquired for their own loads only: folds below that
            // read peer bytes in place need the stream-wide acquire
            bool peer_ops = false;
            for (const auto &sg : segs) peer_ops |= sg.used;
            if (fuse_ok && peer_ops && be.acquire() != 0) return SOSX_ERR_HIP;
        } else {
            if (step_pending) {
                rc = flush();
                if (rc) return rc;
            }
            if (!gs.empty()) {
                rc = be.gather((int)gs.size(), gs.data(), gd.data(), gb.data());
                if (rc) return rc;
            }
        }
        if (fuse_ok) {
            rc = be.run_ops(r, ins, local_ptr);
            if (rc) return rc;
        }
        // this round's receives are read: mark them consumed; this PE's sends must be
        // consumed before anything overwrites them (the next round's ops or the caller)
        for (const auto &x : r.xfers) {
            const int pw = world_of(x.peer);
            if (x.send) pw_wait[&sh->dconsumed[my_world][pw]] = sl.posted[pw];
            else pw_store[&sh->dconsumed[pw][my_world]] = sl.seen[pw];
        }
        if (!fuse_ok) {
            rc = flush();
            if (rc) return rc;
            rc = be.run_ops(r, ins, local_ptr);
            if (rc) return rc;
        }
    }
    // the exit boundary (the last round's consumed marks) on the host, after completion
    be.phase(PH_ENQUEUE);
    const int e = be.complete();
    if (be.device_wait_failed()) return SOSX_ERR_STATE;
    if (e == 0) host_flush();
    be.phase(PH_SYNC_END);
    return e == 0 ? SOSX_OK : SOSX_ERR_HIP;
}

}  // namespace sosp2p
