// p2p_proto_harness.cpp -- the p2p transport's pairing protocol in both signalling modes
// (the product's own sosp2p::exec_host and sosp2p::exec_stream, sos_amd/csrc/p2p_proto.h)
// on CPU threads, for ThreadSanitizer.
//
// Test infrastructure (tests/test_p2p_proto.py builds and runs it; no GPU).  Each PE is a
// host thread with a "stream": a worker thread that runs the PE's queued copies and folds
// in order, as the GPU runs its stream.  Each PE's device heap is a host buffer every
// thread can read (the IPC mapping); the node-shared counters are sosp2p::Shared.  The
// plans are the product's (plan.cpp), the arithmetic is uint32 wrapping addition (order-
// independent, so every schedule's result is the plain sum / prefix / root's bytes).
// Every call's result is checked; under -fsanitize=thread every byte a worker reads from
// a peer must be ordered after the peer's writes, and every overwrite after the peers'
// reads, by the protocol's counters alone.  In stream mode the signal steps are queued on
// the worker like any kernel: their stores and (blocking) waits run in stream order, as
// the GPU's k_p2p_signal does, so a step that waits too early deadlocks here as there.
//
// Build with -DBROKEN_DRAIN to drop the drain before a round's receives are marked
// consumed (step 4): the sanitizer must then report the race (the negative control).
//
// The consumer half of the memory-visibility rule is checked too:
// the backend classifies every wait (a `posted` / `dposted` counter: a peer's bytes) and
// every queued copy or fold (does it read another PE's heap?) on its own, and a peer read
// with a wait since the protocol's last acquire() ends the run ("peer read without an
// acquire").  As in the HIP backend (sos_amd/csrc/carry.h), acquire() only marks the
// acquire owed and the next peer-reading launch pays it: carried in its own workgroups
// (the acquire stays owed for the launches after it) or as the stream-wide kernel first
// (settled); here the choice is a per-launch coin instead of the grid size, so both forms
// and their mixtures within one round are exercised.  Build with -DBROKEN_ACQUIRE to drop
// the acquires: the run must then fail that way (the negative control).
//
// Stream mode runs with the entry boundary on the host, queued, and mixed across PEs.
//
// Usage: p2p_proto_harness [iters]     prints "p2p protocol harness: N calls OK", exit 0
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "p2p_proto.h"

namespace {

struct Stream {
    std::mutex m;
    std::condition_variable cv, idle;
    std::deque<std::function<void()>> q;
    bool stop = false;
    int busy = 0;
    std::thread th;
    Stream()
    {
        th = std::thread([this] {
            for (;;) {
                std::function<void()> f;
                {
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] { return stop || !q.empty(); });
                    if (q.empty()) return;
                    f = std::move(q.front());
                    q.pop_front();
                    busy = 1;
                }
                f();
                {
                    std::lock_guard<std::mutex> lk(m);
                    busy = 0;
                    if (q.empty()) idle.notify_all();
                }
            }
        });
    }
    ~Stream()
    {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void push(std::function<void()> f)
    {
        std::lock_guard<std::mutex> lk(m);
        q.push_back(std::move(f));
        cv.notify_all();
    }
    void drain()
    {
        std::unique_lock<std::mutex> lk(m);
        idle.wait(lk, [&] { return q.empty() && !busy; });
    }
};

std::vector<char *> g_heaps;
constexpr size_t kHeap = 8u << 20;

[[noreturn]] void die(const char *what, int a = 0, int b = 0)
{
    fprintf(stderr, "p2p protocol harness: %s (%d %d)\n", what, a, b);
    fflush(stderr);
    abort();
}

bool in_peer_heap(int me, const void *p)
{
    for (size_t q = 0; q < g_heaps.size(); ++q)
        if ((int)q != me && (const char *)p >= g_heaps[q] && (const char *)p < g_heaps[q] + kHeap) return true;
    return false;
}

std::atomic<long> g_acquires{0}, g_peer_reads{0}, g_carried{0}, g_stream_wide{0};

struct CpuBackend {
    Stream *s;
    bool entry_on_host;
    int me;
    sosp2p::Shared *sh;
    sosp2p::AcquireTrack trk;
    bool owed = false;       // carry.h `want`: acquire() ran, no stream-wide acquire since
    uint64_t coin = 0x9E3779B97F4A7C15ull;
    void read(bool own)
    {
        trk.read(own);
        g_peer_reads++;
        if (own) g_acquires++;
        if (trk.unacquired) die("peer read without an acquire", me);
    }
    // a launch that reads a peer's heap, as HipBackend::peer_launch + carry_acquire
    void peer_launch_read()
    {
        if (!owed) {
            read(false);
            return;
        }
        coin ^= coin << 13;
        coin ^= coin >> 7;
        coin ^= coin << 17;
        if (coin & 1) {  // a small grid: each workgroup acquires; still owed afterwards
            g_carried++;
            read(true);
        } else {  // a streaming grid: the acquire kernel first, which settles it
            owed = false;
            trk.acquired();
            g_acquires++;
            g_stream_wide++;
            s->push([] { std::atomic_thread_fence(std::memory_order_acquire); });
            read(false);
        }
    }
    int acquire()
    {
#ifndef BROKEN_ACQUIRE
        owed = true;
#endif
        return 0;
    }
    bool data_wait(int nq, const uint64_t *const *qa)
    {
        for (int i = 0; i < nq; ++i)
            if (sosp2p::in_dposted(sh, (const char *)sh, qa[i])) return true;
        return false;
    }
    int complete()
    {
        s->drain();
        return 0;
    }
    bool merge_syncs() { return true; }
    int drain(bool)
    {
#ifndef BROKEN_DRAIN
        s->drain();
#endif
        return 0;
    }
    int gather(int n, const void *const *srcs, void *const *dsts, const size_t *bytes)
    {
        bool peer = false;
        for (int i = 0; i < n; ++i) peer |= in_peer_heap(me, srcs[i]);
        if (peer) peer_launch_read();
        std::vector<const void *> sv(srcs, srcs + n);
        std::vector<void *> dv(dsts, dsts + n);
        std::vector<size_t> bv(bytes, bytes + n);
        s->push([sv, dv, bv] {
            for (size_t i = 0; i < sv.size(); ++i) memcpy(dv[i], sv[i], bv[i]);
        });
        return 0;
    }
    int run_ops(const sosplan::Round &r, const std::vector<std::vector<const void *>> &ins,
                const sosp2p::LocalPtr &local_ptr)
    {
        for (size_t i = 0; i < r.ops.size(); ++i) {
            const sosplan::Local l = r.ops[i];
            const std::vector<const void *> in = ins[i];
            bool peer = false;
            for (const void *p : in) peer |= in_peer_heap(me, p);
            if (peer) peer_launch_read();
            if (l.kind == sosplan::COPY) {
                char *o = local_ptr(l.out_buf, l.out_off);
                s->push([o, in, l] { if (o != in[0]) memmove(o, in[0], l.count); });
            } else if (l.kind == sosplan::ZERO) {
                char *o = local_ptr(l.out_buf, l.out_off);
                s->push([o, l] { memset(o, 0, l.count); });
            } else if (l.kind == sosplan::FOLD) {
                char *o = local_ptr(l.out_buf, l.out_off);
                s->push([o, in, l] {
                    for (uint64_t e = 0; e < l.count; ++e) {
                        uint32_t acc = 0, v;
                        for (int k = 0; k < l.nin; ++k) {
                            memcpy(&v, (const char *)in[(size_t)k] + 4 * e, 4);
                            acc += v;
                        }
                        memcpy(o + 4 * e, &acc, 4);
                    }
                });
            } else {  // PREFIX: every input of an element before the first store
                std::vector<char *> outs;
                for (int k = 0; k < l.nout; ++k) outs.push_back(local_ptr(l.outs_buf[k], l.outs_off[k]));
                s->push([outs, in, l] {
                    std::vector<uint32_t> v((size_t)l.nin);
                    for (uint64_t e = 0; e < l.count; ++e) {
                        for (int k = 0; k < l.nin; ++k) memcpy(&v[(size_t)k], (const char *)in[(size_t)k] + 4 * e, 4);
                        uint32_t acc = 0;
                        for (int k = 0; k < l.nin; ++k) {
                            acc += v[(size_t)k];
                            memcpy(outs[(size_t)k] + 4 * e, &acc, 4);
                        }
                    }
                });
            }
        }
        return 0;
    }
    // stream mode
    int release() { return 0; }  // stream order is program order on the worker
    static void step(const std::vector<uint64_t *> &wa, const std::vector<uint64_t> &wv,
                     const std::vector<const uint64_t *> &qa, const std::vector<uint64_t> &qv)
    {
        for (size_t i = 0; i < wa.size(); ++i) __atomic_store_n(wa[i], wv[i], __ATOMIC_RELEASE);
        const auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < qa.size(); ++i)
            while (__atomic_load_n(qa[i], __ATOMIC_ACQUIRE) < qv[i]) {
                std::this_thread::yield();
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) die("device wait");
            }
    }
    int signal(int nw, uint64_t *const *wa, const uint64_t *wv, int nq, const uint64_t *const *qa,
               const uint64_t *qv)
    {
        if (data_wait(nq, qa)) trk.waited();
        std::vector<uint64_t *> a(wa, wa + nw);
        std::vector<uint64_t> av(wv, wv + nw);
        std::vector<const uint64_t *> q(qa, qa + nq);
        std::vector<uint64_t> qv2(qv, qv + nq);
        s->push([a, av, q, qv2] { step(a, av, q, qv2); });
        return 0;
    }
    int gather_signalled(int n, const void *const *srcs, void *const *dsts, const size_t *bytes, int nw,
                         uint64_t *const *wa, const uint64_t *wv, int nq, const uint64_t *const *qa,
                         const uint64_t *qv)
    {
        // the gather's workgroups acquire after the step's waits (copy.hip k_gather<true>)
        const bool own = data_wait(nq, qa);
        signal(nw, wa, wv, nq, qa, qv);
        bool peer = false;
        for (int i = 0; i < n; ++i) peer |= in_peer_heap(me, srcs[i]);
        if (peer) {
            if (own) read(true);
            else peer_launch_read();
        }
        std::vector<const void *> sv(srcs, srcs + n);
        std::vector<void *> dv(dsts, dsts + n);
        std::vector<size_t> bv(bytes, bytes + n);
        s->push([sv, dv, bv] {
            for (size_t i = 0; i < sv.size(); ++i) memcpy(dv[i], sv[i], bv[i]);
        });
        return 0;
    }
    uint64_t *dev(uint64_t *p) { return p; }
    const uint64_t *dev(const uint64_t *p) { return p; }
    void spin_u64(const uint64_t *a, uint64_t want, const char *what)
    {
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(a, __ATOMIC_ACQUIRE) < want) {
            std::this_thread::yield();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) die(what);
        }
        if (sosp2p::in_dposted(sh, (const char *)sh, a)) trk.waited();
    }
    void entry_hook() {}
    bool host_entry() { return entry_on_host; }
    bool device_wait_failed() { return false; }
    const char *peer_base(int pw) { return g_heaps[(size_t)pw]; }
    void spin(std::atomic<uint64_t> &a, uint64_t want, const char *what)
    {
        const auto t0 = std::chrono::steady_clock::now();
        while (a.load(std::memory_order_acquire) < want) {
            std::this_thread::yield();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) die(what);
        }
        if (sosp2p::in_posted(sh, &a)) trk.waited();
    }
    void plan_mismatch(int pw) { die("plan mismatch", pw); }
    void phase(int) {}
};

uint32_t val(uint64_t call, int pe, uint64_t i)
{
    uint64_t x = call * 0x9E3779B97F4A7C15ull ^ (uint64_t)pe << 40 ^ i;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return (uint32_t)x;
}

struct Case {
    int alg;
    uint64_t n;
    bool inplace;
    unsigned soff, doff;  // byte offsets of src/dst in their heap regions
};

// One PE: `cases` calls in order, every result checked.
// mode 0: host signalling; stream signalling with the entry boundary 1: on the host,
// 2: queued, 3: queued on odd PEs only (the two interoperate)
void pe_main(int P, int me, int mode, const std::vector<Case> &cases, sosp2p::Shared *sh,
             long *ok_calls)
{
    Stream st;
    const bool stream_mode = mode > 0;
    CpuBackend be{&st, mode == 1 || (mode == 3 && me % 2 == 0), me, sh, {}};
    sosp2p::Local loc;
    sosp2p::StreamLocal sl;
    char *heap = g_heaps[(size_t)me];
    const size_t region = kHeap / 4;
    std::vector<char> scratch_private;
    uint64_t call = 0;
    for (const Case &c : cases) {
        ++call;
        const uint64_t ts = 4, bytes = c.n * ts;
        char *src = heap + c.soff;
        char *dst = c.inplace ? src : heap + region + c.doff;
        // this call's source (the caller's write, after the previous call returned)
        for (uint64_t i = 0; i < c.n; ++i) {
            const uint32_t v = val(call, me, i);
            memcpy(src + 4 * i, &v, 4);
        }
        const uint32_t sentinel = 0xA5A5A5A5u;
        if (!c.inplace)
            for (uint64_t i = 0; i < c.n; ++i) memcpy(dst + 4 * i, &sentinel, 4);
        const unsigned smis = (unsigned)((uintptr_t)src & 15), dmis = (unsigned)((uintptr_t)dst & 15);
        sosplan::Plan plan;
        if (sosplan::build(c.alg, P, me, c.n, ts, smis, dmis, &plan) != SOSX_OK) die("plan", c.alg, P);
        char *scr = nullptr;
        uint64_t scr_off = 0;
        if (plan.scratch_bytes) {
            if (plan.scr_sent) {  // peers read it: in the heap, after both operands
                scr_off = 2 * region;
                if (scr_off + plan.scratch_bytes > kHeap) die("heap too small", (int)plan.scratch_bytes);
                scr = heap + scr_off;
            } else {
                scratch_private.assign(plan.scratch_bytes + 64, 0);
                scr = scratch_private.data();
            }
        }
        const sosp2p::Bufs b{src, dst, scr, (uint64_t)(src - heap), (uint64_t)(dst - heap), scr_off, smis, dmis};
        auto world_of = [](int i) { return i; };
        const int rc = stream_mode
                           ? sosp2p::exec_stream(plan, P, me, world_of, c.alg, c.n, ts, b, sh, sl, be)
                           : sosp2p::exec_host(plan, P, me, world_of, c.alg, c.n, ts, b, sh, loc, be);
        if (rc) die("exec_host failed", rc);
        // expected result at this PE
        const bool bcast = c.alg >= 32;
        const int root = bcast ? (c.alg - 32) >> 1 : 0;
        const bool copy_root = bcast && ((c.alg - 32) & 1);
        for (uint64_t i = 0; i < c.n; ++i) {
            uint32_t want = 0, got;
            if (c.alg == SOSX_PLAN_INSCAN || c.alg == SOSX_PLAN_EXSCAN) {
                const int last = c.alg == SOSX_PLAN_INSCAN ? me : me - 1;
                for (int p = 0; p <= last; ++p) want += val(call, p, i);
            } else if (bcast) {
                want = me != root ? val(call, root, i) : copy_root || c.inplace ? val(call, me, i) : sentinel;
            } else {
                for (int p = 0; p < P; ++p) want += val(call, p, i);
            }
            memcpy(&got, dst + 4 * i, 4);
            if (got != want) die("wrong result", c.alg, (int)i);
        }
        ++*ok_calls;
    }
}

}  // namespace

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2;
    long total = 0;
    auto *sh = (sosp2p::Shared *)calloc(1, sizeof(sosp2p::Shared));
    const int algs[] = {SOSX_ALG_RING, SOSX_ALG_RECDBL, SOSX_ALG_RECHALVING, SOSX_ALG_RECDBL_DIRECT,
                        SOSX_ALG_RECDBL_GATHER, SOSX_PLAN_INSCAN, SOSX_PLAN_EXSCAN};
    for (int mode = 0; mode < 4; ++mode)
    for (int P : {2, 3, 4, 5, 8, 12}) {
        g_heaps.clear();
        for (int q = 0; q < P; ++q) {
            char *h = (char *)aligned_alloc(4096, kHeap);
            memset(h, 0, kHeap);
            g_heaps.push_back(h);
        }
        std::vector<Case> cases;
        for (int it = 0; it < iters; ++it)
            for (uint64_t n : {1ull, 7ull, 1001ull, 65539ull}) {
                for (int alg : algs)
                    for (int inplace = 0; inplace < 2; ++inplace)
                        cases.push_back(Case{alg, n, inplace != 0, inplace ? 4u * (unsigned)it % 16 : 0u,
                                             inplace ? 0u : 8u});
                for (int root : {0, P - 1})
                    for (int copy = 0; copy < 2; ++copy)
                        cases.push_back(Case{SOSX_PLAN_BCAST(root, copy), n, false, 0, 4});
            }
        // every PE starts with fresh counters: a new job
        memset((void *)sh, 0, sizeof(*sh));
        std::vector<long> ok((size_t)P, 0);
        std::vector<std::thread> th;
        for (int q = 0; q < P; ++q)
            th.emplace_back(pe_main, P, q, mode, std::cref(cases), sh, &ok[(size_t)q]);
        for (auto &t : th) t.join();
        for (long v : ok) total += v;
        for (char *h : g_heaps) free(h);
    }
    free(sh);
    if (g_peer_reads.load() == 0) die("no launch read a peer's bytes");
#ifndef BROKEN_ACQUIRE
    if (g_carried.load() == 0 || g_stream_wide.load() == 0) die("one form of the acquire never ran");
#endif
    printf("p2p protocol harness: %ld calls OK (host and stream signalling, both entries); "
           "%ld peer reads, each after an acquire (%ld acquires: %ld carried by the launch, %ld "
           "stream-wide)\n", total, g_peer_reads.load(), g_acquires.load(), g_carried.load(),
           g_stream_wide.load());
    return 0;
}
