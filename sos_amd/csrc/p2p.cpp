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
//      own plan (built here: plans are deterministic) and its published offsets; then
//      a system-scope acquire in stream order -- carried by the consuming launches' own
//      workgroups when their grids are small, else the acquire kernel first (carry.h) --
//      so no launch below reads a line this GPU's L2s kept from an earlier call
//      (DESIGN.md section 7.3);
//   3. folds whose inputs are received chunks read them IN PLACE from peer memory
//      (no staging copy) -- allowed when the round's outputs do not overlap the
//      bytes this PE is sending in the same round; the other receives are copied by
//      one multi-segment gather launch (all peers' links at once);
//   4. stream sync, mark every receive consumed; wait until the peers consumed every
//      send of this round; run the remaining local ops.
// For the SOS ring plan this is: fold chunk `me` straight from the P-1 peers' sources
// over their xGMI links (P+1 HBM/xGMI streams, one launch), then gather the P-1 owned
// chunks -- the RCCL version's scratch round trip disappears.
//
// Two signalling modes, agreed by every PE when the heap is mapped:
//   stream (the default): between rounds the counters move in stream
//     order, written and awaited by a one-workgroup kernel (sosx_p2p_signal) on
//     host-registered node shared memory, so the rounds are enqueued back to back and
//     the host synchronises once; the launches after a step that awaited posts owe the
//     acquire (a small gather that carries the step acquires in each workgroup).  The
//     call's entry and exit boundaries stay on the host (there is nothing queued for a
//     signal kernel to overlap there).  Each PE's buffer offsets for the
//     call travel ahead of the data through a small descriptor ring per ordered pair
//     (host handshake only, never waiting on a GPU).
//   host (SHMEMX_P2P_SIGNAL=host, or when HIP cannot register the segment): the host
//     synchronises the stream and moves the counters itself every round, as steps 1-4.
#include <time.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <functional>
#include <map>
#include <tuple>
#include <vector>

#include "carry.h"
#include "p2p_proto.h"
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

using sosp2p::kMaxPE;
using P2PShared = sosp2p::Shared;

sosp2p::Local g_local;

// stream-mode signalling state
struct Sig {
    bool on = false;                // stream mode in use
    bool capable = false;           // every PE registered the segment (agreed)
    bool registered = false;
    char *dbase = nullptr;          // device view of the shared segment
    long long limit_ticks = 0;      // device wall-clock ticks of SHMEMX_P2P_TIMEOUT
    sosp2p::StreamLocal sl;         // pair counters and descriptor indices (cumulative)
    bool host_entry = true;         // SHMEMX_P2P_ENTRY: the entry boundary on the host
};
Sig g_sig;

P2PShared *shared()
{
    return (P2PShared *)st().shm.extra;
}

template <class X> X *dev(X *host)
{
    return (X *)(g_sig.dbase + ((char *)host - (char *)shared()));
}

// Wall-clock bound of one wait (SHMEMX_P2P_TIMEOUT seconds, default 300): a peer that
// never posts ends the job with a message instead of hanging it.
// Test hook (tests/test_gpu_multipe.py::test_p2p_stall_mid_call): the PE named by
// SOSX_P2P_TEST_STALL_PE stops for 60 s right after the entry boundary of its first
// multi-round call, so its peers meet the bounded DEVICE waits of the later rounds.
// Compiled into the test build of the library only (-DSOSX_TEST_HOOKS,
// tests/fakerccl/libsos_amd_fakerccl.so); a no-op in the product.
void stall_hook()
{
#ifdef SOSX_TEST_HOOKS
    static const int pe = [] {
        const char *e = getenv("SOSX_P2P_TEST_STALL_PE");
        return e && *e ? atoi(e) : -1;
    }();
    static bool done = false;
    if (pe == st().my_pe && !done) {
        done = true;
        fprintf(stderr, "[%04d] test hook: stalling 60 s after the call's entry boundary\n", pe);
        sleep(60);
    }
#endif
}

// Completion of a round's sends / of the call: sync_system (runtime.h).  Test build only:
// SOSX_TEST_PLAIN_SYNC=1 restores round 4's plain hipStreamSynchronize, for the A/B of
// tools/p2p_stress.py.
hipError_t complete(hipStream_t stream)
{
#ifdef SOSX_TEST_HOOKS
    static const bool plain = [] {
        const char *e = getenv("SOSX_TEST_PLAIN_SYNC");
        return e && *e == '1';
    }();
    if (plain) return hipStreamSynchronize(stream);
#endif
    return sync_system(stream);
}

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

// The same bound for a counter the GPUs also write (stream mode).
void spin_until_u64(const uint64_t *a, uint64_t want, const char *what)
{
    unsigned spins = 0;
    double t0 = 0;
    while (__atomic_load_n(a, __ATOMIC_ACQUIRE) < want) {
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
// to stderr every N calls, with the host time spent inside the backend's release, signal,
// gather and local-op calls (the launches themselves).
struct Trace {
    int every = -1;  // -1: not read yet, 0: off
    double t[6] = {0, 0, 0, 0, 0, 0};
    double b[4] = {0, 0, 0, 0};  // host time inside the backend: release, signal, gather, ops
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

namespace {

// One local op of a round (copy, zero fill, fold, prefix); fold/prefix inputs come from
// `in` (received chunks may point into peer memory).
int run_round_op(const sosplan::Local &l, const std::vector<const void *> &in,
                 const std::function<char *(int, uint64_t)> &local_ptr, int op, int dt,
                 hipStream_t stream)
{
    if (l.kind == sosplan::COPY) {
        if (in[0] == local_ptr(l.out_buf, l.out_off)) return SOSX_OK;
        if (sos::carry_acquire(stream, 0, false) < 0) return SOSX_ERR_HIP;  // a library copy
        return hipMemcpyAsync(local_ptr(l.out_buf, l.out_off), in[0], l.count, hipMemcpyDeviceToDevice,
                              stream) == hipSuccess
                   ? SOSX_OK
                   : SOSX_ERR_HIP;
    }
    if (l.kind == sosplan::ZERO)
        return hipMemsetAsync(local_ptr(l.out_buf, l.out_off), 0, l.count, stream) == hipSuccess ? SOSX_OK
                                                                                                 : SOSX_ERR_HIP;
    prof_mark(0, false, stream);
    int rc;
    if (l.kind == sosplan::PREFIX) {
        void *outs[sosplan::PLAN_MAX_PE];
        for (int k = 0; k < l.nout; ++k) outs[k] = local_ptr(l.outs_buf[k], l.outs_off[k]);
        rc = sosx_prefix(op, dt, outs, in.data(), l.nin, l.own, l.count, stream);
    } else {
        rc = sosx_fold(op, dt, l.order, local_ptr(l.out_buf, l.out_off), in.data(), l.nin, l.count, stream);
    }
    prof_mark(0, true, stream);
    return rc;
}

}  // namespace

// Signalling setup (runtime.cpp ensure_device_heap, collective): register the shared
// segment with HIP on every PE and agree through the bootstrap whether stream mode is
// possible everywhere.  The mode in use starts as SHMEMX_P2P_SIGNAL; unset, it is stream
// when every PE drives the same GPU (equal or faster than host mode in every one-GPU
// measurement, profiles/r2_p2p_signal_latency.txt) and host when the PEs span several
// GPUs (stream mode across xGMI is unmeasured).  It can be switched collectively
// (sosx_set_p2p_signal_mode).
void p2p_signal_setup()
{
    State &s = st();
    // a fresh (zero-filled) segment: every pair's counters restart from 0 here too
    const bool reg = g_sig.registered;
    g_sig = Sig();
    g_sig.registered = reg;
    g_local = sosp2p::Local();
    if (!s.shm.extra || s.n_pes <= 1) return;
    int ok = 1;
    void *dptr = nullptr;
    if (!g_sig.registered) {
        const size_t bytes = (sizeof(P2PShared) + 4095) & ~(size_t)4095;
        hipError_t he = hipHostRegister(s.shm.extra, bytes, kP2PHostRegisterFlags);
        if (he == hipSuccess) g_sig.registered = true;
        else {
            (void)hipGetLastError();
            debug_msg("p2p: hipHostRegister of the shared segment failed (%s)", hipGetErrorString(he));
        }
    }
    if (g_sig.registered) {
        ok = hipHostGetDevicePointer(&dptr, s.shm.extra, 0) == hipSuccess && dptr;
        if (!ok) (void)hipGetLastError();
    } else {
        ok = 0;
    }
    int rate_khz = 0;
    if (ok && (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, s.device) != hipSuccess ||
               rate_khz <= 0)) {
        (void)hipGetLastError();
        ok = 0;
    }
    // which GPU this PE drives (PCI bus id): stream mode is the default only when every
    // PE shares one device -- the configuration every stream-mode measurement and test
    // ran in.  Across GPUs the device-side flags cross xGMI through host memory, which
    // no run has covered yet, so the default there is host signalling.
    struct Vote { int ok; char bus[20]; } mine, *votes;
    memset(&mine, 0, sizeof(mine));
    mine.ok = ok;
    if (hipDeviceGetPCIBusId(mine.bus, (int)sizeof(mine.bus) - 1, s.device) != hipSuccess) {
        (void)hipGetLastError();
        snprintf(mine.bus, sizeof(mine.bus), "dev%d", s.device);
    }
    std::vector<Vote> all((size_t)s.n_pes);
    votes = all.data();
    if (sosboot::hub_allgather(&s.hub, &mine, sizeof(mine), votes) != 0)
        raise_error("p2p: signalling mode agreement failed");
    bool one_device = true;
    for (const Vote &v : all) {
        ok &= v.ok;
        one_device &= strncmp(v.bus, all[0].bus, sizeof(v.bus)) == 0;
    }
    g_sig.capable = ok != 0;
    g_sig.dbase = (char *)dptr;
    g_sig.limit_ticks = (long long)(wait_limit_s() * 1e3 * (double)rate_khz);
    // SHMEMX_P2P_SIGNAL = stream | host (the same on every PE: job environment); unset:
    // stream on one device, host across devices
    const char *e = getenv("SHMEMX_P2P_SIGNAL");
    const bool want = e && *e ? strcmp(e, "host") != 0 : one_device;
    g_sig.on = g_sig.capable && want;
    // SHMEMX_P2P_ENTRY = host | device: where stream mode runs the call's entry boundary
    // (either mode interoperates with the other: the same counters, the same values)
    const char *en = getenv("SHMEMX_P2P_ENTRY");
    g_sig.host_entry = !(en && strcmp(en, "device") == 0);
    debug_msg("p2p transport signalling: %s (stream mode %s; PEs on %s)", g_sig.on ? "stream" : "host",
              g_sig.capable ? "available" : "unavailable", one_device ? "one device" : "several devices");
}

void p2p_signal_teardown()
{
    if (g_sig.registered && st().shm.extra) (void)hipHostUnregister(st().shm.extra);
    g_sig.registered = false;
    g_sig.on = false;
}

bool p2p_stream_signalling() { return g_sig.on; }
bool p2p_stream_capable() { return g_sig.capable; }
void p2p_set_stream_signalling(bool on) { g_sig.on = on && g_sig.capable; }

}  // namespace sosrt

// 1 = stream-ordered device signals, 0 = host synchronisation, -1 = no p2p transport
extern "C" int sosx_p2p_signal_mode(void)
{
    const sosrt::State &s = sosrt::st();
    if (!s.p2p_ready || s.n_pes <= 1) return -1;
    return sosrt::p2p_stream_signalling() ? 1 : 0;
}

// Switch the p2p signalling mode (1 stream, 0 host) between calls; collective: every PE
// switches at the same point of its call sequence.  Returns the previous mode, or -1
// (nothing changed) when the mode is unavailable.
extern "C" int sosx_set_p2p_signal_mode(int mode)
{
    const sosrt::State &s = sosrt::st();
    if (!s.p2p_ready || s.n_pes <= 1 || mode < 0 || mode > 1) return -1;
    if (mode == 1 && !sosrt::p2p_stream_capable()) return -1;
    const int prev = sosrt::p2p_stream_signalling() ? 1 : 0;
    sosrt::p2p_set_stream_signalling(mode == 1);
    return prev;
}

namespace sosrt {

namespace {

// Does p lie in a peer's device heap as mapped here (bytes another PE published)?
bool in_peer_heap(const void *p)
{
    const State &s = st();
    for (size_t q = 0; q < s.peer_heap.size(); ++q) {
        const char *b = s.peer_heap[q];
        if ((int)q != s.my_pe && b && (const char *)p >= b && (const char *)p < b + s.dev_heap_bytes)
            return true;
    }
    return false;
}

// The stream-wide acquire with the runtime's bookkeeping (carry.h stream_wide).
int stream_wide_acquire(hipStream_t st) { return acquire_system(st) == hipSuccess ? 0 : 1; }

// One p2p call's hand-off of the consumer-side acquire (carry.h): nothing owed at entry
// or exit, the runtime's acquire kernel as the stream-wide form.
struct CarryScope {
    CarryScope() { reset(); }
    ~CarryScope() { reset(); }
    static void reset()
    {
        sos::AcquireCarry &c = sos::acquire_carry();
        c.want = false;
        c.peer = false;
        c.stream_wide = &stream_wide_acquire;
    }
};

// The protocol's backend on this PE's HIP stream (p2p_proto.h), both signalling modes.
// It classifies waits and launches itself for the consumer-side check (note_peer_wait /
// note_peer_read, runtime.h): a wait on a `posted` / `dposted` counter is a wait for a
// peer's bytes; a gather or fold reading a peer's heap is a peer read.  acquire() does
// not launch: it marks the acquire owed (carry.h), and the next launch that reads a
// peer's heap carries it in its workgroups when its grid is small, or runs the acquire
// kernel first; a read that did neither after a wait counts as unacquired.
struct HipBackend {
    hipStream_t stream;
    int op, dt;
    int my_world;
    double tp;
    bool tr;
    int complete() { return sosrt::complete(stream) == hipSuccess ? 0 : 1; }
    bool merge_syncs()
    {
#ifdef SOSX_TEST_HOOKS
        // A/B (test build only, tools/host_sync_ab.sh): every drain and completion separate
        static const bool separate = [] {
            const char *e = getenv("SOSX_TEST_SEPARATE_SYNCS");
            return e && *e == '1';
        }();
        return !separate;
#else
        return true;
#endif
    }
    int drain(bool release)
    {
        return (release ? sosrt::complete(stream) : hipStreamSynchronize(stream)) == hipSuccess ? 0 : 1;
    }
    // host time of one backend call into the trace (SOSX_P2P_TRACE)
    template <class F> int timed(int slot, F &&f)
    {
        if (!tr) return f();
        const double t0 = now_s();
        const int rc = f();
        g_trace.b[slot] += now_s() - t0;
        return rc;
    }
    int release()
    {
        return timed(0, [&] { return release_system(stream) == hipSuccess ? 0 : 1; });
    }
    int acquire()
    {
#ifdef SOSX_TEST_HOOKS
        // A/B of the acquire's price (test build only, tools/acquire_cost.sh): skip it
        static const bool skip = [] {
            const char *e = getenv("SOSX_TEST_NO_ACQUIRE");
            return e && *e == '1';
        }();
        if (skip) return 0;
#endif
        sos::acquire_carry().want = true;
        return 0;
    }
    // a launch that reads peer bytes or not (`peer`): mark it for the launchers, then
    // count the read -- acquired in its own workgroups if any of its launches carried
    template <class F> int peer_launch(bool peer, F &&launch)
    {
        sos::AcquireCarry &c = sos::acquire_carry();
        c.peer = peer;
        const long c0 = c.carried;
        const int rc = launch();
        c.peer = false;
        if (peer) note_peer_read(c.carried > c0);
        return rc;
    }
    bool device_data_wait(int nq, const uint64_t *const *qa)
    {
        for (int i = 0; i < nq; ++i)
            if (sosp2p::in_dposted(shared(), g_sig.dbase, qa[i])) return true;
        return false;
    }
    int gather(int n, const void *const *srcs, void *const *dsts, const size_t *bytes)
    {
        bool peer = false;
        for (int i = 0; i < n; ++i) peer |= in_peer_heap(srcs[i]);
        prof_mark(1, false, stream);
        const int rc = timed(2, [&] { return peer_launch(peer, [&] { return sosx_gather(n, srcs, dsts, bytes, stream); }); });
        prof_mark(1, true, stream);
        return rc;
    }
    int signal(int nw, uint64_t *const *wa, const uint64_t *wv, int nq, const uint64_t *const *qa,
               const uint64_t *qv)
    {
        if (device_data_wait(nq, qa)) note_peer_wait();
        return timed(1, [&] {
            return sosx_p2p_signal(nw, wa, wv, nq, qa, qv, dev(&shared()->sig_err[my_world]), g_sig.limit_ticks,
                                   stream);
        });
    }
    int gather_signalled(int n, const void *const *srcs, void *const *dsts, const size_t *bytes, int nw,
                         uint64_t *const *wa, const uint64_t *wv, int nq, const uint64_t *const *qa,
                         const uint64_t *qv)
    {
        // the step's waits run inside the launch; with a wait for peers' bytes every
        // workgroup acquires before its loads (copy.hip k_gather<true>), or -- a step too
        // large to ride in the copy -- the copies carry the acquire after it
        const bool own = device_data_wait(nq, qa);
        if (own) note_peer_wait();
        bool peer = false;
        for (int i = 0; i < n; ++i) peer |= in_peer_heap(srcs[i]);
        prof_mark(1, false, stream);
        const int rc = timed(2, [&] {
            return peer_launch(peer, [&] {
                return sosx_gather_signalled(n, srcs, dsts, bytes, nw, wa, wv, nq, qa, qv,
                                             dev(&shared()->sig_err[my_world]), g_sig.limit_ticks, stream);
            });
        });
        prof_mark(1, true, stream);
        return rc;
    }
    int run_ops(const sosplan::Round &r, const std::vector<std::vector<const void *>> &ins,
                const sosp2p::LocalPtr &local_ptr)
    {
        for (size_t i = 0; i < r.ops.size(); ++i) {
            bool peer = false;
            for (const void *p : ins[i]) peer |= in_peer_heap(p);
            const int rc = timed(3, [&] {
                return peer_launch(peer, [&] { return run_round_op(r.ops[i], ins[i], local_ptr, op, dt, stream); });
            });
            if (rc) return rc;
        }
        return SOSX_OK;
    }
    uint64_t *dev(uint64_t *p) { return sosrt::dev(p); }
    const uint64_t *dev(const uint64_t *p) { return sosrt::dev(p); }
    const char *peer_base(int pw) { return st().peer_heap[(size_t)pw]; }
    void spin(std::atomic<uint64_t> &a, uint64_t want, const char *what)
    {
        spin_until(a, want, what);
        if (sosp2p::in_posted(shared(), &a)) note_peer_wait();
    }
    void spin_u64(const uint64_t *a, uint64_t want, const char *what)
    {
        spin_until_u64(a, want, what);
        if (sosp2p::in_dposted(shared(), (const char *)shared(), a)) note_peer_wait();
    }
    void entry_hook() { stall_hook(); }
    bool host_entry() { return g_sig.host_entry; }
    bool device_wait_failed()
    {
        if (__atomic_load_n(&shared()->sig_err[my_world], __ATOMIC_ACQUIRE))
            raise_error("p2p transport: timed out after %.0f s waiting for a peer (device wait)",
                        wait_limit_s());
        return false;
    }
    void plan_mismatch(int pw) { raise_error("p2p transport: plan mismatch with PE %d", pw); }
    void phase(int ph)
    {
        if (!tr) return;
        const double now = now_s();
        g_trace.t[ph] += now - tp;
        tp = now;
    }
};

}  // namespace

int p2p_exec(const sosplan::Plan &plan, const Team &t, int alg, uint64_t count, uint64_t ts,
             const P2PBufs &b, int op, int dt, hipStream_t stream)
{
    State &s = st();
    P2PShared *sh = shared();
    if (!sh) return SOSX_ERR_STATE;
    const bool tr = trace_on();
    HipBackend be{stream, op, dt, t.world_rank(t.my_idx), tr ? now_s() : 0, tr};
    CarryScope carry_scope;
    const sosp2p::Bufs pb{b.src, b.dst, b.scr, b.src_off, b.dst_off, b.scr_off, b.smis, b.dmis};
    auto world_of = [&](int i) { return t.world_rank(i); };
    if (g_sig.on) {
        const int rc = sosp2p::exec_stream(plan, t.size, t.my_idx, world_of, alg, count, ts, pb, sh,
                                           g_sig.sl, be);
        if (tr && ++g_trace.calls % g_trace.every == 0) {
            const double k = 1e6 / (double)g_trace.every;
            fprintf(stderr, "[%04d] p2p trace, stream mode (calls %ld-%ld, us/call): descriptors %.1f "
                    "enqueue %.1f (release %.1f signal %.1f gather %.1f ops %.1f) sync-end %.1f\n", s.my_pe,
                    g_trace.calls - g_trace.every + 1, g_trace.calls, g_trace.t[1] * k, g_trace.t[2] * k,
                    g_trace.b[0] * k, g_trace.b[1] * k, g_trace.b[2] * k, g_trace.b[3] * k, g_trace.t[5] * k);
            for (double &v : g_trace.t) v = 0;
            for (double &v : g_trace.b) v = 0;
        }
        return rc;
    }
    const int rc = sosp2p::exec_host(plan, t.size, t.my_idx, world_of, alg, count, ts, pb, sh, g_local, be);
    if (tr && ++g_trace.calls % g_trace.every == 0) {  // window averages, then reset
        const double k = 1e6 / (double)g_trace.every;
        fprintf(stderr, "[%04d] p2p trace (calls %ld-%ld, us/call): sync-send %.1f wait-post %.1f "
                "enqueue %.1f (gather %.1f ops %.1f) sync-ops %.1f wait-consumed %.1f sync-end %.1f\n", s.my_pe,
                g_trace.calls - g_trace.every + 1, g_trace.calls, g_trace.t[0] * k, g_trace.t[1] * k,
                g_trace.t[2] * k, g_trace.b[2] * k, g_trace.b[3] * k, g_trace.t[3] * k, g_trace.t[4] * k,
                g_trace.t[5] * k);
        for (double &v : g_trace.t) v = 0;
        for (double &v : g_trace.b) v = 0;
    }
    return rc;
}

}  // namespace sosrt
