// smallpath.cpp -- team reductions of small operands through node shared memory, without
// DMA copies: host-resident operands (SOS's own case) and, below a smaller limit, device
// ones.
//
// SOS runs a reduction below SHMEM_COLL_SIZE_CROSSOVER as recdbl_sw on host memory
// (src/shmem_collectives.h:192-195, src/collectives.c:850-984).  On the general path a
// host operand here costs an H2D copy, the exchange, a D2H copy and their DMA-engine
// latencies: 52 us per call at P = 2 and 290 us at P = 8 for a few bytes
// (profiles/r3_small_latency.txt).  This path keeps the bytes where SOS keeps them:
//   1. each PE copies its source into its slot of the node shared segment (host
//      memory every PE maps, registered with HIP on every GPU: fine-grained, mapped);
//   2. host flags (release/acquire) publish the slot to the team;
//   3. ONE kernel per PE (small.hip) reads all P slots in place over the host link and
//      writes the PE's result, as the schedule SOS would run prescribes:
//      - recdbl_sw (AUTO below the crossover, sosx_small_fold): every PE computes ITS OWN
//        recdbl_sw expression (the extra-PE folds, then the TREE over the leaves
//        permuted by my_idx; see plan.cpp build_recdbl_gather), bit for bit, +-0 ties
//        and NaN payloads included;
//      - the ring (AUTO above it, sosx_small_ring): chunk c folded from PE c, every
//        chunk evaluated by every PE (the allgather's result);
//      - the team scans (sosx_small_linear): the in-order prefix of the team's sources;
//      - the broadcasts (sosx_small_linear over one operand): the root's bytes;
//   4. the result lands in `target` directly when it is in the (device-mapped) host
//      symmetric heap, else in a pinned slot copied out; the host learns that the kernel
//      finished from per-workgroup completion words in pinned memory, not from a
//      stream synchronisation (about 5 us less per call).
// The arithmetic stays on the GPU; the host only moves the caller's bytes into and out
// of shared memory, as SOS's puts do.
//
// Device-resident operands (HBM) take the same path with two launches instead of one: a
// one-workgroup copy kernel moves the source into the slot and then stores the posts
// itself (steps 1-2 on the device), and the fold kernel, queued behind it, writes the
// result into the device target directly: one more launch, against the executors'
// exchange, fold and call-completion wait.  Measured with P PEs on one GPU, fp32 sum under AUTO
// (profiles/r3_small_latency.txt, runs dx and dx2): 20-24 / 23-27 / 71-72 us per 4-byte
// call at P = 2 / 4 / 8 against 40 / 46 / 173 on the p2p executor; from P * bytes =
// 256 KiB at P = 4 (53-64 vs 56 us) and 512 KiB at P = 2 (72-81 vs 49) the slot traffic
// over the host link costs as much as the exchange saves, or more.  The path takes device
// operands while P * bytes <= SHMEMX_SMALL_DEVICE (default 128 KiB).  The GPU-side posts
// do not shorten the critical path (a peer's fold still launches after the post arrives);
// they save the host a completion round trip.
//
// Memory visibility, consumer side: every kernel that reads the
// peers' slots runs a system-scope acquire in each workgroup before its first slot load
// (small.hip slot_acquire), after the host saw the peers' posts.
//
// Slot reuse: each PE alternates between two data slots.  A post to receiver r carries
// a per-pair index k (posted[q][r] = k) and the slot id (ring[q][r][k % 2]); receiver r
// acknowledges with consumed[r][q] = k after its kernel has read the slot.  Before a PE
// rewrites a slot it waits until every receiver of that slot's previous post has
// consumed it, so at most two posts per ordered pair are outstanding and the depth-2
// ring of slot ids never overwrites an unread entry.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <functional>
#include <map>
#include <vector>

#include "plan.h"
#include "runtime.h"
#include "sosx.h"

namespace sosrt {

namespace {

constexpr int kMaxPE = 64;
constexpr size_t kSlotsCap = (size_t)32 << 20;  // all PEs' two slots together
constexpr size_t kRingMaxPE = 8;                // sosx_small_ring's team sizes
// A call reads P operands over the host link (staging moves 2 per PE) after a host
// memcpy of its own, so above about a MiB per PE staging + the exchange wins: measured
// with P PEs on one GPU (profiles/r3_small_latency.txt, crossover runs), P = 2 at 256 KiB
// operands 50 us here vs 98 staged, at 1 MiB 231 vs 157; P = 4 at 256 KiB 141 vs 186.
// The path takes P * bytes <= this.
constexpr size_t kTeamBytes = (size_t)1 << 20;
constexpr size_t kLatencyBytes = 16 * 1024;     // always taken when it fits a slot
constexpr size_t kLocalCombineBytes = 64 * 1024;  // shmemx_reduce_local's small path
constexpr size_t kDeviceTeamBytes = 128 * 1024;   // default P * bytes limit, device operands

// Slot bytes (the largest operand the path takes): SHMEMX_SMALL_HOST_BYTES (default
// 1 MiB), capped so that 2 slots per PE stay within kSlotsCap, in 4 KiB units, at
// most SOSX_SMALL_FOLD_MAX 1-byte elements.  The same on every PE (job environment).
size_t slot_bytes_for(int npes)
{
    size_t b = env_size("SHMEMX_SMALL_HOST_BYTES", (size_t)1 << 20);
    const size_t cap = kSlotsCap / (2 * (size_t)(npes > 0 ? npes : 1));
    if (b > cap) b = cap;
    if (b > (size_t)SOSX_SMALL_FOLD_MAX) b = SOSX_SMALL_FOLD_MAX;
    return (b + 4095) & ~(size_t)4095;
}

struct alignas(64) PairWord {
    std::atomic<uint64_t> v;
    char pad[56];
};

// Per world PE q: posts to every receiver r, their slot ids, and q's acknowledgements
// of every sender's posts.  Cache-line separated: a PE spins on words others write.
struct SmallCtl {
    PairWord posted[kMaxPE];      // [r]: posts q made for r (count)
    PairWord consumed[kMaxPE];    // [s]: posts from s that q has read (count)
    PairWord route[kMaxPE];       // [r]: (k << 8) | tag of q's k-th routed call with r
    uint32_t ring[kMaxPE][2];     // [r][k % 2]: data slot of q's k-th post for r
};

// Route tags (the low byte of a route word): which path a PE took for a call, and the
// residency of its operands, so that a disagreement names both PEs' operands.
constexpr uint64_t kRouteSmall = 1, kRouteDevSrc = 2, kRouteDevDst = 4;

struct Small {
    bool ready = false;          // every PE registered the region (agreed at init)
    bool registered = false;
    char *host = nullptr;        // region base (host view)
    char *dev = nullptr;         // the same bytes, device view
    size_t bytes = 0;
    size_t slot = 0;             // bytes per data slot
    int npes = 0;
    uint64_t seq = 0;            // my posts (slot = seq % 2)
    uint64_t posted_to[kMaxPE] = {0};
    uint64_t seen_from[kMaxPE] = {0};
    std::vector<std::pair<int, uint64_t>> slot_users[2];  // receivers of each slot's last post
    void *out = nullptr;         // pinned result slot (hipHostMalloc, device-mapped)
    uint32_t *flags = nullptr;   // per-workgroup completion words (pinned, coherent)
    uint32_t fseq = 0;           // the value the current launch's workgroups store
    uint64_t routed[kMaxPE] = {0};  // routed calls shared with each world PE (both count)
    uint64_t route_k[kMaxPE] = {0};  // this call's index with each team peer (small path)
    uint64_t route_tag = 0;          // this call's route tag
    size_t dev_team_bytes = 0;   // device operands: P * bytes limit (0: host operands only)
    long calls = 0;
    long dev_calls = 0;          // of which with a device operand
};
Small g;

size_t ctl_bytes(int npes) { return ((size_t)npes * sizeof(SmallCtl) + 4095) & ~(size_t)4095; }

SmallCtl *ctl(int pe) { return (SmallCtl *)(g.host + (size_t)pe * sizeof(SmallCtl)); }

size_t slot_off(int pe, int sl) { return ctl_bytes(g.npes) + ((size_t)pe * 2 + (size_t)sl) * g.slot; }

double limit_s()
{
    const char *e = getenv("SHMEMX_P2P_TIMEOUT");
    const double v = e ? atof(e) : 0.0;
    return v > 0 ? v : 300.0;
}

double now_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

void wait_ge(const std::atomic<uint64_t> &w, uint64_t v, const char *what)
{
    if (w.load(std::memory_order_acquire) >= v) return;
    const double t0 = now_s();
    unsigned spins = 0;
    while (w.load(std::memory_order_acquire) < v) {
        __builtin_ia32_pause();
        if ((++spins & 0xFFFF) == 0 && now_s() - t0 > limit_s())
            raise_error("small shared-memory path: timed out after %.0f s waiting for %s",
                        limit_s(), what);
    }
}

// Wait until workgroups [0, nb) of the small fold stored `seq`.  The host polls pinned
// memory instead of synchronising the stream (a launch + hipStreamSynchronize costs
// ~12 us, a launch + flag poll ~6.6 us: profiles/r3_sync_probe.json).  Every 4096 polls
// the stream is queried: an error, or a drained stream whose flags are still missing,
// ends the job with a message, as does SHMEMX_P2P_TIMEOUT.
void wait_flags(const uint32_t *flags, int nb, uint32_t seq, const char *fn)
{
    const double t0 = now_s();
    unsigned spins = 0;
    for (int b = 0; b < nb;) {
        if (__atomic_load_n(flags + b, __ATOMIC_ACQUIRE) == seq) {
            ++b;
            continue;
        }
        __builtin_ia32_pause();
        if ((++spins & 0xFFF) != 0) continue;
        const hipError_t e = hipStreamQuery(st().stream);
        if (e == hipSuccess) {  // drained: every flag must be visible by now (after the
                                // runtime's own synchronisation at the latest)
            hip_check(sync_system(st().stream), fn);
            for (int k = b; k < nb; ++k)
                if (__atomic_load_n(flags + k, __ATOMIC_ACQUIRE) != seq)
                    raise_error("%s: small shared-memory path: workgroup %d of %d did not "
                                "signal completion", fn, k, nb);
            return;
        }
        if (e != hipErrorNotReady) hip_check(e, fn);
        if (now_s() - t0 > limit_s())
            raise_error("%s: small shared-memory path: timed out after %.0f s", fn, limit_s());
    }
}

// SOSX_SMALL_TRACE=N (diagnostics): host time per phase of small_path_reduce, averaged
// over windows of N calls and printed to stderr (slot free, copy + post, peers' posts,
// launch call, completion words, acks + copy out).
struct SmallTrace {
    int every = -1;
    long calls = 0;
    double t[6] = {0, 0, 0, 0, 0, 0};
    bool on()
    {
        if (every < 0) {
            const char *e = getenv("SOSX_SMALL_TRACE");
            every = e ? atoi(e) : 0;
        }
        return every > 0;
    }
};
SmallTrace g_strace;

}  // namespace

size_t small_shared_bytes(int npes)
{
    if (npes < 2 || npes > kMaxPE) return 0;
    return ctl_bytes(npes) + (size_t)npes * 2 * slot_bytes_for(npes);
}

// Collective (init_common, every PE): register this PE's view of the region with HIP
// and agree over the bootstrap that every PE could; otherwise the path stays off.
void small_path_setup(void *region, size_t bytes)
{
    State &s = st();
    g = Small();
    const char *e = getenv("SHMEMX_SMALL_HOST");
    const bool want = !(e && !strcmp(e, "0"));
    if (!s.hub.up || s.n_pes < 2 || s.n_pes > kMaxPE) return;
    int ok = region != nullptr && bytes >= small_shared_bytes(s.n_pes) && want;
    const size_t slot = slot_bytes_for(s.n_pes);
    const size_t flag_words = slot / 256 + kRingMaxPE;  // a 1-byte fold's workgroups
    void *dptr = nullptr;
    if (ok) {
        if (hipHostRegister(region, bytes, kP2PHostRegisterFlags) == hipSuccess) {
            g.registered = true;
            ok = hipHostGetDevicePointer(&dptr, region, 0) == hipSuccess && dptr;
        } else {
            ok = 0;
        }
        if (!ok) (void)hipGetLastError();
    }
    if (ok && hipHostMalloc(&g.out, slot, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        g.out = nullptr;
        ok = 0;
    }
    if (ok && hipHostMalloc((void **)&g.flags, flag_words * sizeof(uint32_t), hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        g.flags = nullptr;
        ok = 0;
    }
    if (g.flags) memset(g.flags, 0, flag_words * sizeof(uint32_t));
    std::vector<int> oks((size_t)s.n_pes);
    if (sosboot::hub_allgather(&s.hub, &ok, sizeof(ok), oks.data()) != 0)
        raise_error("shmem_init: small-path agreement failed");
    for (int v : oks) ok &= v;
    g.host = (char *)region;
    g.dev = (char *)dptr;
    g.bytes = bytes;
    g.slot = slot;
    g.npes = s.n_pes;
    g.dev_team_bytes = env_size("SHMEMX_SMALL_DEVICE", kDeviceTeamBytes);
    g.ready = ok != 0;
    if (!g.ready) small_path_teardown();
    debug_msg("small shared-memory path: %s", g.ready ? "on" : "off");
}

void small_path_teardown()
{
    if (g.registered && g.host) (void)hipHostUnregister(g.host);
    if (g.out) (void)hipHostFree(g.out);
    if (g.flags) (void)hipHostFree(g.flags);
    g = Small();
}

long small_path_calls() { return g.calls; }
long small_path_device_calls() { return g.dev_calls; }

// Collective over the world when the job is up: every PE passes the same limit (checked
// through the bootstrap), so the path choice for device operands stays uniform.  Without
// the bootstrap hub (shmemx_init_attr) there is no node shared segment, so the small
// path never sets up (small_path_setup returns at once) and the limit routes nothing:
// a disagreement there cannot split a call between paths, and no check is needed.
size_t small_path_set_device_bytes(size_t team_bytes)
{
    State &s = st();
    if (s.initialized && s.hub.up && s.n_pes > 1) {
        std::vector<uint64_t> all((size_t)s.n_pes);
        const uint64_t mine = team_bytes;
        if (sosboot::hub_allgather(&s.hub, &mine, sizeof(mine), all.data()) != 0)
            raise_error("sosx_set_small_device_bytes: agreement failed");
        for (int q = 0; q < s.n_pes; ++q)
            if (all[(size_t)q] != mine)
                raise_error("sosx_set_small_device_bytes: PE %d passed %llu, PE %d passed %llu (the call "
                            "is collective: every PE passes the same limit)", s.my_pe,
                            (unsigned long long)mine, q, (unsigned long long)all[(size_t)q]);
    }
    const size_t prev = g.dev_team_bytes;
    g.dev_team_bytes = team_bytes;
    return prev;
}

namespace {
bool takes(int alg, const void *target, const void *source, size_t bytes, const Team &t, bool dev_src,
           bool dev_dst)
{
    if (!g.ready || bytes == 0 || bytes > g.slot || t.size < 2 || t.size > kMaxPE) return false;
    const size_t team_bytes = (size_t)t.size * bytes;
    if (dev_src || dev_dst) {
        // the copy and fold kernels touch device operands directly: this GPU's HBM only
        if (team_bytes > g.dev_team_bytes) return false;
        if ((dev_src && !is_local_device_ptr(source)) || (dev_dst && !is_local_device_ptr(target)))
            return false;
    } else if (sosplan::is_bcast(alg)) {  // every PE reads one operand, the root's
        if (bytes > kTeamBytes) return false;
    } else if (bytes > kLatencyBytes && team_bytes > kTeamBytes) {
        return false;
    }
    if (sosplan::is_bcast(alg)) return true;
    if (alg == SOSX_ALG_RING || sosplan::is_scan(alg)) {
        if ((size_t)t.size > kRingMaxPE) return false;
    } else if (alg != SOSX_ALG_RECDBL && alg != SOSX_ALG_RECDBL_GATHER) {
        return false;
    }
    return sosplan::pow2_floor(t.size) <= SOSX_MAX_FOLD;
}
}  // namespace

// Does a reduction of `bytes` with these operands over team t take the small path?
bool small_path_takes(int alg, const void *target, const void *source, size_t bytes, const Team &t)
{
    if (!g.ready || bytes == 0 || bytes > g.slot || t.size < 2 || t.size > kMaxPE) return false;
    return takes(alg, target, source, bytes, t, is_device_ptr(source), is_device_ptr(target));
}

namespace {

const char *route_text(uint64_t tag)
{
    return (tag & kRouteSmall) ? "small shared-memory path" : "executor";
}

[[noreturn]] void route_mismatch(const char *fn, uint64_t mine, int q, uint64_t theirs, bool known)
{
    char other[160];
    if (known)
        snprintf(other, sizeof(other), "PE %d the %s (source %s, target %s)", q, route_text(theirs),
                 (theirs & kRouteDevSrc) ? "device" : "host", (theirs & kRouteDevDst) ? "device" : "host");
    else
        snprintf(other, sizeof(other), "PE %d the executor (it finished the call without posting)", q);
    raise_error("%s: the PEs of a team took different paths for the same call: PE %d the %s "
                "(source %s, target %s), %s.  Every PE of the team must pass operands of the same "
                "residency, and SHMEMX_SMALL_DEVICE / sosx_set_small_device_bytes must agree",
                fn, st().my_pe, route_text(mine), (mine & kRouteDevSrc) ? "device" : "host",
                (mine & kRouteDevDst) ? "device" : "host", other);
}

// Wait for peer q's k-th post of a small-path call (kp), checking q's route word: a
// peer that took the executor for this call (its route word for the call says so, or it
// has moved past the call without posting) ends the job at once with both PEs' operands
// named, instead of after SHMEMX_P2P_TIMEOUT.
// While q's kp-th post is missing: q's route word says whether it took the other path
// for this call (ends the job at once, both PEs' operands named).  `past`: when q was
// first seen past the call with the post missing.
void route_check(int q, uint64_t kp, uint64_t mine, const char *fn, double &past)
{
    const int mw = st().my_pe;
    const std::atomic<uint64_t> &w = ctl(q)->posted[mw].v;
    const uint64_t v = ctl(q)->route[mw].v.load(std::memory_order_acquire);
    const uint64_t ik = v >> 8, rk = g.route_k[q];
    if (ik == rk && !(v & kRouteSmall)) route_mismatch(fn, mine, q, v & 0xFF, true);
    if (ik > rk && w.load(std::memory_order_acquire) < kp) {
        // q finished this call: on the small path its post came first (a device post
        // is stored by the copy kernel before q's fold can finish); allow the write
        // 10 ms to arrive before calling it a disagreement
        if (past == 0) past = now_s();
        else if (now_s() - past > 0.01) route_mismatch(fn, mine, q, 0, false);
    }
}

void wait_post(int q, uint64_t kp, uint64_t mine, const char *fn)
{
    const int mw = st().my_pe;
    const std::atomic<uint64_t> &w = ctl(q)->posted[mw].v;
    if (w.load(std::memory_order_acquire) >= kp) return;
    const double t0 = now_s();
    double past = 0;
    unsigned spins = 0;
    while (w.load(std::memory_order_acquire) < kp) {
        __builtin_ia32_pause();
        if ((++spins & 0xFF) != 0) continue;
        route_check(q, kp, mine, fn, past);
        if ((spins & 0xFFFF) == 0 && now_s() - t0 > limit_s())
            raise_error("small shared-memory path: timed out after %.0f s waiting for a peer's operand",
                        limit_s());
    }
}

}  // namespace

// Pick the small path or the executor for one team call and publish the choice to the
// team (route words in node shared memory): SOS's schedule choice depends only on the
// call's size (src/shmem_collectives.h:179-200), so all PEs agree by construction; this
// build's choice also depends on each PE's operand residency, so it is verified.  A PE
// on the small path waits for every peer's post (broadcasts included), and while it
// waits it reads the peer's route word (wait_post): a peer on the executor ends the job
// at once, with both PEs' operands named -- the executor PEs, blocked in the exchange,
// are then reaped by the launcher.  So a disagreement is always seen by a small-path PE,
// and the executor path pays one store per peer, no wait.  Every team call that can take
// the small path goes through here on every member PE, so the per-pair counts agree.
bool small_path_route(int alg, const void *target, const void *source, size_t bytes, const Team &t,
                      bool allowed, const char *fn)
{
    if (!g.ready || t.size < 2 || t.size > kMaxPE || t.my_idx < 0)
        return allowed && small_path_takes(alg, target, source, bytes, t);
    const bool dev_src = is_device_ptr(source), dev_dst = target == source ? dev_src : is_device_ptr(target);
    const bool take = allowed && takes(alg, target, source, bytes, t, dev_src, dev_dst);
    const int mw = st().my_pe;
    const uint64_t tag = (take ? kRouteSmall : 0) | (dev_src ? kRouteDevSrc : 0) | (dev_dst ? kRouteDevDst : 0);
    SmallCtl *mine = ctl(mw);
    for (int i = 0; i < t.size; ++i) {
        if (i == t.my_idx) continue;
        const int r = t.world_rank(i);
        const uint64_t k = ++g.routed[r];
        g.route_k[r] = k;
        mine->route[r].v.store(k << 8 | tag, std::memory_order_release);
    }
    g.route_tag = tag;
    return take;
}

// recdbl_sw's (or, for alg RING, the ring's; for the scan plans, the scan's) value for
// this PE over team t (see the file comment); returns when done.
void small_path_reduce(int alg, void *target, const void *source, size_t count, size_t ts,
                       const Team &t, int op, int dt, const char *fn)
{
    State &s = st();
    const size_t bytes = count * ts;
    const int P = t.size, me = t.my_idx, mw = s.my_pe;
    const int sl = (int)(g.seq++ % 2);
    const bool tr = g_strace.on();
    double tp = tr ? now_s() : 0;
    auto phase = [&](int ph) {
        if (!tr) return;
        const double now = now_s();
        g_strace.t[ph] += now - tp;
        tp = now;
    };
    auto trace_end = [&]() {  // a call's phases into the window; print every `every` calls
        if (!tr) return;
        phase(5);
        if (++g_strace.calls % g_strace.every == 0) {
            const double k = 1e6 / (double)g_strace.every;
            fprintf(stderr, "[%04d] small-path trace (calls %ld-%ld, us/call): slot %.2f copy+post %.2f "
                    "peers %.2f launch %.2f done %.2f acks+out %.2f\n", s.my_pe,
                    g_strace.calls - g_strace.every + 1, g_strace.calls, g_strace.t[0] * k,
                    g_strace.t[1] * k, g_strace.t[2] * k, g_strace.t[3] * k, g_strace.t[4] * k,
                    g_strace.t[5] * k);
            for (double &v : g_strace.t) v = 0;
        }
    };
    // 1. my slot is free once every receiver of its previous post has read it
    for (const auto &u : g.slot_users[sl]) wait_ge(ctl(u.first)->consumed[mw].v, u.second, "a peer to read a slot");
    g.slot_users[sl].clear();
    phase(0);
    const bool bcast = sosplan::is_bcast(alg);
    const int root = bcast ? (alg - sosplan::PLAN_BCAST) / 2 : -1;
    const bool dev_src = is_device_ptr(source), dev_dst = is_device_ptr(target);
    // a broadcast reads only the root's operand; the others post an empty slot.  A device
    // source reaches the slot through a one-workgroup copy launch that then makes the
    // posts itself (sosx_small_stage), so the host goes straight on to the peers' posts
    // and the fold launch queues behind the copy on the stream.
    const bool staged = dev_src && (!bcast || me == root);
    if ((!bcast || me == root) && !staged) memcpy(g.host + slot_off(mw, sl), source, bytes);
    // 2. publish it to the team, then take the peers' posts
    std::atomic_thread_fence(std::memory_order_release);
    SmallCtl *mine = ctl(mw);
    uint64_t *words[kMaxPE];
    uint64_t vals[kMaxPE];
    int nw = 0;
    for (int i = 0; i < P; ++i) {
        if (i == me) continue;
        const int r = t.world_rank(i);
        const uint64_t k = ++g.posted_to[r];
        mine->ring[r][k % 2] = (uint32_t)sl;
        if (staged) {  // the copy kernel's post: the device view of the same word
            words[nw] = (uint64_t *)(g.dev + ((char *)&mine->posted[r].v - g.host));
            vals[nw++] = k;
        } else {
            mine->posted[r].v.store(k, std::memory_order_release);
        }
        g.slot_users[sl].push_back({r, k});
    }
    if (staged) {
        std::atomic_thread_fence(std::memory_order_seq_cst);  // the slot ids before the launch
        const int rc = sosx_small_stage(g.dev + slot_off(mw, sl), source, bytes, words, vals, nw, s.stream);
        if (rc) raise_error("%s: small-path copy of a device operand failed (status %d)", fn, rc);
    }
    phase(1);
    const void *in[kMaxPE];
    int from[kMaxPE];
    for (int i = 0; i < P; ++i) {
        from[i] = -1;
        const int q = t.world_rank(i);
        if (i == me) {
            in[i] = g.dev + slot_off(mw, sl);
            continue;
        }
        const uint64_t k = ++g.seen_from[q];
        wait_post(q, k, g.route_tag, fn);
        const int qs = (int)ctl(q)->ring[mw][k % 2];
        in[i] = g.dev + slot_off(q, qs);
        from[i] = q;
    }
    phase(2);
    // the result goes straight into a device target or the host symmetric heap
    // (device-mapped pinned memory), else into the pinned result slot
    const bool direct = dev_dst || s.host_heap.contains(target, bytes);
    void *out = direct ? target : g.out;  // null when this PE writes nothing
    if (++g.fseq == 0) g.fseq = 1;
    int rc = SOSX_OK, nblocks = 0;
    if (bcast) {
        // 3. one launch: the root's bytes into this PE's target -- every non-root, and the
        //    root itself for the team forms (copy_root, src/collectives_c.c4:390-397); the
        //    active-set forms leave the root's target untouched (:342-378)
        const bool copy_root = ((alg - sosplan::PLAN_BCAST) & 1) != 0;
        if (me != root || copy_root)
            rc = sosx_small_linear(SOSX_OP_BOR, SOSX_DT_UCHAR, out, &in[root], 1, bytes, g.flags,
                                   g.fseq, &nblocks, 1, s.stream);
        else
            out = nullptr;  // nothing written: no copy out either
    } else if (sosplan::is_scan(alg)) {
        // 3. one launch: the in-order prefix of the team's sources 0..me (inscan) or
        //    0..me-1 (exscan), the running value the left operand; exscan's PE 0 gets
        //    zeros, as SOS's memset (src/collectives.c:1111-1209)
        const int np = alg == sosplan::PLAN_INSCAN ? me + 1 : me;
        if (np > 0) {
            rc = sosx_small_linear(op, dt, out, in, np, count, g.flags, g.fseq, &nblocks, 1, s.stream);
        } else if (dev_dst) {
            hip_check(hipMemsetAsync(out, 0, bytes, s.stream), fn);
            hip_check(sync_system(s.stream), fn);
        } else {
            memset(out, 0, bytes);
        }
    } else if (alg == SOSX_ALG_RING) {
        // 3. one launch: every ring chunk c folded LINEAR from PE c (the reduce-scatter's
        //    order), all chunks by every PE (the allgather's result)
        rc = sosx_small_ring(op, dt, out, in, P, count, g.flags, g.fseq, &nblocks, s.stream);
    } else {
        // 3. one launch: this PE's recdbl_sw tree over the leaves w[y] = v[y ^ mp], where
        //    v[x] = in[x] OP in[x + p2] for the extra PEs (x < P - p2), else in[x]
        const int p2 = sosplan::pow2_floor(P), nx = P - p2;
        const int mp = me < p2 ? me : me - p2;
        const void *leaves[kMaxPE], *extras[kMaxPE];
        for (int y = 0; y < p2; ++y) {
            const int x = y ^ mp;
            leaves[y] = in[x];
            extras[y] = x < nx ? in[x + p2] : nullptr;
        }
        rc = sosx_small_fold(op, dt, out, leaves, extras, p2, count, g.flags, g.fseq, &nblocks, s.stream);
    }
    if (rc) raise_error("%s: small-path reduction failed (status %d)", fn, rc);
    // the launch read the peers' slots after their posts, each workgroup behind its own
    // system-scope acquire (small.hip slot_acquire)
    if (nblocks > 0) note_peer_read(true);
    // no fold launch followed the copy kernel (an active-set broadcast's root, exscan's
    // PE 0 with a host target): the call must not return while it still reads `source`
    if (staged && nblocks == 0) hip_check(sync_system(s.stream), fn);
    phase(3);
    // 4. completion from the workgroups' flags (no stream synchronisation); then the
    //    peers' slots are read: acknowledge; my result out
    wait_flags(g.flags, nblocks, g.fseq, fn);
    phase(4);
    for (int i = 0; i < P; ++i)
        if (from[i] >= 0) mine->consumed[from[i]].v.store(g.seen_from[from[i]], std::memory_order_release);
    if (!direct && out) memcpy(target, g.out, bytes);
    g.calls++;
    if (dev_src || dev_dst) g.dev_calls++;
    trace_end();
}

// ---------------------------------------------------------------------------------
// Small local combines (shmemx_reduce_local, shmem_internal_reduce_local's slot in this
// build): one launch of the LINEAR two-operand fold, out = inout OP in, with completion
// words instead of a stream synchronisation.  Host operands in the host symmetric heap
// (pinned, device-mapped) are read and written in place; other host memory goes through
// two pinned staging buffers.  Per process, any number of PEs.
// ---------------------------------------------------------------------------------
namespace {
struct LocalSmall {
    char *stage = nullptr;     // 2 x kLocalBytes, pinned
    uint32_t *flags = nullptr; // pinned, coherent
    uint32_t seq = 0;
    bool failed = false;
};
LocalSmall g_local_small;
constexpr size_t kLocalFlagWords = kLocalCombineBytes / 256 + 8;
}  // namespace

bool small_local_combine(int op, int dt, void *inout, const void *in, size_t count, size_t ts,
                         bool dev_io, bool dev_in)
{
    State &s = st();
    const size_t bytes = count * ts;
    if (bytes == 0 || bytes > kLocalCombineBytes || dev_io != dev_in) return false;
    LocalSmall &L = g_local_small;
    if (!L.flags && !L.failed) {
        if (hipHostMalloc((void **)&L.flags, kLocalFlagWords * sizeof(uint32_t), hipHostMallocCoherent) != hipSuccess ||
            hipHostMalloc((void **)&L.stage, 2 * kLocalCombineBytes, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            if (L.flags) (void)hipHostFree(L.flags);
            L = LocalSmall();
            L.failed = true;  // the general path serves every call
        } else {
            memset(L.flags, 0, kLocalFlagWords * sizeof(uint32_t));
        }
    }
    if (L.failed) return false;
    // operands: HBM and the host symmetric heap in place, other host memory staged
    const bool stage_io = !dev_io && !s.host_heap.contains(inout, bytes);
    const bool stage_in = !dev_in && !s.host_heap.contains(in, bytes);
    void *io = stage_io ? L.stage : inout;
    const void *ii = stage_in ? (const void *)(L.stage + kLocalCombineBytes) : in;
    if (stage_io) memcpy(L.stage, inout, bytes);
    if (stage_in) memcpy(L.stage + kLocalCombineBytes, in, bytes);
    if (++L.seq == 0) L.seq = 1;
    const void *ins[2] = {io, ii};
    int nblocks = 0;
    const int rc = sosx_small_linear(op, dt, io, ins, 2, count, L.flags, L.seq, &nblocks, 0, s.stream);
    if (rc) raise_error("shmemx_reduce_local: small combine failed (status %d)", rc);
    wait_flags(L.flags, nblocks, L.seq, "shmemx_reduce_local");
    if (stage_io) memcpy(inout, L.stage, bytes);
    return true;
}

void small_local_release()
{
    LocalSmall &L = g_local_small;
    if (L.flags) (void)hipHostFree(L.flags);
    if (L.stage) (void)hipHostFree(L.stage);
    L = LocalSmall();
}

}  // namespace sosrt

extern "C" long sosx_small_path_calls(void) { return sosrt::small_path_calls(); }
extern "C" long sosx_small_path_device_calls(void) { return sosrt::small_path_device_calls(); }
extern "C" size_t sosx_set_small_device_bytes(size_t team_bytes)
{
    return sosrt::small_path_set_device_bytes(team_bytes);
}
