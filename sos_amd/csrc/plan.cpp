// plan.cpp -- the SOS team-reduction schedules as per-PE plans (see plan.h).
#include "plan.h"

#include <string.h>

namespace sosplan {

namespace {

inline uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

Xfer xf(int send, int peer, int buf, uint64_t off, uint64_t bytes)
{
    Xfer x;
    x.send = send;
    x.peer = peer;
    x.buf = buf;
    x.off = off;
    x.bytes = bytes;
    return x;
}

Local fold2(int out_buf, uint64_t out_off, int a_buf, uint64_t a_off, int b_buf, uint64_t b_off,
            uint64_t count)
{
    Local l;
    memset(&l, 0, sizeof(l));
    l.kind = FOLD;
    l.order = SOSX_ORDER_LINEAR;
    l.out_buf = out_buf;
    l.out_off = out_off;
    l.nin = 2;
    l.in_buf[0] = a_buf;
    l.in_off[0] = a_off;
    l.in_buf[1] = b_buf;
    l.in_off[1] = b_off;
    l.count = count;
    return l;
}

// Stride between the scratch slots a fold or prefix reads together.  Large slots: a
// multiple of 32 KiB plus 4 KiB, so slot k starts k * 4 KiB into HBM's 32 KiB channel
// interleave and the P-1 slots walk different channels (tools/offset_probe.py --multi,
// profiles/r4_offset_probe.txt: the 8-input fold over 4 KiB-staggered streams 6.13-6.18
// TB/s, over streams 0 mod 32 KiB apart 5.80-5.91; the 16-stream prefix 5.95 vs 5.68-5.72).
// Small slots keep the 1 KiB step (the fold over them is latency-bound).
static uint64_t slot_stride(uint64_t bytes)
{
    if (bytes < ((uint64_t)1 << 20)) return round_up(bytes + 16, 1024);
    return round_up(bytes + 16, 32768) + 4096;
}

// RING and RECDBL_DIRECT share the data movement: a direct reduce-scatter of the SOS
// ring chunks (chunk c is owned, folded and broadcast by team index c), then a
// direct allgather.  Only the fold order differs.
int build_direct(int alg, int P, int me, uint64_t count, uint64_t ts, unsigned src_mis,
                 unsigned dst_mis, Plan *plan)
{
    if (P > SOSX_MAX_FOLD) return SOSX_ERR_ARG;
    uint64_t n_me, first_me;
    ring_chunk(count, P, me, &n_me, &first_me);
    const uint64_t my_bytes = n_me * ts;
    // Scratch slot for each peer's copy of my chunk, 16-B congruent with my DST chunk,
    // slot_stride apart (round 3: chunk + 1 KiB, ~2 % faster than 256-B skews,
    // profiles/r3_fold_layout_probe.json; round 4: 4 KiB steps in the channel interleave
    // for chunks of 1 MiB and more).
    const uint64_t mis = (dst_mis + first_me * ts) & 15;
    const uint64_t stride = slot_stride(my_bytes);
    auto slot = [&](int peer) { return (uint64_t)((peer - me - 1 + P) % P) * stride + mis; };
    (void)src_mis;
    plan->scratch_bytes = (uint64_t)(P - 1) * stride;

    Round rs;  // reduce-scatter exchange
    for (int k = 1; k < P; ++k) {
        const int peer = (me + k) % P;
        uint64_t n_p, first_p;
        ring_chunk(count, P, peer, &n_p, &first_p);
        if (n_p) rs.xfers.push_back(xf(1, peer, SRC, first_p * ts, n_p * ts));
        if (n_me) rs.xfers.push_back(xf(0, peer, SCR, slot(peer), my_bytes));
    }
    if (n_me) {
        Local l;
        memset(&l, 0, sizeof(l));
        l.kind = FOLD;
        l.out_buf = DST;
        l.out_off = first_me * ts;
        l.nin = P;
        l.count = n_me;
        if (alg == SOSX_ALG_RING) {
            // ring fold of chunk c starts at PE c (= me) and walks right:
            // ((s_me OP s_me+1) OP ...) OP s_me-1  (src/collectives.c:711-726)
            l.order = SOSX_ORDER_LINEAR;
            for (int k = 0; k < P; ++k) {
                const int pe = (me + k) % P;
                l.in_buf[k] = pe == me ? SRC : SCR;
                l.in_off[k] = pe == me ? first_me * ts : slot(pe);
            }
        } else {
            // recdbl_sw tree over team indices 0..P-1
            l.order = SOSX_ORDER_TREE;
            for (int pe = 0; pe < P; ++pe) {
                l.in_buf[pe] = pe == me ? SRC : SCR;
                l.in_off[pe] = pe == me ? first_me * ts : slot(pe);
            }
        }
        rs.ops.push_back(l);
    }
    plan->rounds.push_back(rs);

    Round ag;  // direct allgather of the owned chunks
    for (int k = 1; k < P; ++k) {
        const int peer = (me + k) % P;
        uint64_t n_p, first_p;
        ring_chunk(count, P, peer, &n_p, &first_p);
        if (n_me) ag.xfers.push_back(xf(1, peer, DST, first_me * ts, my_bytes));
        if (n_p) ag.xfers.push_back(xf(0, peer, DST, first_p * ts, n_p * ts));
    }
    plan->rounds.push_back(ag);
    return SOSX_OK;
}

// recdbl_sw butterfly, step for step (src/collectives.c:850-984).  The current vector
// lives in DST (the reference keeps it in a malloc'd copy and uses the target as the
// receive buffer; here the receive buffer is scratch, so no final copy is needed).
int build_recdbl(int P, int me, uint64_t count, uint64_t ts, unsigned dst_mis, Plan *plan)
{
    const int pow2 = pow2_floor(P);
    const uint64_t bytes = count * ts;
    const uint64_t soff = dst_mis & 15;  // scratch congruent with DST
    plan->scratch_bytes = round_up(bytes + 16, 256);
    if (me >= pow2) {
        // extra PE: hand the vector to its partner (:905-917), receive the result (:966-975)
        Round a;
        a.xfers.push_back(xf(1, me - pow2, SRC, 0, bytes));
        plan->rounds.push_back(a);
        Round b;
        b.xfers.push_back(xf(0, me - pow2, DST, 0, bytes));
        plan->rounds.push_back(b);
        return SOSX_OK;
    }
    int cur = SRC;
    if (me < P - pow2) {
        // fold the extra PE's vector: current = current OP extra (:920-926)
        Round a;
        a.xfers.push_back(xf(0, me + pow2, SCR, soff, bytes));
        a.ops.push_back(fold2(DST, 0, cur, 0, SCR, soff, count));
        plan->rounds.push_back(a);
        cur = DST;
    }
    for (int d = 1; d < pow2; d <<= 1) {
        // pairwise exchange at distance d: current = current OP peer (:932-963)
        Round r;
        r.xfers.push_back(xf(1, me ^ d, cur, 0, bytes));
        r.xfers.push_back(xf(0, me ^ d, SCR, soff, bytes));
        r.ops.push_back(fold2(DST, 0, cur, 0, SCR, soff, count));
        plan->rounds.push_back(r);
        cur = DST;
    }
    if (me < P - pow2) {
        Round b;
        b.xfers.push_back(xf(1, me + pow2, DST, 0, bytes));
        plan->rounds.push_back(b);
    }
    return SOSX_OK;
}

// recdbl_sw's result for every PE after ONE direct all-gather round (the latency-bound
// small-message case: 1 exchange round instead of log2(P), + 2 for a non-power-of-2 P).
// recdbl_sw at PE me < p2 (src/collectives.c:878-963) computes
//   v[x] = in[x] OP in[x + p2] for x < P - p2, else in[x]        (fold of the extra PEs)
//   T(x, 0) = v[x];  T(x, l) = T(x, l-1) OP T(x ^ 2^(l-1), l-1)   (left operand = own)
// and hands T(me, log2 p2) to its extra partner me + p2.  Relabelling y = x ^ me turns
// T(me, .) into the standard left-to-right pairwise tree over w[y] = v[y ^ me], which is
// the fold kernel's TREE order over p2 inputs: so every PE evaluates ITS OWN recdbl_sw
// expression (NaN payloads and +-0 ties included) from the gathered inputs, bit for bit.
int build_recdbl_gather(int P, int me, uint64_t count, uint64_t ts, unsigned dst_mis, Plan *plan)
{
    const int p2 = pow2_floor(P);
    const int nx = P - p2;  // extra PEs
    if (p2 > SOSX_MAX_FOLD) return SOSX_ERR_ARG;
    const uint64_t bytes = count * ts;
    const uint64_t soff = dst_mis & 15;  // scratch slots congruent with DST
    const uint64_t stride = round_up(bytes + 16, 256);
    // slots: P-1 received vectors (indexed by distance), then nx pre-folded extras
    auto rslot = [&](int pe) { return (uint64_t)((pe - me - 1 + P) % P) * stride + soff; };
    auto vslot = [&](int x) { return (uint64_t)(P - 1 + x) * stride + soff; };
    plan->scratch_bytes = (uint64_t)(P - 1 + nx) * stride;
    auto in_buf = [&](int pe) { return pe == me ? SRC : SCR; };
    auto in_off = [&](int pe) { return pe == me ? (uint64_t)0 : rslot(pe); };
    Round r;
    for (int k = 1; k < P; ++k) {
        const int peer = (me + k) % P;
        r.xfers.push_back(xf(1, peer, SRC, 0, bytes));
        r.xfers.push_back(xf(0, peer, SCR, rslot(peer), bytes));
    }
    for (int x = 0; x < nx; ++x)
        r.ops.push_back(fold2(SCR, vslot(x), in_buf(x), in_off(x), in_buf(x + p2), in_off(x + p2),
                              count));
    const int mp = me < p2 ? me : me - p2;  // an extra PE receives its partner's result
    Local l;
    memset(&l, 0, sizeof(l));
    l.kind = FOLD;
    l.order = SOSX_ORDER_TREE;
    l.out_buf = DST;
    l.out_off = 0;
    l.nin = p2;
    l.count = count;
    for (int y = 0; y < p2; ++y) {
        const int x = y ^ mp;
        l.in_buf[y] = x < nx ? SCR : in_buf(x);
        l.in_off[y] = x < nx ? vslot(x) : in_off(x);
    }
    if (p2 == 1) {  // P == 1 is handled by build(); P >= 2 always has p2 >= 2
        return SOSX_ERR_ARG;
    }
    r.ops.push_back(l);
    plan->rounds.push_back(r);
    return SOSX_OK;
}

// Recursive halving (reduce-scatter at distance 1, 2, 4, ...) + recursive doubling
// (allgather at distance ..., 4, 2, 1), with the recdbl_sw fold of extra PEs.
int build_rechalving(int P, int me, uint64_t count, uint64_t ts, unsigned dst_mis, Plan *plan)
{
    const int pow2 = pow2_floor(P);
    const uint64_t bytes = count * ts;
    plan->scratch_bytes = round_up((count - count / 2) * ts + 16, 256);
    if (me >= pow2) {
        Round a;
        a.xfers.push_back(xf(1, me - pow2, SRC, 0, bytes));
        plan->rounds.push_back(a);
        Round b;
        b.xfers.push_back(xf(0, me - pow2, DST, 0, bytes));
        plan->rounds.push_back(b);
        return SOSX_OK;
    }
    int cur = SRC;
    if (me < P - pow2) {
        plan->scratch_bytes = round_up(bytes + 16, 256);
        const uint64_t soff = dst_mis & 15;
        Round a;
        a.xfers.push_back(xf(0, me + pow2, SCR, soff, bytes));
        a.ops.push_back(fold2(DST, 0, cur, 0, SCR, soff, count));
        plan->rounds.push_back(a);
        cur = DST;
    }
    struct Seg { uint64_t lo, hi, mid; bool low; };
    std::vector<Seg> stack;
    uint64_t lo = 0, hi = count;
    for (int d = 1; d < pow2; d <<= 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        const bool low = (me & d) == 0;
        const uint64_t klo = low ? lo : mid, khi = low ? mid : hi;  // kept
        const uint64_t slo = low ? mid : lo, shi = low ? hi : mid;  // sent
        const uint64_t soff = (dst_mis + klo * ts) & 15;
        Round r;
        if (shi > slo) r.xfers.push_back(xf(1, me ^ d, cur, slo * ts, (shi - slo) * ts));
        if (khi > klo) {
            r.xfers.push_back(xf(0, me ^ d, SCR, soff, (khi - klo) * ts));
            r.ops.push_back(fold2(DST, klo * ts, cur, klo * ts, SCR, soff, khi - klo));
        }
        plan->rounds.push_back(r);
        stack.push_back(Seg{lo, hi, mid, low});
        lo = klo;
        hi = khi;
        cur = DST;
    }
    // recursive doubling: undo the halving in reverse
    for (int d = pow2 >> 1; d >= 1; d >>= 1) {
        const Seg parent = stack.back();
        stack.pop_back();
        // my range is the half of `parent` I kept; the partner owns the other half
        const uint64_t olo = parent.low ? parent.mid : parent.lo;
        const uint64_t ohi = parent.low ? parent.hi : parent.mid;
        Round r;
        if (hi > lo) r.xfers.push_back(xf(1, me ^ d, DST, lo * ts, (hi - lo) * ts));
        if (ohi > olo) r.xfers.push_back(xf(0, me ^ d, DST, olo * ts, (ohi - olo) * ts));
        plan->rounds.push_back(r);
        lo = parent.lo;
        hi = parent.hi;
    }
    if (me < P - pow2) {
        Round b;
        b.xfers.push_back(xf(1, me + pow2, DST, 0, bytes));
        plan->rounds.push_back(b);
    }
    return SOSX_OK;
}

// Team prefix scan (SOS scan_ring semantics, src/collectives.c:1111-1209): PE i's result
// is ((s_0 OP s_1) OP ...) OP s_i (inscan) or the same over s_0..s_{i-1} with PE 0
// zeroed (exscan).  Ring chunk c of every source is gathered at PE c, one PREFIX pass
// yields chunk c of all P results, a direct all-to-all hands them out.
int build_scan(bool exclusive, int P, int me, uint64_t count, uint64_t ts, unsigned src_mis,
               unsigned dst_mis, Plan *plan)
{
    if (P > PLAN_MAX_PE) return SOSX_ERR_ARG;
    uint64_t n_me, first_me;
    ring_chunk(count, P, me, &n_me, &first_me);
    const uint64_t my_bytes = n_me * ts;
    const uint64_t mis = (dst_mis + first_me * ts) & 15;
    const uint64_t stride = my_bytes < ((uint64_t)1 << 20) ? round_up(my_bytes + 16, 256) : slot_stride(my_bytes);
    (void)src_mis;
    // SCR: P-1 slots for the peers' copies of my chunk, then P-1 slots for my chunk of
    // the peers' results
    auto idx = [&](int peer) { return (uint64_t)((peer - me - 1 + P) % P); };
    auto slot_in = [&](int peer) { return idx(peer) * stride + mis; };
    auto slot_out = [&](int peer) { return ((uint64_t)(P - 1) + idx(peer)) * stride + mis; };
    plan->scratch_bytes = 2 * (uint64_t)(P - 1) * stride;
    plan->scr_sent = true;

    Round g;  // gather chunk `me` of every source
    for (int k = 1; k < P; ++k) {
        const int peer = (me + k) % P;
        uint64_t n_p, first_p;
        ring_chunk(count, P, peer, &n_p, &first_p);
        if (n_p) g.xfers.push_back(xf(1, peer, SRC, first_p * ts, n_p * ts));
        if (n_me) g.xfers.push_back(xf(0, peer, SCR, slot_in(peer), my_bytes));
    }
    if (n_me) {
        auto in_of = [&](int pe, int *b, uint64_t *o) {
            *b = pe == me ? SRC : SCR;
            *o = pe == me ? first_me * ts : slot_in(pe);
        };
        auto out_of = [&](int pe, int *b, uint64_t *o) {
            *b = pe == me ? DST : SCR;
            *o = pe == me ? first_me * ts : slot_out(pe);
        };
        Local l;
        memset(&l, 0, sizeof(l));
        l.kind = PREFIX;
        l.count = n_me;
        l.own = -1;
        // inscan: outs[k] (PE k) = prefix(ins[0..k]); exscan: outs[k] (PE k+1) = prefix(ins[0..k])
        const int nin = exclusive ? P - 1 : P;
        l.nin = l.nout = nin;
        for (int k = 0; k < nin; ++k) {
            in_of(k, &l.in_buf[k], &l.in_off[k]);
            out_of(exclusive ? k + 1 : k, &l.outs_buf[k], &l.outs_off[k]);
            if (k == me) l.own = k;
        }
        l.out_buf = l.outs_buf[0];
        l.out_off = l.outs_off[0];
        g.ops.push_back(l);
        if (exclusive) {
            // PE 0's result is zero (src/collectives.c:1145-1155); after the PREFIX pass,
            // which may still read my source chunk where it aliases the target
            Local z;
            memset(&z, 0, sizeof(z));
            z.kind = ZERO;
            out_of(0, &z.out_buf, &z.out_off);
            z.count = my_bytes;
            g.ops.push_back(z);
        }
    }
    plan->rounds.push_back(g);

    Round a;  // all-to-all of the result chunks
    for (int k = 1; k < P; ++k) {
        const int peer = (me + k) % P;
        uint64_t n_p, first_p;
        ring_chunk(count, P, peer, &n_p, &first_p);
        if (n_me) a.xfers.push_back(xf(1, peer, SCR, slot_out(peer), my_bytes));
        if (n_p) a.xfers.push_back(xf(0, peer, DST, first_p * ts, n_p * ts));
    }
    plan->rounds.push_back(a);
    return SOSX_OK;
}

// Broadcast from team index `root` (src/collectives.c:429-485).  Payloads of at least
// kBcastSplitBytes over P > 2 PEs: the root scatters P-1 chunks (one per non-root, each
// over its own link), the non-roots exchange them directly -- every link carries ~1/(P-1)
// of the payload per round instead of the root's link(s) carrying P-1 copies.
constexpr uint64_t kBcastSplitBytes = 64 * 1024;

int build_bcast(int root, bool copy_root, int P, int me, uint64_t count, uint64_t ts, Plan *plan)
{
    if (root < 0 || root >= P) return SOSX_ERR_ARG;
    const uint64_t bytes = count * ts;
    plan->reads_src = me == root;
    plan->writes_dst = me != root || copy_root;
    Round r;
    if (me == root && copy_root) {
        Local l;
        memset(&l, 0, sizeof(l));
        l.kind = COPY;
        l.out_buf = DST;
        l.nin = 1;
        l.in_buf[0] = SRC;
        l.count = bytes;
        r.ops.push_back(l);
    }
    if (P == 1) {
        plan->rounds.push_back(r);
        return SOSX_OK;
    }
    if (P == 2 || bytes < kBcastSplitBytes) {
        for (int k = 1; k < P; ++k) {
            const int peer = (root + k) % P;
            if (me == root) r.xfers.push_back(xf(1, peer, SRC, 0, bytes));
            else if (me == peer) r.xfers.push_back(xf(0, root, DST, 0, bytes));
        }
        plan->rounds.push_back(r);
        return SOSX_OK;
    }
    // chunk j (j = 0..P-2) belongs to the j-th non-root in ring order after the root;
    // chunks are cut in 64-B units when the element size divides 64
    const uint64_t unit = (64 % ts == 0) ? 64 / ts : 1;
    const uint64_t units = (count + unit - 1) / unit;
    auto chunk = [&](int j, uint64_t *off, uint64_t *len) {
        uint64_t n, first;
        ring_chunk(units, P - 1, j, &n, &first);
        uint64_t lo = first * unit, hi = (first + n) * unit;
        if (lo > count) lo = count;
        if (hi > count) hi = count;
        *off = lo * ts;
        *len = (hi - lo) * ts;
    };
    auto owner = [&](int j) { return (root + 1 + j) % P; };
    const int mine = me == root ? -1 : (me - root - 1 + P) % P;
    for (int j = 0; j < P - 1; ++j) {  // scatter
        uint64_t off, len;
        chunk(j, &off, &len);
        if (!len) continue;
        if (me == root) r.xfers.push_back(xf(1, owner(j), SRC, off, len));
        else if (j == mine) r.xfers.push_back(xf(0, root, DST, off, len));
    }
    plan->rounds.push_back(r);
    if (me == root) return SOSX_OK;
    Round ag;  // allgather among the non-roots
    uint64_t moff, mlen;
    chunk(mine, &moff, &mlen);
    for (int k = 1; k < P - 1; ++k) {
        const int j = (mine + k) % (P - 1);
        uint64_t off, len;
        chunk(j, &off, &len);
        if (mlen) ag.xfers.push_back(xf(1, owner(j), DST, moff, mlen));
        if (len) ag.xfers.push_back(xf(0, owner(j), DST, off, len));
    }
    plan->rounds.push_back(ag);
    return SOSX_OK;
}

}  // namespace

// Largest power of two <= P (src/collectives.c:878-882 for P >= 2).
int pow2_floor(int P)
{
    int p = 1;
    while (p * 2 <= P) p *= 2;
    return p;
}

void ring_chunk(uint64_t count, int P, int c, uint64_t *n, uint64_t *first)
{
    const uint64_t rem = count % (uint64_t)P;
    const uint64_t extra = (uint64_t)c < rem;
    const uint64_t cnt = count / (uint64_t)P + extra;
    *n = cnt;
    *first = extra ? (uint64_t)c * cnt : (uint64_t)c * cnt + rem;
}

int resolve_alg(int alg, uint64_t bytes, uint64_t crossover)
{
    // below the crossover SOS runs recdbl_sw; the one-round gather form gives the same
    // bits with fewer exchange rounds
    if (alg == SOSX_ALG_AUTO) return bytes < crossover ? SOSX_ALG_RECDBL_GATHER : SOSX_ALG_RING;
    return alg;
}

int build(int alg, int P, int me, uint64_t count, uint64_t ts, unsigned src_mis,
          unsigned dst_mis, Plan *out)
{
    if (!out || P < 1 || me < 0 || me >= P || ts == 0) return SOSX_ERR_ARG;
    out->alg = alg;
    out->rounds.clear();
    out->scratch_bytes = 0;
    out->reads_src = out->writes_dst = true;
    out->scr_sent = false;
    if (count == 0) return SOSX_OK;
    if (is_bcast(alg))
        return build_bcast((alg - PLAN_BCAST) >> 1, (alg - PLAN_BCAST) & 1, P, me, count, ts, out);
    if (is_scan(alg) && P == 1) {
        // PE_size 1: inscan copies, exscan zeroes (src/collectives.c:1145-1166)
        Round r;
        Local l;
        memset(&l, 0, sizeof(l));
        l.kind = alg == PLAN_EXSCAN ? ZERO : COPY;
        l.out_buf = DST;
        l.nin = alg == PLAN_EXSCAN ? 0 : 1;
        l.in_buf[0] = SRC;
        l.count = count * ts;
        r.ops.push_back(l);
        out->rounds.push_back(r);
        out->reads_src = alg != PLAN_EXSCAN;
        return SOSX_OK;
    }
    if (is_scan(alg)) return build_scan(alg == PLAN_EXSCAN, P, me, count, ts, src_mis, dst_mis, out);
    if (P == 1) {
        // PE_size == 1: the reference copies source to target (src/collectives.c:664-668)
        Round r;
        Local l;
        memset(&l, 0, sizeof(l));
        l.kind = COPY;
        l.out_buf = DST;
        l.nin = 1;
        l.in_buf[0] = SRC;
        l.count = count * ts;
        r.ops.push_back(l);
        out->rounds.push_back(r);
        return SOSX_OK;
    }
    switch (alg) {
        case SOSX_ALG_RING:
        case SOSX_ALG_RECDBL_DIRECT:
            return build_direct(alg, P, me, count, ts, src_mis, dst_mis, out);
        case SOSX_ALG_RECDBL:
            return build_recdbl(P, me, count, ts, dst_mis, out);
        case SOSX_ALG_RECDBL_GATHER:
            return build_recdbl_gather(P, me, count, ts, dst_mis, out);
        case SOSX_ALG_RECHALVING:
            return build_rechalving(P, me, count, ts, dst_mis, out);
        default:
            return SOSX_ERR_ARG;
    }
}

}  // namespace sosplan

// --------------------------------------------------------------------------------
// C ABI: plan introspection (CPU tests simulate every PE's plan against the oracle)
// Encoding (int64 words): [alg, nrounds, scratch_bytes,
//   per round: nx, nops, nx * (send, peer, buf, off, bytes),
//              nops * (kind, order, out_buf, out_off, nin, count, nin * (buf, off),
//                      nout, nout * (buf, off))]
// Returns the number of words (the buffer is filled only if cap >= that), or < 0.
// --------------------------------------------------------------------------------
extern "C" long long sosx_plan_encode(int alg, int P, int me, unsigned long long count,
                                      unsigned long long ts, unsigned src_mis,
                                      unsigned dst_mis, long long *out, unsigned long long cap)
{
    sosplan::Plan p;
    int rc = sosplan::build(alg, P, me, count, ts, src_mis, dst_mis, &p);
    if (rc) return rc;
    std::vector<long long> w;
    w.push_back(p.alg);
    w.push_back((long long)p.rounds.size());
    w.push_back((long long)p.scratch_bytes);
    for (const auto &r : p.rounds) {
        w.push_back((long long)r.xfers.size());
        w.push_back((long long)r.ops.size());
        for (const auto &x : r.xfers) {
            w.push_back(x.send);
            w.push_back(x.peer);
            w.push_back(x.buf);
            w.push_back((long long)x.off);
            w.push_back((long long)x.bytes);
        }
        for (const auto &l : r.ops) {
            w.push_back(l.kind);
            w.push_back(l.order);
            w.push_back(l.out_buf);
            w.push_back((long long)l.out_off);
            w.push_back(l.nin);
            w.push_back((long long)l.count);
            for (int k = 0; k < l.nin; ++k) {
                w.push_back(l.in_buf[k]);
                w.push_back((long long)l.in_off[k]);
            }
            w.push_back(l.kind == sosplan::PREFIX ? l.nout : 0);
            for (int k = 0; l.kind == sosplan::PREFIX && k < l.nout; ++k) {
                w.push_back(l.outs_buf[k]);
                w.push_back((long long)l.outs_off[k]);
            }
        }
    }
    if (out && cap >= w.size()) memcpy(out, w.data(), w.size() * sizeof(long long));
    return (long long)w.size();
}

extern "C" int sosx_resolve_alg(int alg, unsigned long long bytes, unsigned long long crossover)
{
    return sosplan::resolve_alg(alg, bytes, crossover);
}
