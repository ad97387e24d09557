// Host-side check of the plan builder (sos_amd/csrc/plan.cpp) under AddressSanitizer and
// UBSan, built and run by tests/test_plan_bounds.py.
//
// For every schedule (the five reduction algorithms, inscan/exscan, broadcast from
// every root with and without the root copy), team sizes 1..12, 16, 31-33 and 64, ragged counts and element sizes 1..16, and every PE index, it checks
// the invariants the executors rely on when they turn a plan into raw pointers:
//   * every transfer and local operation stays inside its buffer: SRC/DST within
//     count*ts bytes, SCR within the plan's scratch_bytes;
//   * transfers carry > 0 bytes to a valid peer other than the PE itself;
//   * fold/prefix arities are within the kernels' limits;
//   * the sizes PE a sends to PE b, in plan order, equal what b receives from a, in order
//     (FIFO per ordered pair, the matching rule of RCCL and of the p2p counters).
// Prints "plan bounds: N plans OK" or the first violation, exit 0/1.
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <utility>
#include <vector>

#include "plan.h"

using namespace sosplan;

static long g_checked = 0;

static bool fail(const char *what, int alg, int P, int me, unsigned long long n, unsigned long long ts)
{
    fprintf(stderr, "VIOLATION %s: alg %d P %d me %d count %llu ts %llu\n", what, alg, P, me, n, ts);
    return false;
}

static bool in_buf(const Plan &p, int buf, uint64_t off, uint64_t bytes, uint64_t vec_bytes)
{
    const uint64_t lim = buf == SCR ? p.scratch_bytes : vec_bytes;
    return buf >= SRC && buf <= SCR && off <= lim && bytes <= lim - off;
}

static bool check_one(int alg, int P, unsigned long long n, unsigned long long ts, unsigned mis)
{
    std::vector<Plan> plans((size_t)P);
    for (int me = 0; me < P; ++me) {
        if (build(alg, P, me, n, ts, mis, mis, &plans[(size_t)me]) != SOSX_OK)
            return fail("build failed", alg, P, me, n, ts);
        const Plan &p = plans[(size_t)me];
        const uint64_t vb = n * ts;
        for (const Round &r : p.rounds) {
            for (const Xfer &x : r.xfers) {
                if (x.bytes == 0) return fail("empty transfer", alg, P, me, n, ts);
                if (x.peer < 0 || x.peer >= P || x.peer == me) return fail("bad peer", alg, P, me, n, ts);
                if (!in_buf(p, x.buf, x.off, x.bytes, vb)) return fail("transfer out of bounds", alg, P, me, n, ts);
            }
            for (const Local &l : r.ops) {
                const bool typed = l.kind == FOLD || l.kind == PREFIX;
                const uint64_t bytes = typed ? l.count * ts : l.count;
                if (l.kind == FOLD && (l.nin < 1 || l.nin > SOSX_MAX_FOLD))
                    return fail("fold arity", alg, P, me, n, ts);
                if (l.kind == PREFIX && (l.nin < 1 || l.nin > PLAN_MAX_PE || l.nout != l.nin))
                    return fail("prefix arity", alg, P, me, n, ts);
                if (l.kind == PREFIX) {
                    for (int k = 0; k < l.nout; ++k)
                        if (!in_buf(p, l.outs_buf[k], l.outs_off[k], bytes, vb))
                            return fail("prefix output out of bounds", alg, P, me, n, ts);
                } else if (!in_buf(p, l.out_buf, l.out_off, bytes, vb)) {
                    return fail("op output out of bounds", alg, P, me, n, ts);
                }
                const int nin = l.kind == ZERO ? 0 : l.nin;
                for (int k = 0; k < nin; ++k)
                    if (!in_buf(p, l.in_buf[k], l.in_off[k], bytes, vb))
                        return fail("op input out of bounds", alg, P, me, n, ts);
            }
        }
    }
    // pairwise agreement, FIFO per ordered pair as RCCL and the p2p counters match them:
    // the sizes a sends b, in plan order, equal the sizes b receives from a, in order
    std::map<std::pair<int, int>, std::vector<uint64_t>> sent, recv;
    for (int me = 0; me < P; ++me)
        for (const Round &r : plans[(size_t)me].rounds)
            for (const Xfer &x : r.xfers)
                (x.send ? sent[{me, x.peer}] : recv[{x.peer, me}]).push_back(x.bytes);
    if (sent != recv) return fail("send/receive mismatch", alg, P, -1, n, ts);
    ++g_checked;
    return true;
}

int main()
{
    const unsigned long long counts[] = {1, 2, 3, 7, 8, 63, 64, 65, 1000, 4097};
    const unsigned long long sizes[] = {1, 2, 4, 8, 16};
    const int teams[] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 11, 12, 16, 31, 32, 33, 64};
    bool ok = true;
    for (int P : teams) {
        if (!ok) break;
        std::vector<int> algs;
        if (P <= SOSX_MAX_FOLD) {
            const int red[] = {SOSX_ALG_RECDBL, SOSX_ALG_RING, SOSX_ALG_RECHALVING,
                               SOSX_ALG_RECDBL_DIRECT, SOSX_ALG_RECDBL_GATHER};
            if (P <= 8 || P == 16 || P == 64) algs.insert(algs.end(), red, red + 5);
        }
        algs.push_back(PLAN_INSCAN);
        algs.push_back(PLAN_EXSCAN);
        for (int root = 0; root < P; root += (P > 9 ? 7 : 1)) {
            algs.push_back(bcast_alg(root, false));
            algs.push_back(bcast_alg(root, true));
        }
        for (int alg : algs)
            for (unsigned long long n : counts)
                for (unsigned long long ts : sizes)
                    for (unsigned mis : {0u, 4u})
                        if (ok) ok = check_one(alg, P, n, ts, mis);
    }
    if (!ok) return 1;
    printf("plan bounds: %ld plans OK\n", g_checked);
    return 0;
}
