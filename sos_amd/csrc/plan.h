// plan.h -- per-PE execution plans for the SOS team reduction (pure host code).
//
// A plan is what ONE PE (team index `me` of `P`) does for one
// shmem_internal_op_to_all call: a list of rounds, each a group of point-to-point
// transfers with team peers (carried by RCCL ncclSend/ncclRecv inside one
// ncclGroupStart/End, or by the loopback transport in tests) followed by local
// device operations (fused folds / copies) on the same stream.  Buffers are named,
// not addressed: SRC (the caller's source), DST (the caller's target) and SCR (the
// library's device scratch), so the same plan drives the RCCL executor, the
// single-GPU loopback executor and the CPU test simulators.
//
// Schedules (SOS references):
//   RING          bit-exact with SOS ring (src/collectives.c:647-764, SOS AUTO at
//                 >= 16 KiB): every element of ring chunk c is folded
//                 ((s_c OP s_c+1) OP ...) OP s_c-1, left operand the running partial.
//                 The bytes move by a DIRECT exchange (each PE sends chunk q to PE q
//                 over its own xGMI link, all P-1 links at once), the owner folds its
//                 chunk in one fused pass, then a direct allgather.
//   RECDBL        SOS recdbl_sw butterfly (src/collectives.c:850-984) step for step:
//                 full vector per step, current = current OP peer; per-PE exact.
//   RECHALVING    recursive halving (distance 1, 2, 4, ...) + recursive doubling:
//                 the recdbl_sw tree, each element finished by one PE in its own
//                 perspective; 2(P-1)/P of the vector on the wire instead of log2(P).
//   RECDBL_DIRECT the recdbl_sw tree evaluated by the chunk owner after a direct
//                 exchange (all links at once), then a direct allgather.
//   INSCAN/EXSCAN the team prefix ((s_0 OP s_1) OP ...) OP s_i of SOS scan_ring
//                 (src/collectives.c:1111-1209: PE_start's put, then PE 1, 2, ... apply
//                 target = target OP source in turn), computed chunk-wise: PE c gathers
//                 ring chunk c of every source, one fused PREFIX pass produces chunk c of
//                 all P results, and a direct all-to-all returns them (2(P-1)/P of the
//                 vector on every link instead of SOS's P-1 sequential atomic puts).
//   BCAST         root -> all (src/collectives.c:429-485); large payloads as a
//                 scatter of P-1 chunks to the non-roots + their direct allgather.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "sosx.h"

namespace sosplan {

enum Buf : int { SRC = 0, DST = 1, SCR = 2 };
// FOLD:   out = fold_order(ins[0..nin))                         (count elements)
// COPY:   out = ins[0]                                          (count bytes)
// PREFIX: outs[k] = ins[0] OP ... OP ins[k], k < nin            (count elements)
// ZERO:   out = all-zero bytes                                  (count bytes)
enum Kind : int { FOLD = 0, COPY = 1, PREFIX = 2, ZERO = 3 };

// Non-reduction collectives share the plan machinery; their "algorithm" ids sit
// above the SOSX_ALG_* range.  Broadcast: PLAN_BCAST + 2*root + copy_root.
constexpr int PLAN_INSCAN = 16;
constexpr int PLAN_EXSCAN = 17;
constexpr int PLAN_BCAST = 32;
constexpr int PLAN_MAX_PE = 64;   // inputs of one local op: SOSX_MAX_FOLD folds, scan prefixes
inline bool is_scan(int alg) { return alg == PLAN_INSCAN || alg == PLAN_EXSCAN; }
inline bool is_bcast(int alg) { return alg >= PLAN_BCAST; }
inline int bcast_alg(int root, bool copy_root) { return PLAN_BCAST + 2 * root + (copy_root ? 1 : 0); }

struct Xfer {
    int send;        // 1 = send to peer, 0 = receive from peer
    int peer;        // team index
    int buf;         // Buf
    uint64_t off;    // byte offset into buf
    uint64_t bytes;  // > 0
};

struct Local {
    int kind;        // Kind
    int order;       // FOLD: SOSX_ORDER_*
    int out_buf;     // FOLD/COPY/ZERO output (PREFIX: outs[0])
    uint64_t out_off;
    int nin;         // FOLD: <= SOSX_MAX_FOLD; PREFIX: <= PLAN_MAX_PE
    int in_buf[PLAN_MAX_PE];
    uint64_t in_off[PLAN_MAX_PE];
    uint64_t count;
    int nout;        // PREFIX: one output per input (outs[0] == out)
    int outs_buf[PLAN_MAX_PE];
    uint64_t outs_off[PLAN_MAX_PE];
    int own;         // PREFIX: input that may alias an output (read before any store), or -1
};

struct Round {
    std::vector<Xfer> xfers;
    std::vector<Local> ops;
};

struct Plan {
    int alg = 0;
    std::vector<Round> rounds;
    uint64_t scratch_bytes = 0;
    bool reads_src = true;     // false: a broadcast non-root never reads its source
    bool writes_dst = true;    // false: a broadcast root without copy leaves its target
    bool scr_sent = false;     // true: some transfer sends out of SCR (scans)
};

// Largest power of two <= P (src/collectives.c:878-882).
int pow2_floor(int P);

// SOS ring chunk c of `count` elements over P PEs (src/collectives.c:697-709).
void ring_chunk(uint64_t count, int P, int c, uint64_t *n, uint64_t *first);

// Build the plan of team index `me` (0 <= me < P, 2 <= P <= SOSX_MAX_FOLD for the
// direct reduction schedules, P <= PLAN_MAX_PE for scans).  `alg` is a SOSX_ALG_*
// (reduction), PLAN_INSCAN / PLAN_EXSCAN (sum scans, SOS src/collectives.c:1111-1209)
// or bcast_alg(root, copy_root) (src/collectives.c:429-551 bcast_linear/tree).  src_mis/dst_mis = caller pointer addresses mod 16, so scratch
// slots can be placed 16-B congruent with the caller's chunks (vector path).
// Returns SOSX_OK or SOSX_ERR_ARG.
int build(int alg, int P, int me, uint64_t count, uint64_t ts, unsigned src_mis,
          unsigned dst_mis, Plan *out);

// Resolve SOSX_ALG_AUTO the way SOS AUTO does without NIC atomics
// (src/shmem_collectives.h:180-199): recdbl below `crossover` bytes, else ring.
int resolve_alg(int alg, uint64_t bytes, uint64_t crossover);

}  // namespace sosplan
