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
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "sosx.h"

namespace sosplan {

enum Buf : int { SRC = 0, DST = 1, SCR = 2 };
enum Kind : int { FOLD = 0, COPY = 1 };

struct Xfer {
    int send;        // 1 = send to peer, 0 = receive from peer
    int peer;        // team index
    int buf;         // Buf
    uint64_t off;    // byte offset into buf
    uint64_t bytes;  // > 0
};

struct Local {
    int kind;        // FOLD: out = fold_order(ins[0..nin)) over `count` elements
    int order;       // COPY: copy `count` bytes from ins[0] to out
    int out_buf;
    uint64_t out_off;
    int nin;
    int in_buf[SOSX_MAX_FOLD];
    uint64_t in_off[SOSX_MAX_FOLD];
    uint64_t count;
};

struct Round {
    std::vector<Xfer> xfers;
    std::vector<Local> ops;
};

struct Plan {
    int alg = 0;
    std::vector<Round> rounds;
    uint64_t scratch_bytes = 0;
};

// SOS ring chunk c of `count` elements over P PEs (src/collectives.c:697-709).
void ring_chunk(uint64_t count, int P, int c, uint64_t *n, uint64_t *first);

// Build the plan of team index `me` (0 <= me < P, 2 <= P <= SOSX_MAX_FOLD for the
// direct schedules).  src_mis/dst_mis = caller pointer addresses mod 16, so scratch
// slots can be placed 16-B congruent with the caller's chunks (vector path).
// Returns SOSX_OK or SOSX_ERR_ARG.
int build(int alg, int P, int me, uint64_t count, uint64_t ts, unsigned src_mis,
          unsigned dst_mis, Plan *out);

// Resolve SOSX_ALG_AUTO the way SOS AUTO does without NIC atomics
// (src/shmem_collectives.h:180-199): recdbl below `crossover` bytes, else ring.
int resolve_alg(int alg, uint64_t bytes, uint64_t crossover);

}  // namespace sosplan
