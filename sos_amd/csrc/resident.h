// resident.h -- the resident small-collective executor's shared words (smallpath.cpp on
// the host, k_resident in small.hip on the GPU).
//
// A launch + completion wait costs 10-13 us on MI355X whatever the wait primitive
// (profiles/r5_sync_cost.json); a request/answer round trip through a kernel that stays
// resident and polls pinned host memory costs 1.7 us (profiles/r5_resident.txt).  With
// SHMEMX_SMALL_RESIDENT=1 the small shared-memory path's recdbl_sw folds and linear folds
// (scans, broadcasts), the staging of device operands into their slots, and
// shmemx_reduce_local's small combines run on such a kernel: one per (type, op) used, one workgroup, launched on the first request
// and exiting on its own after SHMEMX_SMALL_RESIDENT_IDLE_US of idleness (default 2000)
// or at shmem_finalize.  Measured gain at P = 2 / 4 on one GPU: 0.5-2 us of a 10-13 us
// call -- the request's host-link round trips (descriptor, slots, result + fence) cost
// what the launch saved -- so it stays opt-in (profiles/r5_resident.txt).
//
// Protocol (every word in pinned, coherent host memory):
//   host  : write the descriptor d, then req = k (release);
//   kernel: req > last -> copy d (after the acquire), compute, fence at system scope,
//           done = k (release); exits on stop or idleness, storing exited = 1 last;
//   host  : wait for done >= k; a kernel seen exited with done < k is relaunched (the new
//           one reads done at start and takes request k), so a request is never lost to
//           an idle exit racing the host's post.
#pragma once
#include <stdint.h>

#define SOSX_RESIDENT_FOLD 0    /* recdbl_sw tree over np leaves (+ extras): k_small_fold's value */
#define SOSX_RESIDENT_LINEAR 1  /* in[0] OP in[1] ... OP in[np-1]: k_small_ring's single chunk */
#define SOSX_RESIDENT_STAGE 2   /* stage_bytes stage_src -> stage_dst (a device operand into its slot),
                                   a system-scope fence, then *post_word[k] = post_val[k], k < nposts
                                   (the posts): k_small_stage's work */
#define SOSX_RESIDENT_STAGE_FOLD 3  /* STAGE, then for each team member i < npeers wait until
                                   *wait_word[i] >= wait_val[i] (bounded by `limit` ticks), take its
                                   slot slot[i][*ring_word[i]] (wait_word null: slot[i][0], the PE's
                                   own), and FOLD over leaves leaf_idx[y] (+ extras extra_idx[y] >= 0)
                                   of those: the device-operand recdbl_sw call in one request */
#define SOSX_RESIDENT_MAX_BYTES 4096   /* one pass of the workgroup (256 lanes x 16 B); larger calls launch */

struct SosxResidentDesc {
    uint32_t kind;
    uint32_t np;                 /* leaves (FOLD: 1, 2, 4, 8) or inputs (LINEAR: 1..8) */
    uint64_t count;              /* fold elements, count * size <= SOSX_RESIDENT_MAX_BYTES */
    void *out;
    const void *in[8];
    const void *extra[8];        /* FOLD: null where the leaf has no extra PE */
    uint32_t vec;                /* every fold operand 16-B aligned: 16-B vectors per lane */
    uint32_t nposts;
    /* STAGE / STAGE_FOLD */
    const void *stage_src;
    void *stage_dst;
    uint64_t stage_bytes;
    uint32_t stage_vec;
    uint32_t npeers;
    uint64_t *post_word[8];      /* device views */
    uint64_t post_val[8];
    /* STAGE_FOLD */
    const uint64_t *wait_word[8];
    uint64_t wait_val[8];
    const uint32_t *ring_word[8];
    const void *slot[8][2];
    int8_t leaf_idx[8];
    int8_t extra_idx[8];         /* -1: none */
    long long limit;
};

#ifdef __cplusplus
/* k_resident copies the descriptor one 8-byte word per lane of its 256-lane workgroup */
static_assert(sizeof(struct SosxResidentDesc) % 8 == 0, "descriptor: whole 8-byte words");
static_assert(sizeof(struct SosxResidentDesc) / 8 <= 256, "descriptor: one word per lane");
#endif

struct SosxResidentCtl {
    uint64_t req;
    uint64_t done;
    uint64_t stop;
    uint64_t exited;
    uint64_t err;                /* a STAGE_FOLD wait timed out (the host turns it into an error) */
    uint64_t pad[3];
    struct SosxResidentDesc d;
};

#ifdef __cplusplus
extern "C" {
#endif
/* Launch the resident executor of (op, dtype) on `stream` over `ctl` (device view of
 * pinned host memory): one workgroup, until ctl->stop or `idle_ticks` device wall-clock
 * ticks without a request. */
int sosx_resident_launch(int op, int dtype, struct SosxResidentCtl *ctl, long long idle_ticks, void *stream);
#ifdef __cplusplus
}
#endif
