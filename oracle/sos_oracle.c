/*
 * sos_oracle.c -- CPU restatement of the Sandia OpenSHMEM (SOS v1.5.3) team-reduction
 * path, used ONLY as test infrastructure.
 *
 *   *** TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
 *   *** cpu_baseline leg may load this library, and only as the checker / the timed
 *   *** CPU baseline.  The product (sos_amd/libsos_amd.so) never links or calls it.
 *
 * Parity pinning: the reference's combine header cannot be compiled from its own
 * sources here (src/shmem_internal_op.h -> transport.h -> transport_none.h ->
 * shmem_internal.h needs configure-generated config.h and m4-generated shmemx.h), so
 * oracle/_ref is not built.  This file restates the same C expressions, compiled by
 * the same gcc with SOS's default flags (-std=gnu11 -O2), and is pinned by the
 * known-answer tests listed in SURVEY.md 8(c) (examples/pi_reduce.c outputs) and the
 * man/shmem_reductions.3 example, evaluated in tests/test_oracle_kat.py.
 *
 * Contents
 *   oracle_reduce_local  -- src/shmem_internal_op.h:305-339 (+ FUNC_OP_CREATE :23-33,
 *                           op macros :37-43, dtype classes :225-303)
 *   oracle_ring          -- src/collectives.c:647-764 (P PEs simulated in one process)
 *   oracle_recdbl        -- src/collectives.c:850-984 (P PEs simulated in one process)
 *   oracle_scan          -- src/collectives.c:1111-1209 (inscan / exscan, P PEs)
 *   oracle_bcast         -- src/collectives.c:429-485 + src/collectives_c.c4:342-429
 *   oracle_*_time        -- single-core timing helpers for bench.py's cpu_baseline
 *   oracle_pe_ring       -- src/collectives.c:647-764 as ONE PE of a real P-process job
 *                           over a shared segment (bench.py N > 1 cpu_baseline)
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <complex.h>

/* shm_internal_op_t, src/transport_none.h:25-33 */
enum { O_BAND = 0, O_BOR, O_BXOR, O_MIN, O_MAX, O_SUM, O_PROD };

/* shm_internal_datatype_t, src/transport.h:19-49 */
enum {
    D_SIGNED_BYTE = 0, D_CHAR, D_SCHAR, D_SHORT, D_INT, D_LONG, D_LONG_LONG,
    D_FORTRAN_INTEGER, D_INT8, D_INT16, D_INT32, D_INT64, D_PTRDIFF_T, D_UCHAR,
    D_USHORT, D_UINT, D_ULONG, D_ULONG_LONG, D_UINT8, D_UINT16, D_UINT32, D_UINT64,
    D_SIZE_T, D_FLOAT, D_DOUBLE, D_LONG_DOUBLE, D_FLOAT_COMPLEX, D_DOUBLE_COMPLEX,
    D_COUNT
};

/* Elementwise loop: out = calc(out, in), left operand is the in/out buffer
 * (src/shmem_internal_op.h:23-33). */
#define O_MAXF(a, b) ((a) > (b) ? (a) : (b))
#define O_MINF(a, b) ((a) < (b) ? (a) : (b))
#define O_SUMF(a, b) ((a) + (b))
#define O_PRODF(a, b) ((a) * (b))
#define O_ANDF(a, b) ((a) & (b))
#define O_ORF(a, b) ((a) | (b))
#define O_XORF(a, b) ((a) ^ (b))

#define O_LOOP(ctype, calc)                                           \
    do {                                                              \
        ctype *o_ = (ctype *) inout;                                  \
        const ctype *i_ = (const ctype *) in;                         \
        for (int k_ = 0; k_ < count; ++k_) o_[k_] = calc(o_[k_], i_[k_]); \
    } while (0)

/* op classes of src/shmem_internal_op.h:225-303 */
#define O_CASE_FP(ctype)                                   \
    switch (op) {                                          \
        case O_MIN: O_LOOP(ctype, O_MINF); return 0;       \
        case O_MAX: O_LOOP(ctype, O_MAXF); return 0;       \
        case O_SUM: O_LOOP(ctype, O_SUMF); return 0;       \
        case O_PROD: O_LOOP(ctype, O_PRODF); return 0;     \
        default: return -2;                                \
    }
#define O_CASE_CPLX(ctype)                                 \
    switch (op) {                                          \
        case O_SUM: O_LOOP(ctype, O_SUMF); return 0;       \
        case O_PROD: O_LOOP(ctype, O_PRODF); return 0;     \
        default: return -2;                                \
    }
#define O_CASE_INT(ctype)                                  \
    switch (op) {                                          \
        case O_MIN: O_LOOP(ctype, O_MINF); return 0;       \
        case O_MAX: O_LOOP(ctype, O_MAXF); return 0;       \
        case O_SUM: O_LOOP(ctype, O_SUMF); return 0;       \
        case O_PROD: O_LOOP(ctype, O_PRODF); return 0;     \
        case O_BAND: O_LOOP(ctype, O_ANDF); return 0;      \
        case O_BOR: O_LOOP(ctype, O_ORF); return 0;        \
        case O_BXOR: O_LOOP(ctype, O_XORF); return 0;      \
        default: return -2;                                \
    }

/* Returns 0, -1 for an invalid datatype (RAISE_ERROR_MSG "invalid data type"),
 * -2 for an op the datatype's class does not support (RAISE_ERROR_STR
 * "unsupported reduction on ..."). `count` is int, as in the reference. */
int oracle_reduce_local(int op, int dt, int count, const void *in, void *inout)
{
    switch (dt) {
        case D_CHAR: O_CASE_FP(char);
        case D_SCHAR: O_CASE_FP(signed char);
        case D_SHORT: O_CASE_INT(short);
        case D_INT: O_CASE_INT(int);
        case D_LONG: O_CASE_INT(long);
        case D_LONG_LONG: O_CASE_INT(long long);
        case D_PTRDIFF_T: O_CASE_FP(ptrdiff_t);
        case D_UCHAR: O_CASE_INT(unsigned char);
        case D_USHORT: O_CASE_INT(unsigned short);
        case D_UINT: O_CASE_INT(unsigned int);
        case D_ULONG: O_CASE_INT(unsigned long);
        case D_ULONG_LONG: O_CASE_INT(unsigned long long);
        case D_INT8: O_CASE_INT(int8_t);
        case D_INT16: O_CASE_INT(int16_t);
        case D_INT32: O_CASE_INT(int32_t);
        case D_INT64: O_CASE_INT(int64_t);
        case D_UINT8: O_CASE_INT(uint8_t);
        case D_UINT16: O_CASE_INT(uint16_t);
        case D_UINT32: O_CASE_INT(uint32_t);
        case D_UINT64: O_CASE_INT(uint64_t);
        case D_SIZE_T: O_CASE_INT(size_t);
        case D_FLOAT: O_CASE_FP(float);
        case D_DOUBLE: O_CASE_FP(double);
        case D_LONG_DOUBLE: O_CASE_FP(long double);
        case D_FLOAT_COMPLEX: O_CASE_CPLX(float _Complex);
        case D_DOUBLE_COMPLEX: O_CASE_CPLX(double _Complex);
        default: return -1;
    }
}

/* sizeof the C type behind each datatype on x86-64 (0 = not reducible). */
size_t oracle_type_size(int dt)
{
    static const size_t sz[D_COUNT] = {
        0, 1, 1, 2, 4, 8, 8, 0, 1, 2, 4, 8, 8, 1, 2, 4, 8, 8, 1, 2, 4, 8, 8, 4, 8,
        sizeof(long double), 8, 16 };
    return (dt >= 0 && dt < D_COUNT) ? sz[dt] : 0;
}

/* ------------------------------------------------------------------------------
 * Ring all-reduce, src/collectives.c:647-764, with P PEs simulated in order.
 * src[p] / dst[p] are PE p's source and target buffers (dst[p] == src[p] means an
 * in-place call, handled by the tmp copy of :672-683).  The simulation runs each
 * step's puts for every PE, then each PE's combine: the pSync waits of :717-722 make
 * every PE's step-i combine depend only on the step-i put from its left neighbour.
 * ------------------------------------------------------------------------------ */
static void ring_chunk(size_t count, int P, size_t c, size_t ts, size_t *n, size_t *disp)
{
    /* chunk math, src/collectives.c:697-709 */
    size_t extra = c < count % (size_t) P;
    size_t cnt = count / (size_t) P + extra;
    *n = cnt;
    *disp = extra ? c * cnt * ts : (c * cnt + count % (size_t) P) * ts;
}

int oracle_ring(int P, size_t count, int op, int dt, void **src, void **dst)
{
    size_t ts = oracle_type_size(dt);
    if (!ts) return -1;
    if (count == 0) return 0;
    if (P == 1) {   /* :664-668 */
        if (dst[0] != src[0]) memcpy(dst[0], src[0], count * ts);
        return 0;
    }
    void **s = malloc(sizeof(void *) * P);
    int *tmp = calloc(P, sizeof(int));
    for (int p = 0; p < P; p++) {
        s[p] = src[p];
        if (dst[p] == src[p]) {  /* :672-683 */
            s[p] = malloc(count * ts);
            memcpy(s[p], dst[p], count * ts);
            tmp[p] = 1;
        }
    }
    int rc = 0;
    /* reduce-scatter, :693-727 */
    for (int i = 0; i < P - 1; i++) {
        for (int r = 0; r < P; r++) {
            int peer = (r + 1) % P;
            size_t chunk_out = (size_t) ((r - i + P) % P), n, disp;
            ring_chunk(count, P, chunk_out, ts, &n, &disp);
            memcpy((uint8_t *) dst[peer] + disp,
                   i == 0 ? (uint8_t *) s[r] + disp : (uint8_t *) dst[r] + disp, n * ts);
        }
        for (int r = 0; r < P; r++) {
            size_t chunk_in = (size_t) ((r - i - 1 + P) % P), n, disp;
            ring_chunk(count, P, chunk_in, ts, &n, &disp);
            rc |= oracle_reduce_local(op, dt, (int) n, (uint8_t *) s[r] + disp,
                                      (uint8_t *) dst[r] + disp);
        }
    }
    /* all-gather, :737-756 */
    for (int i = 0; i < P - 1; i++) {
        for (int r = 0; r < P; r++) {
            int peer = (r + 1) % P;
            size_t chunk_out = (size_t) ((r + 1 - i + P) % P), n, disp;
            ring_chunk(count, P, chunk_out, ts, &n, &disp);
            memcpy((uint8_t *) dst[peer] + disp, (uint8_t *) dst[r] + disp, n * ts);
        }
    }
    for (int p = 0; p < P; p++) if (tmp[p]) free(s[p]);
    free(s);
    free(tmp);
    return rc;
}

/* ------------------------------------------------------------------------------
 * Recursive doubling all-reduce, src/collectives.c:850-984, P PEs simulated.
 * Each PE works on a private copy (current_target, :860/:888) and receives the
 * peer's full vector into its target (:936-959), then
 * reduce_local(in = target, inout = current_target) (:961-962): own value is the
 * left operand.  Non-power-of-two P: PEs >= pow2 fold into PE (id - pow2) first
 * (:905-926) and receive the final vector from it at the end (:966-975).
 * ------------------------------------------------------------------------------ */
int oracle_recdbl(int P, size_t count, int op, int dt, void **src, void **dst)
{
    size_t ts = oracle_type_size(dt), bytes;
    if (!ts) return -1;
    bytes = count * ts;
    if (P == 1) {
        if (dst[0] != src[0]) memcpy(dst[0], src[0], bytes);
        return 0;
    }
    if (count == 0) return 0;
    int pow2 = 2, log2p = 1, i = P >> 1;
    while (i != 1) { i >>= 1; pow2 <<= 1; log2p++; }   /* :878-882 */
    /* The loop above yields pow2 = largest power of two <= P for P >= 2. */
    void **cur = malloc(sizeof(void *) * P);
    for (int p = 0; p < P; p++) { cur[p] = malloc(bytes); memcpy(cur[p], src[p], bytes); }
    int rc = 0;
    /* extra-peer fold, :905-926 */
    for (int p = pow2; p < P; p++) {
        int partner = p - pow2;
        memcpy(dst[partner], cur[p], bytes);
        rc |= oracle_reduce_local(op, dt, (int) count, dst[partner], cur[partner]);
    }
    /* pairwise exchange, :932-963 */
    for (int s = 0; s < log2p; s++) {
        for (int r = 0; r < pow2; r++) memcpy(dst[r ^ (1 << s)], cur[r], bytes);
        for (int r = 0; r < pow2; r++)
            rc |= oracle_reduce_local(op, dt, (int) count, dst[r], cur[r]);
    }
    /* final result to the extra peers, :966-975; memcpy(target, current), :977 */
    for (int p = pow2; p < P; p++) memcpy(dst[p], cur[p - pow2], bytes);
    for (int r = 0; r < pow2; r++) memcpy(dst[r], cur[r], bytes);
    for (int p = 0; p < P; p++) free(cur[p]);
    free(cur);
    return rc;
}

/* ------------------------------------------------------------------------------
 * Team prefix scans, src/collectives.c:1111-1209 (scan_ring).  In-place calls work on
 * a copy of the source (:1123-1134).  PE_start zeroes its own target for exscan
 * (:1145-1155) and puts its source into the targets of team PEs exclusive..P-1
 * (:1158-1166); then PE 1, 2, ... in turn (each waits for its left neighbour's
 * pSync, :1181-1185) apply target = target OP source -- shmem_internal_atomicv, the
 * running target is the left operand -- to the targets of PEs i+exclusive..P-1
 * (:1188-1196).  scan_linear (:991-1108) posts the same atomics without the ordering;
 * its result is this one whenever OP is associative and commutative on the values.
 * ------------------------------------------------------------------------------ */
int oracle_scan(int P, size_t count, int op, int dt, int exclusive, void **src, void **dst)
{
    size_t ts = oracle_type_size(dt), bytes;
    if (!ts) return -1;
    if (count == 0) return 0;
    bytes = count * ts;
    void **in = malloc(sizeof(void *) * P);
    for (int p = 0; p < P; p++) { in[p] = malloc(bytes); memcpy(in[p], src[p], bytes); }
    if (exclusive) memset(dst[0], 0, bytes);
    for (int i = exclusive; i < P; i++) memcpy(dst[i], in[0], bytes);
    int rc = 0;
    for (int pe = 1; pe < P; pe++)
        for (int i = pe + exclusive; i < P; i++)
            rc |= oracle_reduce_local(op, dt, (int) count, in[pe], dst[i]);
    for (int p = 0; p < P; p++) free(in[p]);
    free(in);
    return rc;
}

/* ------------------------------------------------------------------------------
 * Broadcast, src/collectives.c:429-485 (bcast_linear; bcast_tree :489-551 moves the
 * same bytes): every non-root target receives the root's source.  The team forms
 * (shmem_broadcastmem / shmem_<T>_broadcast, src/collectives_c.c4:380-429) also copy
 * source to dest on the root; the active-set shmem_broadcast32/64 (:342-378) do not.
 * ------------------------------------------------------------------------------ */
int oracle_bcast(int P, size_t bytes, int root, int copy_root, void **src, void **dst)
{
    if (root < 0 || root >= P) return -3;
    for (int p = 0; p < P; p++) {
        if (p == root) {
            if (copy_root && dst[p] != src[p]) memcpy(dst[p], src[p], bytes);
        } else {
            memcpy(dst[p], src[root], bytes);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------
 * Timing helpers for bench.py's cpu_baseline (single core, CLOCK_MONOTONIC as
 * shmem_internal_wtime, src/shmem_internal.h:549-565).
 * ------------------------------------------------------------------------------ */
static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

/* Runs reduce_local `reps` times over (in, inout) and returns total seconds. */
double oracle_time_reduce_local(int op, int dt, int count, const void *in, void *inout, int reps)
{
    double t0 = now_s();
    for (int r = 0; r < reps; r++) oracle_reduce_local(op, dt, count, in, inout);
    return now_s() - t0;
}

/* ------------------------------------------------------------------------------
 * Synthetic inputs: splitmix64 of (seed, pe, i), the CPU twin of
 * sosx_fill (sos_amd/csrc/kernels.hip).  Values are built from bits or by exact
 * dyadic arithmetic so both sides agree bit for bit.
 * dist 0: fp uniform [-1,1), ints full-range; dist 1: fp [0.5,2) (complex parts
 * +-[0.5,1)), ints [-3,3].
 * ------------------------------------------------------------------------------ */
static uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static float f32_of(uint64_t h, int dist, int cplx)
{
    if (dist == 1) {
        uint32_t bits = cplx ? (((uint32_t) (h >> 63) << 31) | (126u << 23) | (uint32_t) (h & 0x7FFFFFu))
                             : (((126u + (uint32_t) (h >> 63)) << 23) | (uint32_t) (h & 0x7FFFFFu));
        float f;
        memcpy(&f, &bits, 4);
        return f;
    }
    return (float) (uint32_t) (h >> 40) * 0x1p-23f - 1.0f;
}

static double f64_of(uint64_t h, int dist, int cplx)
{
    if (dist == 1) {
        uint64_t bits = cplx ? (((h >> 63) << 63) | (1022ull << 52) | (h & 0xFFFFFFFFFFFFFull))
                             : (((1022ull + (h >> 63)) << 52) | (h & 0xFFFFFFFFFFFFFull));
        double d;
        memcpy(&d, &bits, 8);
        return d;
    }
    return (double) (h >> 11) * 0x1p-52 - 1.0;
}

int oracle_fill(int dt, int dist, uint64_t seed, int pe, void *dst, size_t count, size_t index0)
{
    size_t ts = oracle_type_size(dt);
    if (!ts || dt == D_LONG_DOUBLE) return -1;
    const uint64_t key = mix64(seed ^ ((uint64_t) (uint32_t) pe << 40));
    for (size_t j = 0; j < count; j++) {
        uint64_t i = index0 + j;
        switch (dt) {
            case D_FLOAT: ((float *) dst)[j] = f32_of(mix64(key ^ i), dist, 0); break;
            case D_DOUBLE: ((double *) dst)[j] = f64_of(mix64(key ^ i), dist, 0); break;
            case D_FLOAT_COMPLEX:
                ((float *) dst)[2 * j] = f32_of(mix64(key ^ (2 * i)), dist, 1);
                ((float *) dst)[2 * j + 1] = f32_of(mix64(key ^ (2 * i + 1)), dist, 1);
                break;
            case D_DOUBLE_COMPLEX:
                ((double *) dst)[2 * j] = f64_of(mix64(key ^ (2 * i)), dist, 1);
                ((double *) dst)[2 * j + 1] = f64_of(mix64(key ^ (2 * i + 1)), dist, 1);
                break;
            default: {
                uint64_t h = mix64(key ^ i);
                uint64_t v = dist == 1 ? (uint64_t) ((int64_t) (h % 7u) - 3) : h;
                memcpy((uint8_t *) dst + j * ts, &v, ts);  /* little-endian low bytes */
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------
 * One PE of SOS's ring (src/collectives.c:647-764) run by a real process: the CPU
 * baseline of bench.py's N > 1 line (P single-threaded processes, one
 * core each, shared-memory puts are memcpy as with XPMEM, src/transport_xpmem.h:95).
 *
 * `seg` is a MAP_SHARED segment every PE process maps, laid out as
 *   [header: 64-B lines; line 0 = barrier counter, line 1 + 2p / 2 + 2p = PE p's
 *    pSync[0] / pSync[1]] [PE 0 target][PE 1 target]...  (targets `stride` apart)
 * so a PE's symmetric target and pSync sit at the same offsets in every PE's view.
 * Put + fence + atomic add on the peer's pSync (:711-716 / :744-749) become memcpy
 * into the peer's target, a release fence and an atomic fetch-add; SHMEM_WAIT_UNTIL
 * (:719 / :752) spins on the PE's own pSync.  The source is the PE's private buffer
 * (never the target, so the in-place tmp copy of :672-683 does not arise).
 * ------------------------------------------------------------------------------ */
#define PE_LINE 64
#define PE_SYNC 35   /* SHMEM_REDUCE_SYNC_SIZE words per PE (configure.ac:653-694) */

size_t oracle_pe_header_bytes(int P)
{
    size_t h = (size_t) (1 + PE_SYNC * P) * PE_LINE;
    return (h + 4095) & ~(size_t) 4095;
}

/* PE pe's pSync[k], one 64-B line per word so spinning PEs do not share lines */
static long *pe_psync(void *seg, int pe, int k)
{
    return (long *) ((uint8_t *) seg + (size_t) (1 + PE_SYNC * pe + k) * PE_LINE);
}

static void pe_wait_ge(long *p, long v)
{
    while (__atomic_load_n(p, __ATOMIC_ACQUIRE) < v) __builtin_ia32_pause();
}

/* Sense-free barrier: the epoch-th barrier completes when the counter reaches epoch*P. */
void oracle_pe_barrier(void *seg, int P, long epoch)
{
    long *c = (long *) seg;
    __atomic_fetch_add(c, 1, __ATOMIC_ACQ_REL);
    pe_wait_ge(c, epoch * (long) P);
}

int oracle_pe_ring(void *seg, size_t stride, int P, int me, size_t count, int op, int dt,
                   const void *source)
{
    size_t ts = oracle_type_size(dt);
    if (!ts || me < 0 || me >= P) return -1;
    uint8_t *base = (uint8_t *) seg + oracle_pe_header_bytes(P);
    uint8_t *target = base + (size_t) me * stride;
    if (count == 0) return 0;
    if (P == 1) { memcpy(target, source, count * ts); return 0; }  /* :664-668 */
    int peer = (me + 1) % P;
    uint8_t *peer_target = base + (size_t) peer * stride;
    long *my0 = pe_psync(seg, me, 0), *my1 = pe_psync(seg, me, 1);
    long *peer0 = pe_psync(seg, peer, 0), *peer1 = pe_psync(seg, peer, 1);
    int rc = 0;
    for (int i = 0; i < P - 1; i++) {          /* reduce-scatter, :693-727 */
        size_t out_n, out_d, in_n, in_d;
        ring_chunk(count, P, (size_t) ((me - i + P) % P), ts, &out_n, &out_d);
        ring_chunk(count, P, (size_t) ((me - i - 1 + P) % P), ts, &in_n, &in_d);
        memcpy(peer_target + out_d, i == 0 ? (const uint8_t *) source + out_d : target + out_d,
               out_n * ts);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        __atomic_fetch_add(peer0, 1, __ATOMIC_RELEASE);
        pe_wait_ge(my0, i + 1);
        rc |= oracle_reduce_local(op, dt, (int) in_n, (const uint8_t *) source + in_d, target + in_d);
    }
    __atomic_store_n(my0, 0, __ATOMIC_RELEASE);     /* :730-731 */
    for (int i = 0; i < P - 1; i++) {          /* all-gather, :737-756 */
        size_t out_n, out_d;
        ring_chunk(count, P, (size_t) ((me + 1 - i + P) % P), ts, &out_n, &out_d);
        memcpy(peer_target + out_d, target + out_d, out_n * ts);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        __atomic_fetch_add(peer1, 1, __ATOMIC_RELEASE);
        pe_wait_ge(my1, i + 1);
    }
    __atomic_store_n(my1, 0, __ATOMIC_RELEASE);     /* :759-760 */
    return rc;
}

/* ------------------------------------------------------------------------------
 * One PE of SOS's recdbl_sw (src/collectives.c:850-984) run by a real process: the CPU
 * side of the small-message latency comparison (SOS AUTO below COLL_SIZE_CROSSOVER,
 * src/shmem_collectives.h:192-195).  Same segment layout as oracle_pe_ring.  Puts are
 * memcpy into the peer's target + release fence; put_scalar of the ready flags is an
 * atomic store into the peer's pSync word; SHMEM_WAIT_UNTIL(.., CMP_EQ, v) spins on the
 * PE's own word.  current_target is malloc'd per call, as in the reference (:860).
 * pSync words: [i] step i (:933), [33] the extra-peer word (:862), all reset at :982.
 * ------------------------------------------------------------------------------ */
static void pe_wait_eq(long *p, long v)
{
    while (__atomic_load_n(p, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
}

int oracle_pe_recdbl(void *seg, size_t stride, int P, int me, size_t count, int op, int dt,
                     const void *source)
{
    size_t ts = oracle_type_size(dt);
    if (!ts || me < 0 || me >= P) return -1;
    uint8_t *base = (uint8_t *) seg + oracle_pe_header_bytes(P);
    uint8_t *target = base + (size_t) me * stride;
    const size_t wrk = count * ts;
    const long target_ready = 1, data_ready = 2;
    if (P == 1) { if (count) memcpy(target, source, wrk); return 0; }   /* :865-871 */
    if (count == 0) return 0;                                          /* :873-876 */
    int log2p = 1, pow2 = 2, i = P >> 1;
    while (i != 1) { i >>= 1; pow2 <<= 1; log2p++; }                   /* :878-882 */
    uint8_t *cur = malloc(wrk);                                        /* :860, :888 */
    if (!cur) return -1;
    memcpy(cur, source, wrk);
    long *extra = pe_psync(seg, me, PE_SYNC - 2);                      /* :862 */
    int rc = 0;
    if (me >= pow2) {                                                  /* :905-918 */
        int peer = me - pow2;
        pe_wait_eq(extra, target_ready);
        memcpy(base + (size_t) peer * stride, cur, wrk);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        __atomic_store_n(pe_psync(seg, peer, PE_SYNC - 2), data_ready, __ATOMIC_RELEASE);
        pe_wait_eq(extra, data_ready);
    } else {
        if (me < P - pow2) {                                           /* :920-926 */
            int peer = me + pow2;
            __atomic_store_n(pe_psync(seg, peer, PE_SYNC - 2), target_ready, __ATOMIC_RELEASE);
            pe_wait_eq(extra, data_ready);
            rc |= oracle_reduce_local(op, dt, (int) count, target, cur);
        }
        for (i = 0; i < log2p; i++) {                                  /* :932-963 */
            long *step = pe_psync(seg, me, i);
            int peer = me ^ (1 << i);
            long *peer_step = pe_psync(seg, peer, i);
            uint8_t *peer_target = base + (size_t) peer * stride;
            if (me < peer) {
                __atomic_store_n(peer_step, target_ready, __ATOMIC_RELEASE);
                pe_wait_eq(step, data_ready);
                memcpy(peer_target, cur, wrk);
                __atomic_thread_fence(__ATOMIC_RELEASE);
                __atomic_store_n(peer_step, data_ready, __ATOMIC_RELEASE);
            } else {
                pe_wait_eq(step, target_ready);
                memcpy(peer_target, cur, wrk);
                __atomic_thread_fence(__ATOMIC_RELEASE);
                __atomic_store_n(peer_step, data_ready, __ATOMIC_RELEASE);
                pe_wait_eq(step, data_ready);
            }
            rc |= oracle_reduce_local(op, dt, (int) count, target, cur);  /* :961-962 */
        }
        if (me < P - pow2) {                                           /* :966-975 */
            int peer = me + pow2;
            memcpy(base + (size_t) peer * stride, cur, wrk);
            __atomic_thread_fence(__ATOMIC_RELEASE);
            __atomic_store_n(pe_psync(seg, peer, PE_SYNC - 2), data_ready, __ATOMIC_RELEASE);
        }
        memcpy(target, cur, wrk);                                      /* :977 */
    }
    free(cur);
    for (i = 0; i < PE_SYNC; i++)                                      /* :982-983 */
        __atomic_store_n(pe_psync(seg, me, i), 0, __ATOMIC_RELEASE);
    return rc;
}

/* `reps` calls of the ring (alg 0) or recdbl_sw (alg 1), each preceded by a barrier (the
 * team API's pSync slot reuse rule, src/shmem_team.c:540-585); barrier epochs continue
 * from *epoch.  Returns seconds. */
double oracle_pe_time(int alg, void *seg, size_t stride, int P, int me, size_t count, int op,
                      int dt, const void *source, int reps, long *epoch)
{
    double t0 = now_s();
    for (int r = 0; r < reps; r++) {
        oracle_pe_barrier(seg, P, ++*epoch);
        int rc = alg == 1 ? oracle_pe_recdbl(seg, stride, P, me, count, op, dt, source)
                          : oracle_pe_ring(seg, stride, P, me, count, op, dt, source);
        if (rc) return -1.0;
    }
    return now_s() - t0;
}

double oracle_pe_ring_time(void *seg, size_t stride, int P, int me, size_t count, int op, int dt,
                           const void *source, int reps, long *epoch)
{
    return oracle_pe_time(0, seg, stride, P, me, count, op, dt, source, reps, epoch);
}
