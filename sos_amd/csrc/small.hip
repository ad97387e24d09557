// small.hip -- the kernels of the small host-resident path (smallpath.cpp).
//
// Below a few MiB per team, a reduction whose operands live in host memory (SOS's
// symmetric heap) is latency bound: staging it through HBM costs two DMA round trips and
// the exchange's rounds.  The small path puts every PE's operand in a slot of node shared
// memory that every GPU maps, and ONE kernel per PE reads all P slots over the host link
// and writes that PE's result:
//   k_small_fold : recdbl_sw (AUTO below SHMEM_COLL_SIZE_CROSSOVER), this PE's own tree;
//   k_small_ring : the ring (AUTO above it), every chunk folded from its owner.
// Each lane handles one 16-B vector of every operand when the operands are 16-B aligned
// (the slots are), so a wave moves 1 KiB per load over PCIe instead of 256 B; the few
// elements that do not fill a vector go one per lane.  Completion is signalled without a
// stream synchronisation: every lane fences its stores at system scope and each
// workgroup then stores the call's sequence number into its own word of pinned host
// memory, which the host polls.
//
// The consumer half of the memory-visibility rule: the host
// launches these kernels after it saw the peers' posts, and a kernel dispatch does not
// promise to drop the lines an earlier call left in this GPU's L2s (tools/acquire_probe.hip,
// profiles/r6_acquire_probe.txt).  So each workgroup of a kernel that reads the peers'
// slots starts with a system-scope acquire (slot_acquire): lane 0 fences, waits for the
// invalidate, and the workgroup's loads follow the barrier.
#include "fold_kernels.h"

namespace sos {

// recdbl_sw from one PE's perspective: leaf y is leaf[y] OP extra[y] (the extra PE folded
// in first, src/collectives.c:905-926) or leaf[y] alone; the leaves are then reduced by
// the butterfly's tree (:932-963, fold_elem TREE).  P2 = 0: a runtime leaf count of 16..64
// (several PEs per GPU), walked with the binary-counter stack of k_fold_dyn.
// MAXP = 8 for the P2 <= 8 kernels (one PE per GPU on a node): 150 B of kernel
// arguments instead of 1 KiB, which the host launch call copies every time
// (SOSX_SMALL_TRACE measured the launch call at 3.0 us with the 1 KiB block).
__device__ __forceinline__ void slot_acquire() { wg_acquire(); }

template <int MAXP> struct SmallFoldArgsT {
    const void *leaf[MAXP];
    const void *extra[MAXP];           // null: the leaf has no extra PE
    uint32_t *flags;                   // one word per workgroup
    uint32_t seq;
    int p2;
    int vec_out;                       // out is 16-B aligned: vector stores
};
using SmallFoldArgs = SmallFoldArgsT<SOSX_MAX_FOLD>;
using SmallFoldArgs8 = SmallFoldArgsT<8>;

template <class T, class OP, int P2, class A>
__device__ __forceinline__ T small_tree_elem(const A &a, size_t i)
{
    if constexpr (P2 > 0) {
        T v[P2], x[P2];
#pragma unroll
        for (int y = 0; y < P2; ++y) {
            v[y] = ((const T *)a.leaf[y])[i];
            if (a.extra[y]) x[y] = ((const T *)a.extra[y])[i];
        }
#pragma unroll
        for (int y = 0; y < P2; ++y)
            if (a.extra[y]) v[y] = OP::f(v[y], x[y]);
        return fold_elem<T, OP, P2, SOSX_ORDER_TREE>(v);
    } else {
        T val[8];
        int height[8];
        int top = 0;
        for (int y = 0; y < a.p2; ++y) {
            T leaf = ((const T *)a.leaf[y])[i];
            if (a.extra[y]) leaf = OP::f(leaf, ((const T *)a.extra[y])[i]);
            val[top] = leaf;
            height[top] = 0;
            ++top;
            while (top >= 2 && height[top - 1] == height[top - 2]) {
                val[top - 2] = OP::f(val[top - 2], val[top - 1]);
                height[top - 2]++;
                --top;
            }
        }
        return val[0];
    }
}

__device__ __forceinline__ void signal_done(uint32_t *flags, uint32_t seq)
{
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class T>
__device__ __forceinline__ void store_pack(T *out, size_t i0, const Pack<T> &r, bool vec)
{
    if (vec) {
        *reinterpret_cast<u32x4 *>(out + i0) = __builtin_bit_cast(u32x4, r);
    } else {
#pragma unroll
        for (int j = 0; j < Pack<T>::N; ++j) out[i0 + j] = r.e[j];
    }
}

// VEC: lane L handles elements [L*V, L*V + V) as 16-B vectors (every leaf/extra 16-B
// aligned); the last, partial vector goes element by element.  Otherwise one element per
// lane.  (One lane's share: k_small_fold.)
template <class T, class OP, int P2, bool VEC, class A>
__device__ __forceinline__ void small_fold_lane(T *out, const A &a, size_t n, size_t lane)
{
    if constexpr (VEC && P2 > 0) {
        constexpr int V = Pack<T>::N;
        const size_t i0 = lane * V;
        if (i0 + V <= n) {
            u32x4 lv[P2], xv[P2];
#pragma unroll
            for (int y = 0; y < P2; ++y) {
                lv[y] = reinterpret_cast<const u32x4 *>(a.leaf[y])[lane];
                if (a.extra[y]) xv[y] = reinterpret_cast<const u32x4 *>(a.extra[y])[lane];
            }
            Pack<T> r;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                T v[P2];
#pragma unroll
                for (int y = 0; y < P2; ++y) {
                    v[y] = __builtin_bit_cast(Pack<T>, lv[y]).e[j];
                    if (a.extra[y]) v[y] = OP::f(v[y], __builtin_bit_cast(Pack<T>, xv[y]).e[j]);
                }
                r.e[j] = fold_elem<T, OP, P2, SOSX_ORDER_TREE>(v);
            }
            store_pack<T>(out, i0, r, a.vec_out != 0);
        } else {
            for (size_t i = i0; i < n; ++i) out[i] = small_tree_elem<T, OP, P2, A>(a, i);
        }
    } else {
        if (lane < n) out[lane] = small_tree_elem<T, OP, P2, A>(a, lane);
    }
}

template <class T, class OP, int P2, bool VEC, class A>
__global__ __launch_bounds__(kThreads) void k_small_fold(T *out, A a, size_t n)
{
    slot_acquire();
    small_fold_lane<T, OP, P2, VEC, A>(out, a, n, (size_t)blockIdx.x * kThreads + threadIdx.x);
    signal_done(a.flags, a.seq);
}

// The ring's value of every element: element i of ring chunk c is the LINEAR fold
// ((in[c] OP in[c+1]) OP ...) OP in[c-1] (the reduce-scatter's order, src/collectives.c:
// 693-727; chunk math :697-709), and every PE evaluates every chunk (the allgather's
// result, :737-756).  Workgroups are dealt per chunk, so the rotation is uniform per
// workgroup.  In chunk c, the first workgroup also takes the `head` elements before
// the first 16-B boundary and the elements after the last whole vector.
struct SmallRingArgs {
    const void *in[8];    // team order
    uint64_t first[9];    // chunk c = elements [first[c], first[c + 1])
    uint64_t head[8];     // elements of chunk c before its first vector
    uint64_t nvec[8];     // whole vectors of chunk c (VEC) or its elements (not VEC)
    uint64_t tstart[9];   // chunk c = workgroups [tstart[c], tstart[c + 1])
    uint32_t *flags;
    uint32_t seq;
    int vec_out;
    int acquire;          // the operands are peers' slots: slot_acquire first
};

template <class T, class OP, int NP>
__device__ __forceinline__ T ring_elem(const SmallRingArgs &a, int c, size_t i)
{
    T v[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const int pe = c + k < NP ? c + k : c + k - NP;
        v[k] = ((const T *)a.in[pe])[i];
    }
    return fold_elem<T, OP, NP, SOSX_ORDER_LINEAR>(v);
}

// The same, team size at run time, one element per lane (operands not 16-B aligned).
template <class T, class OP>
__global__ __launch_bounds__(kThreads) void k_small_ring_dyn(T *out, SmallRingArgs a, int np)
{
    if (a.acquire) slot_acquire();
    const uint64_t b = blockIdx.x;
    int c = 0;
    while (b >= a.tstart[c + 1]) ++c;
    const uint64_t j = (b - a.tstart[c]) * kThreads + threadIdx.x;
    if (j < a.nvec[c]) {
        const size_t i = a.first[c] + j;
        T acc = ((const T *)a.in[c])[i];
        for (int k = 1; k < np; ++k) {
            const int pe = c + k < np ? c + k : c + k - np;
            acc = OP::f(acc, ((const T *)a.in[pe])[i]);
        }
        out[i] = acc;
    }
    signal_done(a.flags, a.seq);
}

template <class T, class OP, int NP, bool VEC>
__global__ __launch_bounds__(kThreads) void k_small_ring(T *out, SmallRingArgs a)
{
    if (a.acquire) slot_acquire();
    const uint64_t b = blockIdx.x;
    int c = 0;
    while (b >= a.tstart[c + 1]) ++c;
    const uint64_t local = b - a.tstart[c];
    const uint64_t j = local * kThreads + threadIdx.x;
    if constexpr (VEC) {
        constexpr int V = Pack<T>::N;
        const uint64_t body = a.first[c] + a.head[c];
        if (j < a.nvec[c]) {
            const size_t i0 = body + j * V;
            u32x4 x[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const int pe = c + k < NP ? c + k : c + k - NP;
                x[k] = reinterpret_cast<const u32x4 *>((const T *)a.in[pe] + i0)[0];
            }
            Pack<T> r = __builtin_bit_cast(Pack<T>, fold_pack<T, OP, NP, SOSX_ORDER_LINEAR>(x));
            store_pack<T>(out, i0, r, a.vec_out != 0);
        }
        if (local == 0) {
            for (uint64_t i = a.first[c] + threadIdx.x; i < body; i += kThreads)
                out[i] = ring_elem<T, OP, NP>(a, c, i);
            for (uint64_t i = body + a.nvec[c] * V + threadIdx.x; i < a.first[c + 1]; i += kThreads)
                out[i] = ring_elem<T, OP, NP>(a, c, i);
        }
    } else {
        if (j < a.nvec[c]) out[a.first[c] + j] = ring_elem<T, OP, NP>(a, c, a.first[c] + j);
    }
    signal_done(a.flags, a.seq);
}

// Staging of a device-resident operand (smallpath.cpp): one workgroup copies `bytes` from
// HBM into the PE's slot of node shared memory (host memory, device view), fences at
// system scope, and then publishes the slot itself: word k <- val[k] (release, system
// scope), the posts the host makes for host operands.  With one workgroup the posts follow
// every lane's stores without a grid-wide barrier; a slot is at most a few tens of KiB.
// N = 8: 136 B of arguments for teams of up to 9 PEs (the launch call copies them).
template <int N> struct SmallStageArgsT {
    const void *src;
    void *dst;
    uint64_t bytes;
    uint64_t *word[N];
    uint64_t val[N];
    int nwords;
    int vec;                           // src and dst 16-B aligned
};
constexpr int kStageThreads = 1024;

template <class A>
__global__ __launch_bounds__(kStageThreads) void k_small_stage(A a)
{
    const uint8_t *s = (const uint8_t *)a.src;
    uint8_t *d = (uint8_t *)a.dst;
    uint64_t done = 0;
    if (a.vec) {  // four 16-B loads in flight per lane (64 KiB per pass)
        const uint64_t nv = a.bytes / 16;
        for (uint64_t i = threadIdx.x; i < nv; i += 4 * kStageThreads) {
            u32x4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * kStageThreads < nv) x[u] = reinterpret_cast<const u32x4 *>(s)[i + u * kStageThreads];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * kStageThreads < nv) reinterpret_cast<u32x4 *>(d)[i + u * kStageThreads] = x[u];
        }
        done = nv * 16;
    }
    for (uint64_t i = done + threadIdx.x; i < a.bytes; i += kStageThreads) d[i] = s[i];
    __threadfence_system();
    __syncthreads();
    if ((int)threadIdx.x < a.nwords)
        __hip_atomic_store(a.word[threadIdx.x], a.val[threadIdx.x], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace sos

using namespace sos;

namespace {

struct SmallFoldFn {
    template <class T, class OP>
    static int run(void *out, const SmallFoldArgs *a, size_t n, bool vec, unsigned blocks, hipStream_t st)
    {
        SmallFoldArgs8 a8;
        memset(&a8, 0, sizeof(a8));
        if (a->p2 <= 8) {
            for (int y = 0; y < a->p2; ++y) {
                a8.leaf[y] = a->leaf[y];
                a8.extra[y] = a->extra[y];
            }
            a8.flags = a->flags;
            a8.seq = a->seq;
            a8.p2 = a->p2;
            a8.vec_out = a->vec_out;
        }
        switch (a->p2) {
#define SOS_SMALL(P2)                                                                              \
    case P2:                                                                                       \
        if (vec)                                                                                   \
            hipLaunchKernelGGL((k_small_fold<T, OP, P2, true, SmallFoldArgs8>), dim3(blocks),       \
                               dim3(kThreads), 0, st, (T *)out, a8, n);                            \
        else  /* unaligned operands: one element per lane, leaf count at run time */             \
            hipLaunchKernelGGL((k_small_fold<T, OP, 0, false, SmallFoldArgs8>), dim3(blocks),       \
                               dim3(kThreads), 0, st, (T *)out, a8, n);                            \
        break;
            SOS_SMALL(1)
            SOS_SMALL(2)
            SOS_SMALL(4)
            SOS_SMALL(8)
#undef SOS_SMALL
            default:
                hipLaunchKernelGGL((k_small_fold<T, OP, 0, false, SmallFoldArgs>), dim3(blocks),
                                   dim3(kThreads), 0, st, (T *)out, *a, n);
        }
        return hip_ok(hipGetLastError());
    }
};

struct SmallRingFn {
    template <class T, class OP>
    static int run(void *out, const SmallRingArgs *a, int np, bool vec, unsigned blocks, hipStream_t st)
    {
        if (!vec) {  // unaligned operands: one element per lane, team size at run time
            if (np < 1 || np > 8) return SOSX_ERR_ARG;
            hipLaunchKernelGGL((k_small_ring_dyn<T, OP>), dim3(blocks), dim3(kThreads), 0, st, (T *)out, *a, np);
            return hip_ok(hipGetLastError());
        }
        switch (np) {
#define SOS_RING(NP)                                                                               \
    case NP:                                                                                       \
        hipLaunchKernelGGL((k_small_ring<T, OP, NP, true>), dim3(blocks), dim3(kThreads), 0, st,     \
                           (T *)out, *a);                                                          \
        break;
            SOS_RING(1)
            SOS_RING(2)
            SOS_RING(3)
            SOS_RING(4)
            SOS_RING(5)
            SOS_RING(6)
            SOS_RING(7)
            SOS_RING(8)
#undef SOS_RING
            default:
                return SOSX_ERR_ARG;
        }
        return hip_ok(hipGetLastError());
    }
};

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

// One PE's recdbl_sw value over p2 leaves (leaves[y], each folded first with extras[y]
// when that is not null), written to `out`; workgroup b then stores `seq` into flags[b]
// (pinned host memory), b < *nblocks.  count <= SOSX_SMALL_FOLD_MAX.
int sosx_small_fold(int op, int dtype, void *out, const void *const *leaves,
                    const void *const *extras, int p2, size_t count, uint32_t *flags, uint32_t seq,
                    int *nblocks, void *stream)
{
    if (p2 < 1 || p2 > SOSX_MAX_FOLD || (p2 & (p2 - 1)) || count > SOSX_SMALL_FOLD_MAX || !flags ||
        !nblocks)
        return SOSX_ERR_ARG;
    int rc = sos_check_op(op, dtype);
    if (rc) return rc;
    *nblocks = 0;
    if (count == 0) return SOSX_OK;
    if (!out || !leaves) return SOSX_ERR_ARG;
    SmallFoldArgs a;
    memset(&a, 0, sizeof(a));
    bool vec = p2 <= 8;
    for (int y = 0; y < p2; ++y) {
        if (!leaves[y]) return SOSX_ERR_ARG;
        a.leaf[y] = leaves[y];
        a.extra[y] = extras ? extras[y] : nullptr;
        vec &= aligned16(a.leaf[y]) && (!a.extra[y] || aligned16(a.extra[y]));
    }
    a.flags = flags;
    a.seq = seq;
    a.p2 = p2;
    a.vec_out = aligned16(out);
    const size_t V = vec ? 16 / sos_dtype_info(dtype).size : 1;
    const size_t lanes = (count + V - 1) / V;
    const unsigned blocks = (unsigned)((lanes + kThreads - 1) / kThreads);
    *nblocks = (int)blocks;
    return dispatch<SmallFoldFn>(op, dtype, out, (const SmallFoldArgs *)&a, count, vec, blocks,
                                 as_stream(stream));
}

// Every element's SOS ring value for one PE (np = 2..8 team operands in team order),
// written to `out` (count elements); workgroup b then stores `seq` into flags[b],
// b < *nblocks.
int sosx_small_ring(int op, int dtype, void *out, const void *const *ins, int np, size_t count,
                    uint32_t *flags, uint32_t seq, int *nblocks, void *stream)
{
    if (np < 2 || np > 8 || count > SOSX_SMALL_FOLD_MAX || !flags || !nblocks) return SOSX_ERR_ARG;
    int rc = sos_check_op(op, dtype);
    if (rc) return rc;
    *nblocks = 0;
    if (count == 0) return SOSX_OK;
    if (!out || !ins) return SOSX_ERR_ARG;
    SmallRingArgs a;
    memset(&a, 0, sizeof(a));
    bool vec = true;
    for (int c = 0; c < np; ++c) {
        if (!ins[c]) return SOSX_ERR_ARG;
        a.in[c] = ins[c];
        vec &= aligned16(ins[c]);
    }
    const uint64_t V = vec ? 16 / sos_dtype_info(dtype).size : 1;
    const uint64_t q = count / (uint64_t)np, r = count % (uint64_t)np;
    uint64_t first = 0, tiles = 0;
    for (int c = 0; c < np; ++c) {
        const uint64_t len = q + ((uint64_t)c < r ? 1 : 0);  // src/collectives.c:697-709
        a.first[c] = first;
        a.tstart[c] = tiles;
        uint64_t head = vec ? (V - first % V) % V : 0;
        if (head > len) head = len;
        a.head[c] = head;
        a.nvec[c] = (len - head) / V;
        if (len) tiles += a.nvec[c] ? (a.nvec[c] + kThreads - 1) / kThreads : 1;
        first += len;
    }
    a.first[np] = first;
    a.tstart[np] = tiles;
    for (int c = np + 1; c <= 8; ++c) {  // sentinels: the chunk search never passes np
        a.first[c] = first;
        a.tstart[c] = ~(uint64_t)0;
    }
    a.flags = flags;
    a.seq = seq;
    a.vec_out = aligned16(out);
    a.acquire = 1;
    *nblocks = (int)tiles;
    return dispatch<SmallRingFn>(op, dtype, out, (const SmallRingArgs *)&a, np, vec, (unsigned)tiles,
                                 as_stream(stream));
}

// The LINEAR fold ((ins[0] OP ins[1]) OP ...) OP ins[np-1] of every element (np = 1..8:
// the team scans' value at one PE, src/collectives.c:1111-1209 -- inscan folds the team's
// sources 0..me, exscan 0..me-1), written to `out`; completion words as above.  This is
// the ring kernel with a single chunk: every workgroup folds from ins[0].  acquire != 0:
// the operands are peers' slots (team calls), each workgroup acquires first; 0 for local
// operands (shmemx_reduce_local).
int sosx_small_linear(int op, int dtype, void *out, const void *const *ins, int np, size_t count,
                      uint32_t *flags, uint32_t seq, int *nblocks, int acquire, void *stream)
{
    if (np < 1 || np > 8 || count > SOSX_SMALL_FOLD_MAX || !flags || !nblocks) return SOSX_ERR_ARG;
    int rc = sos_check_op(op, dtype);
    if (rc) return rc;
    *nblocks = 0;
    if (count == 0) return SOSX_OK;
    if (!out || !ins) return SOSX_ERR_ARG;
    SmallRingArgs a;
    memset(&a, 0, sizeof(a));
    bool vec = true;
    for (int k = 0; k < np; ++k) {
        if (!ins[k]) return SOSX_ERR_ARG;
        a.in[k] = ins[k];
        vec &= aligned16(ins[k]);
    }
    const uint64_t V = vec ? 16 / sos_dtype_info(dtype).size : 1;
    a.first[0] = 0;
    a.head[0] = 0;
    a.nvec[0] = count / V;
    const uint64_t tiles = a.nvec[0] ? (a.nvec[0] + kThreads - 1) / kThreads : 1;
    a.tstart[0] = 0;
    for (int c = 1; c <= 8; ++c) {  // chunk 0 holds everything; the others are empty
        a.first[c] = count;
        a.tstart[c] = c <= np ? tiles : ~(uint64_t)0;
    }
    a.flags = flags;
    a.seq = seq;
    a.vec_out = aligned16(out);
    a.acquire = acquire != 0;
    *nblocks = (int)tiles;
    return dispatch<SmallRingFn>(op, dtype, out, (const SmallRingArgs *)&a, np, vec, (unsigned)tiles,
                                 as_stream(stream));
}

// Copy `bytes` from src (device) to dst (a node-shared slot, device view) in one
// workgroup, then store vals[k] into *words[k] for k < nwords (release, system scope):
// the small path's staging + post of a device operand.  bytes <= SOSX_SMALL_FOLD_MAX,
// 1 <= nwords <= SOSX_MAX_FOLD.
int sosx_small_stage(void *dst, const void *src, size_t bytes, uint64_t *const *words,
                     const uint64_t *vals, int nwords, void *stream)
{
    if (!dst || !src || bytes > SOSX_SMALL_FOLD_MAX || nwords < 1 || nwords > SOSX_MAX_FOLD || !words ||
        !vals)
        return SOSX_ERR_ARG;
    for (int k = 0; k < nwords; ++k)
        if (!words[k]) return SOSX_ERR_ARG;
    const hipStream_t st = as_stream(stream);
    const int vec = aligned16(src) && aligned16(dst);
    if (nwords <= 8) {
        SmallStageArgsT<8> a;
        memset(&a, 0, sizeof(a));
        a.src = src;
        a.dst = dst;
        a.bytes = bytes;
        for (int k = 0; k < nwords; ++k) {
            a.word[k] = words[k];
            a.val[k] = vals[k];
        }
        a.nwords = nwords;
        a.vec = vec;
        hipLaunchKernelGGL((k_small_stage<SmallStageArgsT<8>>), dim3(1), dim3(kStageThreads), 0, st, a);
    } else {
        SmallStageArgsT<SOSX_MAX_FOLD> a;
        memset(&a, 0, sizeof(a));
        a.src = src;
        a.dst = dst;
        a.bytes = bytes;
        for (int k = 0; k < nwords; ++k) {
            a.word[k] = words[k];
            a.val[k] = vals[k];
        }
        a.nwords = nwords;
        a.vec = vec;
        hipLaunchKernelGGL((k_small_stage<SmallStageArgsT<SOSX_MAX_FOLD>>), dim3(1), dim3(kStageThreads), 0,
                           st, a);
    }
    return hip_ok(hipGetLastError());
}

}  // extern "C"
