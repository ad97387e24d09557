// runtime.h -- process-wide state of the MI355X SOS reduction runtime.
//
// One PE = one process = one GPU (device = LOCAL_RANK, else pe % device count).
// What SOS's init (src/init.c:221-550) sets up for the reduction path, rebuilt
// MI355X-first:
//   * rank/size discovery + a TCP bootstrap that broadcasts the RCCL unique id
//     (replaces the PMI KVS exchange of src/runtime-pmi.c);
//   * one RCCL communicator over all PEs (xGMI peer links on one node), carrying
//     every inter-PE byte of the team reductions (replaces the one-sided put/atomic
//     layer, src/shmem_comm.h, and the XPMEM/CMA/OFI transports);
//   * one non-blocking HIP stream per PE on which RCCL transfers and the combine
//     kernels are ordered (no host round trip between schedule steps);
//   * symmetric heaps: pinned host memory (shmem_malloc, SOS semantics: CPU
//     accessible, src/symmetric_heap_c.c) and device HBM (shmemx_malloc_device /
//     shmemx_heap_create with SHMEMX_EXTERNAL_HEAP_HIP);
//   * teams (start, stride, size) with SOS's pSync bookkeeping.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stddef.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "bootstrap.h"
#include "shmem.h"
#include "sosx.h"

namespace sosrt {

enum Transport : int {
    TRANSPORT_RCCL = 0,  // RCCL ncclSend/ncclRecv over xGMI (default, any device buffer)
    TRANSPORT_P2P = 1,   // kernels read peers' HBM through the IPC-mapped device heap
};

struct Team {
    int start = 0, stride = 1, size = 1;
    int my_idx = -1;          // index of this PE in the team, -1 if not a member
    int psync_avail[2] = {1, 1};  // SOS N_PSYNCS_PER_TEAM (src/shmem_team.h:18)
    int psync_idx = -1;           // team slot (src/shmem_team.c:21-24, :381-405)
    long config_mask = 0;         // shmem_team_config_t given at creation
    int num_contexts = 0;
    bool valid = false;
    bool predefined = false;
    int world_rank(int idx) const { return start + idx * stride; }
};

struct Heap {
    char *base = nullptr;
    size_t size = 0;
    bool device = false;
    bool external = false;
    std::map<size_t, size_t> free_blocks;  // offset -> size
    std::map<size_t, size_t> used_blocks;  // offset -> size
    uint64_t colour_seq = 0;               // large device allocations so far (Heap::alloc)
    void init(char *b, size_t s, bool dev, bool ext);
    void *alloc(size_t bytes, size_t align);
    bool release(void *p);
    bool contains(const void *p, size_t bytes) const
    {
        return base && (const char *)p >= base && (const char *)p + bytes <= base + size;
    }
};

struct State {
    bool initialized = false;
    bool finalized = false;
    int my_pe = 0;
    int n_pes = 1;
    int device = 0;
    int thread_level = 0;
    hipStream_t stream = nullptr;     // library stream (or the user's, shmemx_set_stream)
    hipStream_t own_stream = nullptr;
    ncclComm_t comm = nullptr;
    // device workspaces, grown on demand
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    void *stage = nullptr;            // staging for host-resident source/target
    size_t stage_bytes = 0;
    int *dbar = nullptr;              // 1-int device word for barriers
    // host-resident ring reductions, pipelined in stripes (collectives.cpp): copy streams,
    // per-slot events, three device stripe slots (the RCCL path's; p2p uses the stage)
    hipStream_t pipe_h2d = nullptr, pipe_d2h = nullptr;
    hipEvent_t pipe_ev[3][3] = {};    // [slot][h2d done, exchange done, d2h done]
    hipEvent_t sys_ev = nullptr;      // system-scope release marker (sync_system)
    long sys_releases = 0;            // how many sync_system / release_system markers ran
    // consumer half of the visibility rule (acquire_system, note_peer_wait/read)
    long sys_acquires = 0, peer_reads = 0, peer_reads_unacquired = 0;
    long acquire_kernels = 0;         // of sys_acquires: stream-wide acquire kernels
    bool acq_pending = false;         // a peer wait since the last acquire (stream order)
    unsigned *acq_mask = nullptr;     // device word: XCD ids the acquire kernels ran on
    void *stripes = nullptr;
    size_t stripes_bytes = 0;
    size_t host_stripe_bytes = 256u << 10; // SHMEMX_HOST_STRIPE_BYTES: min slice (0 = off)
    bool host_stripe_explicit = false;     // set in the environment
    Heap host_heap;                   // shmem_malloc (pinned host)
    Heap dev_heap;                    // shmemx_malloc_device / external HIP heap
    // device symmetric heap layout: [stage region | user allocations]
    size_t dev_heap_bytes = 2ull << 30;
    size_t sym_stage_bytes = 512ull << 20;
    char *sym_stage = nullptr;            // reserved at the heap start, same offset on every PE
    std::vector<char *> peer_heap;        // each PE's heap base as mapped here (IPC)
    // control plane
    sosboot::Hub hub;                 // TCP star to PE 0 (shmem_init path)
    sosboot::ShmBarrier shm;          // node-local barrier + transport counters
    int transport = TRANSPORT_RCCL;   // the transport calls use now
    bool rccl_allgather = false;      // SHMEMX_RCCL_ALLGATHER: equal-chunk allgather rounds
                                      // of a world-team plan as one ncclAllGather
    int rccl_allreduce = 0;           // SHMEMX_RCCL_ALLREDUCE: world-team reductions as one
                                      // ncclAllReduce: 1 integer sum/prod/min/max (bit-exact
                                      // in any order), 2 also fp32/fp64 sum/prod (tolerance)
    bool want_rccl = true;            // create the RCCL communicator
    bool want_p2p = false;            // IPC-map the device heap on every PE
    bool p2p_ready = false;           // heap mapped (or single PE)
    std::map<void *, size_t> dev_allocs;  // direct device allocations (no heap)
    // external heap registered before init (shmemx_heap_create)
    void *ext_base = nullptr;
    size_t ext_size = 0;
    int ext_type = -1;
    // parameters (SOS env table subset, src/shmem_env_defs.h)
    int reduce_alg = SOSX_ALG_AUTO;
    size_t coll_size_crossover = 16384;
    size_t symmetric_size = 512u << 20;
    bool debug = false;
    bool error_checking = true;
    bool heap_on_device = false;
    bool register_data = true;        // SHMEMX_REGISTER_DATA: register the data segment
    void *data_reg = nullptr;         // the registered page range of [__data_start, _end)
    size_t data_reg_bytes = 0;
    // teams (src/shmem_team.c): predefined WORLD / SHARED / SHMEMX_TEAM_NODE occupy slots
    // 0..2 of SHMEM_TEAMS_MAX; team_avail has a bit per free slot
    Team world, shared, node;
    long teams_max = 10;
    uint64_t team_avail = 0;
    std::vector<Team *> team_pool;
    std::mutex mu;
};

State &st();

// Abort the job with an SOS-style message ("[%04d] ERROR: ..."), like RAISE_ERROR_MSG
// (src/shmem_internal.h:124-128) -> shmem_runtime_abort.
[[noreturn]] void raise_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void warn(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void debug_msg(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

void check_initialized(const char *fn);
// A size from the environment (K/M/G suffixes, as SOS's size parameters), or `dflt`.
size_t env_size(const char *name, size_t dflt);
void hip_check(hipError_t e, const char *what);

void nccl_check(ncclResult_t r, const char *what);

// Completion with a SYSTEM-scope release: record an event created with
// hipEventReleaseToSystem on `stream` and wait for the stream (which waits for it).  The marker's release writes every
// XCD's L2 back to memory, so what the stream's kernels stored is in HBM when this
// returns: visible to DMA reads (hipMemcpy on any stream, the host), to peer GPUs reading
// over xGMI and to other processes.  A plain hipStreamSynchronize only promises the
// kernels finished; under multi-process queue time-slicing their nontemporal stores were
// seen still in L2 by a following DMA read ("The 12-PE wrong
// results").  Every call returns, and every p2p post is made, after this.
hipError_t sync_system(hipStream_t stream);
// The same release in stream order, without a host wait (stream-mode p2p posts).
hipError_t release_system(hipStream_t stream);

// The consumer half: a launch that reads bytes a peer published
// must follow, in stream order, a system-scope acquire issued after the wait that saw the
// peer's post.  A kernel dispatch does not promise one (tools/acquire_probe.hip: a
// kernel queued behind a device-side wait read every line of a rewritten buffer stale,
// and an acquire between the two removed it).  acquire_system enqueues the acquire kernel
// (sosx_acquire_system) and clears the pending wait; note_peer_wait records a wait for a
// peer's post (host spin or queued device wait); note_peer_read counts a consuming launch
// -- own_acquire: the launch runs its own per-workgroup acquire (the small path, the
// p2p gather that carries its signalling step) -- and flags one that follows a wait with
// no acquire in between.  Counters: sosx_acquire_stats.
hipError_t acquire_system(hipStream_t stream);
void note_peer_wait();
void note_peer_read(bool own_acquire);

// Device workspaces (grown, never shrunk).
void *scratch(size_t bytes);
void *stage(size_t bytes);

// Is `p` a device (HBM) pointer?  Host pageable, pinned and static data are not.
bool is_device_ptr(const void *p);
// HBM of this PE's own GPU (the library's device heaps, or a runtime query): what a kernel
// on the PE's stream may read without peer access.
bool is_local_device_ptr(const void *p);

// Symmetric check (SHMEM_ERR_CHECK_SYMMETRIC, src/shmem_internal.h:250-290).
bool is_symmetric(const void *p, size_t bytes);

// Barrier across a team: dissemination over RCCL point-to-point, host-synchronous.
void team_barrier(const Team &t);

// shmem_team_t is SOS's opaque `struct shmem_impl_team_t *` (mpp/shmem-def.h.in:94-96);
// the object behind it is a Team.
// Flags of the p2p transport's two cross-process mappings:
//  * the node shared segment of pair counters is registered with hipHostRegister:
//    Mapped (a device pointer through hipHostGetDevicePointer on the PE's own GPU) and
//    NOT hipExtHostRegisterCoarseGrained, so it is fine-grained system memory, coherent
//    for the device's system-scope atomic loads/stores (the device only loads and
//    stores these words, no read-modify-write, so no PCIe AtomicOp support is needed);
//  * a peer's device heap is opened with hipIpcOpenMemHandle(hipIpcMemLazyEnablePeerAccess),
//    which enables peer access from this PE's GPU to the exporter's GPU (required when
//    they differ; hipDeviceCanAccessPeer is checked first).
constexpr unsigned kP2PHostRegisterFlags = hipHostRegisterMapped;
constexpr unsigned kP2PIpcOpenFlags = hipIpcMemLazyEnablePeerAccess;

Team *team_from_handle(shmem_team_t handle);
inline shmem_team_t team_handle(Team *t) { return reinterpret_cast<shmem_team_t>(t); }

// The device symmetric heap (created collectively; IPC-exported to every PE when the
// peer-to-peer transport is on).
void ensure_device_heap();

// Per-pair transport counters living in the shared-memory segment (p2p.cpp).
size_t p2p_shared_bytes();
// Small host-resident team reductions through the node shared segment (smallpath.cpp).
size_t small_shared_bytes(int npes);
void small_path_setup(void *region, size_t bytes);   // collective (init_common)
void small_path_teardown();
bool small_path_takes(int alg, const void *target, const void *source, size_t bytes, const Team &t);
// small_path_takes (when `allowed`) for one team call, published to the team and checked
// against every peer's choice: a disagreement ends the job with both PEs' operands named.
bool small_path_route(int alg, const void *target, const void *source, size_t bytes, const Team &t,
                      bool allowed, const char *fn);
void small_path_reduce(int alg, void *target, const void *source, size_t count, size_t ts,
                       const Team &t, int op, int dt, const char *fn);
long small_path_calls();
long small_path_device_calls();
size_t small_path_set_device_bytes(size_t team_bytes);
// shmemx_reduce_local on operands of <= 64 KiB that are both in HBM or both in host memory:
// one launch + completion words (smallpath.cpp); false = not taken, use the general path.
bool small_local_combine(int op, int dt, void *inout, const void *in, size_t count, size_t ts,
                         bool dev_io, bool dev_in);
void small_local_release();
void team_word_put(int which, int world_pe, uint64_t v);   // node shm (p2p.cpp)
uint64_t team_word_get(int which, int world_pe);
// p2p signalling mode (p2p.cpp): stream-ordered device signals on the registered shm
// segment, or host synchronisation every round.  setup is collective.
void p2p_signal_setup();
void p2p_signal_teardown();
bool p2p_stream_signalling();
bool p2p_stream_capable();
void p2p_set_stream_signalling(bool on);

}  // namespace sosrt

// peer-to-peer executor (p2p.cpp)
namespace sosplan { struct Plan; }
namespace sosrt {
struct P2PBufs {
    const char *src;
    char *dst;
    char *scr;
    size_t src_off, dst_off;  // heap offsets of src/dst (published to the peers)
    size_t scr_off;           // heap offset of scr when the plan sends out of it
    unsigned smis, dmis;      // src/dst address mod 16 the plan was built with
};
int p2p_exec(const sosplan::Plan &plan, const Team &t, int alg, uint64_t count, uint64_t ts,
             const P2PBufs &b, int op, int dt, hipStream_t stream);
}  // namespace sosrt
