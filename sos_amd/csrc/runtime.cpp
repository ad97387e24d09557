// runtime.cpp -- init/finalize, symmetric heaps, teams, barriers and diagnostics of
// the MI355X SOS reduction runtime.  See runtime.h for the design.
#include "runtime.h"

#include <execinfo.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>

#include "bootstrap.h"
#include "shmem.h"
#include "shmemx.h"

// The executable's data segment, as SOS uses for its symmetric-address check
// (src/init.c:341-346); weak so a loader without them still links.
extern "C" char __data_start[] __attribute__((weak));
extern "C" char _end[] __attribute__((weak));

extern "C" {
shmem_team_t SHMEM_TEAM_WORLD = nullptr;
shmem_team_t SHMEM_TEAM_SHARED = nullptr;
shmem_team_t SHMEMX_TEAM_NODE = nullptr;
}

namespace sosrt {

State &st()
{
    static State s;
    return s;
}

// ---------------------------------------------------------------------------------
// diagnostics (src/shmem_internal.h:60-180)
// ---------------------------------------------------------------------------------
// SHMEM_BACKTRACE (src/backtrace.c:181-206): "" (default) off, "execinfo" or "auto" the
// glibc backtrace of the failing PE on stderr; "gdb" is not offered by this build (a
// debugger attached to a process holding a GPU context is not something to start from
// an abort path), and any other value is ignored with SOS's warning.
static void print_backtrace()
{
    const char *m = getenv("SHMEM_BACKTRACE");
    if (!m) m = getenv("SMA_BACKTRACE");
    if (!m || !*m) return;
    if (strcmp(m, "execinfo") && strcmp(m, "auto")) {
        if (!strcmp(m, "gdb"))
            fprintf(stderr, "[%04d] WARN:  Backtrace support through gdb is not available.\n", st().my_pe);
        else
            fprintf(stderr, "[%04d] WARN:  Ignoring invalid backtrace method '%s'.\n", st().my_pe, m);
        return;
    }
    void *frames[64];
    const int n = backtrace(frames, 64);
    fprintf(stderr, "[%04d] backtrace (%d frames):\n", st().my_pe, n);
    backtrace_symbols_fd(frames, n, 2);
}

void raise_error(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[%04d] ERROR: %s\n", st().my_pe, buf);
    print_backtrace();
    fprintf(stderr, "[%04d] ERROR: Sandia OpenSHMEM (MI355X reduction path) exited in error\n",
            st().my_pe);
    fflush(stderr);
    _exit(1);  // shmem_runtime_abort(1, ...): no atexit handlers, the launcher reaps the job
}

void warn(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[%04d] WARN:  %s\n", st().my_pe, buf);
}

void debug_msg(const char *fmt, ...)
{
    if (!st().debug) return;
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[%04d] DEBUG: %s\n", st().my_pe, buf);
}

void check_initialized(const char *fn)
{
    if (!st().initialized) raise_error("%s called before shmem_init or after shmem_finalize", fn);
}

void hip_check(hipError_t e, const char *what)
{
    if (e != hipSuccess) raise_error("HIP error in %s: %s", what, hipGetErrorString(e));
}

void nccl_check(ncclResult_t r, const char *what)
{
    if (r != ncclSuccess) raise_error("RCCL error in %s: %s", what, ncclGetErrorString(r));
}

// ---------------------------------------------------------------------------------
// environment (src/shmem_env_defs.h, src/shmem_env.c:34-117)
// ---------------------------------------------------------------------------------
static size_t atol_scaled(const char *s, size_t dflt)
{
    if (!s || !*s) return dflt;
    char *end = nullptr;
    double v = strtod(s, &end);
    if (end == s || v < 0) return dflt;
    switch (*end) {
        case 'k': case 'K': v *= 1024.0; break;
        case 'm': case 'M': v *= 1024.0 * 1024.0; break;
        case 'g': case 'G': v *= 1024.0 * 1024.0 * 1024.0; break;
        case 't': case 'T': v *= 1024.0 * 1024.0 * 1024.0 * 1024.0; break;
        default: break;
    }
    return (size_t)v;
}

size_t env_size(const char *name, size_t dflt) { return atol_scaled(getenv(name), dflt); }

static const char *getenv2(const char *name)
{
    // SOS accepts SHMEM_<X> and SMA_<X> (src/shmem_env.c:90-117)
    const char *v = getenv((std::string("SHMEM_") + name).c_str());
    if (!v) v = getenv((std::string("SMA_") + name).c_str());
    return v;
}

int parse_reduce_alg(const char *type, int dflt)
{
    if (!type) return dflt;
    if (!strcmp(type, "auto")) return SOSX_ALG_AUTO;
    // linear and tree need NIC atomics; without them SOS runs recdbl_sw
    // (src/shmem_collectives.h:200-221)
    if (!strcmp(type, "linear") || !strcmp(type, "tree") || !strcmp(type, "recdbl"))
        return SOSX_ALG_RECDBL;
    if (!strcmp(type, "ring")) return SOSX_ALG_RING;
    if (!strcmp(type, "rechalving")) return SOSX_ALG_RECHALVING;
    if (!strcmp(type, "recdbl_direct")) return SOSX_ALG_RECDBL_DIRECT;
    if (!strcmp(type, "recdbl_gather")) return SOSX_ALG_RECDBL_GATHER;
    warn("Ignoring bad reduction algorithm '%s'", type);
    return dflt;
}

// SHMEM_INFO / SHMEM_VERSION (src/init.c:240-255, src/shmem_env.c:177-220): PE 0 prints
// the package string, and with SHMEM_INFO the parameters this build reads, in SOS's
// format: name, current value, kind, default, description.
struct EnvDef {
    const char *name, *kind, *dflt, *cat, *desc;
};
static const EnvDef kEnv[] = {
    {"SHMEM_INFO", "bool", "false", "openshmem", "Print library information message at startup"},
    {"SHMEM_VERSION", "bool", "false", "openshmem", "Print library version at startup"},
    {"SHMEM_DEBUG", "bool", "false", "openshmem", "Enable debugging messages"},
    {"SHMEM_SYMMETRIC_SIZE", "size", "536870912", "openshmem", "Symmetric heap size (pinned host memory)"},
    {"SHMEM_TEAMS_MAX", "long", "10", "other", "Maximum number of teams per PE"},
    {"SHMEM_BACKTRACE", "string", "", "other", "Method for backtraces on error (execinfo, auto)"},
    {"SHMEM_COLL_SIZE_CROSSOVER", "size", "16384", "collectives",
     "Crossover between latency and bandwidth optimized collectives (msg. size)"},
    {"SHMEM_REDUCE_ALGORITHM", "string", "auto", "collectives",
     "Algorithm for reductions.  Options are auto, linear, tree, recdbl, ring, rechalving, "
     "recdbl_direct, recdbl_gather"},
    {"SHMEMX_TRANSPORT", "string", "rccl", "device", "Inter-PE transport: rccl, p2p or both"},
    {"SHMEMX_DEVICE", "long", "local rank % GPUs", "device", "GPU of this PE"},
    {"SHMEMX_DEVICE_HEAP_SIZE", "size", "2147483648", "device", "Device symmetric heap size (HBM)"},
    {"SHMEMX_STAGE_BYTES", "size", "536870912", "device",
     "Stage region of the device heap (host operands, p2p exchange scratch)"},
    {"SHMEMX_HEAP_ON_DEVICE", "bool", "false", "device", "shmem_malloc returns device memory"},
    {"SHMEMX_CHECK_SYMMETRIC", "bool", "false", "device", "Check that collective buffers are symmetric"},
    {"SHMEMX_HOST_STRIPE_BYTES", "size", "262144", "device",
     "Slice size of the striped host-resident ring (H2D || exchange || D2H)"},
    {"SHMEMX_RCCL_ALLGATHER", "long", "0", "device", "1: equal-chunk allgather rounds as ncclAllGather"},
    {"SHMEMX_RCCL_ALLREDUCE", "long", "0", "device",
     "1: integer world reductions as ncclAllReduce; 2: also fp sum/prod (RCCL's order)"},
    {"SHMEMX_P2P_SIGNAL", "string", "stream on one GPU, host across GPUs", "device",
     "p2p round signalling: stream (device) or host"},
    {"SHMEMX_P2P_ENTRY", "string", "host", "device",
     "Stream signalling: the call's entry boundary on the host or queued (device)"},
    {"SHMEMX_P2P_TIMEOUT", "long", "300", "device", "Seconds before a p2p wait ends the job"},
    {"SHMEMX_SMALL_HOST", "bool", "true", "device",
     "Small team collectives through node shared memory (host operands; device ones too, below)"},
    {"SHMEMX_SMALL_HOST_BYTES", "size", "1048576", "device",
     "Largest operand of that path (its slots: at most 32 MiB over all PEs)"},
    {"SHMEMX_SMALL_DEVICE", "size", "131072", "device",
     "Device-resident operands take that path when team size * bytes <= this (0: never)"},
    {"SHMEMX_REGISTER_DATA", "bool", "true", "device",
     "Register the executable's data segment with HIP (static symmetric objects DMA as pinned)"},
};

static void print_env()
{
    static const struct { const char *cat, *title; } sections[] = {
        {"openshmem", nullptr}, {"other", "Additional options"},
        {"collectives", "Collectives options"}, {"device", "MI355X (HIP / RCCL) options"}};
    for (const auto &sec : sections) {
        if (sec.title) printf("\n%s:\n", sec.title);
        for (const EnvDef &e : kEnv) {
            if (strcmp(e.cat, sec.cat)) continue;
            const char *v = getenv(e.name);
            if (!v && !strncmp(e.name, "SHMEM_", 6)) v = getenv((std::string("SMA_") + (e.name + 6)).c_str());
            printf("  %-27s %s (type: %s, default: %s)\n\t%s\n", e.name, v ? v : e.dflt, e.kind,
                   e.dflt, e.desc);
        }
    }
    printf("\nNetwork transport: none (intra-node: RCCL over xGMI / IPC-mapped HBM)\n\n");
    fflush(stdout);
}

static bool env_flag(const char *name)
{
    const char *v = getenv2(name);
    return v && *v && strcmp(v, "0") && strcasecmp(v, "false") && strcasecmp(v, "no");
}

static void read_env(State &s)
{
    s.reduce_alg = parse_reduce_alg(getenv2("REDUCE_ALGORITHM"), SOSX_ALG_AUTO);
    s.coll_size_crossover = atol_scaled(getenv2("COLL_SIZE_CROSSOVER"), 16384);
    // SHMEM_TEAMS_MAX (src/shmem_env_defs.h:75, default 10; src/shmem_team.c:171-178)
    const char *tm = getenv2("TEAMS_MAX");
    s.teams_max = tm && *tm ? atol(tm) : 10;
    s.symmetric_size = atol_scaled(getenv2("SYMMETRIC_SIZE"), 512u << 20);
    const char *d = getenv2("DEBUG");
    s.debug = d && *d && strcmp(d, "0") && strcasecmp(d, "false");
    const char *h = getenv("SHMEMX_HEAP_ON_DEVICE");
    s.heap_on_device = h && *h && strcmp(h, "0");
    const char *c = getenv("SHMEMX_CHECK_SYMMETRIC");
    s.error_checking = c && *c && strcmp(c, "0");
    // rccl (default) | p2p | both (RCCL communicator AND IPC-mapped heap; calls use RCCL
    // until shmemx_set_transport(SOSX_TRANSPORT_P2P))
    const char *t = getenv("SHMEMX_TRANSPORT");
    s.transport = (t && !strcmp(t, "p2p")) ? TRANSPORT_P2P : TRANSPORT_RCCL;
    s.want_rccl = !(t && !strcmp(t, "p2p"));
    s.want_p2p = t && (!strcmp(t, "p2p") || !strcmp(t, "both"));
    if (t && strcmp(t, "p2p") && strcmp(t, "rccl") && strcmp(t, "both"))
        warn("Ignoring bad SHMEMX_TRANSPORT '%s'", t);
    s.dev_heap_bytes = atol_scaled(getenv("SHMEMX_DEVICE_HEAP_SIZE"), 2ull << 30);
    s.host_stripe_bytes = atol_scaled(getenv("SHMEMX_HOST_STRIPE_BYTES"), 256u << 10);
    s.host_stripe_explicit = getenv("SHMEMX_HOST_STRIPE_BYTES") != nullptr;
    s.sym_stage_bytes = atol_scaled(getenv("SHMEMX_STAGE_BYTES"), 512ull << 20);
    const char *ag = getenv("SHMEMX_RCCL_ALLGATHER");
    s.rccl_allgather = ag && atoi(ag) != 0;
    const char *ar = getenv("SHMEMX_RCCL_ALLREDUCE");
    s.rccl_allreduce = ar ? std::min(std::max(atoi(ar), 0), 2) : 0;
    s.sym_stage_bytes = (s.sym_stage_bytes + 4095) & ~(size_t)4095;
    if (s.sym_stage_bytes >= s.dev_heap_bytes) s.dev_heap_bytes = s.sym_stage_bytes + (256u << 20);
    const char *rd = getenv("SHMEMX_REGISTER_DATA");
    s.register_data = !(rd && (!strcmp(rd, "0") || !strcasecmp(rd, "false") || !strcasecmp(rd, "no")));
}

// ---------------------------------------------------------------------------------
// The executable's data segment.  SOS registers it with every transport at init
// (src/init.c:341-346 takes [__data_start, _end); src/transport_ofi.c:741 fi_mr_reg of
// shmem_internal_data_base, src/transport_xpmem.c:56-64), so static symmetric objects
// move like heap memory.  Here the same range is registered with HIP: its pages are
// pinned and mapped for the DMA engines, so H2D/D2H copies of static operands run at the
// pinned rate instead of through HIP's pageable bounce buffers (sosx_combine_host's chunk
// pipeline and the team path's staging copies detect it as host-registered memory).  The
// range is rounded out to whole pages; if HIP refuses it (a read-only page at the start),
// the start is rounded in instead; if that fails too the segment stays pageable: correct,
// slower, reported under SHMEM_DEBUG.  Unregistered at shmem_finalize.
// ---------------------------------------------------------------------------------
static void register_data_segment(State &s)
{
    s.data_reg = nullptr;
    s.data_reg_bytes = 0;
    if (!s.register_data || !__data_start || !_end || _end <= __data_start) return;
    const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t lo = (uintptr_t)__data_start, hi = ((uintptr_t)_end + pg - 1) & ~(pg - 1);
    for (uintptr_t start : {lo & ~(pg - 1), (lo + pg - 1) & ~(pg - 1)}) {
        if (start >= hi) break;
        const hipError_t e = hipHostRegister((void *)start, hi - start, hipHostRegisterDefault);
        if (e == hipSuccess) {
            s.data_reg = (void *)start;
            s.data_reg_bytes = hi - start;
            debug_msg("data segment [%p, %p) registered with HIP (%zu B)", (void *)start, (void *)hi,
                      (size_t)(hi - start));
            return;
        }
        (void)hipGetLastError();
        debug_msg("hipHostRegister of the data segment from %p failed (%s)", (void *)start,
                  hipGetErrorString(e));
    }
}

static void unregister_data_segment(State &s)
{
    if (s.data_reg) (void)hipHostUnregister(s.data_reg);
    s.data_reg = nullptr;
    s.data_reg_bytes = 0;
}

// ---------------------------------------------------------------------------------
// symmetric heaps: first-fit allocator over one region (same call sequence on every
// PE => same offsets, as SOS's dlmalloc heap at a fixed base, src/malloc.c)
// ---------------------------------------------------------------------------------
void Heap::init(char *b, size_t s, bool dev, bool ext)
{
    base = b;
    size = s;
    device = dev;
    external = ext;
    free_blocks.clear();
    used_blocks.clear();
    free_blocks[0] = s;
    colour_seq = 0;
}

// Colours of large device-heap allocations.  The HBM rate of a streaming kernel depends on
// how far apart its operands start (tools/offset_probe.py, profiles/r4_offset_probe.txt,
// 128Mi fp32 combine, in = inout + 512 MiB + delta): delta a multiple of 32 KiB below
// 1 MiB, or a multiple of 16 MiB, runs at 6.22-6.32 TB/s (the two read streams walk the
// same HBM channels in step); every odd multiple of 4 KiB probed runs at 6.55-6.67.  So
// the k-th allocation of at least kColorMin bytes starts at (k mod 8) * 4 KiB mod 32 KiB
// from the heap base: consecutive large buffers (a source and its target, a fold's
// inputs) are an odd multiple of 4 KiB apart.  The colour depends only on the allocation
// sequence, which SOS makes collective, so offsets stay symmetric across PEs.
constexpr size_t kColorMin = (size_t)1 << 20, kColorStep = 4096, kColorPeriod = 32768;

void *Heap::alloc(size_t bytes, size_t align)
{
    if (!base) return nullptr;
    if (align < 256) align = 256;
    if (bytes == 0) bytes = 1;
    bytes = (bytes + 255) & ~(size_t)255;
    const bool colour = device && bytes >= kColorMin && align <= kColorStep;
    const size_t want = colour ? (size_t)(colour_seq % (kColorPeriod / kColorStep)) * kColorStep : 0;
    // first fit at the colour; when no free block holds the coloured placement (a heap
    // sized tightly), first fit without it: the colour is a rate preference, never a
    // reason to fail.  The choice depends only on the allocation sequence, so it is the
    // same on every PE and offsets stay symmetric.
    for (int pass = colour ? 0 : 1; pass < 2; ++pass) {
        for (auto it = free_blocks.begin(); it != free_blocks.end(); ++it) {
            size_t off = it->first, len = it->second;
            size_t aoff = (off + align - 1) / align * align;
            if (pass == 0) aoff += (want + kColorPeriod - aoff % kColorPeriod) % kColorPeriod;
            if (aoff + bytes > off + len) continue;
            free_blocks.erase(it);
            if (aoff > off) free_blocks[off] = aoff - off;
            if (off + len > aoff + bytes) free_blocks[aoff + bytes] = off + len - (aoff + bytes);
            used_blocks[aoff] = bytes;
            if (colour) ++colour_seq;
            return base + aoff;
        }
    }
    return nullptr;
}

bool Heap::release(void *p)
{
    if (!contains(p, 1)) return false;
    size_t off = (size_t)((char *)p - base);
    auto u = used_blocks.find(off);
    if (u == used_blocks.end()) return false;
    size_t len = u->second;
    used_blocks.erase(u);
    auto nx = free_blocks.lower_bound(off);
    if (nx != free_blocks.end() && nx->first == off + len) {
        len += nx->second;
        free_blocks.erase(nx);
    }
    auto pv = free_blocks.lower_bound(off);
    if (pv != free_blocks.begin()) {
        --pv;
        if (pv->first + pv->second == off) {
            pv->second += len;
            return true;
        }
    }
    free_blocks[off] = len;
    return true;
}

static void ensure_host_heap(State &s)
{
    if (s.host_heap.base) return;
    void *p = nullptr;
    hip_check(hipHostMalloc(&p, s.symmetric_size, hipHostMallocDefault), "hipHostMalloc(heap)");
    s.host_heap.init((char *)p, s.symmetric_size, false, false);
}

// Collective: every PE creates its device heap [stage | allocations]; when the
// peer-to-peer transport is on, the heaps are IPC-exported and every PE maps every
// other PE's heap (xGMI peer memory on the 8-GPU node; the same device in tests).
void ensure_device_heap()
{
    State &s = st();
    if (s.dev_heap.base) return;
    char *base = nullptr;
    // HIP runtimes before 7.2 (torch 2.10's bundled 7.0.2 among them) hang in
    // hipIpcOpenMemHandle when the exported allocation's size has bit 31 set (2-4 GiB,
    // 6-8 GiB, ...: measured with tests/heap_init_pe.py and tools/diag/heap_probe.c); 7.2 maps every size.  An
    // exported heap is therefore rounded up past such sizes on those runtimes.
    const bool exported = s.want_p2p && s.n_pes > 1;
    int rtv = 0;
    (void)hipRuntimeGetVersion(&rtv);
    const bool ipc_size_bug = rtv < 70200000;
    if (s.ext_base) {
        base = (char *)s.ext_base;
        s.dev_heap_bytes = s.ext_size;
        if (s.sym_stage_bytes >= s.ext_size) s.sym_stage_bytes = s.ext_size / 2;
    } else {
        if (exported && ipc_size_bug && (s.dev_heap_bytes & 0x80000000ull)) {
            const size_t want = s.dev_heap_bytes;
            s.dev_heap_bytes = (s.dev_heap_bytes | 0xFFFFFFFFull) + 1;
            debug_msg("device heap %zu B rounded up to %zu B (HIP %d IPC size limitation)", want,
                      s.dev_heap_bytes, rtv);
        }
        hip_check(hipMalloc((void **)&base, s.dev_heap_bytes), "hipMalloc(device heap)");
    }
    debug_msg("device heap %zu B at %p (stage %zu B)", s.dev_heap_bytes, (void *)base,
              s.sym_stage_bytes);
    s.sym_stage = base;
    s.dev_heap.init(base + s.sym_stage_bytes, s.dev_heap_bytes - s.sym_stage_bytes, true,
                    s.ext_base != nullptr);
    s.peer_heap.assign((size_t)s.n_pes, nullptr);
    s.peer_heap[(size_t)s.my_pe] = base;
    s.p2p_ready = s.n_pes == 1;
    if (!s.want_p2p || s.n_pes == 1) return;
    if (!s.hub.up) raise_error("SHMEMX_TRANSPORT=p2p needs the shmem_init bootstrap");
    // p2p-only mode cannot run without the mapping; in `both` mode a failure on any PE
    // turns the p2p transport off on every PE (agreed through the hub)
    const bool fatal = s.transport == TRANSPORT_P2P;
    if (s.ext_base && ipc_size_bug && (s.dev_heap_bytes & 0x80000000ull)) {
        // an external heap of such a size cannot be mapped on this runtime
        if (fatal)
            raise_error("shmemx_heap_create: a %zu-byte external heap cannot be IPC-mapped by HIP "
                        "runtime %d (sizes with bit 31 set hang before 7.2); use another size",
                        s.dev_heap_bytes, rtv);
        warn("external heap of %zu B cannot be IPC-mapped by HIP %d: p2p transport off",
             s.dev_heap_bytes, rtv);
        return;
    }
    struct Export { hipIpcMemHandle_t h; int device; } mine;
    memset(&mine, 0, sizeof(mine));
    mine.device = s.device;
    hipError_t e = hipIpcGetMemHandle(&mine.h, base);
    if (e != hipSuccess && fatal) hip_check(e, "hipIpcGetMemHandle(device heap)");
    debug_msg("device heap: IPC handle %s", e == hipSuccess ? "ok" : hipGetErrorString(e));
    std::vector<Export> all((size_t)s.n_pes);
    if (sosboot::hub_allgather(&s.hub, &mine, sizeof(mine), all.data()) != 0)
        raise_error("device heap: IPC handle exchange failed");
    int ok = e == hipSuccess;
    for (int q = 0; q < s.n_pes && ok; ++q) {
        if (q == s.my_pe) continue;
        // a heap on another GPU (device ordinals are node-global: one process per GPU,
        // no HIP_VISIBLE_DEVICES remapping) is read in place only with peer access
        const int pd = all[(size_t)q].device;
        int can = 1;
        if (pd != s.device && (hipDeviceCanAccessPeer(&can, s.device, pd) != hipSuccess || !can)) {
            (void)hipGetLastError();
            if (fatal)
                raise_error("p2p transport: GPU %d cannot access PE %d's GPU %d (hipDeviceCanAccessPeer)",
                            s.device, q, pd);
            warn("GPU %d cannot access PE %d's GPU %d: p2p transport off", s.device, q, pd);
            ok = 0;
            break;
        }
        void *p = nullptr;
        debug_msg("device heap: opening PE %d's handle (GPU %d)", q, pd);
        hipError_t eo = hipIpcOpenMemHandle(&p, all[(size_t)q].h, kP2PIpcOpenFlags);
        debug_msg("device heap: PE %d mapped at %p (%s)", q, p, hipGetErrorString(eo));
        if (eo != hipSuccess) {
            if (fatal) hip_check(eo, "hipIpcOpenMemHandle(peer device heap)");
            (void)hipGetLastError();
            warn("cannot map PE %d's device heap (%s): p2p transport off", q, hipGetErrorString(eo));
            ok = 0;
            break;
        }
        s.peer_heap[(size_t)q] = (char *)p;
    }
    std::vector<int> oks((size_t)s.n_pes);
    if (sosboot::hub_allgather(&s.hub, &ok, sizeof(ok), oks.data()) != 0)
        raise_error("device heap: mapping agreement failed");
    for (int v : oks) ok &= v;
    if (!ok) {
        for (int q = 0; q < s.n_pes; ++q)
            if (q != s.my_pe && s.peer_heap[(size_t)q]) {
                (void)hipIpcCloseMemHandle(s.peer_heap[(size_t)q]);
                s.peer_heap[(size_t)q] = nullptr;
            }
        return;
    }
    s.p2p_ready = true;
    debug_msg("device heap %zu B (stage %zu B) mapped on %d PEs", s.dev_heap_bytes,
              s.sym_stage_bytes, s.n_pes);
    p2p_signal_setup();
}

// ---------------------------------------------------------------------------------
// device workspaces
// ---------------------------------------------------------------------------------
static void *grow(void **buf, size_t *have, size_t need, const char *what)
{
    if (need <= *have && *buf) return *buf;
    State &s = st();
    if (*buf) {
        hip_check(hipStreamSynchronize(s.stream), "hipStreamSynchronize");
        hip_check(hipFree(*buf), "hipFree");
        *buf = nullptr;
    }
    size_t sz = need < (1u << 20) ? (1u << 20) : need;
    hip_check(hipMalloc(buf, sz), what);
    *have = sz;
    return *buf;
}

hipError_t release_system(hipStream_t stream)
{
    State &s = st();
    if (!s.sys_ev) {
        const hipError_t e =
            hipEventCreateWithFlags(&s.sys_ev, hipEventReleaseToSystem | hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    ++s.sys_releases;
    return hipEventRecord(s.sys_ev, stream);
}

hipError_t acquire_system(hipStream_t stream)
{
    State &s = st();
    if (!s.acq_mask) {
        hipError_t e = hipMalloc(&s.acq_mask, sizeof(unsigned));
        if (e == hipSuccess) e = hipMemsetAsync(s.acq_mask, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
    }
    ++s.sys_acquires;
    ++s.acquire_kernels;
    s.acq_pending = false;
    return sosx_acquire_system(s.acq_mask, stream) == SOSX_OK ? hipSuccess : hipErrorLaunchFailure;
}

void note_peer_wait() { st().acq_pending = true; }

void note_peer_read(bool own_acquire)
{
    State &s = st();
    ++s.peer_reads;
    if (own_acquire) ++s.sys_acquires;
    else if (s.acq_pending) ++s.peer_reads_unacquired;
}

// The release event, then a stream synchronisation: it waits for the event too, and
// costs what a plain hipStreamSynchronize does, 1.5-4.5 us less per call than waiting on
// the event itself (profiles/r5_sync_cost.json).  Test build only: SOSX_TEST_EVENT_WAIT=1
// waits with hipEventSynchronize, as round 5 first did (the A/B in
// profiles/r5_p2p_small_call_ab.txt: 0.3-1 us per p2p call with two PEs on one GPU).
hipError_t sync_system(hipStream_t stream)
{
    hipError_t e = release_system(stream);
#ifdef SOSX_TEST_HOOKS
    static const bool event_wait = [] {
        const char *v = getenv("SOSX_TEST_EVENT_WAIT");
        return v && *v == '1';
    }();
    if (event_wait) return e == hipSuccess ? hipEventSynchronize(st().sys_ev) : e;
#endif
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e;
}

void *scratch(size_t bytes) { return grow(&st().scratch, &st().scratch_bytes, bytes, "hipMalloc(scratch)"); }
void *stage(size_t bytes) { return grow(&st().stage, &st().stage_bytes, bytes, "hipMalloc(stage)"); }

bool is_device_ptr(const void *p)
{
    if (!p) return false;
    // the symmetric regions this library created answer without a runtime query (a
    // hipPointerGetAttributes costs about a microsecond; every call asks for two)
    State &s = st();
    const char *c = (const char *)p;
    if (s.dev_heap.contains(p, 1) || (s.sym_stage && c >= s.sym_stage && c < s.sym_stage + s.sym_stage_bytes))
        return true;
    if (s.ext_base && c >= (char *)s.ext_base && c < (char *)s.ext_base + s.ext_size) return true;
    if (s.host_heap.contains(p, 1)) return false;
    if (__data_start && _end && c >= __data_start && c < _end) return false;
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // pageable host memory: not registered with HIP
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

bool is_local_device_ptr(const void *p)
{
    State &s = st();
    const char *c = (const char *)p;
    if (!p) return false;
    if (s.dev_heap.contains(p, 1) || (s.ext_base && c >= (char *)s.ext_base && c < (char *)s.ext_base + s.ext_size))
        return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice && a.device == s.device;
}

bool is_symmetric(const void *p, size_t bytes)
{
    State &s = st();
    if (s.host_heap.contains(p, bytes) || s.dev_heap.contains(p, bytes)) return true;
    if (__data_start && _end && (const char *)p >= __data_start && (const char *)p + bytes <= _end)
        return true;
    for (auto &kv : s.dev_allocs)
        if ((const char *)p >= (char *)kv.first && (const char *)p + bytes <= (char *)kv.first + kv.second)
            return true;
    if (s.ext_base && (const char *)p >= (char *)s.ext_base &&
        (const char *)p + bytes <= (char *)s.ext_base + s.ext_size)
        return true;
    return false;
}

// ---------------------------------------------------------------------------------
// barriers: dissemination over RCCL point-to-point (ceil(log2 P) rounds), so any
// strided team can synchronise without a communicator of its own
// ---------------------------------------------------------------------------------
void team_barrier(const Team &t)
{
    State &s = st();
    if (s.shm.base) {
        // node-local: the stream first (SOS barrier also completes outstanding work),
        // then the shared-memory arrival counters of this member set
        hip_check(sync_system(s.stream), "hipStreamSynchronize(barrier)");
        if (t.size > 1 && t.my_idx >= 0 && !s.shm.wait(t.start, t.stride, t.size, 600.0))
            raise_error("barrier timed out (team start %d stride %d size %d)", t.start, t.stride,
                        t.size);
        return;
    }
    if (t.size > 1 && t.my_idx >= 0) {
        for (int d = 1; d < t.size; d <<= 1) {
            const int to = t.world_rank((t.my_idx + d) % t.size);
            const int from = t.world_rank((t.my_idx - d + t.size) % t.size);
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            nccl_check(ncclSend(s.dbar, 1, ncclInt32, to, s.comm, s.stream), "ncclSend(barrier)");
            nccl_check(ncclRecv(s.dbar + 1, 1, ncclInt32, from, s.comm, s.stream), "ncclRecv(barrier)");
            nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        }
    }
    hip_check(sync_system(s.stream), "hipStreamSynchronize(barrier)");
}

Team *team_from_handle(shmem_team_t handle) { return reinterpret_cast<Team *>(handle); }

// ---------------------------------------------------------------------------------
// init (src/init.c:221-567, condensed to what the reduction path needs)
// ---------------------------------------------------------------------------------
// The shared segment's p2p region, rounded to whole pages (the small-path region
// follows it, so the two HIP registrations never share a page).
static size_t shm_p2p_region_bytes() { return (p2p_shared_bytes() + 4095) & ~(size_t)4095; }

static void init_common(int pe, int npes, const ncclUniqueId *uid)
{
    State &s = st();
    s.my_pe = pe;
    s.n_pes = npes;
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev < 1) raise_error("no AMD GPU visible: this SOS build runs the reduction path on HIP");
    const char *dv = getenv("SHMEMX_DEVICE");
    s.device = dv ? atoi(dv) : sosboot::local_rank(pe) % ndev;
    hip_check(hipSetDevice(s.device), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&s.own_stream, hipStreamNonBlocking), "hipStreamCreate");
    s.stream = s.own_stream;
    hip_check(hipMalloc((void **)&s.dbar, 64), "hipMalloc(barrier word)");
    hip_check(hipMemset(s.dbar, 0, 64), "hipMemset");
    if (uid) {
        const ncclResult_t r = ncclCommInitRank(&s.comm, npes, *uid, pe);
        // SHMEMX_TRANSPORT=both: an RCCL communicator that fails to come up leaves the
        // job on the p2p transport (agreed over the bootstrap, so every PE switches)
        const bool can_fall_back = s.want_p2p && s.hub.up && npes > 1;
        if (r != ncclSuccess && !can_fall_back) nccl_check(r, "ncclCommInitRank");
        if (r != ncclSuccess) {
            warn("RCCL communicator init failed (%s)", ncclGetErrorString(r));
            s.comm = nullptr;
        }
        if (can_fall_back) {
            int ok = s.comm != nullptr;
            std::vector<int> oks((size_t)npes);
            if (sosboot::hub_allgather(&s.hub, &ok, sizeof(ok), oks.data()) != 0)
                raise_error("shmem_init: RCCL status agreement failed");
            for (int v : oks) ok &= v;
            if (!ok) {
                if (s.comm) (void)ncclCommDestroy(s.comm);
                s.comm = nullptr;
                s.want_rccl = false;
                s.transport = TRANSPORT_P2P;
                warn("RCCL unavailable on some PE: every PE runs on the p2p transport");
            }
        }
    }
    s.world = Team();
    s.world.start = 0;
    s.world.stride = 1;
    s.world.size = npes;
    s.world.my_idx = pe;
    s.world.valid = true;
    s.world.predefined = true;
    s.world.psync_idx = 0;
    s.shared = s.world;  // one node: every PE shares it (src/shmem_team.c:88-140)
    s.shared.psync_idx = 1;
    s.node = s.world;    // SHMEMX_TEAM_NODE (:101-164)
    s.node.psync_idx = 2;
    SHMEM_TEAM_WORLD = team_handle(&s.world);
    SHMEM_TEAM_SHARED = team_handle(&s.shared);
    SHMEMX_TEAM_NODE = team_handle(&s.node);
    // team slots (src/shmem_team.c:171-226): 64 at most, 3 at least, 0..2 predefined
    if (s.teams_max > 64) raise_error("Requested %ld teams, but only 64 are supported", s.teams_max);
    if (s.teams_max < 3) s.teams_max = 3;
    s.team_avail = 0;
    for (long i = 3; i < s.teams_max; ++i) s.team_avail |= 1ull << i;
    s.team_pool.assign((size_t)s.teams_max, nullptr);
    s.initialized = true;
    s.finalized = false;
    register_data_segment(s);
    if (s.want_p2p || s.ext_base) ensure_device_heap();
    if (s.shm.extra && npes > 1)
        small_path_setup((char *)s.shm.extra + shm_p2p_region_bytes(), small_shared_bytes(npes));
    if (pe == 0 && (env_flag("VERSION") || env_flag("INFO") || s.debug)) {
        printf("Sandia OpenSHMEM 1.5.3 (MI355X reduction path, libsos_amd)\n");
        if (env_flag("INFO")) print_env();
        fflush(stdout);
    }
    debug_msg("PE %d of %d on device %d, transport %s, reduce algorithm %d, crossover %zu", pe,
              npes, s.device, s.transport == TRANSPORT_P2P ? "p2p" : "rccl", s.reduce_alg,
              s.coll_size_crossover);
    team_barrier(s.world);
}

}  // namespace sosrt

using namespace sosrt;

extern "C" {

void shmem_init(void)
{
    State &s = st();
    if (s.initialized) return;
    read_env(s);
    int rank, size;
    sosboot::discover(&rank, &size);
    s.my_pe = rank;
    char err[256] = {0};
    if (sosboot::hub_connect(&s.hub, rank, size, err, sizeof(err)) != 0)
        raise_error("shmem_init: %s", err);
    // PE 0 decides the transport, creates the RCCL id and names the shm segment
    struct Blob {
        ncclUniqueId uid;
        char shm_name[64];
        int transport, want_rccl, want_p2p;
    } blob;
    memset(&blob, 0, sizeof(blob));
    if (rank == 0) {
        blob.transport = s.transport;
        blob.want_rccl = s.want_rccl;
        blob.want_p2p = s.want_p2p;
        // one PE has no peers: no communicator (RCCL's init also prints a banner to stdout)
        if (blob.want_rccl && size > 1) nccl_check(ncclGetUniqueId(&blob.uid), "ncclGetUniqueId");
        snprintf(blob.shm_name, sizeof(blob.shm_name), "/sosx_%d_%lx", (int)getpid(),
                 (unsigned long)time(nullptr));
    }
    if (sosboot::hub_bcast(&s.hub, &blob, sizeof(blob)) != 0) raise_error("shmem_init: bootstrap broadcast failed");
    s.transport = blob.transport;
    s.want_rccl = blob.want_rccl;
    s.want_p2p = blob.want_p2p;
    char host[64] = {0};
    gethostname(host, sizeof(host) - 1);
    std::string recs((size_t)size * sizeof(host), '\0');
    if (sosboot::hub_allgather(&s.hub, host, sizeof(host), &recs[0]) != 0)
        raise_error("shmem_init: bootstrap all-gather failed");
    for (int r = 0; r < size; ++r)
        if (strncmp(&recs[(size_t)r * sizeof(host)], host, sizeof(host)) != 0)
            raise_error("shmem_init: PE %d runs on another node; this build is single-node "
                        "(one PE per MI355X over xGMI)", r);
    if (size > 1) {
        // node-local shared memory: barriers + peer-to-peer transport counters
        int dummy = 0;
        std::vector<int> all((size_t)size);
        // [p2p counters | small-path control words and slots] after the barrier slots
        const size_t extra = shm_p2p_region_bytes() + small_shared_bytes(size);
        if (rank == 0 && !s.shm.attach(blob.shm_name, true, rank, extra))
            raise_error("shmem_init: cannot create shared memory %s", blob.shm_name);
        sosboot::hub_allgather(&s.hub, &dummy, sizeof(dummy), all.data());
        if (rank != 0 && !s.shm.attach(blob.shm_name, false, rank, extra))
            raise_error("shmem_init: cannot attach shared memory %s", blob.shm_name);
        sosboot::hub_allgather(&s.hub, &dummy, sizeof(dummy), all.data());
        if (rank == 0) shm_unlink(blob.shm_name);
    }
    init_common(rank, size, s.want_rccl && size > 1 ? &blob.uid : nullptr);
}

int shmem_init_thread(int requested, int *provided)
{
    shmem_init();
    // collectives are serialised by the caller, as in SOS (pSync selection is unlocked)
    st().thread_level = requested > SHMEM_THREAD_SERIALIZED ? SHMEM_THREAD_SERIALIZED : requested;
    if (provided) *provided = st().thread_level;
    return 0;
}

void shmem_query_thread(int *provided)
{
    if (provided) *provided = st().thread_level;
}

int shmemx_get_unique_id(void *uid, size_t len)
{
    if (!uid || len < sizeof(ncclUniqueId)) return SOSX_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SOSX_ERR_RCCL;
    memcpy(uid, &id, sizeof(id));
    return SOSX_OK;
}

int shmemx_init_attr(int my_pe, int n_pes, const void *uid, size_t len)
{
    if (st().initialized) return SOSX_ERR_STATE;
    if (!uid || len < sizeof(ncclUniqueId) || n_pes < 1 || my_pe < 0 || my_pe >= n_pes)
        return SOSX_ERR_ARG;
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    State &s = st();
    read_env(s);
    s.my_pe = my_pe;
    if (s.want_p2p) {
        warn("SHMEMX_TRANSPORT=p2p/both needs the shmem_init bootstrap; using RCCL only");
        s.transport = TRANSPORT_RCCL;
        s.want_p2p = false;
    }
    s.want_rccl = true;
    init_common(my_pe, n_pes, &id);
    return SOSX_OK;
}

void shmem_finalize(void)
{
    State &s = st();
    if (!s.initialized) return;
    team_barrier(s.world);
    // destroy the teams the program left (src/shmem_team.c:238-247)
    for (size_t i = 3; i < s.team_pool.size(); ++i)
        if (s.team_pool[i]) {
            s.team_pool[i]->valid = false;
            delete s.team_pool[i];
            s.team_pool[i] = nullptr;
        }
    if (s.comm) ncclCommDestroy(s.comm);
    s.comm = nullptr;
    if (s.scratch) (void)hipFree(s.scratch);
    if (s.stage) (void)hipFree(s.stage);
    if (s.dbar) (void)hipFree(s.dbar);
    s.scratch = s.stage = nullptr;
    s.scratch_bytes = s.stage_bytes = 0;
    s.dbar = nullptr;
    sosx_combine_host_release();
    small_local_release();
    if (s.stripes) (void)hipFree(s.stripes);
    s.stripes = nullptr;
    s.stripes_bytes = 0;
    for (auto &slot : s.pipe_ev)
        for (hipEvent_t &e : slot) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
    if (s.sys_ev) (void)hipEventDestroy(s.sys_ev);
    s.sys_ev = nullptr;
    unregister_data_segment(s);
    if (s.acq_mask) (void)hipFree(s.acq_mask);
    s.acq_mask = nullptr;
    for (hipStream_t *ps : {&s.pipe_h2d, &s.pipe_d2h}) {
        if (*ps) (void)hipStreamDestroy(*ps);
        *ps = nullptr;
    }
    if (s.host_heap.base) (void)hipHostFree(s.host_heap.base);
    for (size_t q = 0; q < s.peer_heap.size(); ++q)
        if ((int)q != s.my_pe && s.peer_heap[q]) (void)hipIpcCloseMemHandle(s.peer_heap[q]);
    s.peer_heap.clear();
    if (s.sym_stage && !s.dev_heap.external) (void)hipFree(s.sym_stage);
    s.sym_stage = nullptr;
    s.host_heap = Heap();
    s.dev_heap = Heap();
    p2p_signal_teardown();
    small_path_teardown();
    s.shm.detach();
    sosboot::hub_close(&s.hub);
    for (auto &kv : s.dev_allocs) (void)hipFree(kv.first);
    s.dev_allocs.clear();
    if (s.own_stream) (void)hipStreamDestroy(s.own_stream);
    s.own_stream = s.stream = nullptr;
    s.initialized = false;
    s.finalized = true;
}

void shmem_global_exit(int status)
{
    fflush(stdout);
    fflush(stderr);
    _exit(status);
}

int shmem_my_pe(void) { return st().initialized ? st().my_pe : -1; }
int shmem_n_pes(void) { return st().initialized ? st().n_pes : -1; }

int shmem_pe_accessible(int pe) { return st().initialized && pe >= 0 && pe < st().n_pes; }

int shmem_addr_accessible(const void *addr, int pe)
{
    return shmem_pe_accessible(pe) && is_symmetric(addr, 1);
}

void shmem_info_get_version(int *major, int *minor)
{
    if (major) *major = SHMEM_MAJOR_VERSION;
    if (minor) *minor = SHMEM_MINOR_VERSION;
}

void shmem_info_get_name(char *name)
{
    if (name) {
        strncpy(name, SHMEM_VENDOR_STRING, SHMEM_MAX_NAME_LEN - 1);
        name[SHMEM_MAX_NAME_LEN - 1] = 0;
    }
}

// ---- symmetric memory (src/symmetric_heap_c.c:285-432: allocation + barrier) ----
void *shmem_malloc(size_t size)
{
    check_initialized("shmem_malloc");
    State &s = st();
    void *p;
    {
        std::lock_guard<std::mutex> g(s.mu);
        if (s.heap_on_device) {
            ensure_device_heap();
            p = s.dev_heap.alloc(size, 256);
        } else {
            ensure_host_heap(s);
            p = s.host_heap.alloc(size, 256);
        }
    }
    if (!p && size)
        raise_error("shmem_malloc(%zu): symmetric heap exhausted (SHMEM_SYMMETRIC_SIZE=%zu)", size,
                    s.symmetric_size);
    team_barrier(s.world);
    return p;
}

void *shmem_calloc(size_t count, size_t size)
{
    void *p = shmem_malloc(count * size);
    if (p) {
        if (st().heap_on_device)
            hip_check(hipMemset(p, 0, count * size), "hipMemset");
        else
            memset(p, 0, count * size);
    }
    return p;
}

void *shmem_align(size_t alignment, size_t size)
{
    check_initialized("shmem_align");
    State &s = st();
    if (alignment == 0 || (alignment & (alignment - 1))) return nullptr;
    void *p;
    {
        std::lock_guard<std::mutex> g(s.mu);
        Heap &h = s.heap_on_device ? s.dev_heap : s.host_heap;
        if (s.heap_on_device) ensure_device_heap(); else ensure_host_heap(s);
        p = h.alloc(size, alignment);
    }
    team_barrier(s.world);
    return p;
}

void shmem_free(void *ptr)
{
    if (!ptr) return;
    check_initialized("shmem_free");
    State &s = st();
    team_barrier(s.world);
    std::lock_guard<std::mutex> g(s.mu);
    if (!s.host_heap.release(ptr) && !s.dev_heap.release(ptr))
        raise_error("shmem_free: %p is not a symmetric heap address", ptr);
}

void *shmem_realloc(void *ptr, size_t size)
{
    if (!ptr) return shmem_malloc(size);
    if (size == 0) {
        shmem_free(ptr);
        return nullptr;
    }
    State &s = st();
    Heap &h = s.host_heap.contains(ptr, 1) ? s.host_heap : s.dev_heap;
    size_t old = 0;
    {
        auto it = h.used_blocks.find((size_t)((char *)ptr - h.base));
        if (it == h.used_blocks.end()) raise_error("shmem_realloc: %p is not a heap address", ptr);
        old = it->second;
    }
    void *np = shmem_malloc(size);
    size_t n = old < size ? old : size;
    if (h.device)
        hip_check(hipMemcpy(np, ptr, n, hipMemcpyDeviceToDevice), "hipMemcpy");
    else
        memcpy(np, ptr, n);
    shmem_free(ptr);
    return np;
}

void *shmemx_malloc_device(size_t size)
{
    check_initialized("shmemx_malloc_device");
    State &s = st();
    void *p = nullptr;
    ensure_device_heap();  // collective, like the call itself
    {
        std::lock_guard<std::mutex> g(s.mu);
        p = s.dev_heap.alloc(size, 256);
    }
    if (!p && size)
        raise_error("shmemx_malloc_device(%zu): device heap exhausted (SHMEMX_DEVICE_HEAP_SIZE=%zu)",
                    size, s.dev_heap_bytes);
    team_barrier(s.world);
    return p;
}

void shmemx_free_device(void *ptr)
{
    if (!ptr) return;
    State &s = st();
    team_barrier(s.world);
    std::lock_guard<std::mutex> g(s.mu);
    if (!s.dev_heap.release(ptr))
        raise_error("shmemx_free_device: %p was not allocated by shmemx_malloc_device", ptr);
}

void shmemx_heap_create(void *base, size_t size, int device_type, int device_index)
{
    State &s = st();
    if (s.initialized) {
        warn("Ignoring pre-setup. Heap already initialized");
        return;
    }
    if (!base || size == 0 || device_type != SHMEMX_EXTERNAL_HEAP_HIP)
        raise_error("shmemx_heap_create: this build accepts HIP device heaps "
                    "(SHMEMX_EXTERNAL_HEAP_HIP) only");
    (void)device_index;
    s.ext_base = base;
    s.ext_size = size;
    s.ext_type = device_type;
}

void shmemx_set_stream(void *hip_stream)
{
    State &s = st();
    s.stream = hip_stream ? (hipStream_t)hip_stream : s.own_stream;
}

void *shmemx_get_stream(void) { return (void *)st().stream; }

int shmemx_get_device(void) { return st().device; }

int shmemx_set_transport(int transport)
{
    State &s = st();
    const int prev = s.transport;
    if (transport == TRANSPORT_RCCL && (s.comm || s.n_pes == 1)) s.transport = TRANSPORT_RCCL;
    else if (transport == TRANSPORT_P2P && s.p2p_ready && (s.shm.base || s.n_pes == 1))
        s.transport = TRANSPORT_P2P;
    else return -1;
    return prev;
}

// RCCL executor: run equal-chunk allgather rounds of world-team plans as ncclAllGather
// (1) or as grouped send/receive pairs (0, the default).  Same bytes either way; every
// PE must switch at the same point of its call sequence.  Returns the previous setting.
int sosx_set_rccl_allgather(int on)
{
    State &s = st();
    const int prev = s.rccl_allgather ? 1 : 0;
    s.rccl_allgather = on != 0;
    return prev;
}

// The rank count RCCL's own communicator reports (ncclCommCount), or -1 when this job has
// no RCCL communicator (p2p-only, or one PE): what a bench line names so a reader can see
// that RCCL, and not only the launcher, saw every PE.
int sosx_rccl_comm_count(void)
{
    State &s = st();
    int n = -1;
    if (!s.comm || ncclCommCount(s.comm, &n) != ncclSuccess) return -1;
    return n;
}

// How many system-scope completion markers (sync_system / release_system) this PE has
// issued: every call that returns data ends with one (introspection for tests).
long sosx_sys_releases(void) { return st().sys_releases; }

// The executable's data segment as registered with HIP at shmem_init (null / 0: not
// registered: SHMEMX_REGISTER_DATA=0, or HIP refused it).
size_t sosx_data_segment(void **base)
{
    if (base) *base = st().data_reg;
    return st().data_reg_bytes;
}

void sosx_acquire_stats(long *acquires, long *peer_reads, long *unacquired, unsigned *xcc_mask)
{
    State &s = st();
    if (acquires) *acquires = s.sys_acquires;
    if (peer_reads) *peer_reads = s.peer_reads;
    if (unacquired) *unacquired = s.peer_reads_unacquired;
    if (xcc_mask) {
        *xcc_mask = 0;
        if (s.acq_mask && s.stream && hipStreamSynchronize(s.stream) == hipSuccess)
            (void)hipMemcpy(xcc_mask, s.acq_mask, sizeof(unsigned), hipMemcpyDeviceToHost);
    }
}

long sosx_acquire_kernels(void) { return st().acquire_kernels; }

// Return this PE's private device workspaces (exchange scratch, staging for host
// operands) to the runtime after the library stream drains; the next call that needs one
// allocates it afresh.  Local, not collective.  Returns the bytes released.
size_t sosx_release_workspaces(void)
{
    State &s = st();
    if (!s.initialized) return 0;
    hip_check(hipStreamSynchronize(s.stream), "hipStreamSynchronize");
    const size_t had = (s.scratch ? s.scratch_bytes : 0) + (s.stage ? s.stage_bytes : 0);
    if (s.scratch) hip_check(hipFree(s.scratch), "hipFree(scratch)");
    if (s.stage) hip_check(hipFree(s.stage), "hipFree(stage)");
    s.scratch = s.stage = nullptr;
    s.scratch_bytes = s.stage_bytes = 0;
    return had;
}

// RCCL executor: world-team reductions as one ncclAllReduce where RCCL has the type and
// op (0 off, the default; 1 integer sum/prod/min/max, bit-exact; 2 also fp32/fp64
// sum/prod, within the fp tolerance of DESIGN.md section 5).  Collective; returns the
// previous mode, or -1 for a mode out of range.
int sosx_set_rccl_allreduce(int mode)
{
    State &s = st();
    if (mode < 0 || mode > 2) return -1;
    const int prev = s.rccl_allreduce;
    s.rccl_allreduce = mode;
    return prev;
}

int shmemx_set_reduce_algorithm(int alg)
{
    int prev = st().reduce_alg;
    if (alg >= SOSX_ALG_AUTO && alg <= SOSX_ALG_RECDBL_GATHER) st().reduce_alg = alg;
    return prev;
}

// ---- synchronisation -------------------------------------------------------------
void shmem_barrier_all(void)
{
    check_initialized("shmem_barrier_all");
    team_barrier(st().world);
}

void shmem_sync_all(void) { shmem_barrier_all(); }

void shmem_quiet(void)
{
    if (st().initialized) hip_check(sync_system(st().stream), "hipStreamSynchronize");
}

void shmem_fence(void) { shmem_quiet(); }

static Team active_set(int PE_start, int logPE_stride, int PE_size, const char *fn)
{
    State &s = st();
    const int stride = 1 << logPE_stride;
    // SHMEM_ERR_CHECK_ACTIVE_SET (src/shmem_internal.h:214-227).  SOS tests the last PE
    // with `> num_pes`, which admits PE num_pes (no such PE: SOS then waits on it forever);
    // here that set is refused, since a transfer to it would index past the PE tables.
    if (PE_start < 0 || stride < 1 || PE_size < 0 || PE_start + ((PE_size - 1) * stride) >= s.n_pes)
        raise_error("%s: Invalid active set (PE_start = %d, PE_stride = %d, PE_size = %d)", fn,
                    PE_start, stride, PE_size);
    if (!(s.my_pe >= PE_start && s.my_pe <= PE_start + ((PE_size - 1) * stride) &&
          (s.my_pe - PE_start) % stride == 0))
        raise_error("%s: Calling PE (%d) is not a member of the active set", fn, s.my_pe);
    Team t;
    t.start = PE_start;
    t.stride = stride;
    t.size = PE_size;
    t.my_idx = (s.my_pe - PE_start) / stride;
    t.valid = true;
    return t;
}

void shmem_sync(int PE_start, int logPE_stride, int PE_size, long *pSync)
{
    check_initialized("shmem_sync");
    (void)pSync;
    team_barrier(active_set(PE_start, logPE_stride, PE_size, "shmem_sync"));
}

void shmem_barrier(int PE_start, int logPE_stride, int PE_size, long *pSync)
{
    shmem_sync(PE_start, logPE_stride, PE_size, pSync);
}

// ---- teams (src/shmem_team.c, src/teams_c.c4) -------------------------------------
static Team *team_checked(shmem_team_t team, const char *fn)
{
    check_initialized(fn);
    Team *t = team_from_handle(team);
    if (!t || !t->valid) raise_error("%s: invalid team", fn);  // SHMEM_ERR_CHECK_TEAM_VALID
    return t;
}

int shmem_team_my_pe(shmem_team_t team)
{
    if (team == SHMEM_TEAM_INVALID) return -1;
    return team_checked(team, "shmem_team_my_pe")->my_idx;
}

int shmem_team_n_pes(shmem_team_t team)
{
    if (team == SHMEM_TEAM_INVALID) return -1;
    return team_checked(team, "shmem_team_n_pes")->size;
}

int shmem_team_get_config(shmem_team_t team, long config_mask, shmem_team_config_t *config)
{
    // src/teams_c.c4:76-100
    check_initialized("shmem_team_get_config");
    if (team == SHMEM_TEAM_INVALID) return -1;
    Team *t = team_checked(team, "shmem_team_get_config");
    if (config_mask != 0) {
        if (config_mask != SHMEM_TEAM_NUM_CONTEXTS) {
            warn("Invalid team config mask (%ld)", config_mask);
            return -1;
        }
        if (!config) {
            warn("NULL config pointer passed to shmem_team_get_config");
            return -1;
        }
        config->num_contexts = t->num_contexts;
    } else if (config) {
        warn("shmem_team_get_config encountered an unexpected non-NULL config structure "
             "passed with a config_mask of 0.");
    }
    return 0;
}

int shmem_team_translate_pe(shmem_team_t src_team, int src_pe, shmem_team_t dest_team)
{
    // src/shmem_team.c:262-283
    check_initialized("shmem_team_translate_pe");
    if (src_team == SHMEM_TEAM_INVALID || dest_team == SHMEM_TEAM_INVALID) return -1;
    Team *s = team_checked(src_team, "shmem_team_translate_pe");
    Team *d = team_checked(dest_team, "shmem_team_translate_pe");
    if (src_pe < 0 || src_pe >= s->size) return -1;
    const int off = s->world_rank(src_pe) - d->start;  // shmem_internal_pe_in_active_set
    if ((d->stride > 0 ? off < 0 : off > 0) || off % d->stride) return -1;
    const int idx = off / d->stride;
    return idx < d->size ? idx : -1;
}

// All-gather of one 64-bit word per member of team `t` over RCCL (the path without node
// shared memory, e.g. shmemx_init_attr): grouped ncclSend/ncclRecv with every other
// member, one word each way.  Collective over `t`; returns the words in team order.
static std::vector<uint64_t> team_allgather_word(const Team &t, uint64_t mine)
{
    State &s = st();
    std::vector<uint64_t> out((size_t)t.size, 0);
    out[(size_t)t.my_idx] = mine;
    if (t.size <= 1) return out;
    uint64_t *d = nullptr;
    hip_check(hipMalloc(&d, (size_t)t.size * sizeof(uint64_t)), "hipMalloc(team words)");
    hip_check(hipMemcpyAsync(d + t.my_idx, &mine, sizeof mine, hipMemcpyHostToDevice, s.stream),
              "team words H2D");
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int i = 0; i < t.size; ++i) {
        if (i == t.my_idx) continue;
        nccl_check(ncclSend(d + t.my_idx, sizeof mine, ncclUint8, t.world_rank(i), s.comm, s.stream),
                   "ncclSend(team words)");
        nccl_check(ncclRecv(d + i, sizeof mine, ncclUint8, t.world_rank(i), s.comm, s.stream),
                   "ncclRecv(team words)");
    }
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    hip_check(hipMemcpyAsync(out.data(), d, out.size() * sizeof(uint64_t), hipMemcpyDeviceToHost,
                             s.stream), "team words D2H");
    hip_check(hipStreamSynchronize(s.stream), "hipStreamSynchronize(team words)");
    hip_check(hipFree(d), "hipFree(team words)");
    return out;
}

// Team creation agreement over the parent (src/shmem_team.c:354-432): the members AND
// their free-slot masks and take the lowest common slot; every parent PE then returns
// the MAX of the members' status, so all agree.  Node shared memory carries the words;
// without it (shmemx_init_attr) they are all-gathered over RCCL.
static int team_agree_slot(const Team &parent, const Team &child, bool member, int *slot)
{
    State &s = st();
    *slot = -1;
    if (parent.size <= 1 || !s.shm.extra) {
        // non-members contribute all ones, the neutral word of the AND
        uint64_t all = s.team_avail;
        if (parent.size > 1)
            for (uint64_t w : team_allgather_word(parent, member ? s.team_avail : ~0ull)) all &= w;
        int status = 0;
        if (member) {
            const int idx = all ? __builtin_ctzll(all) : -1;
            if (idx < 0 || idx >= s.teams_max) {
                warn("No more teams available (max = %ld), try increasing SHMEM_TEAMS_MAX",
                     s.teams_max);
                status = 1;
            } else {
                *slot = idx;
            }
        }
        if (parent.size <= 1) return status;
        int agreed = 0;
        for (uint64_t w : team_allgather_word(parent, (uint64_t)status))
            agreed = std::max(agreed, (int)w);
        return agreed;
    }
    const int me_world = s.my_pe;
    team_word_put(0, me_world, member ? s.team_avail : 0);
    team_barrier(parent);
    int status = 0;
    if (member) {
        uint64_t all = s.team_avail;
        for (int i = 0; i < child.size; ++i) all &= team_word_get(0, child.world_rank(i));
        const int idx = all ? __builtin_ctzll(all) : -1;
        if (idx < 0 || idx >= s.teams_max) {
            warn("No more teams available (max = %ld), try increasing SHMEM_TEAMS_MAX", s.teams_max);
            status = 1;
        } else {
            *slot = idx;
        }
    }
    team_word_put(1, me_world, (uint64_t)status);
    team_barrier(parent);
    int agreed = 0;
    for (int i = 0; i < parent.size; ++i)
        agreed = std::max(agreed, (int)team_word_get(1, parent.world_rank(i)));
    return agreed;
}

int shmem_team_split_strided(shmem_team_t parent_team, int PE_start, int PE_stride, int PE_size,
                             const shmem_team_config_t *config, long config_mask,
                             shmem_team_t *new_team)
{
    check_initialized("shmem_team_split_strided");
    if (new_team) *new_team = SHMEM_TEAM_INVALID;
    if (parent_team == SHMEM_TEAM_INVALID) return 1;  // src/shmem_team.c:296-298
    Team *parent = team_checked(parent_team, "shmem_team_split_strided");
    State &s = st();
    // argument rules of src/shmem_team.c:300-321: a stride of 0 (or a 1-PE team) is 1,
    // and the child's first/last PE must be valid world PEs; no collective on error
    PE_stride = (PE_stride == 0 || PE_size == 1) ? 1 : PE_stride;
    if (PE_start < 0 || PE_start >= parent->size || PE_size <= 0 || PE_size > parent->size) {
        warn("Invalid <start, stride, size>: child <%d, %d, %d>, parent <%d, %d, %d>", PE_start,
             PE_stride, PE_size, parent->start, parent->stride, parent->size);
        return -1;
    }
    const int gstart = parent->world_rank(PE_start);
    const int gstride = parent->stride * PE_stride;
    const int gend = gstart + gstride * (PE_size - 1);
    if (gstart < 0 || gstart >= s.n_pes) {
        warn("Starting global PE (%d) is invalid", gstart);
        return -1;
    }
    if (gend < 0 || gend >= s.n_pes) {
        warn("Ending global PE (%d) is invalid", gend);
        return -1;
    }
    if (config_mask != 0 && config_mask != SHMEM_TEAM_NUM_CONTEXTS) {
        warn("Invalid team_split_strided config_mask (%ld)", config_mask);
        return -1;
    }
    Team child;
    child.start = gstart;
    child.stride = PE_size == 1 ? 1 : gstride;
    child.size = PE_size;
    child.valid = true;
    child.config_mask = config_mask;
    child.num_contexts = config_mask && config ? config->num_contexts : 0;
    const int d = s.my_pe - gstart;
    const bool member = gstride > 0 ? (d >= 0 && d % gstride == 0 && d / gstride < PE_size)
                                    : (d <= 0 && (-d) % (-gstride) == 0 && (-d) / (-gstride) < PE_size);
    if (member) child.my_idx = d / gstride;
    int slot = -1;
    const int rc = team_agree_slot(*parent, child, member, &slot);
    if (member && slot >= 0) {
        child.psync_idx = slot;
        if (rc == 0) {
            s.team_avail &= ~(1ull << slot);
            Team *t = new Team(child);
            s.team_pool[(size_t)slot] = t;
            if (new_team) *new_team = team_handle(t);
        }
    }
    team_barrier(*parent);  // src/shmem_team.c:410-414
    return rc;
}

int shmem_team_split_2d(shmem_team_t parent_team, int xrange, const shmem_team_config_t *xaxis_config,
                        long xaxis_mask, shmem_team_t *xaxis_team,
                        const shmem_team_config_t *yaxis_config, long yaxis_mask,
                        shmem_team_t *yaxis_team)
{
    // src/shmem_team.c:436-505: every x team (consecutive runs of xrange) and then every
    // y team (stride xrange) is created by a split over the whole parent, in order
    check_initialized("shmem_team_split_2d");
    if (xaxis_team) *xaxis_team = SHMEM_TEAM_INVALID;
    if (yaxis_team) *yaxis_team = SHMEM_TEAM_INVALID;
    if (parent_team == SHMEM_TEAM_INVALID) return 1;
    Team *parent = team_checked(parent_team, "shmem_team_split_2d");
    if (xrange <= 0) {  // SOS divides by xrange (:455)
        warn("Invalid xrange (%d)", xrange);
        return -1;
    }
    if (xrange > parent->size) xrange = parent->size;
    const int psize = parent->size;
    const int num_xteams = (psize + xrange - 1) / xrange;
    int start = 0;
    for (int i = 0; i < num_xteams; ++i) {
        const int xsize = (i == num_xteams - 1 && psize % xrange) ? psize % xrange : xrange;
        shmem_team_t t = SHMEM_TEAM_INVALID;
        if (shmem_team_split_strided(parent_team, start, 1, xsize, xaxis_config, xaxis_mask, &t))
            raise_error("Creation of x-axis team %d of %d failed", i + 1, num_xteams);
        start += xrange;
        if (t != SHMEM_TEAM_INVALID && xaxis_team) *xaxis_team = t;
    }
    start = 0;
    for (int i = 0; i < xrange; ++i) {
        const int rem = psize % xrange, yrange = psize / xrange;
        const int ysize = (rem && i < rem) ? yrange + 1 : yrange;
        shmem_team_t t = SHMEM_TEAM_INVALID;
        if (shmem_team_split_strided(parent_team, start, xrange, ysize, yaxis_config, yaxis_mask, &t))
            raise_error("Creation of y-axis team %d of %d failed", i + 1, xrange);
        start += 1;
        if (t != SHMEM_TEAM_INVALID && yaxis_team) *yaxis_team = t;
    }
    team_barrier(*parent);
    return 0;
}

void shmem_team_destroy(shmem_team_t team)
{
    // src/teams_c.c4:138-148, src/shmem_team.c:508-535
    check_initialized("shmem_team_destroy");
    State &s = st();
    if (team == team_handle(&s.world) || team == team_handle(&s.shared))
        raise_error("Cannot destroy a pre-defined team");
    Team *t = team_from_handle(team);
    if (!t || t->predefined) return;
    if (t->psync_idx >= 3 && t->psync_idx < (int)s.team_pool.size() && s.team_pool[(size_t)t->psync_idx] == t) {
        s.team_pool[(size_t)t->psync_idx] = nullptr;
        s.team_avail |= 1ull << t->psync_idx;
    }
    t->valid = false;
    delete t;
}

int shmem_team_sync(shmem_team_t team)
{
    if (team == SHMEM_TEAM_INVALID) return -1;
    team_barrier(*team_checked(team, "shmem_team_sync"));
    return 0;
}

}  // extern "C"

// Introspection for the CPU tests (tests/test_abi.py): the p2p transport's mapping flags.
extern "C" void sosx_p2p_flags(unsigned *host_register, unsigned *ipc_open)
{
    if (host_register) *host_register = sosrt::kP2PHostRegisterFlags;
    if (ipc_open) *ipc_open = sosrt::kP2PIpcOpenFlags;
}
