// hostpipe.cpp -- the local combine on HOST-resident operands, pipelined over PCIe.
//
// SOS's reduction operands live in the host symmetric heap (src/symmetric_heap_c.c;
// here: pinned memory from hipHostMalloc).  Combining them on the GPU costs
// 2*n*s bytes H2D + n*s bytes D2H; done serially (copy in, combine, copy out) that is
// the sum of both directions.  This pipeline splits the vector into chunks and runs
// H2D(chunk k+1) || combine(chunk k) || D2H(chunk k-1) on three streams with three
// device slots, so the time approaches max(H2D, D2H) on a full-duplex PCIe link.
// Chunking is exact: the combine is elementwise.
#include <hip/hip_runtime.h>
#include <string.h>

#include "dtypes.h"
#include "sosx.h"

namespace {

struct Pipe {
    bool ready = false;
    int device = -1;
    hipStream_t s_in = nullptr, s_cmp = nullptr, s_out = nullptr;
    static constexpr int kSlots = 3;
    void *a[kSlots] = {nullptr, nullptr, nullptr};
    void *b[kSlots] = {nullptr, nullptr, nullptr};
    size_t slot_bytes = 0;
    hipEvent_t in_done[kSlots] = {}, cmp_done[kSlots] = {}, out_done[kSlots] = {};
};

Pipe g_pipe;

// Frees everything the pipe holds (slots, events, streams) and marks it not ready, so
// a failed or stale setup can never leave freed slots behind a valid-looking size.
void release()
{
    Pipe &p = g_pipe;
    if (p.ready || p.s_in || p.s_cmp || p.s_out) (void)hipDeviceSynchronize();
    for (int i = 0; i < Pipe::kSlots; ++i) {
        if (p.a[i]) (void)hipFree(p.a[i]);
        if (p.b[i]) (void)hipFree(p.b[i]);
        p.a[i] = p.b[i] = nullptr;
        if (p.in_done[i]) (void)hipEventDestroy(p.in_done[i]);
        if (p.cmp_done[i]) (void)hipEventDestroy(p.cmp_done[i]);
        if (p.out_done[i]) (void)hipEventDestroy(p.out_done[i]);
        p.in_done[i] = p.cmp_done[i] = p.out_done[i] = nullptr;
    }
    for (hipStream_t *s : {&p.s_in, &p.s_cmp, &p.s_out}) {
        if (*s) (void)hipStreamDestroy(*s);
        *s = nullptr;
    }
    p.slot_bytes = 0;
    p.device = -1;
    p.ready = false;
}

int setup(size_t slot_bytes)
{
    Pipe &p = g_pipe;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return SOSX_ERR_HIP;
    if (p.ready && p.device == dev && p.slot_bytes >= slot_bytes) return SOSX_OK;
    if (p.ready && p.device != dev) release();  // streams/events belong to the old device
    if (!p.ready) {
        bool ok = hipStreamCreateWithFlags(&p.s_in, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&p.s_cmp, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&p.s_out, hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; ok && i < Pipe::kSlots; ++i)
            ok = hipEventCreateWithFlags(&p.in_done[i], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&p.cmp_done[i], hipEventDisableTiming | hipEventReleaseToSystem) == hipSuccess &&
                 hipEventCreateWithFlags(&p.out_done[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            release();
            return SOSX_ERR_HIP;
        }
        p.device = dev;
        p.ready = true;
    }
    // grow the slots: free the old ones first (HBM headroom); any failure releases all
    (void)hipDeviceSynchronize();
    for (int i = 0; i < Pipe::kSlots; ++i) {
        if (p.a[i]) (void)hipFree(p.a[i]);
        if (p.b[i]) (void)hipFree(p.b[i]);
        p.a[i] = p.b[i] = nullptr;
    }
    p.slot_bytes = 0;
    for (int i = 0; i < Pipe::kSlots; ++i)
        if (hipMalloc(&p.a[i], slot_bytes) != hipSuccess || hipMalloc(&p.b[i], slot_bytes) != hipSuccess) {
            (void)hipGetLastError();
            release();
            return SOSX_ERR_HIP;
        }
    p.slot_bytes = slot_bytes;
    return SOSX_OK;
}

}  // namespace

extern "C" {

// inout[i] = inout[i] OP in[i] with inout/in in host memory (pinned for full overlap).
// Synchronous; `chunk_bytes` 0 = 16 MiB.
int sosx_combine_host(int op, int dtype, void *inout, const void *in, size_t count,
                      size_t chunk_bytes)
{
    int rc = sosx_check_op(op, dtype);
    if (rc) return rc;
    if (count == 0) return SOSX_OK;
    if (!inout || !in) return SOSX_ERR_ARG;
    const size_t ts = sosx_dtype_size(dtype);
    if (!chunk_bytes) {
        // pinned memory overlaps the three stages; pageable copies are staged through the
        // runtime's bounce buffers synchronously, so there only large chunks pay
        hipPointerAttribute_t at;
        const bool pinned = hipPointerGetAttributes(&at, inout) == hipSuccess &&
                            at.type == hipMemoryTypeHost;
        if (!pinned) (void)hipGetLastError();
        chunk_bytes = pinned ? (16u << 20) : (64u << 20);
    }
    size_t chunk = chunk_bytes / ts;
    if (chunk == 0) chunk = 1;
    chunk_bytes = chunk * ts;
    rc = setup(chunk_bytes);
    if (rc) return rc;
    Pipe &p = g_pipe;
    const size_t nchunks = (count + chunk - 1) / chunk;
    for (size_t k = 0; k < nchunks; ++k) {
        const int s = (int)(k % Pipe::kSlots);
        const size_t first = k * chunk;
        const size_t n = count - first < chunk ? count - first : chunk;
        char *io = (char *)inout + first * ts;
        const char *ii = (const char *)in + first * ts;
        if (k >= (size_t)Pipe::kSlots && hipStreamWaitEvent(p.s_in, p.out_done[s], 0) != hipSuccess)
            return SOSX_ERR_HIP;
        if (hipMemcpyAsync(p.a[s], io, n * ts, hipMemcpyHostToDevice, p.s_in) != hipSuccess ||
            hipMemcpyAsync(p.b[s], ii, n * ts, hipMemcpyHostToDevice, p.s_in) != hipSuccess ||
            hipEventRecord(p.in_done[s], p.s_in) != hipSuccess)
            return SOSX_ERR_HIP;
        if (hipStreamWaitEvent(p.s_cmp, p.in_done[s], 0) != hipSuccess) return SOSX_ERR_HIP;
        rc = sosx_combine(op, dtype, p.a[s], p.b[s], n, p.s_cmp);
        if (rc) return rc;
        if (hipEventRecord(p.cmp_done[s], p.s_cmp) != hipSuccess ||
            hipStreamWaitEvent(p.s_out, p.cmp_done[s], 0) != hipSuccess ||
            hipMemcpyAsync(io, p.a[s], n * ts, hipMemcpyDeviceToHost, p.s_out) != hipSuccess ||
            hipEventRecord(p.out_done[s], p.s_out) != hipSuccess)
            return SOSX_ERR_HIP;
    }
    return hipStreamSynchronize(p.s_out) == hipSuccess ? SOSX_OK : SOSX_ERR_HIP;
}

// Returns the pipeline's device slots (6 x chunk bytes of HBM) and streams; called by
// shmem_finalize.  The next sosx_combine_host sets them up again.
void sosx_combine_host_release(void) { release(); }

}  // extern "C"
