// acquire_probe.hip -- what makes a kernel's first read of memory another agent rewrote
// skip the lines this GPU's L2s still hold from an earlier read (the
// consumer half of the memory-visibility rule).
//
// A peer GPU's HBM (IPC-mapped, read over xGMI) cannot be had on a one-GPU box, so the
// probe uses the one-GPU memory that is mapped the same way: memory that is not local to
// the L2 and not fine-grained, i.e. coarse-grained host memory.  Per trial:
//   1. the CPU rewrites every word of H with the trial number;
//   2. a checker kernel (16 workgroups, each reading ALL of H with plain 16-B loads, so
//      every XCD's L2 has seen every line in earlier trials) counts words != trial.
// Schemes for how the checker learns H is ready:
//   host    the CPU writes, then launches (the p2p host-signalling mode: host waits, then
//           enqueues the consuming kernel);
//   device  waiter kernel (1 workgroup, system-scope acquire poll of a host flag) and the
//           checker are enqueued first, then the CPU writes and sets the flag (stream mode);
// Remedies between the "ready" point and the checker:
//   none     nothing;
//   acqk     a 64-workgroup kernel whose lane 0 runs a system-scope acquire fence;
//   inkernel each checker workgroup's lane 0 runs the acquire before its loads;
//   event    hipEventRecord of a default-flag event (HIP documents a system-scope acquire
//            and release fence for it, hip_runtime_api.h hipEventDisableSystemFence).
// Memory: coarse (hipHostMallocNonCoherent), fine (hipHostMalloc default, coherent),
//         regcoarse (hipHostRegister + hipExtHostRegisterCoarseGrained).
// Also prices the acquire: a 1 GiB streaming read with and without the in-kernel
// acquire per workgroup, and the acquire kernel as an extra launch.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/build/acquire_probe tools/acquire_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <sys/mman.h>

#include <atomic>
#include <chrono>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void acquire_sys()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ unsigned xcc_id()
{
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

__global__ void k_acquire(unsigned *mask)
{
    if (threadIdx.x == 0) {
        acquire_sys();
        atomicOr(mask, 1u << xcc_id());
    }
}

__global__ void k_wait(const unsigned *flag, unsigned want, unsigned long long limit)
{
    if (threadIdx.x == 0) {
        const long long t0 = wall_clock64();
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            if ((unsigned long long)(wall_clock64() - t0) > limit) break;
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

// every workgroup reads all nvec vectors of h
// bad[0]: wrong words; bad[1]: workgroups that started while the ready flag was still
// below `want` (an ordering failure, not a stale line); bad[2]/bad[3]: min/max wrong value
template <bool ACQ>
__global__ __launch_bounds__(256) void k_check(const u32x4 *h, size_t nvec, unsigned want, unsigned *bad,
                                               const unsigned *flag)
{
    if (threadIdx.x == 0 && flag &&
        __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want)
        atomicAdd(bad + 1, 1u);
    if constexpr (ACQ) {
        if (threadIdx.x == 0) acquire_sys();
        __syncthreads();
    }
    unsigned n = 0, lo = 0xffffffffu, hi = 0;
    for (size_t i = threadIdx.x; i < nvec; i += 256) {
        const u32x4 v = h[i];
        const unsigned k = (v.x != want) + (v.y != want) + (v.z != want) + (v.w != want);
        if (k) {
            n += k;
            lo = min(lo, min(min(v.x, v.y), min(v.z, v.w)));
            hi = max(hi, max(max(v.x, v.y), max(v.z, v.w)));
        }
    }
    if (n) {
        atomicAdd(bad, n);
        atomicMin(bad + 2, lo);
        atomicMax(bad + 3, hi);
    }
}

// streaming read of nvec vectors, one 4 KiB tile per workgroup (the fold's shape)
template <bool ACQ>
__global__ __launch_bounds__(256) void k_stream(const u32x4 *a, u32x4 *out, size_t nvec)
{
    if constexpr (ACQ) {
        if (threadIdx.x == 0) acquire_sys();
        __syncthreads();
    }
    const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (j < nvec) {
        u32x4 v = __builtin_nontemporal_load(a + j);
        __builtin_nontemporal_store(v, out + j);
    }
}

__global__ void k_empty() {}

int main(int argc, char **argv)
{
    const int trials = argc > 1 ? atoi(argv[1]) : 200;
    const size_t hbytes = 256 << 10;
    const size_t nvec = hbytes / 16;
    const int ngroups = 16;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *bad, *mask;
    CK(hipMalloc(&bad, 16));
    CK(hipMalloc(&mask, 4));
    unsigned *flag;
    CK(hipHostMalloc((void **)&flag, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    hipEvent_t ev_default;
    CK(hipEventCreate(&ev_default));
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const unsigned long long limit = (unsigned long long)rate_khz * 1000ull * 5;  // 5 s

    const char *mems[] = {"coarse", "fine", "regcoarse"};
    const char *schemes[] = {"host", "device"};
    const char *remedies[] = {"none", "acqk", "inkernel", "event"};
    for (int m = 0; m < 3; ++m) {
        unsigned *h = nullptr;
        void *reg = nullptr;
        if (m == 0) CK(hipHostMalloc((void **)&h, hbytes, hipHostMallocNonCoherent | hipHostMallocMapped));
        else if (m == 1) CK(hipHostMalloc((void **)&h, hbytes, hipHostMallocCoherent | hipHostMallocMapped));
        else {
            reg = mmap(nullptr, hbytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (reg == MAP_FAILED) { perror("mmap"); return 1; }
            memset(reg, 0, hbytes);
            hipError_t e = hipHostRegister(reg, hbytes, hipHostRegisterMapped | hipExtHostRegisterCoarseGrained);
            if (e != hipSuccess) {
                printf("mem=%s: hipHostRegister failed: %s\n", mems[m], hipGetErrorString(e));
                (void)hipGetLastError();
                munmap(reg, hbytes);
                continue;
            }
            h = (unsigned *)reg;
        }
        unsigned *hd = nullptr;
        CK(hipHostGetDevicePointer((void **)&hd, h, 0));
        unsigned seq = 0;
        for (int sc = 0; sc < 2; ++sc) {
            for (int r = 0; r < 4; ++r) {
                unsigned long long total = 0, early = 0;
                int bad_trials = 0;
                unsigned lo = 0xffffffffu, hi = 0, lag_lo = 0xffffffffu, lag_hi = 0;
                char which[256] = "";
                unsigned mask_or = 0;
                CK(hipMemsetAsync(mask, 0, 4, s));
                // warm: every XCD's L2 sees H
                for (size_t i = 0; i < hbytes / 4; ++i) h[i] = seq;
                std::atomic_thread_fence(std::memory_order_seq_cst);
                const unsigned init[4] = {0, 0, 0xffffffffu, 0};
                CK(hipMemcpy(bad, init, 16, hipMemcpyHostToDevice));
                hipLaunchKernelGGL(k_check<true>, dim3(ngroups), dim3(256), 0, s, (const u32x4 *)hd, nvec, seq, bad,
                                   (const unsigned *)nullptr);
                CK(hipStreamSynchronize(s));
                for (int t = 0; t < trials; ++t) {
                    ++seq;
                    CK(hipMemcpy(bad, init, 16, hipMemcpyHostToDevice));
                    if (sc == 0) {
                        for (size_t i = 0; i < hbytes / 4; ++i) h[i] = seq;
                        std::atomic_thread_fence(std::memory_order_seq_cst);
                    } else {
                        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, flag, seq, limit);
                    }
                    if (r == 1) hipLaunchKernelGGL(k_acquire, dim3(64), dim3(64), 0, s, mask);
                    if (r == 3) CK(hipEventRecord(ev_default, s));
                    const unsigned *fl = sc == 1 ? flag : nullptr;
                    if (r == 2)
                        hipLaunchKernelGGL(k_check<true>, dim3(ngroups), dim3(256), 0, s, (const u32x4 *)hd, nvec, seq, bad, fl);
                    else
                        hipLaunchKernelGGL(k_check<false>, dim3(ngroups), dim3(256), 0, s, (const u32x4 *)hd, nvec, seq, bad, fl);
                    if (sc == 1) {
                        usleep(200);  // the waiter is spinning, the checker queued behind it
                        for (size_t i = 0; i < hbytes / 4; ++i) h[i] = seq;
                        std::atomic_thread_fence(std::memory_order_seq_cst);
                        __atomic_store_n(flag, seq, __ATOMIC_RELEASE);
                    }
                    CK(hipStreamSynchronize(s));
                    unsigned b[4];
                    CK(hipMemcpy(b, bad, 16, hipMemcpyDeviceToHost));
                    total += b[0];
                    early += b[1];
                    bad_trials += b[0] != 0;
                    if (b[0]) {
                        if (strlen(which) < 200) snprintf(which + strlen(which), 56, "%s%d", *which ? "," : "", t);
                        lo = b[2] < lo ? b[2] : lo;
                        hi = b[3] > hi ? b[3] : hi;
                        // how far behind the wrong values were: seq - value
                        const unsigned l1 = seq - b[3], l2 = seq - b[2];
                        lag_lo = l1 < lag_lo ? l1 : lag_lo;
                        lag_hi = l2 > lag_hi ? l2 : lag_hi;
                    }
                }
                CK(hipMemcpy(&mask_or, mask, 4, hipMemcpyDeviceToHost));
                printf("mem=%-9s scheme=%-6s remedy=%-8s trials=%d stale_trials=%d stale_words=%llu "
                       "early_start_wgs=%llu lag=%u..%u acq_xcc_mask=0x%02x stale_at=[%s]\n",
                       mems[m], schemes[sc], remedies[r], trials, bad_trials, total, early,
                       bad_trials ? lag_lo : 0, bad_trials ? lag_hi : 0, mask_or, which);
                fflush(stdout);
            }
        }
        if (m == 2) {
            CK(hipHostUnregister(reg));
            munmap(reg, hbytes);
        } else {
            CK(hipHostFree(h));
        }
    }

    // price of the acquire
    const size_t sbytes = 1ull << 30, snvec = sbytes / 16;
    u32x4 *a, *o;
    CK(hipMalloc(&a, sbytes));
    CK(hipMalloc(&o, sbytes));
    CK(hipMemset(a, 1, sbytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned blocks = (unsigned)((snvec + 255) / 256);
    for (int rep = 0; rep < 3; ++rep) {
        for (int acq = 0; acq < 2; ++acq) {
            for (int w = 0; w < 3; ++w) {
                if (acq) hipLaunchKernelGGL(k_stream<true>, dim3(blocks), dim3(256), 0, s, a, o, snvec);
                else hipLaunchKernelGGL(k_stream<false>, dim3(blocks), dim3(256), 0, s, a, o, snvec);
            }
            CK(hipEventRecord(e0, s));
            const int K = 20;
            for (int k = 0; k < K; ++k) {
                if (acq) hipLaunchKernelGGL(k_stream<true>, dim3(blocks), dim3(256), 0, s, a, o, snvec);
                else hipLaunchKernelGGL(k_stream<false>, dim3(blocks), dim3(256), 0, s, a, o, snvec);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("stream copy 1 GiB, per-workgroup system acquire=%d: %.4f ms/launch = %.3f TB/s\n", acq,
                   ms / K, 2.0 * sbytes / (ms / K * 1e-3) / 1e12);
        }
    }
    // the acquire as an extra step: small kernel chains with nothing, the acquire kernel,
    // a default-flag event record (HIP: system-scope acquire + release fence), or an event
    // without the system fence, before each kernel; GPU time (events) and host wall time
    hipEvent_t ev_nofence;
    CK(hipEventCreateWithFlags(&ev_nofence, hipEventDisableSystemFence | hipEventDisableTiming));
    const char *steps[] = {"nothing", "acquire kernel", "default event record", "event without system fence"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int acq = 0; acq < 4; ++acq) {
            const int K = 200;
            CK(hipStreamSynchronize(s));
            auto w0 = std::chrono::steady_clock::now();
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < K; ++k) {
                if (acq == 1) hipLaunchKernelGGL(k_acquire, dim3(64), dim3(64), 0, s, mask);
                if (acq == 2) CK(hipEventRecord(ev_default, s));
                if (acq == 3) CK(hipEventRecord(ev_nofence, s));
                hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            auto w1 = std::chrono::steady_clock::now();
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("empty-kernel chain, before each: %-28s %.2f us per step (host wall %.2f us)\n", steps[acq],
                   ms * 1e3 / K, std::chrono::duration<double, std::micro>(w1 - w0).count() / K);
        }
    }
    // the acquire kernel's grid: 8 / 16 / 64 one-wave workgroups (XCD mask of each)
    for (int rep = 0; rep < 2; ++rep) {
        for (unsigned wgs : {8u, 16u, 64u}) {
            const int K = 200;
            CK(hipMemset(mask, 0, 4));
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < K; ++k) {
                hipLaunchKernelGGL(k_acquire, dim3(wgs), dim3(64), 0, s, mask);
                hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            unsigned m = 0;
            CK(hipMemcpy(&m, mask, 4, hipMemcpyDeviceToHost));
            printf("empty-kernel chain, acquire kernel of %2u workgroups before each: %.2f us per step, xcc mask 0x%02x\n",
                   wgs, ms * 1e3 / K, m);
        }
    }
    // a small consumer of G workgroups (one 4 KiB tile each): no acquire, the acquire kernel
    // before it, or each workgroup's own acquire -- in a chain and from an idle stream
    const char *forms[] = {"no acquire", "acquire kernel first", "acquire in each workgroup"};
    for (int rep = 0; rep < 2; ++rep) {
        for (unsigned G : {1u, 16u, 64u, 256u, 1024u}) {
            for (int f = 0; f < 3; ++f) {
                const int K = 200;
                auto launch = [&] {
                    if (f == 1) hipLaunchKernelGGL(k_acquire, dim3(64), dim3(64), 0, s, mask);
                    if (f == 2) hipLaunchKernelGGL(k_stream<true>, dim3(G), dim3(256), 0, s, a, o, (size_t)G * 256);
                    else hipLaunchKernelGGL(k_stream<false>, dim3(G), dim3(256), 0, s, a, o, (size_t)G * 256);
                };
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(e0, s));
                for (int k = 0; k < K; ++k) launch();
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                double tot = 0;
                for (int k = 0; k < K; ++k) {
                    CK(hipStreamSynchronize(s));
                    auto w0 = std::chrono::steady_clock::now();
                    launch();
                    CK(hipStreamSynchronize(s));
                    tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count();
                }
                printf("consumer of %4u workgroups, %-26s chain %.2f us per step, idle stream %.2f us host wall\n",
                       G, forms[f], ms * 1e3 / K, tot / K);
            }
        }
    }
    // one call's worth from an idle stream: host waits, then [acquire] + kernel + sync
    for (int rep = 0; rep < 2; ++rep) {
        for (int acq = 0; acq < 3; ++acq) {
            const int K = 200;
            double tot = 0;
            for (int k = 0; k < K; ++k) {
                CK(hipStreamSynchronize(s));
                auto w0 = std::chrono::steady_clock::now();
                if (acq == 1) hipLaunchKernelGGL(k_acquire, dim3(64), dim3(64), 0, s, mask);
                if (acq == 2) CK(hipEventRecord(ev_default, s));
                hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                CK(hipStreamSynchronize(s));
                tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count();
            }
            printf("idle stream, launch + sync, before the kernel: %-22s %.2f us host wall\n", steps[acq], tot / K);
        }
    }
    printf("done\n");
    return 0;
}
