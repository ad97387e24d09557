// synth.hip -- synthetic-input generator and bitwise compare (bench / self-check).
#include <stdlib.h>

#include "elementwise.h"

namespace sos {

// ---------------------------------------------------------------------------------
// Synthetic inputs: counter-based splitmix64 of (seed, pe, i),
// bit-identical to oracle_fill in oracle/sos_oracle.c.  FP values are built from
// bits or by exact dyadic arithmetic, so CPU and GPU agree bit for bit.
// ---------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t synth_hash(uint64_t key, uint64_t i) { return mix64(key ^ i); }

__device__ __forceinline__ float synth_f32(uint64_t h, int dist)
{
    if (dist == SOSX_DIST_PROD) {  // [0.5, 2): exponent 126 or 127, 23 random mantissa bits
        uint32_t bits = ((126u + (uint32_t)(h >> 63)) << 23) | (uint32_t)(h & 0x7FFFFFu);
        return __builtin_bit_cast(float, bits);
    }
    return (float)(uint32_t)(h >> 40) * 0x1p-23f - 1.0f;  // uniform [-1, 1), exact
}
__device__ __forceinline__ double synth_f64(uint64_t h, int dist)
{
    if (dist == SOSX_DIST_PROD) {
        uint64_t bits = ((1022ull + (h >> 63)) << 52) | (h & 0xFFFFFFFFFFFFFull);
        return __builtin_bit_cast(double, bits);
    }
    return (double)(h >> 11) * 0x1p-52 - 1.0;
}
// complex parts for DIST_PROD: +-[0.5, 1)
__device__ __forceinline__ float synth_c32_part(uint64_t h, int dist)
{
    if (dist == SOSX_DIST_PROD) {
        uint32_t bits = ((uint32_t)(h >> 63) << 31) | (126u << 23) | (uint32_t)(h & 0x7FFFFFu);
        return __builtin_bit_cast(float, bits);
    }
    return synth_f32(h, dist);
}
__device__ __forceinline__ double synth_c64_part(uint64_t h, int dist)
{
    if (dist == SOSX_DIST_PROD) {
        uint64_t bits = ((h >> 63) << 63) | (1022ull << 52) | (h & 0xFFFFFFFFFFFFFull);
        return __builtin_bit_cast(double, bits);
    }
    return synth_f64(h, dist);
}
template <class T> __device__ __forceinline__ T synth_int(uint64_t h, int dist)
{
    if (dist == SOSX_DIST_PROD) return (T)((int64_t)(h % 7u) - 3);
    return (T)h;
}

template <int KIND>
__global__ __launch_bounds__(kThreads) void k_fill(void *dst, size_t n, size_t index0,
                                                     uint64_t key, int dist)
{
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t j = (size_t)blockIdx.x * kThreads + threadIdx.x; j < n; j += stride) {
        const uint64_t i = index0 + j;
        if constexpr (KIND == K_F32) {
            ((float *)dst)[j] = synth_f32(synth_hash(key, i), dist);
        } else if constexpr (KIND == K_F64) {
            ((double *)dst)[j] = synth_f64(synth_hash(key, i), dist);
        } else if constexpr (KIND == K_C32) {
            ((float *)dst)[2 * j] = synth_c32_part(synth_hash(key, 2 * i), dist);
            ((float *)dst)[2 * j + 1] = synth_c32_part(synth_hash(key, 2 * i + 1), dist);
        } else if constexpr (KIND == K_C64) {
            ((double *)dst)[2 * j] = synth_c64_part(synth_hash(key, 2 * i), dist);
            ((double *)dst)[2 * j + 1] = synth_c64_part(synth_hash(key, 2 * i + 1), dist);
        } else if constexpr (KIND == K_U8) {
            ((uint8_t *)dst)[j] = synth_int<uint8_t>(synth_hash(key, i), dist);
        } else if constexpr (KIND == K_U16) {
            ((uint16_t *)dst)[j] = synth_int<uint16_t>(synth_hash(key, i), dist);
        } else if constexpr (KIND == K_U32) {
            ((uint32_t *)dst)[j] = synth_int<uint32_t>(synth_hash(key, i), dist);
        } else {
            ((uint64_t *)dst)[j] = synth_int<uint64_t>(synth_hash(key, i), dist);
        }
    }
}

// ---------------------------------------------------------------------------------
// Bitwise compare (verification helper used by bench.py's self-check)
// ---------------------------------------------------------------------------------
template <class W>
__global__ __launch_bounds__(kThreads) void k_mismatch(const W *a, const W *b, size_t nw,
                                                         int words_per_elem,
                                                         unsigned long long *count)
{
    unsigned long long local = 0;
    const size_t ne = nw / (size_t)words_per_elem;
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < ne; e += stride) {
        bool diff = false;
        for (int w = 0; w < words_per_elem; ++w)
            diff |= a[e * words_per_elem + w] != b[e * words_per_elem + w];
        local += diff;
    }
    // wave-level sum by DPP/shuffle, one atomic per wave
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) local += __shfl_xor(local, off, 64);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(count, local);
}

}  // namespace sos

using namespace sos;

extern "C" {

int sosx_fill(int dtype, int dist, uint64_t seed, int pe, void *dst, size_t count, size_t index0,
              void *stream)
{
    const SosDtypeInfo d = sos_dtype_info(dtype);
    if (d.kind == K_INVALID) return SOSX_ERR_DTYPE;
    if (d.kind == K_LDBL) return SOSX_ERR_UNSUPPORTED;
    if (count == 0) return SOSX_OK;
    if (!dst) return SOSX_ERR_ARG;
    const uint64_t key = mix64(seed ^ ((uint64_t)(uint32_t)pe << 40));
    size_t blocks = (count + kThreads - 1) / kThreads;
    if (blocks > 16384) blocks = 16384;
    hipStream_t st = as_stream(stream);
    dim3 gr((unsigned)blocks), bl(kThreads);
    switch (d.kind) {
        case K_F32: hipLaunchKernelGGL(k_fill<K_F32>, gr, bl, 0, st, dst, count, index0, key, dist); break;
        case K_F64: hipLaunchKernelGGL(k_fill<K_F64>, gr, bl, 0, st, dst, count, index0, key, dist); break;
        case K_C32: hipLaunchKernelGGL(k_fill<K_C32>, gr, bl, 0, st, dst, count, index0, key, dist); break;
        case K_C64: hipLaunchKernelGGL(k_fill<K_C64>, gr, bl, 0, st, dst, count, index0, key, dist); break;
        default:
            switch (d.size) {
                case 1: hipLaunchKernelGGL(k_fill<K_U8>, gr, bl, 0, st, dst, count, index0, key, dist); break;
                case 2: hipLaunchKernelGGL(k_fill<K_U16>, gr, bl, 0, st, dst, count, index0, key, dist); break;
                case 4: hipLaunchKernelGGL(k_fill<K_U32>, gr, bl, 0, st, dst, count, index0, key, dist); break;
                default: hipLaunchKernelGGL(k_fill<K_U64>, gr, bl, 0, st, dst, count, index0, key, dist); break;
            }
    }
    return hip_ok(hipGetLastError());
}

// Test/bench helper: a system-scope release (an event created with
// hipEventReleaseToSystem) so that earlier kernel stores are in HBM for the copy's DMA
// reads, the copy, and the same release after it (a device destination written by a
// blit kernel is then in HBM for a following DMA read; see sync_system in runtime.h).
int sosx_memcpy(void *dst, const void *src, size_t bytes, void *stream)
{
    static hipEvent_t ev = nullptr;
    hipStream_t st = as_stream(stream);
    hipError_t e = ev ? hipSuccess
                      : hipEventCreateWithFlags(&ev, hipEventReleaseToSystem | hipEventDisableTiming);
    // what kernels stored before (on any stream) in HBM first, then the copy
    if (e == hipSuccess) e = hipEventRecord(ev, st);
    if (e == hipSuccess) e = hipEventSynchronize(ev);
    if (e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st);
    if (e == hipSuccess) e = hipEventRecord(ev, st);
    if (e == hipSuccess) e = hipEventSynchronize(ev);
    return hip_ok(e);
}

int sosx_count_mismatch(const void *a, const void *b, size_t count, size_t elem_size,
                        unsigned long long *mismatches, void *stream)
{
    if (!mismatches || elem_size == 0) return SOSX_ERR_ARG;
    *mismatches = 0;
    if (count == 0) return SOSX_OK;
    hipStream_t st = as_stream(stream);
    unsigned long long *dcount = nullptr;
    if (hipMallocAsync((void **)&dcount, sizeof(*dcount), st) != hipSuccess) return SOSX_ERR_HIP;
    (void)hipMemsetAsync(dcount, 0, sizeof(*dcount), st);
    const size_t bytes = count * elem_size;
    size_t w = (elem_size % 8 == 0) ? 8 : (elem_size % 4 == 0) ? 4 : (elem_size % 2 == 0) ? 2 : 1;
    if (((uintptr_t)a | (uintptr_t)b) % w) w = 1;
    const size_t nw = bytes / w;
    const int wpe = (int)(elem_size / w);
    size_t blocks = (count + kThreads - 1) / kThreads;
    if (blocks > 8192) blocks = 8192;
    dim3 gr((unsigned)blocks), bl(kThreads);
    switch (w) {
        case 8: hipLaunchKernelGGL(k_mismatch<uint64_t>, gr, bl, 0, st, (const uint64_t *)a, (const uint64_t *)b, nw, wpe, dcount); break;
        case 4: hipLaunchKernelGGL(k_mismatch<uint32_t>, gr, bl, 0, st, (const uint32_t *)a, (const uint32_t *)b, nw, wpe, dcount); break;
        case 2: hipLaunchKernelGGL(k_mismatch<uint16_t>, gr, bl, 0, st, (const uint16_t *)a, (const uint16_t *)b, nw, wpe, dcount); break;
        default: hipLaunchKernelGGL(k_mismatch<uint8_t>, gr, bl, 0, st, (const uint8_t *)a, (const uint8_t *)b, nw, wpe, dcount); break;
    }
    hipError_t e = hipMemcpyAsync(mismatches, dcount, sizeof(*dcount), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFreeAsync(dcount, st);
    (void)hipStreamSynchronize(st);
    return hip_ok(e);
}

}  // extern "C"
