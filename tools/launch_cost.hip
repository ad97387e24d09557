// launch_cost.hip -- host time of one hipLaunchKernelGGL by kernel-argument size, and of
// the release-event record the p2p transport makes before each post (DESIGN.md section
// 7.3).  Each figure: mean host wall time per call over `reps` calls on one stream, the
// stream drained between batches (the calls queue behind each other, as a p2p call's).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/build/launch_cost tools/launch_cost.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

template <int B> struct Blob {
    unsigned long long w[B / 8];
};

template <int B> __global__ void k_args(Blob<B> b, unsigned long long *sink)
{
    if (threadIdx.x == 0 && b.w[0] == 0xdeadbeefull) *sink = b.w[B / 8 - 1];
}

template <int B> double launch_us(hipStream_t s, unsigned long long *sink, int reps)
{
    Blob<B> b{};
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_args<B>, dim3(1), dim3(64), 0, s, b, sink);
    CK(hipStreamSynchronize(s));
    double tot = 0;
    for (int k = 0; k < reps; k += 20) {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_args<B>, dim3(1), dim3(64), 0, s, b, sink);
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        CK(hipStreamSynchronize(s));
    }
    return tot / reps;
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 2000;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long *sink;
    CK(hipMalloc(&sink, 8));
    hipEvent_t rel, plain;
    CK(hipEventCreateWithFlags(&rel, hipEventReleaseToSystem | hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&plain, hipEventDisableTiming));
    for (int rep = 0; rep < 3; ++rep) {
        printf("launch, %4d B of arguments: %.2f us host\n", 64, launch_us<64>(s, sink, reps));
        printf("launch, %4d B of arguments: %.2f us host\n", 256, launch_us<256>(s, sink, reps));
        printf("launch, %4d B of arguments: %.2f us host\n", 512, launch_us<512>(s, sink, reps));
        printf("launch, %4d B of arguments: %.2f us host\n", 1024, launch_us<1024>(s, sink, reps));
        printf("launch, %4d B of arguments: %.2f us host\n", 2048, launch_us<2048>(s, sink, reps));
        for (int which = 0; which < 2; ++which) {
            hipEvent_t ev = which ? rel : plain;
            double tot = 0;
            for (int k = 0; k < reps; k += 20) {
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < 20; ++i) CK(hipEventRecord(ev, s));
                tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                CK(hipStreamSynchronize(s));
            }
            printf("event record, %s: %.2f us host\n", which ? "hipEventReleaseToSystem" : "plain", tot / reps);
        }
    }
    printf("done\n");
    return 0;
}
