/*
 * static_reduce.c -- reductions on STATIC symmetric objects (SOS programs keep symmetric
 * data in .data/.bss as often as in the heap; src/init.c:341-346 registers that segment
 * with every transport).  shmem_init here registers [__data_start, _end) with HIP, so
 * these arrays move over PCIe like pinned heap memory.
 *
 *   static_reduce team <count> <out-file>
 *       dest = shmem_float_sum_reduce(SHMEM_TEAM_WORLD, source) on two static float
 *       arrays; source[i] = float((i * 2654435761 + pe * 40503) mod 1000003) * 0.001f;
 *       every PE writes its dest bytes to <out-file>.<pe> (tests/test_gpu_team.py
 *       compares them with the oracle).
 *   static_reduce local <count> <reps>
 *       times shmemx_reduce_local(SUM, FLOAT) of one static array into another (the
 *       H2D || combine || D2H pipeline), checks the exact result and prints one JSON
 *       line: payload GiB/s and the registered segment (bench.py's host_resident block).
 *
 * The arrays hold up to 128Mi floats each (1 GiB of .bss in all).
 */
#include <shmem.h>
#include <shmemx.h>
#include <sosx.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define MAXN (128u << 20)

static float source[MAXN];
static float dest[MAXN];

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static float value(size_t i, int pe)
{
    const uint64_t k = ((uint64_t) i * 2654435761ull + (uint64_t) pe * 40503ull) % 1000003ull;
    return (float) k * 0.001f;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s team <count> <out-file> | local <count> <reps>\n", argv[0]);
        return 2;
    }
    const size_t n = strtoull(argv[2], NULL, 0);
    if (n == 0 || n > MAXN) {
        fprintf(stderr, "count must be 1..%u\n", MAXN);
        return 2;
    }
    shmem_init();
    const int me = shmem_my_pe();
    int rc = 0;
    if (!strcmp(argv[1], "team")) {
        for (size_t i = 0; i < n; ++i) source[i] = value(i, me);
        memset(dest, 0xA5, n * sizeof(float));
        shmem_barrier_all();
        if (shmem_float_sum_reduce(SHMEM_TEAM_WORLD, dest, source, n) != 0) rc = 1;
        char path[4096];
        snprintf(path, sizeof(path), "%s.%d", argv[3], me);
        FILE *f = fopen(path, "wb");
        if (!f || fwrite(dest, sizeof(float), n, f) != n) rc = 1;
        if (f) fclose(f);
        void *base = NULL;
        const size_t reg = sosx_data_segment(&base);
        printf("PE %d/%d: static team reduce of %zu floats written; data segment registered %zu B\n", me,
               shmem_n_pes(), n, reg);
    } else if (!strcmp(argv[1], "local")) {
        const int reps = atoi(argv[3]) > 0 ? atoi(argv[3]) : 5;
        for (size_t i = 0; i < n; ++i) {
            dest[i] = (float) (i % 7);
            source[i] = (float) (i % 5);
        }
        /* one untimed call (pipeline setup), then reps timed ones */
        double t0 = 0;
        for (int r = 0; r <= reps; ++r) {
            if (r == 1) t0 = now_s();
            if (shmemx_reduce_local(SOSX_OP_SUM, SOSX_DT_FLOAT, n, source, dest) != 0) rc = 1;
        }
        const double t = (now_s() - t0) / reps;
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i)
            if (dest[i] != (float) (i % 7) + (float) (reps + 1) * (float) (i % 5)) ++bad;
        void *base = NULL;
        const size_t reg = sosx_data_segment(&base);
        if (bad) rc = 1;
        printf("{\"static_pipelined_GiBs\": %.3f, \"static_pipelined_ms\": %.3f, \"count\": %zu, "
               "\"registered_bytes\": %zu, \"wrong\": %zu}\n",
               (double) n * sizeof(float) / t / (double) (1u << 30), t * 1e3, n, reg, bad);
    } else {
        fprintf(stderr, "unknown mode %s\n", argv[1]);
        rc = 2;
    }
    shmem_finalize();
    return rc;
}
