/*
 * reduce_types.c -- end-to-end check of the public reduction API on one or more PEs:
 * team *_reduce and active-set *_to_all calls over several types and ops, on host
 * (static, heap) and device (shmemx_malloc_device) buffers, against closed forms.
 * Prints "reduce_types: OK" on PE 0 and exits 0, or reports the first mismatch.
 */
#include <shmem.h>
#include <shmemx.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define N 5000

static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static double pWrk[N / 2 + 1];
static int64_t a64[N], b64[N];
static double ad[N];

static int fail(const char *what, size_t i)
{
    fprintf(stderr, "reduce_types: MISMATCH in %s at %zu (PE %d)\n", what, i, shmem_my_pe());
    return 1;
}

int main(void)
{
    shmem_init();
    const int me = shmem_my_pe(), np = shmem_n_pes();
    int bad = 0;

    /* int64 xor / sum on static (host) data */
    for (size_t i = 0; i < N; i++) a64[i] = (int64_t) ((me + 1) * 1000003LL) ^ (int64_t) i;
    shmem_int64_xor_reduce(SHMEM_TEAM_WORLD, b64, a64, N);
    for (size_t i = 0; i < N && !bad; i++) {
        int64_t x = 0;
        for (int p = 0; p < np; p++) x ^= (int64_t) ((p + 1) * 1000003LL) ^ (int64_t) i;
        if (b64[i] != x) bad = fail("int64_xor_reduce", i);
    }

    /* double sum via the active-set API with pWrk/pSync, in place */
    for (size_t i = 0; i < N; i++) ad[i] = (double) (me + 1) * (double) i;
    shmem_double_sum_to_all(ad, ad, N, 0, 0, np, pWrk, pSync);
    for (size_t i = 0; i < N && !bad; i++)
        if (ad[i] != (double) i * np * (np + 1) / 2) bad = fail("double_sum_to_all", i);
    for (int k = 0; k < SHMEM_REDUCE_SYNC_SIZE && !bad; k++)
        if (pSync[k] != SHMEM_SYNC_VALUE) bad = fail("pSync restored", (size_t) k);

    /* int max on the symmetric heap */
    int *hi = shmem_malloc(N * sizeof(int)), *ho = shmem_malloc(N * sizeof(int));
    for (size_t i = 0; i < N; i++) hi[i] = (int) i * (me % 2 ? -1 : 1) + me;
    shmem_int_max_reduce(SHMEM_TEAM_WORLD, ho, hi, N);
    for (size_t i = 0; i < N && !bad; i++) {
        int m = hi[i];
        for (int p = 0; p < np; p++) { int v = (int) i * (p % 2 ? -1 : 1) + p; if (v > m) m = v; }
        if (ho[i] != m) bad = fail("int_max_reduce", i);
    }
    shmem_free(ho);
    shmem_free(hi);

    /* float prod on device memory */
    float *dsrc = shmemx_malloc_device(N * sizeof(float)), *ddst = shmemx_malloc_device(N * sizeof(float));
    float *h = malloc(N * sizeof(float));
    for (size_t i = 0; i < N; i++) h[i] = (i % 2) ? 2.0f : 0.5f;
    hipMemcpy(dsrc, h, N * sizeof(float), hipMemcpyHostToDevice);
    shmem_float_prod_reduce(SHMEM_TEAM_WORLD, ddst, dsrc, N);
    hipMemcpy(h, ddst, N * sizeof(float), hipMemcpyDeviceToHost);
    for (size_t i = 0; i < N && !bad; i++) {
        float x = 1.0f;
        for (int p = 0; p < np; p++) x *= (i % 2) ? 2.0f : 0.5f;
        if (h[i] != x) bad = fail("float_prod_reduce(device)", i);
    }
    free(h);
    shmemx_free_device(ddst);
    shmemx_free_device(dsrc);

    /* sub-arrays at different 16-B offsets on device memory: an int sum of M elements from
       src + 3 into dst + 1 (the realigning kernels), and reduce_local between the two */
    enum { M = 300007 };
    int *isrc = shmemx_malloc_device((M + 8) * sizeof(int)), *idst = shmemx_malloc_device((M + 8) * sizeof(int));
    int *hv = malloc((M + 8) * sizeof(int));
    for (size_t i = 0; i < M; i++) hv[i] = (int) (i % 1000) * (me + 1) - 7 * me;
    hipMemcpy(isrc + 3, hv, M * sizeof(int), hipMemcpyHostToDevice);
    shmem_int_sum_reduce(SHMEM_TEAM_WORLD, idst + 1, isrc + 3, M);
    hipMemcpy(hv, idst + 1, M * sizeof(int), hipMemcpyDeviceToHost);
    for (size_t i = 0; i < M && !bad; i++) {
        int x = 0;
        for (int p = 0; p < np; p++) x += (int) (i % 1000) * (p + 1) - 7 * p;
        if (hv[i] != x) bad = fail("int_sum_reduce(misaligned sub-arrays)", i);
    }
    /* idst + 1 += isrc + 3 (inout and in at different 16-B offsets) */
    if (shmemx_reduce_local(SOSX_OP_SUM, SOSX_DT_INT, M, isrc + 3, idst + 1) != SOSX_OK)
        bad = fail("reduce_local status", 0);
    hipMemcpy(hv, idst + 1, M * sizeof(int), hipMemcpyDeviceToHost);
    for (size_t i = 0; i < M && !bad; i++) {
        int x = (int) (i % 1000) * (me + 1) - 7 * me;
        for (int p = 0; p < np; p++) x += (int) (i % 1000) * (p + 1) - 7 * p;
        if (hv[i] != x) bad = fail("reduce_local(misaligned sub-arrays)", i);
    }
    free(hv);
    shmemx_free_device(idst);
    shmemx_free_device(isrc);

    shmem_barrier_all();
    if (me == 0 && !bad) printf("reduce_types: OK (%d PEs)\n", np);
    shmem_finalize();
    return bad;
}
