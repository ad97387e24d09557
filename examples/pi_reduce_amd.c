/*
 * pi_reduce_amd.c -- Monte Carlo pi with a team sum reduction (config #1 acceptance
 * program; same computation as SOS's examples/pi_reduce.c, written for this build).
 * Every PE draws NUM_POINTS points from glibc rand() seeded with 1 + pe, counts the
 * hits inside the unit circle, and the counts are summed in place with the C11
 * generic shmem_sum_reduce on long long (SHMEM_TEAM_WORLD).
 * Known answers (glibc 2.35): 1 PE 3.171200, 2 PEs 3.164400, 4 PEs 3.154100,
 * 8 PEs 3.150200.
 */
#include <shmem.h>
#include <stdio.h>
#include <stdlib.h>

#define NUM_POINTS 10000

static long long hits = 0, points = 0;

int main(void)
{
    shmem_init();
    const int npes = shmem_n_pes();
    const int me = shmem_my_pe();

    srand(1 + me);
    for (points = 0; points < NUM_POINTS; ++points) {
        const double x = rand() / (double) RAND_MAX;
        const double y = rand() / (double) RAND_MAX;
        if (x * x + y * y < 1) ++hits;
    }
    shmem_barrier_all();

    shmem_sum_reduce(SHMEM_TEAM_WORLD, &hits, &hits, 1);
    shmem_sum_reduce(SHMEM_TEAM_WORLD, &points, &points, 1);

    if (me == 0)
        printf("Pi from %llu points on %d PEs: %lf\n", points, npes, 4.0 * hits / (double) points);
    shmem_finalize();
    return 0;
}
