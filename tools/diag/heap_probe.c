/* Diagnostic: shmem_init (device heap + IPC mapping) from C, i.e. on /opt/rocm's HIP
 * runtime rather than torch's.  Run under tools/oshrun with SHMEMX_TRANSPORT=p2p. */
#include <stdio.h>
#include <shmem.h>

int main(void)
{
    shmem_init();
    printf("PE %d of %d: init ok\n", shmem_my_pe(), shmem_n_pes());
    fflush(stdout);
    shmem_barrier_all();
    shmem_finalize();
    return 0;
}
