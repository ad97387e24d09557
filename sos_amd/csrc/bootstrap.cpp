// bootstrap.cpp -- minimal TCP bootstrap for shmem_init().
//
// SOS bootstraps through PMI/PMIx (src/runtime-pmi.c:53-288: rank, size, KVS put/get,
// barrier).  The MI355X build needs one thing from it: every PE must receive the RCCL
// unique id created by PE 0.  PE 0 listens on addr:port, the others connect, send
// their rank, and PE 0 answers each with the id; an all-gather of a small per-PE
// record (device bus id, host name) rides the same sockets.
//
// Rank/size come from the first of: SHMEM_PE/SHMEM_NPES (tools/oshrun), torchrun's
// RANK/WORLD_SIZE, PMI_RANK/PMI_SIZE, OMPI_COMM_WORLD_RANK/SIZE, SLURM_PROCID/NTASKS;
// none -> a singleton job.  Address: SHMEM_BOOTSTRAP_ADDR/PORT, else MASTER_ADDR and
// MASTER_PORT + 1 (torchrun's own store owns MASTER_PORT).
#include "bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <vector>

namespace sosboot {

namespace {

bool env_int(const char *name, int *out)
{
    const char *v = getenv(name);
    if (!v || !*v) return false;
    *out = atoi(v);
    return true;
}

bool send_all(int fd, const void *buf, size_t n)
{
    const char *p = (const char *)buf;
    while (n) {
        ssize_t k = send(fd, p, n, MSG_NOSIGNAL);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        p += k;
        n -= (size_t)k;
    }
    return true;
}

bool recv_all(int fd, void *buf, size_t n, int timeout_ms)
{
    char *p = (char *)buf;
    while (n) {
        struct pollfd pfd = {fd, POLLIN, 0};
        int r = poll(&pfd, 1, timeout_ms);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        ssize_t k = recv(fd, p, n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        p += k;
        n -= (size_t)k;
    }
    return true;
}

double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

}  // namespace

bool discover(int *rank, int *size)
{
    static const char *pairs[][2] = {{"SHMEM_PE", "SHMEM_NPES"},
                                     {"RANK", "WORLD_SIZE"},
                                     {"PMI_RANK", "PMI_SIZE"},
                                     {"OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE"},
                                     {"SLURM_PROCID", "SLURM_NTASKS"}};
    for (auto &p : pairs) {
        int r, s;
        if (env_int(p[0], &r) && env_int(p[1], &s) && s >= 1 && r >= 0 && r < s) {
            *rank = r;
            *size = s;
            return true;
        }
    }
    *rank = 0;
    *size = 1;
    return false;
}

int local_rank(int rank)
{
    int lr;
    if (env_int("SHMEM_LOCAL_PE", &lr)) return lr;
    if (env_int("LOCAL_RANK", &lr)) return lr;
    if (env_int("OMPI_COMM_WORLD_LOCAL_RANK", &lr)) return lr;
    if (env_int("SLURM_LOCALID", &lr)) return lr;
    return rank;
}

// Exchange: PE 0 broadcasts `root_blob` (root_len bytes) and gathers every PE's
// `my_rec` (rec_len bytes) into `all_recs` (size*rec_len), which it broadcasts too.
int exchange(int rank, int size, const void *root_blob, size_t root_len, void *out_blob,
             const void *my_rec, size_t rec_len, void *all_recs, char *err, size_t errlen)
{
    if (size == 1) {
        if (out_blob && root_blob) memcpy(out_blob, root_blob, root_len);
        if (all_recs) memcpy(all_recs, my_rec, rec_len);
        return 0;
    }
    const char *addr = getenv("SHMEM_BOOTSTRAP_ADDR");
    int port = 0;
    if (!env_int("SHMEM_BOOTSTRAP_PORT", &port)) {
        int mp;
        if (env_int("MASTER_PORT", &mp)) port = mp + 1;
    }
    if (!addr) addr = getenv("MASTER_ADDR");
    if (!addr || port <= 0) {
        snprintf(err, errlen,
                 "multi-PE job without a bootstrap address (set SHMEM_BOOTSTRAP_ADDR/PORT or "
                 "MASTER_ADDR/MASTER_PORT, or launch with tools/oshrun)");
        return -1;
    }
    int timeout_s = 120;
    env_int("SHMEM_BOOTSTRAP_TIMEOUT", &timeout_s);
    const double deadline = now_s() + timeout_s;

    struct addrinfo hints, *res = nullptr;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    char portstr[16];
    snprintf(portstr, sizeof(portstr), "%d", port);
    if (getaddrinfo(addr, portstr, &hints, &res) != 0 || !res) {
        snprintf(err, errlen, "cannot resolve bootstrap address %s:%d", addr, port);
        return -1;
    }

    if (rank == 0) {
        int ls = socket(AF_INET, SOCK_STREAM, 0);
        int one = 1;
        setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        struct sockaddr_in sa;
        memset(&sa, 0, sizeof(sa));
        sa.sin_family = AF_INET;
        sa.sin_addr.s_addr = htonl(INADDR_ANY);
        sa.sin_port = htons((uint16_t)port);
        freeaddrinfo(res);
        if (bind(ls, (struct sockaddr *)&sa, sizeof(sa)) != 0 || listen(ls, 1024) != 0) {
            snprintf(err, errlen, "bootstrap bind/listen on port %d failed: %s", port,
                     strerror(errno));
            close(ls);
            return -1;
        }
        std::vector<int> fds(size, -1);
        std::vector<char> recs((size_t)size * rec_len);
        memcpy(recs.data(), my_rec, rec_len);
        for (int got = 1; got < size;) {
            struct pollfd pfd = {ls, POLLIN, 0};
            int left_ms = (int)((deadline - now_s()) * 1000);
            if (left_ms <= 0 || poll(&pfd, 1, left_ms) <= 0) {
                snprintf(err, errlen, "bootstrap: only %d of %d PEs connected", got, size);
                close(ls);
                return -1;
            }
            int fd = accept(ls, nullptr, nullptr);
            if (fd < 0) continue;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            int32_t r = -1;
            if (!recv_all(fd, &r, sizeof(r), 10000) || r <= 0 || r >= size || fds[r] >= 0) {
                close(fd);
                continue;
            }
            if (!recv_all(fd, recs.data() + (size_t)r * rec_len, rec_len, 10000)) {
                close(fd);
                continue;
            }
            fds[r] = fd;
            ++got;
        }
        bool ok = true;
        for (int r = 1; r < size; ++r) {
            ok &= send_all(fds[r], root_blob, root_len);
            ok &= send_all(fds[r], recs.data(), recs.size());
            close(fds[r]);
        }
        close(ls);
        if (out_blob) memcpy(out_blob, root_blob, root_len);
        if (all_recs) memcpy(all_recs, recs.data(), recs.size());
        if (!ok) {
            snprintf(err, errlen, "bootstrap: send to a PE failed");
            return -1;
        }
        return 0;
    }

    int fd = -1;
    while (true) {
        fd = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
        close(fd);
        fd = -1;
        if (now_s() > deadline) break;
        usleep(50 * 1000);
    }
    freeaddrinfo(res);
    if (fd < 0) {
        snprintf(err, errlen, "bootstrap: cannot connect to %s:%d", addr, port);
        return -1;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int32_t r = rank;
    bool ok = send_all(fd, &r, sizeof(r)) && send_all(fd, my_rec, rec_len);
    int left_ms = (int)((deadline - now_s()) * 1000);
    if (left_ms < 1000) left_ms = 1000;
    ok = ok && recv_all(fd, out_blob, root_len, left_ms);
    ok = ok && recv_all(fd, all_recs, (size_t)size * rec_len, left_ms);
    close(fd);
    if (!ok) {
        snprintf(err, errlen, "bootstrap: exchange with PE 0 failed");
        return -1;
    }
    return 0;
}

}  // namespace sosboot

// Test hook (CPU, no GPU): discover rank/size from the launcher environment and run
// one bootstrap exchange in which PE 0 broadcasts a token and every PE contributes its
// rank; `all_ranks` (size ints) receives the gathered ranks.  Returns 0 on success.
extern "C" int sosx_bootstrap_probe(int *rank, int *size, int *all_ranks, int cap,
                                    unsigned long long *token)
{
    int r, s;
    sosboot::discover(&r, &s);
    if (rank) *rank = r;
    if (size) *size = s;
    if (!all_ranks || cap < s) return -3;
    unsigned long long tok = 0x5EED0000ull + (unsigned long long)s;
    unsigned long long got = 0;
    char err[256] = {0};
    int32_t me = r;
    std::vector<int32_t> recs((size_t)s);
    int rc = sosboot::exchange(r, s, &tok, sizeof(tok), &got, &me, sizeof(me), recs.data(), err,
                               sizeof(err));
    if (rc) {
        fprintf(stderr, "bootstrap probe: %s\n", err);
        return rc;
    }
    for (int i = 0; i < s; ++i) all_ranks[i] = recs[(size_t)i];
    if (token) *token = got;
    return 0;
}
