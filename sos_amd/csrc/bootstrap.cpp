// bootstrap.cpp -- rank discovery, the TCP hub and the shared-memory barrier.
//
// SOS bootstraps through PMI/PMIx (src/runtime-pmi.c:53-288: rank, size, KVS put/get,
// barrier).  The MI355X build needs: the RCCL unique id from PE 0 on every PE, a way
// to all-gather small records later (IPC handles of the device symmetric heap), and a
// fast node-local barrier for the peer-to-peer transport.
//
// Rank/size come from the first of: SHMEM_PE/SHMEM_NPES (tools/oshrun), torchrun's
// RANK/WORLD_SIZE, PMI_RANK/PMI_SIZE, OMPI_COMM_WORLD_RANK/SIZE, SLURM_PROCID/NTASKS;
// none -> a singleton job.  Address: SHMEM_BOOTSTRAP_ADDR/PORT, else MASTER_ADDR and
// MASTER_PORT + 1 (torchrun's own store owns MASTER_PORT).
#include "bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
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

constexpr int kHubTimeoutMs = 600000;  // collective calls may be far apart in time

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

// ---------------------------------------------------------------------------------
// TCP hub: PE 0 accepts one connection per PE and relays
// ---------------------------------------------------------------------------------
int hub_connect(Hub *h, int rank, int size, char *err, size_t errlen)
{
    h->rank = rank;
    h->size = size;
    h->fds.assign(size > 1 ? (rank == 0 ? size : 1) : 0, -1);
    h->up = true;
    if (size == 1) return 0;
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
        h->up = false;
        return -1;
    }
    int timeout_s = 120;
    env_int("SHMEM_BOOTSTRAP_TIMEOUT", &timeout_s);
    const double deadline = now_s() + timeout_s;
    const int one = 1;

    if (rank == 0) {
        int ls = socket(AF_INET, SOCK_STREAM, 0);
        setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        struct sockaddr_in sa;
        memset(&sa, 0, sizeof(sa));
        sa.sin_family = AF_INET;
        sa.sin_addr.s_addr = htonl(INADDR_ANY);
        sa.sin_port = htons((uint16_t)port);
        if (bind(ls, (struct sockaddr *)&sa, sizeof(sa)) != 0 || listen(ls, 1024) != 0) {
            snprintf(err, errlen, "bootstrap bind/listen on port %d failed: %s", port, strerror(errno));
            close(ls);
            h->up = false;
            return -1;
        }
        for (int got = 1; got < size;) {
            struct pollfd pfd = {ls, POLLIN, 0};
            int left_ms = (int)((deadline - now_s()) * 1000);
            if (left_ms <= 0 || poll(&pfd, 1, left_ms) <= 0) {
                snprintf(err, errlen, "bootstrap: only %d of %d PEs connected", got, size);
                close(ls);
                h->up = false;
                return -1;
            }
            int fd = accept(ls, nullptr, nullptr);
            if (fd < 0) continue;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            int32_t r = -1;
            if (!recv_all(fd, &r, sizeof(r), 10000) || r <= 0 || r >= size || h->fds[r] >= 0) {
                close(fd);
                continue;
            }
            h->fds[r] = fd;
            ++got;
        }
        close(ls);
        return 0;
    }

    struct addrinfo hints, *res = nullptr;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    char portstr[16];
    snprintf(portstr, sizeof(portstr), "%d", port);
    if (getaddrinfo(addr, portstr, &hints, &res) != 0 || !res) {
        snprintf(err, errlen, "cannot resolve bootstrap address %s:%d", addr, port);
        h->up = false;
        return -1;
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
        h->up = false;
        return -1;
    }
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int32_t r = rank;
    if (!send_all(fd, &r, sizeof(r))) {
        close(fd);
        snprintf(err, errlen, "bootstrap: cannot register with PE 0");
        h->up = false;
        return -1;
    }
    h->fds[0] = fd;
    return 0;
}

int hub_bcast(Hub *h, void *buf, size_t len)
{
    if (!h->up) return -1;
    if (h->size == 1) return 0;
    if (h->rank == 0) {
        bool ok = true;
        for (int r = 1; r < h->size; ++r) ok &= send_all(h->fds[r], buf, len);
        return ok ? 0 : -1;
    }
    return recv_all(h->fds[0], buf, len, kHubTimeoutMs) ? 0 : -1;
}

int hub_allgather(Hub *h, const void *rec, size_t len, void *all)
{
    if (!h->up) return -1;
    char *out = (char *)all;
    memcpy(out + (size_t)h->rank * len, rec, len);
    if (h->size == 1) return 0;
    if (h->rank == 0) {
        for (int r = 1; r < h->size; ++r)
            if (!recv_all(h->fds[r], out + (size_t)r * len, len, kHubTimeoutMs)) return -1;
        return hub_bcast(h, out, (size_t)h->size * len);
    }
    if (!send_all(h->fds[0], rec, len)) return -1;
    return recv_all(h->fds[0], out, (size_t)h->size * len, kHubTimeoutMs) ? 0 : -1;
}

void hub_close(Hub *h)
{
    for (int fd : h->fds)
        if (fd >= 0) close(fd);
    h->fds.clear();
    h->up = false;
}

int exchange(int rank, int size, const void *root_blob, size_t root_len, void *out_blob,
             const void *my_rec, size_t rec_len, void *all_recs, char *err, size_t errlen)
{
    Hub h;
    if (hub_connect(&h, rank, size, err, errlen)) return -1;
    std::vector<char> blob((const char *)root_blob, (const char *)root_blob + root_len);
    int rc = hub_bcast(&h, blob.data(), root_len);
    if (!rc) rc = hub_allgather(&h, my_rec, rec_len, all_recs);
    if (!rc && out_blob) memcpy(out_blob, blob.data(), root_len);
    hub_close(&h);
    if (rc) snprintf(err, errlen, "bootstrap exchange failed");
    return rc;
}

// ---------------------------------------------------------------------------------
// shared-memory barrier
// ---------------------------------------------------------------------------------
namespace {
constexpr int kMaxPE = 64;
constexpr int kSlots = 256;
struct Slot {
    std::atomic<uint64_t> key;
    std::atomic<uint64_t> arrive[kMaxPE];
};
}  // namespace

bool ShmBarrier::attach(const char *name, bool create, int my_rank, size_t extra_bytes)
{
    rank = my_rank;
    const size_t slots_bytes = (sizeof(Slot) * kSlots + 4095) & ~(size_t)4095;
    bytes = slots_bytes + ((extra_bytes + 4095) & ~(size_t)4095);
    int fd = shm_open(name, O_RDWR | (create ? O_CREAT | O_EXCL : 0), 0600);
    if (fd < 0) return false;
    if (create && ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        return false;
    }
    void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return false;
    base = p;  // a fresh segment is zero-filled: every key 0, every counter 0
    extra = extra_bytes ? (char *)p + slots_bytes : nullptr;
    return true;
}

void ShmBarrier::detach()
{
    if (base) munmap(base, bytes);
    base = nullptr;
}

bool ShmBarrier::wait(int start, int stride, int size, double timeout_s)
{
    if (!base || size > kMaxPE || start + (size - 1) * stride >= kMaxPE) return false;
    if (size <= 1) return true;
    const uint64_t key = (((uint64_t)start << 42) | ((uint64_t)stride << 21) | (uint64_t)size) + 1;
    Slot *slots = (Slot *)base;
    uint64_t hsh = key * 0x9E3779B97F4A7C15ull;
    Slot *s = nullptr;
    for (int probe = 0; probe < kSlots; ++probe) {
        Slot *c = &slots[(hsh >> 32) % kSlots];
        hsh += 0x632BE59BD9B4E019ull;
        uint64_t k = c->key.load(std::memory_order_acquire);
        if (k == 0) {
            uint64_t zero = 0;
            if (c->key.compare_exchange_strong(zero, key)) k = key;
            else k = zero;
        }
        if (k == key) {
            s = c;
            break;
        }
    }
    if (!s) return false;
    uint64_t *mine = nullptr;
    for (auto &e : seq)
        if (e.first == key) mine = &e.second;
    if (!mine) {
        seq.push_back({key, 0});
        mine = &seq.back().second;
    }
    const uint64_t want = ++*mine;
    s->arrive[rank].store(want, std::memory_order_release);
    const double deadline = now_s() + timeout_s;
    for (int i = 0; i < size; ++i) {
        const int q = start + i * stride;
        unsigned spins = 0;
        while (s->arrive[q].load(std::memory_order_acquire) < want) {
            if (++spins < 2048) {
                __builtin_ia32_pause();
                continue;
            }
            sched_yield();
            if ((spins & 1023) == 0 && now_s() > deadline) return false;
        }
    }
    return true;
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

// Test hook: shared-memory barrier across the launcher's PEs (CPU only).  PE 0 creates
// the segment `name`, everyone attaches after a hub barrier, then runs `iters` barriers
// over the full set and over the even PEs; returns 0 if all completed.
extern "C" int sosx_shm_barrier_probe(const char *name, int iters)
{
    int r, s;
    sosboot::discover(&r, &s);
    sosboot::Hub h;
    char err[256];
    if (sosboot::hub_connect(&h, r, s, err, sizeof(err))) return -1;
    sosboot::ShmBarrier b;
    if (r == 0 && !b.attach(name, true, r)) return -2;
    int dummy = 0;
    std::vector<int> all((size_t)s);
    sosboot::hub_allgather(&h, &dummy, sizeof(int), all.data());
    if (r != 0 && !b.attach(name, false, r)) return -3;
    sosboot::hub_allgather(&h, &dummy, sizeof(int), all.data());
    if (r == 0) shm_unlink(name);
    for (int i = 0; i < iters; ++i) {
        if (!b.wait(0, 1, s, 30.0)) return -4;
        if (r % 2 == 0 && !b.wait(0, 2, (s + 1) / 2, 30.0)) return -5;
    }
    b.detach();
    hub_close(&h);
    return 0;
}
