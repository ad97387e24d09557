// TEST INFRASTRUCTURE ONLY -- never linked into sos_amd/libsos_amd.so.
//
// A stand-in for the ten RCCL entry points libsos_amd.so calls (ncclGetUniqueId,
// ncclCommInitRank, ncclCommDestroy, ncclGetErrorString, ncclGroupStart/End, ncclSend,
// ncclRecv, ncclAllGather, ncclAllReduce), linked with hidden visibility into a test copy of the library,
// tests/fakerccl/libsos_amd_fakerccl.so.  Real RCCL refuses two ranks on one GPU
// ("Duplicate GPU detected"), and the GPU box has one, so without this the RCCL executor
// (collectives.cpp exec_rccl, the RCCL device barrier and team words in runtime.cpp) only
// ever runs with several PEs on the driver's 8-GPU node.  With it, the same executor code
// runs with P real PE processes on one GPU, and every plan's send/receive pairing, byte
// offsets and stream ordering are checked bit-exactly by the same checkers as the p2p runs.
//
// Semantics (stricter than RCCL's, which is what a correctness harness wants):
//   * ncclSend/ncclRecv outside a group run as a group of one;
//   * ncclGroupEnd synchronises every stream named in the group (so the send buffers hold
//     what the stream order says they hold), then posts every send as a file
//     /dev/shm/fakerccl_<id>_<src>_<dst>_<seq> (written under a temporary name, then
//     renamed), then waits for each receive's file, copies it into the receive buffer
//     and unlinks it.  It returns with all transfers complete.
//   * ncclAllGather is a group of one send of the contribution to every peer and one
//     receive from every peer into its slot, plus the local copy when not in place;
//   * ncclAllReduce sends the whole send buffer to every peer, receives every peer's,
//     and folds the P buffers on the host in rank order (sum/prod/min/max of the 8/32/64-bit
//     integer and fp32/fp64 types; integers in two's complement);
//   * messages of one ordered pair match in issue order through per-pair sequence numbers,
//     RCCL's FIFO rule; a size mismatch or a wait longer than FAKERCCL_TIMEOUT seconds
//     (default 120) returns an error, which libsos_amd.so turns into an abort.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

struct ncclComm {
    int nranks, rank;
    char key[33];
    std::vector<unsigned long long> sent, recvd;  // per-peer sequence numbers
};

namespace {

struct Op {
    bool send;
    void *buf;
    size_t bytes;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};

int g_depth = 0;
std::vector<Op> g_ops;
unsigned long long g_msgs = 0, g_bytes = 0, g_allgathers = 0, g_allreduces = 0;
int g_rank = -1;

// FAKERCCL_STATS=1: each process reports how much went through the stand-in, so a test can
// tell that the RCCL executor really ran.
__attribute__((destructor)) void report()
{
    const char *e = getenv("FAKERCCL_STATS");
    if (e && *e == '1' && g_rank >= 0)
        fprintf(stderr, "fakerccl stats: rank %d sent %llu messages, %llu bytes, %llu allgathers, "
                "%llu allreduces\n", g_rank, g_msgs, g_bytes, g_allgathers, g_allreduces);
}

double now_s()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

size_t type_size(ncclDataType_t t)
{
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

std::string msg_path(const ncclComm *c, int src, int dst, unsigned long long seq)
{
    char p[160];
    snprintf(p, sizeof p, "/dev/shm/fakerccl_%s_%d_%d_%llu", c->key, src, dst, seq);
    return p;
}

bool write_all(int fd, const char *p, size_t n)
{
    while (n) {
        const ssize_t w = write(fd, p, n);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return false;
        p += w;
        n -= (size_t)w;
    }
    return true;
}

bool read_all(int fd, char *p, size_t n)
{
    while (n) {
        const ssize_t r = read(fd, p, n);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        p += r;
        n -= (size_t)r;
    }
    return true;
}

ncclResult_t post_send(const Op &o, std::vector<char> &tmp)
{
    ncclComm *c = o.comm;
    tmp.resize(o.bytes);
    if (o.bytes && hipMemcpy(tmp.data(), o.buf, o.bytes, hipMemcpyDefault) != hipSuccess)
        return ncclUnhandledCudaError;
    const std::string fin = msg_path(c, c->rank, o.peer, c->sent[(size_t)o.peer]++);
    const std::string part = fin + ".part";
    const int fd = open(part.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0600);
    if (fd < 0) return ncclSystemError;
    const bool ok = write_all(fd, tmp.data(), o.bytes);
    close(fd);
    if (!ok || rename(part.c_str(), fin.c_str()) != 0) return ncclSystemError;
    ++g_msgs;
    g_bytes += o.bytes;
    return ncclSuccess;
}

ncclResult_t complete_recv(const Op &o, std::vector<char> &tmp)
{
    ncclComm *c = o.comm;
    const std::string fin = msg_path(c, o.peer, c->rank, c->recvd[(size_t)o.peer]++);
    const char *e = getenv("FAKERCCL_TIMEOUT");
    const double limit = e ? atof(e) : 120.0, t0 = now_s();
    int fd;
    while ((fd = open(fin.c_str(), O_RDONLY)) < 0) {
        if (now_s() - t0 > limit) {
            fprintf(stderr, "fakerccl error: rank %d timed out waiting for %s\n", c->rank, fin.c_str());
            return ncclSystemError;
        }
        usleep(20);
    }
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size != o.bytes) {
        fprintf(stderr, "fakerccl error: rank %d: %s holds %lld bytes, receive expects %zu\n", c->rank,
                fin.c_str(), (long long)st.st_size, o.bytes);
        close(fd);
        return ncclInvalidUsage;
    }
    tmp.resize(o.bytes);
    const bool ok = read_all(fd, tmp.data(), o.bytes);
    close(fd);
    unlink(fin.c_str());
    if (!ok) return ncclSystemError;
    if (o.bytes && hipMemcpy(o.buf, tmp.data(), o.bytes, hipMemcpyDefault) != hipSuccess)
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

ncclResult_t run_group()
{
    std::vector<Op> ops;
    ops.swap(g_ops);
    std::vector<hipStream_t> synced;
    for (const Op &o : ops) {
        bool seen = false;
        for (hipStream_t s : synced) seen |= s == o.stream;
        if (seen) continue;
        if (hipStreamSynchronize(o.stream) != hipSuccess) return ncclUnhandledCudaError;
        synced.push_back(o.stream);
    }
    std::vector<char> tmp;
    for (const Op &o : ops)
        if (o.send) {
            const ncclResult_t r = post_send(o, tmp);
            if (r != ncclSuccess) return r;
        }
    for (const Op &o : ops)
        if (!o.send) {
            const ncclResult_t r = complete_recv(o, tmp);
            if (r != ncclSuccess) return r;
        }
    return ncclSuccess;
}

ncclResult_t enqueue(bool send, const void *buf, size_t count, ncclDataType_t t, int peer,
                     ncclComm_t comm, hipStream_t stream)
{
    const size_t ts = type_size(t);
    if (!comm || !ts || peer < 0 || peer >= comm->nranks || peer == comm->rank)
        return ncclInvalidArgument;
    g_ops.push_back({send, const_cast<void *>(buf), count * ts, peer, comm, stream});
    return g_depth ? ncclSuccess : run_group();
}

}  // namespace

ncclResult_t ncclGetUniqueId(ncclUniqueId *id)
{
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof *id);
    timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    snprintf(id->internal, sizeof id->internal, "%08x%08lx%08lx%08x", (unsigned)getpid(),
             (unsigned long)t.tv_sec & 0xffffffffUL, (unsigned long)t.tv_nsec, (unsigned)rand());
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank)
{
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks || !id.internal[0])
        return ncclInvalidArgument;
    ncclComm *c = new ncclComm;
    c->nranks = nranks;
    c->rank = rank;
    snprintf(c->key, sizeof c->key, "%.32s", id.internal);
    c->sent.assign((size_t)nranks, 0);
    c->recvd.assign((size_t)nranks, 0);
    g_rank = rank;
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int *count)
{
    if (!comm || !count) return ncclInvalidArgument;
    *count = comm->nranks;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm)
{
    delete comm;
    return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t r)
{
    switch (r) {
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "fakerccl: HIP call failed";
    case ncclSystemError: return "fakerccl: system error or timeout";
    case ncclInvalidArgument: return "fakerccl: invalid argument";
    case ncclInvalidUsage: return "fakerccl: send/receive size mismatch";
    default: return "fakerccl: error";
    }
}

ncclResult_t ncclGroupStart()
{
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd()
{
    if (g_depth <= 0) return ncclInvalidUsage;
    return --g_depth ? ncclSuccess : run_group();
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                      hipStream_t stream)
{
    return enqueue(true, buf, count, t, peer, comm, stream);
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                      hipStream_t stream)
{
    return enqueue(false, buf, count, t, peer, comm, stream);
}

ncclResult_t ncclAllGather(const void *sendbuff, void *recvbuff, size_t sendcount,
                           ncclDataType_t t, ncclComm_t comm, hipStream_t stream)
{
    const size_t ts = type_size(t);
    if (!comm || !ts || g_depth) return ncclInvalidArgument;
    const size_t bytes = sendcount * ts;
    char *mine = (char *)recvbuff + (size_t)comm->rank * bytes;
    ++g_allgathers;
    ncclGroupStart();
    for (int q = 0; q < comm->nranks; ++q) {
        if (q == comm->rank) continue;
        enqueue(true, sendbuff, sendcount, t, q, comm, stream);
        enqueue(false, (char *)recvbuff + (size_t)q * bytes, sendcount, t, q, comm, stream);
    }
    const ncclResult_t r = ncclGroupEnd();
    if (r != ncclSuccess) return r;
    if (mine != sendbuff && bytes &&
        hipMemcpyAsync(mine, sendbuff, bytes, hipMemcpyDefault, stream) != hipSuccess)
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

namespace {

template <class T> void fold_into(T *acc, const T *x, size_t n, ncclRedOp_t op)
{
    for (size_t i = 0; i < n; ++i) {
        switch (op) {
        case ncclSum: acc[i] = (T)(acc[i] + x[i]); break;
        case ncclProd: acc[i] = (T)(acc[i] * x[i]); break;
        case ncclMin: acc[i] = x[i] < acc[i] ? x[i] : acc[i]; break;
        case ncclMax: acc[i] = x[i] > acc[i] ? x[i] : acc[i]; break;
        default: break;
        }
    }
}

// integer sum/prod in the unsigned type of the same width (two's-complement wrap, no UB)
bool fold_typed(char *acc, const char *x, size_t n, ncclDataType_t t, ncclRedOp_t op)
{
    const bool arith = op == ncclSum || op == ncclProd;
    switch (t) {
    case ncclInt8: arith ? fold_into((uint8_t *)acc, (const uint8_t *)x, n, op)
                         : fold_into((int8_t *)acc, (const int8_t *)x, n, op); return true;
    case ncclUint8: fold_into((uint8_t *)acc, (const uint8_t *)x, n, op); return true;
    case ncclInt32: arith ? fold_into((uint32_t *)acc, (const uint32_t *)x, n, op)
                          : fold_into((int32_t *)acc, (const int32_t *)x, n, op); return true;
    case ncclUint32: fold_into((uint32_t *)acc, (const uint32_t *)x, n, op); return true;
    case ncclInt64: arith ? fold_into((uint64_t *)acc, (const uint64_t *)x, n, op)
                          : fold_into((int64_t *)acc, (const int64_t *)x, n, op); return true;
    case ncclUint64: fold_into((uint64_t *)acc, (const uint64_t *)x, n, op); return true;
    case ncclFloat32: fold_into((float *)acc, (const float *)x, n, op); return true;
    case ncclFloat64: fold_into((double *)acc, (const double *)x, n, op); return true;
    default: return false;
    }
}

}  // namespace

ncclResult_t ncclAllReduce(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t t,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream)
{
    const size_t ts = type_size(t);
    if (!comm || !ts || g_depth || op < ncclSum || op > ncclMin) return ncclInvalidArgument;
    const size_t bytes = count * ts;
    const int P = comm->nranks;
    ++g_allreduces;
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    std::vector<std::vector<char>> all((size_t)P, std::vector<char>(bytes));
    if (bytes && hipMemcpy(all[(size_t)comm->rank].data(), sendbuff, bytes, hipMemcpyDefault) != hipSuccess)
        return ncclUnhandledCudaError;
    std::vector<char> tmp;
    for (int q = 0; q < P; ++q) {
        if (q == comm->rank) continue;
        const ncclResult_t r = post_send({true, const_cast<void *>(sendbuff), bytes, q, comm, stream}, tmp);
        if (r != ncclSuccess) return r;
    }
    for (int q = 0; q < P; ++q) {
        if (q == comm->rank) continue;
        // receive into host memory: complete_recv copies with hipMemcpyDefault
        const ncclResult_t r = complete_recv({false, all[(size_t)q].data(), bytes, q, comm, stream}, tmp);
        if (r != ncclSuccess) return r;
    }
    std::vector<char> acc = all[0];
    for (int q = 1; q < P; ++q)
        if (!fold_typed(acc.data(), all[(size_t)q].data(), count, t, op)) return ncclInvalidArgument;
    if (bytes && hipMemcpy(recvbuff, acc.data(), bytes, hipMemcpyDefault) != hipSuccess)
        return ncclUnhandledCudaError;
    return ncclSuccess;
}
