/* Diagnostic: on SIGABRT/SIGSEGV write the interrupted context's RIP/RSP, the raw bytes
 * of the stack above RSP and /proc/self/maps to files, using only async-signal-safe
 * calls (no backtrace(): it can take the loader lock, and a crash inside exit-time
 * teardown may already hold it).  tools/diag/symbolize.py turns the dump into a
 * call chain offline, against the same library files.
 * Output: $SOSX_CRASHTRACE_OUT.{regs,stack,maps} (default /tmp/crashtrace).
 * Loaded by tests/conftest.py when SOSX_CRASHTRACE=1. */
#define _GNU_SOURCE
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <ucontext.h>
#include <unistd.h>

static char g_prefix[512] = "/tmp/crashtrace";

static void put(int fd, const char *s) { if (write(fd, s, strlen(s)) < 0) _exit(98); }

static void puthex(int fd, unsigned long v)
{
    char b[24];
    int i = 23;
    b[i--] = 0;
    do { b[i--] = "0123456789abcdef"[v & 15]; v >>= 4; } while (v && i > 1);
    b[i--] = 'x';
    b[i] = '0';
    put(fd, &b[i]);
}

static int open_out(const char *suffix)
{
    char path[600];
    size_t n = strlen(g_prefix), m = strlen(suffix);
    if (n + m + 1 > sizeof(path)) return -1;
    memcpy(path, g_prefix, n);
    memcpy(path + n, suffix, m + 1);
    return open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
}

/* end of the mapping that holds `addr`, parsed from /proc/self/maps without malloc */
static uintptr_t mapping_end(uintptr_t addr)
{
    int fd = open("/proc/self/maps", O_RDONLY);
    if (fd < 0) return addr;
    char buf[8192];
    char line[512];
    size_t ll = 0;
    uintptr_t found = addr;
    ssize_t r;
    while ((r = read(fd, buf, sizeof buf)) > 0) {
        for (ssize_t i = 0; i < r; ++i) {
            if (buf[i] != '\n') {
                if (ll + 1 < sizeof line) line[ll++] = buf[i];
                continue;
            }
            line[ll] = 0;
            ll = 0;
            uintptr_t lo = 0, hi = 0;
            char *p = line;
            while (*p && *p != '-') { lo = lo * 16 + (uintptr_t)(*p <= '9' ? *p - '0' : *p - 'a' + 10); ++p; }
            if (*p == '-') ++p;
            while (*p && *p != ' ') { hi = hi * 16 + (uintptr_t)(*p <= '9' ? *p - '0' : *p - 'a' + 10); ++p; }
            if (addr >= lo && addr < hi) found = hi;
        }
    }
    close(fd);
    return found;
}

static void handler(int sig, siginfo_t *si, void *ctx)
{
    (void)si;
    ucontext_t *uc = (ucontext_t *)ctx;
    uintptr_t rsp = (uintptr_t)uc->uc_mcontext.gregs[REG_RSP];
    uintptr_t rip = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
    int fd = open_out(".regs");
    if (fd >= 0) {
        put(fd, "sig "); puthex(fd, (unsigned long)sig);
        put(fd, "\nrip "); puthex(fd, rip);
        put(fd, "\nrsp "); puthex(fd, rsp);
        put(fd, "\n");
        close(fd);
    }
    uintptr_t end = mapping_end(rsp);
    if (end - rsp > (1u << 20)) end = rsp + (1u << 20);
    fd = open_out(".stack");
    if (fd >= 0) {
        if (write(fd, (const void *)rsp, end - rsp) < 0) {}
        close(fd);
    }
    fd = open_out(".maps");
    int in = open("/proc/self/maps", O_RDONLY);
    char buf[4096];
    ssize_t r;
    while (fd >= 0 && in >= 0 && (r = read(in, buf, sizeof buf)) > 0)
        if (write(fd, buf, (size_t)r) < 0) break;
    if (in >= 0) close(in);
    if (fd >= 0) close(fd);
    put(2, "\n*** crashtrace: dump written ***\n");
    _exit(97);
}

__attribute__((constructor)) static void install(void)
{
    const char *p = getenv("SOSX_CRASHTRACE_OUT");
    if (p && strlen(p) + 8 < sizeof g_prefix) strcpy(g_prefix, p);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigaction(SIGABRT, &sa, 0);
    sigaction(SIGSEGV, &sa, 0);
}
