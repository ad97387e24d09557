/* Diagnostic: on SIGABRT/SIGSEGV print raw return addresses and /proc/self/maps (no
 * malloc, no loader lock: the crash may happen inside exit-time destructors), for
 * offline symbolisation.  Loaded by tests/conftest.py when SOSX_CRASHTRACE=1. */
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void put(const char *s) { if (write(2, s, strlen(s)) < 0) _exit(98); }

static void puthex(unsigned long v)
{
    char b[20];
    int i = 19;
    b[i--] = 0;
    do { b[i--] = "0123456789abcdef"[v & 15]; v >>= 4; } while (v && i > 1);
    b[i--] = 'x';
    b[i] = '0';
    put(&b[i]);
}

static void handler(int sig)
{
    void *frames[64];
    int n = backtrace(frames, 64);
    put("\n*** crashtrace frames ***\n");
    for (int i = 0; i < n; ++i) { puthex((unsigned long)frames[i]); put("\n"); }
    put("*** maps ***\n");
    int fd = open("/proc/self/maps", O_RDONLY);
    char buf[4096];
    ssize_t r;
    while (fd >= 0 && (r = read(fd, buf, sizeof buf)) > 0)
        if (write(2, buf, (size_t)r) < 0) break;
    put("*** end ***\n");
    _exit(97);
}

__attribute__((constructor)) static void install(void)
{
    void *warm[2];
    backtrace(warm, 2);
    signal(SIGABRT, handler);
    signal(SIGSEGV, handler);
}
