/* Diagnostic: print a native backtrace on SIGSEGV / SIGABRT to stderr, then
 * die with the same signal.  A tool loads it with ctypes.CDLL (its
 * constructor installs the handlers) to find where a crash lies when no
 * debugger runs on the GPU box, e.g. in a library's teardown at exit, after
 * Python's faulthandler is gone.  Not part of the product. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig) {
    void* frames[64];
    const char msg[] = "segv_trace: native backtrace\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_fault;
    sa.sa_flags = SA_RESETHAND;
    sigaction(SIGSEGV, &sa, 0);
    sigaction(SIGABRT, &sa, 0);
}
