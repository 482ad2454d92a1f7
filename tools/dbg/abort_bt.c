/* Diagnostic: a SIGABRT handler that prints the native backtrace of the aborting thread to
 * stderr (loaded with ctypes before pytest installs faulthandler, which chains to it). */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_abort(int sig) {
    void* pc[64];
    const int n = backtrace(pc, 64);
    static const char msg[] = "\n==== native backtrace (SIGABRT) ====\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(pc, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_abort;
    sigaction(SIGABRT, &sa, 0);
}
