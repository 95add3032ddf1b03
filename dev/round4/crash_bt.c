// Developer tool (not part of the library): a fatal-signal handler that prints the native
// backtrace (addresses + the nearest exported symbol) on an alternate stack, so a stack
// overflow inside a stripped runtime library still leaves its repeating frame on stderr.
// Load it with ctypes before the code under test:
//   gcc -shared -fPIC -O1 -o /tmp/crash_bt.so crash_bt.c
//   python -c "import ctypes; ctypes.CDLL('/tmp/crash_bt.so'); ..."
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static void on_fatal(int sig) {
    void* frames[48];
    const int n = backtrace(frames, 48);
    static const char hdr[] = "crash_bt: fatal signal, native backtrace:\n";
    (void)!write(2, hdr, sizeof(hdr) - 1);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void crash_bt_install(void) {
    static char alt[1 << 16];
    stack_t ss;
    memset(&ss, 0, sizeof(ss));
    ss.ss_sp = alt;
    ss.ss_size = sizeof(alt);
    sigaltstack(&ss, 0);
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_fatal;
    sa.sa_flags = SA_ONSTACK;
    sigaction(SIGSEGV, &sa, 0);
    sigaction(SIGBUS, &sa, 0);
    sigaction(SIGABRT, &sa, 0);
}
