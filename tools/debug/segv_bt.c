// Debug aid: loaded with ctypes into a repro script, prints the native
// backtrace when the process takes SIGSEGV (then dies as before).
//   gcc -shared -fPIC -O1 -g -o /tmp/segv_bt.so tools/debug/segv_bt.c
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>
static void h(int sig) {
    void *b[64];
    int n = backtrace(b, 64);
    const char msg[] = "\n=== SIGSEGV native backtrace ===\n";
    if (write(2, msg, sizeof msg - 1) < 0) return;
    backtrace_symbols_fd(b, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
// Call after the runtimes are loaded (they may install handlers of their own).
void segv_bt_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = h;
    sa.sa_flags = SA_RESETHAND;
    sigaction(SIGSEGV, &sa, 0);
}
