/* Diagnostic only: a SIGSEGV / SIGBUS handler that prints the native stack as
 * "object(symbol+offset) [address]" lines (backtrace_symbols_fd: no malloc; resolve
 * further with addr2line -f -e <object> <offset>), then re-raises with the default action.  Loaded by tests/conftest.py
 * when RT_SEGV_BT=1 (after pytest's faulthandler, which shows Python frames only).
 *     gcc -O1 -g -shared -fPIC -o tools/libsegv_bt.so tools/segv_bt.c -ldl */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <fcntl.h>
#include <stdlib.h>

static int g_fd = 2;                            /* RT_SEGV_BT_FILE, else stderr (pytest may capture fd 2) */

static void on_fault(int sig, siginfo_t* si, void* uc) {
    (void)uc;
    alarm(10);                                   /* a handler stuck on a lock still ends the process */
    static const char hdr[] = "\nsegv_bt: native stack (object(+offset) [address]):\n";
    (void)!write(g_fd, hdr, sizeof hdr - 1);
    char line[64];
    const int m = snprintf(line, sizeof line, "segv_bt: signal %d, fault address %p\n", sig, si ? si->si_addr : NULL);
    if (m > 0) (void)!write(g_fd, line, (size_t)m);
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, g_fd);         /* no malloc: usable after heap corruption */
    signal(sig, SIG_DFL);
    raise(sig);
}

int segv_bt_install(void) {
    const char* path = getenv("RT_SEGV_BT_FILE");
    if (path && g_fd == 2) {
        const int fd = open(path, O_WRONLY | O_CREAT | O_APPEND, 0644);
        if (fd >= 0) g_fd = fd;
    }
    void* warm[4];
    (void)backtrace(warm, 4);                   /* loads libgcc_s now, not inside the handler */
    static char alt[1 << 16];                   /* this thread's faults run here, a stack overflow included */
    stack_t ss;
    memset(&ss, 0, sizeof ss);
    ss.ss_sp = alt;
    ss.ss_size = sizeof alt;
    if (sigaltstack(&ss, NULL) != 0) return -1;
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_fault;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGSEGV, &sa, NULL) != 0) return -1;
    if (sigaction(SIGBUS, &sa, NULL) != 0) return -1;
    return 0;
}
