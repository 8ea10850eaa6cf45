/* SIGSEGV diagnostics for host-side crashes inside the HIP runtime.
 *
 * Loaded with ctypes (never LD_PRELOAD); segv_trace_install() installs a
 * SIGSEGV handler that prints, for every frame of the native backtrace, the
 * shared object, the address's offset inside it and the nearest dynamic
 * symbol, plus the faulting address -- so a crash in a stripped library can be
 * located with llvm-objdump offline -- and then chains to the handler that was
 * installed before (Python's faulthandler), which prints the Python stack.
 *
 * Build: gcc -O1 -g -shared -fPIC -o tools/_segv_trace.so tools/segv_trace.c -ldl
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_prev;

static void on_segv(int sig, siginfo_t *si, void *uc) {
    char line[512];
    int n = snprintf(line, sizeof line, "segv_trace: signal %d, fault address %p\n", sig, si->si_addr);
    write(2, line, n);
    void *frames[64];
    int k = backtrace(frames, 64);
    for (int i = 0; i < k; ++i) {
        Dl_info d;
        memset(&d, 0, sizeof d);
        if (dladdr(frames[i], &d) && d.dli_fname) {
            unsigned long off = (unsigned long)frames[i] - (unsigned long)d.dli_fbase;
            long soff = d.dli_saddr ? (long)((char *)frames[i] - (char *)d.dli_saddr) : -1;
            n = snprintf(line, sizeof line, "  #%02d %p %s+0x%lx (%s+%ld)\n", i, frames[i], d.dli_fname, off,
                         d.dli_sname ? d.dli_sname : "?", soff);
        } else {
            n = snprintf(line, sizeof line, "  #%02d %p ?\n", i, frames[i]);
        }
        write(2, line, n);
    }
    sigaction(SIGSEGV, &g_prev, NULL);
    if (g_prev.sa_flags & SA_SIGINFO) {
        if (g_prev.sa_sigaction) g_prev.sa_sigaction(sig, si, uc);
    } else if (g_prev.sa_handler != SIG_IGN && g_prev.sa_handler != SIG_DFL) {
        g_prev.sa_handler(sig);
    }
    raise(sig);
}

int segv_trace_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    return sigaction(SIGSEGV, &sa, &g_prev);
}
