// crash_trace.cpp — BAGUA_SEGV_TRACE=1: on SIGSEGV / SIGBUS print the native
// backtrace (frames as library+offset; addr2line -f -e lib/libbagua_core.so
// <offset> names them) to stderr, then hand the signal to the handler installed
// before (Python's faulthandler prints the Python stacks).  A diagnostic for host
// faults seen only on the GPU box; off by default.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>

namespace {

struct sigaction g_prev_segv, g_prev_bus;

void on_fault(int sig, siginfo_t* si, void* ctx) {
    static const char msg[] = "[bagua-core] fatal signal in the process; native backtrace:\n";
    ssize_t w = write(2, msg, sizeof msg - 1);
    (void)w;
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    const struct sigaction& prev = sig == SIGSEGV ? g_prev_segv : g_prev_bus;
    sigaction(sig, &prev, nullptr);
    if ((prev.sa_flags & SA_SIGINFO) && prev.sa_sigaction) {
        prev.sa_sigaction(sig, si, ctx);
    } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN && prev.sa_handler) {
        prev.sa_handler(sig);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

struct Install {
    Install() {
        const char* e = std::getenv("BAGUA_SEGV_TRACE");
        if (!e || *e != '1') return;
        // backtrace()'s first call may dlopen the unwinder and allocate, which a signal
        // handler must not do: call it once now, so the handler's call is the cheap one
        void* warm[4];
        (void)backtrace(warm, 4);
        // an alternate stack, so a stack overflow is reported too
        static char alt[64 * 1024];
        stack_t ss;
        std::memset(&ss, 0, sizeof ss);
        ss.ss_sp = alt;
        ss.ss_size = sizeof alt;
        (void)sigaltstack(&ss, nullptr);
        struct sigaction sa;
        std::memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = on_fault;
        sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
        sigemptyset(&sa.sa_mask);
        sigaction(SIGSEGV, &sa, &g_prev_segv);
        sigaction(SIGBUS, &sa, &g_prev_bus);
    }
} g_install;

}  // namespace
