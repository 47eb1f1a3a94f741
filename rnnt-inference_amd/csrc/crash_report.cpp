// crash_report.cpp -- rnnt_install_crash_report(): on a fatal signal, print every stack frame as
// shared object + offset (dladdr), then hand the signal to the handler that was installed before (a
// profiler's, or the default core dump).  Round 5 saw one SIGSEGV inside __cxa_finalize at the exit of a
// rocprofv3-traced bench run whose report named no library ("teardown"); with this
// installed, a recurrence names the object whose static destructor faulted.  Host code only.
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>

#include "../../include/rnnt_mi355x.h"

namespace {

constexpr int kSignals[] = {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT};
struct sigaction g_prev[65];
volatile sig_atomic_t g_installed = 0;

void put(const char* s) { (void)!write(2, s, strlen(s)); }

void put_num(uintptr_t v, int base) {
  char buf[32];
  int i = (int)sizeof(buf);
  buf[--i] = 0;
  do {
    const int d = (int)(v % (uintptr_t)base);
    buf[--i] = (char)(d < 10 ? '0' + d : 'a' + d - 10);
    v /= (uintptr_t)base;
  } while (v && i > 2);
  if (base == 16) {
    buf[--i] = 'x';
    buf[--i] = '0';
  }
  put(buf + i);
}

void on_fatal(int sig, siginfo_t* si, void* ctx) {
  put("rnnt crash report: signal ");
  put_num((uintptr_t)sig, 10);
  put(" at address ");
  put_num((uintptr_t)(si ? si->si_addr : nullptr), 16);
  put("\n");
  void* frames[64];
  const int n = backtrace(frames, 64);
  for (int i = 0; i < n; ++i) {
    Dl_info di;
    put("  #");
    put_num((uintptr_t)i, 10);
    put(" ");
    put_num((uintptr_t)frames[i], 16);
    if (dladdr(frames[i], &di) && di.dli_fname) {
      put(" ");
      put(di.dli_fname);
      put("+");
      put_num((uintptr_t)frames[i] - (uintptr_t)di.dli_fbase, 16);
      if (di.dli_sname) {
        put(" (");
        put(di.dli_sname);
        put(")");
      }
    }
    put("\n");
  }
  // the previous disposition takes over (a profiler's report, or the default action): a fault re-executes
  // the faulting instruction on return and arrives there with its own siginfo; a sent signal is re-sent
  (void)ctx;
  sigaction(sig, &g_prev[sig], nullptr);
  if (!si || si->si_code <= 0) raise(sig);
}

}  // namespace

extern "C" int rnnt_install_crash_report(void) {
  if (g_installed) return 0;
  void* warm[2];
  (void)backtrace(warm, 2);  // loads the unwinder now, not inside the handler
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_fatal;
  sa.sa_flags = SA_SIGINFO;
  sigemptyset(&sa.sa_mask);
  for (int s : kSignals)
    if (sigaction(s, &sa, &g_prev[s]) != 0) return RNNT_EINVAL;
  g_installed = 1;
  return 0;
}
