// Native backtrace on a fatal signal.  Python's faulthandler only sees threads that hold a Python thread state;
// a fault on a native thread (the DynamicBatcher instance thread driving the executor, a front-end worker, a HIP
// runtime thread) ends the process with no frame at all (profiles/r4lanes/detection_lanes_dbg.log).  This
// handler prints the faulting thread's native stack (glibc backtrace(): "object(symbol+offset) [address]", and
// each frame's offset inside its object, for addr2line on the host) to stderr, then hands the signal to the
// handler that was installed before it (faulthandler, or the default action -> core).
#include "crash_trace.h"

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

namespace arena {
namespace {

constexpr int kSignals[] = {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT};
constexpr int kNumSignals = sizeof(kSignals) / sizeof(int);
struct sigaction g_prev[kNumSignals];
bool g_installed = false;
alignas(16) char g_altstack[64 * 1024];

void write_str(const char* s) {
  ssize_t r = ::write(2, s, strlen(s));
  (void)r;
}

// async-signal-safe decimal / hex formatting (no stdio in the handler)
void write_num(unsigned long long v, int base) {
  char buf[32];
  int n = 0;
  do {
    const int d = (int)(v % base);
    buf[n++] = (char)(d < 10 ? '0' + d : 'a' + d - 10);
    v /= base;
  } while (v && n < 31);
  char out[34];
  int k = 0;
  if (base == 16) {
    out[k++] = '0';
    out[k++] = 'x';
  }
  while (n) out[k++] = buf[--n];
  out[k] = 0;
  write_str(out);
}

void handler(int sig, siginfo_t* info, void* uctx) {
  write_str("\n[arena crash] fatal signal ");
  write_num((unsigned)sig, 10);
  write_str(" (");
  write_str(sig == SIGSEGV ? "SIGSEGV" : sig == SIGBUS ? "SIGBUS" : sig == SIGABRT ? "SIGABRT" : sig == SIGFPE ? "SIGFPE" : "SIGILL");
  write_str(") on native thread ");
  write_num((unsigned long long)syscall(SYS_gettid), 10);
  if (sig == SIGSEGV || sig == SIGBUS) {
    write_str(", fault address ");
    write_num((unsigned long long)(uintptr_t)info->si_addr, 16);
  }
  write_str("\n");
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  // object-relative offsets: `addr2line -e <object> <offset>` against the same build resolves file:line
  for (int i = 0; i < n; ++i) {
    Dl_info di;
    if (dladdr(frames[i], &di) && di.dli_fname != nullptr) {
      write_str("[arena crash]   #");
      write_num((unsigned)i, 10);
      write_str(" ");
      write_str(di.dli_fname);
      write_str(" +");
      write_num((unsigned long long)((uintptr_t)frames[i] - (uintptr_t)di.dli_fbase), 16);
      write_str("\n");
    }
  }
  // chain: the previous handler (faulthandler prints the Python threads), else the default action
  for (int i = 0; i < kNumSignals; ++i) {
    if (kSignals[i] != sig) continue;
    const struct sigaction& p = g_prev[i];
    if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction != nullptr) {
      p.sa_sigaction(sig, info, uctx);
      return;
    }
    if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler != nullptr) {
      p.sa_handler(sig);
      return;
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

void stack_handler(int, siginfo_t*, void*) {
  write_str("[arena stack] thread ");
  write_num((unsigned long long)syscall(SYS_gettid), 10);
  write_str("\n");
  void* frames[48];
  const int n = backtrace(frames, 48);
  for (int i = 0; i < n; ++i) {
    Dl_info di;
    write_str("[arena stack]   #");
    write_num((unsigned)i, 10);
    write_str(" ");
    if (dladdr(frames[i], &di) && di.dli_fname != nullptr) {
      write_str(di.dli_fname);
      write_str(" +");
      write_num((unsigned long long)((uintptr_t)frames[i] - (uintptr_t)di.dli_fbase), 16);
      if (di.dli_sname != nullptr) {
        write_str(" ");
        write_str(di.dli_sname);
        write_str("+");
        write_num((unsigned long long)((uintptr_t)frames[i] - (uintptr_t)di.dli_saddr), 16);
      }
    } else {
      write_num((unsigned long long)(uintptr_t)frames[i], 16);
    }
    write_str("\n");
  }
}

}  // namespace

bool dump_thread_stack(int tid) {
  static bool installed = false;
  if (!installed) {
    void* warm[2];
    backtrace(warm, 2);
    struct sigaction sa{};
    sa.sa_sigaction = stack_handler;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGUSR2, &sa, nullptr);
    installed = true;
  }
  return syscall(SYS_tgkill, getpid(), tid, SIGUSR2) == 0;
}

bool install_crash_trace() {
  if (g_installed) return false;
  // backtrace() loads libgcc_s on first use (malloc): do that now, not inside the handler
  void* warm[2];
  backtrace(warm, 2);
  stack_t ss{};
  ss.ss_sp = g_altstack;
  ss.ss_size = sizeof(g_altstack);
  sigaltstack(&ss, nullptr);
  for (int i = 0; i < kNumSignals; ++i) {
    struct sigaction sa{};
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kSignals[i], &sa, &g_prev[i]);
  }
  g_installed = true;
  return true;
}

bool crash_trace_installed() { return g_installed; }

}  // namespace arena
