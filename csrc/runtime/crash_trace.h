// Native backtrace on fatal signals (SIGSEGV/SIGBUS/SIGFPE/SIGILL/SIGABRT), chained to the previous handler.
#pragma once

namespace arena {

// Installs the handler once per process (false when already installed).  The alternate signal stack is
// registered for the calling thread only; other threads run the handler on their own stacks.
bool install_crash_trace();
bool crash_trace_installed();
// Diagnostics: the native stack of thread `tid` of this process, printed to stderr by that thread (SIGUSR2).
bool dump_thread_stack(int tid);

}  // namespace arena
