/* Debug aid for tools/rccl_capture_probe.py: print the native backtrace of a SIGSEGV to
 * stderr (there is no gdb on the GPU box), then re-raise so faulthandler and the default
 * action still run.  Built by the probe with gcc -shared; never part of the product. */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_segv(int sig) {
  void* frames[64];
  int n = backtrace(frames, 64);
  const char msg[] = "---- native backtrace (segv_bt) ----\n";
  write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void segv_bt_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_segv;
  sigaction(SIGSEGV, &sa, 0);
}
