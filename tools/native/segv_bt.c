/* Host-side crash diagnostics: a SIGSEGV/SIGABRT handler that prints the native backtrace
 * (glibc backtrace_symbols_fd) to stderr before the default action. Loaded into a Python process by
 * ctypes when MX_SEGV_BT=1 (tests/conftest.py); touches no GPU state.
 * Build: gcc -O1 -g -shared -fPIC -rdynamic tools/native/segv_bt.c -o tools/native/libsegvbt.so */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void handler(int sig) {
  void* frames[64];
  const char msg[] = "\n[segv_bt] native backtrace:\n";
  write(2, msg, sizeof(msg) - 1);
  int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int mx_segv_bt_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = handler;
  sa.sa_flags = SA_RESETHAND | SA_NODEFER;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGABRT, &sa, 0);
  void* warm[2];
  backtrace(warm, 2); /* load libgcc's unwinder now, not inside the handler */
  return 0;
}
