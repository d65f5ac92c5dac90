// Crash attribution for exit-time faults: loaded into a Python worker with
// ctypes.CDLL (not LD_PRELOAD), its constructor installs SIGSEGV / SIGABRT / SIGBUS handlers on
// an alternate stack.  On a fault the handler writes, to stderr and to $FISDF_CRASH_OUT if set:
// the signal, the faulting address, the thread id, the native backtrace (backtrace_symbols_fd:
// exported symbol + offset where the library has one) and, per frame, the mapping it falls in
// with its offset into that file, so a stripped frame can be symbolized afterwards with
// `llvm-symbolizer --obj=<file> <offset>` or `nm -D`.  Then the default action runs (core dump).
// Build: gcc -O1 -g -shared -fPIC tools/crashtrace.c -o tools/libcrashtrace.so -ldl
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

static char alt_stack[1 << 16];
static int out_fd = -1;

static void put(int fd, const char* s) {
  if (fd >= 0) {
    ssize_t r = write(fd, s, strlen(s));
    (void)r;
  }
}

static void both(const char* s) {
  put(2, s);
  put(out_fd, s);
}

static void frame_maps(void* pc) {
  // find the /proc/self/maps line holding pc (no stdio: read in chunks)
  int fd = open("/proc/self/maps", O_RDONLY);
  if (fd < 0) return;
  static char buf[1 << 20];
  ssize_t n = 0, r;
  while (n < (ssize_t)sizeof(buf) - 1 && (r = read(fd, buf + n, sizeof(buf) - 1 - n)) > 0) n += r;
  close(fd);
  buf[n] = 0;
  char* line = buf;
  while (line && *line) {
    char* nl = strchr(line, '\n');
    if (nl) *nl = 0;
    unsigned long lo = 0, hi = 0, off = 0;
    char perm[8] = {0};
    if (sscanf(line, "%lx-%lx %7s %lx", &lo, &hi, perm, &off) == 4 && (uintptr_t)pc >= lo &&
        (uintptr_t)pc < hi) {
      char msg[1200];
      const char* path = strchr(line, '/');
      snprintf(msg, sizeof(msg), "    in %s  file offset 0x%lx\n", path ? path : "[anon]",
               (unsigned long)((uintptr_t)pc - lo + off));
      both(msg);
      break;
    }
    line = nl ? nl + 1 : NULL;
  }
}

static void handler(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  char msg[256];
  snprintf(msg, sizeof(msg), "\n=== crashtrace: signal %d (%s) addr %p tid %ld pid %d ===\n", sig,
           strsignal(sig), si ? si->si_addr : NULL, (long)syscall(SYS_gettid), (int)getpid());
  both(msg);
  void* pcs[64];
  int n = backtrace(pcs, 64);
  backtrace_symbols_fd(pcs, n, 2);
  if (out_fd >= 0) backtrace_symbols_fd(pcs, n, out_fd);
  for (int i = 0; i < n; ++i) {
    snprintf(msg, sizeof(msg), "  #%d %p\n", i, pcs[i]);
    both(msg);
    frame_maps(pcs[i]);
  }
  both("=== crashtrace end ===\n");
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void crashtrace_init(void) {
  const char* out = getenv("FISDF_CRASH_OUT");
  if (out && *out) out_fd = open(out, O_WRONLY | O_CREAT | O_APPEND, 0644);
  stack_t ss;
  ss.ss_sp = alt_stack;
  ss.ss_size = sizeof(alt_stack);
  ss.ss_flags = 0;
  sigaltstack(&ss, NULL);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, NULL);
  sigaction(SIGABRT, &sa, NULL);
  sigaction(SIGBUS, &sa, NULL);
  // backtrace() loads libgcc_s on first use: do it now, not inside the handler
  void* warm[2];
  backtrace(warm, 2);
}
