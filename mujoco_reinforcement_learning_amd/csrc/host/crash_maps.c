/* Diagnostics only (no reference counterpart): with PPO_SEGV_MAPS=1 in the environment, a fatal
 * SIGSEGV / SIGBUS in the process first writes the faulting address and /proc/self/maps to
 * stderr, then hands the signal to the handler that was installed before (rocprofv3's stack
 * printer, or the default action).  The maps turn the "(unknown)" frames of a profiler crash
 * into library + offset (tools/symbolize_crash.py).  Async-signal-safe: open / read / write only.
 * Built into libppo_hostenv.so, which the engine loads first (host_pool / _lib). */
#define _GNU_SOURCE
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_old_segv, g_old_bus;

static void put(const char *s) {
  ssize_t n = (ssize_t)strlen(s);
  while (n > 0) {
    const ssize_t w = write(2, s, (size_t)n);
    if (w <= 0) return;
    s += w;
    n -= w;
  }
}

static void put_hex(uintptr_t v) {
  char buf[2 + 16 + 1];
  buf[0] = '0';
  buf[1] = 'x';
  for (int i = 0; i < 16; ++i) buf[2 + i] = "0123456789abcdef"[(v >> (4 * (15 - i))) & 15];
  buf[18] = 0;
  put(buf);
}

static void on_fault(int sig, siginfo_t *si, void *uc) {
  put("\nppo crash_maps: signal ");
  put(sig == SIGSEGV ? "SIGSEGV" : "SIGBUS");
  put(" at address ");
  put_hex((uintptr_t)si->si_addr);
  put("\n--- /proc/self/maps ---\n");
  const int fd = open("/proc/self/maps", O_RDONLY);
  if (fd >= 0) {
    char buf[4096];
    ssize_t n;
    while ((n = read(fd, buf, sizeof(buf))) > 0) {
      ssize_t off = 0;
      while (off < n) {
        const ssize_t w = write(2, buf + off, (size_t)(n - off));
        if (w <= 0) break;
        off += w;
      }
    }
    close(fd);
  }
  put("--- end maps ---\n");
  struct sigaction *old = sig == SIGSEGV ? &g_old_segv : &g_old_bus;
  if ((old->sa_flags & SA_SIGINFO) && old->sa_sigaction) {
    old->sa_sigaction(sig, si, uc);
    return;
  }
  if (old->sa_handler != SIG_DFL && old->sa_handler != SIG_IGN && old->sa_handler) {
    old->sa_handler(sig);
    return;
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void ppo_crash_maps_init(void) {
  const char *v = getenv("PPO_SEGV_MAPS");
  if (!v || strcmp(v, "1") != 0) return;
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_old_segv);
  sigaction(SIGBUS, &sa, &g_old_bus);
}

/* ppo_crash_maps_installed: 1 when the handler is active (tests / tools). */
int ppo_crash_maps_installed(void) {
  struct sigaction cur;
  if (sigaction(SIGSEGV, NULL, &cur) != 0) return 0;
  return (cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == on_fault;
}
