/* tests/c/boot_fuzz.c -- the bootstrap star and the node-local shared-memory
 * barrier (csrc/pg_boot.c) under AddressSanitizer + UndefinedBehaviorSanitizer:
 * W forked processes join through rank 0, all-gather one int each, meet at
 * the TCP barrier and at 1000 shared-memory barriers (pgx_boot_selftest).
 * Built and run by tests/test_plan_sanitize.py.  usage: boot_fuzz W port */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "pg_impl.h"

/* pg.c is not linked (it needs the GPU runtime): its two helpers used here */
static char g_err[512];
void pg_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char *pg_last_error(void) { return g_err; }

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  int W = atoi(argv[1]), port = atoi(argv[2]);
  char list[4096] = "";
  for (int i = 0; i < W; ++i) strcat(list, "127.0.0.1 ");
  for (int r = 0; r < W; ++r) {
    if (fork() == 0) {
      int *out = calloc((size_t)W, sizeof(int));
      int rc = pgx_boot_selftest(list, r, port, 100 + r, out);
      for (int q = 0; rc == 0 && q < W; ++q)
        if (out[q] != 100 + q) rc = -2;
      if (rc) fprintf(stderr, "rank %d: rc %d: %s\n", r, rc, g_err);
      free(out);
      _exit(rc ? 1 : 0);
    }
  }
  int bad = 0, st;
  for (int r = 0; r < W; ++r) {
    if (wait(&st) < 0 || !WIFEXITED(st) || WEXITSTATUS(st)) bad = 1;
  }
  printf(bad ? "FAIL\n" : "ok\n");
  return bad;
}
