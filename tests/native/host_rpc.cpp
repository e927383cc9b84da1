// Host-sanitizer driver (SURVEY §5 "compile a debug build with -fsanitize=address
// for host code"): the host-only entry points of libpomcp_hip.so
// (posggym-baselines_amd/csrc/host_api.cpp, compiled together with this file
// under -fsanitize=address,undefined) served over stdin / stdout, so the Python
// tests that check them against the oracle (tests/test_env_model.py,
// tests/test_host_exp.py) run them under the sanitizers unchanged
// (tests/sanitized_host.py is the client).  An executable rather than a
// sanitized shared library: an ASan library loaded into an uninstrumented
// python needs its runtime preloaded; this program links it itself.  Any
// sanitizer report aborts the program (-fno-sanitize-recover=all), which the
// client sees as a closed pipe.
//
// Protocol, one request per line: "<fn> <args...>\n" [+ binary payload];
// reply "<rc> <values...>\n" [+ binary payload].  Grids are set once ("G" /
// "P" + hex of the pomcp_grid / pomcp_pe_grid bytes) and used by later calls.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "pomcp.h"
#include "pomcp_debug.h"

static pomcp_grid g_drv;
static pomcp_pe_grid g_pe;

static bool unhex(const char* h, void* out, size_t n) {
  if (strlen(h) != 2 * n) return false;
  unsigned char* o = static_cast<unsigned char*>(out);
  for (size_t i = 0; i < n; ++i) {
    unsigned v = 0;
    if (sscanf(h + 2 * i, "%2x", &v) != 1) return false;
    o[i] = (unsigned char)v;
  }
  return true;
}

static uint64_t bits(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}

static bool read_exact(void* p, size_t n) { return fread(p, 1, n, stdin) == n; }
static void write_exact(const void* p, size_t n) { fwrite(p, 1, n, stdout); }

int main() {
  std::vector<char> line(1 << 16);
  while (fgets(line.data(), (int)line.size(), stdin)) {
    char fn[16] = {0};
    if (sscanf(line.data(), "%15s", fn) != 1) continue;
    const char* a = line.data() + strlen(fn);
    if (!strcmp(fn, "G") || !strcmp(fn, "P")) {
      char* h = const_cast<char*>(a);
      while (*h == ' ') ++h;
      h[strcspn(h, "\r\n")] = 0;
      const bool ok = !strcmp(fn, "G") ? unhex(h, &g_drv, sizeof g_drv) : unhex(h, &g_pe, sizeof g_pe);
      printf("%d\n", ok ? 0 : -1);
    } else if (!strcmp(fn, "dsi") || !strcmp(fn, "pesi")) {
      unsigned long long seed;
      uint32_t tree, ctr, st[2] = {0, 0};
      sscanf(a, "%llu %u %u", &seed, &tree, &ctr);
      const int rc = fn[0] == 'd' ? pomcp_driving_sample_initial_state(&g_drv, seed, tree, &ctr, st)
                                  : pomcp_pe_sample_initial_state(&g_pe, seed, tree, &ctr, st);
      printf("%d %u %u %u\n", rc, ctr, st[0], st[1]);
    } else if (!strcmp(fn, "dstep") || !strcmp(fn, "pestep")) {
      unsigned long long seed = 0;
      uint32_t tree = 0, ctr = 0, st[2], nx[2] = {0, 0};
      int32_t act[2], term[2] = {0, 0};
      double rew[2] = {0, 0};
      uint64_t keys[2] = {0, 0};
      int rc;
      if (fn[0] == 'd') {
        sscanf(a, "%llu %u %u %u %u %d %d", &seed, &tree, &ctr, &st[0], &st[1], &act[0], &act[1]);
        rc = pomcp_driving_step(&g_drv, seed, tree, &ctr, st, act, nx, rew, term, keys);
      } else {
        sscanf(a, "%u %u %d %d", &st[0], &st[1], &act[0], &act[1]);
        rc = pomcp_pe_step(&g_pe, st, act, nx, rew, term, keys);
      }
      printf("%d %u %u %u %llu %llu %d %d %llu %llu\n", rc, ctr, nx[0], nx[1],
             (unsigned long long)bits(rew[0]), (unsigned long long)bits(rew[1]), term[0], term[1],
             (unsigned long long)keys[0], (unsigned long long)keys[1]);
    } else if (!strcmp(fn, "dobs") || !strcmp(fn, "peobs")) {
      uint32_t st[2];
      uint64_t keys[2] = {0, 0};
      sscanf(a, "%u %u", &st[0], &st[1]);
      const int rc = fn[0] == 'd' ? pomcp_driving_obs(&g_drv, st, keys) : pomcp_pe_obs(&g_pe, st, keys);
      printf("%d %llu %llu\n", rc, (unsigned long long)keys[0], (unsigned long long)keys[1]);
    } else if (!strcmp(fn, "philox")) {
      unsigned long long seed;
      uint32_t tree, stream, first;
      int32_t n;
      sscanf(a, "%llu %u %u %u %d", &seed, &tree, &stream, &first, &n);
      std::vector<uint32_t> out((size_t)(n > 0 ? n : 0));
      const int rc = pomcp_philox_words(seed, tree, stream, first, n, n > 0 ? out.data() : nullptr);
      printf("%d %d\n", rc, n);
      fflush(stdout);
      write_exact(out.data(), out.size() * 4);
    } else if (!strcmp(fn, "logtab")) {
      long long first, n;
      sscanf(a, "%lld %lld", &first, &n);
      std::vector<double> out((size_t)(n > 0 ? n : 0));
      const int rc = pomcp_host_log_table(first, n, n > 0 ? out.data() : nullptr);
      printf("%d %lld\n", rc, n);
      fflush(stdout);
      write_exact(out.data(), out.size() * 8);
    } else if (!strcmp(fn, "hexp")) {
      int32_t n;
      sscanf(a, "%d", &n);
      std::vector<double> x((size_t)n), out((size_t)n);
      if (!read_exact(x.data(), x.size() * 8)) return 3;
      const int rc = pomcp_debug_host_exp(x.data(), n, out.data());
      printf("%d %d\n", rc, n);
      fflush(stdout);
      write_exact(out.data(), out.size() * 8);
    } else if (!strcmp(fn, "quit")) {
      break;
    } else {
      printf("-99\n");
    }
    fflush(stdout);
  }
  return 0;
}
