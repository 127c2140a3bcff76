// dw_compat2 (the 2-pair fast path) against dw_compatible (csrc/dewey.h) on every pair of
// canonical versions of <= 2 RLE pairs over small digits; prints the mismatches (none expected)
// and the number of pairs checked.  Built and run by tests/test_lane_cpu.py.
#include <cstdio>
#include <vector>

#include "hip/hip_runtime.h"
#include "dewey.h"

using namespace cep;

int main() {
  std::vector<Dewey> vs;
  for (int n = 1; n <= 2; n++)
    for (int v0 = 0; v0 < 4; v0++)
      for (int c0 = 1; c0 <= 3; c0++)
        for (int v1 = 0; v1 < 4; v1++)
          for (int c1 = 1; c1 <= 3; c1++) {
            if (n == 1 && (v1 || c1 > 1)) continue;
            if (n == 2 && v1 == v0) continue;  // canonical: adjacent pairs differ
            Dewey d;
            dw_init(d, v0);
            d.n = n;
            d.c[0] = c0;
            d.v[1] = n == 2 ? v1 : 0;
            d.c[1] = n == 2 ? c1 : 0;
            d.len = c0 + (n == 2 ? c1 : 0);
            vs.push_back(d);
          }
  long checked = 0, bad = 0;
  for (const Dewey& a : vs)
    for (const Dewey& b : vs) {
      const bool want = dw_compatible(a, b);
      const bool got = dw_compat2(a.n, a.len, a.v[0], a.c[0], a.v[1], a.c[1], b.n, b.len, b.v[0], b.c[0], b.v[1], b.c[1]);
      checked++;
      if (want != got) {
        bad++;
        if (bad < 10) std::printf("mismatch a n=%u len=%u b n=%u len=%u want %d\n", a.n, a.len, b.n, b.len, want);
      }
    }
  std::printf("checked %ld bad %ld\n", checked, bad);
  return bad != 0;
}
