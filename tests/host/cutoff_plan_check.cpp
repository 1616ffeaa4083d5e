// Host check of the cutoff kernel's chunk plan (gpmdm_amd/csrc/common.h: cutoff_chunk_begin,
// cutoff_chunk_positions, cutoff_split_chunk -- the functions obs_cutoff.h and k_obs_ll
// evaluate on the device), against a direct restatement: chunks tile the list exactly, only
// the first is partial, positions follow the last R tile's diagonal, and the split point
// minimises the larger of the two workgroups' positions.  Built by hipcc, run on the CPU (no
// HIP call is made).
#include <cstdio>
#include <cstdlib>

#include "common.h"

using namespace gpmdm;

static int fails = 0;
#define EXPECT(c, ...)                   \
  do {                                   \
    if (!(c)) {                          \
      if (fails < 20) {                  \
        std::printf(__VA_ARGS__);        \
        std::printf("\n");               \
      }                                  \
      ++fails;                           \
    }                                    \
  } while (0)

int main() {
  const int tpcs[] = {32, 16, 8};
  const int tms[] = {1, 2, 4, 8, 17};
  long long cases = 0;
  for (int tpc : tpcs)
    for (int T_M : tms)
      for (int n_act = 0; n_act <= 700; ++n_act) {
        const int nt = n_act + T_M;
        const int nc = (nt + tpc - 1) / tpc;
        EXPECT(cutoff_chunk_begin(0, nt, tpc) == 0, "begin(0)");
        EXPECT(cutoff_chunk_begin(nc, nt, tpc) == nt, "begin(nc) nt=%d", nt);
        long long tot = 0;
        for (int c = 0; c < nc; ++c) {
          const int b = cutoff_chunk_begin(c, nt, tpc), e = cutoff_chunk_begin(c + 1, nt, tpc);
          EXPECT(e > b && e - b <= tpc, "chunk %d size %d (nt %d)", c, e - b, nt);
          EXPECT(c == 0 || e - b == tpc, "chunk %d not full (nt %d)", c, nt);
          const int last = e - 1;
          const int pos = last < n_act ? last + 1 : n_act;   // R tiles: to the last diagonal
          EXPECT(cutoff_chunk_positions(c, n_act, T_M, tpc) == pos, "positions c=%d nt=%d", c, nt);
          tot += pos + 4;
        }
        const int cs = cutoff_split_chunk(n_act, T_M, tpc);
        if (nc < 2) {
          EXPECT(cs == nc, "no split below two chunks");
        } else {
          EXPECT(cs >= 1 && cs < nc, "split in range: %d of %d", cs, nc);
          long long best = -1, pre = 0;
          for (int c = 1; c < nc; ++c) {
            pre += cutoff_chunk_positions(c - 1, n_act, T_M, tpc) + 4;
            const long long v = pre > tot - pre ? pre : tot - pre;
            if (best < 0 || v < best) best = v;
          }
          long long at = 0;
          for (int c = 0; c < cs; ++c) at += cutoff_chunk_positions(c, n_act, T_M, tpc) + 4;
          const long long v = at > tot - at ? at : tot - at;
          EXPECT(v == best, "split not minimal: n_act %d T_M %d", n_act, T_M);
        }
        ++cases;
      }
  std::printf("%lld cases, %d failures\n", cases, fails);
  if (fails) return 1;
  std::printf("ok\n");
  return 0;
}
