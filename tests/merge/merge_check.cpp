// CPU check of ke::merge_exact (koordinator_amd/csrc/ke_merge.h) against the permutation walk ke::merge_walk on
// random provider lists: upward-closed families like generateResourceHints / DeviceShare's hints produce
// (cpu, memory, DeviceShare copies with NUMA ids outside the zones, unsatisfied nil lists), and arbitrary
// mask sets.  Test infrastructure (tests/test_merge.py builds and runs it); prints one line per failure.
//   usage: merge_check SEED TRIALS
#include <cstdio>
#include <cstdlib>
#include <random>

#define KE_HD
#include "../../koordinator_amd/csrc/ke_merge.h"

static const uint8_t* numa_order() {  // IterateBitMasks order: by size, then combinations in index order
  static uint8_t o[255];
  static bool done = false;
  if (!done) {
    int n = 0;
    for (int k = 1; k <= 8; k++)
      for (int m = 1; m < 256; m++)  // combinations of k bits in lexicographic order of their indices
        if (__builtin_popcount(m) == k) o[n++] = (uint8_t)m;
    // lexicographic order of index tuples: sort each size class by its reversed-bit order
    for (int a = 0, b; a < 255; a = b) {
      for (b = a; b < 255 && __builtin_popcount(o[b]) == __builtin_popcount(o[a]); b++) {}
      auto key = [](uint8_t m) {
        uint32_t r = 0;
        for (int i = 0; i < 8; i++)
          if ((m >> i) & 1) r = r * 8 + (uint32_t)i;
        return r;
      };
      for (int i = a + 1; i < b; i++)
        for (int j = i; j > a && key(o[j]) < key(o[j - 1]); j--) {
          const uint8_t t = o[j];
          o[j] = o[j - 1];
          o[j - 1] = t;
        }
    }
    done = true;
  }
  return o;
}

int main(int argc, char** argv) {
  const unsigned seed = argc > 1 ? (unsigned)atoi(argv[1]) : 1;
  const int trials = argc > 2 ? atoi(argv[2]) : 1000;
  std::mt19937 rng(seed);
  auto U = [&](int n) { return (int)(rng() % (unsigned)n); };
  const uint8_t* ord = numa_order();
  int fails = 0, exact_runs = 0;
  for (int t = 0; t < trials; t++) {
    ke::MergeLists L;
    L.n = 0;
    const int nz = 2 + U(5);  // zones 0..nz-1 (up to 6: keeps the walk fast)
    uint32_t all = (1u << nz) - 1;
    if (U(4) == 0) all &= ~(1u << U(nz));  // a zone missing
    if (!all) all = 1;
    int32_t hs[256];
    for (int m = 0; m < 256; m++) hs[m] = U(3) == 0 ? 0 : U(4) * 25;
    uint64_t S[4] = {rng(), rng(), rng(), rng()};
    const bool generic = U(5) == 0;
    auto family = [&](uint32_t universe, int minsz, double p_keep) {  // upward closed within `universe`
      uint8_t seeds[8];
      int ns = 0;
      for (int r = 0; r < 1 + U(3); r++) {
        uint32_t s = 0;
        for (int z = 0; z < 8; z++)
          if (((universe >> z) & 1) && U(3) == 0) s |= 1u << z;
        if (!s) s = universe & (~universe + 1);
        if (__builtin_popcount(s) < minsz) s = universe;
        seeds[ns++] = (uint8_t)s;
      }
      int n = 0;
      for (int e = 0; e < 255; e++) {
        const uint32_t m = ord[e];
        if (m & ~universe) continue;
        bool up = false;
        for (int q = 0; q < ns; q++) up = up || (m & seeds[q]) == seeds[q];
        if (generic) up = U(1000) < (int)(p_keep * 1000);
        if (up) L.m[L.n][n++] = (uint8_t)m;
      }
      return n;
    };
    auto add = [&](uint32_t universe, bool ds) {
      L.ds[L.n] = ds;
      L.unsat[L.n] = 0;
      L.len[L.n] = family(universe, 1, 0.5);
      if (L.len[L.n] == 0) L.m[L.n][0] = (uint8_t)universe, L.len[L.n] = 1;
      L.n++;
    };
    const int kind = U(4);
    if (kind == 0) {  // a nil unsatisfied list (a resource without hints) + others
      L.m[L.n][0] = 0, L.len[L.n] = 1, L.ds[L.n] = 0, L.unsat[L.n] = 1, L.n++;
    }
    const int nres = 1 + U(2);
    for (int r = 0; r < nres && L.n < ke::MERGE_LISTS; r++) {
      uint32_t lack = U(3) == 0 ? (1u << U(nz)) : 0;
      add(all & ~lack ? all & ~lack : all, false);
    }
    // DeviceShare: identical copies of one family over NUMA ids that may lie outside the zones
    const int copies = U(3);
    if (copies && L.n < ke::MERGE_LISTS) {
      uint32_t uni = all | (U(3) == 0 ? (1u << (nz + U(8 - nz))) & 0xFF : 0);
      const int base = L.n;
      add(uni, true);
      for (int c = 1; c < copies && L.n < ke::MERGE_LISTS; c++) {
        for (int i = 0; i < L.len[base]; i++) L.m[L.n][i] = L.m[base][i];
        L.len[L.n] = L.len[base], L.ds[L.n] = 1, L.unsat[L.n] = 0, L.n++;
      }
    }
    int64_t total = 1;
    for (int l = 0; l < L.n; l++) total *= L.len[l];
    if (total > 3000000) continue;
    auto sc = [&](int l, uint32_t m) -> int32_t { return L.ds[l] ? ((S[m >> 6] >> (m & 63)) & 1 ? 500 : 0) : hs[m]; };
    const uint32_t w = ke::merge_walk(L, all, total, sc);
    const uint32_t x = ke::merge_exact(L, all, sc);
    exact_runs++;
    if (w != x) {
      fails++;
      printf("FAIL trial %d: walk %u exact %u all %u lists %d total %lld\n", t, w, x, all, L.n, (long long)total);
    }
  }
  printf("checked %d fails %d\n", exact_runs, fails);
  return fails ? 1 : 0;
}
