// mergeFilteredHints over every permutation of the provider hint lists (topologymanager/policy.go:198-299)
// for a BestEffort merge without a preferred merged hint.  Host + device code: the kernels
// include it, and tests/merge/merge_check.cpp compiles it with g++ to check the exact fold against the
// permutation-by-permutation one.
//
// The reference folds the permutations in lexicographic order (first list outermost):
//   mg = all & AND of the non-nil masks, skipped when 0; S = sum of the scores of the hints whose mask == mg;
//   u (unsatisfied) = some list is the unsatisfied nil entry, or some non-nil mask != mg;
//   best <- (mg, S, u) when mg is narrower than best, or the same size with S > best's score
// and BestEffort returns `all` when the final hint is unsatisfied.  Beyond MERGE_BUDGET permutations the
// walk is replaced by merge_exact, which computes the same result without enumerating:
//   1. Only hints of the minimal non-zero size c (over every permutation) matter: the first one replaces any
//      wider state and a wider one never replaces a c-sized one.
//   2. The fold's final key (mask, score) equals the fold over the distinct keys taken in the order of their
//      LAST occurrence (a key's earlier occurrences never decide the outcome).
//   3. Its u is the u of the key's first occurrence after Q, the last occurrence of any key that beats it.
// Last / first occurrences are lexicographically extreme permutations producing a key; for a target mask M
// they follow from a greedy over the lists with a feasibility test: which lists pick M itself (their scores
// sum to the key's score; every other list needs a strict superset of M), or, when none does, whether the
// strict supersets can still AND down to M (a backward bitset table over the masks between M and `all`).
#pragma once
#include <stdint.h>

#ifndef KE_HD
#define KE_HD __host__ __device__
#endif

namespace ke {

constexpr int MERGE_LISTS = 5;
constexpr int64_t MERGE_BUDGET = 1 << 20;  // permutations walked one by one; more: merge_exact

// lists[l][0..len[l]) hold masks in IterateBitMasks order; a nil list is one entry 0 (`unsat`: the
// unsatisfied entry of a resource without hints); `ds`: a DeviceShare list (the score function knows)
struct MergeLists {
  uint8_t m[MERGE_LISTS][255];
  uint8_t ds[MERGE_LISTS];
  uint8_t unsat[MERGE_LISTS];
  int len[MERGE_LISTS];
  int n;
};

KE_HD inline bool merge_narrower(uint32_t a, uint32_t b) {  // bitmask.IsNarrowerThan
  const int ca = __builtin_popcount(a), cb = __builtin_popcount(b);
  return ca == cb ? a < b : ca < cb;
}
// the fold's replacement rule for non-preferred hints
KE_HD inline bool merge_beats(uint32_t m, int32_t s, uint32_t bm, int32_t bs) {
  return merge_narrower(m, bm) || (__builtin_popcount(m) == __builtin_popcount(bm) && s > bs);
}
KE_HD inline bool mbit(const uint64_t* b, uint32_t x) { return (b[x >> 6] >> (x & 63u)) & 1u; }
KE_HD inline void mset(uint64_t* b, uint32_t x) { b[x >> 6] |= 1ull << (x & 63u); }

// The permutation walk.  sc(l, mask): the hint score of `mask` in list l.  Returns the merged affinity
// (`all` when the best hint is unsatisfied).
template <class ScoreFn>
KE_HD uint32_t merge_walk(const MergeLists& L, uint32_t all, int64_t total, ScoreFn sc) {
  uint32_t best = all;
  int32_t bsc = 0;
  bool bun = false;
  int idx[MERGE_LISTS] = {0, 0, 0, 0, 0};
  for (int64_t it = 0; it < total; it++) {
    uint32_t mg = all;
    int maxn = 0;
    bool have = false, un = false;
    for (int l = 0; l < L.n; l++) {
      const uint32_t m = L.m[l][idx[l]];
      un = un || L.unsat[l];
      if (m) {
        have = true;
        mg &= m;
        maxn = maxn > __builtin_popcount(m) ? maxn : __builtin_popcount(m);
      }
    }
    un = un || (have && maxn != __builtin_popcount(mg));
    if (mg) {
      int32_t s = 0;
      for (int l = 0; l < L.n; l++) {
        const uint32_t m = L.m[l][idx[l]];
        if (m && m == mg) s += sc(l, m);
      }
      if (merge_beats(mg, s, best, bsc)) {
        best = mg;
        bsc = s;
        bun = un;
      }
    }
    for (int l = L.n - 1; l >= 0; l--) {  // next permutation (last list fastest)
      if (++idx[l] < L.len[l]) break;
      idx[l] = 0;
    }
  }
  return bun ? all : best;
}

// ---- merge_exact ---------------------------------------------------------------------------------------
// One target mask M: per (non-nil) list the position of M itself, its score there, whether a strict
// superset of M exists, and G[j] = the prefix ANDs a (M <= a <= all) from which lists j.. choosing strict
// supersets only reach exactly M.
struct MergeTarget {
  uint32_t M;
  int16_t e[MERGE_LISTS];
  int32_t sc[MERGE_LISTS];
  bool sup[MERGE_LISTS];
  uint64_t G[MERGE_LISTS + 1][4];
};

struct MergeCtx {
  const MergeLists* L;
  int lid[MERGE_LISTS];  // the non-nil lists
  int n;
  uint32_t all;
};

KE_HD inline const uint8_t* mlist(const MergeCtx& C, int j) { return C.L->m[C.lid[j]]; }
KE_HD inline int mlen(const MergeCtx& C, int j) { return C.L->len[C.lid[j]]; }

template <class ScoreFn>
KE_HD void merge_target(const MergeCtx& C, uint32_t M, ScoreFn sc, MergeTarget& T) {
  T.M = M;
  for (int j = 0; j < C.n; j++) {
    T.e[j] = -1;
    T.sup[j] = false;
    const uint8_t* m = mlist(C, j);
    for (int i = 0; i < mlen(C, j); i++) {
      if (m[i] == M) T.e[j] = (int16_t)i;
      else if ((m[i] & M) == M) T.sup[j] = true;
    }
    T.sc[j] = T.e[j] >= 0 ? sc(C.lid[j], M) : 0;
  }
  for (int q = 0; q < 4; q++) T.G[C.n][q] = 0;
  mset(T.G[C.n], M);
  const uint32_t free = C.all & ~M;
  for (int j = C.n - 1; j >= 0; j--) {
    for (int q = 0; q < 4; q++) T.G[j][q] = 0;
    const uint8_t* m = mlist(C, j);
    for (uint32_t sub = free;; sub = (sub - 1) & free) {  // every a with M <= a <= all
      const uint32_t a = M | sub;
      for (int i = 0; i < mlen(C, j); i++)
        if (m[i] != M && (m[i] & M) == M && mbit(T.G[j + 1], a & m[i])) {
          mset(T.G[j], a);
          break;
        }
      if (!sub) break;
    }
  }
}

// lists j.. can complete a prefix (AND a, score acc, some list took M: any) to the key (M, S)
KE_HD inline bool merge_feasible(const MergeCtx& C, const MergeTarget& T, int j, uint32_t a, int32_t acc, bool any,
                                 int32_t S) {
  int ex = 0;
  for (int l = j; l < C.n; l++)
    if (T.e[l] >= 0) ex |= 1 << l;
  for (int E = ex;; E = (E - 1) & ex) {  // the lists after j that take M itself
    int32_t s = acc;
    bool ok = true;
    for (int l = j; l < C.n; l++) {
      if ((E >> l) & 1) s += T.sc[l];
      else ok = ok && T.sup[l];
    }
    if (s == S) {
      if (any || E) {
        if (ok) return true;
      } else if (mbit(T.G[j], a)) {
        return true;
      }
    }
    if (!E) break;
  }
  return false;
}

// Lexicographically last (MAX) or first permutation producing the key (M, S) whose position is above
// `after` (levels 0..n-1, 8 bits each, level 0 highest; after < 0: no bound).  Returns the packed
// permutation or -1; *u = its unsatisfied flag (some non-nil mask differs from M).
template <bool MAX>
KE_HD int64_t merge_extreme(const MergeCtx& C, const MergeTarget& T, int32_t S, int64_t after, bool* u) {
  const uint32_t M = T.M;
  int t[MERGE_LISTS] = {0, 0, 0, 0, 0};
  // the deepest level d at which the permutation leaves `after`'s prefix (MAX: d = -1, no prefix)
  int d0 = -1, dmin = -1;
  if (!MAX && after >= 0) d0 = C.n - 1, dmin = 0;
  for (int d = d0; d >= dmin; d--) {
    // the prefix of `after` before level d
    uint32_t a = C.all;
    int32_t acc = 0;
    bool any = false, ok = true;
    for (int j = 0; j < d && ok; j++) {
      const int i = (int)((after >> (8 * (C.n - 1 - j))) & 0xFF);
      const uint32_t m = mlist(C, j)[i];
      t[j] = i;
      if ((m & M) != M) ok = false;
      else if (m == M) acc += T.sc[j], any = true, a = M;
      else a &= m;
    }
    if (!ok) continue;
    if (d < 0 && !merge_feasible(C, T, 0, a, acc, any, S)) return -1;
    bool found = true;
    for (int j = d < 0 ? 0 : d; j < C.n && found; j++) {
      const uint8_t* m = mlist(C, j);
      const int len = mlen(C, j);
      // a strict superset at level j is feasible iff (some list took / will take M) or (none does and the
      // supersets still reach M); the first test does not depend on the mask
      bool fe_any = false;
      {
        int ex = 0;
        for (int l = j + 1; l < C.n; l++)
          if (T.e[l] >= 0) ex |= 1 << l;
        for (int E = ex;; E = (E - 1) & ex) {
          int32_t s = acc;
          bool sup_ok = true;
          for (int l = j + 1; l < C.n; l++) {
            if ((E >> l) & 1) s += T.sc[l];
            else sup_ok = sup_ok && T.sup[l];
          }
          if (s == S && (any || E) && sup_ok) fe_any = true;
          if (!E || fe_any) break;
        }
      }
      const bool fe_g = !any && acc == S;
      const bool ex_ok = T.e[j] >= 0 && merge_feasible(C, T, j + 1, M, acc + T.sc[j], true, S);
      const int lo = (j == d) ? (int)((after >> (8 * (C.n - 1 - j))) & 0xFF) + 1 : 0;
      int pick = -1;
      for (int s = 0; s < len - (MAX ? 0 : lo); s++) {
        const int i = MAX ? len - 1 - s : lo + s;
        const uint32_t mi = m[i];
        if ((mi & M) != M) continue;
        const bool f = (mi == M) ? ex_ok : (fe_any || (fe_g && mbit(T.G[j + 1], a & mi)));
        if (f) {
          pick = i;
          break;
        }
      }
      if (pick < 0) {
        found = false;
        break;
      }
      t[j] = pick;
      if (m[pick] == M) acc += T.sc[j], any = true, a = M;
      else a &= m[pick];
    }
    if (!found) continue;
    int64_t key = 0;
    bool un = false;
    for (int j = 0; j < C.n; j++) {
      key = (key << 8) | t[j];
      un = un || mlist(C, j)[t[j]] != M;
    }
    if (u) *u = un;
    return key;
  }
  return -1;
}

// the scores of M's keys: one per set of lists taking M itself (valid with the others' strict supersets,
// or, for the empty set, when the supersets alone reach M); returns the number of distinct scores
KE_HD inline int merge_scores(const MergeCtx& C, const MergeTarget& T, int32_t* out) {
  int ex = 0, k = 0;
  for (int l = 0; l < C.n; l++)
    if (T.e[l] >= 0) ex |= 1 << l;
  for (int E = ex;; E = (E - 1) & ex) {
    int32_t s = 0;
    bool ok = true;
    for (int l = 0; l < C.n; l++) {
      if ((E >> l) & 1) s += T.sc[l];
      else ok = ok && T.sup[l];
    }
    const bool valid = E ? ok : mbit(T.G[0], C.all);
    bool dup = false;
    for (int q = 0; q < k; q++) dup = dup || out[q] == s;
    if (valid && !dup) out[k++] = s;
    if (!E) break;
  }
  return k;
}

// the key of target T with the smallest last occurrence above `after` (-1: none); *S = its score
KE_HD inline int64_t merge_next_key(const MergeCtx& C, const MergeTarget& T, int64_t after, int32_t* S) {
  int32_t sv[1 << MERGE_LISTS];
  const int k = merge_scores(C, T, sv);
  int64_t best = -1;
  for (int q = 0; q < k; q++) {
    const int64_t t = merge_extreme<true>(C, T, sv[q], -1, nullptr);
    if (t > after && (best < 0 || t < best)) best = t, *S = sv[q];
  }
  return best;
}

template <class ScoreFn>
KE_HD uint32_t merge_exact(const MergeLists& L, uint32_t all, ScoreFn sc) {
  MergeCtx C;
  C.L = &L;
  C.all = all;
  C.n = 0;
  for (int l = 0; l < L.n; l++)
    if (!(L.len[l] == 1 && L.m[l][0] == 0)) C.lid[C.n++] = l;
  bool unsat = false;
  for (int l = 0; l < L.n; l++) unsat = unsat || L.unsat[l];
  if (C.n == 0) return all;  // every permutation merges to `all` with score 0: the initial best stays
  // 1. the non-zero ANDs every permutation can reach, and their minimal size c
  uint64_t R[4] = {0, 0, 0, 0};
  mset(R, all);
  for (int j = 0; j < C.n; j++) {
    uint64_t R2[4] = {0, 0, 0, 0};
    for (uint32_t a = 0; a < 256; a++)
      if (mbit(R, a))
        for (int i = 0; i < mlen(C, j); i++) mset(R2, a & mlist(C, j)[i]);
    for (int q = 0; q < 4; q++) R[q] = R2[q];
  }
  int c = 9;
  for (uint32_t a = 1; a < 256; a++)
    if (mbit(R, a) && __builtin_popcount(a) < c) c = __builtin_popcount(a);
  if (c == 9) return all;  // no permutation merges to a non-empty affinity
  // 2. fold the c-sized keys in the order of their last occurrence: a K-way merge over the target masks,
  //    each target keeping its next key (smallest last occurrence not yet folded)
  uint8_t tm[70];
  int64_t nt[70];
  int32_t ns[70];
  int nT = 0;
  MergeTarget T;
  for (uint32_t M = 1; M < 256; M++) {
    if (__builtin_popcount(M) != c || !mbit(R, M)) continue;
    merge_target(C, M, sc, T);
    tm[nT] = (uint8_t)M;
    nt[nT] = merge_next_key(C, T, -1, &ns[nT]);
    nT++;
  }
  uint32_t bm = all;
  int32_t bs = 0;
  for (;;) {
    int q = -1;
    for (int r = 0; r < nT; r++)
      if (nt[r] >= 0 && (q < 0 || nt[r] < nt[q])) q = r;
    if (q < 0) break;
    if (merge_beats(tm[q], ns[q], bm, bs)) bm = tm[q], bs = ns[q];
    merge_target(C, tm[q], sc, T);
    nt[q] = merge_next_key(C, T, nt[q], &ns[q]);
  }
  if (bm == all) return all;  // the initial hint, or a hint on `all` itself: the result is `all` either way
  // 3. Q = the last occurrence of any key that beats the final one; the final hint is its first occurrence
  //    after Q
  int64_t Q = -1;
  for (int r = 0; r < nT; r++) {
    merge_target(C, tm[r], sc, T);
    int32_t sv[1 << MERGE_LISTS];
    const int k = merge_scores(C, T, sv);
    for (int z = 0; z < k; z++)
      if (merge_beats(tm[r], sv[z], bm, bs)) {
        const int64_t t = merge_extreme<true>(C, T, sv[z], -1, nullptr);
        if (t > Q) Q = t;
      }
  }
  merge_target(C, bm, sc, T);
  bool u = false;
  const int64_t first = merge_extreme<false>(C, T, bs, Q, &u);
  (void)first;  // exists: the key's last occurrence is after Q (it entered the fold after every beating key)
  return (u || unsat) ? all : bm;
}

}  // namespace ke
