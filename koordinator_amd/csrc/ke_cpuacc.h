// ke_cpuacc.h — NodeNUMAResource's CPU accumulator on the device (one node, one 64-lane workgroup,
// LDS-resident).
//
// Same algorithm as pkg/scheduler/plugins/nodenumaresource/cpu_accumulator.go (takeCPUs :87-232 and
// the cpuAccumulator helpers :234-822).  Per node the CPU table lives in the CPU SoA as one 8-byte
// record per CPU id (CpuRec); core and socket ids are the node's dense ranks of the reference ids (the
// accumulator only compares them), NUMA ids are kept.  Go feeds every list through map iteration but
// sorts each by a total order with the id last; the two length-only sorts in takeCPUs (:142-144,
// :161-163) run on <= 12 sockets, where Go's sort.Slice is an insertion sort (stable) — the insertion
// sorts here are stable too, and the rank sort of freeCPUs' cores reproduces a sort by a total order.
//
// Every function is called by all 64 lanes of the workgroup with the same arguments (control flow is
// uniform: decisions read LDS after a barrier).  Loops over CPUs / cores without a carried dependency
// run lane-strided (counts through LDS atomics or wave sums); the order-dependent list builders run on
// lane 0 between barriers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ke_types.h"

namespace ke {

constexpr int ACC_CPUS = CPU_SLOTS;
constexpr int ACC_TPC = 8;  // max logical CPUs per core (validated by ke_node_cpus_set)

// topology counts (cpu_topology.go:45-105)
struct AccTopo {
  int num_cpus, num_cores, num_nodes, num_sockets;
};

struct AccLds {
  CpuRec cpu[ACC_CPUS];
  uint8_t alloc[ACC_CPUS];    // allocatableCPUs
  uint8_t aref[ACC_CPUS];     // allocatableCPUs[c].RefCount (max_ref > 1)
  uint8_t ex_core[ACC_CPUS];  // exclusiveInCores (core rank)
  uint8_t ex_node[ACC_CPUS];  // exclusiveInNUMANodes (NUMA id)
  uint8_t res[ACC_CPUS];      // result
  // one grouping (cores / NUMA nodes / sockets): CPUs concatenated in group order
  int16_t lst[ACC_CPUS];
  int16_t goff[ACC_CPUS + 1];
  int16_t gkey[ACC_CPUS];
  int16_t gscore[ACC_CPUS];   // per group: the free score the sort used
  int ng;
  // a second grouping (takeCPUs keeps the unsatisfied sockets)
  int16_t lst2[ACC_CPUS];
  int16_t goff2[ACC_CPUS + 1];
  int ng2;
  // per core rank: its allocatable CPUs (kept by the current pass; in no particular order)
  int32_t core_n[ACC_CPUS];
  uint8_t core_cpu[ACC_CPUS][ACC_TPC];
  int32_t cref[ACC_CPUS];     // getCoreRefCount per core rank over the allocatable CPUs (max_ref > 1)
  // counts of the list builders
  int32_t sc_sock[ACC_CPUS], sc_node[ACC_CPUS], sc_colo[ACC_CPUS];  // free / co-located CPUs per socket / node
  int32_t cnt32[ACC_CPUS];                                          // per group key, then bucket cursors
  int16_t p_off[ACC_CPUS + 1], p_key[ACC_CPUS], p_sc[ACC_CPUS];     // permute_groups, bucket starts
  int16_t sp_out[ACC_CPUS];                                         // spread_cpus
  int16_t ord2[ACC_CPUS];
  uint8_t mark[ACC_CPUS];
  // allocateCPUSet around the accumulator: the CPUs it may take, the exclusivity of the allocated
  // CPUs before the pod, the union of its per-NUMA takes
  uint8_t base[ACC_CPUS], ex_core0[ACC_CPUS], ex_node0[ACC_CPUS], uni[ACC_CPUS];
  int16_t order[ACC_CPUS];
  int16_t tmp[ACC_CPUS];
  AccTopo t;
  int max_ref, needed, excl_policy, exclusive, numa_most;
  // loop bounds of the node's table: CPU ids < n_cpu, core ranks < n_core, socket ranks < n_sock, NUMA
  // ids < n_numa (the byte arrays are zero past them)
  int n_cpu, n_core, n_sock, n_numa;
  int bcast;  // lane 0's result for the wave
  // takePreferredCPUs' preferredCPUs (cpu_accumulator.go:29-85), has_pref = 0: none (takeCPUs alone)
  uint8_t pref[ACC_CPUS];
  int has_pref;
};

__device__ __forceinline__ int acc_lane() { return (int)threadIdx.x; }
__device__ __forceinline__ int acc_nkey(const AccLds& a, bool by_socket) { return by_socket ? a.n_sock : a.n_numa; }
__device__ __forceinline__ int acc_wave_sum(int v) { return __ockl_wfred_add_i32(v); }

__device__ __forceinline__ int acc_cpc(const AccTopo& t) { return t.num_cores ? t.num_cpus / t.num_cores : 0; }
__device__ __forceinline__ int acc_cps(const AccTopo& t) { return t.num_sockets ? t.num_cpus / t.num_sockets : 0; }
__device__ __forceinline__ int acc_cpn(const AccTopo& t) { return t.num_nodes ? t.num_cpus / t.num_nodes : 0; }

__device__ __forceinline__ bool strat_less(const AccLds& a, int si, int sj) { return a.numa_most ? si < sj : si > sj; }

// take the n (distinct) CPUs of cpus[] (:290-304)
__device__ inline void acc_take(AccLds& a, const int16_t* cpus, int n) {
  for (int i = acc_lane(); i < n; i += 64) {
    const int c = cpus[i];
    a.res[c] = 1;
    a.alloc[c] = 0;
    if (a.exclusive) {
      if (a.excl_policy == 1) a.ex_core[a.cpu[c].core] = 1;
      else if (a.excl_policy == 2) a.ex_node[a.cpu[c].numa] = 1;
    }
  }
  __syncthreads();
  if (acc_lane() == 0) a.needed -= n;
  __syncthreads();
}
__device__ __forceinline__ int acc_count_alloc(const AccLds& a) {
  int n = 0;
  for (int c = acc_lane(); c < a.n_cpu; c += 64) n += a.alloc[c];
  return acc_wave_sum(n);
}
__device__ __forceinline__ bool excl_pcpu(const AccLds& a, int c) { return a.excl_policy == 1 && a.ex_core[a.cpu[c].core]; }
__device__ __forceinline__ bool excl_numa(const AccLds& a, int c) { return a.excl_policy == 2 && a.ex_node[a.cpu[c].numa]; }

// getCoreRefCount (:776-783) over the allocatable CPUs: cached per core rank by collect_cores (the
// allocatable set only changes in acc_take, between sorts)
__device__ __forceinline__ int core_ref(const AccLds& a, int core) { return a.cref[core]; }

// lane 0's sequential helpers
__device__ inline void sort_i16(int16_t* v, int n) {
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && v[j] < v[j - 1]; j--) {
      const int16_t t = v[j];
      v[j] = v[j - 1];
      v[j - 1] = t;
    }
}
__device__ inline void sort_by_ref(const AccLds& a, int16_t* v, int n) {  // sortCPUsByRefCount :785-796
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0; j--) {
      const int x = v[j], y = v[j - 1];
      const bool less = a.aref[x] != a.aref[y] ? a.aref[x] < a.aref[y] : x < y;
      if (!less) break;
      v[j] = (int16_t)y;
      v[j - 1] = (int16_t)x;
    }
}
__device__ inline int extract_cpu(AccLds& a, int16_t* v, int n) {  // :332-343
  for (int i = 0; i < n; i++) a.mark[a.cpu[v[i]].core] = 0;
  int m = 0;
  for (int i = 0; i < n; i++) {
    const int core = a.cpu[v[i]].core;
    if (a.mark[core]) continue;
    a.mark[core] = 1;
    v[m++] = v[i];
  }
  return m;
}

// cores of the allocatable CPUs passing `keep` (per core rank; a core's CPUs sorted by its users)
template <typename Keep>
__device__ inline void collect_cores(AccLds& a, Keep keep) {
  const int L = acc_lane();
  for (int k = L; k < a.n_core; k += 64) a.core_n[k] = 0, a.cref[k] = 0;
  __syncthreads();
  if (a.max_ref > 1)
    for (int c = L; c < a.n_cpu; c += 64)
      if (a.alloc[c]) atomicAdd(&a.cref[a.cpu[c].core], (int)a.aref[c]);
  for (int c = L; c < a.n_cpu; c += 64)
    if (a.alloc[c] && keep(c)) {
      const int k = a.cpu[c].core;
      const int slot = atomicAdd(&a.core_n[k], 1);
      if (slot < ACC_TPC) a.core_cpu[k][slot] = (uint8_t)c;
    }
  __syncthreads();
}

// sortCores :345-368 on a list of core ranks
__device__ inline bool cores_less(const AccLds& a, int ci, int cj) {
  if (a.core_n[ci] != a.core_n[cj]) return a.core_n[ci] > a.core_n[cj];
  if (a.max_ref > 1) {
    const int ri = core_ref(a, ci), rj = core_ref(a, cj);
    if (ri != rj) return ri < rj;
  }
  return ci < cj;
}

// Group the collected cores by NUMA node (by_socket = 0) or socket (1), full cores only if asked;
// per group the cores sorted (sortCores) and their CPUs appended -> a.lst / a.goff / a.gkey.  Groups
// in ascending key order (the caller's sort is total), cores bucketed by a counting sort.
__device__ inline void group_cores(AccLds& a, bool by_socket, bool filter_full) {
  const int L = acc_lane();
  const int cpc = acc_cpc(a.t), nkey = acc_nkey(a, by_socket);
  auto key = [&](int k) {
    const int c0 = a.core_cpu[k][0];
    return by_socket ? (int)a.cpu[c0].socket : (int)a.cpu[c0].numa;
  };
  auto in = [&](int k) { return a.core_n[k] && !(filter_full && a.core_n[k] != cpc); };
  for (int g = L; g < nkey; g += 64) a.cnt32[g] = 0;
  __syncthreads();
  for (int k = L; k < a.n_core; k += 64)
    if (in(k)) atomicAdd(&a.cnt32[key(k)], 1);
  __syncthreads();
  if (L == 0) {
    int16_t* start = a.p_sc;
    int acc = 0;
    for (int g = 0; g < nkey; g++) {
      start[g] = (int16_t)acc;
      acc += a.cnt32[g];
      a.cnt32[g] = start[g];
    }
    for (int k = 0; k < a.n_core; k++)  // ascending core rank within a bucket
      if (in(k)) a.order[a.cnt32[key(k)]++] = (int16_t)k;
    a.ng = 0;
    int pos = 0;
    for (int g = 0; g < nkey; g++) {
      const int b = start[g], nc = a.cnt32[g] - b;
      if (nc == 0) continue;
      int16_t* o = &a.order[b];
      for (int i = 1; i < nc; i++)
        for (int j = i; j > 0 && cores_less(a, o[j], o[j - 1]); j--) {
          const int16_t t = o[j];
          o[j] = o[j - 1];
          o[j - 1] = t;
        }
      a.gkey[a.ng] = (int16_t)g;
      a.goff[a.ng] = (int16_t)pos;
      for (int i = 0; i < nc; i++) {
        const int k = o[i];
        for (int q = 0; q < a.core_n[k]; q++) a.tmp[q] = a.core_cpu[k][q];
        sort_i16(a.tmp, a.core_n[k]);
        for (int q = 0; q < a.core_n[k]; q++) a.lst[pos++] = a.tmp[q];
      }
      a.ng++;
    }
    a.goff[a.ng] = (int16_t)pos;
  }
  __syncthreads();
}

__device__ __forceinline__ int glen(const AccLds& a, int g) { return a.goff[g + 1] - a.goff[g]; }

// reorder the groups of a.lst by a permutation a.order[0..ng)
__device__ inline void permute_groups(AccLds& a) {
  if (acc_lane() == 0) {
    int pos = 0;
    int16_t *noff = a.p_off, *nkey = a.p_key, *nsc = a.p_sc;
    for (int i = 0; i < a.ng; i++) {
      const int g = a.order[i];
      noff[i] = (int16_t)pos;
      nkey[i] = a.gkey[g];
      nsc[i] = a.gscore[g];
      for (int q = a.goff[g]; q < a.goff[g + 1]; q++) a.tmp[pos++] = a.lst[q];
    }
    noff[a.ng] = (int16_t)pos;
    for (int i = 0; i <= a.ng; i++) a.goff[i] = noff[i];
    for (int i = 0; i < a.ng; i++) a.gkey[i] = nkey[i], a.gscore[i] = nsc[i];
    a.bcast = pos;
  }
  __syncthreads();
  const int pos = a.bcast;
  for (int q = acc_lane(); q < pos; q += 64) a.lst[q] = a.tmp[q];
  __syncthreads();
}

// free-CPU count per socket / NUMA node of the allocatable CPUs passing `keep`
template <typename Keep>
__device__ inline void free_scores(AccLds& a, Keep keep, int32_t* per_socket, int32_t* per_node) {
  const int L = acc_lane();
  for (int k = L; k < a.n_sock; k += 64) per_socket[k] = 0;
  for (int k = L; k < a.n_numa; k += 64) per_node[k] = 0;
  __syncthreads();
  for (int c = L; c < a.n_cpu; c += 64)
    if (a.alloc[c] && keep(c)) atomicAdd(&per_socket[a.cpu[c].socket], 1), atomicAdd(&per_node[a.cpu[c].numa], 1);
  __syncthreads();
}

// freeCoresInNode :371-461
__device__ inline void free_cores_in_node(AccLds& a, bool filter_full, bool filter_excl) {
  auto keep = [&](int c) { return !(filter_excl && excl_numa(a, c)); };
  free_scores(a, keep, a.sc_sock, a.sc_node);
  collect_cores(a, keep);
  group_cores(a, false, filter_full);
  if (acc_lane() == 0) {
    const int32_t* sock = a.sc_sock;
    for (int g = 0; g < a.ng; g++) a.gscore[g] = (int16_t)glen(a, g), a.order[g] = (int16_t)g;
    for (int i = 1; i < a.ng; i++)
      for (int j = i; j > 0; j--) {
        const int gi = a.order[j], gj = a.order[j - 1];
        const int si = sock[a.cpu[a.lst[a.goff[gi]]].socket], sj = sock[a.cpu[a.lst[a.goff[gj]]].socket];
        bool less;
        if (a.gscore[gi] != a.gscore[gj]) less = strat_less(a, a.gscore[gi], a.gscore[gj]);
        else if (si != sj) less = strat_less(a, si, sj);
        else less = a.gkey[gi] < a.gkey[gj];
        if (!less) break;
        a.order[j] = (int16_t)gj;
        a.order[j - 1] = (int16_t)gi;
      }
  }
  __syncthreads();
  permute_groups(a);
}

// freeCoresInSocket :464-527
__device__ inline void free_cores_in_socket(AccLds& a, bool filter_full) {
  collect_cores(a, [](int) { return true; });
  group_cores(a, true, filter_full);
  if (acc_lane() == 0) {
    for (int g = 0; g < a.ng; g++) a.gscore[g] = (int16_t)glen(a, g), a.order[g] = (int16_t)g;
    for (int i = 1; i < a.ng; i++)
      for (int j = i; j > 0; j--) {
        const int gi = a.order[j], gj = a.order[j - 1];
        const bool less = a.gscore[gi] != a.gscore[gj] ? strat_less(a, a.gscore[gi], a.gscore[gj]) : a.gkey[gi] < a.gkey[gj];
        if (!less) break;
        a.order[j] = (int16_t)gj;
        a.order[j - 1] = (int16_t)gi;
      }
  }
  __syncthreads();
  permute_groups(a);
}

// freeCPUsInNode (:530-605, by_socket = false) / freeCPUsInSocket (:608-656, by_socket = true)
__device__ inline void free_cpus_in_group(AccLds& a, bool by_socket, bool filter_excl) {
  const int L = acc_lane();
  auto keep = [&](int c) {
    if (!filter_excl) return true;
    return by_socket ? !excl_pcpu(a, c) : !(excl_pcpu(a, c) || excl_numa(a, c));
  };
  free_scores(a, keep, a.sc_sock, a.sc_node);
  // CPUs bucketed by group key (counting sort, ascending ids within a bucket)
  const int nkey = acc_nkey(a, by_socket);
  auto key = [&](int c) { return by_socket ? (int)a.cpu[c].socket : (int)a.cpu[c].numa; };
  for (int g = L; g < nkey; g += 64) a.cnt32[g] = 0;
  __syncthreads();
  for (int c = L; c < a.n_cpu; c += 64)
    if (a.alloc[c] && keep(c)) atomicAdd(&a.cnt32[key(c)], 1);
  __syncthreads();
  if (L == 0) {
    const int32_t *sock = a.sc_sock, *node = a.sc_node;
    int16_t* first = a.p_sc;
    int acc = 0;
    for (int g = 0; g < nkey; g++) {
      first[g] = (int16_t)acc;
      acc += a.cnt32[g];
      a.cnt32[g] = first[g];
    }
    for (int c = 0; c < a.n_cpu; c++)
      if (a.alloc[c] && keep(c)) a.tmp[a.cnt32[key(c)]++] = (int16_t)c;
    a.ng = 0;
    int pos = 0;
    for (int g = 0; g < nkey; g++) {
      const int b = first[g], m = a.cnt32[g] - b;
      if (m == 0) continue;
      const int start = pos;
      for (int q = 0; q < m; q++) a.lst[pos++] = a.tmp[b + q];
      int n = m;  // ascending already; then by ref count, then one CPU per core
      if (a.max_ref > 1) sort_by_ref(a, &a.lst[start], n);
      if (filter_excl) n = extract_cpu(a, &a.lst[start], n);
      pos = start + n;
      a.gkey[a.ng] = (int16_t)g;
      a.goff[a.ng] = (int16_t)start;
      a.gscore[a.ng] = by_socket ? (int16_t)n : (int16_t)node[g];
      a.ng++;
    }
    a.goff[a.ng] = (int16_t)pos;
    for (int g = 0; g < a.ng; g++) a.order[g] = (int16_t)g;
    for (int i = 1; i < a.ng; i++)
      for (int j = i; j > 0; j--) {
        const int gi = a.order[j], gj = a.order[j - 1];
        bool less;
        if (a.gscore[gi] != a.gscore[gj]) {
          less = strat_less(a, a.gscore[gi], a.gscore[gj]);
        } else if (!by_socket) {
          const int si = sock[a.cpu[a.lst[a.goff[gi]]].socket], sj = sock[a.cpu[a.lst[a.goff[gj]]].socket];
          less = si != sj ? strat_less(a, si, sj) : a.gkey[gi] < a.gkey[gj];
        } else {
          less = a.gkey[gi] < a.gkey[gj];
        }
        if (!less) break;
        a.order[j] = (int16_t)gj;
        a.order[j - 1] = (int16_t)gi;
      }
  }
  __syncthreads();
  permute_groups(a);
}

// freeCPUs :666-774 -> a.lst[0..n)
__device__ inline int free_cpus(AccLds& a, bool filter_excl) {
  const int L = acc_lane();
  auto keep = [&](int c) { return !(filter_excl && (excl_pcpu(a, c) || excl_numa(a, c))); };
  int32_t *sock = a.sc_sock, *node = a.sc_node, *colo = a.sc_colo;
  free_scores(a, keep, sock, node);
  for (int s = L; s < a.n_sock; s += 64) colo[s] = 0;
  __syncthreads();
  for (int c = L; c < a.n_cpu; c += 64)
    if ((a.cpu[c].flags & CR_VALID) && a.res[c]) atomicAdd(&colo[a.cpu[c].socket], 1);
  collect_cores(a, keep);  // its barriers order the counts above
  if (L == 0) {
    int nc = 0;
    for (int k = 0; k < a.n_core; k++)
      if (a.core_n[k]) a.order[nc++] = (int16_t)k;
    a.bcast = nc;
  }
  __syncthreads();
  const int nc = a.bcast;
  // the cores sorted by a total order (its last key is the core rank): a core's place is the number of
  // cores before it
  auto less = [&](int ki, int kj) {
    const int ci = a.core_cpu[ki][0], cj = a.core_cpu[kj][0];
    const int si = a.cpu[ci].socket, sj = a.cpu[cj].socket, ni = a.cpu[ci].numa, nj = a.cpu[cj].numa;
    if (colo[si] != colo[sj]) return colo[si] > colo[sj];
    if (sock[si] != sock[sj]) return strat_less(a, sock[si], sock[sj]);
    if (node[ni] != node[nj]) return strat_less(a, node[ni], node[nj]);
    if (a.core_n[ki] != a.core_n[kj]) return a.core_n[ki] < a.core_n[kj];
    if (si != sj) return si < sj;
    const int ri = a.max_ref > 1 ? core_ref(a, ki) : 0, rj = a.max_ref > 1 ? core_ref(a, kj) : 0;
    return ri != rj ? ri < rj : ki < kj;
  };
  for (int i = L; i < nc; i += 64) {
    const int ki = a.order[i];
    int r = 0;
    for (int j = 0; j < nc; j++) r += less(a.order[j], ki) ? 1 : 0;
    a.p_key[r] = (int16_t)ki;
  }
  __syncthreads();
  if (L == 0) {
    int n = 0;
    for (int i = 0; i < nc; i++) {
      const int k = a.p_key[i];
      const int start = n;
      for (int q = 0; q < a.core_n[k]; q++) a.lst[n++] = a.core_cpu[k][q];
      sort_i16(&a.lst[start], a.core_n[k]);
      if (a.max_ref > 1) sort_by_ref(a, &a.lst[start], a.core_n[k]);
    }
    a.bcast = n;
  }
  __syncthreads();
  return a.bcast;
}

// spreadCPUs :798-822 on v[0..n)
__device__ inline void spread_cpus(AccLds& a, int16_t* v, int n) {
  if (n <= acc_cpc(a.t)) return;
  if (acc_lane() == 0) {
    int16_t* prep = a.tmp;
    for (int i = 0; i < n; i++) prep[i] = v[i];
    int np = n, no = 0;
    int16_t* out = a.sp_out;
    while (np > 0) {
      for (int i = 0; i < np; i++) a.mark[a.cpu[prep[i]].core] = 0;
      int nr = 0;
      for (int i = 0; i < np; i++) {
        const int core = a.cpu[prep[i]].core;
        if (a.mark[core]) {
          prep[nr++] = prep[i];  // reserved for the next pass (nr <= i: in place)
          continue;
        }
        a.mark[core] = 1;
        out[no++] = prep[i];
      }
      np = nr;
    }
    for (int i = 0; i < n; i++) v[i] = out[i];
  }
  __syncthreads();
}

// takeCPUs :87-232 on the accumulator state prepared by the caller (alloc, aref, ex_*, res = 0,
// needed, policies).  Returns true on success (a.res = the cpuset).
__device__ inline bool acc_take_cpus(AccLds& a, int bind) {
  if (a.needed < 1) return true;
  if (a.needed > acc_count_alloc(a)) return false;
  const bool full = bind == XB_FULL;
  const int cpc = acc_cpc(a.t);
  if (full || cpc == 1) {
    if (a.needed <= acc_cpn(a.t))
      for (int fe = 1; fe >= 0; fe--) {
        free_cores_in_node(a, true, fe == 1);
        for (int g = 0; g < a.ng; g++)
          if (glen(a, g) >= a.needed) {
            acc_take(a, &a.lst[a.goff[g]], a.needed);
            return true;
          }
      }
    if (a.needed <= acc_cps(a.t)) {
      free_cores_in_socket(a, true);
      for (int g = 0; g < a.ng; g++)
        if (glen(a, g) >= a.needed) {
          acc_take(a, &a.lst[a.goff[g]], a.needed);
          return true;
        }
    }
    free_cores_in_socket(a, true);
    if (acc_lane() == 0) {
      for (int g = 0; g < a.ng; g++) a.order[g] = (int16_t)g;
      for (int i = 1; i < a.ng; i++)  // sort.Slice by length desc (stable on few sockets)
        for (int j = i; j > 0 && glen(a, a.order[j]) > glen(a, a.order[j - 1]); j--) {
          const int16_t t = a.order[j];
          a.order[j] = a.order[j - 1];
          a.order[j - 1] = t;
        }
    }
    __syncthreads();
    permute_groups(a);
    int ng2 = 0, pos2 = 0;
    for (int g = 0; g < a.ng; g++) {
      const int len = glen(a, g);
      if (a.needed < len) {  // !needs(len): kept for the per-core pass
        if (acc_lane() == 0) {
          a.goff2[ng2] = (int16_t)pos2;
          for (int q = 0; q < len; q++) a.lst2[pos2 + q] = a.lst[a.goff[g] + q];
        }
        ng2++;
        pos2 += len;
      } else {
        acc_take(a, &a.lst[a.goff[g]], len);
        if (a.needed < 1) return true;
      }
    }
    if (acc_lane() == 0) a.goff2[ng2] = (int16_t)pos2, a.ng2 = ng2;
    __syncthreads();
    if (a.needed >= cpc) {
      int16_t* ord = a.ord2;
      if (acc_lane() == 0) {
        for (int g = 0; g < ng2; g++) ord[g] = (int16_t)g;
        for (int i = 1; i < ng2; i++)  // by length asc, stable
          for (int j = i; j > 0; j--) {
            const int li = a.goff2[ord[j] + 1] - a.goff2[ord[j]], lj = a.goff2[ord[j - 1] + 1] - a.goff2[ord[j - 1]];
            if (!(li < lj)) break;
            const int16_t t = ord[j];
            ord[j] = ord[j - 1];
            ord[j - 1] = t;
          }
      }
      __syncthreads();
      for (int i = 0; i < ng2; i++) {
        const int g = ord[i];
        for (int q = a.goff2[g]; q < a.goff2[g + 1]; q += cpc) {
          acc_take(a, &a.lst2[q], cpc);
          if (a.needed < 1) return true;
          if (a.needed < cpc) break;
        }
      }
    }
  }
  if (!full) {
    if (a.needed <= acc_cpn(a.t))
      for (int fe = 1; fe >= 0; fe--) {
        free_cpus_in_group(a, false, fe == 1);
        for (int g = 0; g < a.ng; g++)
          if (glen(a, g) >= a.needed) {
            spread_cpus(a, &a.lst[a.goff[g]], glen(a, g));
            acc_take(a, &a.lst[a.goff[g]], a.needed);
            return true;
          }
      }
    if (a.needed <= acc_cps(a.t))
      for (int fe = 1; fe >= 0; fe--) {
        free_cpus_in_group(a, true, fe == 1);
        for (int g = 0; g < a.ng; g++)
          if (glen(a, g) >= a.needed) {
            spread_cpus(a, &a.lst[a.goff[g]], glen(a, g));
            acc_take(a, &a.lst[a.goff[g]], a.needed);
            return true;
          }
      }
  }
  for (int fe = 1; fe >= 0; fe--) {
    const int n = free_cpus(a, fe == 1);
    spread_cpus(a, a.lst, n);
    for (int i = 0; i < n; i++) {
      if (a.needed >= 1) acc_take(a, &a.lst[i], 1);
      if (a.needed < 1) return true;
    }
  }
  return false;
}

}  // namespace ke
