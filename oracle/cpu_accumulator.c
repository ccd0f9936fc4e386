/* Oracle (test infrastructure only): plain-C restatement of NodeNUMAResource's CPU accumulator,
 * pkg/scheduler/plugins/nodenumaresource/cpu_accumulator.go (takePreferredCPUs :29-85, takeCPUs
 * :87-232, cpuAccumulator :234-822), with the CPU topology helpers of cpu_topology.go:24-105.
 *
 * Go map iteration feeds every list here, but each list is sorted afterwards by a total order
 * (ids last), except two sort.Slice calls in takeCPUs (:142-144, :161-163) whose comparators tie on
 * equal lengths: sockets are few (< 12), where Go's sort.Slice is an insertion sort and therefore
 * stable, so ties keep the socket order freeCoresInSocket produced.  That is what acc_sort_stable does.
 */
#include "cpu_accumulator.h"

#include <string.h>

/* ---- sets of CPU ids --------------------------------------------------------------------------- */
static int bs_has(const uint64_t* s, int c) { return (int)((s[c >> 6] >> (c & 63)) & 1u); }
static void bs_add(uint64_t* s, int c) { s[c >> 6] |= 1ull << (c & 63); }
static void bs_del(uint64_t* s, int c) { s[c >> 6] &= ~(1ull << (c & 63)); }
static int bs_count(const uint64_t* s) {
  int n = 0;
  for (int w = 0; w < ACC_WORDS; w++) n += __builtin_popcountll(s[w]);
  return n;
}

/* CPUTopology counts (cpu_topology.go:45-105): sockets, (socket, node) pairs, (socket, node, core) triples */
void acc_topo_finish(acc_topo* t) {
  t->num_cpus = t->num_sockets = t->num_nodes = t->num_cores = 0;
  int socks[ACC_MAX_CPUS], ns = 0;
  int sn[ACC_MAX_CPUS][2], nn = 0;
  int snc[ACC_MAX_CPUS][3], nc = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) {
    if (!t->valid[c]) continue;
    t->num_cpus++;
    int f = 0;
    for (int i = 0; i < ns && !f; i++) f = socks[i] == t->socket[c];
    if (!f) socks[ns++] = t->socket[c];
    f = 0;
    for (int i = 0; i < nn && !f; i++) f = sn[i][0] == t->socket[c] && sn[i][1] == t->node[c];
    if (!f) sn[nn][0] = t->socket[c], sn[nn][1] = t->node[c], nn++;
    f = 0;
    for (int i = 0; i < nc && !f; i++)
      f = snc[i][0] == t->socket[c] && snc[i][1] == t->node[c] && snc[i][2] == t->core[c];
    if (!f) snc[nc][0] = t->socket[c], snc[nc][1] = t->node[c], snc[nc][2] = t->core[c], nc++;
  }
  t->num_sockets = ns;
  t->num_nodes = nn;
  t->num_cores = nc;
}
int acc_cpus_per_core(const acc_topo* t) { return t->num_cores ? t->num_cpus / t->num_cores : 0; }
int acc_cpus_per_socket(const acc_topo* t) { return t->num_sockets ? t->num_cpus / t->num_sockets : 0; }
int acc_cpus_per_node(const acc_topo* t) { return t->num_nodes ? t->num_cpus / t->num_nodes : 0; }

/* ---- the accumulator ----------------------------------------------------------------------------- */
typedef struct acc {
  const acc_topo* t;
  int max_ref;
  uint64_t alloc[ACC_WORDS]; /* allocatableCPUs */
  int ref[ACC_MAX_CPUS];     /* allocatableCPUs[c].RefCount (max_ref > 1) */
  int needed;
  int exclusive, excl_policy, numa_most;
  int excl_core[ACC_MAX_CPUS], n_excl_core; /* exclusiveInCores (core ids) */
  int excl_node[ACC_MAX_CPUS], n_excl_node; /* exclusiveInNUMANodes */
  uint64_t result[ACC_WORDS];
} acc;

static int in_list(const int* l, int n, int v) {
  for (int i = 0; i < n; i++)
    if (l[i] == v) return 1;
  return 0;
}

/* newCPUAccumulator :247-288 */
static void acc_init(acc* a, const acc_topo* t, int max_ref, const uint64_t* available, const acc_alloc* allocated,
                     int needed, int excl_policy, int numa_most) {
  memset(a, 0, sizeof *a);
  a->t = t;
  a->max_ref = max_ref;
  for (int c = 0; c < ACC_MAX_CPUS; c++) {
    if (allocated && allocated->present[c]) {
      if (allocated->excl[c] == ACC_EXCL_PCPU && !in_list(a->excl_core, a->n_excl_core, t->core[c]))
        a->excl_core[a->n_excl_core++] = t->core[c];
      else if (allocated->excl[c] == ACC_EXCL_NUMA && !in_list(a->excl_node, a->n_excl_node, t->node[c]))
        a->excl_node[a->n_excl_node++] = t->node[c];
    }
    if (t->valid[c] && bs_has(available, c)) { /* topology.CPUDetails.KeepOnly(availableCPUs) */
      bs_add(a->alloc, c);
      if (max_ref > 1) a->ref[c] = allocated && allocated->present[c] ? allocated->ref[c] : 0;
    }
  }
  a->exclusive = excl_policy == ACC_EXCL_PCPU || excl_policy == ACC_EXCL_NUMA;
  a->excl_policy = excl_policy;
  a->needed = needed;
  a->numa_most = numa_most;
}

static void acc_take(acc* a, const int* cpus, int n) { /* :290-304 */
  for (int i = 0; i < n; i++) {
    const int c = cpus[i];
    bs_add(a->result, c);
    bs_del(a->alloc, c);
    if (a->exclusive) {
      if (a->excl_policy == ACC_EXCL_PCPU && !in_list(a->excl_core, a->n_excl_core, a->t->core[c]))
        a->excl_core[a->n_excl_core++] = a->t->core[c];
      else if (a->excl_policy == ACC_EXCL_NUMA && !in_list(a->excl_node, a->n_excl_node, a->t->node[c]))
        a->excl_node[a->n_excl_node++] = a->t->node[c];
    }
  }
  a->needed -= n;
}
static int acc_needs(const acc* a, int n) { return a->needed >= n; }
static int acc_satisfied(const acc* a) { return a->needed < 1; }
static int acc_failed(const acc* a) { return a->needed > bs_count(a->alloc); }
static int excl_pcpu(const acc* a, int c) {
  return a->excl_policy == ACC_EXCL_PCPU && in_list(a->excl_core, a->n_excl_core, a->t->core[c]);
}
static int excl_numa(const acc* a, int c) {
  return a->excl_policy == ACC_EXCL_NUMA && in_list(a->excl_node, a->n_excl_node, a->t->node[c]);
}

/* getCoreRefCount :776-783 over the allocatable CPUs */
static int core_ref(const acc* a, int core) {
  int r = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++)
    if (bs_has(a->alloc, c) && a->t->core[c] == core) r += a->ref[c];
  return r;
}

/* a group of CPUs (one core, node or socket) */
typedef struct grp {
  int key;  /* core / node / socket id */
  int n;
  int cpu[ACC_MAX_CPUS];
} grp;

static grp* grp_get(grp* g, int* ng, int key) {
  for (int i = 0; i < *ng; i++)
    if (g[i].key == key) return &g[i];
  g[*ng].key = key;
  g[*ng].n = 0;
  return &g[(*ng)++];
}

static void sort_ints(int* v, int n) {
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && v[j] < v[j - 1]; j--) {
      const int t = v[j];
      v[j] = v[j - 1];
      v[j - 1] = t;
    }
}

/* sortCPUsByRefCount :785-796 */
static void sort_by_ref(const acc* a, int* v, int n) {
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0; j--) {
      const int x = v[j], y = v[j - 1];
      const int less = a->ref[x] != a->ref[y] ? a->ref[x] < a->ref[y] : x < y;
      if (!less) break;
      v[j] = y;
      v[j - 1] = x;
    }
}

/* extractCPU :332-343: the first CPU of each core, in list order */
static int extract_cpu(const acc* a, int* v, int n) {
  int cores[ACC_MAX_CPUS], nc = 0, m = 0;
  for (int i = 0; i < n; i++) {
    const int core = a->t->core[v[i]];
    if (in_list(cores, nc, core)) continue;
    cores[nc++] = core;
    v[m++] = v[i];
  }
  return m;
}

/* sortCores :345-368 (a total order: ties end on the core id) */
static int cores_less(const acc* a, const grp* i, const grp* j) {
  if (i->n != j->n) return i->n > j->n;
  if (a->max_ref > 1) {
    const int ri = core_ref(a, i->key), rj = core_ref(a, j->key);
    if (ri != rj) return ri < rj;
  }
  return i->key < j->key;
}

/* the CPUs of the allocatable cores of one group, cores sorted, CPU ids ascending per core */
static void concat_cores(const acc* a, grp* cores, int* idx, int n, grp* out) {
  for (int i = 1; i < n; i++) /* sort the core indices */
    for (int j = i; j > 0 && cores_less(a, &cores[idx[j]], &cores[idx[j - 1]]); j--) {
      const int t = idx[j];
      idx[j] = idx[j - 1];
      idx[j - 1] = t;
    }
  out->n = 0;
  for (int i = 0; i < n; i++) {
    grp* c = &cores[idx[i]];
    sort_ints(c->cpu, c->n);
    for (int k = 0; k < c->n; k++) out->cpu[out->n++] = c->cpu[k];
  }
}

static int strategy_less(const acc* a, int si, int sj) { return a->numa_most ? si < sj : si > sj; }

/* freeCoresInNode :371-461 -> out groups keyed by NUMA node, in order */
static int free_cores_in_node(const acc* a, int filter_full, int filter_excl, grp* out) {
  static __thread grp cores[ACC_MAX_CPUS];
  int nc = 0, sock_key[ACC_MAX_CPUS], sock_score[ACC_MAX_CPUS], ns = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) {
    if (!bs_has(a->alloc, c)) continue;
    if (filter_excl && excl_numa(a, c)) continue;
    grp* g = grp_get(cores, &nc, a->t->core[c]);
    g->cpu[g->n++] = c;
    int s = 0;
    while (s < ns && sock_key[s] != a->t->socket[c]) s++;
    if (s == ns) sock_key[ns] = a->t->socket[c], sock_score[ns++] = 0;
    sock_score[s]++;
  }
  const int cpc = acc_cpus_per_core(a->t);
  int node_key[ACC_MAX_CPUS], nn = 0;
  static __thread int node_cores[ACC_MAX_CPUS][ACC_MAX_CPUS];
  int node_nc[ACC_MAX_CPUS];
  for (int i = 0; i < nc; i++) {
    if (filter_full && cores[i].n != cpc) continue;
    const int node = a->t->node[cores[i].cpu[0]];
    int k = 0;
    while (k < nn && node_key[k] != node) k++;
    if (k == nn) node_key[nn] = node, node_nc[nn++] = 0;
    node_cores[k][node_nc[k]++] = i;
  }
  for (int k = 0; k < nn; k++) {
    out[k].key = node_key[k];
    concat_cores(a, cores, node_cores[k], node_nc[k], &out[k]);
  }
  int order[ACC_MAX_CPUS];
  for (int k = 0; k < nn; k++) order[k] = k;
  for (int i = 1; i < nn; i++) /* total order: node id last */
    for (int j = i; j > 0; j--) {
      const grp *gi = &out[order[j]], *gj = &out[order[j - 1]];
      const int si = a->t->socket[gi->cpu[0]], sj = a->t->socket[gj->cpu[0]];
      int less;
      if (gi->n != gj->n) {
        less = strategy_less(a, gi->n, gj->n);
      } else {
        int fi = 0, fj = 0;
        for (int s = 0; s < ns; s++) {
          if (sock_key[s] == si) fi = sock_score[s];
          if (sock_key[s] == sj) fj = sock_score[s];
        }
        less = fi != fj ? strategy_less(a, fi, fj) : gi->key < gj->key;
      }
      if (!less) break;
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  static __thread grp tmp[ACC_MAX_CPUS];
  for (int k = 0; k < nn; k++) tmp[k] = out[order[k]];
  for (int k = 0; k < nn; k++) out[k] = tmp[k];
  return nn;
}

/* freeCoresInSocket :464-527 */
static int free_cores_in_socket(const acc* a, int filter_full, grp* out) {
  static __thread grp cores[ACC_MAX_CPUS];
  int nc = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) {
    if (!bs_has(a->alloc, c)) continue;
    grp* g = grp_get(cores, &nc, a->t->core[c]);
    g->cpu[g->n++] = c;
  }
  const int cpc = acc_cpus_per_core(a->t);
  int sock_key[ACC_MAX_CPUS], ns = 0, sock_nc[ACC_MAX_CPUS];
  static __thread int sock_cores[ACC_MAX_CPUS][ACC_MAX_CPUS];
  for (int i = 0; i < nc; i++) {
    if (filter_full && cores[i].n != cpc) continue;
    const int s = a->t->socket[cores[i].cpu[0]];
    int k = 0;
    while (k < ns && sock_key[k] != s) k++;
    if (k == ns) sock_key[ns] = s, sock_nc[ns++] = 0;
    sock_cores[k][sock_nc[k]++] = i;
  }
  for (int k = 0; k < ns; k++) {
    out[k].key = sock_key[k];
    concat_cores(a, cores, sock_cores[k], sock_nc[k], &out[k]);
  }
  int order[ACC_MAX_CPUS];
  for (int k = 0; k < ns; k++) order[k] = k;
  for (int i = 1; i < ns; i++)
    for (int j = i; j > 0; j--) {
      const grp *gi = &out[order[j]], *gj = &out[order[j - 1]];
      const int less = gi->n != gj->n ? strategy_less(a, gi->n, gj->n) : gi->key < gj->key;
      if (!less) break;
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  static __thread grp tmp[ACC_MAX_CPUS];
  for (int k = 0; k < ns; k++) tmp[k] = out[order[k]];
  for (int k = 0; k < ns; k++) out[k] = tmp[k];
  return ns;
}

/* freeCPUsInNode :530-605 */
static int free_cpus_in_node(const acc* a, int filter_excl, grp* out) {
  int nn = 0, node_score[ACC_MAX_CPUS], sock_key[ACC_MAX_CPUS], sock_score[ACC_MAX_CPUS], ns = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) {
    if (!bs_has(a->alloc, c)) continue;
    if (filter_excl && (excl_pcpu(a, c) || excl_numa(a, c))) continue;
    int k = 0;
    while (k < nn && out[k].key != a->t->node[c]) k++;
    if (k == nn) out[nn].key = a->t->node[c], out[nn].n = 0, node_score[nn++] = 0;
    out[k].cpu[out[k].n++] = c;
    node_score[k]++;
    int s = 0;
    while (s < ns && sock_key[s] != a->t->socket[c]) s++;
    if (s == ns) sock_key[ns] = a->t->socket[c], sock_score[ns++] = 0;
    sock_score[s]++;
  }
  for (int k = 0; k < nn; k++) {
    sort_ints(out[k].cpu, out[k].n);
    if (a->max_ref > 1) sort_by_ref(a, out[k].cpu, out[k].n);
    if (filter_excl) out[k].n = extract_cpu(a, out[k].cpu, out[k].n);
  }
  int order[ACC_MAX_CPUS];
  for (int k = 0; k < nn; k++) order[k] = k;
  for (int i = 1; i < nn; i++)
    for (int j = i; j > 0; j--) {
      const int ki = order[j], kj = order[j - 1];
      const int si = a->t->socket[out[ki].cpu[0]], sj = a->t->socket[out[kj].cpu[0]];
      int fi = 0, fj = 0;
      for (int s = 0; s < ns; s++) {
        if (sock_key[s] == si) fi = sock_score[s];
        if (sock_key[s] == sj) fj = sock_score[s];
      }
      int less;
      if (node_score[ki] != node_score[kj]) less = strategy_less(a, node_score[ki], node_score[kj]);
      else if (fi != fj) less = strategy_less(a, fi, fj);
      else less = out[ki].key < out[kj].key;
      if (!less) break;
      order[j] = kj;
      order[j - 1] = ki;
    }
  static __thread grp tmp[ACC_MAX_CPUS];
  for (int k = 0; k < nn; k++) tmp[k] = out[order[k]];
  for (int k = 0; k < nn; k++) out[k] = tmp[k];
  return nn;
}

/* freeCPUsInSocket :608-656 */
static int free_cpus_in_socket(const acc* a, int filter_excl, grp* out) {
  int ns = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) {
    if (!bs_has(a->alloc, c)) continue;
    if (filter_excl && excl_pcpu(a, c)) continue;
    grp* g = grp_get(out, &ns, a->t->socket[c]);
    g->cpu[g->n++] = c;
  }
  for (int k = 0; k < ns; k++) {
    sort_ints(out[k].cpu, out[k].n);
    if (a->max_ref > 1) sort_by_ref(a, out[k].cpu, out[k].n);
    if (filter_excl) out[k].n = extract_cpu(a, out[k].cpu, out[k].n);
  }
  int order[ACC_MAX_CPUS];
  for (int k = 0; k < ns; k++) order[k] = k;
  for (int i = 1; i < ns; i++)
    for (int j = i; j > 0; j--) {
      const grp *gi = &out[order[j]], *gj = &out[order[j - 1]];
      const int less = gi->n != gj->n ? strategy_less(a, gi->n, gj->n) : gi->key < gj->key;
      if (!less) break;
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  static __thread grp tmp[ACC_MAX_CPUS];
  for (int k = 0; k < ns; k++) tmp[k] = out[order[k]];
  for (int k = 0; k < ns; k++) out[k] = tmp[k];
  return ns;
}

/* freeCPUs :666-774 -> flat list */
static int free_cpus(const acc* a, int filter_excl, int* out) {
  static __thread grp cores[ACC_MAX_CPUS];
  int nc = 0, node_key[ACC_MAX_CPUS], node_score[ACC_MAX_CPUS], nn = 0;
  int sock_key[ACC_MAX_CPUS], sock_score[ACC_MAX_CPUS], sock_colo[ACC_MAX_CPUS], ns = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) {
    if (!bs_has(a->alloc, c)) continue;
    if (filter_excl && (excl_pcpu(a, c) || excl_numa(a, c))) continue;
    grp* g = grp_get(cores, &nc, a->t->core[c]);
    g->cpu[g->n++] = c;
    int k = 0;
    while (k < nn && node_key[k] != a->t->node[c]) k++;
    if (k == nn) node_key[nn] = a->t->node[c], node_score[nn++] = 0;
    node_score[k]++;
    int s = 0;
    while (s < ns && sock_key[s] != a->t->socket[c]) s++;
    if (s == ns) sock_key[ns] = a->t->socket[c], sock_score[ns++] = 0;
    sock_score[s]++;
  }
  for (int s = 0; s < ns; s++) { /* CPUsInSockets(socket) ∩ result */
    sock_colo[s] = 0;
    for (int c = 0; c < ACC_MAX_CPUS; c++)
      if (a->t->valid[c] && a->t->socket[c] == sock_key[s] && bs_has(a->result, c)) sock_colo[s]++;
  }
  int order[ACC_MAX_CPUS];
  for (int i = 0; i < nc; i++) order[i] = i;
  for (int i = 1; i < nc; i++)
    for (int j = i; j > 0; j--) {
      const grp *gi = &cores[order[j]], *gj = &cores[order[j - 1]];
      const int ci = gi->cpu[0], cj = gj->cpu[0];
      const int si = a->t->socket[ci], sj = a->t->socket[cj], ni = a->t->node[ci], nj = a->t->node[cj];
      int coi = 0, coj = 0, fsi = 0, fsj = 0, fni = 0, fnj = 0;
      for (int s = 0; s < ns; s++) {
        if (sock_key[s] == si) coi = sock_colo[s], fsi = sock_score[s];
        if (sock_key[s] == sj) coj = sock_colo[s], fsj = sock_score[s];
      }
      for (int k = 0; k < nn; k++) {
        if (node_key[k] == ni) fni = node_score[k];
        if (node_key[k] == nj) fnj = node_score[k];
      }
      int less;
      if (coi != coj) less = coi > coj;
      else if (fsi != fsj) less = strategy_less(a, fsi, fsj);
      else if (fni != fnj) less = strategy_less(a, fni, fnj);
      else if (gi->n != gj->n) less = gi->n < gj->n;
      else if (si != sj) less = si < sj;
      else {
        int ri = 0, rj = 0;
        if (a->max_ref > 1) ri = core_ref(a, gi->key), rj = core_ref(a, gj->key);
        less = ri != rj ? ri < rj : gi->key < gj->key;
      }
      if (!less) break;
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  int n = 0;
  for (int i = 0; i < nc; i++) {
    grp* g = &cores[order[i]];
    sort_ints(g->cpu, g->n);
    if (a->max_ref > 1) sort_by_ref(a, g->cpu, g->n);
    for (int k = 0; k < g->n; k++) out[n++] = g->cpu[k];
  }
  return n;
}

/* spreadCPUs :798-822 (in place) */
static void spread_cpus(const acc* a, int* v, int n) {
  if (n <= acc_cpus_per_core(a->t)) return;
  int prep[ACC_MAX_CPUS], np = n, out[ACC_MAX_CPUS], no = 0;
  memcpy(prep, v, sizeof(int) * (size_t)n);
  while (np > 0) {
    int res[ACC_MAX_CPUS], nr = 0, cores[ACC_MAX_CPUS], nc = 0;
    for (int i = 0; i < np; i++) {
      const int core = a->t->core[prep[i]];
      if (in_list(cores, nc, core)) {
        res[nr++] = prep[i];
        continue;
      }
      out[no++] = prep[i];
      cores[nc++] = core;
    }
    memcpy(prep, res, sizeof(int) * (size_t)nr);
    np = nr;
  }
  memcpy(v, out, sizeof(int) * (size_t)n);
}

/* stable sort of groups by length (sort.Slice on <= 12 sockets is Go's insertion sort) */
static void sort_groups_by_len(grp* g, int n, int desc) {
  static __thread grp t;
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0; j--) {
      const int less = desc ? g[j].n > g[j - 1].n : g[j].n < g[j - 1].n;
      if (!less) break;
      t = g[j];
      g[j] = g[j - 1];
      g[j - 1] = t;
    }
}

/* takeCPUs :87-232.  Returns 0 and `result` on success, -1 on failure. */
int acc_take_cpus(const acc_topo* t, int max_ref, const uint64_t* available, const acc_alloc* allocated, int needed,
                  int bind, int excl_policy, int numa_most, uint64_t* result) {
  static __thread acc a;
  static __thread grp groups[ACC_MAX_CPUS];
  acc_init(&a, t, max_ref, available, allocated, needed, excl_policy, numa_most);
  memset(result, 0, sizeof(uint64_t) * ACC_WORDS);
  if (acc_satisfied(&a)) return 0;
  if (acc_failed(&a)) return -1;
  const int full = bind == ACC_BIND_FULL_PCPUS;
  const int cpc = acc_cpus_per_core(t);
  if (full || cpc == 1) {
    if (a.needed <= acc_cpus_per_node(t))
      for (int fe = 1; fe >= 0; fe--) {
        const int n = free_cores_in_node(&a, 1, fe, groups);
        for (int k = 0; k < n; k++)
          if (groups[k].n >= a.needed) {
            acc_take(&a, groups[k].cpu, a.needed);
            memcpy(result, a.result, sizeof a.result);
            return 0;
          }
      }
    if (a.needed <= acc_cpus_per_socket(t)) {
      const int n = free_cores_in_socket(&a, 1, groups);
      for (int k = 0; k < n; k++)
        if (groups[k].n >= a.needed) {
          acc_take(&a, groups[k].cpu, a.needed);
          memcpy(result, a.result, sizeof a.result);
          return 0;
        }
    }
    int n = free_cores_in_socket(&a, 1, groups);
    sort_groups_by_len(groups, n, 1);
    static __thread grp unsat[ACC_MAX_CPUS];
    int nu = 0;
    for (int k = 0; k < n; k++) {
      if (!acc_needs(&a, groups[k].n)) {
        unsat[nu++] = groups[k];
      } else {
        acc_take(&a, groups[k].cpu, groups[k].n);
        if (acc_satisfied(&a)) {
          memcpy(result, a.result, sizeof a.result);
          return 0;
        }
      }
    }
    if (acc_needs(&a, cpc)) {
      sort_groups_by_len(unsat, nu, 0);
      for (int k = 0; k < nu; k++)
        for (int i = 0; i < unsat[k].n; i += cpc) {
          acc_take(&a, &unsat[k].cpu[i], cpc);
          if (acc_satisfied(&a)) {
            memcpy(result, a.result, sizeof a.result);
            return 0;
          }
          if (!acc_needs(&a, cpc)) break;
        }
    }
  }
  if (!full) {
    if (a.needed <= acc_cpus_per_node(t))
      for (int fe = 1; fe >= 0; fe--) {
        const int n = free_cpus_in_node(&a, fe, groups);
        for (int k = 0; k < n; k++)
          if (groups[k].n >= a.needed) {
            spread_cpus(&a, groups[k].cpu, groups[k].n);
            acc_take(&a, groups[k].cpu, a.needed);
            memcpy(result, a.result, sizeof a.result);
            return 0;
          }
      }
    if (a.needed <= acc_cpus_per_socket(t))
      for (int fe = 1; fe >= 0; fe--) {
        const int n = free_cpus_in_socket(&a, fe, groups);
        for (int k = 0; k < n; k++)
          if (groups[k].n >= a.needed) {
            spread_cpus(&a, groups[k].cpu, groups[k].n);
            acc_take(&a, groups[k].cpu, a.needed);
            memcpy(result, a.result, sizeof a.result);
            return 0;
          }
      }
  }
  for (int fe = 1; fe >= 0; fe--) {
    int cpus[ACC_MAX_CPUS];
    const int n = free_cpus(&a, fe, cpus);
    spread_cpus(&a, cpus, n);
    for (int i = 0; i < n; i++) {
      if (acc_needs(&a, 1)) acc_take(&a, &cpus[i], 1);
      if (acc_satisfied(&a)) {
        memcpy(result, a.result, sizeof a.result);
        return 0;
      }
    }
  }
  return -1;
}

/* takePreferredCPUs :29-85 */
int acc_take_preferred_cpus(const acc_topo* t, int max_ref, const uint64_t* available, const uint64_t* preferred,
                            const acc_alloc* allocated, int needed, int bind, int excl_policy, int numa_most,
                            uint64_t* result) {
  uint64_t avail[ACC_WORDS], pref[ACC_WORDS], res[ACC_WORDS] = {0};
  int any = 0;
  for (int w = 0; w < ACC_WORDS; w++) {
    avail[w] = available[w];
    pref[w] = preferred ? available[w] & preferred[w] : 0;
    any |= pref[w] != 0;
  }
  if (any) {
    int n = needed;
    if (n > bs_count(pref)) n = bs_count(pref);
    if (acc_take_cpus(t, max_ref, pref, allocated, n, bind, excl_policy, numa_most, res) != 0) {
      memcpy(result, res, sizeof res);
      return -1;
    }
    needed -= bs_count(res);
    for (int w = 0; w < ACC_WORDS; w++) avail[w] &= ~pref[w];
  }
  if (needed > 0) {
    uint64_t more[ACC_WORDS];
    if (acc_take_cpus(t, max_ref, avail, allocated, needed, bind, excl_policy, numa_most, more) != 0) {
      memset(result, 0, sizeof(uint64_t) * ACC_WORDS);
      return -1;
    }
    for (int w = 0; w < ACC_WORDS; w++) res[w] |= more[w];
  }
  memcpy(result, res, sizeof res);
  return 0;
}

/* freeCPUs + spreadCPUs order (TestCPUSpreadByPCPUs): the accumulator's spread list of `available` */
int acc_spread_order(const acc_topo* t, const uint64_t* available, int numa_most, int* out) {
  static __thread acc a;
  acc_init(&a, t, 1, available, NULL, 0, ACC_EXCL_NONE, numa_most);
  const int n = free_cpus(&a, 0, out);
  spread_cpus(&a, out, n);
  return n;
}
