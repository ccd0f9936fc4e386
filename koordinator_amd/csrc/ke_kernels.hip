// ke_kernels.hip — gfx950 kernels of the koord-scheduler Filter/Score evaluator and the device side
// of a context (GPU-resident node SoA, pod queue, speculative-batch buffers).
//
// Per speculative batch of B pods:
//   k_eval_batch  nodes x pods: fused LoadAware + NodeNUMAResource filter predicates and int64
//                 scores -> one 9-bit framework score per (pod,node) (0 = filtered out).  Lane = node,
//                 pod parameters are wave-uniform (scalar loads), the node row lives in VGPRs for
//                 the whole pod group.  HBM-streaming over the SoA; no MFMA (not a contraction).
//   k_select      one workgroup per pod: exact top-k_j (k_j = j+1) by a 9-step threshold search on
//                 the score plus an index-ordered tie break (ballot/mbcnt prefix), i.e. selectHost's
//                 order with ties to the lowest node index.
//   k_resolve     one wavefront: replays the batch sequentially — for pod j the best unchanged
//                 candidate vs an exact re-evaluation of the <= j nodes already changed by earlier
//                 pods of the batch — then Reserve-patches the chosen rows in LDS and writes them back.
// The three kernels are chained on one stream; nothing returns to the host between batches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "ke_host.h"
#include "ke_types.h"

namespace ke {

#define HIP_OK(expr)                                                                 \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      return fail(KE_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e));  \
    }                                                                                \
  } while (0)

constexpr int EVAL_BLOCK = 256;
constexpr int SELECT_BLOCK = 1024;
constexpr int SELECT_WAVES = SELECT_BLOCK / 64;
constexpr int KMAX = MAX_BATCH;

struct SoA {
  int64_t* f;       // NUM_I64_FIELDS arrays of `stride` int64
  uint32_t* flags;  // `stride` u32
  int64_t stride;
};

// ---------------------------------------------------------------------------------------------
// the fused per-(pod,node) evaluation
// ---------------------------------------------------------------------------------------------
struct NodeRegs {
  int64_t ut, fh[2][2], sa[2][2], cap[2], nalloc[2], nreq[2], csm, csaf, csas;
  uint32_t flags;
  double rcap[2], ralloc[2];  // reciprocals for the exact score divisions
};

__device__ __forceinline__ void load_row(const SoA& s, int64_t i, NodeRegs& r) {
  const int64_t st = s.stride;
  const int64_t* f = s.f + i;
  r.ut = f[F_UT * st];
#pragma unroll
  for (int v = 0; v < 2; v++)
#pragma unroll
    for (int q = 0; q < 2; q++) {
      r.fh[v][q] = f[(F_FH + 2 * v + q) * st];
      r.sa[v][q] = f[(F_SA + 2 * v + q) * st];
    }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    r.cap[q] = f[(F_CAP + q) * st];
    r.nalloc[q] = f[(F_NALLOC + q) * st];
    r.nreq[q] = f[(F_NREQ + q) * st];
  }
  r.csm = f[F_CSM * st];
  r.csaf = f[F_CSAF * st];
  r.csas = f[F_CSAS * st];
  r.flags = s.flags[i];
}

__device__ __forceinline__ void prepare_row(NodeRegs& r) {
#pragma unroll
  for (int q = 0; q < 2; q++) {
    r.rcap[q] = r.cap[q] > 0 ? 1.0 / (double)r.cap[q] : 0.0;
    r.ralloc[q] = r.nalloc[q] > 0 ? 1.0 / (double)r.nalloc[q] : 0.0;
  }
}

// floor(num / den) for num >= 0, den > 0: double estimate from a reciprocal, then exact integer
// correction (the estimate is within +-1 for the operand ranges of a scheduler score).
__device__ __forceinline__ int64_t div_exact(int64_t num, int64_t den, double rden) {
  int64_t q = (int64_t)((double)num * rden);
  int64_t rem = num - q * den;
  while (rem < 0) {
    q--;
    rem += den;
  }
  while (rem >= den) {
    q++;
    rem -= den;
  }
  return q;
}

__device__ __forceinline__ bool node_expired(const NodeRegs& r, const KArgs& k) {
  // isNodeMetricExpired  helper.go:35-40
  if (!(r.flags & NF_HAS_UT)) return true;
  return k.exp_s > 0 && (k.now - r.ut) >= k.exp_s * 1000000000LL;
}

struct EvalOut {
  int32_t total;  // -1 = filtered out
  uint8_t status, reason;
  int16_t la, numa;
};

template <bool FULL>
__device__ __forceinline__ EvalOut eval_pair(const NodeRegs& n, bool expired, const DevPod& p, const KArgs& k) {
  EvalOut o;
  o.status = KE_CODE_SUCCESS;
  o.reason = KE_REASON_NONE;
  o.la = o.numa = 0;
  const uint32_t nf = n.flags;
  if (!(nf & NF_VALID)) {
    o.status = KE_CODE_ERROR;
    o.total = -1;
    return o;
  }
  // ---- LoadAwareScheduling.Filter  load_aware.go:122-186
  if (!(p.flags & PF_DAEMONSET) && (nf & NF_HAS_METRIC)) {
    if ((k.flags & AF_FILTER_EXPIRED) && (k.flags & AF_EXP_PRESENT) && expired) {
      if (!(k.flags & AF_ENABLE_WHEN_EXPIRED)) {
        o.status = KE_CODE_UNSCHEDULABLE;
        o.reason = KE_REASON_LA_NODEMETRIC_EXPIRED;
      }
    } else if (!(nf & NF_NM_NIL)) {
      const int v = ((nf & NF_HAS_PROD_THR) && (p.flags & PF_PROD)) ? 1 : 0;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        if (o.status == KE_CODE_SUCCESS && (nf & nf_fh_on(v, q)) && p.est[q] > n.fh[v][q]) {
          o.status = KE_CODE_UNSCHEDULABLE;
          const bool agg = v == 0 && (nf & NF_FILTER_AGG);
          o.reason = (uint8_t)(agg ? KE_REASON_LA_AGG_USAGE_CPU + q : KE_REASON_LA_USAGE_CPU + q);
        }
      }
    }
  }
  // ---- NodeNUMAResource.Filter -> filterAmplifiedCPUs  plugin.go:318-442
  if (o.status == KE_CODE_SUCCESS && !(p.flags & PF_NUMA_SKIP) && p.req[0] != 0) {
    if (nf & NF_NUMA_AMP_ERR) {
      o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      o.reason = KE_REASON_NUMA_INVALID_AMPLIFICATION_RATIO;
    } else if (nf & NF_NUMA_RATIO_F) {
      if (nf & NF_NUMA_TOPO_INVALID) {
        o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
        o.reason = KE_REASON_NUMA_INVALID_CPU_TOPOLOGY;
      } else {
        int64_t req = n.nreq[0];
        if (req >= n.csm && n.csm > 0) req = req - n.csm + n.csaf;
        if (p.req[0] > n.nalloc[0] - req) {
          o.status = KE_CODE_UNSCHEDULABLE;
          o.reason = KE_REASON_NUMA_INSUFFICIENT_AMPLIFIED_CPU;
        }
      }
    }
  }
  if (o.status != KE_CODE_SUCCESS) {
    o.total = -1;
    return o;
  }
  // ---- LoadAwareScheduling.Score  load_aware.go:201-249,387-406
  int32_t la = 0;
  if ((nf & NF_HAS_METRIC) && !((k.flags & AF_EXP_PRESENT) && expired) && !(nf & NF_NM_NIL) && k.wsum_la > 0) {
    const int v = (p.flags & PF_LA_SCORE_PROD) ? 1 : 0;
    int32_t s = 0;
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const int64_t cap = n.cap[q];
      const int64_t room = n.sa[v][q] - p.est[q];  // cap - used
      int32_t sc = 0;
      if (cap != 0 && room >= 0) sc = (int32_t)div_exact(room * 100, cap, n.rcap[q]);
      s += sc * k.w_la[q];
    }
    la = (int32_t)((uint32_t)s / (uint32_t)k.wsum_la);
  }
  // ---- NodeNUMAResource.Score  scoring.go:66-139,210-249
  int32_t nu = 0;
  if (!(p.flags & PF_NUMA_SKIP) && !(nf & NF_NUMA_SCORE_ZERO)) {
    bool zero = false;
    int64_t reqc = n.nreq[0];
    if (p.req[0] != 0 && (nf & NF_NUMA_RATIO_S)) {
      if (nf & NF_NUMA_TOPO_INVALID) zero = true;
      else reqc = n.nreq[0] - n.csm + n.csas;
    }
    if (!zero) {
      int32_t s = 0, ws = 0;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int32_t w = k.w_numa[q];
        const int64_t alloc = n.nalloc[q];
        if (w == 0 || alloc == 0) continue;
        const int64_t req = (q == 0 ? reqc : n.nreq[1]) + p.req[q];
        int32_t sc;
        if (k.flags & AF_NUMA_MOST) {
          const int64_t rq = req > alloc ? alloc : req;
          sc = (int32_t)div_exact(rq * 100, alloc, n.ralloc[q]);
        } else {
          sc = req > alloc ? 0 : (int32_t)div_exact((alloc - req) * 100, alloc, n.ralloc[q]);
        }
        s += sc * w;
        ws += w;
      }
      nu = ws > 0 ? (int32_t)((uint32_t)s / (uint32_t)ws) : 0;
    }
  }
  o.la = (int16_t)la;
  o.numa = (int16_t)nu;
  o.total = k.wp_la * la + k.wp_numa * nu;
  return o;
}

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
__global__ void k_scatter_rows(SoA s, const Row* __restrict__ rows, const int32_t* __restrict__ idx, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t i = idx[t];
  const Row& r = rows[t];
#pragma unroll
  for (int f = 0; f < NUM_I64_FIELDS; f++) s.f[f * s.stride + i] = r.f[f];
  s.flags[i] = r.flags;
}

__global__ void k_gather_rows(SoA s, Row* __restrict__ rows, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Row r;
#pragma unroll
  for (int f = 0; f < NUM_I64_FIELDS; f++) r.f[f] = s.f[f * s.stride + i];
  r.flags = s.flags[i];
  r.pad = 0;
  rows[i] = r;
}

// parity mode: full status / score matrices [pod][node] + selectHost per pod
__global__ __launch_bounds__(EVAL_BLOCK) void k_eval_parity(SoA s, int n_nodes, const DevPod* __restrict__ pods,
                                                            int n_pods, int pods_per_block, KArgs k,
                                                            uint8_t* status, uint8_t* reason, int16_t* la,
                                                            int16_t* numa, int16_t* total, uint32_t* best_key) {
  const int i = blockIdx.x * EVAL_BLOCK + threadIdx.x;
  const bool live = i < n_nodes;
  NodeRegs n;
  if (live) {
    load_row(s, i, n);
    prepare_row(n);
  }
  const bool expired = live ? node_expired(n, k) : false;
  const int p0 = blockIdx.y * pods_per_block;
  const int p1 = min(n_pods, p0 + pods_per_block);
  for (int p = p0; p < p1; p++) {
    uint32_t key = 0;
    if (live) {
      const EvalOut o = eval_pair<true>(n, expired, pods[p], k);
      const int64_t o_idx = (int64_t)p * n_nodes + i;
      if (status) status[o_idx] = o.status;
      if (reason) reason[o_idx] = o.reason;
      if (la) la[o_idx] = o.la;
      if (numa) numa[o_idx] = o.numa;
      if (total) total[o_idx] = (int16_t)o.total;
      key = make_key(o.total, i);
    }
    // wave max, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) key = max(key, (uint32_t)__shfl_xor((int)key, off, 64));
    if ((threadIdx.x & 63) == 0 && key) atomicMax(&best_key[p], key);
  }
}

// batch mode: 9-bit score per (pod,node): (total+1) or 0 when filtered out
__global__ __launch_bounds__(EVAL_BLOCK) void k_eval_batch(SoA s, int n_nodes, const DevPod* __restrict__ pods,
                                                           const int32_t* __restrict__ batch_base, int batch_pods,
                                                           int pods_per_block, KArgs k, uint16_t* __restrict__ scores,
                                                           int64_t score_stride) {
  const int i = blockIdx.x * EVAL_BLOCK + threadIdx.x;
  if (i >= n_nodes) return;
  NodeRegs n;
  load_row(s, i, n);
  prepare_row(n);
  const bool expired = node_expired(n, k);
  const int base = *batch_base;
  const int p0 = blockIdx.y * pods_per_block;
  const int p1 = min(batch_pods, p0 + pods_per_block);
  for (int p = p0; p < p1; p++) {
    const EvalOut o = eval_pair<false>(n, expired, pods[base + p], k);
    scores[(int64_t)p * score_stride + i] = (uint16_t)(o.total + 1);
  }
}

__device__ __forceinline__ int wave_popc(bool pred) { return __popcll(__ballot(pred)); }

// exact top-k_j per pod, k_j = min(j+1, KMAX), ordered by (score desc, node index asc)
__global__ __launch_bounds__(SELECT_BLOCK) void k_select(const uint16_t* __restrict__ scores, int64_t score_stride,
                                                         int n_nodes, uint32_t* __restrict__ cand,
                                                         int32_t* __restrict__ cand_cnt) {
  __shared__ int32_t s_cnt[SELECT_WAVES];
  __shared__ int32_t s_tie[SELECT_WAVES];
  __shared__ int32_t s_out;
  const int j = blockIdx.x;
  const int k = min(j + 1, KMAX);
  const uint16_t* sc = scores + (int64_t)j * score_stride;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int seg = ((n_nodes + SELECT_WAVES - 1) / SELECT_WAVES + 63) & ~63;
  const int w0 = wave * seg;
  const int w1 = min(n_nodes, w0 + seg);

  auto count_ge = [&](int t) -> int {
    int c = 0;
    for (int b = w0; b < w1; b += 64) {
      const int i = b + lane;
      const int v = i < w1 ? sc[i] : 0;
      c += wave_popc(v >= t);
    }
    if (lane == 0) s_cnt[wave] = c;
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int w = 0; w < SELECT_WAVES; w++) tot += s_cnt[w];
    __syncthreads();
    return tot;
  };

  const int feasible = count_ge(1);
  int thr, need_ties;  // select all v > thr, plus the first `need_ties` with v == thr
  if (feasible <= k) {
    thr = 0;  // everything feasible, no tie selection at 0 (score 0 = filtered out)
    need_ties = 0;
  } else {
    int lo = 1, hi = 512, cnt_hi = 0;  // count(>=lo) >= k > count(>=hi)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      const int c = count_ge(mid);
      if (c >= k) lo = mid;
      else {
        hi = mid;
        cnt_hi = c;
      }
    }
    thr = lo;
    need_ties = k - cnt_hi;
  }
  // per-wave tie counts -> exclusive prefix over waves (index order)
  int ties = 0;
  if (need_ties > 0) {
    for (int b = w0; b < w1; b += 64) {
      const int i = b + lane;
      const int v = i < w1 ? sc[i] : 0;
      ties += wave_popc(v == thr);
    }
  }
  if (lane == 0) s_tie[wave] = ties;
  if (threadIdx.x == 0) s_out = 0;
  __syncthreads();
  int tie_base = 0;
  for (int w = 0; w < wave; w++) tie_base += s_tie[w];
  uint32_t* out = cand + (int64_t)j * KMAX;
  int running = tie_base;
  for (int b = w0; b < w1; b += 64) {
    const int i = b + lane;
    const int v = i < w1 ? sc[i] : 0;
    bool sel = v > thr;
    const bool tie = need_ties > 0 && v == thr && v > 0;
    const uint64_t tmask = __ballot(tie);
    if (tie) {
      const int rank = running + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(tmask >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)tmask, 0));
      sel = rank < need_ties;
    }
    running += __popcll(tmask);
    const uint64_t smask = __ballot(sel);
    if (smask) {
      int wbase = 0;
      if (lane == 0) wbase = atomicAdd(&s_out, __popcll(smask));
      wbase = __shfl(wbase, 0, 64);
      if (sel) {
        const int pos = wbase + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(smask >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)smask, 0));
        out[pos] = ((uint32_t)v << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)i);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) cand_cnt[j] = s_out;
}

// --- resolve: one wavefront replays the batch sequentially -------------------------------------
struct LdsRow {
  int64_t f[NUM_I64_FIELDS];
  uint32_t flags;
  uint32_t pad;
};

__device__ __forceinline__ void regs_from_lds(const LdsRow& r, NodeRegs& n) {
  n.ut = r.f[F_UT];
#pragma unroll
  for (int v = 0; v < 2; v++)
#pragma unroll
    for (int q = 0; q < 2; q++) {
      n.fh[v][q] = r.f[F_FH + 2 * v + q];
      n.sa[v][q] = r.f[F_SA + 2 * v + q];
    }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    n.cap[q] = r.f[F_CAP + q];
    n.nalloc[q] = r.f[F_NALLOC + q];
    n.nreq[q] = r.f[F_NREQ + q];
  }
  n.csm = r.f[F_CSM];
  n.csaf = r.f[F_CSAF];
  n.csas = r.f[F_CSAS];
  n.flags = r.flags;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}

constexpr int HASH_SLOTS = 256;

__global__ __launch_bounds__(64) void k_resolve(SoA s, const DevPod* __restrict__ pods, int32_t* __restrict__ batch_base,
                                                int batch_pods, KArgs k, const uint32_t* __restrict__ cand,
                                                const int32_t* __restrict__ cand_cnt, int32_t* __restrict__ chosen,
                                                int32_t* __restrict__ chosen_score, int32_t global_offset,
                                                uint64_t* __restrict__ stamps, int batch_index) {
  __shared__ uint32_t s_cand[MAX_BATCH * KMAX];
  __shared__ LdsRow s_chg[MAX_BATCH];
  __shared__ LdsRow s_pref[MAX_BATCH];
  __shared__ int32_t s_pref_node[MAX_BATCH];
  __shared__ int32_t s_chg_node[MAX_BATCH];
  __shared__ int32_t s_hash_key[HASH_SLOTS];
  __shared__ int32_t s_hash_val[HASH_SLOTS];
  __shared__ DevPod s_pod[MAX_BATCH];
  const int lane = threadIdx.x;
  const int base = *batch_base;
  const int B = batch_pods;

  for (int t = lane; t < B * KMAX; t += 64) {
    const int j = t / KMAX, c = t % KMAX;
    s_cand[t] = c < cand_cnt[j] ? cand[t] : 0u;
  }
  for (int t = lane; t < HASH_SLOTS; t += 64) s_hash_key[t] = -1;
  if (lane < B) s_pod[lane] = pods[base + lane];
  __syncthreads();
  // prefetch the row of each pod's best candidate (the most likely choice)
  if (lane < B) {
    uint32_t best = 0;
    for (int c = 0; c < KMAX; c++) best = max(best, s_cand[lane * KMAX + c]);
    const int node = best ? key_node(best) : -1;
    s_pref_node[lane] = node;
    if (node >= 0) {
#pragma unroll
      for (int f = 0; f < NUM_I64_FIELDS; f++) s_pref[lane].f[f] = s.f[f * s.stride + node];
      s_pref[lane].flags = s.flags[node];
    }
  }
  __syncthreads();

  int n_chg = 0;
  for (int j = 0; j < B; j++) {
    const DevPod pod = s_pod[j];
    // best snapshot candidate not changed earlier in this batch
    const uint32_t ck = s_cand[j * KMAX + lane];
    bool in_chg = false;
    if (ck) {
      const int node = key_node(ck);
      int h = (node * 0x9E3779B1u) >> 24;
      while (true) {
        const int kk = s_hash_key[h];
        if (kk < 0) break;
        if (kk == node) {
          in_chg = true;
          break;
        }
        h = (h + 1) & (HASH_SLOTS - 1);
      }
    }
    const uint32_t bu = wave_max_u32(in_chg ? 0u : ck);
    // exact re-evaluation of the changed nodes against their patched rows
    uint32_t kc = 0;
    if (lane < n_chg) {
      NodeRegs n;
      regs_from_lds(s_chg[lane], n);
      prepare_row(n);
      const EvalOut o = eval_pair<false>(n, node_expired(n, k), pod, k);
      kc = make_key(o.total, s_chg_node[lane]);
    }
    const uint32_t bc = wave_max_u32(kc);
    const uint32_t w = max(bu, bc);
    int slot = -1;
    if (w != 0) {
      const int node = key_node(w);
      if (w == bc) {
        const uint64_t m = __ballot(kc == w && lane < n_chg);
        slot = __ffsll((unsigned long long)m) - 1;
      } else {
        slot = n_chg;
        if (lane == 0) s_chg_node[slot] = node;
        if (s_pref_node[j] == node) {
          if (lane < NUM_I64_FIELDS) s_chg[slot].f[lane] = s_pref[j].f[lane];
          if (lane == 0) s_chg[slot].flags = s_pref[j].flags;
        } else {
          if (lane < NUM_I64_FIELDS) s_chg[slot].f[lane] = s.f[lane * s.stride + node];
          if (lane == 0) s_chg[slot].flags = s.flags[node];
        }
        if (lane == 0) {
          int h = (node * 0x9E3779B1u) >> 24;
          while (s_hash_key[h] >= 0) h = (h + 1) & (HASH_SLOTS - 1);
          s_hash_key[h] = node;
          s_hash_val[h] = slot;
        }
        n_chg++;
      }
      __syncthreads();
      // Reserve: LoadAware assign (the new pod has no PodMetric -> counted at its estimate in every
      // non-prod term, and in the prod terms when it is prod), NodeInfo.Requested += requests.
      if (lane == 0) {
        LdsRow& r = s_chg[slot];
        const int vmax = (r.flags & NF_HAS_METRIC) && !(r.flags & NF_NM_NIL) ? ((pod.flags & PF_PROD) ? 2 : 1) : 0;
        for (int v = 0; v < vmax; v++)
          for (int q = 0; q < 2; q++) {
            if (r.flags & nf_fh_on(v, q)) r.f[F_FH + 2 * v + q] -= pod.est[q];
            r.f[F_SA + 2 * v + q] -= pod.est[q];
          }
        r.f[F_NREQ + 0] += pod.req[0];
        r.f[F_NREQ + 1] += pod.req[1];
      }
    }
    if (lane == 0) {
      chosen[base + j] = w ? key_node(w) + global_offset : -1;
      chosen_score[base + j] = w ? key_score(w) : -1;
    }
    __syncthreads();
  }
  // write the patched rows back to the SoA
  if (lane < n_chg) {
    const int node = s_chg_node[lane];
#pragma unroll
    for (int f = 0; f < NUM_I64_FIELDS; f++) s.f[f * s.stride + node] = s_chg[lane].f[f];
  }
  if (lane == 0) {
    *batch_base = base + B;
    stamps[batch_index + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void k_stamp(uint64_t* stamps) { stamps[0] = __builtin_amdgcn_s_memrealtime(); }

// ---------------------------------------------------------------------------------------------
// device state
// ---------------------------------------------------------------------------------------------
struct DeviceState {
  int device = 0;
  hipStream_t stream = nullptr;
  SoA soa{};
  int64_t capacity = 0;
  // staging for row uploads
  Row* d_rows = nullptr;
  int32_t* d_idx = nullptr;
  int64_t staging_cap = 0;
  // pods
  DevPod* d_pods = nullptr;
  int64_t pods_cap = 0;
  // batch buffers
  uint16_t* d_scores = nullptr;  // [MAX_BATCH][capacity]
  uint32_t* d_cand = nullptr;    // [MAX_BATCH][KMAX]
  int32_t* d_cand_cnt = nullptr;
  int32_t* d_batch_base = nullptr;
  int32_t* d_chosen = nullptr;
  int32_t* d_chosen_score = nullptr;
  uint64_t* d_stamps = nullptr;
  int64_t out_cap = 0;
  // parity outputs
  void* d_parity = nullptr;
  int64_t parity_cap = 0;
  uint32_t* d_best = nullptr;
  int64_t best_cap = 0;
  int profile_every = 0;
};

static int ensure(void** p, int64_t* cap, int64_t bytes) {
  if (*cap >= bytes) return KE_OK;
  if (*p) HIP_OK(hipFree(*p));
  *p = nullptr;
  *cap = 0;
  HIP_OK(hipMalloc(p, (size_t)bytes));
  *cap = bytes;
  return KE_OK;
}

int device_available() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
  return 1;
}

int device_create(Context* ctx) {
  if (!device_available()) return fail(KE_ERR_NO_DEVICE, "no HIP device available (the evaluator has no CPU path)");
  auto* d = new DeviceState();
  ctx->dev = d;
  d->device = ctx->cfg.device_ordinal;
  HIP_OK(hipSetDevice(d->device));
  HIP_OK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
  d->capacity = ((int64_t)ctx->cfg.node_capacity + 255) & ~255LL;
  d->soa.stride = d->capacity;
  HIP_OK(hipMalloc(&d->soa.f, sizeof(int64_t) * NUM_I64_FIELDS * d->capacity));
  HIP_OK(hipMalloc(&d->soa.flags, sizeof(uint32_t) * d->capacity));
  HIP_OK(hipMemsetAsync(d->soa.f, 0, sizeof(int64_t) * NUM_I64_FIELDS * d->capacity, d->stream));
  HIP_OK(hipMemsetAsync(d->soa.flags, 0, sizeof(uint32_t) * d->capacity, d->stream));
  HIP_OK(hipMalloc(&d->d_scores, sizeof(uint16_t) * MAX_BATCH * d->capacity));
  HIP_OK(hipMalloc(&d->d_cand, sizeof(uint32_t) * MAX_BATCH * KMAX));
  HIP_OK(hipMalloc(&d->d_cand_cnt, sizeof(int32_t) * MAX_BATCH));
  HIP_OK(hipMalloc(&d->d_batch_base, sizeof(int32_t)));
  HIP_OK(hipStreamSynchronize(d->stream));
  return KE_OK;
}

void device_destroy(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->stream) (void)hipStreamSynchronize(d->stream);
  void* ptrs[] = {d->soa.f, d->soa.flags, d->d_rows, d->d_idx, d->d_pods, d->d_scores, d->d_cand, d->d_cand_cnt,
                  d->d_batch_base, d->d_chosen, d->d_chosen_score, d->d_stamps, d->d_parity, d->d_best};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (d->stream) (void)hipStreamDestroy(d->stream);
  delete d;
  ctx->dev = nullptr;
}

static KArgs make_kargs(const Context* ctx, int64_t now) {
  KArgs k = ctx->kargs_template;
  k.now = now;
  return k;
}

// Re-derive rows of dirty / time-expired nodes and scatter them into the SoA.
int device_refresh(Context* ctx, int64_t now) {
  DeviceState* d = ctx->dev;
  std::vector<Row> rows;
  std::vector<int32_t> idx;
  for (int32_t i = 0; i < ctx->n_nodes; i++) {
    NodeState& ns = ctx->nodes[i];
    if (!ns.dirty && now < ns.valid_until) continue;
    Row r;
    int64_t vu;
    derive_row(ctx->cfg, ns, now, &r, &vu);
    ns.valid_until = vu;
    ns.dirty = false;
    rows.push_back(r);
    idx.push_back(i);
  }
  if (rows.empty()) return KE_OK;
  HIP_OK(hipSetDevice(d->device));
  const int64_t n = (int64_t)rows.size();
  if (d->staging_cap < n) {
    if (d->d_rows) HIP_OK(hipFree(d->d_rows));
    if (d->d_idx) HIP_OK(hipFree(d->d_idx));
    HIP_OK(hipMalloc(&d->d_rows, sizeof(Row) * n));
    HIP_OK(hipMalloc(&d->d_idx, sizeof(int32_t) * n));
    d->staging_cap = n;
  }
  HIP_OK(hipMemcpyAsync(d->d_rows, rows.data(), sizeof(Row) * n, hipMemcpyHostToDevice, d->stream));
  HIP_OK(hipMemcpyAsync(d->d_idx, idx.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, d->stream));
  hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, d->stream, d->soa, d->d_rows,
                     d->d_idx, (int)n);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(d->stream));  // `rows` is a local host vector
  return KE_OK;
}

static int upload_pods(Context* ctx, int32_t n_pods, const ke_pod* pods) {
  DeviceState* d = ctx->dev;
  std::vector<DevPod> dp((size_t)n_pods);
  for (int32_t p = 0; p < n_pods; p++) dp[p] = make_dev_pod(ctx->cfg, pods[p]);
  int rc = ensure((void**)&d->d_pods, &d->pods_cap, sizeof(DevPod) * (int64_t)std::max(n_pods, 1));
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(d->d_pods, dp.data(), sizeof(DevPod) * n_pods, hipMemcpyHostToDevice, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  return KE_OK;
}

int device_eval(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, uint8_t* status, uint8_t* reason,
                int16_t* la, int16_t* numa, int16_t* total, int32_t* best) {
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  int rc = device_refresh(ctx, now);
  if (rc) return rc;
  if (n_pods == 0) return KE_OK;
  rc = upload_pods(ctx, n_pods, pods);
  if (rc) return rc;
  const int64_t N = ctx->n_nodes, P = n_pods, M = N * P;
  // parity buffers: status u8, reason u8, la i16, numa i16, total i16 = 8 B per pair
  rc = ensure(&d->d_parity, &d->parity_cap, std::max<int64_t>(M, 1) * 8 + 16);
  if (rc) return rc;
  rc = ensure((void**)&d->d_best, &d->best_cap, sizeof(uint32_t) * P);
  if (rc) return rc;
  uint8_t* d_status = (uint8_t*)d->d_parity;
  uint8_t* d_reason = d_status + M;
  int16_t* d_la = (int16_t*)(d_reason + M + (M & 1));
  int16_t* d_numa = d_la + M;
  int16_t* d_total = d_numa + M;
  HIP_OK(hipMemsetAsync(d->d_best, 0, sizeof(uint32_t) * P, d->stream));
  const KArgs k = make_kargs(ctx, now);
  const int ppb = 8;
  dim3 grid((unsigned)((N + EVAL_BLOCK - 1) / EVAL_BLOCK), (unsigned)((P + ppb - 1) / ppb));
  if (N > 0) {
    hipLaunchKernelGGL(k_eval_parity, grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, (int)N, d->d_pods, (int)P, ppb,
                       k, d_status, d_reason, d_la, d_numa, d_total, d->d_best);
    HIP_OK(hipGetLastError());
  }
  if (status) HIP_OK(hipMemcpyAsync(status, d_status, M, hipMemcpyDeviceToHost, d->stream));
  if (reason) HIP_OK(hipMemcpyAsync(reason, d_reason, M, hipMemcpyDeviceToHost, d->stream));
  if (la) HIP_OK(hipMemcpyAsync(la, d_la, M * 2, hipMemcpyDeviceToHost, d->stream));
  if (numa) HIP_OK(hipMemcpyAsync(numa, d_numa, M * 2, hipMemcpyDeviceToHost, d->stream));
  if (total) HIP_OK(hipMemcpyAsync(total, d_total, M * 2, hipMemcpyDeviceToHost, d->stream));
  std::vector<uint32_t> bk((size_t)P);
  HIP_OK(hipMemcpyAsync(bk.data(), d->d_best, sizeof(uint32_t) * P, hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  if (best)
    for (int64_t p = 0; p < P; p++) best[p] = bk[p] ? key_node(bk[p]) + ctx->cfg.global_node_offset : -1;
  return KE_OK;
}

int device_schedule(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, int32_t* chosen, int32_t* score) {
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  int rc = device_refresh(ctx, now);
  if (rc) return rc;
  ctx->last_batch_ms.clear();
  ctx->last_total_ms = 0;
  if (n_pods == 0) return KE_OK;
  rc = upload_pods(ctx, n_pods, pods);
  if (rc) return rc;
  const int B = ctx->cfg.pod_batch;
  const int n_batches = (n_pods + B - 1) / B;
  const int64_t out_bytes = sizeof(int32_t) * (int64_t)n_pods;
  if (d->out_cap < n_pods) {
    if (d->d_chosen) HIP_OK(hipFree(d->d_chosen));
    if (d->d_chosen_score) HIP_OK(hipFree(d->d_chosen_score));
    if (d->d_stamps) HIP_OK(hipFree(d->d_stamps));
    HIP_OK(hipMalloc(&d->d_chosen, out_bytes));
    HIP_OK(hipMalloc(&d->d_chosen_score, out_bytes));
    HIP_OK(hipMalloc(&d->d_stamps, sizeof(uint64_t) * ((int64_t)n_pods + 2)));
    d->out_cap = n_pods;
  }
  const KArgs k = make_kargs(ctx, now);
  const int N = ctx->n_nodes;
  const int ppb = 8;
  HIP_OK(hipMemsetAsync(d->d_batch_base, 0, sizeof(int32_t), d->stream));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, d->stream));
  hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, d->stream, d->d_stamps);
  // sampled per-kernel HIP event pairs (ke_set_profiling)
  const int every = d->profile_every;
  std::vector<hipEvent_t> ev;
  if (every > 0) {
    const int samples = (n_batches + every - 1) / every;
    ev.resize((size_t)samples * 4);
    for (auto& e : ev) HIP_OK(hipEventCreate(&e));
  }
  for (int b = 0; b < n_batches; b++) {
    const int bp = std::min(B, n_pods - b * B);
    const bool prof = every > 0 && b % every == 0;
    hipEvent_t* pe = prof ? &ev[(size_t)(b / every) * 4] : nullptr;
    if (prof) HIP_OK(hipEventRecord(pe[0], d->stream));
    if (N > 0) {
      dim3 grid((unsigned)((N + EVAL_BLOCK - 1) / EVAL_BLOCK), (unsigned)((bp + ppb - 1) / ppb));
      hipLaunchKernelGGL(k_eval_batch, grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, N, d->d_pods, d->d_batch_base, bp,
                         ppb, k, d->d_scores, d->capacity);
      if (prof) HIP_OK(hipEventRecord(pe[1], d->stream));
      hipLaunchKernelGGL(k_select, dim3((unsigned)bp), dim3(SELECT_BLOCK), 0, d->stream, d->d_scores, d->capacity, N,
                         d->d_cand, d->d_cand_cnt);
    } else {
      if (prof) HIP_OK(hipEventRecord(pe[1], d->stream));
      HIP_OK(hipMemsetAsync(d->d_cand_cnt, 0, sizeof(int32_t) * MAX_BATCH, d->stream));
    }
    if (prof) HIP_OK(hipEventRecord(pe[2], d->stream));
    hipLaunchKernelGGL(k_resolve, dim3(1), dim3(64), 0, d->stream, d->soa, d->d_pods, d->d_batch_base, bp, k,
                       d->d_cand, d->d_cand_cnt, d->d_chosen, d->d_chosen_score, ctx->cfg.global_node_offset,
                       d->d_stamps, b);
    if (prof) HIP_OK(hipEventRecord(pe[3], d->stream));
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(e1, d->stream));
  HIP_OK(hipMemcpyAsync(chosen, d->d_chosen, out_bytes, hipMemcpyDeviceToHost, d->stream));
  if (score) HIP_OK(hipMemcpyAsync(score, d->d_chosen_score, out_bytes, hipMemcpyDeviceToHost, d->stream));
  std::vector<uint64_t> st((size_t)n_batches + 1);
  HIP_OK(hipMemcpyAsync(st.data(), d->d_stamps, sizeof(uint64_t) * (n_batches + 1), hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  ctx->last_total_ms = ms;
  // s_memrealtime ticks -> ms, calibrated against the event-timed span of the whole queue
  const double span = (double)(st[n_batches] - st[0]);
  const double ms_per_tick = span > 0 ? ms / span : 1e-5;
  ctx->last_batch_ms.resize(n_batches);
  for (int b = 0; b < n_batches; b++) ctx->last_batch_ms[b] = (double)(st[b + 1] - st[b]) * ms_per_tick;
  ctx->kstat_samples = 0;
  ctx->kstat_eval_ms = ctx->kstat_select_ms = ctx->kstat_resolve_ms = 0;
  for (size_t s = 0; s + 3 < ev.size(); s += 4) {
    float a = 0, b = 0, c = 0;
    HIP_OK(hipEventElapsedTime(&a, ev[s], ev[s + 1]));
    HIP_OK(hipEventElapsedTime(&b, ev[s + 1], ev[s + 2]));
    HIP_OK(hipEventElapsedTime(&c, ev[s + 2], ev[s + 3]));
    ctx->kstat_eval_ms += a;
    ctx->kstat_select_ms += b;
    ctx->kstat_resolve_ms += c;
    ctx->kstat_samples++;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  if (ctx->kstat_samples) {
    ctx->kstat_eval_ms /= ctx->kstat_samples;
    ctx->kstat_select_ms /= ctx->kstat_samples;
    ctx->kstat_resolve_ms /= ctx->kstat_samples;
  }
  return KE_OK;
}

int device_set_profiling(Context* ctx, int32_t every) {
  ctx->dev->profile_every = every < 0 ? 0 : every;
  return KE_OK;
}

int device_bench_eval(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, int32_t iters, double* avg_ms) {
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  if (n_pods < 1 || n_pods > MAX_BATCH || iters < 1) return fail(KE_ERR_INVALID, "bench: 1 <= n_pods <= 64, iters >= 1");
  int rc = device_refresh(ctx, now);
  if (rc) return rc;
  rc = upload_pods(ctx, n_pods, pods);
  if (rc) return rc;
  const int N = ctx->n_nodes;
  if (N == 0) return fail(KE_ERR_INVALID, "bench: no nodes");
  const KArgs k = make_kargs(ctx, now);
  const int ppb = 8;
  HIP_OK(hipMemsetAsync(d->d_batch_base, 0, sizeof(int32_t), d->stream));
  dim3 grid((unsigned)((N + EVAL_BLOCK - 1) / EVAL_BLOCK), (unsigned)((n_pods + ppb - 1) / ppb));
  hipLaunchKernelGGL(k_eval_batch, grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, N, d->d_pods, d->d_batch_base, n_pods,
                     ppb, k, d->d_scores, d->capacity);  // warm
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, d->stream));
  for (int it = 0; it < iters; it++)
    hipLaunchKernelGGL(k_eval_batch, grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, N, d->d_pods, d->d_batch_base,
                       n_pods, ppb, k, d->d_scores, d->capacity);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(e1, d->stream));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *avg_ms = ms / iters;
  return KE_OK;
}

int device_debug_rows(Context* ctx, int32_t n, Row* out) {
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  Row* tmp = nullptr;
  HIP_OK(hipMalloc(&tmp, sizeof(Row) * std::max(n, 1)));
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, d->stream, d->soa, tmp, n);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(out, tmp, sizeof(Row) * n, hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  HIP_OK(hipFree(tmp));
  return KE_OK;
}

}  // namespace ke
