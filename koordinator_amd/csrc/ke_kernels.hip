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
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ke_cpuacc.h"
#include "ke_merge.h"
#include "ke_host.h"
#include "ke_types.h"

namespace ke {

// wave-wide reductions from the device library (DPP)
extern "C" __device__ uint32_t __ockl_wfred_max_u32(uint32_t);
extern "C" __device__ int32_t __ockl_wfred_add_i32(int32_t);

#define HIP_OK(expr)                                                                 \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      return fail(KE_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e));  \
    }                                                                                \
  } while (0)

constexpr int EVAL_BLOCK = 256;
constexpr int PST = 16;  // replay stamps / counters per batch (ke_debug_resolve_phases)
// k_eval_batch grid: node tiles padded to a multiple of the 8 XCDs (x) x pod groups (y)
inline dim3 eval_grid(int n_nodes, int block, int pods, int ppb) {
  const int tiles = (n_nodes + block - 1) / block;
  return dim3((unsigned)((tiles + 7) / 8 * 8), (unsigned)((pods + ppb - 1) / ppb));
}
constexpr int SELECT_BLOCK = 1024;
constexpr int SELECT_WAVES = SELECT_BLOCK / 64;
constexpr int KMAX = MAX_BATCH;

struct SoA {
  int64_t* f;       // NUM_I64_FIELDS arrays of `stride` int64
  uint32_t* flags;  // `stride` u32
  int64_t stride;
  int64_t* ds;      // DeviceShare: NUM_DS_FIELDS arrays of `stride` int64 (nullptr until a device cache appears)
  uint64_t* dsm;    // DeviceShare: NUM_DS_MASKS arrays of `stride` uint64
  int64_t* nf;      // NUMA topology: NUM_NUMA_FIELDS arrays of `stride` int64 (nullptr until a NUMA node appears)
  uint64_t* nm;     // NUMA topology: `stride` uint64 zone / key masks (ke_types.h NUMA_M_*)
  int64_t* cs;      // CPU tables: NUM_CS_FIELDS arrays of `stride` int64 (nullptr until a cpuset pod / CPU table)
  CpuRec* cpu;      // CPU tables: CPU_SLOTS records per node, node-major
  int64_t* qt;      // ElasticQuota: NUM_QF arrays of QT_STRIDE int64 (nullptr until a tree is loaded)
  int32_t* qm;      // ElasticQuota: QT_STRIDE meta words (ke_types.h qm_*)
  int64_t* rec;     // replay records: NUM_RW int64 words per node, row-major (RecWord)
  uint64_t* pt;     // GPU partition tables: PT_WORDS words per table (ke_types.h), nullptr until one is set
  int32_t* kerr;    // device error word of the context (KERR_* bits; the host reads it after a call)
  int64_t* xf;      // NodeResourcesFitPlus / ScarceResourceAvoidance: NUM_XF arrays of `stride` int64 (XF_*)
  uint64_t* xm;     //   and `stride` uint64 masks of the resource ids with Allocatable > 0 (nullptr when off)
  // DeviceShare batches (nullptr until a device cache appears): per pod of the batch 1 + the snapshot max raw
  // score over its feasible nodes (DSB_MAX), how many feasible nodes attain it (DSB_CNT), and the replay's cut
  // word (DSB_CUT: the first pod it left unplaced, -1 = none)
  uint32_t* dsb;
  uint16_t* dsraw;  // DeviceShare batch: per pod, 1 + each node's raw score in the batch's snapshot (0 = infeasible)
  // DeviceShare hints: per node NUM_DSX words (DSX_*, field-major, allocated with the device
  // SoA), the hinted pods' records of the current call (DevPod::ring_bw = slot), and per pod of the call the VF
  // ranks its Reserve took ([pod][type - 1][minor], -1 = none)
  int64_t* dsx;
  const DevPodHint* ph;
  int8_t* vfo;
  // a KE_RSV_MATCHED segment's allocate-from-reservation decisions (RsvOvr) for its NF_RSV_CS nodes
  const RsvOvr* rovr;
  int32_t n_rovr;
};
__device__ __forceinline__ const RsvOvr* rsv_ovr_of(const SoA& s, int64_t node) {
  for (int q = 0; q < s.n_rovr; q++)
    if (s.rovr[q].node == node) return &s.rovr[q];
  return nullptr;
}
constexpr int DSB_MAX = 0, DSB_CNT = 64, DSB_CUT = 128, DSB_WORDS = 129;
// kerr bits: an input the kernels refuse mid-call (the call returns KE_ERR_UNSUPPORTED)
constexpr int32_t KERR_HINT_ROUTE = 2;  // a hinted pod reached a kernel instantiated without the hint path (H)
constexpr int32_t KERR_LDS_WAIT = 4;    // a bounded intra-workgroup LDS wait of the replay expired (internal)

// ---------------------------------------------------------------------------------------------
// ElasticQuota PreFilter / Reserve (elasticquota/plugin.go:223-275,345-359; plugin_helper.go:281-301;
// core/group_quota_manager.go:700-760,943-963).  Used limits come from the host (ke_host.cpp
// quota_compute_limits); the request is Mask(PodRequests, Max names of the pod's quota).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t qtf(const SoA& s, int f, int q) { return s.qt[f * QT_STRIDE + q]; }

// one thread, global memory (singleton batches)
__device__ bool quota_admit_g(const SoA& s, const DevPod& p, const KArgs& k, int64_t req[2]) {
  const int qi = (int)p.quota - 1;
  const int32_t m = s.qm[qi];
  for (int r = 0; r < 2; r++) req[r] = qm_max(m, r) ? p.req[r] : 0;
  for (int r = 0; r < 2; r++)
    if (qm_lim(m, r) && qtf(s, QF_USED + r, qi) + req[r] > qtf(s, QF_LIM + r, qi)) return false;
  if (p.flags & PF_QUOTA_NP)
    for (int r = 0; r < 2; r++)
      if (qm_min(m, r) && qtf(s, QF_NP + r, qi) + req[r] > qtf(s, QF_MIN + r, qi)) return false;
  if (k.flags & AF_QUOTA_PARENT)
    for (int a = qm_parent(m); a >= 0; a = qm_parent(s.qm[a]))
      for (int r = 0; r < 2; r++)
        if (req[r] != 0 && qm_lim(s.qm[a], r) && qtf(s, QF_USED + r, a) + req[r] > qtf(s, QF_LIM + r, a)) return false;
  return true;
}
__device__ void quota_reserve_g(const SoA& s, const DevPod& p, const int64_t req[2]) {
  for (int a = (int)p.quota - 1; a >= 0; a = qm_parent(s.qm[a]))
    for (int r = 0; r < 2; r++) {
      s.qt[(QF_USED + r) * QT_STRIDE + a] += req[r];
      if (p.flags & PF_QUOTA_NP) s.qt[(QF_NP + r) * QT_STRIDE + a] += req[r];
    }
}

// the replay's copy: lane l holds used / non-preemptible used of quotas l, 64+l, 128+l, 192+l
struct QuotaRegs {
  int64_t u[4][2], n[4][2];
};
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t qreg_get(const int64_t (&a)[4][2], int q, int r) {  // q wave-uniform
  const int b = q >> 6;
  const int64_t v = b == 0 ? a[0][r] : b == 1 ? a[1][r] : b == 2 ? a[2][r] : a[3][r];
  return readlane64(v, q & 63);
}
__device__ __forceinline__ bool quota_admit_r(const SoA& s, const DevPod& p, const KArgs& k, const QuotaRegs& Q,
                                              int64_t req[2]) {
  const int qi = (int)p.quota - 1;
  const int32_t m = s.qm[qi];
#pragma unroll
  for (int r = 0; r < 2; r++) req[r] = qm_max(m, r) ? p.req[r] : 0;
  bool ok = true;
#pragma unroll
  for (int r = 0; r < 2; r++)
    ok = ok && !(qm_lim(m, r) && qreg_get(Q.u, qi, r) + req[r] > qtf(s, QF_LIM + r, qi));
  if (p.flags & PF_QUOTA_NP)
#pragma unroll
    for (int r = 0; r < 2; r++)
      ok = ok && !(qm_min(m, r) && qreg_get(Q.n, qi, r) + req[r] > qtf(s, QF_MIN + r, qi));
  if (ok && (k.flags & AF_QUOTA_PARENT))
    for (int a = qm_parent(m); a >= 0 && ok; a = qm_parent(s.qm[a]))
#pragma unroll
      for (int r = 0; r < 2; r++)
        ok = ok && !(req[r] != 0 && qm_lim(s.qm[a], r) && qreg_get(Q.u, a, r) + req[r] > qtf(s, QF_LIM + r, a));
  return ok;
}
__device__ __forceinline__ void quota_reserve_r(const SoA& s, const DevPod& p, QuotaRegs& Q, const int64_t req[2],
                                                int lane) {
  const bool np = (p.flags & PF_QUOTA_NP) != 0;
  for (int a = (int)p.quota - 1; a >= 0; a = qm_parent(s.qm[a])) {
    if (lane != (a & 63)) continue;
#pragma unroll
    for (int b = 0; b < 4; b++)
      if (b == (a >> 6))
#pragma unroll
        for (int r = 0; r < 2; r++) {
          Q.u[b][r] += req[r];
          if (np) Q.n[b][r] += req[r];
        }
  }
}

// Amplify (node_resource_amplification.go:170-175) with the ratio's IEEE bits from the CPU SoA
__device__ __forceinline__ int64_t amplify_bits(int64_t q, int64_t ratio_bits) {
  const double r = __longlong_as_double(ratio_bits);
  if (r <= 1.0) return q;
  return (int64_t)ceil((double)q * r);
}

// ---------------------------------------------------------------------------------------------
// the fused per-(pod,node) evaluation
// ---------------------------------------------------------------------------------------------
struct NodeRegs {
  int64_t ut, fh[2][2], sa[2][2], cap[2], nalloc[2], nreq[2], csm, csaf, csas;
  uint32_t flags;
  double dcap[2], rcap[2], dalloc[2], ralloc[2];  // cap/alloc as double and approximate reciprocals
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
    r.dcap[q] = (double)r.cap[q];
    r.rcap[q] = __builtin_amdgcn_rcp(r.dcap[q]);
    r.dalloc[q] = (double)r.nalloc[q];
    r.ralloc[q] = __builtin_amdgcn_rcp(r.dalloc[q]);
  }
}

// x * 100 / c for 0 < c < 2^42 and 0 <= x <= 16c (Go int64 division, truncating) — the
// framework.MaxNodeScore scaling of every least/most scorer.  On that range x, c, x*100 and every
// q*c below are integers < 2^53, so each double product and comparison is exact: the reciprocal
// estimate is off by at most one (q <= 1600, relative error << 2^-12) and one exact test in each
// direction fixes it.  No 64-bit integer multiply (quarter-rate on the VALU).
constexpr int64_t DIV_FAST_CAP = 1LL << 42;
__device__ __forceinline__ bool div100_fast_ok(int64_t x, int64_t c) { return c > 0 && c < DIV_FAST_CAP && x >= 0 && x <= 16 * c; }
__device__ __forceinline__ int32_t div100_f(int64_t x, double dc, double rc) {
  const double dx = (double)x * 100.0;
  const int32_t q = (int32_t)(dx * rc);
  const double t = (double)q * dc;
  return q - (int32_t)(t > dx) + (int32_t)(t + dc <= dx);
}
__device__ __forceinline__ int32_t div100(int64_t x, int64_t c, double dc, double rc) {
  if (!div100_fast_ok(x, c)) return (int32_t)(x * 100 / c);
  return div100_f(x, dc, rc);
}

// floor(s / d) for 0 <= s < 2^22, 0 < d < 2^22 (weighted means of per-resource scores); 24-bit
// multiplies are full rate
__device__ __forceinline__ int32_t div_small(int32_t s, int32_t d) {
  int32_t q = (int32_t)((float)s * __builtin_amdgcn_rcpf((float)d));
  q -= (int32_t)(__mul24(q, d) > s);
  q += (int32_t)(__mul24(q + 1, d) <= s);
  return q;
}

__device__ __forceinline__ bool node_expired(const NodeRegs& r, const KArgs& k) {
  // isNodeMetricExpired  helper.go:35-40
  if (!(r.flags & NF_HAS_UT)) return true;
  return k.exp_s > 0 && (k.now - r.ut) >= k.exp_s * 1000000000LL;
}

struct EvalOut {
  int32_t total;  // -1 = filtered out; else Σ weight·score of LoadAware + NodeNUMAResource (DeviceShare
                  // enters after NormalizeScore, once the pod's max over feasible nodes is known)
  uint8_t status, reason;
  uint8_t aff;           // NUMA policy: the affinity Admit stored for the node (0 = nil)
  int16_t la, numa, ds;  // ds: DeviceShare.Score before NormalizeScore
};

// ---------------------------------------------------------------------------------------------
// DeviceShare on one node (pkg/scheduler/plugins/deviceshare).  The device
// cache of node i is read straight from the device SoA (L1/L2-resident across the pods of a block).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t dsf(const SoA& s, int field, int64_t i) { return s.ds[field * s.stride + i]; }
__device__ __forceinline__ uint64_t dsmask(const SoA& s, int w, int64_t i) { return s.dsm[w * s.stride + i]; }

__device__ __forceinline__ bool pod_req_has(const DevPod& p, int t, int k) {
  if (t != KE_DEV_GPU) return true;
  return (p.flags & (k == 0 ? PF_DS_H_CORE : (k == 1 ? PF_DS_H_MEM : PF_DS_H_RATIO))) != 0;
}

// One device instance as nodeDevice.filter leaves it (device_cache.go:360-415): free_orig =
// SubtractWithNonNegativeResult(total, used); used' = total - free_orig (dropped when zero);
// free' = used' zero ? total : total - used'.  Keys: presence bits.
struct DsInst {
  int64_t tv[3], fv[3];
  uint32_t th, fh;  // key presence of total / free'
  bool used_nz;     // used' kept (non-zero): the minor is in getRealUsed (allocator_gpu.go:59-70)
};
#ifndef KE_DS_GRP
#define KE_DS_GRP 2
#endif
// the instance's total / used words (0 for absent keys), loaded ahead of their use (ds_type_view issues a
// group of instances' loads together: one memory round trip per group instead of per instance)
struct DsRaw {
  int64_t tv[3], uv[3];
};
// rv (k_ds_views): the view's preemptible beyond the row's restore leaves max(0, used - pre) (the caller's msk
// carries the pre keys as used keys)
__device__ __forceinline__ void ds_load(const SoA& s, int64_t i, int t, int m, const uint64_t msk[4], DsRaw& r,
                                        const DsView* rv = nullptr) {
  const int nk = DS_NK[t];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const bool ht = k < nk && ((msk[ds_ht_word(t)] >> ds_ht_bit(t, m, k)) & 1);
    const bool hu = k < nk && ((msk[ds_hu_word(t)] >> ds_hu_bit(t, m, k)) & 1);
    r.tv[k] = ht ? dsf(s, DS_TBASE[t] + m * nk + k, i) : 0;
    r.uv[k] = hu ? dsf(s, DS_UBASE[t] + m * nk + k, i) : 0;
    if (rv && k < nk && ((rv->pre_keys[k] >> (16 * t + m)) & 1)) {
      const int64_t u = r.uv[k] - rv->pre[t][m][k];
      r.uv[k] = u > 0 ? u : 0;
    }
  }
}
// rv with the instance in cap_in (a Restricted reservation's requiredDeviceResources): free_orig =
// MinResourceList(free_orig, cap) -- the keys of both, the smaller value (pkg/util/resource.go:64-78)
__device__ __forceinline__ void ds_instance_from(const DsRaw& r, int t, int m, const uint64_t msk[4], DsInst& d,
                                                 const DsView* rv = nullptr) {
  const int nk = DS_NK[t];
  int64_t up[3];
  uint32_t uh = 0;
  d.th = 0;
  const bool capped = rv && ((rv->cap_in[t] >> m) & 1u);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    d.tv[k] = 0;
    up[k] = 0;
    d.fv[k] = 0;
    if (k >= nk) continue;
    const bool ht = (msk[ds_ht_word(t)] >> ds_ht_bit(t, m, k)) & 1;
    const bool hu = (msk[ds_hu_word(t)] >> ds_hu_bit(t, m, k)) & 1;
    const int64_t tv = r.tv[k];
    const int64_t uv = r.uv[k];
    int64_t fo = ht ? (tv - uv > 0 ? tv - uv : 0) : 0;  // free_orig (used-only keys: 0)
    bool fh = ht || hu;                                  // its keys
    if (capped) {
      const bool ch = (rv->cap_keys[k] >> (16 * t + m)) & 1;
      fh = fh && ch;
      fo = fh ? (fo < rv->cap[t][m][k] ? fo : rv->cap[t][m][k]) : 0;
    }
    up[k] = ht ? (tv - fo > 0 ? tv - fo : 0) : 0;  // used' = total - free_orig (keys of both)
    d.tv[k] = tv;
    d.th |= (uint32_t)ht << k;
    uh |= (uint32_t)(ht || fh) << k;
  }
  bool up_zero = true;
#pragma unroll
  for (int k = 0; k < 3; k++) up_zero = up_zero && !(((uh >> k) & 1) && up[k] != 0);
  d.used_nz = !up_zero;
  d.fh = up_zero ? d.th : uh;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const bool ht = (d.th >> k) & 1;
    d.fv[k] = up_zero ? d.tv[k] : (ht ? (d.tv[k] - up[k] > 0 ? d.tv[k] - up[k] : 0) : 0);
  }
}

// quotav1.IsZero(free')
__device__ __forceinline__ bool ds_free_zero(const DsInst& d) {
  bool zero = true;
#pragma unroll
  for (int k = 0; k < 3; k++) zero = zero && !(((d.fh >> k) & 1) && d.fv[k] != 0);
  return zero;
}
// quotav1.LessThanOrEqual(request, free'): the keys of free' the request also has
__device__ __forceinline__ bool ds_leq(const DsInst& d, const DevPod& p, int t) {
  bool leq = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const bool fh = (d.fh >> k) & 1;
    if (fh && k < DS_NK[t] && pod_req_has(p, t, k) && p.ds_req[ds_req_slot(t, k)] > d.fv[k]) leq = false;
  }
  return leq;
}
// defaultAllocateDevices' test: !IsZero(free') && LessThanOrEqual(request, free')
__device__ __forceinline__ bool ds_satisfied(const DsInst& d, const DevPod& p, int t) {
  return !ds_free_zero(d) && ds_leq(d, p, t);
}
// removeZeroDevice: the instance's total is not zero
__device__ __forceinline__ bool ds_total_nz(const DsInst& d) {
  bool nz = false;
#pragma unroll
  for (int k = 0; k < 3; k++) nz = nz || (((d.th >> k) & 1) && d.tv[k] != 0);
  return nz;
}

// x*100/cap exactly (Go int64 division) without the 64-bit division routine on the usual range (div100)
__device__ __forceinline__ int64_t ds_div100(int64_t x, int64_t cap) {
  const double dc = (double)cap;
  return div100(x, cap, dc, __builtin_amdgcn_rcp(dc));
}
__device__ __forceinline__ int64_t ds_res_score(bool most, int64_t req, int64_t cap) {  // scoring.go:283-322
  if (cap == 0) return 0;
  if (most) return ds_div100(req > cap ? cap : req, cap);
  return req > cap ? 0 : ds_div100(cap - req, cap);
}

// resourceAllocationScorer.scorer over per-key (requested, allocatable) with weights (scoring.go:268-297)
__device__ __forceinline__ int64_t ds_weighted(const KArgs& k, int t, const int64_t* tot, const int64_t* fre,
                                               const DevPod& p) {
  int64_t sc = 0, ws = 0;
  for (int key = 0; key < DS_NK[t]; key++) {
    const int wi = ds_weight_index(t, key);
    if (wi < 0 || k.w_ds[wi] < 0 || tot[key] == 0) continue;
    const int64_t pr = pod_req_has(p, t, key) ? p.ds_req[ds_req_slot(t, key)] : 0;
    const int64_t req = tot[key] >= fre[key] ? tot[key] - fre[key] + pr : tot[key];
    sc += ds_res_score(k.flags & AF_DS_MOST, req, tot[key]) * k.w_ds[wi];
    ws += k.w_ds[wi];
  }
  if (!ws) return 0;
  return (sc >= 0 && sc < (1 << 22) && ws < (1 << 22)) ? div_small((int32_t)sc, (int32_t)ws) : sc / ws;
}

// bitmask.IterateBitMasks order over NUMA ids 0..7: by popcount, then lexicographic on the ascending
// id list.  Restricted to the subsets of a node's zones it is the order over those zones.
__constant__ uint8_t NUMA_ORDER[255] = {
    1, 2, 4, 8, 16, 32, 64, 128, 3, 5, 9, 17, 33, 65, 129, 6, 10, 18, 34, 66, 130, 12, 20, 36, 68, 132, 24,
    40, 72, 136, 48, 80, 144, 96, 160, 192, 7, 11, 19, 35, 67, 131, 13, 21, 37, 69, 133, 25, 41, 73, 137,
    49, 81, 145, 97, 161, 193, 14, 22, 38, 70, 134, 26, 42, 74, 138, 50, 82, 146, 98, 162, 194, 28, 44, 76,
    140, 52, 84, 148, 100, 164, 196, 56, 88, 152, 104, 168, 200, 112, 176, 208, 224, 15, 23, 39, 71, 135,
    27, 43, 75, 139, 51, 83, 147, 99, 163, 195, 29, 45, 77, 141, 53, 85, 149, 101, 165, 197, 57, 89, 153,
    105, 169, 201, 113, 177, 209, 225, 30, 46, 78, 142, 54, 86, 150, 102, 166, 198, 58, 90, 154, 106, 170,
    202, 114, 178, 210, 226, 60, 92, 156, 108, 172, 204, 116, 180, 212, 228, 120, 184, 216, 232, 240, 31,
    47, 79, 143, 55, 87, 151, 103, 167, 199, 59, 91, 155, 107, 171, 203, 115, 179, 211, 227, 61, 93, 157,
    109, 173, 205, 117, 181, 213, 229, 121, 185, 217, 233, 241, 62, 94, 158, 110, 174, 206, 118, 182, 214,
    230, 122, 186, 218, 234, 242, 124, 188, 220, 236, 244, 248, 63, 95, 159, 111, 175, 207, 119, 183, 215,
    231, 123, 187, 219, 235, 243, 125, 189, 221, 237, 245, 249, 126, 190, 222, 238, 246, 250, 252, 127, 191,
    223, 239, 247, 251, 253, 254, 255};
__constant__ uint8_t NUMA_OFF[10] = {0, 0, 8, 36, 92, 162, 218, 246, 254, 255};  // first entry of each size

// Diagnostic build (-DKE_PROF_REPLAY, tools/replay_phases.sh): shader-clock cycles of each phase of
// the per-pod replay loop, summed over every pod into g_rprof (ke_debug_replay_phases).  Off in the
// product build (the macro expands to nothing).
#ifdef KE_PROF_REPLAY
__device__ unsigned long long g_rprof[4][8];  // per kernel: k_resolve, k_numa_fallback, k_cpuset_reserve, k_select
#define RPROF_DECL uint64_t rp_[7] = {0, 0, 0, 0, 0, 0, 0}, rp_t = __builtin_amdgcn_s_memtime();
#define RPROF(i)                                         \
  {                                                      \
    const uint64_t rp_n = __builtin_amdgcn_s_memtime(); \
    rp_[i] += rp_n - rp_t;                               \
    rp_t = rp_n;                                         \
  }
#define RPROF_FLUSH(blk, npods)                                                           \
  if (lane == 0) {                                                                        \
    for (int u_ = 0; u_ < 7; u_++) atomicAdd(&g_rprof[blk][u_], (unsigned long long)rp_[u_]); \
    atomicAdd(&g_rprof[blk][7], (unsigned long long)(npods));                             \
  }
#else
#define RPROF_DECL
#define RPROF(i)
#define RPROF_FLUSH(blk, npods)
#endif

// ---- GPUAllocator.Allocate (allocator_gpu.go:72-451) ------------------------------------------------
// The node's GPUs as AllocateContext sees them, as minor masks.
struct GpuMasks {
  uint32_t minors;  // every GPU device (DeviceInfos; the scope tree's minors)
  uint32_t total;   // removeZeroDevice(deviceTotal[GPU]); 0 when the filtered view dropped the type
  uint32_t used;    // deviceUsedMinorsHash
  uint32_t sat;     // allocateFromScope: LessThanOrEqual(request, deviceFree) && in deviceTotal
  uint32_t dflt;    // defaultAllocateDevices: !IsZero(free') && LessThanOrEqual(request, free')
  uint32_t pref;    // defaultAllocateDevices' preferred minors (a matched reservation's, k_ds_views; else 0)
};

// minors whose 4-bit rank in `w` equals r (SWAR nibble compare)
__device__ __forceinline__ uint32_t rank_mask(uint64_t w, int r) {
  const uint64_t x = w ^ ((uint64_t)(uint32_t)r * 0x1111111111111111ull);
  const uint64_t lo = 0x7777777777777777ull;
  const uint64_t t = ~(((x & lo) + lo) | x | lo);  // bit 4k+3 set iff nibble k == 0
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) m |= (uint32_t)((t >> (4 * k + 3)) & 1) << k;
  return m;
}

enum GpuSt : int { GS_OK = 0, GS_NONE = 1 };  // a stage allocated / fell through

// allocateByPartition (allocator_gpu.go:177-237) + selectPartitionByBinPack (:261-296) over the node's table.
// Returns the chosen minors, 0 = none; *why = the failure reason (MISSING/UNSUPPORTED/INSUFFICIENT).
__device__ uint32_t gpu_partition(const SoA& s, uint64_t ex0, const DevPod& p, int want, const GpuMasks& g,
                                  bool select, int* why) {
  if (!(ex0 & DSX_TABLE)) {
    *why = KE_REASON_DS_MISSING_PARTITION_TABLE;
    return 0;
  }
  const uint64_t* tab = s.pt + (int64_t)(ex0 >> DSX_TABLE_SHIFT) * PT_WORDS;
  const bool restricted = p.flags & PF_GPU_PART_RESTRICTED;
  int group = -1, nf = 0;
  uint32_t best = 0;
  int64_t best_score = 0;
  for (int e = 0; e < PT_SLOTS; e++) {
    const uint64_t w = tab[e];
    if (pt_gpus(w) == 0) break;
    if (pt_gpus(w) != want) continue;
    if (pt_group(w) != group) {
      if (nf > 0 || (restricted && group >= 0)) break;  // the first group with a feasible partition
      group = pt_group(w);
    }
    const uint32_t pm = pt_minors(w);
    if (pm & g.used) continue;
    if ((g.total & pm) != pm) continue;
    if (p.flags & PF_GPU_RING_BW) {
      const int64_t bw = (int64_t)tab[PT_SLOTS + e];
      if (bw == KE_ABSENT || p.ring_bw > bw) continue;
    }
    nf++;
    if (!select) return pm;
    // BinPackScore: the 8/4/2-GPU partitions of each lowest-score group that stay free
    const uint32_t alloc = g.used | pm;
    int64_t score = 0;
    for (int f = 0; f < PT_SLOTS; f++) {
      const uint64_t q = tab[f];
      const int c = pt_gpus(q);
      if (c == 0) break;
      if ((c != 8 && c != 4 && c != 2) || c < want || pt_group(q) != 0 || (pt_minors(q) & alloc)) continue;
      score += (int64_t)(c == 8 ? 10000 : c == 4 ? 100 : 1) * pt_score(q);
    }
    if (nf == 1 || score > best_score) {  // stable descending sort: first of the maxima
      best = pm;
      best_score = score;
    }
  }
  *why = group < 0 ? KE_REASON_DS_UNSUPPORTED_GPU_REQUESTS : KE_REASON_DS_INSUFFICIENT_PARTITIONED;
  return best;
}

// One scope's own candidates (allocator_gpu.go:393-450): the first `want` satisfied minors ascending, or
// for a shared GPU the satisfied minor of the highest scoreDevice (first on ties).
struct ScopeRes {
  uint32_t minors;  // 0 = no result
  int depth, cum;
  int64_t score;
};
__device__ __forceinline__ void scope_take(uint32_t mask, int level, int depth, int cum, int req_level, int want,
                                           bool shared, const GpuMasks& g, const int64_t* dscore, ScopeRes& r) {
  r.minors = 0;
  if (req_level > level) return;
  const uint32_t sm = g.sat & mask;
  if (!shared) {
    if (__builtin_popcount(sm) < want) return;
    uint32_t c = 0, rest = sm;
    for (int n = 0; n < want; n++) {
      c |= rest & (0u - rest);
      rest &= rest - 1;
    }
    r.minors = c;
    r.score = -1;
  } else {
    if (!sm) return;
    int bm = -1;
    int64_t bs = -1;
    for (uint32_t rest = sm; rest; rest &= rest - 1) {
      const int m = __builtin_ctz(rest);
      const int64_t sc = dscore ? dscore[m] : 0;  // no scorer (Filter, hints): every score 0
      if (sc > bs) bm = m, bs = sc;
    }
    r.minors = 1u << bm;
    r.score = bs;
  }
  r.depth = depth;
  r.cum = cum;
}
__device__ __forceinline__ bool scope_better(const ScopeRes& best, const ScopeRes& r, bool shared) {
  if (!best.minors) return true;
  if (best.depth < r.depth || (best.depth == r.depth && best.cum < r.cum)) return true;
  return shared && best.depth == r.depth && best.cum == r.cum && best.score < r.score;
}

// allocateFromScope over the tree Node > NUMANode > PCIe (allocator_gpu.go:357-451; tree from
// GetGPUTopologyScope, allocator_gpu_helper.go:202-263).  dscore: per-minor scoreDevice (shared GPUs).
__device__ uint32_t gpu_topology(const SoA& s, int64_t i, const DevPod& p, int want, const GpuMasks& g,
                                 const int64_t* dscore) {
  const bool shared = p.flags & PF_GPU_SHARED;
  const int req_level = scope_level(pod_scope(p.flags));
  if (__builtin_popcount(g.minors) < want) return 0;
  const uint64_t topo = dsmask(s, DSM_TOPO, i), pcie = dsmask(s, DSM_PCIE, i);
  const int cum0 = (g.minors & g.used) ? 1 : 0;
  ScopeRes best;
  best.minors = 0;
  for (int a = 0; a < DS_MINORS; a++) {  // NUMA scopes by NodeID
    const uint32_t nm = rank_mask(topo, a) & g.minors;
    if (!nm) break;
    if (__builtin_popcount(nm) < want) continue;
    const int cum1 = cum0 + ((nm & g.used) ? 1 : 0);
    int lo = DS_MINORS, hi = -1;  // this NUMA node's PCIe scope ranks
    for (uint32_t rest = nm; rest; rest &= rest - 1) {
      const int r = (int)((pcie >> (4 * __builtin_ctz(rest))) & 15u);
      lo = r < lo ? r : lo;
      hi = r > hi ? r : hi;
    }
    ScopeRes nb;
    nb.minors = 0;
    for (int b = lo; b <= hi; b++) {
      const uint32_t pm = rank_mask(pcie, b) & nm;
      if (__builtin_popcount(pm) < want) continue;
      ScopeRes r;
      scope_take(pm, 3, 3, cum1 + ((pm & g.used) ? 1 : 0), req_level, want, shared, g, dscore, r);
      if (r.minors && scope_better(nb, r, shared)) nb = r;
    }
    if (!nb.minors) scope_take(nm, 2, 2, cum1, req_level, want, shared, g, dscore, nb);
    if (nb.minors && scope_better(best, nb, shared)) best = nb;
  }
  if (!best.minors) scope_take(g.minors, 1, 1, cum0, req_level, want, shared, g, dscore, best);
  return best.minors;
}

// Filter feasibility of allocateFromScope: some scope at or below the required level has enough
// satisfied minors (a deeper result always exists when a shallower one does, so no tree search).
__device__ bool gpu_topology_feasible(const SoA& s, int64_t i, const DevPod& p, int want, const GpuMasks& g) {
  const bool shared = p.flags & PF_GPU_SHARED;
  const int need = shared ? 1 : want;
  const int req_level = scope_level(pod_scope(p.flags));
  if (__builtin_popcount(g.minors) < want) return false;
  if (req_level <= 1) return __builtin_popcount(g.sat) >= need;
  if (req_level > 3) return false;
  const uint64_t w = dsmask(s, req_level == 2 ? DSM_TOPO : DSM_PCIE, i);
  for (int r = 0; r < DS_MINORS; r++) {
    const uint32_t m = rank_mask(w, r) & g.minors;
    if (!m) break;
    if (__builtin_popcount(m) >= want && __builtin_popcount(g.sat & m) >= need) return true;
  }
  return false;
}

// defaultAllocateDevices' choice among the satisfiable instances `ok`: (scoreDevice desc, minor asc)
// (device_resources.go:171-208), the first `want`; without a scorer the lowest minors.
// `pref`: sortDeviceResourcesByMinor's preferred minors go first (device_resources.go:187-193)
__device__ __forceinline__ uint32_t default_pick(uint32_t ok, int want, const int64_t* score, uint32_t pref = 0) {
  uint32_t take = 0;
  for (int c = 0; c < want && ok; c++) {
    int best = -1;
    for (uint32_t r = (ok & pref) ? (ok & pref) : ok; r; r &= r - 1) {
      const int m = __builtin_ctz(r);
      if (best < 0 || (score && score[m] > score[best])) best = m;  // ascending minors: ties keep the lower
    }
    ok &= ~(1u << best);
    take |= 1u << best;
  }
  return take;
}

// GPUAllocator.Allocate after allocateByTemplate (refused at the boundary).  Returns the framework code
// (0 = allocated); with `select` *minors = the chosen minors (dscore: scoreDevice per minor, nullptr = no
// scorer), else only feasibility is decided.
__device__ int gpu_allocate(const SoA& s, int64_t i, uint64_t ex0, const DevPod& p, const GpuMasks& g, bool select,
                            const int64_t* dscore, uint32_t* minors, int* reason, int tmode = 0) {
  const int want = p.ds_cnt[KE_DEV_GPU];
  const bool shared = p.flags & PF_GPU_SHARED;
  const bool honor = (p.flags & PF_GPU_PART_SPEC) || (ex0 & DSX_HONOR);
  *minors = 0;
  if (tmode == 2) {  // allocateByTemplate: no candidate template of the node's GPU model (allocator_gpu.go:141-143)
    *reason = KE_REASON_DS_NO_MATCHED_TEMPLATE;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  if (!shared && tmode == 0) {  // allocateByPartition (one candidate template: generalAllocate only, :144-154)
    int why = 0;
    const uint32_t pm = gpu_partition(s, ex0, p, want, g, select, &why);
    if (pm) {
      *minors = pm;
      return 0;
    }
    if (honor) {
      *reason = why;
      return why == KE_REASON_DS_INSUFFICIENT_PARTITIONED ? KE_CODE_UNSCHEDULABLE : KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
  }
  const bool required = pod_scope(p.flags) != KE_SCOPE_NONE;  // generalAllocate -> allocateByDeviceTopology
  if (!(ex0 & DSX_TOPO) || (shared && want > 1)) {
    if (required) {
      *reason = (ex0 & DSX_TOPO) ? KE_REASON_DS_MULTI_SHARED_GPU : KE_REASON_DS_MISSING_TOPOLOGY_TREE;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
  } else {
    const bool ok = select ? (*minors = gpu_topology(s, i, p, want, g, dscore)) != 0
                           : gpu_topology_feasible(s, i, p, want, g);
    if (ok) return 0;
    *reason = required ? KE_REASON_DS_INSUFFICIENT_TOPOLOGY_SCOPED : KE_REASON_DS_INSUFFICIENT_GPU_TOPOLOGY;
    return KE_CODE_UNSCHEDULABLE;
  }
  if (__builtin_popcount(g.dflt) >= want) {  // defaultAllocateDevices
    if (select) *minors = default_pick(g.dflt, want, dscore, g.pref);
    return 0;
  }
  *reason = KE_REASON_DS_INSUFFICIENT_GPU;
  return KE_CODE_UNSCHEDULABLE;
}

// AutopilotAllocator.numaNodes (nil = off): the NUMA affinity the devices are restricted to
struct DsAff {
  bool on;
  uint32_t mask;  // NUMA ids
};
// filterNodeDevice's device choice (device_allocator.go:137-166): with numaNodes set, a device needs a
// topology whose NodeID is -1 or in the affinity (DSM_DNUMA codes: 0 none, 1 + NodeID, 9 = -1)
__device__ __forceinline__ uint32_t ds_allowed(const SoA& s, int64_t i, int t, DsAff a) {
  if (!a.on) return 0xFFFFu;
  const uint64_t w = dsmask(s, DSM_DNUMA + t, i);
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const uint32_t c = (uint32_t)(w >> (4 * q)) & 15u;
    const bool ok = c == DN_ANY || (c >= 1 && c <= 8 && ((a.mask >> (c - 1)) & 1u));
    m |= (uint32_t)ok << q;
  }
  return m;
}

// One device type of the filtered nodeDevice (nodeDevice.filter, device_cache.go:360-415): the type is kept
// when some instance has a free (over every instance) and some instance passes the affinity; the masks of
// the passing instances, their summed total / free' (scoreNode), scoreDevice per minor (`score`, optional),
// and the used hash over realUsed (allocator_gpu.go:59-70: the original used minors outside the refined
// total, the refined used' inside).
// rv (k_ds_views): a reservation view -- the preemptible beyond the row's (ds_load), a Restricted reservation's
// requiredDeviceResources (only the cap_in instances take part, their free capped: ds_instance_from), its required
// minors (defaultAllocateDevices takes only those) and preferred minors (g.pref)
__device__ __forceinline__ bool ds_type_view(const SoA& s, int64_t i, int t, const uint64_t msk[4], const DevPod& p,
                                             const KArgs& k, DsAff a, GpuMasks& g, int64_t (&tot)[3],
                                             int64_t (&fre)[3], int64_t* score, uint32_t sel = 0xFFFFu,
                                             const DsView* rv = nullptr) {
  const int nk = DS_NK[t];
  uint64_t ex = (msk[DSM_EXISTS] >> (16 * t)) & 0xFFFF;
  const uint32_t keep = (rv && rv->cap_in[t]) ? (uint32_t)rv->cap_in[t] : 0xFFFFu;  // requiredDeviceResources
  const uint32_t allowed = (uint32_t)ex & ds_allowed(s, i, t, a) & sel & keep;  // sel: a hint Selector's devices
  g.minors = (uint32_t)ex;
  g.total = g.used = g.sat = g.dflt = 0;
  g.pref = rv ? (uint32_t)rv->pref[t] : 0u;
  uint32_t orig_used = 0, used_p = 0, tot_m = 0, sat = 0, dflt = 0;
  bool present = false;
#pragma unroll
  for (int q = 0; q < 3; q++) tot[q] = fre[q] = 0;
  constexpr int GRP = KE_DS_GRP;  // instances whose words are loaded together
  while (ex) {
    int ms[GRP];
    DsRaw raw[GRP];
#pragma unroll
    for (int u = 0; u < GRP; u++) {
      ms[u] = ex ? __builtin_ctzll(ex) : -1;
      ex &= ex ? ex - 1 : 0;
    }
#pragma unroll
    for (int u = 0; u < GRP; u++)
      if (ms[u] >= 0) ds_load(s, i, t, ms[u], msk, raw[u], rv);
#pragma unroll
    for (int u = 0; u < GRP; u++) {
      const int m = ms[u];
      if (m < 0) continue;
      bool hu = false;
#pragma unroll
      for (int q = 0; q < 3; q++) hu = hu || (q < nk && ((msk[ds_hu_word(t)] >> ds_hu_bit(t, m, q)) & 1));
      orig_used |= (uint32_t)hu << m;
      if (!((keep >> m) & 1u)) continue;  // outside requiredDeviceResources: not in the filtered view at all
      DsInst d;
      ds_instance_from(raw[u], t, m, msk, d, rv);
      const bool fz = ds_free_zero(d);
      present = present || !fz;
      if (!((allowed >> m) & 1u)) continue;
      const bool leq = ds_leq(d, p, t), tnz = ds_total_nz(d);
      dflt |= (uint32_t)(!fz && leq) << m;
      sat |= (uint32_t)(leq && tnz) << m;
      tot_m |= (uint32_t)tnz << m;
      used_p |= (uint32_t)d.used_nz << m;
      int64_t tv[3], fv[3];
#pragma unroll
      for (int q = 0; q < 3; q++) {
        tv[q] = ((d.th >> q) & 1) ? d.tv[q] : 0;
        fv[q] = ((d.fh >> q) & 1) ? d.fv[q] : 0;
        tot[q] += tv[q];
        fre[q] += fv[q];
      }
      if (score) score[m] = ds_weighted(k, t, tv, fv, p);  // scoreDevice
    }
  }
  present = present && allowed != 0;
  if (rv && rv->rreq[t]) dflt &= (uint32_t)rv->rreq[t];  // required.Len() > 0 && !required.Has(minor)
  if (present) {
    g.dflt = dflt;
    g.sat = sat;
    g.total = tot_m;
    g.used = (orig_used & ~allowed) | used_p;
  } else {
    g.used = orig_used;
  }
  return present;
}

__device__ int hint_allocate(const SoA& s, int64_t i, const DevPod& p0, const KArgs& k, DsAff a, bool reserve,
                             bool scored, uint32_t* out, int8_t (*vf)[DS_MINORS], int* reason);
__device__ bool hint_score(const SoA& s, int64_t i, const DevPod& p0, const KArgs& k, DsAff a, int64_t* raw);
__device__ __forceinline__ uint64_t dsxw(const SoA& s, int w, int64_t i);

// AutopilotAllocator.Allocate (device_allocator.go:87-135) on the devices the affinity leaves: Prepare (a
// requested type without devices in the cache), then every requested type in the fixed order GPU, RDMA,
// FPGA.  *gpu = the GPU minors (no scorer) when `gpu` is given.
// H: the hint path is compiled in (hinted pods run only in kernels instantiated with H; elsewhere a hinted pod
// is an internal routing error: KERR_HINT_ROUTE, the call fails loudly).  Keeping hint_allocate / hint_score
// out of the batch kernels keeps them free of call frames and scratch.
__device__ __forceinline__ bool hint_misrouted(const SoA& s, const DevPod& p) {
  if (!(p.flags & PF_DS_HINT)) return false;
  __hip_atomic_fetch_or(s.kerr, KERR_HINT_ROUTE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}
template <bool H = true>
__device__ int ds_try_allocate(const SoA& s, int64_t i, const DevPod& p, const KArgs& k, DsAff a, uint32_t* gpu,
                               int* reason) {
  if constexpr (H) {
    if (p.flags & PF_DS_HINT) {  // Filter's trial allocation (no scorer, Prepare outside Reserve)
      uint32_t out[3];
      int8_t vf[2][DS_MINORS];
      const int st = hint_allocate(s, i, p, k, a, false, false, out, vf, reason);
      if (gpu) *gpu = st ? 0u : out[KE_DEV_GPU];
      return st;
    }
  } else if (hint_misrouted(s, p)) {
    *reason = KE_REASON_DS_INSUFFICIENT_GPU;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  uint64_t msk[4];
#pragma unroll
  for (int w = 0; w < 4; w++) msk[w] = dsmask(s, w, i);
  for (int t = 0; t < 3; t++)
    if (p.ds_cnt[t] && !((msk[DSM_EXISTS] >> (16 * t)) & 0xFFFF)) {
      *reason = KE_REASON_DS_INSUFFICIENT_GPU + t;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
  if (gpu) *gpu = 0;
#pragma unroll
  for (int t = 0; t < 3; t++) {
    if (!p.ds_cnt[t]) continue;
    GpuMasks g;
    int64_t tot[3], fre[3];
    ds_type_view(s, i, t, msk, p, k, a, g, tot, fre, nullptr);
    if (t == KE_DEV_GPU) {
      uint32_t take = 0;
      int why = 0;
      const int st = gpu_allocate(s, i, msk[DSM_EXISTS], p, g, gpu != nullptr, nullptr, &take, &why);
      if (st) {
        *reason = why;
        return st;
      }
      if (gpu) *gpu = take;
    } else if (__builtin_popcount(g.dflt) < p.ds_cnt[t]) {
      *reason = KE_REASON_DS_INSUFFICIENT_GPU + t;
      return KE_CODE_UNSCHEDULABLE;
    }
  }
  return 0;
}

// Filter (Prepare + per-type allocation feasibility) and raw Score of DeviceShare for a pod with PF_DS on
// a node with a cache entry.  `a`: the affinity the topology manager stored (Score and Reserve read it;
// Filter then passes: topology_hint.go Allocate already ran).  Types in the fixed order GPU, RDMA, FPGA.
template <bool H>
__device__ __forceinline__ void ds_filter_score(const SoA& s, int64_t i, const DevPod& p, const KArgs& k, EvalOut& o,
                                             bool stored, DsAff a) {
  if constexpr (H) {
    if (p.flags & PF_DS_HINT) {
      if (!stored) {
        int why = 0;
        const int st = ds_try_allocate<true>(s, i, p, k, DsAff{false, 0u}, nullptr, &why);
        if (st) {
          o.status = (uint8_t)st;
          o.reason = (uint8_t)why;
          return;
        }
      }
      int64_t raw = 0;
      hint_score(s, i, p, k, a, &raw);
      o.ds = (int16_t)raw;
      return;
    }
  } else if (hint_misrouted(s, p)) {
    o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    o.reason = KE_REASON_DS_INSUFFICIENT_GPU;
    return;
  }
  uint64_t msk[4];
#pragma unroll
  for (int w = 0; w < 4; w++) msk[w] = dsmask(s, w, i);
  for (int t = 0; t < 3; t++)  // AutopilotAllocator.Prepare: a requested type without devices
    if (p.ds_cnt[t] && !((msk[DSM_EXISTS] >> (16 * t)) & 0xFFFF)) {
      if (!stored) {
        o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
        o.reason = (uint8_t)(KE_REASON_DS_INSUFFICIENT_GPU + t);
      }
      return;  // Score: 0 with an error status
    }
  int64_t raw = 0;
  // GPUs on a node without partition table / honor policy / topology tree, for a pod without a partition
  // spec or required scope, go straight to defaultAllocateDevices: only its count is needed
  const bool gpu_default = !(msk[DSM_EXISTS] & (DSX_TOPO | DSX_TABLE | DSX_HONOR)) &&
                           !(p.flags & (PF_GPU_PART_SPEC | 7u * PF_GPU_SCOPE0));
#pragma unroll  // the type as a constant: key counts, field bases and mask bits fold per instance
  for (int t = 0; t < 3; t++) {
    if (!p.ds_cnt[t]) continue;
    GpuMasks g;
    int64_t tot[3], fre[3];
    const bool present = ds_type_view(s, i, t, msk, p, k, a, g, tot, fre, nullptr);
    if (!stored) {
      int st = 0, reason = KE_REASON_DS_INSUFFICIENT_GPU + t;
      if (t == KE_DEV_GPU && !gpu_default) {
        uint32_t unused;
        st = gpu_allocate(s, i, msk[DSM_EXISTS], p, g, false, nullptr, &unused, &reason);
      } else if (__builtin_popcount(g.dflt) < p.ds_cnt[t]) {  // defaultAllocateDevices: "Insufficient <type> devices"
        st = KE_CODE_UNSCHEDULABLE;
      }
      if (st) {
        o.status = (uint8_t)st;
        o.reason = (uint8_t)reason;
        return;
      }
    }
    if (present) raw += ds_weighted(k, t, tot, fre, p);  // resourceAllocationScorer.scoreNode
  }
  o.ds = (int16_t)raw;
}

// DeviceShare Reserve (plugin.go:426-492) on the devices the affinity leaves: per type the allocator's
// minors -- GPUs through GPUAllocator (partition, topology scope, then default), other types
// defaultAllocateDevices -- with the plugin's scorer.  The allocation (request + fillGPUTotalMem,
// devicehandler_gpu.go:98-133) is added to `used` in the SoA (updateCacheUsed).  Returns the minors mask
// (bit 16*type + minor).
// ro: a reservation-matched / -ignored pod's Reserve on the node as k_ds_views decided it (RsvOvr.ds_res 1: the
// minors of the nominated reservation's / the node's view; allocateWithNominatedReservation, reservation.go:368-415)
template <bool H>
__device__ __noinline__ uint64_t ds_reserve(const SoA& s, int64_t i, const DevPod& p, const KArgs& k, DsAff a,
                                            int8_t* vf_out = nullptr, const RsvOvr* ro = nullptr) {
  uint64_t msk[4], out = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) msk[w] = dsmask(s, w, i);
  uint32_t hout[3] = {0, 0, 0};
  int8_t hvf[2][DS_MINORS];
  const bool hinted = H && (p.flags & PF_DS_HINT) != 0;
  if constexpr (!H) {
    if (hint_misrouted(s, p)) return 0;
  }
  if (hinted) {  // the hinted allocation with the scorer in the Reserve phase (feasibility checked by the caller)
    for (int t = 0; t < 2; t++)
      for (int m = 0; m < DS_MINORS; m++) hvf[t][m] = -1;
    int why = 0;
    if (hint_allocate(s, i, p, k, a, true, true, hout, hvf, &why)) hout[0] = hout[1] = hout[2] = 0;
    if (vf_out)
      for (int t = 0; t < 2; t++)
        for (int m = 0; m < DS_MINORS; m++) vf_out[t * DS_MINORS + m] = ((hout[t + 1] >> m) & 1u) ? hvf[t][m] : (int8_t)-1;
  }
  for (int t = 0; t < 3; t++) {
    if (!p.ds_cnt[t]) continue;
    const int nk = DS_NK[t];
    uint32_t take = 0;
    if (hinted) {
      take = hout[t];
      for (uint32_t rest = take; t > 0 && rest; rest &= rest - 1) {  // updateVFAllocations: the VF is held
        const int m = __builtin_ctz(rest);
        if (hvf[t - 1][m] < 0) continue;
        const int w = DSX_VFFREE + 16 * (t - 1) + m;
        s.dsx[w * s.stride + i] = (int64_t)(dsxw(s, w, i) & ~(1ull << hvf[t - 1][m]));
      }
    } else if (ro && ro->ds_res) {
      take = ro->ds_res == 1 ? (uint32_t)((ro->ds_minors >> (16 * t)) & 0xFFFFu) : 0u;
    } else {
      int64_t score[DS_MINORS];
      GpuMasks g;
      int64_t tot[3], fre[3];
      ds_type_view(s, i, t, msk, p, k, a, g, tot, fre, score);
      if (t == KE_DEV_GPU) {
        int reason = 0;
        if (gpu_allocate(s, i, msk[DSM_EXISTS], p, g, true, score, &take, &reason) != 0) take = 0;  // passed Filter
      } else {
        take = default_pick(g.dflt, p.ds_cnt[t], score);
      }
    }
    for (uint32_t rest = take; rest; rest &= rest - 1) {
      const int best = __builtin_ctz(rest);
      out |= 1ull << (16 * t + best);
      int64_t alloc[3] = {0, 0, 0};
      bool has[3] = {false, false, false};
      if (t == KE_DEV_GPU) {
        const bool htm = (msk[DSM_GPU_HT] >> ds_ht_bit(0, best, 1)) & 1;
        const int64_t tm = htm ? dsf(s, DS_TBASE[0] + best * 3 + 1, i) : 0;
        if (p.flags & PF_DS_H_CORE) has[0] = true, alloc[0] = p.ds_req[0];
        if (p.flags & PF_DS_H_RATIO) {  // memoryRatioToBytes
          has[2] = true, alloc[2] = p.ds_req[2];
          has[1] = true, alloc[1] = p.ds_req[2] * tm / 100;
        } else if (p.flags & PF_DS_H_MEM) {  // memoryBytesToRatio: int64(float64(b)/float64(total)*100)
          has[1] = true, alloc[1] = p.ds_req[1];
          has[2] = true, alloc[2] = (int64_t)((double)p.ds_req[1] / (double)tm * 100.0);
        }
      } else {
        has[0] = true, alloc[0] = p.ds_req[2 + t];
      }
      for (int key = 0; key < nk; key++) {
        if (!has[key]) continue;
        const int w = ds_hu_word(t), b = ds_hu_bit(t, best, key);
        const int field = DS_UBASE[t] + best * nk + key;
        const int64_t prev = ((msk[w] >> b) & 1) ? dsf(s, field, i) : 0;
        s.ds[field * s.stride + i] = prev + alloc[key];  // quotav1.Add
        msk[w] |= 1ull << b;
      }
    }
  }
#pragma unroll
  for (int w = 1; w < 4; w++) s.dsm[w * s.stride + i] = msk[w];
  return out;
}

// ---- DeviceShare hints (deviceshare/utils.go:414-482, device_allocator.go:74-455) --------------
// Pods with DeviceAllocateHints / DeviceJointAllocate (PF_DS_HINT) are singleton batches; their DeviceShare
// Filter / Score / Reserve / NUMA hints run these functions on one lane.  The node's label-set ids, PCIe ranks,
// VF state and template model key live in the DSX SoA; the pod's Selector / VFSelector / template candidates
// are 256-bit sets over the context's interned ids (the host evaluates the selectors once per call).
__device__ __forceinline__ uint64_t dsxw(const SoA& s, int w, int64_t i) { return (uint64_t)s.dsx[w * s.stride + i]; }
__device__ __forceinline__ bool in256(const uint64_t* b, uint32_t x) { return (b[x >> 6] >> (x & 63u)) & 1u; }
__device__ __forceinline__ uint32_t dsx_byte(const SoA& s, int base, int64_t i, int t, int m) {
  return (uint32_t)(dsxw(s, base + 2 * t + (m >> 3), i) >> (8 * (m & 7))) & 0xFFu;
}
// filterNodeDevice's Selector (device_allocator.go:150-161): minors of type t whose labels it matches
__device__ uint32_t hint_sel_minors(const SoA& s, int64_t i, const DevPodHint& h, int t) {
  if (!(h.flags & (PH_SEL0 << t))) return 0xFFFFu;
  uint32_t m = 0;
  for (int q = 0; q < DS_MINORS; q++) m |= (uint32_t)in256(h.sel[t], dsx_byte(s, DSX_LBL, i, t, q)) << q;
  return m;
}
// allocateVF (device_allocator.go:426-455): the VF ranks of minor m (type 1..2) free and in a group the
// VFSelector matches; the lowest rank is the lowest BusID
__device__ uint64_t hint_vf_cand(const SoA& s, int64_t i, const DevPodHint& h, int t, int m) {
  const int d = 16 * (t - 1) + m;
  const uint64_t lw = dsxw(s, DSX_VFL + (d >> 1), i) >> (32 * (d & 1));
  uint64_t c = 0;
  for (int g = 0; g < KE_MAX_VF_GROUPS; g++) {
    const uint64_t vfs = dsxw(s, DSX_VFG + 4 * d + g, i);
    if (vfs && in256(h.vfsel[t], (uint32_t)(lw >> (8 * g)) & 0xFFu)) c |= vfs;
  }
  return c & dsxw(s, DSX_VFFREE + d, i);
}
// newPreferredPCIes (device_allocator.go:456-467): the PCIe ranks of `minors` (devices with a topology)
__device__ uint64_t hint_pcie_set(const SoA& s, int64_t i, int t, uint32_t minors) {
  uint64_t r = 0;
  for (uint32_t rest = minors; rest; rest &= rest - 1) {
    const uint32_t pr = dsx_byte(s, DSX_PCIE, i, t, __builtin_ctz(rest));
    if (pr < 64) r |= 1ull << pr;
  }
  return r;
}

// AutopilotAllocator.Prepare (device_allocator.go:74-94, calcRequestsAndCountByDeviceType :171-203): the types
// of requestsPerInstance (a joint pod's secondary types are left out outside Reserve on a node with well-planned
// secondary devices) and their desired counts (ApplyForAll: the node's devices matching the Selector,
// devicehandler_default.go:62-80), then mustAllocateVF's hasVirtualFunctions.  Types in the order GPU, RDMA, FPGA.
struct DsPrep {
  uint32_t inc;
  int want[3];
};
__device__ int hint_prepare(const SoA& s, int64_t i, const DevPod& p, const DevPodHint& h, uint64_t ex0, bool reserve,
                            DsPrep& pr, int* reason) {
  const uint64_t node = dsxw(s, DSX_NODE, i);
  pr.inc = 0;
  for (int t = 0; t < 3; t++) {
    pr.want[t] = 0;
    if (!p.ds_cnt[t]) continue;
    if (h.joint_n && t != h.joint[0] && (h.flags & PH_FITS_WELL_PLANNED) && (node & 1u) && !reserve) continue;
    const uint32_t ex = (uint32_t)(ex0 >> (16 * t)) & 0xFFFFu;
    int w = p.ds_cnt[t];
    if (w == DS_CNT_ALL) w = __builtin_popcount(ex & hint_sel_minors(s, i, h, t));
    if (!ex || w == 0) {
      *reason = KE_REASON_DS_INSUFFICIENT_GPU + t;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    pr.want[t] = w;
    pr.inc |= 1u << t;
  }
  for (int t = 1; t < 3; t++)
    if (((pr.inc >> t) & 1u) && (h.flags & (PH_VF0 << t)) && !((node >> t) & 1u)) {
      *reason = t == KE_DEV_RDMA ? KE_REASON_DS_INSUFFICIENT_RDMA_VF : KE_REASON_DS_INSUFFICIENT_FPGA_VF;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
  return 0;
}

// defaultAllocateDevices (device_allocator.go:352-424) with sortDeviceResourcesByPreferredPCIe (preferred PCIe
// first, then scoreDevice desc, minor asc) and one VF per device for a VF pod: up to max_count of `ok`.
__device__ int hint_default_pick(const SoA& s, int64_t i, const DevPodHint& h, int t, uint32_t ok, int max_count,
                                 uint64_t pref, const int64_t* score, uint32_t* take, int8_t* vf) {
  int8_t rank[DS_MINORS];
  uint32_t pf = 0;
  for (uint32_t rest = ok; rest; rest &= rest - 1) {
    const int m = __builtin_ctz(rest);
    rank[m] = -1;
    if (t > 0 && (h.flags & (PH_VF0 << t))) {
      const uint64_t c = hint_vf_cand(s, i, h, t, m);
      if (!c) {
        ok &= ~(1u << m);
        continue;
      }
      rank[m] = (int8_t)__builtin_ctzll(c);
    }
    const uint32_t pr = dsx_byte(s, DSX_PCIE, i, t, m);
    if (pr < 64 && ((pref >> pr) & 1u)) pf |= 1u << m;
  }
  *take = 0;
  int n = 0;
  for (; n < max_count && ok; n++) {
    int best = -1;
    for (uint32_t rest = ok; rest; rest &= rest - 1) {
      const int m = __builtin_ctz(rest);
      if (best < 0) {
        best = m;
        continue;
      }
      const bool pm = (pf >> m) & 1u, pb = (pf >> best) & 1u;
      const int64_t sm = score ? score[m] : 0, sb = score ? score[best] : 0;
      if (pm != pb ? pm : sm > sb) best = m;  // ascending minors: ties keep the lower
    }
    ok &= ~(1u << best);
    *take |= 1u << best;
    if (vf) vf[best] = rank[best];
  }
  return n;
}

// AutopilotAllocator.Allocate (device_allocator.go:96-138) for a hinted pod on the devices the NUMA affinity and
// the Selectors leave: Prepare, tryJointAllocate (:205-299: the primary type, then the secondary types preferring
// the primary's PCIe switches, SamePCIe validated) when more than one type is requested, then the other types.
// `scored`: the plugin's scorer (Reserve), else every score 0.  out[type] = minors, vf[type-1][minor] = VF ranks.
__device__ __noinline__ int hint_allocate(const SoA& s, int64_t i, const DevPod& p0, const KArgs& k, DsAff a,
                                          bool reserve, bool scored, uint32_t* out, int8_t (*vf)[DS_MINORS],
                                          int* reason) {
  const DevPodHint& h = s.ph[p0.ring_bw];
  DevPod p = p0;
  p.ring_bw = h.ring_bw;
  uint64_t msk[4];
  for (int w = 0; w < 4; w++) msk[w] = dsmask(s, w, i);
  for (int t = 0; t < 3; t++) out[t] = 0;
  DsPrep pr;
  int st = hint_prepare(s, i, p, h, msk[DSM_EXISTS], reserve, pr, reason);
  if (st) return st;
  int tmode = 0;
  if (h.flags & PH_TMPL) {
    const uint32_t key = (uint32_t)(dsxw(s, DSX_NODE, i) >> 8) & 0xFFu;
    tmode = in256(h.tmpl1, key) ? 1 : in256(h.tmplm, key) ? 0 : 2;
  }
  // allocateDevices (:320-350) of one type with its desired count and preferred PCIe ranks
  auto alloc_type = [&](int t, int desired, uint64_t pref) -> int {
    int max_count = desired;
    const int np = __builtin_popcountll(pref);
    if (np > max_count) max_count = np;
    if (desired == 0) desired = 1;
    if (max_count < desired) max_count = desired;
    GpuMasks g;
    int64_t tot[3], fre[3], score[DS_MINORS];
    ds_type_view(s, i, t, msk, p, k, a, g, tot, fre, scored ? score : nullptr, hint_sel_minors(s, i, h, t));
    if (t == KE_DEV_GPU) {
      DevPod q = p;
      q.ds_cnt[KE_DEV_GPU] = (uint8_t)desired;
      return gpu_allocate(s, i, msk[DSM_EXISTS], q, g, true, scored ? score : nullptr, &out[t], reason, tmode);
    }
    const int n = hint_default_pick(s, i, h, t, g.dflt, max_count, pref, scored ? score : nullptr, &out[t], vf[t - 1]);
    if (n < desired) {
      out[t] = 0;
      *reason = KE_REASON_DS_INSUFFICIENT_GPU + t;
      return KE_CODE_UNSCHEDULABLE;
    }
    return 0;
  };
  uint32_t done = 0;
  if (__builtin_popcount(pr.inc) > 1 && h.joint_n) {
    const int pt = h.joint[0];
    st = alloc_type(pt, pr.want[pt], 0);
    if (st) return st;
    if (!out[pt]) {
      *reason = KE_REASON_DS_INSUFFICIENT_PRIMARY;
      return KE_CODE_UNSCHEDULABLE;
    }
    done |= 1u << pt;
    const uint64_t pcie = hint_pcie_set(s, i, pt, out[pt]);
    const int npcie = __builtin_popcountll(pcie);
    for (int j = 1; j < h.joint_n; j++) {
      const int t = h.joint[j];
      int desired = pr.want[t];
      if ((h.flags & PH_JOINT_PCIE) && desired < npcie) desired = npcie;
      st = alloc_type(t, desired, pcie);
      if (st) return st;
      if (out[t]) done |= 1u << t;
    }
    if (h.flags & PH_JOINT_PCIE)
      for (int j = 1; j < h.joint_n; j++)
        if (hint_pcie_set(s, i, h.joint[j], out[h.joint[j]]) != pcie) {  // validateJointAllocation (:223-252)
          *reason = KE_REASON_DS_JOINT_VIOLATION;
          return KE_CODE_UNSCHEDULABLE;
        }
  }
  for (int t = 0; t < 3; t++) {
    if (!((pr.inc >> t) & 1u) || ((done >> t) & 1u)) continue;
    st = alloc_type(t, pr.want[t], 0);
    if (st) return st;
  }
  return 0;
}

// DeviceShare Score of a hinted pod (AutopilotAllocator.score, device_allocator.go:469-492): scoreNode over the
// types of requestsPerInstance on the Selector-filtered view; false when Prepare fails (Score 0 with an error)
__device__ __noinline__ bool hint_score(const SoA& s, int64_t i, const DevPod& p0, const KArgs& k, DsAff a,
                                        int64_t* raw) {
  const DevPodHint& h = s.ph[p0.ring_bw];
  uint64_t msk[4];
  for (int w = 0; w < 4; w++) msk[w] = dsmask(s, w, i);
  DsPrep pr;
  int why = 0;
  *raw = 0;
  if (hint_prepare(s, i, p0, h, msk[DSM_EXISTS], false, pr, &why)) return false;
  for (int t = 0; t < 3; t++) {
    if (!((pr.inc >> t) & 1u)) continue;
    GpuMasks g;
    int64_t tot[3], fre[3];
    if (ds_type_view(s, i, t, msk, p0, k, a, g, tot, fre, nullptr, hint_sel_minors(s, i, h, t)))
      *raw += ds_weighted(k, t, tot, fre, p0);
  }
  return true;
}

// ---- DeviceShare as a NUMA topology hint provider (topology_hint.go:38-236) ----------------------------
// The hints of one pod on one node, as sets over mask values of the device NUMA ids: F = the feasible
// masks, S = those whose GPU allocation equals the one on every device NUMA node (score 500); preferred =
// popcount == dmin; one identical list per requested device type (`copies`).
struct DsHints {
  uint8_t status, reason;  // a provider error (Admit reason)
  bool none;               // no preference (nil hints)
  uint8_t copies, dmin;
  uint64_t F[4], S[4];
};
__device__ __forceinline__ bool bit256(const uint64_t (&b)[4], uint32_t m) {
  const uint64_t w = m < 64 ? b[0] : m < 128 ? b[1] : m < 192 ? b[2] : b[3];
  return (w >> (m & 63u)) & 1u;
}
__device__ __forceinline__ void set256(uint64_t (&b)[4], uint32_t m) {
  const uint64_t bit = 1ull << (m & 63u);
  const int w = (int)(m >> 6);
#pragma unroll
  for (int q = 0; q < 4; q++) b[q] |= q == w ? bit : 0ull;
}

// generateTopologyHints (topology_hint.go:119-212) for a pod with PF_DS on a node with a device cache
template <bool H>
__device__ __noinline__ void ds_numa_hints(const SoA& s, int64_t i, const DevPod& p, const KArgs& k, DsHints& h) {
  h.status = h.reason = 0;
  h.none = true;
  h.copies = h.dmin = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) h.F[q] = h.S[q] = 0;
  if (k.flags & AF_DS_NO_NUMA) return;
  uint32_t ids = 0;  // numaTopology.nodes: NodeIDs of devices with a topology, -1 excluded
#pragma unroll
  for (int t = 0; t < 3; t++) {
    const uint64_t w = dsmask(s, DSM_DNUMA + t, i);
    for (int q = 0; q < 16; q++) {
      const uint32_t c = (uint32_t)(w >> (4 * q)) & 15u;
      if (c >= 1 && c <= 8) ids |= 1u << (c - 1);
    }
  }
  if (!ids) return;  // an empty hint map
  const uint64_t ex = dsmask(s, DSM_EXISTS, i);
  // Prepare fails on every mask alike; a hinted pod's requestsPerInstance / desired counts (hint_prepare)
  DsPrep pr;
  pr.inc = 0;
  for (int t = 0; t < 3; t++) {
    pr.want[t] = p.ds_cnt[t];
    pr.inc |= p.ds_cnt[t] ? 1u << t : 0u;
  }
  if constexpr (H) {
    if (p.flags & PF_DS_HINT) {
      int why = 0;
      const int st = hint_prepare(s, i, p, s.ph[p.ring_bw], ex, false, pr, &why);
      if (st) {
        h.status = (uint8_t)st;
        h.reason = (uint8_t)why;
        return;
      }
    }
  } else if (hint_misrouted(s, p)) {
    h.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    h.reason = KE_REASON_DS_INSUFFICIENT_GPU;
    return;
  }
  for (int t = 0; t < 3; t++)
    if (p.ds_cnt[t] && !((ex >> (16 * t)) & 0xFFFF)) {
      h.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      h.reason = (uint8_t)(KE_REASON_DS_INSUFFICIENT_GPU + t);
      return;
    }
  // one mask: calcTotalDevicesByNUMA's count check, then the trial allocation
  auto try_mask = [&](uint32_t m, uint32_t* gpu, int* why) -> int {
#pragma unroll
    for (int t = 0; t < 3; t++) {
      if (!((pr.inc >> t) & 1u)) continue;
      const uint64_t w = dsmask(s, DSM_DNUMA + t, i);
      int cnt = 0;
      for (int q = 0; q < 16; q++) {
        const uint32_t c = (uint32_t)(w >> (4 * q)) & 15u;
        cnt += (c >= 1 && c <= 8 && ((m >> (c - 1)) & 1u)) ? 1 : 0;
      }
      if (cnt > 0 && cnt < pr.want[t]) {
        *why = KE_REASON_DS_INSUFFICIENT_NUMA_SCOPED;
        return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      }
    }
    return ds_try_allocate<H>(s, i, p, k, DsAff{true, m}, gpu, why);
  };
  uint32_t best_gpu = 0;
  int why = 0;
  const int full = try_mask(ids, &best_gpu, &why);  // statusUnsatisfied / bestAllocationResult
  if (full) {
    h.status = (uint8_t)full;
    h.reason = (uint8_t)why;
    return;
  }
  int dmin = 9;
  for (int e = 0; e < 255; e++) {
    const uint32_t m = NUMA_ORDER[e];
    if (m & ~ids) continue;
    uint32_t gpu = 0;
    int w2 = 0;
    if (try_mask(m, &gpu, &w2)) continue;
    set256(h.F, m);
    if (gpu == best_gpu) set256(h.S, m);
    dmin = min(dmin, __popc(m));
  }
  h.none = false;
  h.dmin = (uint8_t)dmin;
  h.copies = (uint8_t)__builtin_popcount(pr.inc);  // minAffinitySize: the types of requestsPerInstance
}

// ---------------------------------------------------------------------------------------------
// NodeNUMAResource under a NUMA topology policy, non-cpuset pods: hint generation
// (resource_manager.go:525-622), topologymanager merge + admit (policy*.go), allocation by the merged
// hint (tryBestToDistributeEvenly, resource_manager.go:260-314) and the NUMA-scope score
// (scoring.go:101-119).  The zones of node i are read from the NUMA SoA once per lane into registers.
// ---------------------------------------------------------------------------------------------

struct NumaNode {
  uint32_t zm, ch[2], ak[2];  // zones present, capacity keys, allocated keys per resource (bit = NUMA id)
  uint32_t single, shared;    // NUMANodeSharedStatus single / shared (ids < number of zones)
  int64_t av[2][8];        // totalAvailable[r][id] (0 for absent zones / keys)
  uint32_t perm[2][8];     // perm[r][nb-1]: slot order of an nb-zone hint after the distribute sort
};

__device__ __forceinline__ int64_t pick8(const int64_t (&a)[8], int z) {
  int64_t v = a[0];
#pragma unroll
  for (int t = 1; t < 8; t++) v = z == t ? a[t] : v;
  return v;
}
__device__ __forceinline__ uint32_t pick8u(const uint32_t (&a)[8], int z) {
  uint32_t v = a[0];
#pragma unroll
  for (int t = 1; t < 8; t++) v = z == t ? a[t] : v;
  return v;
}
__device__ __forceinline__ int64_t numa_cap(const SoA& s, int64_t i, int z, int r) {
  return s.nf[(NUMA_CAP + 2 * z + r) * s.stride + i];
}
__device__ __forceinline__ int64_t numa_al(const SoA& s, int64_t i, const NumaNode& v, int z, int r) {
  const int64_t a = s.nf[(NUMA_AL + 2 * z + r) * s.stride + i];  // SubtractWithNonNegativeResult(allocated, {})
  return ((v.ak[r] >> z) & 1u) && a > 0 ? a : 0;
}

// The sort order of tryBestToDistributeEvenly for resource r: perm[r][nb-1] after insertion passes
// 1..nb-1 over av[r][0..7] (positions, the reference quirk below).
__device__ __forceinline__ void numa_perm(NumaNode& v, int r) {
  uint32_t st = 0x76543210u;
  v.perm[r][0] = st;
#pragma unroll
  for (int ii = 1; ii < 8; ii++) {
    bool go = true;
#pragma unroll
    for (int j = ii; j > 0; j--) {
      go = go && v.av[r][j] < v.av[r][j - 1];
      if (go) {
        const uint32_t a = (st >> (4 * j)) & 15u, b = (st >> (4 * (j - 1))) & 15u;
        st = (st & ~(0xFFu << (4 * (j - 1)))) | (a << (4 * (j - 1))) | (b << (4 * j));
      }
    }
    v.perm[r][ii] = st;
  }
}

// getAvailableNUMANodeResources (node_allocation.go:221-243) and the sort order of
// tryBestToDistributeEvenly: sort.Slice's insertion sort compares totalAvailable indexed by slice
// POSITION (a reference quirk), so the permutation of an nb-zone hint depends only on av[r][0..nb-1]
// and is the state after insertion passes 1..nb-1 — computed once for all hints.
__device__ __forceinline__ void numa_load(const SoA& s, int64_t i, NumaNode& v) {
  const uint64_t m = s.nm[i];
  v.zm = (uint32_t)m & 0xFFu;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    v.ch[r] = (uint32_t)(m >> (NUMA_M_CAP + 8 * r)) & 0xFFu;
    v.ak[r] = (uint32_t)(m >> (NUMA_M_AL + 8 * r)) & 0xFFu;
  }
  v.single = (uint32_t)(m >> NUMA_M_ST) & 0xFFu;
  v.shared = (uint32_t)(m >> (NUMA_M_ST + 8)) & 0xFFu;
#pragma unroll
  for (int z = 0; z < 8; z++)
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int64_t a = numa_cap(s, i, z, r) - numa_al(s, i, v, z, r);
      v.av[r][z] = a > 0 ? a : 0;
    }
#pragma unroll
  for (int r = 0; r < 2; r++) numa_perm(v, r);
}

// A pod that binds CPUs on the node (requestCPUBind): the cpuset part of ResourceOptions
// (getResourceOptions plugin.go:629-668, getCPUBindPolicy util.go:101-119) and, per NUMA id, the CPUs
// allocateCPUSet may take there (GetAvailableCPUs after a required policy's filter, CS_Z* words).
struct NumaCs {
  bool rcb, req, full;  // binding; required policy; required FullPCPUs
  int num, cpc, total;  // numCPUsNeeded, CPUs per core, the node's CPUs allocateCPUSet may take
  int64_t zlo, zhi;     // per NUMA id (16 bits each) the same in the zone
};
__device__ __forceinline__ int cs_zc(const NumaCs& c, int z) { return cs_zone(c.zlo, c.zhi, z); }

// the same from a CS_CNT word and the three CS_Z* word pairs (cs_fill's layout; a view's availability, k_numa_views)
__device__ __forceinline__ NumaCs numa_cs_words(int64_t cnt, const int64_t (&z6)[6], uint32_t nf, const DevPod& p) {
  NumaCs c;
  const int preq = pf_cpu_required(p.flags), nb = nf_cpu_bind(nf);
  int bind = preq;
  c.req = true;
  if (preq == XB_NONE) {
    if (nb == KE_NODE_CPU_BIND_SPREAD_BY_PCPUS) bind = XB_SPREAD;
    else if (nb == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY) bind = XB_FULL;
    else c.req = false, bind = pf_cpu_preferred(p.flags);
  }
  c.rcb = true;
  c.full = c.req && bind == XB_FULL;
  c.num = (int)(p.req[0] / 1000);
  c.cpc = cs_cpc(cnt);
  const int zw = !c.req ? 0 : (bind == XB_FULL ? 2 : 4);
  c.total = !c.req ? cs_all(cnt) : (bind == XB_FULL ? cs_full(cnt) : cs_spread(cnt));
  c.zlo = z6[zw];
  c.zhi = z6[zw + 1];
  return c;
}
__device__ __forceinline__ NumaCs numa_cs_load(const SoA& s, int64_t i, uint32_t nf, const DevPod& p) {
  NumaCs c;
  const int64_t cnt = s.cs[CS_CNT * s.stride + i];
  const int preq = pf_cpu_required(p.flags), nb = nf_cpu_bind(nf);
  int bind = preq;
  c.req = true;
  if (preq == XB_NONE) {
    if (nb == KE_NODE_CPU_BIND_SPREAD_BY_PCPUS) bind = XB_SPREAD;
    else if (nb == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY) bind = XB_FULL;
    else c.req = false, bind = pf_cpu_preferred(p.flags);
  }
  c.rcb = true;
  c.full = c.req && bind == XB_FULL;
  c.num = (int)(p.req[0] / 1000);
  c.cpc = cs_cpc(cnt);
  const int zw = !c.req ? CS_ZALL : (bind == XB_FULL ? CS_ZFULL : CS_ZSPREAD);
  c.total = !c.req ? cs_all(cnt) : (bind == XB_FULL ? cs_full(cnt) : cs_spread(cnt));
  c.zlo = s.cs[zw * s.stride + i];
  c.zhi = s.cs[(zw + 1) * s.stride + i];
  return c;
}

// trimNUMANodeResources (resource_manager.go:166-192): a required policy caps a zone's available cpu at
// its CPUs the policy leaves; the distribute order follows the trimmed availability.
__device__ __forceinline__ void numa_trim(NumaNode& v, const NumaCs& c) {
  if (!c.req) return;
#pragma unroll
  for (int z = 0; z < 8; z++) {
    const int64_t cap = (int64_t)cs_zc(c, z) * 1000;
    if (v.av[0][z] != 0 && cap < v.av[0][z]) v.av[0][z] = cap;
  }
  numa_perm(v, 0);
}

// q / d for 1 <= d <= 8 (Go int64 division): constant divisors become multiply-high sequences
__device__ __forceinline__ int64_t div_upto8(int64_t q, int d) {
  switch (d) {
    case 1: return q;
    case 2: return q / 2;
    case 3: return q / 3;
    case 4: return q / 4;
    case 5: return q / 5;
    case 6: return q / 6;
    case 7: return q / 7;
    default: return q / 8;
  }
}

// the resources tryBestToDistributeEvenly splits: keys of some zone's totalAvailable, requested
__device__ __forceinline__ bool numa_checked(const NumaNode& v, const DevPod& p, int r) {
  return ((v.ch[r] | v.ak[r]) & v.zm) != 0 && p.req[r] != 0;
}

// Necessary condition of a successful split (allocateRes never takes more than a zone has): every
// checked request fits in the summed availability of the mask's zones.
__device__ __forceinline__ bool numa_sum_fits(const NumaNode& v, uint32_t m, const DevPod& p) {
#pragma unroll
  for (int r = 0; r < 2; r++) {
    if (!numa_checked(v, p, r)) continue;
    int64_t sum = 0;
#pragma unroll
    for (int z = 0; z < 8; z++) sum += ((m >> z) & 1u) ? v.av[r][z] : 0;
    if (sum < p.req[r]) return false;
  }
  return true;
}

// Smallest hint size that can pass numa_sum_fits (sum of the largest zones), 9 if none: the masks
// below it are skipped without changing any hint list.
__device__ __forceinline__ int numa_min_size(const NumaNode& v, const DevPod& p) {
  int smin = 1;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    if (!numa_checked(v, p, r) || p.req[r] <= 0) continue;
    int64_t sum = 0;
    uint32_t used = 0;
    int s = 0;
    while (sum < p.req[r] && s < 8) {
      int64_t best = -1;
      int bz = 0;
#pragma unroll
      for (int z = 0; z < 8; z++)
        if (((v.zm & ~used) >> z & 1u) && v.av[r][z] > best) {
          best = v.av[r][z];
          bz = z;
        }
      if (best < 0) break;
      used |= 1u << bz;
      sum += best;
      s++;
    }
    if (sum < p.req[r]) return 9;
    smin = max(smin, s);
  }
  return smin;
}

// tryBestToDistributeEvenly over the zones of mask m: true when every requested resource is fully
// split; OUT: per resource the zones that received a non-zero amount and the amounts (out[r][id]).
// CS: the pod may bind CPUs (`cs` non-null): a binding pod splits whole CPUs (whole cores under a
// required FullPCPUs, splitQuantity :316-330) and its allocateCPUSet must then take numCPUsNeeded CPUs
// from the zones that received resources — per zone min(cpu/1000, its CPUs), whole cores each under a
// required FullPCPUs — or from the node when none did.  *split_ok: the split alone.
template <bool OUT, bool CS = false>
__device__ __forceinline__ bool numa_distribute(const NumaNode& v, uint32_t m, const DevPod& p, uint32_t* got_mask,
                                                int64_t (&out)[2][8], const NumaCs* cs = nullptr,
                                                bool* split_ok = nullptr) {
  if (!OUT && !numa_sum_fits(v, m, p)) {
    if (split_ok) *split_ok = false;
    return false;
  }
  const bool bind = CS && cs->rcb;
  const int nb = __popc(m);
  uint32_t bl = 0;  // zone ids of m, ascending, one nibble each
  for (uint32_t mm = m, t = 0; mm; mm &= mm - 1, t++) bl |= (uint32_t)(__ffs(mm) - 1) << (4 * t);
  bool ok = true, any = false, aligned = true;
  int taken = 0;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    if (!OUT && !ok) break;
    if (!numa_checked(v, p, r)) continue;  // resourceNamesByNUMA x requests
    const uint32_t perm = pick8u(v.perm[r], nb - 1);
    int64_t q = p.req[r];
    for (int t = 0; t < nb; t++) {
      const int z = (int)((bl >> (4 * ((perm >> (4 * t)) & 15u))) & 15u);
      const int64_t a = pick8(v.av[r], z);
      int64_t split = div_upto8(q, nb - t);  // splitQuantity
      if (bind && r == 0) {
        const int64_t val = q >= 0 ? (q + 999) / 1000 : -((-q + 999) / 1000);  // Quantity.Value()
        split = cs->full ? div_upto8(div_upto8(val, cs->cpc), nb - t) * cs->cpc * 1000 : div_upto8(val, nb - t) * 1000;
      }
      const int64_t got = a > split ? split : a;  // allocateRes
      q -= got;
      if (got != 0) {
        any = true;
        if (bind && r == 0) {
          const int k = min((int)(got / 1000), cs_zc(*cs, z));
          if (k > 0) {
            taken += k;
            if (k % cs->cpc) aligned = false;
          }
        }
      }
      if (OUT && got != 0) {
        got_mask[r] |= 1u << z;
#pragma unroll
        for (int zz = 0; zz < 8; zz++) out[r][zz] += zz == z ? got : 0;
      }
    }
    if (q != 0) ok = false;
  }
  if (split_ok) *split_ok = ok;
  if (bind) ok = ok && cs->total >= cs->num && (!any || (taken == cs->num && (!cs->full || aligned)));
  return ok;
}

// numa_distribute<false, CS>'s result (the hint loops' feasibility test).  A one-zone mask (the common
// case: hint sizes are tried smallest first) takes the split in one step — splitQuantity by 1, one zone,
// no sort — as straight-line code on its uniform zone id; larger masks run the general split.
// A binding pod whose cpu is split (requested, some zone keyed) must take numCPUsNeeded CPUs from the
// zones that received cpu (taken == num): the mask's zones need that many CPUs allocateCPUSet may take.
template <bool CS>
__device__ __forceinline__ bool numa_cs_counts_ok(const NumaNode& v, uint32_t m, const DevPod& p, const NumaCs* cs) {
  if (!CS || !cs->rcb || cs->num <= 0 || p.req[0] <= 0 || !numa_checked(v, p, 0)) return true;
  int n = 0;
#pragma unroll
  for (int z = 0; z < 8; z++) n += ((m >> z) & 1u) ? cs_zc(*cs, z) : 0;
  return n >= cs->num;
}

// The smallest mask size whose zones can hold numCPUsNeeded such CPUs (1 when the bound does not apply).
template <bool CS>
__device__ __forceinline__ int numa_cs_min_size(const NumaNode& v, const DevPod& p, const NumaCs* cs) {
  if (!CS || !cs->rcb || cs->num <= 0 || p.req[0] <= 0 || !numa_checked(v, p, 0)) return 1;
  int c[8];
#pragma unroll
  for (int z = 0; z < 8; z++) c[z] = ((v.zm >> z) & 1u) ? cs_zc(*cs, z) : 0;
  int sum = 0, k = 0;
  uint32_t used = 0;
  while (sum < cs->num && k < 8) {  // the largest counts first
    int best = -1, bz = 0;
#pragma unroll
    for (int z = 0; z < 8; z++)
      if (!((used >> z) & 1u) && c[z] > best) best = c[z], bz = z;
    used |= 1u << bz;
    sum += best;
    k++;
  }
  return sum >= cs->num ? k : 9;
}

// numa_distribute<false, CS> for a two-zone mask: the two split steps unrolled; the zones' availability
// read at their uniform ids, the distribute order (per lane) picks between them.
template <bool CS>
__device__ __forceinline__ bool numa_fits2(const NumaNode& v, uint32_t m, const DevPod& p, const NumaCs* cs) {
  if (!numa_sum_fits(v, m, p)) return false;
  const int za = __ffs(m) - 1, zb = 31 - __clz(m);
  const bool bind = CS && cs->rcb;
  bool ok = true, any = false, aligned = true;
  int taken = 0;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    if (!ok) break;
    if (!numa_checked(v, p, r)) continue;
    const uint32_t perm = v.perm[r][1];  // slots 0, 1 hold positions 0 / 1 of the mask's zones
    const int64_t aa = pick8(v.av[r], za), ab = pick8(v.av[r], zb);
    int64_t q = p.req[r];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const bool first_zone = ((perm >> (4 * t)) & 15u) == 0;
      const int z = first_zone ? za : zb;
      const int64_t a = first_zone ? aa : ab;
      int64_t split = t == 0 ? q / 2 : q;  // splitQuantity
      if (bind && r == 0) {
        const int val = (int)(q >= 0 ? (q + 999) / 1000 : -((-q + 999) / 1000));  // Quantity.Value()
        split = cs->full ? (int64_t)((val / cs->cpc) / (2 - t)) * cs->cpc * 1000 : (int64_t)(val / (2 - t)) * 1000;
      }
      const int64_t got = a > split ? split : a;  // allocateRes
      q -= got;
      if (got != 0) {
        any = true;
        if (bind && r == 0) {
          const int kk = min((int)(got / 1000), cs_zc(*cs, z));
          if (kk > 0) {
            taken += kk;
            if (kk % cs->cpc) aligned = false;
          }
        }
      }
    }
    if (q != 0) ok = false;
  }
  if (bind) ok = ok && cs->total >= cs->num && (!any || (taken == cs->num && (!cs->full || aligned)));
  return ok;
}

template <bool CS = false>
__device__ __forceinline__ bool numa_fits(const NumaNode& v, uint32_t m, const DevPod& p, const NumaCs* cs = nullptr) {
  if (!numa_cs_counts_ok<CS>(v, m, p, cs)) return false;
  const int nb = __popc(m);
  if (nb == 2 && (!CS || !cs->rcb || (p.req[0] >= 0 && p.req[0] < (1ll << 40)))) return numa_fits2<CS>(v, m, p, cs);
  if (nb != 1) {
    int64_t dummy[2][8];
    return numa_distribute<false, CS>(v, m, p, nullptr, dummy, cs);
  }
  const int z = __ffs(m) - 1;
  const bool bind = CS && cs->rcb;
  bool ok = true, any = false, aligned = true;
  int taken = 0;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    if (!ok) break;
    if (!numa_checked(v, p, r)) continue;
    const int64_t q = p.req[r];
    const int64_t a = pick8(v.av[r], z);
    int64_t split = q;
    if (bind && r == 0) {
      const int64_t val = q >= 0 ? (q + 999) / 1000 : -((-q + 999) / 1000);  // Quantity.Value()
      split = cs->full ? (val / cs->cpc) * cs->cpc * 1000 : val * 1000;
    }
    const int64_t got = a > split ? split : a;
    if (got != 0) {
      any = true;
      if (bind && r == 0) {
        const int k = min((int)(got / 1000), cs_zc(*cs, z));
        if (k > 0) {
          taken = k;
          if (k % cs->cpc) aligned = false;
        }
      }
    }
    if (q - got != 0) ok = false;
  }
  if (bind) ok = ok && cs->total >= cs->num && (!any || (taken == cs->num && (!cs->full || aligned)));
  return ok;
}

// resourceAllocationScorer.score with least/mostResourceScorer (scoring.go:210-226) in plain int64
__device__ __forceinline__ int32_t numa_scope_score(bool most, const int64_t (&req)[2], const int64_t (&alloc)[2],
                                                    const DevPod& p, const KArgs& k) {
  int64_t sc = 0, ws = 0;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int64_t w = k.w_numa[r], a = alloc[r];
    if (w == 0 || a == 0) continue;
    const int64_t rq = req[r] + p.req[r];
    int64_t x;
    if (most) x = ((rq > a ? a : rq) * 100) / a;
    else x = rq > a ? 0 : ((a - rq) * 100) / a;
    sc += x * w;
    ws += w;
  }
  return ws ? (int32_t)(sc / ws) : 0;
}

// the hint's score: numaScorer over requested = total - available of the hint's zones
__device__ __forceinline__ int32_t numa_hint_score(const SoA& s, int64_t i, const NumaNode& v, uint32_t m,
                                                   const DevPod& p, const KArgs& k) {
  int64_t tot[2] = {0, 0}, av[2] = {0, 0}, req[2];
#pragma unroll
  for (int z = 0; z < 8; z++)
    if ((m >> z) & 1u)
#pragma unroll
      for (int r = 0; r < 2; r++) {
        tot[r] += numa_cap(s, i, z, r);
        av[r] += v.av[r][z];
      }
#pragma unroll
  for (int r = 0; r < 2; r++) req[r] = tot[r] - av[r] > 0 ? tot[r] - av[r] : 0;
  return numa_scope_score((k.flags & AF_NUMA_HINT_MOST) != 0, req, tot, p, k);
}

__device__ __forceinline__ bool narrower(uint32_t a, uint32_t b) {  // bitmask.IsNarrowerThan
  const int ca = __popc(a), cb = __popc(b);
  return ca == cb ? a < b : ca < cb;
}

__device__ __forceinline__ bool in_list(const uint64_t (&l)[4], uint32_t m) {
  const uint64_t w = m < 64 ? l[0] : m < 128 ? l[1] : m < 192 ? l[2] : l[3];
  return (w >> (m & 63u)) & 1u;
}

struct NumaPick {
  uint8_t status, reason;
  uint32_t aff;  // merged NUMANodeAffinity, 0 = nil
};

// checkExclusivePolicy (policy.go:73-93) for a non-empty mask: with SingleNUMANodeExclusive Required a
// multi-zone hint may not touch a "single" zone and a one-zone hint may not be a "shared" zone.
__device__ __forceinline__ bool exclusive_ok(const NumaNode& v, uint32_t m, bool required) {
  if (!required) return true;
  return __popc(m) > 1 ? (m & v.single) == 0 : (m & v.shared) == 0;
}

// BestEffort without a preferred merged hint: mergeFilteredHints over the full provider lists
// (policy.go:198-260), every merged hint non-preferred; an unsatisfied result (or a resource without
// hints) -> any NUMA node.  Lists in resource-name order (cpu, memory): the reference ranges over a Go
// map here, so its order — and with it this tie-break — is not deterministic.
// ps: the requests the hint scores see (options.requests; a binding pod's cpu amplified)
template <bool CS = false>
__device__ __forceinline__ uint32_t numa_best_effort_fallback(const SoA& s, int64_t i, const NumaNode& v, const DevPod& p,
                                                           const KArgs& k, const bool (&present)[2],
                                                           const uint32_t (&lack)[2], const NumaCs* cs = nullptr,
                                                           const DevPod* ps = nullptr) {
  const DevPod& sp = CS ? *ps : p;
  uint64_t L[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int e = 0; e < 255; e++) {
    const uint32_t m = NUMA_ORDER[e];
    if (m & ~v.zm) continue;
    const bool in0 = present[0] && !(m & lack[0]), in1 = present[1] && !(m & lack[1]);
    if (!in0 && !in1) continue;
    if (!numa_fits<CS>(v, m, p, cs)) continue;
    const uint64_t bit = 1ull << (m & 63u);
    const int w = (int)(m >> 6);
#pragma unroll
    for (int ww = 0; ww < 4; ww++) {
      if (in0 && w == ww) L[0][ww] |= bit;
      if (in1 && w == ww) L[1][ww] |= bit;
    }
  }
  const bool e0 = !(L[0][0] | L[0][1] | L[0][2] | L[0][3]), e1 = !(L[1][0] | L[1][1] | L[1][2] | L[1][3]);
  if ((present[0] && e0) || (present[1] && e1)) return v.zm;  // filterProvidersHints reasons
  uint32_t best = v.zm;
  int32_t bsc = 0;
  bool bun = false;
  if (!(present[0] && present[1])) {  // one list (+ DeviceShare's any-NUMA hint): merged = the hint
    const int r = present[0] ? 0 : 1;
    for (int e = 0; e < 255; e++) {
      const uint32_t m = NUMA_ORDER[e];
      if ((m & ~v.zm) || !in_list(L[r], m)) continue;
      const int32_t sc = numa_hint_score(s, i, v, m, sp, k);
      if (narrower(m, best) || (__popc(m) == __popc(best) && sc > bsc)) {
        best = m;
        bsc = sc;
      }
    }
    return best;
  }
  for (int e1i = 0; e1i < 255; e1i++) {
    const uint32_t m1 = NUMA_ORDER[e1i];
    if ((m1 & ~v.zm) || !in_list(L[0], m1)) continue;
    int32_t s1 = -1;
    for (int e2i = 0; e2i < 255; e2i++) {
      const uint32_t m2 = NUMA_ORDER[e2i];
      if ((m2 & ~v.zm) || !in_list(L[1], m2)) continue;
      const uint32_t mg = m1 & m2;
      if (!mg) continue;
      const bool un = max(__popc(m1), __popc(m2)) != __popc(mg);
      int32_t sc = 0;
      if (m1 == mg) {
        if (s1 < 0) s1 = numa_hint_score(s, i, v, m1, sp, k);
        sc += s1;
      }
      if (m2 == mg) sc += numa_hint_score(s, i, v, m2, sp, k);
      if (narrower(mg, best) || (__popc(mg) == __popc(best) && sc > bsc)) {
        best = mg;
        bsc = sc;
        bun = un;
      }
    }
  }
  return bun ? v.zm : best;
}

constexpr uint8_t STATUS_DEFERRED = 0xFF;  // pair left to k_numa_fallback
constexpr int NUMA_DEFER_SIZE = 1;         // largest hint size the batch eval's lanes search
constexpr uint32_t NFB_FOUND = 1, NFB_FAIL = 2, NFB_BEST_EFFORT = 3;  // k_numa_fallback's merge outcome

// generateResourceHints' resource lists: present[r] = the pod requests r and some zone has the key;
// lack[r] = numaNodesLackResource (zones without r available)
__device__ __forceinline__ void numa_present_lack(const NumaNode& v, const DevPod& p, bool (&present)[2],
                                                  uint32_t (&lack)[2]) {
#pragma unroll
  for (int r = 0; r < 2; r++) {
    present[r] = p.req[r] != 0 && (v.ch[r] & v.zm) != 0;
    uint32_t l = 0;
    if (v.ch[r] & v.zm)
#pragma unroll
      for (int z = 0; z < 8; z++)
        if (((v.zm >> z) & 1u) && (!(((v.ch[r] | v.ak[r]) >> z) & 1u) || v.av[r][z] == 0)) l |= 1u << z;
    lack[r] = l;
  }
}

// mergeFilteredHints over every permutation of the provider lists (policy.go:198-299) when no merged hint
// is preferred (ke_merge.h): up to MERGE_BUDGET permutations are walked in order, beyond it merge_exact
// computes the same fold without enumerating them.  DeviceShare lists score 500 where their hint carries it
// (dh.S), the NodeNUMAResource lists numa_hint_score.
__device__ __noinline__ uint32_t merge_all_permutations(const SoA& s, int64_t i, const NumaNode& v, const DevPod& sp,
                                                         const KArgs& k, const MergeLists& L, const DsHints& dh,
                                                         bool excl) {
  (void)excl;  // every merged hint is non-preferred here: the exclusive check changes nothing
  int64_t total = 1;
  for (int l = 0; l < L.n; l++) total *= L.len[l];
  auto sc = [&](int l, uint32_t m) -> int32_t {
    return L.ds[l] ? (bit256(dh.S, m) ? 500 : 0) : numa_hint_score(s, i, v, m, sp, k);
  };
  if (total <= MERGE_BUDGET) return merge_walk(L, v.zm, total, sc);
  return merge_exact(L, v.zm, sc);
}

// topologymanager Admit with DeviceShare's hint lists (topology_hint.go:38-212, manager.go:64-129): the
// provider lists in order [cpu, memory] (NodeNUMAResource; one preferred any-NUMA hint when it has none),
// then `copies` identical DeviceShare lists.  A merged hint is preferred only on the diagonal (every list
// holds the mask, preferred), so the preferred candidates are scanned in IterateBitMasks order with
// mergeFilteredHints' replacement rule; without one, BestEffort folds every permutation.  The NUMA
// allocation on the result follows; DeviceShare's Allocate is the caller's.
template <bool CS>
__device__ __noinline__ NumaPick numa_admit_ds(const SoA& s, int64_t i, int policy, const NumaNode& v, const DevPod& p,
                                               const KArgs& k, const NumaCs* cs, const DevPod* ps, const DsHints& dh) {
  NumaPick o{KE_CODE_SUCCESS, KE_REASON_NONE, 0u};
  const DevPod& sp = CS ? *ps : p;
  if (dh.status) {  // the provider's error is an Admit reason (manager.go:110-125)
    o.status = KE_CODE_UNSCHEDULABLE;
    o.reason = dh.reason;
    return o;
  }
  const bool excl = (p.flags & PF_NUMA_EXCL_REQ) != 0;
  const uint32_t all = v.zm;
  bool present[2];
  uint32_t lack[2];
  numa_present_lack(v, p, present, lack);
  const int R = (int)present[0] + (int)present[1];
  uint64_t L[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  int minr[2] = {9, 9};
  for (int e = 0; e < 255; e++) {  // generateResourceHints: the feasible masks per resource
    const uint32_t m = NUMA_ORDER[e];
    if (m & ~all) continue;
    const bool in0 = present[0] && !(m & lack[0]), in1 = present[1] && !(m & lack[1]);
    if (!in0 && !in1) continue;
    if (!numa_fits<CS>(v, m, p, cs)) continue;
    if (in0) set256(L[0], m), minr[0] = min(minr[0], __popc(m));
    if (in1) set256(L[1], m), minr[1] = min(minr[1], __popc(m));
  }
  const bool single = policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE, restricted = policy == KE_NUMA_POLICY_RESTRICTED;
  const bool empty0 = present[0] && minr[0] == 9, empty1 = present[1] && minr[1] == 9;  // filterProvidersHints reasons
  const int copies = dh.copies;
  uint32_t best = all;
  int32_t bsc = 0;
  bool found = false, bun = false;  // bun: the best merged hint is narrower than its masks (unsatisfied)
  if (!empty0 && !empty1) {
    for (int e = 0; e < 255; e++) {
      const uint32_t m = NUMA_ORDER[e];
      if (!bit256(dh.F, m) || __popc(m) != dh.dmin) continue;  // DeviceShare: preferred = the minimal size
      if (single && __popc(m) != 1) continue;                   // filterSingleNumaHints
      bool cand = true;
#pragma unroll
      for (int r = 0; r < 2; r++)
        if (present[r]) cand = cand && !(m & ~all) && bit256(L[r], m) && (restricted || (int)__popc(m) == minr[r]);
      if (!cand) continue;
      const uint32_t mg = m & all;  // mergePermutation ANDs the default affinity
      if (!mg || !exclusive_ok(v, mg, excl)) continue;
      const int32_t sc = (R ? R * numa_hint_score(s, i, v, m, sp, k) : 0) + (mg == m && bit256(dh.S, m) ? 500 * copies : 0);
      if (!found || narrower(mg, best) || (__popc(mg) == __popc(best) && sc > bsc)) {
        best = mg;
        bsc = sc;
        found = true;
        bun = mg != m;  // a hint on NUMA ids without a zone: maxNUMANodeNum != merged count
      }
    }
  }
  if (found && bun && policy == KE_NUMA_POLICY_BEST_EFFORT) best = all;  // policy_best_effort.go: unsatisfied -> any
  if (!found) {
    if (policy != KE_NUMA_POLICY_BEST_EFFORT) {
      o.status = KE_CODE_UNSCHEDULABLE;
      o.reason = KE_REASON_NUMA_HINT_UNALIGNED;
      return o;
    }
    MergeLists ml;
    ml.n = 0;
    auto add_set = [&](const uint64_t (&b)[4], bool ds) {
      int n = 0;
      for (int e = 0; e < 255; e++)
        if (bit256(b, NUMA_ORDER[e])) ml.m[ml.n][n++] = NUMA_ORDER[e];
      ml.len[ml.n] = n;
      ml.ds[ml.n] = ds;
      ml.unsat[ml.n] = 0;
      ml.n++;
    };
    if (R == 0) {
      ml.m[0][0] = 0, ml.len[0] = 1, ml.ds[0] = 0, ml.unsat[0] = 0, ml.n = 1;
    } else {
      for (int r = 0; r < 2; r++) {
        if (!present[r]) continue;
        if (r == 0 ? empty0 : empty1) {
          ml.m[ml.n][0] = 0, ml.len[ml.n] = 1, ml.ds[ml.n] = 0, ml.unsat[ml.n] = 1, ml.n++;
        } else {
          add_set(L[r], false);
        }
      }
    }
    for (int c = 0; c < copies; c++) add_set(dh.F, true);
    best = merge_all_permutations(s, i, v, sp, k, ml, dh, excl);
  }
  o.aff = (single && best == all) ? 0u : best;
  // topologymanager allocateResources -> NodeNUMAResource.Allocate (tryAllocateFromNode with the hint)
  int64_t dummy2[2][8];
  bool split = true;
  const bool fits = o.aff ? numa_distribute<false, CS>(v, o.aff, p, nullptr, dummy2, cs, &split)
                          : (!CS || cs->total >= cs->num);
  if (!fits) {
    o.status = KE_CODE_UNSCHEDULABLE;
    o.reason = split ? KE_REASON_NUMA_INSUFFICIENT_CPUS : KE_REASON_NUMA_INSUFFICIENT_RESOURCES;
  }
  return o;
}

// FilterByNUMANode + RunNUMATopologyManagerAdmit for a pod whose requests are not all zero, under
// the merged topology `policy` (node / pod, util.go:58-74).  DEFER: a BestEffort pair without a
// preferred merged hint returns STATUS_DEFERRED instead of running the full merge here (one lane
// needing it would hold its whole wavefront; k_numa_fallback runs those pairs compacted).
// The deferral also caps the in-lane search at hints of NUMA_DEFER_SIZE zones: a pair whose lists need
// larger hints (a few per wave, but the wave waits for its slowest lane) goes to k_numa_fallback, whose
// wave lists every mask of the pair at once.
// FB_AFF: k_numa_fallback computed the Admit's merge for the pair: `fb_aff` = FB_* kind << 8 | affinity.
// CS: a binding pod (`cs`, `ps` = its amplified requests for the hint scores): every allocation check
// includes allocateCPUSet's take, a nil affinity the node-wide one.
template <bool DEFER, bool FB_AFF = false, bool CS = false>
__device__ __forceinline__ NumaPick numa_admit(const SoA& s, int64_t i, uint32_t nf, int policy, const NumaNode& v,
                                               const DevPod& p, const KArgs& k, uint32_t fb_aff = 0,
                                               const NumaCs* cs = nullptr, const DevPod* ps = nullptr,
                                               const DsHints* dh = nullptr) {
  NumaPick o{KE_CODE_SUCCESS, KE_REASON_NONE, 0u};
  const DevPod& sp = CS ? *ps : p;
  // Allocate on the chosen affinity (topologymanager allocateResources -> tryAllocateFromNode)
  auto allocate_on = [&](uint32_t aff) {
    int64_t dummy2[2][8];
    bool split = true;
    const bool fits = aff ? numa_distribute<false, CS>(v, aff, p, nullptr, dummy2, cs, &split)
                          : (!CS || cs->total >= cs->num);
    if (!fits) {
      o.status = KE_CODE_UNSCHEDULABLE;
      o.reason = split ? KE_REASON_NUMA_INSUFFICIENT_CPUS : KE_REASON_NUMA_INSUFFICIENT_RESOURCES;
    }
  };
  const bool excl = (p.flags & PF_NUMA_EXCL_REQ) != 0;
  if (v.zm == 0) {  // topology_hint.go:31-41
    o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    o.reason = KE_REASON_NUMA_MISSING_RESOURCES;
    return o;
  }
  if (nf & NF_NUMA_OPT_ERR) {  // GetPodTopologyHints error -> admit reasons
    o.status = KE_CODE_UNSCHEDULABLE;
    o.reason = KE_REASON_NUMA_HINT_UNALIGNED;
    return o;
  }
  if (dh && (dh->status || !dh->none)) return numa_admit_ds<CS>(s, i, policy, v, p, k, cs, ps, *dh);
  const uint32_t all = v.zm;
  bool present[2];
  uint32_t lack[2];
  numa_present_lack(v, p, present, lack);
  const int R = (int)present[0] + (int)present[1];
  if (R == 0) {  // no hints: one preferred any-NUMA hint per provider -> merged = all zones
    if (policy != KE_NUMA_POLICY_BEST_EFFORT && !exclusive_ok(v, all, excl)) {
      o.status = KE_CODE_UNSCHEDULABLE;
      o.reason = KE_REASON_NUMA_HINT_UNALIGNED;
      return o;
    }
    o.aff = policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE ? 0u : all;  // best == all -> nil affinity
    allocate_on(o.aff);
    return o;
  }
  if (FB_AFF) {  // the merge k_numa_fallback ran over the pair's full lists
    const uint32_t kind = fb_aff >> 8, aff = fb_aff & 0xFFu;
    if (kind == NFB_FAIL) {
      o.status = KE_CODE_UNSCHEDULABLE;
      o.reason = KE_REASON_NUMA_HINT_UNALIGNED;
      return o;
    }
    o.aff = aff;
    if (kind == NFB_FOUND) {
      if (CS && !o.aff) allocate_on(0u);
    } else {
      allocate_on(o.aff);
    }
    return o;
  }
  // Preferred merged hints are the masks in every present list that are preferred in each (of the
  // list's minimum size, or any size under Restricted); scanned in IterateBitMasks order with
  // mergeFilteredHints' replacement rule (narrower, else same size and higher score).
  int minr[2] = {0, 0};
  uint32_t best = 0;
  int32_t bsc = 0;
  bool found = false, stop = false;
  const int smax = policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE ? 1 : __popc(all);
  for (int sz = max(numa_min_size(v, p), numa_cs_min_size<CS>(v, p, cs)); sz <= smax && !stop; sz++) {
    if (DEFER && sz > NUMA_DEFER_SIZE) {
      o.status = STATUS_DEFERRED;
      return o;
    }
    const bool first0 = minr[0] == 0, first1 = minr[1] == 0;
    for (int e = NUMA_OFF[sz]; e < NUMA_OFF[sz + 1]; e++) {
      const uint32_t m = NUMA_ORDER[e];
      if (m & ~all) continue;
      const bool in0 = present[0] && !(m & lack[0]), in1 = present[1] && !(m & lack[1]);
      if (!in0 && !in1) continue;
      if (!numa_fits<CS>(v, m, p, cs)) continue;
      if (in0 && !minr[0]) minr[0] = sz;
      if (in1 && !minr[1]) minr[1] = sz;
      bool cand = (!present[0] || in0) && (!present[1] || in1);
      if (policy != KE_NUMA_POLICY_RESTRICTED) cand = cand && (!present[0] || first0) && (!present[1] || first1);
      if (!cand || !exclusive_ok(v, m, excl)) continue;
      const int32_t sc = R * numa_hint_score(s, i, v, m, sp, k);
      if (!found || narrower(m, best) || (__popc(m) == __popc(best) && sc > bsc)) {
        best = m;
        bsc = sc;
        found = true;
      }
    }
    stop = policy == KE_NUMA_POLICY_RESTRICTED ? found : ((!present[0] || minr[0]) && (!present[1] || minr[1]));
  }
  if (found) {
    o.aff = (policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE && best == all) ? 0u : best;
    if (CS && !o.aff) allocate_on(0u);  // a hint passed its allocation already
    return o;
  }
  if (policy != KE_NUMA_POLICY_BEST_EFFORT) {
    o.status = KE_CODE_UNSCHEDULABLE;
    o.reason = KE_REASON_NUMA_HINT_UNALIGNED;
    return o;
  }
  if (DEFER) {
    o.status = STATUS_DEFERRED;
    return o;
  }
  o.aff = numa_best_effort_fallback<CS>(s, i, v, p, k, present, lack, cs, ps);
  allocate_on(o.aff);
  return o;
}

// Score under a NUMA policy (scoring.go:101-119): the allocation on the affinity, NUMA-scope
// allocatable / requested of the zones it touches, else the node's.
// CS: a binding pod's requested cpu is Amplify(the node's allocated CPUs * 1000) (scoring.go:179-185),
// scored with its amplified requests `ps`.
template <bool CS = false>
__device__ __forceinline__ int32_t numa_policy_score(const SoA& s, int64_t i, const NumaNode& v, uint32_t aff,
                                                     const DevPod& p, const KArgs& k, const NodeRegs& n,
                                                     const NumaCs* cs = nullptr, const DevPod* ps = nullptr) {
  int64_t out[2][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0}};
  uint32_t got[2] = {0, 0};
  if (aff) numa_distribute<true, CS>(v, aff, p, got, out, cs);
  const uint32_t zs = got[0] | got[1];
  int64_t req[2] = {n.nreq[0], n.nreq[1]}, alloc[2] = {n.nalloc[0], n.nalloc[1]};
  if (zs) {
    req[0] = req[1] = alloc[0] = alloc[1] = 0;
#pragma unroll
    for (int z = 0; z < 8; z++)
      if ((zs >> z) & 1u)
#pragma unroll
        for (int r = 0; r < 2; r++) {
          alloc[r] += numa_cap(s, i, z, r);
          req[r] += numa_al(s, i, v, z, r);
        }
  }
  if (CS) req[0] = amplify_bits(n.csm, s.cs[CS_RS * s.stride + i]);
  return numa_scope_score((k.flags & AF_NUMA_MOST) != 0, req, alloc, CS ? *ps : p, k);
}

// NodeNUMAResource Reserve of a pod in a CPU batch on a NUMA-policy node: the allocation (`dist`) joins
// the zones' entries (quotav1.Add keys, numa_reserve); under a cpu ratio > 1 an entry's cpu is the
// allocated cpu - cpusets + Amplify(cpusets) of its zone (node_allocation.go:221-243), re-adjusted for
// the zones whose cpuset count changed (`cs_old` -> `cs_new`, CPUs per NUMA id); the cpuset's NUMA ids
// become single / shared (node_allocation.go:111-156 and GetAllNUMANodeStatus).
__device__ void numa_reserve_cs(const SoA& s, int64_t i, uint32_t nf, const NumaNode& v, const uint32_t (&got)[2],
                                const int64_t (&dist)[2][8], const int (&cs_old)[8], const int (&cs_new)[8],
                                uint32_t used, int n_used, int64_t* out16) {
  // the cpuset counts come from CPU tables; without the CPU SoA they are zero (a zone without an
  // allocation entry holds no cpusets, ke_node_numa_set) and the ratio is never read
  if (out16)
    for (int z = 0; z < 8; z++)
      for (int r = 0; r < 2; r++) out16[2 * z + r] = dist[r][z];
  // resourceManager.Update records the allocation only on a node with a valid CPU topology
  // (resource_manager.go:461-466); the pod still carries it (state.allocation -> PreBind)
  if (!(nf & NF_CPUS_VALID)) return;
  const int64_t ratio = s.cs ? s.cs[CS_RS * s.stride + i] : 0;
  for (int z = 0; z < 8; z++) {
    for (int r = 0; r < 2; r++) {
      int64_t* f = s.nf + (NUMA_AL + 2 * z + r) * s.stride + i;
      const bool entry_before = (v.ak[0] >> z) & 1u, entry_after = entry_before || (((got[0] | got[1]) >> z) & 1u);
      if (r == 0 && (nf & NF_NUMA_AL_AMP)) {
        if (!entry_after) continue;
        const int64_t o = (int64_t)cs_old[z] * 1000, n = (int64_t)cs_new[z] * 1000;
        const int64_t raw = entry_before ? *f + o - amplify_bits(o, ratio) : 0;
        *f = raw + dist[0][z] - n + amplify_bits(n, ratio);
      } else if ((got[r] >> z) & 1u) {
        *f = (((v.ak[r] >> z) & 1u) ? *f : 0) + dist[r][z];
      }
    }
  }
  uint32_t ak0 = v.ak[0] | got[0];
  if (nf & NF_NUMA_AL_AMP) ak0 |= got[1];
  const uint32_t ak1 = v.ak[1] | got[1];
  uint32_t single = v.single, shared = v.shared;
  const uint32_t tracked = v.zm & ((1u << __popc(v.zm)) - 1u);  // ids < len(numaNodes) with a zone
  for (int z = 0; z < 8; z++) {
    if (!((used >> z) & 1u) || !((tracked >> z) & 1u)) continue;
    if (n_used > 1 || ((shared >> z) & 1u)) shared |= 1u << z, single &= ~(1u << z);
    else single |= 1u << z;
  }
  uint64_t m = s.nm[i];
  m |= ((uint64_t)ak0 << NUMA_M_AL) | ((uint64_t)ak1 << (NUMA_M_AL + 8));
  m &= ~((uint64_t)0xFFFF << NUMA_M_ST);
  m |= ((uint64_t)single << NUMA_M_ST) | ((uint64_t)shared << (NUMA_M_ST + 8));
  s.nm[i] = m;
}

// allocated CPUs per NUMA id of node i from its CPU table (zeros without the CPU SoA)
__device__ __forceinline__ void zone_cpusets(const SoA& s, int64_t i, int (&cs)[8]) {
#pragma unroll
  for (int z = 0; z < 8; z++) cs[z] = 0;
  if (!s.cpu) return;
  const CpuRec* recs = s.cpu + i * CPU_SLOTS;
  for (int c = 0; c < CPU_SLOTS; c++) {
    const CpuRec r = recs[c];
    if ((r.flags & CR_VALID) && r.ref > 0 && r.numa < 8) cs[r.numa]++;
  }
}

// NodeNUMAResource Reserve of a non-cpuset pod under a NUMA policy: NodeAllocation.addPodAllocation
// (node_allocation.go:111-156) adds the allocation on the affinity to the zones (numa_reserve_cs with
// unchanged cpusets; a new entry under a cpu ratio > 1 carries its zone's cpuset adjustment).
__device__ __forceinline__ void numa_reserve(const SoA& s, int64_t i, uint32_t nf, const NumaNode& v, uint32_t aff,
                                             const DevPod& p, int64_t* out16) {
  int64_t out[2][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0}};
  uint32_t got[2] = {0, 0};
  if (aff) numa_distribute<true>(v, aff, p, got, out);
  int cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if ((nf & NF_NUMA_AL_AMP) && ((got[0] | got[1]) & ~v.ak[0])) zone_cpusets(s, i, cs);  // a new entry
  numa_reserve_cs(s, i, nf, v, got, out, cs, cs, 0u, 0, out16);
}

// numa_reserve with an allocation given per NUMA id ([2*id + r], k_numa_views' choice for a reservation-matched pod)
__device__ __noinline__ void numa_reserve_dist(const SoA& s, int64_t i, uint32_t nf, const NumaNode& v,
                                               const int64_t* dist16, int64_t* out16) {
  int64_t out[2][8];
  uint32_t got[2] = {0, 0};
  for (int z = 0; z < 8; z++)
    for (int r = 0; r < 2; r++) {
      out[r][z] = dist16[2 * z + r];
      if (out[r][z] != 0) got[r] |= 1u << z;
    }
  int cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if ((nf & NF_NUMA_AL_AMP) && ((got[0] | got[1]) & ~v.ak[0])) zone_cpusets(s, i, cs);  // a new entry
  numa_reserve_cs(s, i, nf, v, got, out, cs, cs, 0u, 0, out16);
}

// `s`/`i` locate the node's DeviceShare state (read only for pods with PF_DS, and only when DS: the
// batch replay never evaluates a DeviceShare pod — such a pod is alone in its batch).
// NUMA: some node may carry a NUMA topology policy; `nv` holds node i's zones when its policy is set.
// CPU: the pod may bind CPUs (PF_CPUSET: a singleton batch) — cpuset PreFilter state, requestCPUBind,
// the amplified pod cpu and the required-bind-policy checks read the CPU SoA.
// ---- NodeResourcesFitPlus + ScarceResourceAvoidance + NodeResourcesFit -----------
// Weighted framework contribution of the Score plugins that read NodeInfo by resource id, for a feasible (pod,
// node), and NodeResourcesFit's Filter.  Go int64 arithmetic (wrapping products, truncating division) on the ext
// slots (KArgs::xs_id): xa / xr = the node's Allocatable / (NonZero)Requested of slot q, xm = its ids with
// Allocatable > 0.
__device__ __forceinline__ int64_t mul100_wrap(int64_t x) { return (int64_t)((uint64_t)x * 100u); }
// `get(q, a, r)` yields slot q's Allocatable / (NonZero)Requested: from registers (NodeFast: unrolled, constant
// indices) or straight from the SoA one slot at a time (ROLLED: a loop, so the row-path kernels -- whose registers
// the DeviceShare / NUMA evaluation already fills -- keep one slot's int64 division live, not eight)
template <bool ROLLED, typename F>
__device__ __forceinline__ void for_slots(F&& f) {
  if constexpr (ROLLED) {
#pragma unroll 1
    for (int q = 0; q < NUM_XS; q++) f(q);
  } else {
#pragma unroll
    for (int q = 0; q < NUM_XS; q++) f(q);
  }
}
template <bool ROLLED = false, typename G>
__device__ __forceinline__ int32_t ext_score_gen(uint64_t xm, G&& get, const DevPod& p, const KArgs& k) {
  int32_t t = 0;
  if (k.wp_fp) {  // resourceScorer (node_resource_fit_plus_utils.go:57-89) over the pod's requested names
    int64_t ns = 0, ws = 0;
    for_slots<ROLLED>([&](int q) {
      if (!((k.fp_mask >> q) & 1) || !((p.xmask >> k.xs_id[q]) & 1)) return;
      int64_t cap, req;
      get(q, cap, req);
      req += p.xreq[q];
      int64_t sc = 0;
      if ((k.fp_most >> q) & 1) {  // mostRequestedScore (:35-44)
        if (req > cap) req = cap;
        sc = cap == 0 ? 0 : mul100_wrap(req) / cap;
      } else {  // leastRequestedScore (:46-55)
        sc = (cap == 0 || req > cap) ? 0 : mul100_wrap(cap - req) / cap;
      }
      ns += sc * k.fp_w[q];
      ws += k.fp_w[q];
    });
    t += k.wp_fp * (int32_t)(ws == 0 ? 100 : ns / ws);
  }
  if (k.wp_sra) {  // scarce_resource_avoidance.go:70-90,159-161
    const uint64_t diff = xm & ~p.xmask;
    const int nd = __popcll(diff), ni = __popcll(diff & k.sra_mask);
    t += k.wp_sra * ((nd == 0 || ni == 0) ? 100 : (nd - ni) * 100 / nd);
  }
  if (k.wp_fit) {  // NodeResourcesFit Score (k8s v1.28.7 resource_allocation.go score, least/most_allocated.go)
    int64_t ns = 0, ws = 0;
    const bool most = (k.flags & AF_FIT_MOST) != 0;
    for_slots<ROLLED>([&](int q) {
      if (!((k.fit_mask >> q) & 1)) return;
      const int64_t preq = p.xreq[q];
      if (k.xs_id[q] >= 2 && preq == 0) return;  // a scalar the pod does not request: (0, 0)
      int64_t cap, req;
      get(q, cap, req);
      if (cap == 0) return;
      req += preq;
      int64_t sc;
      if (most) {
        if (req > cap) req = cap;
        sc = mul100_wrap(req) / cap;
      } else {
        sc = req > cap ? 0 : mul100_wrap(cap - req) / cap;
      }
      ns += sc * k.fit_w[q];
      ws += k.fit_w[q];
    });
    t += k.wp_fit * (int32_t)(ws == 0 ? 0 : ns / ws);
  }
  return t;
}
__device__ __forceinline__ int32_t ext_score_vals(uint64_t xm, const int64_t (&xa)[NUM_XS], const int64_t (&xr)[NUM_XS],
                                                  const DevPod& p, const KArgs& k) {
  return ext_score_gen(xm, [&](int q, int64_t& a, int64_t& r) { a = xa[q], r = xr[q]; }, p, k);
}
// NodeResourcesFit Filter (k8s v1.28.7 fit.go fitsRequest): the pod room, then cpu / memory requests > 0 against
// Allocatable - Requested (the row's NodeInfo), then the scalar slots; returns the reason (0 = fits)
template <bool ROLLED = false, typename G>
__device__ __forceinline__ uint8_t fit_filter_gen(int64_t room, G&& get, bool cpu_over, bool mem_over, const DevPod& p,
                                                  const KArgs& k) {
  if (room < 1) return KE_REASON_FIT_TOO_MANY_PODS;
  if (cpu_over) return KE_REASON_FIT_INSUFFICIENT_CPU;
  if (mem_over) return KE_REASON_FIT_INSUFFICIENT_MEMORY;
  bool sc = false;
  for_slots<ROLLED>([&](int q) {
    if (!((k.fit_scalar >> q) & 1) || p.xreq[q] <= 0) return;
    int64_t a, r;
    get(q, a, r);
    sc |= p.xreq[q] > a - r;
  });
  return sc ? KE_REASON_FIT_INSUFFICIENT_SCALAR : 0;
}
__device__ __forceinline__ uint8_t fit_filter(int64_t room, const int64_t (&xa)[NUM_XS], const int64_t (&xr)[NUM_XS],
                                              bool cpu_over, bool mem_over, const DevPod& p, const KArgs& k) {
  return fit_filter_gen(room, [&](int q, int64_t& a, int64_t& r) { a = xa[q], r = xr[q]; }, cpu_over, mem_over, p, k);
}
// slot q's words from the SoA (plain loads: no kernel writes them while this one runs)
struct ExtSoaGet {
  const SoA& s;
  int64_t i;
  __device__ __forceinline__ void operator()(int q, int64_t& a, int64_t& r) const {
    a = s.xf[(XF_ALLOC + q) * s.stride + i];
    r = s.xf[(XF_REQ + q) * s.stride + i];
  }
};
// NodeResourcesFit's Filter reason on a row (eval_pair / lite_total)
__device__ __forceinline__ uint8_t fit_filter_row(const SoA& s, int64_t i, const NodeRegs& n, const DevPod& p,
                                                  const KArgs& k) {
  const bool co = p.req[0] > 0 && p.req[0] > n.nalloc[0] - n.nreq[0];
  const bool mo = p.req[1] > 0 && p.req[1] > n.nalloc[1] - n.nreq[1];
  return fit_filter_gen<true>(s.xf[XF_PODS * s.stride + i], ExtSoaGet{s, i}, co, mo, p, k);
}
__device__ __forceinline__ int32_t ext_score(const SoA& s, int64_t i, const DevPod& p, const KArgs& k) {
  return ext_score_gen<true>(s.xm[i], ExtSoaGet{s, i}, p, k);
}
// Reserve: NodeInfo (NonZero)Requested += the pod's requests of the slots' resources, one pod more
__device__ __forceinline__ void ext_reserve(const SoA& s, int64_t i, const DevPod& p, const KArgs& k) {
#pragma unroll
  for (int q = 0; q < NUM_XS; q++)
    if (q < k.xs_n) s.xf[(XF_REQ + q) * s.stride + i] += p.xreq[q];
  s.xf[XF_PODS * s.stride + i] -= 1;
}

template <bool DS, bool NUMA, bool DEFER = false, bool FB_AFF = false, bool CPU = false, bool H = false>
__device__ __forceinline__ EvalOut eval_pair(const NodeRegs& n, bool expired, const DevPod& p, const KArgs& k,
                                             const SoA& s, int64_t i, const NumaNode& nv, uint32_t fb_aff = 0) {
  EvalOut o;
  o.status = KE_CODE_SUCCESS;
  o.reason = KE_REASON_NONE;
  o.aff = 0;
  o.la = o.numa = o.ds = 0;
  const uint32_t nf = n.flags;
  if (!(nf & NF_VALID)) {
    o.status = KE_CODE_ERROR;
    o.total = -1;
    return o;
  }
  if (CPU && (p.flags & PF_CPU_INVALID)) {  // NodeNUMAResource PreFilter failed (plugin.go:296-298)
    o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    o.reason = KE_REASON_NUMA_INVALID_REQUESTED_CPUS;
    o.total = -1;
    return o;
  }
  if (p.flags & PF_DS_INVALID) {  // DeviceShare PreFilter failed: the pod fits nowhere (utils.go:355-390)
    o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    o.reason = p.ds_req[0] ? (uint8_t)p.ds_req[0] : (uint8_t)KE_REASON_DS_INVALID_REQUEST;  // the host's reason
    o.total = -1;
    return o;
  }
  // ---- NodeResourcesFit.Filter (a default plugin: before the profile's own Filters)
  if (k.flags & AF_FIT_FILTER) {
    const uint8_t why = fit_filter_row(s, i, n, p, k);
    if (why) {
      o.status = KE_CODE_UNSCHEDULABLE;
      o.reason = why;
      o.total = -1;
      return o;
    }
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
        const int64_t fh = v ? n.fh[1][q] : n.fh[0][q];  // select, not a runtime index (no scratch)
        if (o.status == KE_CODE_SUCCESS && (nf & nf_fh_on(v, q)) && p.est[q] > fh) {
          o.status = KE_CODE_UNSCHEDULABLE;
          const bool agg = v == 0 && (nf & NF_FILTER_AGG);
          o.reason = (uint8_t)(agg ? KE_REASON_LA_AGG_USAGE_CPU + q : KE_REASON_LA_USAGE_CPU + q);
        }
      }
    }
  }
  // ---- NodeNUMAResource.Filter: node / pod topology policy merge (plugin.go:337-341), then
  // filterAmplifiedCPUs (plugin.go:408-442)
  const int pod_pol = NUMA ? pf_numa_policy(p.flags) : 0, node_pol = nf_numa_policy(nf);
  if (NUMA && o.status == KE_CODE_SUCCESS && !(p.flags & PF_NUMA_SKIP) && pod_pol && node_pol && pod_pol != node_pol) {
    o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    o.reason = KE_REASON_NUMA_POLICY_CONFLICT;
  }
  // requestCPUBind (util.go:121-138): the pod's own cpuset state, else a node CPU bind policy binds
  // any whole-CPU request (-1: a fractional one there is UnschedulableAndUnresolvable)
  int rcb = 0;
  if (CPU && !(p.flags & PF_NUMA_SKIP)) {
    if (p.flags & PF_CPU_RCB) rcb = 1;
    else if (p.req[0] != 0 && nf_cpu_bind(nf) != KE_NODE_CPU_BIND_NONE) rcb = (p.flags & PF_CPU_INT) ? 1 : -1;
  }
  if (CPU && o.status == KE_CODE_SUCCESS && rcb < 0) {
    o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    o.reason = KE_REASON_NUMA_INVALID_REQUESTED_CPUS;
  }
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
        const int64_t pcpu = (CPU && rcb > 0) ? amplify_bits(p.req[0], s.cs[CS_RF * s.stride + i]) : p.req[0];
        if (pcpu > n.nalloc[0] - req) {
          o.status = KE_CODE_UNSCHEDULABLE;
          o.reason = KE_REASON_NUMA_INSUFFICIENT_AMPLIFIED_CPU;
        }
      }
    }
  }
  const int eff_pol = pod_pol ? pod_pol : node_pol;
  // ---- cpuset binding (plugin.go:351-398): topology, bind-policy conflict, SMT alignment, and the
  // required policies' trial allocation, which on a regular topology is a count check
  if (CPU && rcb > 0 && o.status == KE_CODE_SUCCESS) {
    if (!(nf & NF_CPUS_VALID)) {
      o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      o.reason = KE_REASON_NUMA_INVALID_CPU_TOPOLOGY;
    } else {
      const int64_t cnt = s.cs[CS_CNT * s.stride + i];
      const int preq = pf_cpu_required(p.flags), nb = nf_cpu_bind(nf);
      const int req = nb == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY ? XB_FULL : nb == KE_NODE_CPU_BIND_SPREAD_BY_PCPUS ? XB_SPREAD : preq;
      const int64_t ncpu = p.req[0] / 1000;
      if (preq != XB_NONE && preq != req) {
        o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
        o.reason = KE_REASON_NUMA_CPU_BIND_POLICY_CONFLICT;
      } else if (req == XB_FULL && ncpu % cs_cpc(cnt) != 0) {
        o.status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
        o.reason = KE_REASON_NUMA_SMT_ALIGNMENT;
      } else if (req != XB_NONE && eff_pol == KE_NUMA_POLICY_NONE && (nf & NF_RSV_CS) &&
                 rsv_ovr_of(s, i) && rsv_ovr_of(s, i)->filter != 0) {
        // the matched pod's reservations first (plugin.go:381-390): satisfied by one (k_rsv_views), or none under
        // a reservation affinity ("Reservation(s) ...", reservation.go:420-422)
        if (rsv_ovr_of(s, i)->filter == 2) {
          o.status = KE_CODE_UNSCHEDULABLE;
          o.reason = KE_REASON_RSV_INSUFFICIENT_CPUS;
        }
      } else if (req != XB_NONE && eff_pol == KE_NUMA_POLICY_NONE &&
                 ncpu > (req == XB_FULL ? cs_full(cnt) : cs_spread(cnt))) {
        o.status = KE_CODE_UNSCHEDULABLE;
        o.reason = KE_REASON_NUMA_INSUFFICIENT_CPUS;
      }
    }
  }
  // ---- NodeNUMAResource.Filter under a NUMA topology policy: FilterByNUMANode + topologymanager Admit
  const bool npol = NUMA && !(p.flags & PF_NUMA_SKIP) && eff_pol != KE_NUMA_POLICY_NONE;
  int32_t npol_score = 0;
  // DeviceShare is a second hint provider for a pod with device requests on a node with a device cache
  // (topology_hint.go:38-58); such a pair is never deferred (its batch runs no k_numa_fallback)
  const bool ds_here = DS && (p.flags & PF_DS) && (nf & NF_DS_CACHE);
  bool stored = false;  // the topology manager stored an affinity for the node
  // a reservation-matched pod on a node of its reservations holding NUMA resources / CPUs: the outcome k_numa_views
  // computed over the allocate-from-reservation trials (RsvOvr.numa_on)
  const RsvOvr* nro = (npol && (nf & NF_RSV_CS)) ? rsv_ovr_of(s, i) : nullptr;
  if (nro && !nro->numa_on) nro = nullptr;
  if (nro && o.status == KE_CODE_SUCCESS) {
    if (nro->numa_st != KE_CODE_SUCCESS) {
      o.status = nro->numa_st;
      o.reason = nro->numa_reason;
    } else {
      o.aff = nro->numa_aff;
      npol_score = nro->numa_score;
      stored = true;
    }
  } else if (npol && o.status == KE_CODE_SUCCESS) {
    DsHints dh;
    dh.status = 0;
    dh.none = true;
    if (ds_here) ds_numa_hints<H>(s, i, p, k, dh);
    const DsHints* dhp = ds_here ? &dh : nullptr;
    NumaPick pk;
    if (CPU && rcb > 0) {  // a binding pod: cpuset hints and allocation (resource_manager.go:166-192,353-459)
      const NumaCs cs = numa_cs_load(s, i, nf, p);
      DevPod ps = p;  // options.requests: cpu amplified (plugin.go:634-640)
      ps.req[0] = amplify_bits(p.req[0], s.cs[CS_RS * s.stride + i]);
      NumaNode tv = nv;
      numa_trim(tv, cs);
      pk = ds_here ? numa_admit<false, false, true>(s, i, nf, eff_pol, tv, p, k, 0u, &cs, &ps, dhp)
                   : numa_admit<DEFER, FB_AFF, true>(s, i, nf, eff_pol, tv, p, k, fb_aff, &cs, &ps);
      if (DEFER && pk.status == STATUS_DEFERRED) {
        o.status = STATUS_DEFERRED;
        o.total = -1;
        return o;
      }
      if (pk.status == KE_CODE_SUCCESS) npol_score = numa_policy_score<true>(s, i, tv, pk.aff, p, k, n, &cs, &ps);
    } else {
      pk = ds_here ? numa_admit<false>(s, i, nf, eff_pol, nv, p, k, 0u, nullptr, nullptr, dhp)
                   : numa_admit<DEFER, FB_AFF>(s, i, nf, eff_pol, nv, p, k, fb_aff);
      if (DEFER && pk.status == STATUS_DEFERRED) {
        o.status = STATUS_DEFERRED;
        o.total = -1;
        return o;
      }
      if (pk.status == KE_CODE_SUCCESS) npol_score = numa_policy_score(s, i, nv, pk.aff, p, k, n);
    }
    if (pk.status == KE_CODE_SUCCESS && ds_here && !(k.flags & AF_DS_NO_NUMA)) {
      int why = 0;  // allocateResources -> DeviceShare.Allocate on the affinity (topology_hint.go:60-117)
      const int st = ds_try_allocate<H>(s, i, p, k, DsAff{pk.aff != 0, pk.aff}, nullptr, &why);
      if (st) pk.status = (uint8_t)st, pk.reason = (uint8_t)why;
    }
    if (pk.status != KE_CODE_SUCCESS) {
      o.status = pk.status;
      o.reason = pk.reason;
    } else {
      o.aff = (uint8_t)pk.aff;
      stored = true;
    }
  }
  // ---- DeviceShare.Filter + raw Score  plugin.go:311-365, scoring.go:45-103 (Filter passes and Score
  // reads the devices of the affinity when the topology manager stored one)
  // a reservation-matched / -ignored pod on a node of its device-holding reservations: the allocate-from-reservation
  // outcome k_ds_views computed (deviceshare/plugin.go:350-364, scoring.go:83-102; no NUMA policy on pod or node)
  const RsvOvr* ro = (nf & NF_RSV_CS) ? rsv_ovr_of(s, i) : nullptr;
  if (ds_here && o.status == KE_CODE_SUCCESS) {
    if (ro && ro->ds_on) {
      o.status = ro->ds_st;
      o.reason = ro->ds_reason;
      o.ds = ro->ds_raw;
    } else {
      ds_filter_score<H>(s, i, p, k, o, stored, DsAff{stored && o.aff != 0, o.aff});
    }
  }
  // the Reservation Filter of a pod with a reservation affinity (reservation/plugin.go:316-318, 351-442): only the
  // nodes of its matched reservations where one fits
  if ((k.flags & AF_RSV_ONLY) && o.status == KE_CODE_SUCCESS && !(ro && ro->rfilter == 1)) {
    o.status = KE_CODE_UNSCHEDULABLE;
    o.reason = KE_REASON_RSV_AFFINITY;
  }
  if (o.status != KE_CODE_SUCCESS) {
    o.total = -1;
    o.ds = 0;
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
      const int64_t room = (v ? n.sa[1][q] : n.sa[0][q]) - p.est[q];  // cap - used
      const int32_t sc = (cap > 0 && room >= 0) ? div100(room, cap, n.dcap[q], n.rcap[q]) : 0;  // leastUsedScore
      s += sc * k.w_la[q];
    }
    la = div_small(s, k.wsum_la);
  }
  // ---- NodeNUMAResource.Score  scoring.go:66-139,210-249
  int32_t nu = 0;
  if (npol) {
    nu = npol_score;
  } else if (!(p.flags & PF_NUMA_SKIP) && !(nf & NF_NUMA_SCORE_ZERO)) {
    bool zero = false;
    int64_t reqc = n.nreq[0], preq0 = p.req[0];
    if (p.req[0] != 0 && (nf & NF_NUMA_RATIO_S)) {
      if (nf & NF_NUMA_TOPO_INVALID) zero = true;
      else reqc = n.nreq[0] - n.csm + n.csas;
    }
    if (CPU && rcb != 0) {  // scoring.go:86-92: a binding pod scores its amplified cpu, 0 without a topology
      if (rcb < 0 || !(nf & NF_CPUS_VALID)) zero = true;
      else if (nf & NF_NUMA_RATIO_S) preq0 = amplify_bits(p.req[0], s.cs[CS_RS * s.stride + i]);
    }
    if (!zero) {
      int32_t s = 0, ws = 0;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int32_t w = k.w_numa[q];
        const int64_t alloc = n.nalloc[q];
        if (w == 0 || alloc == 0) continue;
        const int64_t req = (q == 0 ? reqc + preq0 : n.nreq[1] + p.req[1]);
        int32_t sc;
        if (k.flags & AF_NUMA_MOST) {  // mostRequestedScore  most_allocated.go:53-62
          const int64_t rq = req > alloc ? alloc : req;
          sc = alloc > 0 ? div100(rq, alloc, n.dalloc[q], n.ralloc[q]) : (int32_t)((rq * 100) / alloc);
        } else {  // leastRequestedScore  least_allocated.go:49-58
          sc = req > alloc ? 0 : (alloc > 0 ? div100(alloc - req, alloc, n.dalloc[q], n.ralloc[q]) : (int32_t)(((alloc - req) * 100) / alloc));
        }
        s += sc * w;
        ws += w;
      }
      nu = ws > 0 ? div_small(s, ws) : 0;
    }
  }
  o.la = (int16_t)la;
  o.numa = (int16_t)nu;
  o.total = k.wp_la * la + k.wp_numa * nu;
  if (k.flags & AF_EXT) o.total += ext_score(s, i, p, k);
  return o;
}

// use ? x*100/c : 0 (Go int64 division) as straight-line code: div100's estimate + corrections always,
// the native division only for lanes outside the estimate's range (exec-masked, skipped when none).
__device__ __forceinline__ int32_t div100_sel(bool use, int64_t x, int64_t c, double dc, double rc) {
  int32_t q = div100_f(x, dc, rc);
  if (use & !div100_fast_ok(x, c)) q = (int32_t)(x * 100 / c);
  return use ? q : 0;
}

// eval_pair<false, false>(...).total without exec-mask branches: every predicate is a lane boolean and
// every score term is computed and selected.  Plain pods on nodes seen through the LoadAware +
// NodeNUMAResource (policy None) path — k_resolve's replay re-evaluation and k_eval_batch's plain
// batches.  Same arithmetic as eval_pair (load_aware.go:122-249,387-406; plugin.go:408-442;
// scoring.go:66-139,210-249); a failing filter gives -1 whatever the reason.
__device__ __forceinline__ int32_t lite_total(const NodeRegs& n, bool expired, const DevPod& p, const KArgs& k) {
  const uint32_t nf = n.flags, pf = p.flags, af = k.flags;
  bool fail = !(nf & NF_VALID) | ((pf & PF_DS_INVALID) != 0);
  // LoadAwareScheduling.Filter
  const bool la_on = !(pf & PF_DAEMONSET) & ((nf & NF_HAS_METRIC) != 0);
  const bool exp_f = ((af & AF_FILTER_EXPIRED) != 0) & ((af & AF_EXP_PRESENT) != 0) & expired;
  fail |= la_on & exp_f & !(af & AF_ENABLE_WHEN_EXPIRED);
  const bool thr_on = la_on & !exp_f & !(nf & NF_NM_NIL);
  const bool v = ((nf & NF_HAS_PROD_THR) != 0) & ((pf & PF_PROD) != 0);
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int64_t fh = v ? n.fh[1][q] : n.fh[0][q];
    const bool on = (nf & (v ? nf_fh_on(1, q) : nf_fh_on(0, q))) != 0;
    fail |= thr_on & on & (p.est[q] > fh);
  }
  // filterAmplifiedCPUs
  const bool amp = !(pf & PF_NUMA_SKIP) & (p.req[0] != 0);
  fail |= amp & ((nf & NF_NUMA_AMP_ERR) != 0);
  const bool rf = amp & !(nf & NF_NUMA_AMP_ERR) & ((nf & NF_NUMA_RATIO_F) != 0);
  fail |= rf & ((nf & NF_NUMA_TOPO_INVALID) != 0);
  const int64_t areq = ((n.nreq[0] >= n.csm) & (n.csm > 0)) ? n.nreq[0] - n.csm + n.csaf : n.nreq[0];
  fail |= rf & !(nf & NF_NUMA_TOPO_INVALID) & (p.req[0] > n.nalloc[0] - areq);
  // LoadAwareScheduling.Score
  const bool las = ((nf & NF_HAS_METRIC) != 0) & !(((af & AF_EXP_PRESENT) != 0) & expired) & !(nf & NF_NM_NIL) & (k.wsum_la > 0);
  const bool vs = (pf & PF_LA_SCORE_PROD) != 0;
  int32_t sl = 0;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int64_t cap = n.cap[q];
    const int64_t room = (vs ? n.sa[1][q] : n.sa[0][q]) - p.est[q];
    sl += div100_sel(las & (cap > 0) & (room >= 0), room, cap, n.dcap[q], n.rcap[q]) * k.w_la[q];
  }
  const int32_t la = las ? div_small(sl, k.wsum_la) : 0;
  // NodeNUMAResource.Score (policy None)
  const bool rs = (p.req[0] != 0) & ((nf & NF_NUMA_RATIO_S) != 0);
  const bool zero = ((pf & PF_NUMA_SKIP) != 0) | ((nf & NF_NUMA_SCORE_ZERO) != 0) | (rs & ((nf & NF_NUMA_TOPO_INVALID) != 0));
  const int64_t reqc = rs ? n.nreq[0] - n.csm + n.csas : n.nreq[0];
  const bool most = (af & AF_NUMA_MOST) != 0;
  int32_t sn = 0, ws = 0;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int32_t w = k.w_numa[q];
    const int64_t alloc = n.nalloc[q];
    const bool on = !zero & (w != 0) & (alloc != 0);
    const int64_t req = q == 0 ? reqc + p.req[0] : n.nreq[1] + p.req[1];
    const int64_t x = most ? (req > alloc ? alloc : req) : alloc - req;
    const int32_t sc = div100_sel(on & (most | (req <= alloc)), x, alloc, n.dalloc[q], n.ralloc[q]);
    sn += on ? sc * w : 0;
    ws += on ? w : 0;
  }
  const int32_t nu = ws > 0 ? div_small(sn, ws) : 0;
  return fail ? -1 : k.wp_la * la + k.wp_numa * nu;
}

// a packed row into registers
__device__ __forceinline__ void regs_from_row(const Row& r, NodeRegs& n) {
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

// Words one workgroup hands to another while both run (k_fixup -> k_resolve_run: the exact lists;
// k_resolve_run -> k_fixup: the changed rows; -> later eval launches: the patched SoA rows) are
// written and read with sc1 (relaxed agent-scope atomics: global_store / global_load ... sc1), i.e.
// write-through past the storing CU and read past the reading CU's L1: no release (L2 write-back) and
// no acquire (L1/L2 invalidate) fence on the hand-off path (MI355X_MICROARCH.md § visibility,
// cdna_hip_programming.md Guideline 16).  The storing wave drains (vmcnt(0)) before the flag.
__device__ __forceinline__ int64_t ld_sc1(const int64_t* p) {
  return __hip_atomic_load(const_cast<int64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_sc1(const int32_t* p) {
  return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)

// Device-side hand-off between the eval stream and the persistent Reserve kernel (k_resolve_run):
// counters / flags in global memory polled with relaxed sc1 loads, payloads sc1 (above), every wait
// bounded in time and abandoned when the run's error word is set.
constexpr uint64_t HANDOFF_TIMEOUT_TICKS = 200000000ull;  // 2 s of s_memrealtime (100 MHz)
__device__ __forceinline__ bool wait_at_least(const int32_t* flag, int32_t want, int32_t* err) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > HANDOFF_TIMEOUT_TICKS) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  // the hand-off's words are read with sc1 loads from here on: no acquire fence, only a compiler
  // ordering point (cdna_hip_programming.md Guideline 16)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return true;
}


// ---- the replay's fast path: per-node records with the node-only terms precomputed --------------
// In the replay a changed node is re-evaluated for every later pod of its batch, while its row changes
// only at its own Reserves; and almost every pod adopts a node it has not touched yet.  Each node
// therefore has a row-major replay record (NUM_RW words, RecWord) next to the SoA: the static node-only
// terms of lite_total (KArgs weights, capacities as doubles with their reciprocals, flag bits) and the
// Reserve-dependent ones (the LoadAware filter headrooms, score bases and NodeInfo.Requested as exact
// doubles).  k_scatter_rows derives it with the row, every Reserve rewrites it.  Adopting a node is 13
// contiguous 16-byte loads plus the `now`-dependent bits; re-evaluating it (fast_total) is a handful of
// compares and four exact x*100/c divisions.  Doubles are exact: every value is an integer below 2^53
// (ingestion rejects larger quantities) and only sums / differences of them are formed.
constexpr int64_t THR_NONE = INT64_MAX;
enum : uint32_t {
  FB_FAIL = 1u,       // not a valid node
  FB_EXP_FAIL = 2u,   // LoadAware: NodeMetric expired and FilterExpiredNodeMetrics (non-DaemonSet pods)
  FB_AMP_BAD = 4u,    // filterAmplifiedCPUs fails for any cpu request (unparsable ratio / invalid topology)
  FB_LAS = 8u,        // LoadAware Score computes (metric present, not expired, NodeMetric set, weights)
  FB_NZERO = 16u,     // NodeNUMAResource Score is 0 (getResourceOptions error)
  FB_RSZERO = 32u,    // ... when the pod requests cpu (score ratio > 1 with an invalid topology)
  FB_CAP0 = 64u,      // 2 bits: EstimateNode allocatable > 0 per resource
  FB_AL0 = 256u,      // 2 bits: NodeInfo.Allocatable != 0 per resource
  FB_SLOW = 1024u,    // a capacity >= 2^42: x*100/c in int64 (outside the reciprocal estimate's range)
  FB_RF = 2048u,      // filterAmplifiedCPUs checks the amplified room (ratio > 1, parsable, valid topology)
};
// record words (int64 / double)
enum RecWord : int {
  RW_FH = 0,       // 4: LoadAware filter headroom fh[variant][res] (int64)
  RW_SA = 4,       // 4: LoadAware score base sa[variant][res] (double)
  RW_CAP = 8,      // 2: EstimateNode allocatable (double)
  RW_RCAP = 10,    // 2: its approximate reciprocal
  RW_AL = 12,      // 2: NodeInfo.Allocatable (double)
  RW_RAL = 14,     // 2: its approximate reciprocal
  RW_NREQ = 16,    // 2: NodeInfo.Requested (double)
  RW_NREQ0S = 18,  // cpu requested, cpuset CPUs at the score amplification (double)
  RW_NALLOC0 = 19, // cpu allocatable (int64), RW_CSM / RW_CSAF: cpuset milli and its filter amplification
  RW_CSM = 20,
  RW_CSAF = 21,
  RW_UT = 22,      // NodeMetric UpdateTime
  RW_FLAGS = 23,   // node flags (low 32) | static FB_* bits (high 32)
  RW_NWS = 24,     // Σ NUMA score weights over resources with allocatable != 0
  RW_PAD = 25,
  NUM_RW = 26
};
static_assert(NUM_RW % 2 == 0, "records are 16-byte granules");

struct NodeFast {
  int64_t fh[2][2];
  double sa[2][2];
  double cap[2], rcap[2], al[2], ral[2];
  double nreq[2], nreq0s;
  int64_t nalloc0, csm, csaf, ut;
  uint32_t nflags, sbits;  // node flags, static FB bits
  int32_t nws;
  // derived at adoption / after each Reserve
  int64_t thr[2][2];  // [pod is prod][res]: LoadAware filter passes iff est <= thr (THR_NONE = no check)
  int64_t amp_room;   // filterAmplifiedCPUs passes iff req0 <= amp_room (THR_NONE = no check)
  uint32_t bits;      // sbits + the `now`-dependent FB bits
  bool thr_node;      // the LoadAware filter thresholds apply (metric, not expired-filtered, NodeMetric set)
  // NodeResourcesFitPlus / ScarceResourceAvoidance / NodeResourcesFit (AF_EXT): the node's ext SoA words (ext_load)
  uint64_t xm;
  int64_t xa[NUM_XS], xr[NUM_XS];
  int64_t room;  // AllowedPodNumber - len(Pods)
};

// the node's ext words (sc1: a Reserve kernel of this or a concurrent launch may have written them)
__device__ __forceinline__ void ext_load(const SoA& s, int64_t node, const KArgs& k, NodeFast& f) {
  f.xm = (uint64_t)ld_sc1(reinterpret_cast<const int64_t*>(s.xm) + node);
#pragma unroll
  for (int q = 0; q < NUM_XS; q++) {
    f.xa[q] = q < k.xs_n ? ld_sc1(s.xf + (XF_ALLOC + q) * s.stride + node) : 0;
    f.xr[q] = q < k.xs_n ? ld_sc1(s.xf + (XF_REQ + q) * s.stride + node) : 0;
  }
  f.room = ld_sc1(s.xf + XF_PODS * s.stride + node);
}
// a Reserve on the node's ext words in registers, and their write-back (sc1: read by later launches)
__device__ __forceinline__ void ext_fast_reserve(NodeFast& f, const DevPod& p, const KArgs& k) {
#pragma unroll
  for (int q = 0; q < NUM_XS; q++) f.xr[q] += q < k.xs_n ? p.xreq[q] : 0;
  f.room -= 1;
}
__device__ __forceinline__ void ext_store(const SoA& s, int64_t node, const NodeFast& f, const KArgs& k) {
#pragma unroll
  for (int q = 0; q < NUM_XS; q++)
    if (q < k.xs_n) st_sc1(s.xf + (XF_REQ + q) * s.stride + node, f.xr[q]);
  st_sc1(s.xf + XF_PODS * s.stride + node, f.room);
}

// the record of a prepared row (rcap / ralloc set), static bits from the args
__device__ __forceinline__ void rec_from_regs(const NodeRegs& n, const KArgs& k, int64_t (&w)[NUM_RW]) {
  const uint32_t nf = n.flags;
  uint32_t b = 0;
  b |= !(nf & NF_VALID) ? FB_FAIL : 0u;
  b |= ((nf & NF_NUMA_AMP_ERR) || ((nf & NF_NUMA_RATIO_F) && (nf & NF_NUMA_TOPO_INVALID))) ? FB_AMP_BAD : 0u;
  b |= (!(nf & NF_NUMA_AMP_ERR) && (nf & NF_NUMA_RATIO_F) && !(nf & NF_NUMA_TOPO_INVALID)) ? FB_RF : 0u;
  b |= (nf & NF_NUMA_SCORE_ZERO) ? FB_NZERO : 0u;
  b |= ((nf & NF_NUMA_RATIO_S) && (nf & NF_NUMA_TOPO_INVALID)) ? FB_RSZERO : 0u;
  int32_t nws = 0;
  for (int q = 0; q < 2; q++) {
    b |= n.cap[q] > 0 ? (FB_CAP0 << q) : 0u;
    b |= n.nalloc[q] != 0 ? (FB_AL0 << q) : 0u;
    nws += (n.nalloc[q] != 0 && k.w_numa[q] != 0) ? k.w_numa[q] : 0;
    // the reciprocal division's range: 0 < c < 2^42 (x <= 16c holds: x <= sa <= cap for LoadAware,
    // x <= alloc for the NUMA scorers)
    if ((n.cap[q] > 0 && n.cap[q] >= DIV_FAST_CAP) || n.nalloc[q] < 0 || n.nalloc[q] >= DIV_FAST_CAP) b |= FB_SLOW;
  }
  for (int v = 0; v < 2; v++)
    for (int q = 0; q < 2; q++) {
      w[RW_FH + 2 * v + q] = n.fh[v][q];
      w[RW_SA + 2 * v + q] = __double_as_longlong((double)n.sa[v][q]);
    }
  for (int q = 0; q < 2; q++) {
    w[RW_CAP + q] = __double_as_longlong(n.dcap[q]);
    w[RW_RCAP + q] = __double_as_longlong(n.rcap[q]);
    w[RW_AL + q] = __double_as_longlong(n.dalloc[q]);
    w[RW_RAL + q] = __double_as_longlong(n.ralloc[q]);
    w[RW_NREQ + q] = __double_as_longlong((double)n.nreq[q]);
  }
  w[RW_NREQ0S] = __double_as_longlong((nf & NF_NUMA_RATIO_S) ? (double)(n.nreq[0] - n.csm + n.csas) : (double)n.nreq[0]);
  w[RW_NALLOC0] = n.nalloc[0];
  w[RW_CSM] = n.csm;
  w[RW_CSAF] = n.csaf;
  w[RW_UT] = n.ut;
  w[RW_FLAGS] = (int64_t)(((uint64_t)b << 32) | nf);
  w[RW_NWS] = nws;
  w[RW_PAD] = 0;
}

// the LoadAware filter bounds and the amplified room from the current headrooms / requested
__device__ __forceinline__ void fast_bounds(NodeFast& f) {
  const uint32_t nf = f.nflags;
  const bool v1 = (nf & NF_HAS_PROD_THR) != 0;  // the prod pods' profile (register selects, no indexing)
#pragma unroll
  for (int q = 0; q < 2; q++) {
    f.thr[0][q] = (f.thr_node & ((nf & nf_fh_on(0, q)) != 0)) ? f.fh[0][q] : THR_NONE;
    const bool on1 = v1 ? (nf & nf_fh_on(1, q)) != 0 : (nf & nf_fh_on(0, q)) != 0;
    f.thr[1][q] = (f.thr_node & on1) ? (v1 ? f.fh[1][q] : f.fh[0][q]) : THR_NONE;
  }
  const int64_t nreq0 = (int64_t)f.nreq[0];
  const int64_t areq = ((nreq0 >= f.csm) & (f.csm > 0)) ? nreq0 - f.csm + f.csaf : nreq0;
  f.amp_room = (f.sbits & FB_RF) ? f.nalloc0 - areq : THR_NONE;
}

// the `now`-dependent parts after loading a record (isNodeMetricExpired, helper.go:35-40)
__device__ __forceinline__ void fast_adopt(NodeFast& f, const KArgs& k) {
  const uint32_t nf = f.nflags, af = k.flags;
  const bool expired = !(nf & NF_HAS_UT) || (k.exp_s > 0 && (k.now - f.ut) >= k.exp_s * 1000000000LL);
  const bool exp_f = ((af & AF_FILTER_EXPIRED) != 0) & ((af & AF_EXP_PRESENT) != 0) & expired;
  uint32_t b = f.sbits;
  b |= (((nf & NF_HAS_METRIC) != 0) & exp_f & !(af & AF_ENABLE_WHEN_EXPIRED)) ? FB_EXP_FAIL : 0u;
  const bool las = ((nf & NF_HAS_METRIC) != 0) & !(((af & AF_EXP_PRESENT) != 0) & expired) & !(nf & NF_NM_NIL) &
                   (k.wsum_la > 0);
  b |= las ? FB_LAS : 0u;
  f.bits = b;
  f.thr_node = ((nf & NF_HAS_METRIC) != 0) & !exp_f & !(nf & NF_NM_NIL);
  fast_bounds(f);
}

// a record from the replay's record array (workgroup-scope loads: this workgroup may have rewritten it
// in an earlier batch; another launch wrote it before this one started)
__device__ __forceinline__ void rec_unpack(const int64_t (&w)[NUM_RW], NodeFast& f);
template <int SCOPE = __HIP_MEMORY_SCOPE_WORKGROUP>
__device__ __forceinline__ void rec_load(const int64_t* __restrict__ rec, NodeFast& f) {
  int64_t w[NUM_RW];
  // every loaded word is consumed (a dead load's register would be reused while the load is in flight,
  // and the reuse would wait for it)
#pragma unroll
  for (int u = 0; u < RW_PAD; u++) w[u] = __hip_atomic_load(const_cast<int64_t*>(rec + u), __ATOMIC_RELAXED, SCOPE);
  w[RW_PAD] = 0;
  rec_unpack(w, f);
}
// a record no running kernel writes (k_eval_plain): 13 plain 16-byte loads
__device__ __forceinline__ void rec_load_plain(const int64_t* __restrict__ rec, NodeFast& f) {
  int64_t w[NUM_RW];
  const int4* r4 = reinterpret_cast<const int4*>(rec);
#pragma unroll
  for (int u = 0; u < NUM_RW / 2; u++) {
    const int4 q = r4[u];
    w[2 * u] = (int64_t)(((uint64_t)(uint32_t)q.y << 32) | (uint32_t)q.x);
    w[2 * u + 1] = (int64_t)(((uint64_t)(uint32_t)q.w << 32) | (uint32_t)q.z);
  }
  rec_unpack(w, f);
}
__device__ __forceinline__ void rec_unpack(const int64_t (&w)[NUM_RW], NodeFast& f) {
#pragma unroll
  for (int v = 0; v < 2; v++)
#pragma unroll
    for (int q = 0; q < 2; q++) {
      f.fh[v][q] = w[RW_FH + 2 * v + q];
      f.sa[v][q] = __longlong_as_double(w[RW_SA + 2 * v + q]);
    }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    f.cap[q] = __longlong_as_double(w[RW_CAP + q]);
    f.rcap[q] = __longlong_as_double(w[RW_RCAP + q]);
    f.al[q] = __longlong_as_double(w[RW_AL + q]);
    f.ral[q] = __longlong_as_double(w[RW_RAL + q]);
    f.nreq[q] = __longlong_as_double(w[RW_NREQ + q]);
  }
  f.nreq0s = __longlong_as_double(w[RW_NREQ0S]);
  f.nalloc0 = w[RW_NALLOC0];
  f.csm = w[RW_CSM];
  f.csaf = w[RW_CSAF];
  f.ut = w[RW_UT];
  f.nflags = (uint32_t)w[RW_FLAGS];
  f.sbits = (uint32_t)((uint64_t)w[RW_FLAGS] >> 32);
  f.nws = (int32_t)w[RW_NWS];
}

// write a record back (the Reserve-dependent words; the static ones never change)
template <int SCOPE>
__device__ __forceinline__ void rec_store_dyn(int64_t* rec, const NodeFast& f) {
#pragma unroll
  for (int v = 0; v < 2; v++)
#pragma unroll
    for (int q = 0; q < 2; q++) {
      __hip_atomic_store(rec + RW_FH + 2 * v + q, f.fh[v][q], __ATOMIC_RELAXED, SCOPE);
      __hip_atomic_store(rec + RW_SA + 2 * v + q, (int64_t)__double_as_longlong(f.sa[v][q]), __ATOMIC_RELAXED, SCOPE);
    }
#pragma unroll
  for (int q = 0; q < 2; q++)
    __hip_atomic_store(rec + RW_NREQ + q, (int64_t)__double_as_longlong(f.nreq[q]), __ATOMIC_RELAXED, SCOPE);
  __hip_atomic_store(rec + RW_NREQ0S, (int64_t)__double_as_longlong(f.nreq0s), __ATOMIC_RELAXED, SCOPE);
}

// a full record with the node index in RW_PAD
template <typename W>
__device__ __forceinline__ void rec_to_words(const NodeFast& f, int node, W& w) {
#pragma unroll
  for (int v = 0; v < 2; v++)
#pragma unroll
    for (int q = 0; q < 2; q++) {
      w[RW_FH + 2 * v + q] = f.fh[v][q];
      w[RW_SA + 2 * v + q] = __double_as_longlong(f.sa[v][q]);
    }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    w[RW_CAP + q] = __double_as_longlong(f.cap[q]);
    w[RW_RCAP + q] = __double_as_longlong(f.rcap[q]);
    w[RW_AL + q] = __double_as_longlong(f.al[q]);
    w[RW_RAL + q] = __double_as_longlong(f.ral[q]);
    w[RW_NREQ + q] = __double_as_longlong(f.nreq[q]);
  }
  w[RW_NREQ0S] = __double_as_longlong(f.nreq0s);
  w[RW_NALLOC0] = f.nalloc0;
  w[RW_CSM] = f.csm;
  w[RW_CSAF] = f.csaf;
  w[RW_UT] = f.ut;
  w[RW_FLAGS] = (int64_t)(((uint64_t)f.sbits << 32) | f.nflags);
  w[RW_NWS] = f.nws;
  w[RW_PAD] = node;
}
// ... stored sc1: the compact changed list k_fixup reads
__device__ __forceinline__ void rec_store_full(int64_t* r, const NodeFast& f, int node) {
  int64_t w[NUM_RW];
  rec_to_words(f, node, w);
#pragma unroll
  for (int u = 0; u < NUM_RW; u++) st_sc1(r + u, w[u]);
}

// the owner lane's Reserve of pod p (load_aware.go:192-195, NodeInfo.Requested += requests): the same
// updates k_resolve's int64 path makes, the doubles moved by the same exact amounts
__device__ __forceinline__ void fast_reserve(NodeFast& f, const DevPod& p, const double (&estd)[2],
                                             const double (&reqd)[2]) {
  const uint32_t nf = f.nflags;
  if ((nf & NF_HAS_METRIC) && !(nf & NF_NM_NIL)) {
#pragma unroll
    for (int q = 0; q < 2; q++) {
      if (nf & nf_fh_on(0, q)) f.fh[0][q] -= p.est[q];
      f.sa[0][q] -= estd[q];
      if (p.flags & PF_PROD) {
        if (nf & nf_fh_on(1, q)) f.fh[1][q] -= p.est[q];
        f.sa[1][q] -= estd[q];
      }
    }
  }
  f.nreq[0] += reqd[0];
  f.nreq[1] += reqd[1];
  f.nreq0s += reqd[0];
  fast_bounds(f);
}

// x * 100 / c on the fast range, x and c exact doubles (div100_f without the int64 -> double step)
__device__ __forceinline__ int32_t div100_d(double x, double dc, double rc) {
  const double dx = x * 100.0;
  const int32_t q = (int32_t)(dx * rc);
  const double t = (double)q * dc;
  return q - (int32_t)(t > dx) + (int32_t)(t + dc <= dx);
}

// lite_total(n, expired, p, k) from the node's record (fast_adopt'ed, current).  `estd` / `reqd`: the
// pod's estimate / requests as doubles.
template <bool EXT = true>
__device__ __forceinline__ int32_t fast_total(const NodeFast& f, const DevPod& p, const double (&estd)[2],
                                              const double (&reqd)[2], const KArgs& k) {
  const uint32_t b = f.bits, pf = p.flags;
  bool fail = (b & FB_FAIL) | ((pf & PF_DS_INVALID) != 0);
  const bool pp = (pf & PF_PROD) != 0;  // pod-uniform: scalar selects
  if (!(pf & PF_DAEMONSET))
    fail |= ((b & FB_EXP_FAIL) != 0) | (p.est[0] > (pp ? f.thr[1][0] : f.thr[0][0])) |
            (p.est[1] > (pp ? f.thr[1][1] : f.thr[0][1]));
  if (!(pf & PF_NUMA_SKIP) & (p.req[0] != 0)) fail |= ((b & FB_AMP_BAD) != 0) | (p.req[0] > f.amp_room);
  if (EXT && (k.flags & AF_FIT_FILTER)) {  // NodeResourcesFit.Filter on the record's exact doubles
    const bool co = (p.req[0] > 0) & (reqd[0] > f.al[0] - f.nreq[0]);
    const bool mo = (p.req[1] > 0) & (reqd[1] > f.al[1] - f.nreq[1]);
    fail |= fit_filter(f.room, f.xa, f.xr, co, mo, p, k) != 0;
  }
  // LoadAwareScheduling.Score
  const bool vs = (pf & PF_LA_SCORE_PROD) != 0;
  int32_t sl = 0;
  double xs[4];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const double room = (vs ? f.sa[1][q] : f.sa[0][q]) - estd[q];
    xs[q] = room;
    const bool use = ((b & (FB_CAP0 << q)) != 0) & (room >= 0.0);
    sl += (use ? div100_d(room, f.cap[q], f.rcap[q]) : 0) * k.w_la[q];
  }
  // NodeNUMAResource.Score (policy None)
  const bool rs = p.req[0] != 0;
  const bool zero = ((pf & PF_NUMA_SKIP) != 0) | ((b & FB_NZERO) != 0) | (rs & ((b & FB_RSZERO) != 0));
  const bool most = (k.flags & AF_NUMA_MOST) != 0;
  const double rq[2] = {(rs ? f.nreq0s : f.nreq[0]) + reqd[0], f.nreq[1] + reqd[1]};
  int32_t sn = 0;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const bool on = ((b & (FB_AL0 << q)) != 0) & (k.w_numa[q] != 0);
    const double x = most ? fmin(rq[q], f.al[q]) : f.al[q] - rq[q];
    xs[2 + q] = x;
    sn += (on & (most | (rq[q] <= f.al[q]))) ? div100_d(x, f.al[q], f.ral[q]) * k.w_numa[q] : 0;
  }
  if (b & FB_SLOW) {  // exec-masked, rare: capacities >= 2^42, the int64 division (as lite_total)
    sl = sn = 0;
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const bool use = ((b & (FB_CAP0 << q)) != 0) & (xs[q] >= 0.0);
      sl += (use ? (int32_t)((int64_t)xs[q] * 100 / (int64_t)f.cap[q]) : 0) * k.w_la[q];
      const bool on = ((b & (FB_AL0 << q)) != 0) & (k.w_numa[q] != 0);
      sn += (on & (most | (rq[q] <= f.al[q]))) ? (int32_t)((int64_t)xs[2 + q] * 100 / (int64_t)f.al[q]) * k.w_numa[q] : 0;
    }
  }
  const int32_t la = (b & FB_LAS) ? div_small(sl, k.wsum_la) : 0;
  const int32_t nu = (!zero & (f.nws > 0)) ? div_small(sn, f.nws) : 0;
  if (fail) return -1;
  int32_t tot = k.wp_la * la + k.wp_numa * nu;
  if (EXT && (k.flags & AF_EXT)) tot += ext_score_vals(f.xm, f.xa, f.xr, p, k);
  return tot;
}

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
__global__ void k_scatter_rows(SoA s, const Row* __restrict__ rows, const int32_t* __restrict__ idx, int n, KArgs k,
                               const int32_t* __restrict__ gate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n || (gate && *gate)) return;
  const int64_t i = idx[t];
  const Row& r = rows[t];
#pragma unroll
  for (int f = 0; f < NUM_I64_FIELDS; f++) s.f[f * s.stride + i] = r.f[f];
  s.flags[i] = r.flags;
  NodeRegs nr;  // the node's replay record
  regs_from_row(r, nr);
  prepare_row(nr);
  int64_t w[NUM_RW];
  rec_from_regs(nr, k, w);
#pragma unroll
  for (int u = 0; u < NUM_RW; u++) s.rec[i * NUM_RW + u] = w[u];
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

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v);
__device__ __forceinline__ int lanes_below(uint64_t m);

// Append `item` to a deferred-pair list (one atomic per wavefront).
__device__ __forceinline__ void defer_push(bool want, uint64_t item, uint64_t* __restrict__ list, uint32_t* cnt) {
  const uint64_t bal = __ballot(want);
  if (!bal) return;
  const int leader = __ffsll((unsigned long long)bal) - 1;
  uint32_t base = 0;
  if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(cnt, (uint32_t)__popcll(bal));
  base = __shfl(base, leader, 64);
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
  if (want) list[base + below] = item;
}

// parity mode: full status / score matrices [pod][node]; `total` holds the LoadAware + NUMA part
// until k_parity_finalize adds the normalized DeviceShare score.  dsmax[p] = 1 + max raw DeviceShare
// score over the pod's feasible nodes (DefaultNormalizeScore's maxCount).
template <bool NUMA, bool CPU>
__global__ __launch_bounds__(EVAL_BLOCK) void k_eval_parity(SoA s, int n_nodes, const DevPod* __restrict__ pods,
                                                            int n_pods, int pods_per_block, KArgs k,
                                                            uint8_t* status, uint8_t* reason, int16_t* la,
                                                            int16_t* numa, int16_t* ds, int16_t* total,
                                                            uint32_t* dsmax, uint64_t* defer_list,
                                                            uint32_t* defer_cnt) {
  const int i = blockIdx.x * EVAL_BLOCK + threadIdx.x;
  const bool live = i < n_nodes;
  NodeRegs n;
  if (live) {
    load_row(s, i, n);
    prepare_row(n);
  }
  const bool expired = live ? node_expired(n, k) : false;
  NumaNode nv;
  if (NUMA && live) numa_load(s, i, nv);  // a pod's own policy reaches nodes without one
  const int p0 = blockIdx.y * pods_per_block;
  const int p1 = min(n_pods, p0 + pods_per_block);
  for (int p = p0; p < p1; p++) {
    uint32_t m = 0;
    bool deferred = false;
    if (live) {
      const EvalOut o = eval_pair<true, NUMA, NUMA, false, CPU, true>(n, expired, pods[p], k, s, i, nv);
      deferred = NUMA && o.status == STATUS_DEFERRED;
      const int64_t o_idx = (int64_t)p * n_nodes + i;
      status[o_idx] = o.status;
      reason[o_idx] = o.reason;
      la[o_idx] = o.la;
      numa[o_idx] = o.numa;
      ds[o_idx] = o.ds;
      total[o_idx] = (int16_t)o.total;
      m = o.total >= 0 ? (uint32_t)o.ds + 1 : 0u;
    }
    if (NUMA) defer_push(deferred, ((uint64_t)p << 32) | (uint32_t)i, defer_list, defer_cnt);
    m = __ockl_wfred_max_u32(m);
    if ((threadIdx.x & 63) == 0 && m) atomicMax(&dsmax[p], m);
  }
}

// DeviceShare NormalizeScore (DefaultNormalizeScore(MaxNodeScore, false): score*100/max when max > 0)
__device__ __forceinline__ int32_t ds_norm(int32_t raw, uint32_t dsmax1) {
  const int32_t mx = dsmax1 > 0 ? (int32_t)dsmax1 - 1 : 0;
  return mx > 0 ? raw * 100 / mx : raw;
}

// normalized DeviceShare score into the weighted sum, then selectHost's packed-key max per pod
__global__ __launch_bounds__(EVAL_BLOCK) void k_parity_finalize(int n_nodes, KArgs k, const int16_t* ds,
                                                                int16_t* total, const uint32_t* dsmax,
                                                                uint32_t* best_key) {
  const int i = blockIdx.x * EVAL_BLOCK + threadIdx.x;
  const int p = blockIdx.y;
  uint32_t key = 0;
  if (i < n_nodes) {
    const int64_t o = (int64_t)p * n_nodes + i;
    int32_t t = total[o];
    if (t >= 0) {
      t += k.wp_ds * ds_norm(ds[o], dsmax[p]);
      total[o] = (int16_t)t;
    }
    key = make_key(t, i);
  }
  key = __ockl_wfred_max_u32(key);
  if ((threadIdx.x & 63) == 0 && key) atomicMax(&best_key[p], key);
}

// batch mode: 9-bit score per (pod,node): (total+1) or 0 when filtered out; for a DeviceShare pod
// (always alone in its batch) also dsraw[node] = raw DeviceShare score + 1 (0 when filtered out).
// Nodes [lo, hi) of the SoA (this rank's shard); scores stay indexed by the global node index.
// DS: the batch's pod is a DeviceShare pod (the DeviceShare path stays out of plain batches' code).
template <bool DS, bool NUMA, bool CPU, bool EXT = false, bool H = false>
__global__ __launch_bounds__(EVAL_BLOCK) void k_eval_batch(SoA s, int lo, int hi, const DevPod* __restrict__ pods,
                                                           const int32_t* __restrict__ batch_base, int batch_pods,
                                                           int pods_per_block, KArgs k, uint16_t* __restrict__ scores,
                                                           int64_t score_stride, uint16_t* __restrict__ dsraw,
                                                           uint64_t* __restrict__ defer_list, uint32_t* defer_cnt,
                                                           uint8_t* __restrict__ aff_out, uint32_t* __restrict__ dsmax1,
                                                           uint64_t* __restrict__ stamp) {
  // a plain batch's eval-start stamp (per-pod latency counts from here; else k_batch_begin wrote it)
  if (stamp && (blockIdx.x | blockIdx.y | threadIdx.x) == 0) stamp[0] = __builtin_amdgcn_s_memrealtime();
  // XCD-aware block mapping (eval_grid): workgroups are dealt to the 8 XCDs round-robin by linear id,
  // so every pod group of one node tile is given ids of the same residue mod 8 — the tile's rows are
  // fetched into one XCD's L2 once instead of once per pod group.
  const int G = (int)gridDim.y;
  const int b = (int)(blockIdx.x + blockIdx.y * gridDim.x), r = b >> 3;
  const int tile = (r / G) * 8 + (b & 7), group = r % G;
  const int i = lo + tile * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  NodeRegs n;
  load_row(s, i, n);
  prepare_row(n);
  const bool expired = node_expired(n, k);
  NumaNode nv;
  if (NUMA) numa_load(s, i, nv);  // a pod's own policy reaches nodes without one
  const int base = *batch_base;
  const int p0 = group * pods_per_block;
  const int p1 = min(batch_pods, p0 + pods_per_block);
  for (int p = p0; p < p1; p++) {
    const DevPod& pod = pods[base + p];
    if constexpr (!DS && !NUMA && !CPU) {  // plain batch: straight-line evaluation
      int32_t tot = lite_total(n, expired, pod, k);
      if (EXT && tot >= 0 && (k.flags & AF_FIT_FILTER) && fit_filter_row(s, i, n, pod, k)) tot = -1;
      if (EXT && tot >= 0) tot += ext_score(s, i, pod, k);  // FitPlus / SRA / Fit: its own variant
      scores[(int64_t)p * score_stride + i] = (uint16_t)(tot + 1);
      continue;
    }
    const EvalOut o = eval_pair<DS, NUMA, NUMA, false, CPU, H>(n, expired, pod, k, s, i, nv);
    scores[(int64_t)p * score_stride + i] = (uint16_t)(o.total + 1);
    if (NUMA) defer_push(o.status == STATUS_DEFERRED, ((uint64_t)p << 32) | (uint32_t)i, defer_list, defer_cnt);
    if (DS && (pod.flags & PF_DS)) {  // DefaultNormalizeScore's max: 1 + max raw score over feasible nodes
      const uint32_t r = o.total >= 0 ? (uint32_t)(o.ds + 1) : 0u;
      dsraw[(int64_t)p * score_stride + i] = (uint16_t)r;
      const uint32_t m = __ockl_wfred_max_u32(r);
      if ((threadIdx.x & 63) == 0 && m) atomicMax(dsmax1 + p, m);
    } else if (DS) {  // a plain pod of a DeviceShare batch: raw 0, no normalisation
      dsraw[(int64_t)p * score_stride + i] = (uint16_t)(o.total >= 0 ? 1u : 0u);
    }
    if (CPU && NUMA) aff_out[i] = o.aff;  // singleton batch: the affinity its Reserve allocates on
  }
}

// Plain batches (LoadAware + NodeNUMAResource policy None, FitPlus / SRA when EXT): each lane adopts its
// node's replay record (13 16-byte loads + fast_adopt, once per pod group) and scores the group's pods
// with fast_total — k_resolve's exact re-evaluation, equal to lite_total (+ ext_score): the Reserve-
// dependent words are exact doubles, so no int64 -> double conversion or 64-bit subtraction is left per
// (pod, node).  The pods' estimates / requests as doubles are converted once per block into LDS.
// Records are written sc1 by the Reserve kernels, so a pipelined eval sees them like the SoA rows.
constexpr int EVAL_PPB = 8;  // pods per block (eval_grid's pod groups)
// A plain batch of more than 2 pods is evaluated from the 208-B replay records (k_eval_plain: no int64 ->
// double work per pair, the record read once per 8 pods); 1-2 pods stream the 148-B SoA rows
// (k_eval_batch), the smaller read when the pass is bandwidth-bound.
__host__ __device__ constexpr bool use_record_eval(int pods) { return pods > 2; }
template <bool EXT>
__global__ __launch_bounds__(EVAL_BLOCK) void k_eval_plain(SoA s, int lo, int hi, const DevPod* __restrict__ pods,
                                                           const int32_t* __restrict__ batch_base, int batch_pods,
                                                           KArgs k, uint16_t* __restrict__ scores, int64_t score_stride,
                                                           uint64_t* __restrict__ stamp, const int32_t* __restrict__ done_wait,
                                                           int32_t* __restrict__ err) {
  if (done_wait) {  // pipelined: the Reserves of batch b-2 first (every workgroup sees the flag itself)
    __shared__ int32_t s_go;
    if (threadIdx.x == 0) s_go = wait_at_least(done_wait, 1, err);
    __syncthreads();
    if (!s_go) return;  // (a timed-out hand-off: the host discards the queue)
  }
  if (stamp && (blockIdx.x | blockIdx.y | threadIdx.x) == 0) stamp[0] = __builtin_amdgcn_s_memrealtime();
  const int G = (int)gridDim.y;
  const int b = (int)(blockIdx.x + blockIdx.y * gridDim.x), r = b >> 3;
  const int tile = (r / G) * 8 + (b & 7), group = r % G;  // XCD-aware, as k_eval_batch
  const int i = lo + tile * blockDim.x + threadIdx.x;
  const int base = *batch_base;
  const int p0 = group * EVAL_PPB;
  const int np = min(batch_pods, p0 + EVAL_PPB) - p0;
  // the group's pods in LDS once per block: the estimates / requests as doubles, and (without the ext terms) the
  // flags and integer estimates / cpu request fast_total reads -- no scalar-memory load (and its wait) per pod
  __shared__ double s_pd[EVAL_PPB][4];
  __shared__ int64_t s_pi[EVAL_PPB][3];
  __shared__ uint32_t s_pf[EVAL_PPB];
  if ((int)threadIdx.x < 4 * np) {
    const int q = threadIdx.x >> 2, c = threadIdx.x & 3;
    const DevPod& pp = pods[base + p0 + q];
    s_pd[q][c] = (double)(c < 2 ? pp.est[c] : pp.req[c - 2]);
    if (!EXT && c < 3) s_pi[q][c] = c < 2 ? pp.est[c] : pp.req[0];
    if (!EXT && c == 3) s_pf[q] = pp.flags;
  }
  __syncthreads();
  if (i >= hi) return;
  NodeFast f;
  rec_load_plain(s.rec + (int64_t)i * NUM_RW, f);
  if (EXT && (k.flags & AF_EXT)) ext_load(s, i, k, f);
  fast_adopt(f, k);
  uint16_t* const out = scores + (int64_t)p0 * score_stride + i;
  for (int q = 0; q < np; q++) {
    const double ed[2] = {s_pd[q][0], s_pd[q][1]}, rd[2] = {s_pd[q][2], s_pd[q][3]};
    int32_t t;
    if constexpr (EXT) {
      t = fast_total<EXT>(f, pods[base + p0 + q], ed, rd, k);
    } else {
      DevPod pl;  // (fast_total<false> reads these fields only)
      pl.flags = s_pf[q];
      pl.est[0] = s_pi[q][0];
      pl.est[1] = s_pi[q][1];
      pl.req[0] = s_pi[q][2];
      t = fast_total<false>(f, pl, ed, rd, k);
    }
    out[(int64_t)q * score_stride] = (uint16_t)(t + 1);
  }
}

// Batch b's scores of the nodes batch b-2 changed (stale-list runs on two eval streams): batch
// b's eval waited only for batch b-3's done flag; once done[b-2] is published (a k_handoff ahead of this kernel)
// lane t of workgroup j re-evaluates node t of batch b-2's changed list (written with its rows, drained before
// the flag) for pod j from its record, as k_eval_plain does -- the lists then see every Reserve of batches <= b-2.
template <bool EXT>
__global__ __launch_bounds__(64) void k_patch(SoA s, const DevPod* __restrict__ pods, const int32_t* __restrict__ batch_base,
                                              KArgs k, const int32_t* __restrict__ tlist, uint16_t* __restrict__ scores,
                                              int64_t score_stride, const int32_t* __restrict__ done_wait,
                                              int32_t* __restrict__ err) {
  const int j = blockIdx.x, t = threadIdx.x;
  {  // batch b-2's done flag (each one-wave workgroup polls it: no separate wait kernel ahead of this one)
    __shared__ int32_t s_go;
    if (t == 0) s_go = wait_at_least(done_wait, 1, err);
    __syncthreads();
    if (!s_go) return;  // (a timed-out hand-off: the host discards the queue)
  }
  const int n = ld_sc1(tlist);
  if (t >= n) return;
  const int node = ld_sc1(tlist + 1 + t);
  NodeFast f;
  rec_load<__HIP_MEMORY_SCOPE_AGENT>(s.rec + (int64_t)node * NUM_RW, f);
  if (EXT && (k.flags & AF_EXT)) ext_load(s, node, k, f);
  fast_adopt(f, k);
  const DevPod pod = pods[*batch_base + j];
  const double ed[2] = {(double)pod.est[0], (double)pod.est[1]}, rd[2] = {(double)pod.req[0], (double)pod.req[1]};
  scores[(int64_t)j * score_stride + node] = (uint16_t)(fast_total<EXT>(f, pod, ed, rd, k) + 1);
}

// selectHost for a singleton batch: the best packed key over nodes [lo, hi) (ties to the lowest node
// index), one atomicMax per wave; cand[0] must be zero on entry, cand_cnt[0] becomes 1.
template <bool DS>
__global__ __launch_bounds__(256) void k_argmax1(const uint16_t* __restrict__ scores, int lo, int hi,
                                                 const uint16_t* __restrict__ dsraw, const uint32_t* __restrict__ dsmax1,
                                                 int32_t wds, uint32_t* __restrict__ cand, int32_t* __restrict__ cand_cnt) {
  const int i = lo + blockIdx.x * 256 + threadIdx.x;
  uint32_t key = 0;
  if (i < hi) {
    uint32_t v = scores[i];  // total + 1, 0 = filtered out
    if (DS && v) v += (uint32_t)(wds * ds_norm((int32_t)dsraw[i] - 1, *dsmax1));
    key = v ? (v << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)i) : 0u;
  }
  key = __ockl_wfred_max_u32(key);
  if ((threadIdx.x & 63) == 0 && key) atomicMax(cand, key);
  if (blockIdx.x == 0 && threadIdx.x == 0) cand_cnt[0] = 1;
}

// The Reservation plugin for a singleton batch whose pod matches reservations, after
// k_argmax1: one wave over the K nodes holding matched reservations (the other nodes score 0).
//   1. PreScore's preferredNode (reservation/scoring.go:97-107): the feasible node with the smallest
//      reservation order != 0, ties -> lowest node index; it scores mostPreferredScore 1000 (:118-120);
//   2. DefaultNormalizeScore (:134-139): n = 100 * raw / max over the feasible nodes (all 0 when max is 0);
//   3. selectHost over total + w * n: a 64-bit key over the K nodes against k_argmax1's winner (n = 0).
// cand[0] becomes the winner's 32-bit key (its plugin total without the Reservation part); out = {winner
// node or -1, its n, max, preferredNode or -1}.
// With a reservation affinity only the pairs' allowed nodes pass the Reservation Filter: k_argmax1's winner
// does not count and the others are infeasible.
// A DeviceShare pod (dsraw != nullptr): a node's plugin total includes DeviceShare's normalized score, as in
// k_argmax1.  A winner whose pair carries RSV_PAIR_RESERVE_FAILS is not placed (its DeviceShare Reserve fails).
// A reservation-matched pod fused behind the plain pods of its ke_schedule segment: its nomination and
// rows were taken on the host before those pods ran, valid unless one of them was placed on a node of its reservations
// (their Requested / pod count / assign cache feed fitsNode and the rows).  k_rsv_check sets *gate then; the gated
// scatters keep the plain rows, k_rsv_gate_apply empties the pod's candidates (its Reserve places nothing) and the
// host runs the pod again as a segment of its own.
__global__ __launch_bounds__(256) void k_rsv_check(const int32_t* __restrict__ chosen, int n_prev,
                                                   const RsvPair* __restrict__ pr, int K, int32_t global_offset,
                                                   int32_t* __restrict__ gate) {
  __shared__ int32_t hit;
  if (threadIdx.x == 0) hit = 0;
  __syncthreads();
  for (int i = (int)threadIdx.x; i < n_prev; i += (int)blockDim.x) {
    const int32_t c = chosen[i];
    if (c < 0) continue;
    for (int q = 0; q < K; q++)
      if (pr[q].node + global_offset == c) hit = 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) *gate = hit;
}
__global__ void k_rsv_gate_apply(const int32_t* __restrict__ gate, int32_t* __restrict__ cand_cnt) {
  if (threadIdx.x == 0 && *gate) cand_cnt[0] = 0;
}

__global__ __launch_bounds__(64) void k_rsv_pick(const uint16_t* __restrict__ scores, const RsvPair* __restrict__ pr,
                                                 int K, int64_t w, int affinity, uint32_t* __restrict__ cand,
                                                 int32_t* __restrict__ out, const uint16_t* __restrict__ dsraw,
                                                 const uint32_t* __restrict__ dsmax1, int32_t wds) {
  const int l = (int)threadIdx.x;
  auto feasible = [&](const RsvPair& q) { return scores[q.node] != 0 && (q.allowed & RSV_PAIR_ALLOWED) != 0; };
  auto total = [&](int32_t node) -> uint32_t {
    uint32_t v = scores[node];
    if (dsraw && v) v += (uint32_t)(wds * ds_norm((int32_t)dsraw[node] - 1, *dsmax1));
    return v;
  };
  int64_t bo = INT64_MAX;
  int32_t bn = INT32_MAX;
  for (int i = l; i < K; i += 64) {
    const RsvPair q = pr[i];
    if (q.order != 0 && feasible(q) && (q.order < bo || (q.order == bo && q.node < bn))) {
      bo = q.order;
      bn = q.node;
    }
  }
  for (int m = 32; m; m >>= 1) {
    const int64_t o2 = __shfl_xor(bo, m);
    const int32_t n2 = __shfl_xor(bn, m);
    if (o2 < bo || (o2 == bo && n2 < bn)) {
      bo = o2;
      bn = n2;
    }
  }
  const int32_t pref = bo == INT64_MAX ? -1 : bn;
  int32_t mx = 0;
  for (int i = l; i < K; i += 64) {
    const RsvPair q = pr[i];
    if (feasible(q)) mx = max(mx, q.node == pref ? 1000 : (int32_t)q.raw);
  }
  for (int m = 32; m; m >>= 1) mx = max(mx, __shfl_xor(mx, m));
  const uint32_t g = affinity ? 0u : cand[0];  // k_argmax1's key: (total + 1) << KEY_IDX_BITS | (mask - node)
  uint64_t best = g;
  if (mx > 0 || affinity)
    for (int i = l; i < K; i += 64) {
      const RsvPair q = pr[i];
      const uint32_t v = total(q.node);
      if (!feasible(q)) continue;
      const int64_t n = mx > 0 ? 100 * (int64_t)(q.node == pref ? 1000 : q.raw) / mx : 0;
      const uint64_t key = ((uint64_t)(v + w * n) << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)q.node);
      best = key > best ? key : best;
    }
  for (int m = 32; m; m >>= 1) {
    const uint64_t o = __shfl_xor(best, m);
    best = o > best ? o : best;
  }
  const int32_t win = best ? (int32_t)(KEY_IDX_MASK - (uint32_t)(best & KEY_IDX_MASK)) : -1;
  int32_t nw = 0, fails = 0;  // the winner's n (0 unless it holds matched reservations), its Reserve failing
  for (int i = l; i < K; i += 64) {
    const RsvPair q = pr[i];
    if (q.node == win && mx > 0) nw = (int32_t)(100 * (int64_t)(q.node == pref ? 1000 : q.raw) / mx);
    if (q.node == win && (q.allowed & RSV_PAIR_RESERVE_FAILS)) fails = 1;
    if ((q.allowed & RSV_PAIR_SCORE_ERROR) && feasible(q)) fails = 1;  // RunScorePlugins' error: no placement
  }
  for (int m = 32; m; m >>= 1) nw = max(nw, __shfl_xor(nw, m)), fails = max(fails, __shfl_xor(fails, m));
  if (l == 0) {
    const bool placed = win >= 0 && !fails;
    cand[0] = placed ? (total(win) << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)win) : 0u;
    out[0] = placed ? win : -1;
    out[1] = nw;
    out[2] = mx;
    out[3] = pref;
  }
}

// k_rsv_pick across node shards (the pod's reservation nodes may live on any rank; every rank replays the same
// Reserve, so every rank needs the same winner): the same steps in stages over the pairs of this rank's node range
// [lo, hi) (loopback: every node), each stage's word made global by an all-reduce between the launches --
//   0: the smallest order != 0 of a feasible pair (MIN)        1: the smallest such node with it (MIN)
//   2: mx over the feasible pairs, preferredNode at 1000 (MAX)  3: the best 64-bit key against the merged lists' top
//   4: the winner's total and n from the rank that owns it (MAX) 5: cand[0] and the result words, as k_rsv_pick.
struct RsvPickSt {
  int64_t order;
  int32_t node, mx;
  uint64_t best;
  int32_t wt, nw;
};
template <int S>
__global__ __launch_bounds__(64) void k_rsv_stage(const uint16_t* __restrict__ scores, const RsvPair* __restrict__ pr,
                                                  int K, int lo, int hi, int64_t w, int affinity,
                                                  uint32_t* __restrict__ cand, RsvPickSt* __restrict__ st,
                                                  int32_t* __restrict__ out, const uint16_t* __restrict__ dsraw,
                                                  const uint32_t* __restrict__ dsmax1, int32_t wds) {
  const int l = (int)threadIdx.x;
  auto mine = [&](const RsvPair& q) {
    return q.node >= lo && q.node < hi && scores[q.node] != 0 && (q.allowed & RSV_PAIR_ALLOWED) != 0;
  };
  auto total = [&](int32_t node) -> uint32_t {  // as k_rsv_pick
    uint32_t v = scores[node];
    if (dsraw && v) v += (uint32_t)(wds * ds_norm((int32_t)dsraw[node] - 1, *dsmax1));
    return v;
  };
  const int32_t pref = S >= 2 ? (st->order == INT64_MAX ? -1 : st->node) : -1;
  if constexpr (S == 0) {
    int64_t bo = INT64_MAX;
    for (int i = l; i < K; i += 64)
      if (pr[i].order != 0 && mine(pr[i])) bo = min(bo, pr[i].order);
    for (int m = 32; m; m >>= 1) bo = min(bo, (int64_t)__shfl_xor(bo, m));
    if (l == 0) st->order = bo;
  } else if constexpr (S == 1) {
    int32_t bn = INT32_MAX;
    for (int i = l; i < K; i += 64)
      if (st->order != INT64_MAX && pr[i].order == st->order && mine(pr[i])) bn = min(bn, pr[i].node);
    for (int m = 32; m; m >>= 1) bn = min(bn, __shfl_xor(bn, m));
    if (l == 0) st->node = bn;
  } else if constexpr (S == 2) {
    int32_t mx = 0;
    for (int i = l; i < K; i += 64)
      if (mine(pr[i])) mx = max(mx, pr[i].node == pref ? 1000 : (int32_t)pr[i].raw);
    for (int m = 32; m; m >>= 1) mx = max(mx, __shfl_xor(mx, m));
    if (l == 0) st->mx = mx;
  } else if constexpr (S == 3) {
    const int32_t mx = st->mx;
    uint64_t best = affinity ? 0u : cand[0];  // the merged lists' top: (total + 1) << KEY_IDX_BITS | (mask - node)
    if (mx > 0 || affinity)
      for (int i = l; i < K; i += 64) {
        const RsvPair q = pr[i];
        if (!mine(q)) continue;
        const int64_t n = mx > 0 ? 100 * (int64_t)(q.node == pref ? 1000 : q.raw) / mx : 0;
        const uint64_t key = ((uint64_t)(total(q.node) + w * n) << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)q.node);
        best = key > best ? key : best;
      }
    for (int m = 32; m; m >>= 1) {
      const uint64_t o = __shfl_xor(best, m);
      best = o > best ? o : best;
    }
    if (l == 0) st->best = best;
  } else if constexpr (S == 4) {
    const uint64_t best = st->best;
    const int32_t win = best ? (int32_t)(KEY_IDX_MASK - (uint32_t)(best & KEY_IDX_MASK)) : -1;
    int32_t nw = 0;
    if (win >= 0 && st->mx > 0)
      for (int i = l; i < K; i += 64)
        if (pr[i].node == win && win >= lo && win < hi)
          nw = (int32_t)(100 * (int64_t)(pr[i].node == pref ? 1000 : pr[i].raw) / st->mx);
    for (int i = l; i < K; i += 64)  // a feasible pair of this range whose Score errs: bit 30, carried by the MAX
      if ((pr[i].allowed & RSV_PAIR_SCORE_ERROR) && mine(pr[i])) nw |= 1 << 30;
    for (int m = 32; m; m >>= 1) nw = max(nw, __shfl_xor(nw, m));
    if (l == 0) {
      st->wt = win >= lo && win < hi ? (int32_t)total(win) : 0;
      st->nw = nw;
    }
  } else {
    if (l == 0) {
      const uint64_t best = st->best;
      int32_t win = best ? (int32_t)(KEY_IDX_MASK - (uint32_t)(best & KEY_IDX_MASK)) : -1;
      for (int i = 0; win >= 0 && i < K; i++)  // (every rank holds every pair)
        if (pr[i].node == win && (pr[i].allowed & RSV_PAIR_RESERVE_FAILS)) win = -1;
      if ((st->nw >> 30) & 1) win = -1;  // a Score error on some rank's feasible node
      cand[0] = win >= 0 ? ((uint32_t)st->wt << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)win) : 0u;
      out[0] = win;
      out[1] = st->nw & ~(1 << 30);
      out[2] = st->mx;
      out[3] = pref;
    }
  }
}

// The deferred BestEffort pairs of an eval launch: one wavefront per pair computes mergeFilteredHints
// over the full provider lists (numa_best_effort_fallback's result), then lane 0 evaluates the pair
// with it.  A DeviceShare pod's pair is deferred only on a node without a device cache (DeviceShare has
// no hints there, Filter passes, Score is 0).  PARITY: write the parity matrices; else the batch score
// (and for a DeviceShare singleton its raw score + 1 into `dsraw`, the max into `dsmax`).
//   1. lanes split the 255 masks: hint lists L_cpu / L_mem (IterateBitMasks order) and hint scores;
//   2. c* = the smallest popcount of a non-empty merged mask m1 & m2: only merged hints of that size
//      can end as the best (the first one is narrower than anything before it, larger ones never
//      replace it), and between equal sizes the rule is "numerically smaller or higher score";
//   3. FB_ROWS rows of L_cpu at a time, each lane lists its row's size-c* merged hints in L_mem order
//      into LDS; lane 0 folds them in permutation order.
constexpr int FALLBACK_BLOCKS = 4096;
constexpr int FB_ROWS = 16;  // rows of L_cpu per fold chunk (LDS: several pair-waves per CU)
// CS: pods of the launch may bind CPUs — such a pair's lists come from the trimmed zones with the
// cpuset-aware split, its hint scores from the amplified requests (eval_pair's binding branch).
template <bool PARITY, bool CS = false>
__global__ __launch_bounds__(64) void k_numa_fallback(SoA s, const DevPod* __restrict__ pods,
                                                      const int32_t* __restrict__ batch_base, KArgs k,
                                                      const uint64_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                      uint16_t* __restrict__ scores, int64_t score_stride, int n_nodes,
                                                      uint8_t* status, uint8_t* reason, int16_t* la, int16_t* numa,
                                                      int16_t* ds, int16_t* total, uint32_t* dsmax,
                                                      uint8_t* __restrict__ aff_out, uint16_t* __restrict__ dsraw,
                                                      uint32_t* __restrict__ fb_out) {
  __shared__ int32_t s_score[256];     // hint score by mask value
  __shared__ uint8_t s_list[2][256];   // L_cpu / L_mem masks in order
  __shared__ uint16_t s_buf[FB_ROWS][256];  // per-row merged hints of size c*: M | k << 8 | unsatisfied << 10
  __shared__ int32_t s_cnt[FB_ROWS];
  __shared__ uint64_t s_E[2][4];       // list membership by NUMA_ORDER index (LDS: read at runtime indices)
  const int lane = threadIdx.x;
  const uint32_t n = *cnt;
  const int base = PARITY ? 0 : *batch_base;
  for (uint32_t w = blockIdx.x; w < n; w += FALLBACK_BLOCKS) {
    const uint64_t it = list[w];
    const int p = (int)(it >> 32);
    const int64_t i = (int64_t)(uint32_t)it;
    RPROF_DECL
    const DevPod pod = pods[base + p];
    NumaNode nv;
    numa_load(s, i, nv);
    NumaCs cs;
    cs.rcb = false;
    DevPod ps = pod;
    if (CS) {
      const uint32_t nf = s.flags[i];
      const bool rcb = !(pod.flags & PF_NUMA_SKIP) &&
                       ((pod.flags & PF_CPU_RCB) || (pod.req[0] != 0 && nf_cpu_bind(nf) != KE_NODE_CPU_BIND_NONE &&
                                                     (pod.flags & PF_CPU_INT)));
      if (rcb) {
        cs = numa_cs_load(s, i, nf, pod);
        ps.req[0] = amplify_bits(pod.req[0], s.cs[CS_RS * s.stride + i]);
        numa_trim(nv, cs);
      }
    }
    bool present[2];
    uint32_t lack[2];
    numa_present_lack(nv, pod, present, lack);
    RPROF(3)
    // 1. lists and scores, 64 masks (in IterateBitMasks order) per step; E[r][c]: the list membership of
    // NUMA_ORDER[64c + lane].  2. after each step lane 0 runs numa_admit's search for the preferred merged
    // hint over the hint sizes listed completely so far (same scan order and replacement rule, same lists):
    // the lists' minimum sizes, candidates in both present lists (of those sizes unless Restricted),
    // SingleNUMANode one-zone hints only.  A hint found there ends the listing.
    int len[2] = {0, 0};
    if (lane < 8) s_E[lane >> 2][lane & 3] = 0;
    const int pol = pf_numa_policy(pod.flags) ? pf_numa_policy(pod.flags) : nf_numa_policy(s.flags[i]);
    uint32_t fb = 0;
    const bool single = pol == KE_NUMA_POLICY_SINGLE_NUMA_NODE, restricted = pol == KE_NUMA_POLICY_RESTRICTED;
    const bool excl = (pod.flags & PF_NUMA_EXCL_REQ) != 0;
    const int R = (int)present[0] + (int)present[1];
    int cov_done = 0;  // hint sizes folded
    uint32_t best = 0;
    int32_t bsc = 0;
    bool found = false;
    // steps: the one- and two-zone hints (most searches end there), then 64 masks at a time
    for (int c = 0, e0 = 0; e0 < 255 && !fb; c++) {
      const int e1 = c == 0 ? NUMA_OFF[3] : min(e0 + 64, 255);
      const int e = e0 + lane;
      const uint32_t m = e < e1 ? NUMA_ORDER[e] : 0u;
      bool in[2] = {false, false};
      if (m && !(m & ~nv.zm)) {
        in[0] = present[0] && !(m & lack[0]);
        in[1] = present[1] && !(m & lack[1]);
        if ((in[0] || in[1]) && !numa_fits<CS>(nv, m, pod, &cs)) in[0] = in[1] = false;
        if (in[0] || in[1]) s_score[m] = numa_hint_score(s, i, nv, m, ps, k);
      }
#pragma unroll
      for (int r = 0; r < 2; r++) {
        const uint64_t bal = __ballot(in[r]);
        const int sh = e0 & 63;  // lane l's mask is NUMA_ORDER[e0 + l]
        if (lane == 0) {
          s_E[r][e0 >> 6] |= bal << sh;
          if (sh && (e0 >> 6) < 3) s_E[r][(e0 >> 6) + 1] |= bal >> (64 - sh);
        }
        if (in[r]) s_list[r][len[r] + lanes_below(bal)] = (uint8_t)m;
        len[r] += __popcll(bal);
      }
      __syncthreads();
      if (c == 0) {
        RPROF(4)
      }
      int covered = 0;  // hint sizes whose masks are all listed
      while (covered < 8 && NUMA_OFF[covered + 2] <= e1) covered++;
      e0 = e1;
      // fold the candidates of the sizes listed completely since the last step, in IterateBitMasks order
      // (lanes test 64 masks at a time; the fold reads the candidate lanes' registers): a larger hint
      // never replaces a smaller one, so folding every candidate equals the search's early stops
      const int top = single ? min(covered, 1) : covered;
      if (top > cov_done) {
        const int minr0 = len[0] ? __popc(s_list[0][0]) : 9, minr1 = len[1] ? __popc(s_list[1][0]) : 9;
        for (int q0 = NUMA_OFF[cov_done + 1]; q0 < NUMA_OFF[top + 1]; q0 += 64) {
          const int q = q0 + lane;
          bool cand = false;
          uint32_t mq = 0;
          int32_t sc = 0;
          if (q < NUMA_OFF[top + 1]) {
            mq = NUMA_ORDER[q];
            const int sz = __popc(mq);
            const bool in0 = (s_E[0][q >> 6] >> (q & 63)) & 1u, in1 = (s_E[1][q >> 6] >> (q & 63)) & 1u;
            cand = (in0 || in1) && (!present[0] || in0) && (!present[1] || in1);
            if (!restricted) cand = cand && (!present[0] || minr0 == sz) && (!present[1] || minr1 == sz);
            cand = cand && exclusive_ok(nv, mq, excl);
            if (cand) sc = R * s_score[mq];
          }
          for (uint64_t cb = __ballot(cand); cb; cb &= cb - 1) {
            const int l = __ffsll((long long)cb) - 1;
            const uint32_t mm = (uint32_t)__builtin_amdgcn_readlane((int)mq, l);
            const int32_t ss = __builtin_amdgcn_readlane(sc, l);
            if (!found || narrower(mm, best) || (__popc(mm) == __popc(best) && ss > bsc)) {
              best = mm;
              bsc = ss;
              found = true;
            }
          }
        }
        cov_done = top;
      }
      if (found) fb = NFB_FOUND << 8 | ((single && best == nv.zm) ? 0u : best);
      else if (e1 >= 255 && pol != KE_NUMA_POLICY_BEST_EFFORT) fb = NFB_FAIL << 8;
      if (c == 0) {
        RPROF(0)
      } else {
        RPROF(1)
      }
    }
    uint32_t aff = 0;
    if (fb) {
      // the search decided
    } else if ((present[0] && !len[0]) || (present[1] && !len[1])) {
      aff = nv.zm;  // filterProvidersHints reasons: unsatisfied -> any NUMA node
    } else if (!(present[0] && present[1])) {  // one list: the merged hint is the list's hint
      const int r = present[0] ? 0 : 1;
      uint32_t best = nv.zm;
      int32_t bsc = 0;
      if (lane == 0)
        for (int j = 0; j < len[r]; j++) {
          const uint32_t m = s_list[r][j];
          const int32_t sc = s_score[m];
          if (narrower(m, best) || (__popc(m) == __popc(best) && sc > bsc)) {
            best = m;
            bsc = sc;
          }
        }
      aff = best;
    } else {
      // 2. c*
      int cmin = 9;
      for (int j = lane; j < len[0]; j += 64) {
        const uint32_t m1 = s_list[0][j];
        for (int q = 0; q < len[1]; q++) {
          const uint32_t mg = m1 & s_list[1][q];
          if (mg) cmin = min(cmin, __popc(mg));
        }
      }
      const int cs = 9 - (int)wave_max_u32((uint32_t)(9 - cmin));
      // 3. fold the size-c* merged hints in permutation order
      uint32_t best = nv.zm;
      int32_t bsc = 0;
      bool bun = false;
      for (int r0 = 0; cs <= 8 && r0 < len[0]; r0 += FB_ROWS) {
        int c = 0;
        if (lane < FB_ROWS && r0 + lane < len[0]) {
          const uint32_t m1 = s_list[0][r0 + lane];
          for (int q = 0; q < len[1]; q++) {
            const uint32_t m2 = s_list[1][q];
            const uint32_t mg = m1 & m2;
            if ((int)__popc(mg) != cs) continue;
            const uint32_t kk = (uint32_t)(m1 == mg) + (uint32_t)(m2 == mg);
            const uint32_t un = (int)max(__popc(m1), __popc(m2)) != cs;
            s_buf[lane][c++] = (uint16_t)(mg | kk << 8 | un << 10);
          }
        }
        if (lane < FB_ROWS) s_cnt[lane] = c;
        __syncthreads();
        if (lane == 0)
          for (int t = 0; t < FB_ROWS; t++)
            for (int q = 0; q < s_cnt[t]; q++) {
              const uint32_t e = s_buf[t][q];
              const uint32_t mg = e & 0xFFu;
              const int32_t sc = (int32_t)((e >> 8) & 3u) * s_score[mg];
              if (narrower(mg, best) || (__popc(mg) == __popc(best) && sc > bsc)) {
                best = mg;
                bsc = sc;
                bun = (e >> 10) & 1u;
              }
            }
        __syncthreads();
      }
      aff = bun ? nv.zm : best;
    }
    RPROF(2)
    if (!fb) fb = NFB_BEST_EFFORT << 8 | aff;
    if (lane == 0) fb_out[w] = fb;
    RPROF_FLUSH(1, 1)
    __syncthreads();
  }
}

// The deferred pairs evaluated with their merges (k_numa_fallback's fb_in), one lane per pair: the
// Filter / Score of eval_pair with the Admit's outcome given.  PARITY: the parity matrices; else the
// batch score (and for a binding batch the affinity, for a DeviceShare singleton its raw score).
constexpr int FINISH_BLOCKS = 256;
template <bool PARITY, bool CS = false>
__global__ __launch_bounds__(64) void k_numa_finish(SoA s, const DevPod* __restrict__ pods,
                                                    const int32_t* __restrict__ batch_base, KArgs k,
                                                    const uint64_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                    uint16_t* __restrict__ scores, int64_t score_stride, int n_nodes,
                                                    uint8_t* status, uint8_t* reason, int16_t* la, int16_t* numa,
                                                    int16_t* ds, int16_t* total, uint32_t* dsmax,
                                                    uint8_t* __restrict__ aff_out, uint16_t* __restrict__ dsraw,
                                                    const uint32_t* __restrict__ fb_in) {
  const uint32_t n = *cnt;
  const int base = PARITY ? 0 : *batch_base;
  for (uint32_t w = blockIdx.x * 64 + threadIdx.x; w < n; w += FINISH_BLOCKS * 64) {
    const uint64_t it = list[w];
    const int p = (int)(it >> 32);
    const int64_t i = (int64_t)(uint32_t)it;
    const DevPod pod = pods[base + p];
    NumaNode nv;
    numa_load(s, i, nv);
    NodeRegs nr;
    load_row(s, i, nr);
    prepare_row(nr);
    const bool expired = node_expired(nr, k);
    const EvalOut o = eval_pair<false, true, false, true, CS>(nr, expired, pod, k, s, i, nv, fb_in[w]);
    if (PARITY) {
      const int64_t o_idx = (int64_t)p * n_nodes + i;
      status[o_idx] = o.status;
      reason[o_idx] = o.reason;
      la[o_idx] = o.la;
      numa[o_idx] = o.numa;
      ds[o_idx] = o.ds;
      total[o_idx] = (int16_t)o.total;
      if (o.total >= 0) atomicMax(&dsmax[p], (uint32_t)o.ds + 1);
    } else {
      scores[(int64_t)p * score_stride + i] = (uint16_t)(o.total + 1);
      if (CS && aff_out) aff_out[i] = o.aff;
      if (dsraw && (pod.flags & PF_DS)) {  // a DeviceShare singleton: its raw score (0 here) for the normalisation
        dsraw[i] = o.total >= 0 ? (uint16_t)(o.ds + 1) : (uint16_t)0;
        if (o.total >= 0) atomicMax(dsmax, (uint32_t)o.ds + 1);
      }
    }
  }
}

// ---- wave-wide primitives (DPP reductions from the device library, ballots) ---------------------
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) { return __ockl_wfred_max_u32(v); }
__device__ __forceinline__ int wave_sum(int v) { return __ockl_wfred_add_i32(v); }
__device__ __forceinline__ int lanes_below(uint64_t m) {  // popcount of m over lanes < this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}
// exclusive prefix over lanes of a small per-lane count c (0 <= c < 16) and the wave total
__device__ __forceinline__ int lane_prefix16(int c, int* total) {
  int pre = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint64_t m = __ballot((c >> b) & 1);
    pre += lanes_below(m) << b;
    tot += __popcll(m) << b;
  }
  *total = tot;
  return pre;
}

// 8 consecutive u16 values starting at node i (i % 8 == 0), 0 beyond `end`
__device__ __forceinline__ void load8_raw(const uint16_t* sc, int i, int end, uint32_t v[8]) {
  if (i + 8 <= end) {
    const uint4 q = *reinterpret_cast<const uint4*>(sc + i);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int t = 0; t < 4; t++) {
      v[2 * t] = w[t] & 0xFFFFu;
      v[2 * t + 1] = w[t] >> 16;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 8; t++) v[t] = i + t < end ? sc[i + t] : 0u;
  }
}

// DeviceShare NormalizeScore folded into the select: lut[raw] = weight * normalized(raw)
struct DsNorm {
  const uint16_t* raw;  // raw DeviceShare score + 1 per node (0 = filtered out)
  const int16_t* lut;   // LDS, MAX_DS_RAW + 1 entries
};

// 8 consecutive framework scores (total + 1, 0 = filtered out) of one pod starting at node i
template <bool DS>
__device__ __forceinline__ void load8(const uint16_t* sc, int i, int end, uint32_t v[8], const DsNorm& dn) {
  load8_raw(sc, i, end, v);
  if (DS) {
    uint32_t r[8];
    load8_raw(dn.raw, i, end, r);
#pragma unroll
    for (int t = 0; t < 8; t++) v[t] = v[t] ? v[t] + (uint32_t)dn.lut[r[t] - 1] : 0u;
  }
}

constexpr int SEL_WINDOW = 64;  // histogram window below the pod's best score
constexpr int SEL_RC = 8;       // register-resident select: up to SEL_RC * 512 nodes per wave (65,536 per pod)
constexpr int SEL_COPIES = 8;   // histogram copies per wave (pass 2)

// per-wave node segment of k_select over [lo, hi): a multiple of 512 (one 16-B load per lane per step)
__host__ __device__ inline int select_seg(int lo, int hi) { return ((hi - lo + SELECT_WAVES - 1) / SELECT_WAVES + 511) & ~511; }
// workgroups per pod of a plain batch's split k_select over n nodes: >= 256 workgroups in all, parts of
// >= 4096 nodes, at most MAX_WORLD (k_merge's fan-in)
// (parts of >= 24576 nodes: at C3's 50k nodes two parts per pod measured 93.5 G against 92.1 G with four and 91.1 G
// with one -- profiles/r06/ab_select_parts.txt; the split's merge tail costs more than the per-part pass saves.
// KOORDEVAL_SELECT_PARTS = P, an A/B knob: at most P parts of >= 4096 nodes.)
inline int select_parts(int64_t n, int bp, int L = 2 * 64) {
  const char* e = std::getenv("KOORDEVAL_SELECT_PARTS");
  const int cap = e ? std::max(1, std::min(8, std::atoi(e))) : 8;
  const int64_t per = e ? 4096 : 24576;
  return std::max(1, std::min({cap, (255 + bp) / bp, (int)(n / per), 1024 / L}));  // (the merge: parts x L <= 1024)
}
// node part of one of `parts` workgroups of a split k_select (512-aligned, like the shard ranges)
__host__ __device__ inline int select_part(int lo, int hi, int parts) { return ((hi - lo + parts - 1) / parts + 511) & ~511; }

// it = 0 .. iters-1 over a wave's 512-node steps; RC > 0: a constant trip count (registers indexed by it)
template <int RC, typename F>
__device__ __forceinline__ void sel_each(int iters, F&& f) {
  if constexpr (RC > 0) {
#pragma unroll
    for (int it = 0; it < RC; it++)
      if (it < iters) f(it);
  } else {
    for (int it = 0; it < iters; it++) f(it);
  }
}

// two u16 scores per dword (low half = the lower node index): packed VALU, two scores per instruction
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t w) { return __builtin_bit_cast(u16x2, w); }
__device__ __forceinline__ uint32_t as_u32(u16x2 w) { return __builtin_bit_cast(uint32_t, w); }
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  return as_u32(__builtin_elementwise_max(as_u16x2(a), as_u16x2(b)));
}
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {  // kept one instruction (no compare rewrite)
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) { return as_u32(as_u16x2(a) + as_u16x2(b)); }
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b) { return as_u32(as_u16x2(a) - as_u16x2(b)); }
__device__ __forceinline__ uint32_t max_halves(uint32_t w) { return max(w & 0xFFFFu, w >> 16); }

// Exact top-k_j per pod, k_j = min(j+1, KMAX), in (score desc, node index asc) order.  One
// workgroup per pod; each wave owns a contiguous node segment read 16 B per lane (8 scores).
//   pass 1: best score M and the feasible count (DPP reductions)
//   pass 2: per-wave histogram of the 64 scores below M in LDS -> threshold score and, per wave, the
//           number of ties before it in node order (a generic binary search covers the rare case
//           of fewer than k feasible nodes inside the window)
//   pass 3: select score > thr, and the first need_ties nodes with score == thr by node index.
// Every pass works on the scores two per dword with packed u16 instructions; a step whose lanes hold no
// score in the window (pass 2) or none that can be selected (pass 3) is skipped by one ballot, so pass 3
// — k of N nodes selected — costs a max and a ballot per step.
// RC > 0 (segments of <= RC * 512 nodes): pass 1 issues every load of the wave's segment at once and
// keeps the (normalized) scores in registers, so passes 2 and 3 read no memory.  RC = 0 streams the
// segment in every pass.
// Nodes [lo, hi) (lo % 512 == 0: the shard boundaries keep the 16-B loads aligned); keys carry the
// global node index, so per-shard lists merge without translation (k_merge).
// DS: the batch is one DeviceShare pod; its scores get the normalized DeviceShare term (dsmax1 =
// 1 + the max raw score over all feasible nodes, after the all-reduce when node-sharded).
// kext / ostride: the pipelined schedule selects top-(k_j + KMAX) lists of a stale snapshot into
// rows of `ostride` keys (pipelining); otherwise kext = 0, ostride = KMAX.
// gridDim.y > 1 (plain batches): the pod's nodes are split into gridDim.y 512-aligned parts, one workgroup
// each, every part's top-k_j list in its own block of a gather buffer (`ystride` words apart) for k_merge --
// the per-shard lists of the node-sharded path, on one GPU (a batch of 64 pods then fills every CU).
// L = list length (KMAX, or KSTALE for the pipelined schedule's stale lists); outputs use stride L.
constexpr int KSTALE = 2 * KMAX;  // stale-snapshot list length of the pipelined schedule
constexpr int KSTALE2 = 3 * KMAX;  // select-ahead list length (k_fixlist: up to KMAX of them are batch b-2's nodes)
constexpr int gath_words(int L) { return MAX_BATCH * L + MAX_BATCH; }
constexpr int GATH_WORDS_MAX = MAX_BATCH * KSTALE + MAX_BATCH;
constexpr int MAX_WORLD = 8;
static_assert(MAX_WORLD == 8, "select_parts caps the parts at 8");
constexpr int MERGE_BLOCK = MAX_WORLD * KSTALE;

template <bool SC1, bool SORTED = false>
__device__ __forceinline__ void merge_lists(const uint32_t* __restrict__ gath, int64_t gw, int world, int L, int kext,
                                            int j, uint4* s_k, uint32_t* __restrict__ cand,
                                            int32_t* __restrict__ cand_cnt, bool sc1_out = false);
static_assert(SELECT_BLOCK == MERGE_BLOCK, "the last part's workgroup of a split k_select merges");

template <bool DS, int RC>
__global__ __launch_bounds__(SELECT_BLOCK) void k_select(const uint16_t* __restrict__ scores, int64_t score_stride,
                                                         int lo, int hi, uint32_t* __restrict__ cand,
                                                         int32_t* __restrict__ cand_cnt,
                                                         const uint16_t* __restrict__ dsraw,
                                                         uint32_t* __restrict__ dsmax1, int32_t wds, int kext,
                                                         int ostride, int64_t ystride,
                                                         uint32_t* __restrict__ mcand = nullptr,
                                                         int32_t* __restrict__ mcnt = nullptr,
                                                         int32_t* __restrict__ parts_done = nullptr,
                                                         int32_t* __restrict__ ready = nullptr,
                                                         int32_t* __restrict__ started = nullptr) {
  uint32_t* const gath = cand;
  RPROF_DECL
  if (!DS && gridDim.y > 1) {
    const int part = select_part(lo, hi, gridDim.y);
    lo = min(hi, lo + (int)blockIdx.y * part);
    hi = min(hi, lo + part);
    cand += (int64_t)blockIdx.y * ystride;
    cand_cnt += (int64_t)blockIdx.y * ystride;
  }
  // this workgroup of the batch's selection is resident: the other eval stream's next eval waits for all of them,
  // so its grid never holds the CUs a workgroup of this select still needs
  if (started && threadIdx.x == 0) __hip_atomic_fetch_add(started, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __shared__ int16_t s_lut[DS ? MAX_DS_RAW + 1 : 1];
  __shared__ int32_t s_dscnt;
  DsNorm dn{DS ? dsraw + (int64_t)blockIdx.x * score_stride : dsraw, s_lut};
  uint32_t m1 = 0;
  if (DS) {
    m1 = dsmax1[blockIdx.x];
    if (threadIdx.x == 0) s_dscnt = 0;
    for (int x = threadIdx.x; x <= MAX_DS_RAW; x += SELECT_BLOCK) s_lut[x] = (int16_t)(wds * ds_norm(x, m1));
    __syncthreads();
  }
  // per wave SEL_COPIES histograms (lane & 7 picks one), rows padded to 65 words: lanes of one LDS lane group
  // that count the same score go to different copies in different banks instead of one address
  __shared__ __attribute__((aligned(16))) int32_t s_hist[SELECT_WAVES][SEL_COPIES][SEL_WINDOW + 1];
  __shared__ int32_t s_red[2][SELECT_WAVES];
  __shared__ int32_t s_thr[2];
  __shared__ int32_t s_tie[SELECT_WAVES];
  __shared__ int32_t s_out;
  const int j = blockIdx.x;
  const int k = min(j + 1, KMAX) + kext;
  const uint16_t* sc = scores + (int64_t)j * score_stride;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int seg = select_seg(lo, hi);
  const int w0 = min(hi, lo + wave * seg);
  const int w1 = min(hi, w0 + seg);
  const int iters = (w1 - w0 + 511) >> 9;  // wave-uniform; <= RC when RC > 0 (the host picks RC by select_seg)
  for (int x = threadIdx.x; x < SELECT_WAVES * SEL_COPIES * (SEL_WINDOW + 1); x += SELECT_BLOCK)
    reinterpret_cast<int32_t*>(s_hist)[x] = 0;
  int32_t* my_hist = &s_hist[wave][lane & (SEL_COPIES - 1)][0];
  if (threadIdx.x == 0) s_out = 0;
  uint4 cache[RC > 0 ? RC : 1];
  // the 8 scores of this lane at step it (nodes w0 + it*512 + lane*8 ...) as 4 packed dwords, 0 beyond w1
  auto load4 = [&](int it, uint32_t w[4]) {
    const int i = w0 + it * 512 + lane * 8;
    if (!DS && i + 8 <= w1) {
      const uint4 q = *reinterpret_cast<const uint4*>(sc + i);
      w[0] = q.x, w[1] = q.y, w[2] = q.z, w[3] = q.w;
    } else {
      uint32_t v[8];
      load8<DS>(sc, i, w1, v, dn);
#pragma unroll
      for (int t = 0; t < 4; t++) w[t] = v[2 * t] | (v[2 * t + 1] << 16);
    }
  };
  auto get4 = [&](int it, uint32_t w[4]) {
    if constexpr (RC > 0) {
      w[0] = cache[it].x, w[1] = cache[it].y, w[2] = cache[it].z, w[3] = cache[it].w;
    } else {
      load4(it, w);
    }
  };
  auto unpack = [](const uint32_t w[4], uint32_t v[8]) {
#pragma unroll
    for (int t = 0; t < 4; t++) {
      v[2 * t] = w[t] & 0xFFFFu;
      v[2 * t + 1] = w[t] >> 16;
    }
  };
  auto lane_max = [](const uint32_t w[4]) { return max_halves(pk_max_u16(pk_max_u16(w[0], w[1]), pk_max_u16(w[2], w[3]))); };

  // pass 1 (RC > 0: the only pass that reads memory)
  uint32_t mx2 = 0, cnt2 = 0;  // packed: per half, the max and the feasible count
  int at_max = 0;              // DS: feasible nodes whose raw score attains the normalisation max
  sel_each<RC>(iters, [&](int it) {
    uint32_t w[4];
    load4(it, w);
    if constexpr (RC > 0) cache[it] = make_uint4(w[0], w[1], w[2], w[3]);
#pragma unroll
    for (int t = 0; t < 4; t++) {
      mx2 = pk_max_u16(mx2, w[t]);
      cnt2 = pk_add_u16(cnt2, pk_min_u16(w[t], 0x00010001u));
    }
    if (DS && m1) {
      uint32_t r[8];
      load8_raw(dn.raw, w0 + it * 512 + lane * 8, w1, r);
#pragma unroll
      for (int t = 0; t < 8; t++) at_max += r[t] == m1;
    }
  });
  if (DS && m1) {
    at_max = wave_sum(at_max);
    if (lane == 0 && at_max) atomicAdd(&s_dscnt, at_max);
  }
  RPROF(0)
  const uint32_t mx = wave_max_u32(max_halves(mx2));
  const int feas = wave_sum((int)((cnt2 & 0xFFFFu) + (cnt2 >> 16)));
  if (lane == 0) {
    s_red[0][wave] = (int)mx;
    s_red[1][wave] = feas;
  }
  __syncthreads();
  int M = 0, F = 0;
#pragma unroll
  for (int w = 0; w < SELECT_WAVES; w++) {
    M = max(M, s_red[0][w]);
    F += s_red[1][w];
  }
  RPROF(1)
  int thr = 0, need_ties = 0;  // select v > thr, plus the first need_ties with v == thr
  if (F > k) {
    // pass 2: per-wave histogram of d = M - v over the window d < 64.  An infeasible node (v = 0) has
    // d = M exactly, so bins d < M are exact and the scan below ignores the rest.
    const uint32_t MM = (uint32_t)M * 0x00010001u;
    sel_each<RC>(iters, [&](int it) {
      uint32_t w[4];
      get4(it, w);
      if (!__ballot(lane_max(w) + SEL_WINDOW > (uint32_t)M)) return;  // no score of the step in the window
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const uint32_t d2 = pk_sub_u16(MM, w[t]);
        const uint32_t dl = d2 & 0xFFFFu, dh = d2 >> 16;
        if (dl < SEL_WINDOW) atomicAdd(my_hist + dl, 1);
        if (dh < SEL_WINDOW) atomicAdd(my_hist + dh, 1);
      }
    });
    __syncthreads();
    {  // each wave folds its copies into copy 0, lane d = window bin
      int c = 0;
#pragma unroll
      for (int y = 0; y < SEL_COPIES; y++) c += s_hist[wave][y][lane];
      s_hist[wave][0][lane] = c;  // the wave's own row: no other wave reads it before the barrier
    }
    __syncthreads();
    if (wave == 0) {  // cumulative count from the top, lane d = window bin
      int c = 0;
#pragma unroll
      for (int w = 0; w < SELECT_WAVES; w++) c += s_hist[w][0][lane];
      if (lane >= M) c = 0;  // d >= M: score <= 0, infeasible
      int cum = c;  // inclusive prefix over lanes
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(cum, off, 64);
        if (lane >= off) cum += o;
      }
      const uint64_t reach = __ballot(cum >= k);
      if (reach) {
        const int d = __ffsll((unsigned long long)reach) - 1;
        const int above = __shfl(cum - c, d, 64);
        if (lane == 0) {
          s_thr[0] = M - d;
          s_thr[1] = k - above;
        }
      } else if (lane == 0) {
        s_thr[0] = -1;  // fewer than k feasible nodes inside the window
      }
    }
    __syncthreads();
    thr = s_thr[0];
    need_ties = s_thr[1];
    if (thr < 0) {
      // generic threshold search over [1, M - 64]: count(v >= lo) >= k > count(v >= hi)
      auto count_ge = [&](int t) -> int {
        int c = 0;
        sel_each<RC>(iters, [&](int it) {
          uint32_t w[4], v[8];
          get4(it, w);
          unpack(w, v);
#pragma unroll
          for (int q = 0; q < 8; q++) c += v[q] >= (uint32_t)t;
        });
        c = wave_sum(c);
        __syncthreads();
        if (lane == 0) s_red[1][wave] = c;
        __syncthreads();
        int tot = 0;
#pragma unroll
        for (int w = 0; w < SELECT_WAVES; w++) tot += s_red[1][w];
        return tot;
      };
      int lo = 1, hi = M - SEL_WINDOW + 1, cnt_hi = count_ge(hi);
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
      int ties = 0;
      sel_each<RC>(iters, [&](int it) {
        uint32_t w[4], v[8];
        get4(it, w);
        unpack(w, v);
#pragma unroll
        for (int q = 0; q < 8; q++) ties += v[q] == (uint32_t)thr;
      });
      ties = wave_sum(ties);
      if (lane == 0) s_tie[wave] = ties;
    } else if (lane == 0) {
      s_tie[wave] = s_hist[wave][0][M - thr];
    }
    __syncthreads();
  }
  RPROF(2)
  // pass 3: select (a step none of whose scores reaches vmin holds no selected node and no tie)
  const uint32_t vmin = (uint32_t)max(1, need_ties > 0 ? thr : thr + 1);
  uint32_t* const stage = reinterpret_cast<uint32_t*>(&s_hist[0][0][0]);  // (pass 3 reads no histogram)
  int running = 0;  // ties of this wave before the current row
  for (int w = 0; w < wave; w++) running += need_ties > 0 ? s_tie[w] : 0;
  uint32_t* out = cand + (int64_t)j * ostride;
  sel_each<RC>(iters, [&](int it) {
    uint32_t w[4];
    get4(it, w);
    if (!__ballot(lane_max(w) >= vmin)) return;
    const int i0 = w0 + it * 512 + lane * 8;
    uint32_t v[8];
    unpack(w, v);
    int nt = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) nt += (need_ties > 0 && v[t] == (uint32_t)thr && v[t] > 0);
    int tie_tot;
    int rank = running + lane_prefix16(nt, &tie_tot);
    running += tie_tot;
    uint32_t selm = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
      bool sel = v[t] > (uint32_t)thr;
      if (need_ties > 0 && v[t] == (uint32_t)thr && v[t] > 0) {
        sel = rank < need_ties;
        rank++;
      }
      selm |= (uint32_t)sel << t;
    }
    const int ns = __popc(selm);
    int sel_tot;
    const int pre = lane_prefix16(ns, &sel_tot);
    if (sel_tot) {
      int wbase = 0;
      if (lane == 0) wbase = atomicAdd(&s_out, sel_tot);
      wbase = __shfl(wbase, 0, 64);
      int pos = wbase + pre;
#pragma unroll
      for (int t = 0; t < 8; t++)
        if (selm & (1u << t)) {
          const uint32_t key = (v[t] << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)(i0 + t));
          if (mcand) stage[pos] = key;  // (fused merge: sorted below)
          else if (ready) st_sc1(out + pos, key);  // (read by the running Reserve kernel)
          else out[pos] = key;
          pos++;
        }
    }
  });
  __syncthreads();
  RPROF(3)
  if (mcand && !DS) {  // the part's list in descending order (the merge ranks by binary search)
    const int n = s_out;
    if ((int)threadIdx.x < n) {
      const uint32_t key = stage[threadIdx.x];
      int rank = 0;
      for (int x = 0; x < n; x++) rank += stage[x] > key;
      st_sc1(out + rank, key);  // (read by another workgroup of this launch)
    }
  }
  if (threadIdx.x == 0) {
    if (mcand || ready) st_sc1(cand_cnt + j, (int32_t)s_out);
    else cand_cnt[j] = s_out;
    if (DS) dsmax1[DSB_CNT + j] = (uint32_t)s_dscnt;
  }
  if (!DS && !mcand && ready) {  // one workgroup per pod: publish its list to the running Reserve kernel
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  RPROF(4)
  if (DS || !mcand || !parts_done) {  // (no parts_done: the parts stay sorted in place, k_fixlist<PARTS> merges)
    RPROF_FLUSH(3, 1)
    return;
  }
  // split select with the merge fused: the workgroup finishing pod j's last part merges the parts (k_merge's
  // work without its launch).  The lists went out as sc1 stores; every wave drains them before the barrier,
  // then one relaxed count (no agent-scope fence: on this part it would write back the XCD's L2,
  // cdna_hip_programming.md Guideline 16); the merging workgroup reads them with sc1 loads.
  drain_stores();
  __syncthreads();
  __shared__ int32_t s_last;
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(parts_done + j, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (int)gridDim.y - 1;
    if (s_last) parts_done[j] = 0;  // the next batch's count (stream order; no other workgroup touches it now)
  }
  __syncthreads();
  RPROF(5)
  if (!s_last) {
    RPROF_FLUSH(3, 1)
    return;
  }
  __syncthreads();  // (the staging reads above, before the merge reuses the words)
  merge_lists<true, true>(gath, ystride, (int)gridDim.y, ostride, kext, j, reinterpret_cast<uint4*>(&s_hist[0][0][0]),
                          mcand, mcnt, ready != nullptr);
  if (ready) {  // publish the merged list to the running Reserve kernel
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  RPROF(6)
  RPROF_FLUSH(3, 1)
}

// --- node-sharded batches: merge of the per-shard candidate lists ---------------------------------
// Rank r's k_select writes its block of the gather buffer: keys [MAX_BATCH][KMAX] then counts
// [MAX_BATCH].  After the all-gather every rank holds all blocks and merges identically: the global
// top-k_j of pod j is the top-k_j of the union of the per-shard top-k_j lists (each global top-k_j node
// is also top-k_j inside its own shard).  Keys are unique (they embed the node index), so a key's
// rank in the union is the number of larger keys; ranks < k_j are written in order.

// pod j's merged list from `world` blocks `gw` words apart (all MERGE_BLOCK threads of the workgroup; s_k:
// MERGE_BLOCK keys of LDS).  SC1: the blocks were written by other workgroups of the running launch.
// SORTED: every block's list is in descending order, so a key's rank in another block is the length of
// that block's prefix of larger keys (a binary search) instead of a count over all of its keys.
template <bool SC1, bool SORTED>
__device__ __forceinline__ void merge_lists(const uint32_t* __restrict__ gath, int64_t gw, int world, int L, int kext,
                                            int j, uint4* s_k, uint32_t* __restrict__ cand,
                                            int32_t* __restrict__ cand_cnt, bool sc1_out) {
  const int k = min(j + 1, KMAX) + kext;
  const int t = threadIdx.x, r = t / L, c = t % L;
  uint32_t key = 0;
  int n = 0;
  if (r < world) {
    const uint32_t* blk = gath + (int64_t)r * gw;
    n = SC1 ? ld_sc1(reinterpret_cast<const int32_t*>(blk + MAX_BATCH * L + j)) : (int)blk[MAX_BATCH * L + j];
    if (c < n) key = SC1 ? (uint32_t)ld_sc1(reinterpret_cast<const int32_t*>(blk + j * L + c)) : blk[j * L + c];
  }
  uint32_t* const sk = reinterpret_cast<uint32_t*>(s_k);
  sk[t] = key;
  const int nz = __syncthreads_count(key != 0u);
  if (SORTED) {
    if (key) {
      int rank = c;  // the larger keys of its own block come first
      for (int q = 0; q < world; q++) {
        if (q == r) continue;
        const uint32_t* b = sk + q * L;  // descending, zeros after the block's count
        int lo = 0, hi = L;              // the first position holding a key < key
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (b[mid] > key) lo = mid + 1;
          else hi = mid;
        }
        rank += lo;
      }
      if (rank < k) {
        if (sc1_out) st_sc1(cand + j * L + rank, key);
        else cand[j * L + rank] = key;
      }
    }
    if (t == 0) {
      if (sc1_out) st_sc1(cand_cnt + j, min(nz, k));
      else cand_cnt[j] = min(nz, k);
    }
    return;
  }
  if (key) {
    int rank = 0;
    const int n4 = world * L / 4;
    for (int u = 0; u < n4; u++) {
      const uint4 q = s_k[u];
      rank += (int)(q.x > key) + (int)(q.y > key) + (int)(q.z > key) + (int)(q.w > key);
    }
    if (rank < k) cand[j * L + rank] = key;
  }
  if (t == 0) cand_cnt[j] = min(nz, k);
}

__global__ __launch_bounds__(MERGE_BLOCK) void k_merge(const uint32_t* __restrict__ gath, int world, int L, int kext,
                                                       uint32_t* __restrict__ cand, int32_t* __restrict__ cand_cnt) {
  __shared__ uint4 s_k[MERGE_BLOCK / 4];
  merge_lists<false>(gath, gath_words(L), world, L, kext, (int)blockIdx.x, s_k, cand, cand_cnt);
}

// --- pipelined schedule: exact candidate lists from a stale snapshot ------------------------------
// Batch b's eval + select run while batch b-1 is still being resolved (pipelining): they
// see every Reserve of batches <= b-2, and arbitrary (possibly half-written) rows for the <= 64 nodes
// batch b-1 chose ("touched").  Every other row equals the exact pre-b state S.  The select keeps the
// stale top-(k_j + KMAX) per pod.  An untouched node in the exact top-k_j under S has at most k_j - 1
// untouched and T <= KMAX touched nodes above it in the stale order, so it is in the stale list; the
// touched nodes are re-evaluated here against their rows in S (this kernel runs after batch b-1's
// resolve).  The top-k_j of (stale list minus touched) + (touched, fresh keys) is therefore the exact
// top-k_j under S that k_resolve expects.  One workgroup per pod.
constexpr int FIX_BLOCK = KSTALE + KMAX;  // stale keys, then fresh keys of the touched nodes

// wait_b >= 0: the lists need the Reserves of batch wait_b (the touched nodes' rows): wait for its flag
// in `done` first.  When the list is written the workgroup adds 1 to *ready (the Reserve kernel waits
// for all of the batch's pods).
// The touched nodes come as the Reserve kernel's compact list of the rows batch b-1 changed (distinct
// nodes, the node index in Row.pad), so no row gather depends on a node id read after the wait.

template <bool EXT>
__global__ __launch_bounds__(FIX_BLOCK) void k_fixup(SoA s, const DevPod* __restrict__ pods,
                                                     const int32_t* __restrict__ batch_base, KArgs k,
                                                     const uint32_t* __restrict__ stale,
                                                     const int32_t* __restrict__ stale_cnt,
                                                     const int64_t* __restrict__ trows, const int32_t* __restrict__ tcnt,
                                                     uint32_t* __restrict__ cand, int32_t* __restrict__ cand_cnt,
                                                     const int32_t* __restrict__ done, int wait_b,
                                                     int32_t* __restrict__ ready, int32_t* __restrict__ err,
                                                     uint64_t* __restrict__ fstamp) {
  __shared__ int32_t s_tn[KMAX];
  __shared__ uint4 s_k[FIX_BLOCK / 4];
  __shared__ int32_t s_ok, s_nt;
  const int j = blockIdx.x, kj = min(j + 1, KMAX);
  const int t = threadIdx.x;
  // everything that does not depend on batch b-1 is read before the wait
  uint32_t key = 0;
  if (t < KSTALE && t < stale_cnt[j]) key = stale[j * KSTALE + t];
  DevPod pod;
  if (t >= KSTALE) pod = pods[*batch_base + j];
  if (t == 0) {
    s_ok = wait_b < 0 || wait_at_least(done + wait_b, 1, err);
    s_nt = wait_b < 0 ? 0 : ld_sc1(tcnt);
    if (j == 0 && fstamp) fstamp[0] = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  if (!s_ok) return;
  const int nt = s_nt;
  NodeFast n;
  int node = -1;
  if (t >= KSTALE && t - KSTALE < nt) {  // sc1: the Reserve kernel wrote the records while running
    const int64_t* rp = trows + (int64_t)(t - KSTALE) * NUM_RW;
    rec_load<__HIP_MEMORY_SCOPE_AGENT>(rp, n);
    node = (int)ld_sc1(rp + RW_PAD);
    if (EXT && (k.flags & AF_EXT)) ext_load(s, node, k, n);  // written by batch b-1's Reserve before its done flag
    s_tn[t - KSTALE] = node;
  }
  __syncthreads();
  if (t < KSTALE) {
    if (key) {
      const int kn = key_node(key);
      for (int u = 0; u < nt; u++) key = s_tn[u] == kn ? 0u : key;  // broadcast reads
    }
  } else if (node >= 0) {
    fast_adopt(n, k);
    const double estd[2] = {(double)pod.est[0], (double)pod.est[1]}, reqd[2] = {(double)pod.req[0], (double)pod.req[1]};
    key = make_key(fast_total<EXT>(n, pod, estd, reqd, k), node);
  }
  reinterpret_cast<uint32_t*>(s_k)[t] = key;
  const int nz = __syncthreads_count(key != 0u);
  if (key) {
    int rank = 0;
#pragma unroll 4
    for (int u = 0; u < FIX_BLOCK / 4; u++) {
      const uint4 q = s_k[u];
      rank += (int)(q.x > key) + (int)(q.y > key) + (int)(q.z > key) + (int)(q.w > key);
    }
    if (rank < kj) st_sc1(cand + j * KMAX + rank, key);  // sc1: read by the running Reserve kernel
  }
  if (t == 0) st_sc1(cand_cnt + j, min(nz, kj));
  if (ready) {  // publish: every wave drains its sc1 stores before the barrier, then one counter add
    drain_stores();
    __syncthreads();
    if (t == 0) {
      __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (j == 0 && fstamp) fstamp[1] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// Select-ahead (round 5): batch b's eval waited for batch b-3's Reserve, its select ran right after it into top-
// (k_j + 2 KMAX) lists; once batch b-2 is done, workgroup j drops b-2's changed nodes (THelp::tlist, written with
// their records before the flag) from pod j's list, inserts their current keys, and publishes the top-(k_j + KMAX)
// in descending key order as the Reserve kernel's stale list -- exact but for batch b-1's nodes, which the replay
// holds as T slots.  (At most KMAX entries drop, so k_j + KMAX exact keys remain.)  A key of a node that batch
// b-1 changes too may be torn (its record is being rewritten): the replay drops every T node's key anyway.
// PARTS (round 6): the split select left its parts' lists sorted in their blocks of the gather buffer (`pre`, `gw`
// words apart) without merging them -- its sc1 drain, counter and last-arriver merge were its tail -- and this kernel
// merges them before it waits (a key's rank is its position plus a binary search in every other part, as
// merge_lists), so the merge is off the done[b-2] -> ready[b] lap.
constexpr int FIXL_BLOCK = KSTALE2 + KMAX;
constexpr int FIXL_PARTS_BLOCK = 1024;
static_assert((1024 / KSTALE2) * KSTALE2 <= FIXL_PARTS_BLOCK, "every part of a select-ahead split fits a workgroup");
template <bool EXT, bool PARTS = false>
__global__ __launch_bounds__(PARTS ? FIXL_PARTS_BLOCK : FIXL_BLOCK) void k_fixlist(
    SoA s, const DevPod* __restrict__ pods, const int32_t* __restrict__ batch_base, KArgs k,
    const uint32_t* __restrict__ pre, const int32_t* __restrict__ pre_cnt, const int32_t* __restrict__ tlist,
    const int32_t* __restrict__ done_wait, uint32_t* __restrict__ stale, int32_t* __restrict__ stale_cnt,
    int32_t* __restrict__ ready, int32_t* __restrict__ err, int64_t gw = 0, int parts = 1) {
  __shared__ int32_t s_tn[KMAX];
  __shared__ uint4 s_k[FIXL_BLOCK / 4];
  __shared__ int32_t s_ok, s_nt;
  __shared__ uint32_t s_pk[PARTS ? FIXL_PARTS_BLOCK : 1];  // the parts' lists (descending, zeros after each count)
  __shared__ int32_t s_mcnt;
  const int j = blockIdx.x, kj = min(j + 1, KMAX);
  const int t = threadIdx.x;
  uint32_t key = 0;  // (read before the wait: the select before this kernel on the same stream wrote them)
  if constexpr (PARTS) {
    const int L = KSTALE2, r = t / L, c = t - r * L;
    const int kx = kj + 2 * KMAX;  // the merged list's length (the select's k_j + kext)
    uint32_t pk = 0;
    if (r < parts) {
      const uint32_t* blk = pre + (int64_t)r * gw;
      if (c < (int)blk[MAX_BATCH * L + j]) pk = blk[j * L + c];
      s_pk[t] = pk;
    }
    if (t < KSTALE2) reinterpret_cast<uint32_t*>(s_k)[t] = 0u;
    const int nz = __syncthreads_count(pk != 0u);
    if (t == 0) s_mcnt = min(nz, kx);
    if (pk) {
      int rank = c;  // the larger keys of its own part come first
      for (int q = 0; q < parts; q++) {
        if (q == r) continue;
        const uint32_t* b = s_pk + q * L;
        int lo = 0, hi = L;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (b[mid] > pk) lo = mid + 1;
          else hi = mid;
        }
        rank += lo;
      }
      if (rank < kx) reinterpret_cast<uint32_t*>(s_k)[rank] = pk;
    }
    __syncthreads();
    if (t < KSTALE2 && t < s_mcnt) key = reinterpret_cast<uint32_t*>(s_k)[t];
    __syncthreads();  // (s_k is reused below; threads >= FIXL_BLOCK only join the barriers from here)
  } else {
    if (t < KSTALE2 && t < pre_cnt[j]) key = pre[j * KSTALE2 + t];
  }
  DevPod pod;
  if (t >= KSTALE2 && t < FIXL_BLOCK) pod = pods[*batch_base + j];
  if (t == 0) {
    s_ok = done_wait ? wait_at_least(done_wait, 1, err) : 1;
    s_nt = done_wait ? ld_sc1(tlist) : 0;
  }
  __syncthreads();
  if (!s_ok) return;  // (a timed-out hand-off: the host discards the queue)
  const int nt = s_nt;
  NodeFast n;
  int node = -1;
  if (t >= KSTALE2 && t < FIXL_BLOCK && t - KSTALE2 < nt) {
    node = ld_sc1(tlist + 1 + (t - KSTALE2));
    rec_load<__HIP_MEMORY_SCOPE_AGENT>(s.rec + (int64_t)node * NUM_RW, n);
    if (EXT && (k.flags & AF_EXT)) ext_load(s, node, k, n);
    s_tn[t - KSTALE2] = node;
  }
  __syncthreads();
  if (t < KSTALE2) {
    if (key) {
      const int kn = key_node(key);
      for (int u = 0; u < nt; u++) key = s_tn[u] == kn ? 0u : key;  // broadcast reads
    }
  } else if (node >= 0) {
    fast_adopt(n, k);
    const double estd[2] = {(double)pod.est[0], (double)pod.est[1]}, reqd[2] = {(double)pod.req[0], (double)pod.req[1]};
    key = make_key(fast_total<EXT>(n, pod, estd, reqd, k), node);
  }
  if (t < FIXL_BLOCK) reinterpret_cast<uint32_t*>(s_k)[t] = key;
  const int nz = __syncthreads_count(key != 0u);
  const int out = min(nz, kj + KMAX);
  if (key) {
    int rank = 0;
#pragma unroll 4
    for (int u = 0; u < FIXL_BLOCK / 4; u++) {
      const uint4 q = s_k[u];
      rank += (int)(q.x > key) + (int)(q.y > key) + (int)(q.z > key) + (int)(q.w > key);
    }
    if (rank < out) st_sc1(stale + j * KSTALE + rank, key);  // sc1: read by the running Reserve kernel
  }
  if (t == 0) st_sc1(stale_cnt + j, out);
  drain_stores();  // publish: every wave drains its sc1 stores before the barrier, then one counter add
  __syncthreads();
  if (t == 0) __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Pipelined schedule without k_fixup (k_resolve_run's stale-list mode), where the eval / select kernels do not
// do it themselves (node-sharded selects, 1-2-pod batches): publish batch q's lists to the running Reserve
// kernel (ready = its pods; the select / merge kernels before this one on the same stream wrote them), and /
// or hold the eval stream until batch q-1's Reserve is done (done_wait), so that batch q+1's eval sees every
// Reserve of batches <= q-1 -- its stale keys differ from the exact ones only on the nodes batch q changes --
// and its lists may reuse batch q-1's half of the double buffer.
// Dynamic LDS of the eval streams' LDS-free kernels (k_handoff, k_patch): a workgroup holding any LDS cannot
// share a CU with a Reserve workgroup (which leaves 64 B of the CU's LDS), so their waves never take issue
// slots from the replay's latency-bound waves.
constexpr unsigned EXCL_LDS = 1024;
__global__ void k_handoff(int32_t* __restrict__ ready, int32_t n, const int32_t* __restrict__ done_wait,
                          int32_t* __restrict__ err, uint64_t* __restrict__ fstamp, int32_t want) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (ready) __hip_atomic_store(ready, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (fstamp) {
    fstamp[0] = t0;
    fstamp[1] = t0 + 1;
  }
  if (done_wait) (void)wait_at_least(done_wait, want, err);  // a timeout sets *err: the host discards the queue
}

// --- resolve: one wavefront replays the batch sequentially -------------------------------------
// one node row straight from the SoA, past this CU's L1 (rows this workgroup patched earlier)
__device__ __forceinline__ void load_row_sc1(const SoA& s, int64_t i, Row& r) {
  const int64_t st = s.stride;
#pragma unroll
  for (int f = 0; f < NUM_I64_FIELDS; f++) r.f[f] = ld_sc1(s.f + f * st + i);
  r.flags = ld_sc1(s.flags + i);
  r.pad = 0;
}

// Changed-node set of the batch being replayed: a bitmap over node ids, in LDS for ids < 811,008 (else a
// zeroed device bitmap in global memory, sc1-accessed).  Only the replay wave touches it; the bits of a
// batch are cleared when it ends, so it is zero between batches.
constexpr int CHG_LDS_WORDS = 25344;  // node ids < 811,008 (else the global bitmap)
struct ChgSet {
  uint32_t* lds;
  uint32_t* glb;  // non-null: node ids beyond the LDS bitmap
};
__device__ __forceinline__ bool chg_test(const ChgSet& c, int node) {
  const uint32_t w = c.glb ? ld_sc1(c.glb + (node >> 5)) : c.lds[node >> 5];
  return (w >> (node & 31)) & 1u;
}
__device__ __forceinline__ void chg_set(const ChgSet& c, int node) {  // one lane
  if (c.glb) __hip_atomic_fetch_or(c.glb + (node >> 5), 1u << (node & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else c.lds[node >> 5] |= 1u << (node & 31);
}
// several lanes at once (words may be shared)
__device__ __forceinline__ void chg_set_atomic(const ChgSet& c, int node) {
  if (c.glb) __hip_atomic_fetch_or(c.glb + (node >> 5), 1u << (node & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_fetch_or(c.lds + (node >> 5), 1u << (node & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// compile-time placement of the bitmap (the speculative prediction loop: no branch, no vmcnt wait on the
// LDS path); GLB: one lane's atomic is drained before later loads of other lanes may depend on it
template <bool GLB>
__device__ __forceinline__ void chg_or(const ChgSet& c, int node) {
  if (GLB) {
    __hip_atomic_fetch_or(c.glb + (node >> 5), 1u << (node & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    drain_stores();
  } else {
    __hip_atomic_fetch_or(c.lds + (node >> 5), 1u << (node & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
// at the end of a batch every set bit belongs to a changed node: each changed lane zeroes its word
// (lanes sharing a word all store zero)
__device__ __forceinline__ void chg_clear_word(const ChgSet& c, int node) {
  if (c.glb) st_sc1(c.glb + (node >> 5), 0u);
  else c.lds[node >> 5] = 0u;
}

// prologue width (the replay runs on wave 0 alone): 4 waves, one per SIMD, so the replay wave may use
// every register of its SIMD (no scratch spills in any variant)
template <bool NUMA> constexpr int res_threads() { return 256; }

// Ordering point for LDS traffic between the lanes of ONE wavefront: LDS instructions of a wave
// execute in issue order, so only the compiler must be kept from moving accesses across it
// (a workgroup __syncthreads would also drain outstanding global stores).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}

// DeviceShare Reserve of node i on the whole wave, lane m = minor m (ds_reserve spreads nothing: one lane
// walks every instance, scores it and updates it in turn).  The default-allocation case: a node without
// partition table / honor policy / topology tree and a pod without partition spec or required scope, no NUMA
// affinity -- GPUAllocator.Allocate then reduces to defaultAllocateDevices on the instances that fit
// (allocator_gpu.go; device_allocator.go:237-300), other types too.  The same instance views, scores,
// picks (highest scoreDevice, ties to the lower minor) and quotav1.Add of the allocation as ds_reserve;
// anything else goes to ds_reserve on lane 0.  Wave-uniform i / p; returns the minors mask on every lane.
__device__ __forceinline__ uint64_t ds_reserve_wave(const SoA& s, int64_t i, const DevPod& p, const KArgs& k,
                                                    int lane) {
  uint64_t msk[4], out = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) msk[w] = dsmask(s, w, i);
  const RsvOvr* ro = s.n_rovr ? rsv_ovr_of(s, i) : nullptr;  // a matched pod's Reserve from k_ds_views
  if (ro && !ro->ds_res) ro = nullptr;
  if (ro || (msk[DSM_EXISTS] & (DSX_TOPO | DSX_TABLE | DSX_HONOR)) || (p.flags & (PF_GPU_PART_SPEC | 7u * PF_GPU_SCOPE0))) {
    if (lane == 0) out = ds_reserve<false>(s, i, p, k, DsAff{false, 0u}, nullptr, ro);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(out >> 32), 0) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)out, 0);
  }
  const int m = lane & (DS_MINORS - 1);
#pragma unroll
  for (int t = 0; t < 3; t++) {
    if (!p.ds_cnt[t]) continue;
    const int nk = DS_NK[t];
    const uint32_t ex = (uint32_t)(msk[DSM_EXISTS] >> (16 * t)) & 0xFFFFu;
    const bool inst = lane < DS_MINORS && ((ex >> m) & 1u);
    DsRaw raw;
    bool fit = false;
    uint32_t key = 0;  // 1 + (scoreDevice << 4 | 15 - m) for an instance defaultAllocateDevices may take
    if (inst) {
      ds_load(s, i, t, m, msk, raw);
      DsInst d;
      ds_instance_from(raw, t, m, msk, d);
      fit = !ds_free_zero(d) && ds_leq(d, p, t);
      if (fit) {
        int64_t tv[3], fv[3];
#pragma unroll
        for (int q = 0; q < 3; q++) {
          tv[q] = ((d.th >> q) & 1) ? d.tv[q] : 0;
          fv[q] = ((d.fh >> q) & 1) ? d.fv[q] : 0;
        }
        const int64_t sc = ds_weighted(k, t, tv, fv, p);  // in [0, MaxNodeScore]
        key = 1u + (((uint32_t)sc << 4) | (uint32_t)(DS_MINORS - 1 - m));
      }
    }
    const uint32_t ok = (uint32_t)__ballot(fit) & 0xFFFFu;
    const int want = p.ds_cnt[t];
    uint32_t take = 0;
    // GPUAllocator: "Insufficient GPU devices" takes nothing (Reserve follows a passed Filter); other types
    // take what fits, up to the count
    if (t != KE_DEV_GPU || __builtin_popcount(ok) >= want)
      for (int c = 0; c < want && (ok & ~take); c++) {
        const uint32_t best = wave_max_u32(((take >> m) & 1u) ? 0u : key);
        take |= 1u << (DS_MINORS - 1 - (int)((best - 1u) & 15u));
      }
    out |= (uint64_t)take << (16 * t);
    const bool mine = inst && ((take >> m) & 1u);
    int64_t alloc[3] = {0, 0, 0};
    bool has[3] = {false, false, false};
    if (t == KE_DEV_GPU) {
      const int64_t tm = raw.tv[1];  // the instance's total memory (0 without the key)
      if (p.flags & PF_DS_H_CORE) has[0] = true, alloc[0] = p.ds_req[0];
      if (p.flags & PF_DS_H_RATIO) {  // memoryRatioToBytes
        has[2] = true, alloc[2] = p.ds_req[2];
        has[1] = true, alloc[1] = mine ? p.ds_req[2] * tm / 100 : 0;
      } else if (p.flags & PF_DS_H_MEM) {  // memoryBytesToRatio: int64(float64(b)/float64(total)*100)
        has[1] = true, alloc[1] = p.ds_req[1];
        has[2] = true, alloc[2] = mine ? (int64_t)((double)p.ds_req[1] / (double)tm * 100.0) : 0;
      }
    } else {
      has[0] = true, alloc[0] = p.ds_req[2 + t];
    }
    const int w = ds_hu_word(t);
#pragma unroll
    for (int key_i = 0; key_i < 3; key_i++) {
      if (key_i >= nk || !has[key_i]) continue;
      if (mine) {
        const int field = DS_UBASE[t] + m * nk + key_i;
        s.ds[field * s.stride + i] = raw.uv[key_i] + alloc[key_i];  // quotav1.Add (absent used key: 0)
      }
      msk[w] |= (uint64_t)take << ds_hu_bit(t, 0, key_i);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int w = 1; w < 4; w++) s.dsm[w * s.stride + i] = msk[w];
  }
  return out;
}

// The speculative replay's round state (replay_spec): per pod its predicted node / snapshot key, the best
// current key among the nodes earlier pods of the batch took, and the round's first failing pod.
struct SpecLds {
  int32_t xnode[MAX_BATCH];  // pod j's predicted (then committed) node, -1 = none
  uint32_t xkey[MAX_BATCH];  // its snapshot candidate key (the best unchanged candidate), 0 = none
  uint32_t mrow[MAX_BATCH];  // max key of pod j over the nodes pods < j took, in their current state
  int32_t jf;                // first pod of the round whose prediction failed (end of round: none)
  uint32_t tmx[MAX_BATCH];   // stale lists: max key of pod j over the previous batch's changed nodes T ...
  int32_t tver[MAX_BATCH];   // ... valid while no pod of the batch reserved a T node since (-1: never computed)
  int32_t tnext[MAX_BATCH];  // the batch's changed nodes (the next batch's T), in touched-list order
  int32_t tnext_n;
};

constexpr int32_t XN_PENDING = INT32_MIN;  // L.sp.xnode: not predicted yet (the progressive S polls it)
constexpr int PCH = 16;                    // the progressive S: pods a chunk
constexpr uint64_t T_HELP_WAIT_TICKS = 2000;  // wave 0's wait for the helpers' T maxima (20 us), then its own rows
// The T-row helpers of a stale-list run (k_resolve_run workgroups 1..H): batch b's T maxima
// (every pod against the previous batch's changed nodes) evaluated on other CUs while the Reserve workgroup
// predicts, instead of on its own waves.  Global hand-off words, double-buffered by batch parity.
// Co-residency: nothing waits for a helper.  The Reserve workgroup (workgroup 0) waits for tready[b] at most
// T_HELP_WAIT_TICKS and then evaluates the missing T maxima itself, so a helper that is not resident (the grid is
// 1 + H workgroups of one CU each; other launches may hold the CUs) only costs that wait; a helper waits only for
// done[b-1], which workgroup 0 publishes whether or not any helper ran (bounded by HANDOFF_TIMEOUT_TICKS and the
// error word).  Within a workgroup every wait on LDS (the progressive S polling xnode) is on wave 0's prediction
// loop, which writes every xnode of its window before any barrier.  An unbounded LDS wait on a wave that may sit
// at a barrier is the one wait shape the bounded global hand-offs do not cover -- the most likely cause of the
// round-4 hang under per-chunk row claiming (reverted before commit) -- so the xnode poll is
// bounded too (KERR_LDS_WAIT fails the call).
struct THelp {
  int32_t* tlist;   // [2][1 + MAX_BATCH]: a batch's changed nodes (count first; the Reserve workgroup writes them)
  uint32_t* tmx;    // [2][MAX_BATCH]: the T maxima of a batch's pods (the helpers write them)
  int32_t* tready;  // [batch]: helpers done with the batch (relaxed agent adds)
  int H;            // helper workgroups (0: none)
  int ign;          // test hook: the Reserve workgroup ignores the helpers' maxima (its own rows after the barrier)
  int32_t* resident;  // set by the Reserve workgroup when it starts: the run's first eval waits for it (a select
                      // workgroup waiting for a done flag must never be what keeps the Reserve workgroup off the CUs)
};

struct ResLdsCore {
  uint32_t cand[MAX_BATCH * KSTALE];  // exact lists at stride KMAX, or the pipelined schedule's stale lists at KSTALE
  DevPod pod[MAX_BATCH];
  double pd[MAX_BATCH][4];  // the pod's estimate and requests (cpu, memory) as doubles
  int32_t cnt[MAX_BATCH];
  uint32_t dsm[MAX_BATCH];  // DeviceShare batch: 1 + snapshot max raw score of each pod (0: none / not DS)
  int32_t dsc[MAX_BATCH];   // ... and the number of its feasible nodes attaining it
  SpecLds sp;
  int64_t trec[MAX_BATCH][NUM_RW];  // the last batch's changed records (stale lists: the next batch's T slots)
  uint32_t chg[CHG_LDS_WORDS];
};
// The Reserve kernels take the CU's whole LDS (160 KB, less 64 B for a kernel's own words): no workgroup of
// the eval / select kernels (all of which use LDS) is co-resident, so the latency-bound replay waves issue on
// SIMDs of their own instead of queueing behind a concurrent eval's FP64 instructions (pipelined schedule).
constexpr int CU_LDS_BYTES = 163840;
struct ResLds : ResLdsCore {
  uint8_t cu_fill[CU_LDS_BYTES - 64 - sizeof(ResLdsCore)];
};
static_assert(sizeof(ResLds) == CU_LDS_BYTES - 64, "ResLds fills the CU's LDS");

// a changed-set bit that a failed prediction set (several lanes may share a word)
__device__ __forceinline__ void chg_unset(const ChgSet& c, int node) {
  if (c.glb) __hip_atomic_fetch_and(c.glb + (node >> 5), ~(1u << (node & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_fetch_and(c.lds + (node >> 5), ~(1u << (node & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The P phase of the speculative replay (wave 0): pods [start, end) each predict their best candidate whose
// node is not in the changed set, nor predicted by an earlier pod of the round.  A software pipeline keeps
// every LDS access off the per-pod chain: while pod j reduces, pod j+1's changed-set words are read (after
// the set updates of pods < j: a wave's LDS operations execute in order; pod j's own prediction is compared
// in registers) and pod j+2's keys are read; each is consumed one step later.  The three register sets
// rotate by hand (step A, B, C -> B, C, A), so no loop-carried copy of a pending load forces an early wait.
// Lane 0 stores pod j's prediction (L.sp.xnode / xkey) with its changed-set bit.
template <bool GLB>
__device__ __forceinline__ uint32_t chg_load_word(const ChgSet& c, uint32_t key) {
  const int node = key ? key_node(key) : 0;  // (key 0: any word, its bit is masked below)
  return GLB ? ld_sc1(c.glb + (node >> 5)) : c.lds[node >> 5];
}
__device__ __forceinline__ bool chg_word_bit(uint32_t w, uint32_t key) {
  return key != 0 && ((w >> (key_node(key) & 31)) & 1u);
}
// SORTED: every list is in descending key order (the merged lists of a split / sharded select, k_fixup's):
// the prediction is the first unflagged key -- a ballot and a lane read instead of a wave max.
template <bool GLB, bool SORTED>
__device__ __forceinline__ void spec_predict(ResLds& L, const ChgSet& C, int start, int end, int LS, bool two,
                                             int lane) {
  // SORTED: only the first 64 keys of a list are pipelined; the rest are read (with their words, which by then
  // hold every earlier prediction) when those 64 are all taken -- j + |T| of them at most, so rarely
  const bool two_p = two && !SORTED;
  auto keys = [&](int j, uint32_t& k0, uint32_t& k1) {
    k0 = j < end ? L.cand[j * LS + lane] : 0u;
    k1 = two_p && j < end ? L.cand[j * LS + 64 + lane] : 0u;
  };
  // set X: keys k0/k1 of one pod, its changed-set words w0/w1, its keys' matches m0/m1 of the previous pod's
  // prediction (not yet in the words)
  uint32_t ka0, ka1, kb0, kb1, kc0 = 0, kc1 = 0, wa0, wa1, wb0 = 0, wb1 = 0, wc0 = 0, wc1 = 0;
  bool ma0 = false, ma1 = false, mb0 = false, mb1 = false, mc0 = false, mc1 = false;
  keys(start, ka0, ka1);
  keys(start + 1, kb0, kb1);
  wa0 = chg_load_word<GLB>(C, ka0);
  wa1 = two_p ? chg_load_word<GLB>(C, ka1) : 0u;
  // pod j on set A; set B = pod j+1 (words read here); set C = pod j+2 (keys read here)
  auto step = [&](int j, uint32_t& kA0, uint32_t& kA1, uint32_t& wA0, uint32_t& wA1, bool& mA0, bool& mA1,
                  uint32_t& kB0, uint32_t& kB1, uint32_t& wB0, uint32_t& wB1, bool& mB0, bool& mB1,
                  uint32_t& kC0, uint32_t& kC1, bool& mC0, bool& mC1) {
    wB0 = chg_load_word<GLB>(C, kB0);
    if (two_p) wB1 = chg_load_word<GLB>(C, kB1);
    keys(j + 2, kC0, kC1);
    mC0 = mC1 = false;
    const bool f0 = mA0 || chg_word_bit(wA0, kA0);
    uint32_t bu;
    if constexpr (SORTED) {
      const uint64_t u0 = __ballot(kA0 != 0 && !f0);
      if (u0) {
        bu = (uint32_t)__builtin_amdgcn_readlane((int)kA0, __builtin_ctzll(u0));
      } else if (two) {  // the list's second half, read now
        const uint32_t k1 = j < end ? L.cand[j * LS + 64 + lane] : 0u;
        const uint32_t w1 = chg_load_word<GLB>(C, k1);
        const uint64_t u1 = __ballot(k1 != 0 && !chg_word_bit(w1, k1));
        bu = u1 ? (uint32_t)__builtin_amdgcn_readlane((int)k1, __builtin_ctzll(u1)) : 0u;
      } else {
        bu = 0u;
      }
    } else {
      const bool f1 = mA1 || chg_word_bit(wA1, kA1);
      bu = wave_max_u32(max(f0 ? 0u : kA0, two_p && !f1 ? kA1 : 0u));
    }
    const int xn = bu ? key_node(bu) : -1;
    if (lane == 0) {  // pod j's prediction, and its node into the changed set
      ((volatile int32_t*)L.sp.xnode)[j] = xn;  // (in order: the progressive S polls it)
      L.sp.xkey[j] = bu;
      if (xn >= 0) chg_or<GLB>(C, xn);
    }
    mB0 = kB0 != 0 && xn >= 0 && key_node(kB0) == xn;
    if (two_p) mB1 = kB1 != 0 && xn >= 0 && key_node(kB1) == xn;
  };
  for (int j = start; j < end; j += 3) {
    step(j, ka0, ka1, wa0, wa1, ma0, ma1, kb0, kb1, wb0, wb1, mb0, mb1, kc0, kc1, mc0, mc1);
    if (j + 1 >= end) break;
    step(j + 1, kb0, kb1, wb0, wb1, mb0, mb1, kc0, kc1, wc0, wc1, mc0, mc1, ka0, ka1, ma0, ma1);
    if (j + 2 >= end) break;
    step(j + 2, kc0, kc1, wc0, wc1, mc0, mc1, ka0, ka1, wa0, wa1, ma0, ma1, kb0, kb1, mb0, mb1);
  }
}

// The prediction loop for sorted lists and the LDS changed set, shortened to the per-pod instructions the chain
// needs (the loop is issue-bound: one wave per SIMD, ~11 cycles per dependent instruction): pod j's key word is
// read a step ahead (it misses only pod j-1's prediction, compared as a node), the untaken test is one bit
// extract and two compares, the prediction one ballot / find-first / lane read, and lane 0's stores (prediction,
// key, changed-set bit) are one exec-masked group without a branch.  A pod whose first 64 keys are all taken
// reads the second half of its list (rare: j + |T| keys at most precede its prediction).
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ void lane0_record(uint32_t pa, uint32_t xn, uint32_t xk, uint32_t ca, uint32_t cm) {
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_write2_b32 %1, %2, %3 offset1:64\n\t"
      "ds_or_b32 %4, %5\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv)
      : "v"(pa), "v"(xn), "v"(xk), "v"(ca), "v"(cm)
      : "memory");
}
__device__ __forceinline__ void spec_predict_lean(ResLds& L, const ChgSet& C, int start, int end, int LS, bool two,
                                                  int lane) {
  const uint32_t cbase = lds_addr(C.lds), pbase = lds_addr(&L.sp.xnode[0]);
  auto node_of = [](uint32_t k) { return (int32_t)(KEY_IDX_MASK - (k & KEY_IDX_MASK)); };
  auto key_at = [&](int j) -> uint32_t { return j < end ? L.cand[j * LS + lane] : 0u; };
  auto word_of = [&](int n) -> uint32_t { return C.lds[(uint32_t)n >> 5]; };
  auto node_of0 = [&](uint32_t k) { return k ? node_of(k) : 0; };  // (key 0: word 0, masked by the key test)
  uint32_t kA = key_at(start), kB = key_at(start + 1);
  int32_t nA = node_of0(kA);
  uint32_t wA = word_of(nA);
  int32_t xprev = -1;
  for (int j = start; j < end; j++) {
    const int32_t nB = node_of0(kB);
    const uint32_t wB = word_of(nB);     // after the set updates of pods < j (LDS order); misses pod j's
    const uint32_t kC = key_at(j + 2);
    const bool untaken = (kA != 0u) & (((wA >> (nA & 31)) & 1u) == 0u) & (nA != xprev);
    const uint64_t u = __ballot(untaken);
    uint32_t bu;
    int32_t xn;
    if (__builtin_expect(u != 0, 1)) {
      const int l = __builtin_ctzll(u);
      bu = (uint32_t)__builtin_amdgcn_readlane((int)kA, l);
      xn = __builtin_amdgcn_readlane(nA, l);
    } else {  // every one of the first 64 keys taken: the second half, against the set as it is now
      const uint32_t k1 = two && j < end ? L.cand[j * LS + 64 + lane] : 0u;
      const int32_t n1 = node_of0(k1);
      const uint64_t u1 = __ballot(k1 != 0u && !((word_of(n1) >> (n1 & 31)) & 1u) && n1 != xprev);
      bu = u1 ? (uint32_t)__builtin_amdgcn_readlane((int)k1, __builtin_ctzll(u1)) : 0u;
      xn = bu ? node_of(bu) : -1;
    }
    const uint32_t ca = cbase + (xn >= 0 ? ((uint32_t)xn >> 5) << 2 : 0u), cm = xn >= 0 ? 1u << (xn & 31) : 0u;
    lane0_record(pbase + 4u * (uint32_t)j, (uint32_t)xn, bu, ca, cm);
    xprev = xn;
    kA = kB, nA = nB, wA = wB, kB = kC;
  }
}

// Speculative replay of a plain batch (LoadAware + NodeNUMAResource (+ FitPlus / SRA / Fit) pods, no quota) on
// every wave of the workgroup ("speculative replay").  The sequential replay decides pod j as
// max(bu_j, bc_j): bu_j its best candidate no earlier pod of the batch took (exact: its snapshot key), bc_j
// the best current key among the nodes earlier pods took.  Almost every pod takes its bu_j, so a round
//   P  predicts that every pod of a window does (wave 0: bu_j = the max of its list minus the nodes of the
//      earlier predictions -- one wave max per pod),
//   R  builds in lane c of every wave the record of pod c's predicted node after pod c's Reserve,
//   S  evaluates every pod j of the window against the slots c < j in parallel (rows spread over the waves;
//      one fast_total pass per row, wave max -> mrow[j]),
//   V  checks the predictions in order: pod j's holds iff xkey[j] > mrow[j] (keys are unique per node; both
//      0: unschedulable).  Up to the first failing pod jf every prediction is the sequential decision (its
//      state is the predicted one); pod jf takes the changed node of mrow[jf] (Reserve on that slot), the
//      predictions after it are dropped, and the next round starts at jf + 1 with a smaller window.
// Lane c of every wave holds slot c: the node pod c took (valid when pod c took a node no earlier pod had),
// in its current state -- every wave applies the same Reserves, so no slot crosses waves.
//
// Stale lists (`tin`, the pipelined schedule without k_fixup): the lists were selected from a
// snapshot that lacks the Reserves of the previous batch, whose changed nodes T (<= 64, their current records in
// `tin`, node index in RW_PAD) are the only nodes whose snapshot keys are stale; each pod's list holds its top-
// (k_j + 64) of that snapshot (LS = KSTALE keys a pod, two a lane).  Lane t of every wave then also holds T's
// node t as a second slot: T's bits are set in the changed set before P, so a prediction never takes a T node
// (every node outside T and the batch's own slots keeps its exact key, and at most 64 + j of them can precede pod
// j's best such node in its stale list); S evaluates every pod against all of T besides its own slots c < j; a
// pod whose best current key is a T node takes it in V (Reserve on the T slot).  The batch's changed nodes --
// its own slots and the T slots it reserved -- are written back and become the next batch's T.
template <bool EXT>
__device__ __forceinline__ void replay_spec(ResLds& L, const ChgSet& C, const SoA& s, const int base, const int B,
                                            const KArgs& k, int32_t* __restrict__ chosen,
                                            int32_t* __restrict__ chosen_score, int32_t global_offset,
                                            uint64_t* __restrict__ stamps, int batch_index,
                                            uint64_t* __restrict__ dev_alloc, int64_t* __restrict__ touched_out,
                                            int32_t* __restrict__ touched_cnt, uint64_t* __restrict__ pst,
                                            bool has_t, bool keep, int LS, bool sorted, const THelp th) {
  constexpr int NW = res_threads<false>() / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool ext = EXT && (k.flags & AF_EXT);
  const bool two = LS > KMAX;  // stale lists: two keys a lane
  NodeFast slot;  // lane c: the node pod c took, after every Reserve on it so far
  bool sv = false;
  int snode = -1;
  NodeFast tslot;  // lane t: node t of the previous batch's changed set T (stale lists only)
  bool tv = false, tdirty = false;
  int tnode = -1;
  // T: the previous batch of the run left its changed nodes' bits set in the changed set, their ids in
  // L.sp.tnext and their current records in L.trec
  const int64_t* const tin = has_t ? &L.trec[0][0] : nullptr;  // (non-null: T present)
  const int tin_n = has_t ? L.sp.tnext_n : 0;
  if (lane < tin_n) {
    tnode = L.sp.tnext[lane];
    int64_t w[NUM_RW];
#pragma unroll
    for (int u = 0; u < NUM_RW; u++) w[u] = L.trec[lane][u];
    rec_unpack(w, tslot);
    tv = true;
  }
  bool t_adopted = false;
  auto adopt_t = [&]() {  // first use of the T slots (wave-uniform)
    if (t_adopted) return;
    t_adopted = true;
    if (tv) {
      if (ext) ext_load(s, tnode, k, tslot);
      fast_adopt(tslot, k);
    }
  };
  int tres = 0;  // Reserves of this batch's pods on T nodes so far (the version of L.sp.tmx, reset in the prologue)
  if (wave == 0 && lane == 0) pst[8] = __builtin_amdgcn_s_memrealtime();  // T set up
  // pod j's max key over T in its current state, cached in L.sp.tmx until a pod reserves on a T node
  auto t_row = [&](int j) {
    if (L.sp.tver[j] == tres) return;
    const DevPod p = L.pod[j];
    const double ed[2] = {L.pd[j][0], L.pd[j][1]}, rd[2] = {L.pd[j][2], L.pd[j][3]};
    uint32_t tk = tv ? make_key(fast_total<EXT>(tslot, p, ed, rd, k), tnode) : 0u;
    tk = wave_max_u32(tk);
    if (lane == 0) L.sp.tmx[j] = tk, L.sp.tver[j] = tres;
  };
  // two rows at once (j1 < 0: none), independent chains (the P phase's idle waves)
  auto t_row2 = [&](int j, int j1) {
    const bool need0 = L.sp.tver[j] != tres, need1 = j1 >= 0 && L.sp.tver[j1] != tres;
    if (!need1) {
      t_row(j);
      return;
    }
    if (!need0) {
      t_row(j1);
      return;
    }
    const DevPod p = L.pod[j], p1 = L.pod[j1];
    const double ed[2] = {L.pd[j][0], L.pd[j][1]}, rd[2] = {L.pd[j][2], L.pd[j][3]};
    const double ed1[2] = {L.pd[j1][0], L.pd[j1][1]}, rd1[2] = {L.pd[j1][2], L.pd[j1][3]};
    uint32_t tk = 0, tk1 = 0;
    if (tv) {
      tk = make_key(fast_total<EXT>(tslot, p, ed, rd, k), tnode);
      tk1 = make_key(fast_total<EXT>(tslot, p1, ed1, rd1, k), tnode);
    }
    tk = wave_max_u32(tk);
    tk1 = wave_max_u32(tk1);
    if (lane == 0) {
      L.sp.tmx[j] = tk, L.sp.tver[j] = tres;
      L.sp.tmx[j1] = tk1, L.sp.tver[j1] = tres;
    }
  };
  // lane c in [lo, hi) adopts pod c's predicted node and reserves pod c on it (vol: read while wave 0 predicts)
  auto reserve_lanes = [&](int lo, int hi, bool vol) {
    if (lane >= lo && lane < hi) {
      snode = vol ? ((volatile int32_t*)L.sp.xnode)[lane] : L.sp.xnode[lane];
      sv = snode >= 0;
      if (sv) {
        rec_load_plain(s.rec + (int64_t)snode * NUM_RW, slot);  // 16-B loads (this workgroup wrote it sc1, or a
                                                                 // launch before this one)
        if (ext) ext_load(s, snode, k, slot);
        fast_adopt(slot, k);
        const DevPod pc = L.pod[lane];
        const double ed[2] = {L.pd[lane][0], L.pd[lane][1]}, rd[2] = {L.pd[lane][2], L.pd[lane][3]};
        fast_reserve(slot, pc, ed, rd);
        if (ext) ext_fast_reserve(slot, pc, k);
      }
    }
  };
  int32_t o_node = -1, o_score = -1;  // wave 0, lane j: pod j's placement
  int start = 0, win = B, rounds = 0, fetched = 0;
  const bool stamp = wave == 0 && lane == 0;  // phase stamps of the first round (ke_debug_resolve_phases)
  bool first = true;
  while (start < B) {
    const int end = min(B, start + win);
    // the first round of a batch with T whose maxima the helpers evaluate: R + S follow the prediction
    const bool prog = first && tin && th.H > 0;
    // ---- P (wave 0): pods [start, end) each take their best candidate not taken before.  Meanwhile the other
    // waves evaluate the rows' T maxima the S phase would compute (stale lists: the first round, or after a
    // Reserve on a T node).
    if (wave == 0) {
      if (C.glb) {
        if (sorted) spec_predict<true, true>(L, C, start, end, LS, two, lane);
        else spec_predict<true, false>(L, C, start, end, LS, two, lane);
      } else {
        if (sorted) spec_predict_lean(L, C, start, end, LS, two, lane);
        else spec_predict<false, false>(L, C, start, end, LS, two, lane);
      }
      if (first && lane == 0) pst[9] = __builtin_amdgcn_s_memrealtime();  // the prediction loop's end
      adopt_t();  // (its loads landed during the prediction)
      if (prog) {
        reserve_lanes(start, end, false);  // wave 0's own slots (V, write-back)
        fetched += __popcll(__ballot(lane >= start && lane < end && sv));
        if (lane == 0) pst[11] = __builtin_amdgcn_s_memrealtime();
        // the helpers' T maxima of this batch (a bounded wait: rows whose maximum did not arrive are evaluated
        // after the barrier)
        int ok = 0;
        if (lane == 0 && !th.ign) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (true) {
            if (ld_sc1(th.tready + batch_index) >= th.H) {
              ok = 1;
              break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > T_HELP_WAIT_TICKS) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        ok = __builtin_amdgcn_readfirstlane(ok);
        if (ok && lane >= start && lane < end) {
          L.sp.tmx[lane] = ld_sc1(th.tmx + (batch_index & 1) * MAX_BATCH + lane);
          L.sp.tver[lane] = 0;  // (tres == 0: the first round)
        }
        if (lane == 0) {
          pst[10] = __builtin_amdgcn_s_memrealtime();
          pst[12] = ok;
        }
      }
    } else if (prog) {
      // ---- progressive R + S (waves 1..NW-1): once pod hi-1 of a chunk [lo, hi) is predicted, its slots are
      // reserved and evaluated against every later pod of the window
      adopt_t();
      uint64_t w_wait = 0, w_res = 0, w_rows = 0, w_t = __builtin_amdgcn_s_memrealtime();  // wave 1's stamps
      // slot-major: a chunk's 16 slots are held four times a wave (lane l: slot lo + l % 16, group
      // g = 4 (wave - 1) + l / 16 of GW), and group g evaluates its slot c against the pods j = c + 1 + g + GW t:
      // every pair (c, j > c) of the chunk is evaluated once its slot is known, max-reduced into mrow[j] with an
      // LDS atomic -- rows wait for no later prediction, so after the loop only the last chunk's pairs remain
      constexpr int GW = 4 * (NW - 1);
      const int g = 4 * (wave - 1) + (lane >> 4);
      NodeFast pslot;
      int pnode = -1;
      for (int lo = start; lo < end; lo += PCH) {
        const int hi = min(end, lo + PCH);
        if (lane == 0) {  // an LDS wait on wave 0 of the same workgroup (co-resident by construction), bounded
                          // all the same: wave 0 never reaches a barrier before every xnode of [start, end) is
                          // written, and a wait past 2 s fails the call (KERR_LDS_WAIT) instead of hanging it
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (((volatile int32_t*)L.sp.xnode)[hi - 1] == XN_PENDING) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > HANDOFF_TIMEOUT_TICKS) {
              __hip_atomic_fetch_or(s.kerr, KERR_LDS_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        w_wait += t1 - w_t;
        // lane l adopts slot c = lo + l % 16 and reserves pod c on it (lo is a multiple of 16: the first round
        // starts at pod 0); lanes [lo, hi) keep it as their own slot for V and the later rounds
        const int c = lo + (lane & 15);
        pnode = c < hi ? ((volatile int32_t*)L.sp.xnode)[c] : -1;
        const bool pv = pnode >= 0;
        if (pv) {
          rec_load_plain(s.rec + (int64_t)pnode * NUM_RW, pslot);
          if (ext) ext_load(s, pnode, k, pslot);
          fast_adopt(pslot, k);
          const DevPod pc = L.pod[c];
          const double ed[2] = {L.pd[c][0], L.pd[c][1]}, rd[2] = {L.pd[c][2], L.pd[c][3]};
          fast_reserve(pslot, pc, ed, rd);
          if (ext) ext_fast_reserve(pslot, pc, k);
        }
        if (lane >= lo && lane < hi) {
          snode = pnode;
          sv = pv;
          if (pv) slot = pslot;
        }
        w_t = __builtin_amdgcn_s_memrealtime();
        w_res += w_t - t1;
        constexpr int RS = EXT ? 1 : 2;  // chains a pass
        for (int j = c + 1 + g; pv && j < end; j += RS * GW) {
          const DevPod p = L.pod[j];
          const double ed[2] = {L.pd[j][0], L.pd[j][1]}, rd[2] = {L.pd[j][2], L.pd[j][3]};
          const uint32_t kc = make_key(fast_total<EXT>(pslot, p, ed, rd, k), pnode);
          uint32_t kc1 = 0u;
          const int j1 = j + GW;
          if (RS == 2 && j1 < end) {
            const DevPod p1 = L.pod[j1];
            const double ed1[2] = {L.pd[j1][0], L.pd[j1][1]}, rd1[2] = {L.pd[j1][2], L.pd[j1][3]};
            kc1 = make_key(fast_total<EXT>(pslot, p1, ed1, rd1, k), pnode);
          }
          if (kc) atomicMax(&L.sp.mrow[j], kc);
          if (kc1) atomicMax(&L.sp.mrow[j1], kc1);
        }
        t1 = __builtin_amdgcn_s_memrealtime();
        w_rows += t1 - w_t;
        w_t = t1;
      }
      if (wave == 1 && lane == 0) {  // ke_debug_resolve_waves: wave 1's polls, record loads + Reserves, rows
        pst[13] = w_wait;
        pst[14] = w_res | (w_rows << 32);
        pst[15] = w_t;
      }
    } else if (tin) {
      adopt_t();
      constexpr int RT = EXT ? 1 : 2;
      for (int j = start + wave - 1; j < end; j += RT * (NW - 1)) t_row2(j, RT == 2 && j + NW - 1 < end ? j + NW - 1 : -1);
      if (first && wave == 1 && lane == 0) pst[10] = __builtin_amdgcn_s_memrealtime();  // wave 1's T rows
    }
    __syncthreads();
    if (stamp && first) pst[1] = __builtin_amdgcn_s_memrealtime();
    if (prog) {
      // the T maxima into the rows: the helpers' (wave 0 polled them), else evaluated here.  With every row's
      // maximum in (the usual case: the same LDS words on every wave, so the test is uniform) wave 0 merges
      // them one lane a row
      const bool in = lane >= start && lane < end;
      if (!__ballot(in && L.sp.tver[lane] != tres)) {
        if (wave == 0 && in) L.sp.mrow[lane] = max(L.sp.mrow[lane], L.sp.tmx[lane]);
      } else {
        for (int j = start + wave; j < end; j += NW) {
          t_row(j);
          if (lane == 0) L.sp.mrow[j] = max(L.sp.mrow[j], L.sp.tmx[j]);
        }
      }
    } else {
      // ---- R (every wave): lane c in [start, end) adopts pod c's predicted node and reserves pod c on it
      reserve_lanes(start, end, false);
      if (wave == 0) fetched += __popcll(__ballot(lane >= start && lane < end && sv));
      if (stamp && first) pst[11] = __builtin_amdgcn_s_memrealtime();  // wave 0's slots reserved (R)
      // ---- S (rows over the waves): pod j against every slot c < j (and every T slot)
      // Two rows a pass (j and j + NW): two independent evaluation chains for the latency-bound wave (one with
      // the ext slots: their registers would spill).
      constexpr int RS = EXT ? 1 : 2;
      for (int j = start + wave; j < end; j += RS * NW) {
        const int j1 = j + NW;
        const bool has1 = RS == 2 && j1 < end;  // (wave-uniform)
        const DevPod p = L.pod[j];
        const double ed[2] = {L.pd[j][0], L.pd[j][1]}, rd[2] = {L.pd[j][2], L.pd[j][3]};
        uint32_t kc = 0, kc1 = 0;
        if (has1) {
          const DevPod p1 = L.pod[j1];
          const double ed1[2] = {L.pd[j1][0], L.pd[j1][1]}, rd1[2] = {L.pd[j1][2], L.pd[j1][3]};
          if (sv && lane < j) kc = make_key(fast_total<EXT>(slot, p, ed, rd, k), snode);
          if (sv && lane < j1) kc1 = make_key(fast_total<EXT>(slot, p1, ed1, rd1, k), snode);
        } else if (sv && lane < j) {
          kc = make_key(fast_total<EXT>(slot, p, ed, rd, k), snode);
        }
        uint32_t tk = 0, tk1 = 0;
        if (tin) {  // T changes only when a pod of the batch reserves on it: pod j's T max is cached meanwhile
          t_row(j);  // (this wave's own LDS writes: in order)
          tk = L.sp.tmx[j];
          if (has1) {
            t_row(j1);
            tk1 = L.sp.tmx[j1];
          }
        }
        const uint32_t mx = max(wave_max_u32(kc), tk);
        const uint32_t mx1 = has1 ? max(wave_max_u32(kc1), tk1) : 0u;
        if (lane == 0) {
          L.sp.mrow[j] = mx;
          if (has1) L.sp.mrow[j1] = mx1;
        }
      }
    }
    __syncthreads();
    if (stamp && first) pst[2] = __builtin_amdgcn_s_memrealtime();
    // ---- V (wave 0): the first pod whose best changed node beats its prediction
    if (wave == 0) {
      const bool in = lane >= start && lane < end;
      const uint32_t xk = in ? L.sp.xkey[lane] : 0u, mk = in ? L.sp.mrow[lane] : 0u;
      const uint64_t bad = __ballot(in && mk > xk);
      const int jf = bad ? __ffsll((unsigned long long)bad) - 1 : end;
      if (lane >= start && lane < jf) {
        const int xn = L.sp.xnode[lane];
        o_node = xn >= 0 ? xn + global_offset : -1;
        o_score = xk ? key_score(xk) : -1;
      }
      if (lane == jf && jf < end) {  // pod jf takes the changed node of its best current key
        o_node = key_node(mk) + global_offset;
        o_score = key_score(mk);
      }
      if (lane >= jf && lane < end) {  // predictions that did not happen leave the changed set
        const int xn = L.sp.xnode[lane];
        if (xn >= 0) chg_unset(C, xn);
      }
      if (lane == 0) L.sp.jf = jf;
    }
    __syncthreads();
    if (stamp && first) pst[3] = __builtin_amdgcn_s_memrealtime();
    first = false;
    const int jf = L.sp.jf;
    if (jf < end) {
      if (lane >= jf && lane < end) sv = false;
      const int wn = key_node(L.sp.mrow[jf]);
      const bool on_c = sv && snode == wn, on_t = tv && tnode == wn;
      if (on_c || on_t) {  // pod jf's Reserve on that slot (every wave keeps its copy)
        const DevPod pc = L.pod[jf];
        const double ed[2] = {L.pd[jf][0], L.pd[jf][1]}, rd[2] = {L.pd[jf][2], L.pd[jf][3]};
        if (on_c) {
          fast_reserve(slot, pc, ed, rd);
          if (ext) ext_fast_reserve(slot, pc, k);
        } else {
          fast_reserve(tslot, pc, ed, rd);
          if (ext) ext_fast_reserve(tslot, pc, k);
          tdirty = true;
        }
      }
      if (tin && __ballot(on_t)) tres++;  // same T slots on every wave: uniform
      win = max(8, 2 * (jf - start + 1));
      start = jf + 1;
      rounds++;
    } else {
      start = end;
      win = min(MAX_BATCH, 2 * win);
    }
  }
  if (wave != 0) return;  // (T came from `tin` into registers the S phases consumed: the write-back may replace it)
  if (lane == 0) pst[5] = __builtin_amdgcn_s_memrealtime();
  if (lane < B) {
    chosen[base + lane] = o_node;
    chosen_score[base + lane] = o_score;
    dev_alloc[base + lane] = 0;
  }
  // the changed nodes' rows back to the SoA, their replay records, the compact list for the next batch (T of a
  // stale-list batch, or k_fixup's touched rows)
  const uint64_t vm = __ballot(sv), tm = __ballot(tdirty);
  auto write_back = [&](const NodeFast& f, int node, int pos) {
    const int64_t st = s.stride;
    int64_t* fr = s.f + node;
#pragma unroll
    for (int v = 0; v < 2; v++)
#pragma unroll
      for (int q = 0; q < 2; q++) {
        st_sc1(fr + (F_FH + 2 * v + q) * st, f.fh[v][q]);
        st_sc1(fr + (F_SA + 2 * v + q) * st, (int64_t)f.sa[v][q]);
      }
    st_sc1(fr + (F_NREQ + 0) * st, (int64_t)f.nreq[0]);
    st_sc1(fr + (F_NREQ + 1) * st, (int64_t)f.nreq[1]);
    rec_store_dyn<__HIP_MEMORY_SCOPE_AGENT>(s.rec + (int64_t)node * NUM_RW, f);  // sc1: read by k_eval_plain
    if (ext) ext_store(s, node, f, k);
    if (keep) rec_to_words(f, node, L.trec[pos]);  // the next batch's T slot
    else if (touched_out) rec_store_full(touched_out + (int64_t)pos * NUM_RW, f, node);
  };
  if (sv) write_back(slot, snode, lanes_below(vm));
  if (tdirty) write_back(tslot, tnode, __popcll(vm) + lanes_below(tm));
  if (keep) {  // the changed nodes stay in the set as the next batch's T; T nodes no pod reserved leave it
    if (sv) L.sp.tnext[lanes_below(vm)] = snode;
    if (tdirty) L.sp.tnext[__popcll(vm) + lanes_below(tm)] = tnode;
    if (lane == 0) L.sp.tnext_n = __popcll(vm) + __popcll(tm);
    if (th.tlist) {  // ... and for the helpers / k_patch (drained before done[batch_index] is published)
      int32_t* tl = th.tlist + (batch_index & 1) * (1 + MAX_BATCH);
      if (sv) st_sc1(tl + 1 + lanes_below(vm), (int32_t)snode);
      if (tdirty) st_sc1(tl + 1 + __popcll(vm) + lanes_below(tm), (int32_t)tnode);
      if (lane == 0) st_sc1(tl, (int32_t)(__popcll(vm) + __popcll(tm)));
    }
    if (tv && !tdirty) chg_unset(C, tnode);
  } else {  // every bit still set belongs to a taken node or to T
    if (sv) chg_clear_word(C, snode);
    if (tv) chg_clear_word(C, tnode);
  }
  if (touched_out && lane == 0) st_sc1(touched_cnt, (int32_t)(__popcll(vm) + __popcll(tm)));
  if (lane == 0) {
    stamps[batch_index + 1] = __builtin_amdgcn_s_memrealtime();
    pst[6] = (uint64_t)(uint32_t)fetched | ((uint64_t)rounds << 32);  // records fetched | failed rounds
    pst[7] = (uint64_t)(__popcll(vm) + __popcll(tm));
  }
  if (!keep) drain_stores();  // (keep: the next batch's prologue drains them behind its loads, then publishes)
}

// zero the LDS bitmap words of node ids [0, n_nodes) (all threads; once per launch)
__device__ __forceinline__ ChgSet chg_init(ResLds& L, uint32_t* glb, int n_nodes) {
  const int words = glb ? 0 : (n_nodes + 31) >> 5;
  for (int t = threadIdx.x; t < words; t += blockDim.x) L.chg[t] = 0u;
  return ChgSet{L.chg, glb};
}

template <bool DS, bool NUMA, bool QUOTA, bool EXT>
__device__ __forceinline__ void replay_batch(ResLds& L, const ChgSet& C, const SoA& s, const int base, const int B,
                                             const KArgs& k, int32_t* __restrict__ chosen,
                                             int32_t* __restrict__ chosen_score, int32_t global_offset,
                                             uint64_t* __restrict__ stamps, int batch_index,
                                             uint64_t* __restrict__ dev_alloc, int64_t* __restrict__ numa_alloc,
                                             int64_t* __restrict__ touched_out, int32_t* __restrict__ touched_cnt,
                                             uint64_t* __restrict__ pst);

// One batch: prologue on every thread of the workgroup (the batch's pods and exact candidate lists
// into LDS), replay on wave 0 (the other waves skip it).
template <bool DS, bool NUMA, bool QUOTA, bool EXT = true>
__device__ __forceinline__ void resolve_batch(ResLds& L, const ChgSet& C, const SoA& s, const DevPod* __restrict__ pods,
                                              const int base, const int B, const KArgs& k,
                                              const uint32_t* __restrict__ cand, const int32_t* __restrict__ cand_cnt,
                                              int32_t* __restrict__ chosen, int32_t* __restrict__ chosen_score,
                                              int32_t global_offset, uint64_t* __restrict__ stamps,
                                              uint64_t* __restrict__ pstamps, int batch_index,
                                              uint64_t* __restrict__ dev_alloc, int64_t* __restrict__ numa_alloc,
                                              int64_t* __restrict__ touched_out = nullptr,
                                              int32_t* __restrict__ touched_cnt = nullptr,
                                              bool has_t = false, bool keep = false, int LS = KMAX,
                                              bool sorted = false, int32_t* __restrict__ pub_done = nullptr,
                                              const THelp th = THelp{nullptr, nullptr, nullptr, 0, 0, nullptr}) {
  const int tid = threadIdx.x;
  constexpr int RES_THREADS = res_threads<NUMA>();
  if (tid == 0) pstamps[PST * batch_index] = __builtin_amdgcn_s_memrealtime();
  // `pub_done` (stale-list runs): the previous batch's done flag, published once wave 0's stores of it have
  // drained -- here, behind this batch's loads, rather than before them
  // candidate keys at stride LS, 16 B a load, issued together with their counts and the pods' loads (one round
  // trip; sc1 buffer loads: a concurrent launch wrote them), then the slots past a list's count zeroed
  constexpr int U = MAX_BATCH * KSTALE / 4 / RES_THREADS;  // 16-B chunks per thread
  const int lsh = LS == KSTALE ? 7 : 6, nk = MAX_BATCH * LS;
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(cand), 0, nk * 4, 0x00020000);
  uint4 q[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int t = 4 * (u * RES_THREADS + tid), j = t >> lsh;
    if (t < nk && j < B) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(crs, t * 4, 0, 16);  // aux 16: sc1
      q[u] = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
      q[u] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  if (tid < B) {
    L.cnt[tid] = ld_sc1(cand_cnt + tid);
    const DevPod pd = pods[base + tid];
    L.pod[tid] = pd;
    L.pd[tid][0] = (double)pd.est[0];
    L.pd[tid][1] = (double)pd.est[1];
    L.pd[tid][2] = (double)pd.req[0];
    L.pd[tid][3] = (double)pd.req[1];
    if (DS) {  // written by this batch's eval / select, earlier on the same stream
      L.dsm[tid] = s.dsb[DSB_MAX + tid];
      L.dsc[tid] = (int32_t)s.dsb[DSB_CNT + tid];
    }
  }
  if (has_t && tid < B) L.sp.tver[tid] = -1;  // no pod's T max computed yet (replay_spec)
  if (tid < B) L.sp.xnode[tid] = XN_PENDING, L.sp.mrow[tid] = 0u;  // (the progressive S max-reduces into mrow)
  if (pub_done && tid == 0) {  // (wave 0 issued every store of the previous batch)
    drain_stores();
    st_sc1(pub_done, 1);
  }
  __syncthreads();  // the counts
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int t = 4 * (u * RES_THREADS + tid), j = t >> lsh, c = t & (LS - 1);
    if (t < nk) {
      const int n = j < B ? L.cnt[j] : 0;
      uint4 w = q[u];
      w.x = c < n ? w.x : 0u;
      w.y = c + 1 < n ? w.y : 0u;
      w.z = c + 2 < n ? w.z : 0u;
      w.w = c + 3 < n ? w.w : 0u;
      *reinterpret_cast<uint4*>(&L.cand[t]) = w;
    }
  }
  __syncthreads();
  if (tid == 0) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    for (int u = 1; u < 6; u++) pstamps[PST * batch_index + u] = t;
    for (int u = 8; u < 12; u++) pstamps[PST * batch_index + u] = t;
    for (int u = 12; u < 16; u++) pstamps[PST * batch_index + u] = 0;
  }
  if constexpr (!DS && !NUMA && !QUOTA) {  // plain batch: the speculative replay on every wave
    __builtin_amdgcn_s_setprio(3);
    replay_spec<EXT>(L, C, s, base, B, k, chosen, chosen_score, global_offset, stamps, batch_index, dev_alloc,
                     touched_out, touched_cnt, pstamps + PST * batch_index, has_t, keep, LS, sorted, th);
    __builtin_amdgcn_s_setprio(0);
    return;
  }
  if (tid >= 64) return;  // the replay is one wavefront: wave-level ordering only from here on
  // the next batch's eval waves may share this SIMD (pipelined schedule): the replay issues first
  __builtin_amdgcn_s_setprio(3);
  replay_batch<DS, NUMA, QUOTA, EXT>(L, C, s, base, B, k, chosen, chosen_score, global_offset, stamps, batch_index,
                                dev_alloc, numa_alloc, touched_out, touched_cnt, pstamps + PST * batch_index);
  __builtin_amdgcn_s_setprio(0);
}


// The sequential replay of one batch (wave 0).
//   Lane c owns the c-th node changed in this batch: its row lives in that lane's registers, so the
//   per-pod re-evaluation of every changed node is one register-only eval across the lanes.  Per pod j:
//   the best unchanged candidate bu (wave max over its list minus the changed nodes), the exact score
//   of every changed node, the better of the two, Reserve on the owner lane.  The row of bu's node is
//   fetched from the SoA by the next free lane at the start of the pod, into spare registers, so its
//   latency hides under the re-evaluation; it becomes that lane's row if bu wins.  Pod j+1's record
//   and candidates are read during pod j, its changed flags right after pod j's Reserve.
template <bool DS, bool NUMA, bool QUOTA, bool EXT>
__device__ __forceinline__ void replay_batch(ResLds& L, const ChgSet& C, const SoA& s, const int base, const int B,
                                             const KArgs& k, int32_t* __restrict__ chosen,
                                             int32_t* __restrict__ chosen_score, int32_t global_offset,
                                             uint64_t* __restrict__ stamps, int batch_index,
                                             uint64_t* __restrict__ dev_alloc, int64_t* __restrict__ numa_alloc,
                                             int64_t* __restrict__ touched_out, int32_t* __restrict__ touched_cnt,
                                             uint64_t* __restrict__ pst) {
  const uint32_t* const s_cand = L.cand;
  const DevPod* const s_pod = L.pod;
  const int lane = threadIdx.x & 63;
  int n_chg = 0, n_fetch = 0;
  // changed nodes as replay records (fast_total); NUMA / DeviceShare batches: full rows (+ zones / devices)
  constexpr bool FAST = !NUMA && !DS;
  NodeRegs mine;   // NUMA: the changed node's row
  Row spare;       // NUMA, lane n_chg: the row of the pod's best unchanged candidate
  NodeFast fast;   // FAST: the changed node's record
  NodeFast sparef; // FAST, lane n_chg: the record of the pod's best unchanged candidate
  int my_node = -1;
  bool my_expired = false;
  int32_t o_node = -1, o_score = -1;  // lane j: pod j's placement
  uint64_t o_alloc = 0;
  QuotaRegs Q;  // ElasticQuota used / non-preemptible used, lane-distributed (QUOTA only)
  if (QUOTA)
#pragma unroll
    for (int b = 0; b < 4; b++)
#pragma unroll
      for (int r = 0; r < 2; r++) {
        Q.u[b][r] = qtf(s, QF_USED + r, 64 * b + lane);
        Q.n[b][r] = qtf(s, QF_NP + r, 64 * b + lane);
      }
  DevPod pod = s_pod[0];
  double pdd[4] = {L.pd[0][0], L.pd[0][1], L.pd[0][2], L.pd[0][3]};
  uint32_t ck = s_cand[lane];
  bool chg = false;  // changed flag of this lane's candidate (pods < j); nothing is changed at j = 0
  RPROF_DECL
  for (int j = 0; j < B; j++) {
    const bool more = j + 1 < B;
    const DevPod pod_n = s_pod[more ? j + 1 : j];
    const int jn = more ? j + 1 : j;
    const double pdd_n[4] = {L.pd[jn][0], L.pd[jn][1], L.pd[jn][2], L.pd[jn][3]};
    const double estd[2] = {pdd[0], pdd[1]}, reqd[2] = {pdd[2], pdd[3]};
    const uint32_t ck_n = more ? s_cand[(j + 1) * KMAX + lane] : 0u;
    const uint32_t bu = wave_max_u32(chg ? 0u : ck);  // best unchanged snapshot candidate
    RPROF(0)
    if (bu != 0 && lane == n_chg) {
      if constexpr (FAST) {
        rec_load(s.rec + (int64_t)key_node(bu) * NUM_RW, sparef);
        if (EXT && (k.flags & AF_EXT)) ext_load(s, key_node(bu), k, sparef);
      }
      else load_row_sc1(s, key_node(bu), spare);
    }
    n_fetch += bu != 0;
    RPROF(1)
    uint32_t kc = 0;  // exact re-evaluation of the nodes changed earlier in this batch
    uint32_t craw = 0;  // DeviceShare batch: 1 + the changed node's current raw DeviceShare score (0 = infeasible)
    const uint32_t m0 = DS ? L.dsm[j] : 0u;  // the snapshot's normalisation max of pod j (DeviceShare pods)
    uint32_t snap = 0;  // DeviceShare batch: 1 + the changed node's raw score for pod j in the snapshot
    if (DS && (pod.flags & PF_DS) && lane < n_chg) snap = s.dsraw[(int64_t)(j) * s.stride + my_node];
    if (lane < n_chg) {
      int32_t tot;
      if constexpr (NUMA) {
        NumaNode nv;
        numa_load(s, my_node, nv);
        tot = eval_pair<false, NUMA>(mine, my_expired, pod, k, s, my_node, nv).total;
      } else if constexpr (DS) {
        NumaNode nv;  // unused without NUMA policies
        const EvalOut o = eval_pair<true, false>(mine, my_expired, pod, k, s, my_node, nv);
        tot = o.total;
        if (tot >= 0) {
          craw = (uint32_t)o.ds + 1;
          tot += k.wp_ds * ds_norm(o.ds, m0);
        }
      } else {
        tot = fast_total<EXT>(fast, pod, estd, reqd, k);
      }
      kc = make_key(tot, my_node);
    }
    RPROF(2)
    const uint32_t bc = wave_max_u32(kc);
    RPROF(3)
    // DeviceShare batch: pod j's candidate keys used the snapshot max m0.  It still is the max over the
    // feasible nodes when some node that attained it in the snapshot is unchanged (it still does) and no
    // changed node now exceeds it; otherwise the batch stops here and the host re-runs pods j..
    if constexpr (DS) {
      if (pod.flags & PF_DS) {
        const uint32_t cmax = wave_max_u32(craw);
        // snapshot max-attaining nodes that changed since: the rest still attain m0
        const int lost = __popcll(__ballot(lane < n_chg && snap == m0));
        const bool safe = m0 == 0 ? cmax == 0 : (cmax <= m0 && L.dsc[j] > lost);
        if (!safe) {
          if (lane == 0) s.dsb[DSB_CUT] = (uint32_t)(base + j);
          break;
        }
      }
    }
    // ElasticQuota PreFilter: a refused pod is placed nowhere
    int64_t qreq[2] = {0, 0};
    const bool adm = !QUOTA || !pod.quota || quota_admit_r(s, pod, k, Q, qreq);
    const uint32_t w = adm ? max(bu, bc) : 0u;
    if (w != 0) {
      int owner;
      if (w == bc) {
        owner = __ffsll((unsigned long long)__ballot(lane < n_chg && kc == w)) - 1;
      } else {
        owner = n_chg++;
        if (lane == owner) {
          my_node = key_node(w);
          if constexpr (FAST) {
            fast = sparef;
            fast_adopt(fast, k);
          } else {
            regs_from_row(spare, mine);
            prepare_row(mine);
            my_expired = node_expired(mine, k);
          }
          chg_set(C, my_node);
        }
      }
      RPROF(4)
      // Reserve: LoadAware assign (the new pod has no PodMetric -> counted at its estimate in every
      // non-prod term, and in the prod terms when it is prod), NodeInfo.Requested += requests.
      uint64_t al = 0;
      if (DS && (pod.flags & PF_DS)) {  // DeviceShare Reserve (wave-uniform branch), before NodeNUMAResource's
        const uint32_t nfl = (uint32_t)__builtin_amdgcn_readlane((int)(FAST ? fast.nflags : mine.flags), owner);
        const int node = (int)key_node(w);  // the chosen node (my_node of the owner lane)
        // the device SoA is global: a later pod of the batch re-evaluating this node reads it back
        // (wave_lds_sync below)
        if (nfl & NF_DS_CACHE) al = ds_reserve_wave(s, node, pod, k, lane);
      }
      if (lane == owner) {
        if constexpr (FAST) {
          fast_reserve(fast, pod, estd, reqd);
          if (EXT && (k.flags & AF_EXT)) ext_fast_reserve(fast, pod, k);  // NodeInfo (NonZero)Requested, Pods
        } else {
          if ((mine.flags & NF_HAS_METRIC) && !(mine.flags & NF_NM_NIL)) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
              if (mine.flags & nf_fh_on(0, q)) mine.fh[0][q] -= pod.est[q];
              mine.sa[0][q] -= pod.est[q];
              if (pod.flags & PF_PROD) {
                if (mine.flags & nf_fh_on(1, q)) mine.fh[1][q] -= pod.est[q];
                mine.sa[1][q] -= pod.est[q];
              }
            }
          }
          mine.nreq[0] += pod.req[0];
          mine.nreq[1] += pod.req[1];
        }
        if (!FAST && (k.flags & AF_EXT)) ext_reserve(s, my_node, pod, k);  // read back by the next re-evaluations
        // DeviceShare Reserve (the device SoA is global: a later pod of the batch re-evaluating this node
        // reads it back, wave_lds_sync below)
        if (NUMA) {  // NodeNUMAResource Reserve: the zones of a NUMA-policy node
          int64_t* out16 = numa_alloc + (int64_t)(base + j) * 16;
          const int pol = pf_numa_policy(pod.flags) ? pf_numa_policy(pod.flags) : nf_numa_policy(mine.flags);
          const RsvOvr* nro = (mine.flags & NF_RSV_CS) ? rsv_ovr_of(s, my_node) : nullptr;
          if (!(pod.flags & PF_NUMA_SKIP) && pol != KE_NUMA_POLICY_NONE && nro && nro->numa_on) {
            NumaNode nv;  // the nominated reservation's (or the node's own) allocation k_numa_views computed
            numa_load(s, my_node, nv);
            numa_reserve_dist(s, my_node, mine.flags, nv, nro->numa_dist, out16);
          } else if (!(pod.flags & PF_NUMA_SKIP) && pol != KE_NUMA_POLICY_NONE) {
            NumaNode nv;
            numa_load(s, my_node, nv);
            const NumaPick pk = numa_admit<false>(s, my_node, mine.flags, pol, nv, pod, k);
            numa_reserve(s, my_node, mine.flags, nv, pk.status == KE_CODE_SUCCESS ? pk.aff : 0u, pod, out16);
          } else {
#pragma unroll
            for (int t = 0; t < 16; t++) out16[t] = 0;
          }
        }
      }
      if (QUOTA && pod.quota) quota_reserve_r(s, pod, Q, qreq, lane);  // ElasticQuota Reserve
      if (DS) {
        const uint64_t a = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(al >> 32), owner) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)al, owner);
        if (lane == j) o_alloc = a;
      }
      if (lane == j) {
        o_node = key_node(w) + global_offset;
        o_score = key_score(w);
      }
    } else if (NUMA && lane == 0) {
#pragma unroll
      for (int t = 0; t < 16; t++) numa_alloc[(int64_t)(base + j) * 16 + t] = 0;
    }
    RPROF(5)
    // pod j+1's changed flags, read after this Reserve's bitmap update (LDS ops of a wave execute in
    // order), so they already include pod j's new node
    const bool chg_n = ck_n != 0 && chg_test(C, key_node(ck_n));
    if (NUMA || DS) wave_lds_sync();  // the next re-evaluation reads the zones / devices this Reserve patched
    else __atomic_signal_fence(__ATOMIC_SEQ_CST);
    pod = pod_n;
#pragma unroll
    for (int u = 0; u < 4; u++) pdd[u] = pdd_n[u];
    ck = ck_n;
    chg = chg_n;
    RPROF(6)
  }
  RPROF_FLUSH(0, B)
  if (lane < B) {
    chosen[base + lane] = o_node;
    chosen_score[base + lane] = o_score;
    dev_alloc[base + lane] = o_alloc;
  }
  if (QUOTA)
#pragma unroll
    for (int b = 0; b < 4; b++)
#pragma unroll
      for (int r = 0; r < 2; r++) {
        s.qt[(QF_USED + r) * QT_STRIDE + 64 * b + lane] = Q.u[b][r];
        s.qt[(QF_NP + r) * QT_STRIDE + 64 * b + lane] = Q.n[b][r];
      }
  if (lane < n_chg) {
    // the patched rows back to the SoA (sc1: read by the next batches' evals on other CUs), the replay
    // records (this workgroup's later batches, later launches), and the compact list of the changed
    // records for the next batch's k_fixup (pipelined runs; sc1, read by a concurrent launch)
    const int64_t st = s.stride;
    int64_t* f = s.f + my_node;
    int64_t* rec = s.rec + (int64_t)my_node * NUM_RW;
    if constexpr (FAST) {
#pragma unroll
      for (int v = 0; v < 2; v++)
#pragma unroll
        for (int q = 0; q < 2; q++) {
          st_sc1(f + (F_FH + 2 * v + q) * st, fast.fh[v][q]);
          st_sc1(f + (F_SA + 2 * v + q) * st, (int64_t)fast.sa[v][q]);
        }
      st_sc1(f + (F_NREQ + 0) * st, (int64_t)fast.nreq[0]);
      st_sc1(f + (F_NREQ + 1) * st, (int64_t)fast.nreq[1]);
      rec_store_dyn<__HIP_MEMORY_SCOPE_AGENT>(rec, fast);
      if (EXT && (k.flags & AF_EXT)) ext_store(s, my_node, fast, k);
      if (touched_out) rec_store_full(touched_out + (int64_t)lane * NUM_RW, fast, my_node);
    } else {
#pragma unroll
      for (int v = 0; v < 2; v++)
#pragma unroll
        for (int q = 0; q < 2; q++) {
          st_sc1(f + (F_FH + 2 * v + q) * st, mine.fh[v][q]);
          st_sc1(f + (F_SA + 2 * v + q) * st, mine.sa[v][q]);
        }
      st_sc1(f + (F_NREQ + 0) * st, mine.nreq[0]);
      st_sc1(f + (F_NREQ + 1) * st, mine.nreq[1]);
      int64_t w[NUM_RW];
      rec_from_regs(mine, k, w);
#pragma unroll
      for (int u = 0; u < NUM_RW; u++) __hip_atomic_store(rec + u, w[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    chg_clear_word(C, my_node);  // the bitmap is zero again for the next batch
  }
  if (touched_out && lane == 0) st_sc1(touched_cnt, (int32_t)n_chg);
  if (lane == 0) {
    stamps[batch_index + 1] = __builtin_amdgcn_s_memrealtime();
    pst[6] = (uint64_t)n_fetch;  // candidate rows fetched from the SoA
    pst[7] = (uint64_t)n_chg;    // rows changed (written back)
  }
  drain_stores();  // every hand-off store is performed before the workgroup publishes the batch
}

template <bool DS, bool NUMA, bool QUOTA>
__global__ __launch_bounds__(res_threads<NUMA>()) void k_resolve(SoA s, const DevPod* __restrict__ pods, const int32_t* __restrict__ batch_base,
                                                int batch_pods, KArgs k, const uint32_t* __restrict__ cand,
                                                const int32_t* __restrict__ cand_cnt, int32_t* __restrict__ chosen,
                                                int32_t* __restrict__ chosen_score, int32_t global_offset,
                                                uint64_t* __restrict__ stamps, uint64_t* __restrict__ pstamps,
                                                int batch_index, uint64_t* __restrict__ dev_alloc,
                                                int64_t* __restrict__ numa_alloc, uint32_t* __restrict__ chg_glb,
                                                int n_nodes, int sorted) {
  __shared__ ResLds L;
  const ChgSet C = chg_init(L, chg_glb, n_nodes);
  resolve_batch<DS, NUMA, QUOTA>(L, C, s, pods, *batch_base, batch_pods, k, cand, cand_cnt, chosen, chosen_score,
                                 global_offset, stamps, pstamps, batch_index, dev_alloc, numa_alloc, nullptr, nullptr,
                                 false, false, KMAX, sorted != 0);
}

// A T-row helper workgroup (THelp; helper h of H): for every batch b > b0 of the run, once the Reserve
// workgroup has published done[b-1] (the changed nodes' records and list drained), the T slots in registers
// (lane t: changed node t of batch b-1, as replay_spec's tslot) and the T maximum of every pod j of batch b
// whose pair index (j / 2) falls to this helper: max_t key(fast_total(T node t, pod j)).  Published to tmx with
// one relaxed add on tready[b] per helper.  A batch the Reserve workgroup has already finished (done[b]) is
// skipped; the Reserve workgroup falls back to its own rows for any batch whose maxima arrive late, so no
// wait of the run depends on a helper being resident.
template <bool EXT>
__device__ __noinline__ void t_helper(ResLds& L, const SoA& s, const DevPod* __restrict__ pods,
                                      const int32_t* __restrict__ bases, int b0, int nb, const KArgs& k,
                                      const int32_t* __restrict__ done, int32_t* __restrict__ err, const THelp th,
                                      int h, int32_t* s_go) {
  constexpr int NW = res_threads<false>() / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool ext = EXT && (k.flags & AF_EXT);
  for (int b = b0 + 1; b < b0 + nb; b++) {
    const int base = bases[b], B = bases[b + 1] - base;
    if ((int)threadIdx.x < B) {  // the batch's pods (uploaded before the launch): before the wait
      const DevPod pd = pods[base + threadIdx.x];
      L.pod[threadIdx.x] = pd;
      L.pd[threadIdx.x][0] = (double)pd.est[0];
      L.pd[threadIdx.x][1] = (double)pd.est[1];
      L.pd[threadIdx.x][2] = (double)pd.req[0];
      L.pd[threadIdx.x][3] = (double)pd.req[1];
    }
    if (threadIdx.x == 0) {
      int go = -1;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (true) {  // (no error word of its own: a stuck run is the Reserve workgroup's to report)
        if (ld_sc1(done + (b - 1)) != 0) {
          go = ld_sc1(done + b) != 0 ? 0 : 1;
          break;
        }
        if (ld_sc1(err) != 0 || __builtin_amdgcn_s_memrealtime() - t0 > HANDOFF_TIMEOUT_TICKS) break;
        __builtin_amdgcn_s_sleep(1);
      }
      *s_go = go;
    }
    __syncthreads();
    const int go = *s_go;
    if (go < 0) return;
    if (go > 0) {
      // T of batch b: the changed nodes of batch b-1 (count and ids in one round trip, then the records)
      const int32_t* tl = th.tlist + ((b - 1) & 1) * (1 + MAX_BATCH);
      const int tn = ld_sc1(tl);
      const int32_t tid_node = ld_sc1(tl + 1 + lane);
      const bool tv = lane < tn;
      NodeFast tslot;
      const int tnode = tv ? tid_node : -1;
      if (tv) {
        rec_load<__HIP_MEMORY_SCOPE_AGENT>(s.rec + (int64_t)tnode * NUM_RW, tslot);
        if (ext) ext_load(s, tnode, k, tslot);
        fast_adopt(tslot, k);
      }
      uint32_t* out = th.tmx + (b & 1) * MAX_BATCH;
      // pairs of rows (two independent chains a pass): pair q to helper q % H, wave (q / H) % NW
      for (int q = h + th.H * wave; 2 * q < B; q += th.H * NW) {
        const int j = 2 * q, j1 = j + 1;
        const bool has1 = j1 < B;
        const DevPod p = L.pod[j];
        const double ed[2] = {L.pd[j][0], L.pd[j][1]}, rd[2] = {L.pd[j][2], L.pd[j][3]};
        uint32_t tk = tv ? make_key(fast_total<EXT>(tslot, p, ed, rd, k), tnode) : 0u, tk1 = 0u;
        if (has1) {
          const DevPod p1 = L.pod[j1];
          const double ed1[2] = {L.pd[j1][0], L.pd[j1][1]}, rd1[2] = {L.pd[j1][2], L.pd[j1][3]};
          tk1 = tv ? make_key(fast_total<EXT>(tslot, p1, ed1, rd1, k), tnode) : 0u;
        }
        tk = wave_max_u32(tk);
        tk1 = wave_max_u32(tk1);
        if (lane == 0) {
          st_sc1(out + j, tk);
          if (has1) st_sc1(out + j1, tk1);
        }
      }
      drain_stores();
    }
    __syncthreads();  // (every wave's maxima drained; s_go and the pods are rewritten next batch)
    if (go > 0 && threadIdx.x == 0) __hip_atomic_fetch_add(th.tready + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Persistent Reserve chain of a run of pipelined plain batches [b0, b0 + nb): one
// workgroup for the whole run, so no kernel boundary or cross-stream event sits between two batches.
// Per batch: wait until its lists are published (ready[b] == pods of b), resolve it, then publish
// done[b] (rows, placements, the changed-row list).  Every wait is bounded (wait_at_least); on a
// timeout the run stops and the error word tells the host.
//   stale == nullptr (quota runs): k_fixup made the lists exact (cand, stride KMAX).
//   else: the stale top-(k_j + KMAX) lists of the double buffer `stale` (stride KSTALE) go straight to the
//   speculative replay, with the previous batch's changed rows (touched_out, this workgroup wrote them) as
//   its T slots -- no fixup kernel and no hand-off back to the eval stream on the critical path.
template <bool QUOTA, bool EXT>
__global__ __launch_bounds__(res_threads<false>()) void k_resolve_run(SoA s, const DevPod* __restrict__ pods,
                                                                      const int32_t* __restrict__ bases, int b0, int nb,
                                                                      KArgs k, const uint32_t* __restrict__ cand,
                                                                      const int32_t* __restrict__ cand_cnt,
                                                                      int32_t* __restrict__ chosen,
                                                                      int32_t* __restrict__ chosen_score, int32_t global_offset,
                                                                      uint64_t* __restrict__ stamps,
                                                                      uint64_t* __restrict__ pstamps,
                                                                      uint64_t* __restrict__ dev_alloc,
                                                                      const int32_t* __restrict__ ready,
                                                                      int32_t* __restrict__ done, int32_t* __restrict__ err,
                                                                      int64_t* __restrict__ touched_out,
                                                                      int32_t* __restrict__ touched_cnt,
                                                                      uint32_t* __restrict__ chg_glb, int n_nodes,
                                                                      const uint32_t* __restrict__ stale,
                                                                      const int32_t* __restrict__ stale_cnt, int sorted,
                                                                      THelp th) {
  __shared__ ResLds L;
  __shared__ int32_t s_ok;
  const bool nofix = !QUOTA && stale != nullptr;
  if (blockIdx.x == 0 && threadIdx.x == 0 && th.resident) st_sc1(th.resident, 1);
  if (blockIdx.x > 0) {  // a T-row helper
    if (nofix) t_helper<EXT>(L, s, pods, bases, b0, nb, k, done, err, th, (int)blockIdx.x - 1, &s_ok);
    return;
  }
  if (!nofix) th.H = 0, th.tlist = nullptr;
  const ChgSet C = chg_init(L, chg_glb, n_nodes);
  for (int b = b0; b < b0 + nb; b++) {
    const int base = bases[b], B = bases[b + 1] - bases[b];
    if (!nofix || b == b0) {  // (a stale-list batch after the first: polled while its predecessor wrote back)
      if (threadIdx.x == 0) s_ok = wait_at_least(ready + b, B, err);
      __syncthreads();
      if (!s_ok) return;
    }
    const int par = b & 1;
    const bool has_t = nofix && b > b0;       // the previous batch's changed nodes (L.trec)
    const bool keep = nofix && b + 1 < b0 + nb;  // this batch's are the next one's T
    resolve_batch<false, false, QUOTA, EXT>(L, C, s, pods, base, B, k, nofix ? stale + (int64_t)par * MAX_BATCH * KSTALE : cand,
                                       nofix ? stale_cnt + par * MAX_BATCH : cand_cnt, chosen, chosen_score, global_offset,
                                       stamps, pstamps, b, dev_alloc, nullptr, touched_out, touched_cnt, has_t, keep,
                                       nofix ? KSTALE : KMAX, !nofix || sorted != 0,  // (k_fixup's lists: by rank)
                                       has_t ? done + (b - 1) : nullptr, th);
    // the next stale-list batch's lists: wave 1 waits for them while wave 0 writes this batch back (every load
    // of them comes after the barrier below, so after the flag was seen)
    if (keep && threadIdx.x == 64) s_ok = wait_at_least(ready + b + 1, bases[b + 2] - bases[b + 1], err);
    __syncthreads();
    if (keep && !s_ok) return;
    // wave 0 drained its stores (replay_batch / a batch without a successor), so they are performed; a stale-list
    // batch with a successor is published by that successor's prologue
    if (threadIdx.x == 0 && !keep) st_sc1(done + b, 1);
  }
}

// --- cpuset pods: Reserve with the CPU accumulator --------------------------------------------
// LoadAware assign + NodeInfo.Requested on the SoA row of the chosen node (k_resolve's patch)
__device__ void reserve_row(const SoA& s, int64_t node, uint32_t nf, const DevPod& pod) {
  const int64_t st = s.stride;
  int64_t* f = s.f + node;
  if ((nf & NF_HAS_METRIC) && !(nf & NF_NM_NIL)) {
    for (int q = 0; q < 2; q++) {
      if (nf & nf_fh_on(0, q)) f[(F_FH + q) * st] -= pod.est[q];
      f[(F_SA + q) * st] -= pod.est[q];
      if (pod.flags & PF_PROD) {
        if (nf & nf_fh_on(1, q)) f[(F_FH + 2 + q) * st] -= pod.est[q];
        f[(F_SA + 2 + q) * st] -= pod.est[q];
      }
    }
  }
  f[F_NREQ * st] += pod.req[0];
  f[(F_NREQ + 1) * st] += pod.req[1];
}

// One takePreferredCPUs call (no preferred CPUs = takeCPUs, cpu_accumulator.go:29-85) over the CPUs of
// `a.base` in NUMA id `zone` (-1 = all) not yet in `a.uni`, from the pre-pod exclusivity; adds the
// result to a.uni.  needed <= 0 takes nothing.  All lanes (ke_cpuacc.h).
__device__ bool cpuset_take1(AccLds& a, int zone, int needed, int bind, int pref_sel) {
  if (needed <= 0) return true;
  const int L = threadIdx.x;
  for (int c = L; c < a.n_cpu; c += 64) {
    // pref_sel: 0 every available CPU, 1 the preferred ones, 2 the others (availableCPUs.Difference(preferred))
    const bool sel = pref_sel == 0 || (pref_sel == 1) == (a.pref[c] != 0);
    a.alloc[c] = a.base[c] && !a.uni[c] && (zone < 0 || a.cpu[c].numa == zone) && sel;
    a.res[c] = 0;
  }
  for (int k = L; k < a.n_core; k += 64) a.ex_core[k] = a.ex_core0[k];
  for (int z = L; z < a.n_numa; z += 64) a.ex_node[z] = a.ex_node0[z];
  if (L == 0) a.needed = needed;
  __syncthreads();
  if (!acc_take_cpus(a, bind)) return false;
  for (int c = L; c < a.n_cpu; c += 64) a.uni[c] |= a.res[c];
  __syncthreads();
  return true;
}
__device__ bool cpuset_take(AccLds& a, int zone, int needed, int bind) {
  if (!a.has_pref) return cpuset_take1(a, zone, needed, bind, 0);
  // takePreferredCPUs: min(needed, |available ∩ preferred|) from the preferred ones, the rest from the others
  int np = 0, before = 0;
  for (int c = threadIdx.x; c < a.n_cpu; c += 64) {
    np += a.base[c] && !a.uni[c] && (zone < 0 || a.cpu[c].numa == zone) && a.pref[c];
    before += a.uni[c];
  }
  np = acc_wave_sum(np);
  before = acc_wave_sum(before);
  if (np > 0) {
    if (!cpuset_take1(a, zone, min(needed, np), bind, 1)) return false;
    int got = 0;
    for (int c = threadIdx.x; c < a.n_cpu; c += 64) got += a.uni[c];
    needed -= acc_wave_sum(got) - before;
  }
  return cpuset_take1(a, zone, needed, bind, np > 0 ? 2 : 0);
}

// allocateCPUSet (resource_manager.go:353-459) over the node's CPU table in LDS: getAvailableCPUs, the
// required-policy filter (filterCPUsByRequiredCPUBindPolicy :655-695); with a NUMA allocation (zones
// `zmask`, cpu milli `zcpu[id]`) one take per zone in id order of min(cpu/1000, its CPUs) CPUs, which
// must add up to numCPUsNeeded; else one take over the node; then satisfiedRequiredCPUBindPolicy
// (:697-718).  All lanes of the workgroup, same arguments; a.res = the cpuset.
__device__ bool cpuset_allocate(const SoA& s, int64_t node, uint32_t nf, const DevPod& pod, AccLds& a, uint32_t zmask,
                                const int64_t* zcpu) {
  const int L = threadIdx.x;
  const int64_t st = s.stride;
  const int64_t cnt = s.cs[CS_CNT * st + node], topo = s.cs[CS_TOPO * st + node];
  const int max_ref = cs_max_ref(cnt), cpc = cs_cpc(cnt);
  // getCPUBindPolicy (util.go:101-119)
  const int preq = pf_cpu_required(pod.flags), nb = nf_cpu_bind(nf);
  bool required = true;
  int bind = preq;
  if (preq == XB_NONE) {
    if (nb == KE_NODE_CPU_BIND_SPREAD_BY_PCPUS) bind = XB_SPREAD;
    else if (nb == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY) bind = XB_FULL;
    else required = false, bind = pf_cpu_preferred(pod.flags);
  }
  if (L == 0) {
    a.t.num_cpus = (int)(topo & 0xffff);
    a.t.num_cores = (int)((topo >> 16) & 0xffff);
    a.t.num_nodes = (int)((topo >> 32) & 0xffff);
    a.t.num_sockets = (int)((topo >> 48) & 0xffff);
    a.n_core = a.t.num_cores;  // dense ranks
    a.n_sock = a.t.num_sockets;
    a.max_ref = max_ref;
    a.excl_policy = (pod.flags & PF_CPU_RCB) ? pf_cpu_excl(pod.flags) : KE_CPU_EXCL_NONE;
    a.exclusive = a.excl_policy == KE_CPU_EXCL_PCPU_LEVEL || a.excl_policy == KE_CPU_EXCL_NUMA_NODE_LEVEL;
    a.numa_most = (nf & NF_CPU_NUMA_MOST) ? 1 : 0;
  }
  __syncthreads();
  int32_t* navail_core = a.core_n;  // LDS scratch until the accumulator runs
  for (int k = L; k < a.n_core; k += 64) navail_core[k] = 0, a.ex_core0[k] = 0;
  for (int z = L; z < a.n_numa; z += 64) a.ex_node0[z] = 0;
  for (int c = L; c < a.n_cpu; c += 64) a.uni[c] = 0;
  __syncthreads();
  for (int c = L; c < a.n_cpu; c += 64) {  // a.cpu: the node's records (k_cpuset_reserve loaded them)
    const CpuRec r = a.cpu[c];
    a.base[c] = cpu_available(r, max_ref) ? 1 : 0;
    a.aref[c] = r.ref;
    if (a.base[c]) atomicAdd(&navail_core[r.core], 1);
    if ((r.flags & CR_VALID) && r.ref > 0) {  // exclusiveInCores / exclusiveInNUMANodes of the allocated CPUs
      if (r.excl == KE_CPU_EXCL_PCPU_LEVEL) a.ex_core0[r.core] = 1;
      else if (r.excl == KE_CPU_EXCL_NUMA_NODE_LEVEL) a.ex_node0[r.numa] = 1;
    }
  }
  __syncthreads();
  if (required) {  // FullPCPUs: CPUs of fully available cores; SpreadByPCPUs: each core's lowest CPU
    if (L == 0) {
      for (int k = 0; k < a.n_core; k++) a.mark[k] = 0;
      for (int c = 0; c < a.n_cpu; c++) {
        if (!a.base[c]) continue;
        const int k = a.cpu[c].core;
        const bool lowest = !a.mark[k];
        a.mark[k] = 1;
        if ((bind == XB_FULL && navail_core[k] != cpc) || (bind == XB_SPREAD && !lowest)) a.base[c] = 0;
      }
    }
    __syncthreads();
  }
  int navail = 0;
  for (int c = L; c < a.n_cpu; c += 64) navail += a.base[c];
  navail = acc_wave_sum(navail);
  const int ncpu = (int)(pod.req[0] / 1000);
  if (navail < ncpu) return false;
  int needed = ncpu;
  if (zmask) {
    for (int z = 0; z < 8; z++) {
      if (!((zmask >> z) & 1u)) continue;
      int inzone = 0;
      for (int c = L; c < a.n_cpu; c += 64) inzone += a.base[c] && a.cpu[c].numa == z;
      inzone = acc_wave_sum(inzone);
      if (!cpuset_take(a, z, min((int)(zcpu[z] / 1000), inzone), bind)) return false;
    }
    int got = 0;
    for (int c = L; c < a.n_cpu; c += 64) got += a.uni[c];
    needed -= acc_wave_sum(got);
    if (needed != 0) return false;
  }
  if (needed > 0 && !cpuset_take(a, -1, needed, bind)) return false;
  for (int c = L; c < a.n_cpu; c += 64) a.res[c] = a.uni[c];
  __syncthreads();
  if (required) {
    if (L == 0) {
      for (int k = 0; k < a.n_core; k++) a.mark[k] = 0;
      int n = 0, ncore = 0;
      for (int c = 0; c < a.n_cpu; c++) {
        if (!a.res[c]) continue;
        n++;
        const int k = a.cpu[c].core;
        if (!a.mark[k]) ncore++;
        a.mark[k] = 1;
      }
      a.bcast = !((bind == XB_FULL && ncore * cpc != n) || (bind == XB_SPREAD && ncore != n));
    }
    __syncthreads();
    if (!a.bcast) return false;
  }
  return true;
}

// k_cpuset_reserve's hand-off from thread 0 to the wave, and the wave's sums
struct CsrShared {
  int64_t node;
  int64_t zcpu[8];  // the NUMA allocation's cpu per id (cpuset_allocate's zones)
  uint32_t nf, zmask;
  int take, cs_pass, commit, excl, cpc, max_ref, numa_ovr;
  int cs_old[8], cs_add[8];  // allocated CPUs per NUMA id before the pod; newly allocated ones
  uint32_t used[8];          // NUMA ids (0..255) of the cpuset
  int zc[24];                // cs_fill's per-NUMA-id counts: available, in full cores, cores' lowest
  int allocated, all;
  unsigned long long set[4];
  int core_cnt[CPU_SLOTS], core_min[CPU_SLOTS];
};

// resourceManager.Update -> addPodAllocation (node_allocation.go:111-156): RefCount++ and the pod's
// exclusive policy on the new cpuset, the allocated-CPU count of the amplified cpu (row F_CS*) and the
// availability counts (cs_fill's words, one CPU per lane step).  The zones' NUMA status is left to the
// host mirror (re-derived rows).  Every lane of the wave; a.res = the cpuset.
__device__ void cpuset_commit_wave(const SoA& s, AccLds& a, CsrShared& sh, int lane) {
  const int64_t st = s.stride, node = sh.node;
  CpuRec* recs = s.cpu + node * CPU_SLOTS;
  int allocated = 0, all = 0;
  for (int c = lane; c < CPU_SLOTS; c += 64) {
    if (a.res[c]) {
      atomicOr(&sh.set[c >> 6], 1ull << (c & 63));
      CpuRec r = a.cpu[c];
      r.ref++;
      r.excl = (uint8_t)sh.excl;
      a.cpu[c] = r;
      recs[c] = r;
      atomicOr(&sh.used[r.numa >> 5], 1u << (r.numa & 31));
      if (r.numa < 8 && r.ref == 1) atomicAdd(&sh.cs_add[r.numa], 1);  // a CPU newly allocated
    }
    allocated += (a.cpu[c].flags & CR_VALID) && a.cpu[c].ref > 0;
    sh.core_cnt[c] = 0;
    sh.core_min[c] = CPU_SLOTS;
  }
  allocated = wave_sum(allocated);
  __syncthreads();
  for (int c = lane; c < CPU_SLOTS; c += 64)  // available CPUs per core, its lowest available id
    if (cpu_available(a.cpu[c], sh.max_ref)) {
      atomicAdd(&sh.core_cnt[a.cpu[c].core], 1);
      atomicMin(&sh.core_min[a.cpu[c].core], c);
      all++;
    }
  all = wave_sum(all);
  __syncthreads();
  const int cpc = sh.cpc;
  int full = 0, spread = 0;
  for (int kk = lane; kk < CPU_SLOTS; kk += 64) {
    if (sh.core_cnt[kk] == cpc && cpc > 0) full += cpc;
    if (sh.core_cnt[kk] > 0) spread++;
  }
  full = wave_sum(full);
  spread = wave_sum(spread);
  for (int c = lane; c < CPU_SLOTS; c += 64) {
    const CpuRec r = a.cpu[c];
    if (!cpu_available(r, sh.max_ref) || r.numa >= 8) continue;
    atomicAdd(&sh.zc[r.numa], 1);                                     // available
    if (sh.core_cnt[r.core] == cpc) atomicAdd(&sh.zc[8 + r.numa], 1);  // in a fully available core
    if (sh.core_min[r.core] == c) atomicAdd(&sh.zc[16 + r.numa], 1);  // the core's lowest available CPU
  }
  __syncthreads();
  if (lane == 0) {
    int64_t* f = s.f + node;
    const int64_t cs_milli = (int64_t)allocated * 1000;
    f[F_CSM * st] = cs_milli;
    f[F_CSAF * st] = amplify_bits(cs_milli, s.cs[CS_RF * st + node]);
    f[F_CSAS * st] = amplify_bits(cs_milli, s.cs[CS_RS * st + node]);
    s.cs[CS_CNT * st + node] = cs_pack(full, spread, cpc, sh.max_ref, all);
    for (int w = 0; w < 6; w++) {  // CS_Z* words: 16-bit counts of NUMA ids 4 (w & 1) .. 4 (w & 1) + 3
      int64_t word = 0;
      for (int q = 0; q < 4; q++) word |= (int64_t)sh.zc[8 * (w >> 1) + 4 * (w & 1) + q] << (16 * q);
      s.cs[(CS_ZALL + w) * st + node] = word;
    }
  }
}

// The allocate-from-reservation trials of one KE_RSV_MATCHED pod (pods[0]) on the nodes of its matched reservations
// that hold a cpuset / NUMA resources (nodenumaresource/reservation.go:270-424; the node has no NUMA policy, so
// Allocate is allocateCPUSet alone): one workgroup per view, allocateCPUSet over the node's CPU table with
// RefCount-- on the view's preferredCPUs (getAvailableCPUs(preferred), node_allocation.go:192-219) and
// takePreferredCPUs; a Restricted reservation's view then needs numCPUsNeeded <= |remainedCPUs| and a second
// allocation preferring only them, whose cpuset may not outgrow them.
// zmask != 0 or score_on (a pod binding CPUs under a NUMA policy, after k_numa_views and the nomination): one
// allocation with `pref` over the zones of the trial's NUMA allocation, and with score_on the NodeNUMAResource Score of
// it -- requested cpu = Amplify(the CPUs still referenced once `pref2`, the options' preferredCPUs, gives back those
// not in the cpuset, x 1000) (scoring.go:101-119, 179-185).
__global__ __launch_bounds__(64) void k_rsv_views(SoA s, const DevPod* __restrict__ pods, const RsvView* __restrict__ views,
                                                  RsvViewOut* __restrict__ out, KArgs k) {
  __shared__ AccLds a;
  __shared__ int s_ok;
  const RsvView v = views[blockIdx.x];
  const DevPod pod = pods[0];
  const int L = threadIdx.x;
  const uint32_t nf = s.flags[v.node];
  const int64_t ncpu = pod.req[0] / 1000;
  bool ok = s.cpu != nullptr && (nf & NF_CPUS_VALID);
  for (int pass = 0; pass < (v.restricted ? 2 : 1) && ok; pass++) {
    const uint64_t* pw = pass ? v.pref2 : v.pref;
    if (pass) {  // Restricted: numCPUsNeeded > reservedCPUs.Size() fails the reservation
      int nrem = 0;
      for (int w = 0; w < 4; w++) nrem += __popcll(v.pref2[w]);
      if (ncpu > nrem) {
        ok = false;
        break;
      }
    }
    const CpuRec* recs = s.cpu + (int64_t)v.node * CPU_SLOTS;
    int top_cpu = 0, top_numa = 0;
    for (int c = L; c < CPU_SLOTS; c += 64) {
      CpuRec r = recs[c];
      const bool p = (pw[c >> 6] >> (c & 63)) & 1;
      if (p && r.ref > 0 && --r.ref == 0) r.excl = KE_CPU_EXCL_NONE;  // the CPU leaves allocateInfo at 0
      a.cpu[c] = r;
      a.alloc[c] = a.res[c] = a.base[c] = a.uni[c] = a.mark[c] = 0;
      a.pref[c] = p;
      if (r.flags & CR_VALID) top_cpu = c + 1, top_numa = max(top_numa, (int)r.numa + 1);
    }
    top_cpu = (int)wave_max_u32((uint32_t)top_cpu);
    top_numa = (int)wave_max_u32((uint32_t)top_numa);
    if (L == 0) a.n_cpu = top_cpu, a.n_numa = top_numa, a.has_pref = 1;
    __syncthreads();
    const bool took = cpuset_allocate(s, v.node, nf, pod, a, (uint32_t)v.zmask, v.zcpu);
    if (L == 0) s_ok = took;
    __syncthreads();
    ok = s_ok != 0;
    if (ok && pass) {  // result.CPUSet.Size() > reservedCPUs.Size()
      int n = 0, nrem = 0;
      for (int c = L; c < a.n_cpu; c += 64) n += a.res[c];
      n = acc_wave_sum(n);
      for (int w = 0; w < 4; w++) nrem += __popcll(v.pref2[w]);
      ok = n <= nrem;
    }
  }
  uint64_t w4[4] = {0, 0, 0, 0};
  if (ok)
    for (int c = 0; c < CPU_SLOTS; c++)
      if (a.res[c]) w4[c >> 6] |= 1ull << (c & 63);
  int32_t score = 0;
  if (ok && v.score_on) {
    const CpuRec* recs = s.cpu + (int64_t)v.node * CPU_SLOTS;
    int held = 0;
    for (int c = L; c < CPU_SLOTS; c += 64) {
      const CpuRec r = recs[c];
      int ref = (r.flags & CR_VALID) ? r.ref : 0;
      if (ref > 0 && ((v.pref2[c >> 6] >> (c & 63)) & 1) && !((w4[c >> 6] >> (c & 63)) & 1)) ref--;
      held += ref > 0;
    }
    held = acc_wave_sum(held);
    const int64_t rs = s.cs[CS_RS * s.stride + v.node];
    DevPod ps = pod;
    ps.req[0] = amplify_bits(pod.req[0], rs);
    const int64_t req[2] = {amplify_bits((int64_t)held * 1000, rs), v.sreq1}, alloc[2] = {v.salloc[0], v.salloc[1]};
    score = numa_scope_score((k.flags & AF_NUMA_MOST) != 0, req, alloc, ps, k);
  }
  if (L == 0) {
    out[blockIdx.x].ok = ok ? 1 : 0;
    out[blockIdx.x].score = score;
    for (int w = 0; w < 4; w++) out[blockIdx.x].cpus[w] = w4[w];
  }
}

// The DeviceShare allocate-from-reservation views of one reservation-matched / -ignored pod (pods[0]) on the nodes of
// its device-holding reservations (deviceshare/reservation.go:207-366): one view per workgroup, its
// lane 0 runs AutopilotAllocator over the node's row with the view's preemptible / requiredDeviceResources /
// required and preferred minors (ds_type_view with rv) -- Prepare, the Filter's allocation without a scorer (the
// first failing type's status in the order GPU, RDMA, FPGA), score (Σ scoreNode over the types the view keeps) and
// the Reserve-phase allocation with the plugin's scorer (the minors; 0 when it fails).  Reads the SoA only.
__global__ __launch_bounds__(64) void k_ds_views(SoA s, const DevPod* __restrict__ pods, const DsView* __restrict__ views,
                                                 DsViewOut* __restrict__ out, KArgs k) {
  if (threadIdx.x != 0) return;
  const DsView* v = views + blockIdx.x;
  const DevPod p = pods[0];
  const int64_t i = v->node;
  uint64_t msk[4];
#pragma unroll
  for (int w = 0; w < 4; w++) msk[w] = dsmask(s, w, i);
  for (int t = 0; t < 3; t++)  // the view's preemptible keys are used keys of their instances (calcFreeWithPreemptible)
    for (int m = 0; m < DS_MINORS; m++) {
      const int bit = 16 * t + m;
      if (!((v->pre_in >> bit) & 1)) continue;
      for (int q = 0; q < DS_NK[t]; q++)
        if ((v->pre_keys[q] >> bit) & 1) msk[ds_hu_word(t)] |= 1ull << ds_hu_bit(t, m, q);
    }
  DsViewOut o;
  o.st = KE_CODE_SUCCESS;
  o.reason = KE_REASON_NONE;
  o.raw = 0;
  o.minors = 0;
  for (int t = 0; t < 3; t++)  // Prepare: a requested type without devices
    if (p.ds_cnt[t] && !((msk[DSM_EXISTS] >> (16 * t)) & 0xFFFF)) {
      o.st = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      o.reason = KE_REASON_DS_INSUFFICIENT_GPU + t;
      out[blockIdx.x] = o;
      return;
    }
  int64_t raw = 0;
  for (int t = 0; t < 3; t++) {
    if (!p.ds_cnt[t]) continue;
    GpuMasks g;
    int64_t tot[3], fre[3];
    const bool present = ds_type_view(s, i, t, msk, p, k, DsAff{false, 0u}, g, tot, fre, nullptr, 0xFFFFu, v);
    if (o.st == KE_CODE_SUCCESS) {
      int why = KE_REASON_DS_INSUFFICIENT_GPU + t;
      int st = 0;
      if (t == KE_DEV_GPU) {
        uint32_t unused;
        st = gpu_allocate(s, i, msk[DSM_EXISTS], p, g, false, nullptr, &unused, &why);
      } else if (__builtin_popcount(g.dflt) < p.ds_cnt[t]) {
        st = KE_CODE_UNSCHEDULABLE;
      }
      if (st) o.st = st, o.reason = why;
    }
    if (present) raw += ds_weighted(k, t, tot, fre, p);  // resourceAllocationScorer.scoreNode
  }
  o.raw = raw;
  if (o.st == KE_CODE_SUCCESS) {
    uint64_t minors = 0;
    bool ok = true;
    for (int t = 0; t < 3 && ok; t++) {
      if (!p.ds_cnt[t]) continue;
      int64_t score[DS_MINORS];
      GpuMasks g;
      int64_t tot[3], fre[3];
      ds_type_view(s, i, t, msk, p, k, DsAff{false, 0u}, g, tot, fre, score, 0xFFFFu, v);
      uint32_t take = 0;
      if (t == KE_DEV_GPU) {
        int why = 0;
        ok = gpu_allocate(s, i, msk[DSM_EXISTS], p, g, true, score, &take, &why) == 0 && take != 0;
      } else {
        take = default_pick(g.dflt, p.ds_cnt[t], score, g.pref);
        ok = __builtin_popcount(take) >= p.ds_cnt[t];
      }
      minors |= (uint64_t)take << (16 * t);
    }
    o.minors = ok ? minors : 0;
  }
  out[blockIdx.x] = o;
}

// ---- NodeNUMAResource allocate-from-reservation under a NUMA policy (k_numa_views) ------------------------------
// A view of node i's zones with `e` (keys ek: bit 2*id + r) added to the reusable resources of the NUMA ids with an
// allocation entry (getAvailableNUMANodeResources, node_allocation.go:221-243): SubtractWithNonNegativeResult of the
// row's allocated (its unmatched restore already subtracted) -- the allocated amounts al[r][id] and totalAvailable.
__device__ __noinline__ void numa_view_reuse(const SoA& s, int64_t i, const NumaNode& base, uint32_t entry,
                                             const int64_t* e, uint32_t ek, NumaNode& o, int64_t (&al)[2][8]) {
  o = base;
  for (int z = 0; z < 8; z++)
    for (int r = 0; r < 2; r++) {
      int64_t a = numa_al(s, i, base, z, r);
      if (((entry >> z) & 1u) && ((ek >> (2 * z + r)) & 1u)) {
        a -= e[2 * z + r];
        a = a > 0 ? a : 0;
        o.ak[r] |= 1u << z;
      }
      al[r][z] = ((o.ak[r] >> z) & 1u) ? a : 0;
      const int64_t q = numa_cap(s, i, z, r) - al[r][z];
      o.av[r][z] = q > 0 ? q : 0;
    }
  numa_perm(o, 0);
  numa_perm(o, 1);
}
// totalAvailable = requiredResources (allocateResourcesByHint, resource_manager.go:226-254): its NUMA ids and keys,
// signed (quotav1.Subtract); resourceNamesByNUMA = its keys
__device__ __noinline__ void numa_view_req(const NumaNode& base, const int64_t* req, uint32_t rk, NumaNode& o) {
  o = base;
  o.ch[0] = o.ch[1] = o.ak[0] = o.ak[1] = 0;
  for (int z = 0; z < 8; z++)
    for (int r = 0; r < 2; r++) {
      const bool key = (rk >> (2 * z + r)) & 1u;
      if (key) o.ch[r] |= 1u << z;
      o.av[r][z] = key ? req[2 * z + r] : 0;
    }
  numa_perm(o, 0);
  numa_perm(o, 1);
}

// One workgroup per view set (a node of the matched pod's reservations holding NUMA resources / CPUs, a NUMA policy
// merged): the views in LDS; every lane takes masks of IterateBitMasks' order and asks the Allocate of
// generateResourceHints (resource_manager.go:586-594): tryAllocateFromReservation over the trials (the first satisfied
// one), else -- without a reservation affinity -- tryAllocateFromNode; lane 0 merges the hint lists as numa_admit does
// (preferred scan, BestEffort's full fold) and runs Plugin.Allocate on the affinity (topology_hint.go:78-118); lanes
// q <= n then record each trial's (and the node's own) allocation on it and the Score calculateAllocatableAndRequested
// gives with its options (scoring.go:101-119, 141-186).  A pod binding CPUs (round 6): every view has its own
// availability counts (cs_fill with the view's preferredCPUs), trims its zones under a required bind policy and
// checks allocateCPUSet's take by counts as numa_fits<CS>; its Score's cpu needs the cpuset, which the
// cpuset pass (k_rsv_views with zones) adds to sreq1 / salloc.  Reads the SoA only.
__global__ __launch_bounds__(64) void k_numa_views(SoA s, const DevPod* __restrict__ pods,
                                                   const NumaRsvView* __restrict__ views, NumaRsvOut* __restrict__ out,
                                                   KArgs k) {
  const NumaRsvView& w = views[blockIdx.x];
  const DevPod p = pods[0];
  const int64_t i = w.node;
  const int n = min(w.n, NV_MAX);
  const int lane = (int)threadIdx.x;
  constexpr int NVW = 2 + 2 * NV_MAX;  // 0 hint, 1 node, 2 + q trial q, 2 + NV_MAX + q its requiredResources
  static_assert(NVW <= 64, "k_numa_views: one lane per view");
  __shared__ NumaNode s_v[NVW];
  __shared__ NumaCs s_cs[NVW];
  __shared__ uint8_t s_scr[NVW][CPU_SLOTS];
  __shared__ int64_t s_al[NV_MAX + 1][2][8];  // the allocated amounts of trial q / the node (NV_MAX)
  __shared__ unsigned long long s_L[2][4];
  __shared__ uint32_t s_aff;
  __shared__ int32_t s_st, s_reason;
  NodeRegs nr;
  load_row(s, i, nr);
  const uint32_t nf = nr.flags;
  // requestCPUBind (util.go:121-138), as eval_pair; a binding pod's hint scores see its amplified cpu request
  const bool rcb = s.cpu != nullptr && (nf & NF_CPUS_VALID) && !(p.flags & PF_NUMA_SKIP) &&
                   ((p.flags & PF_CPU_RCB) || (p.req[0] != 0 && nf_cpu_bind(nf) != KE_NODE_CPU_BIND_NONE &&
                                               (p.flags & PF_CPU_INT)));
  DevPod ps = p;
  if (rcb) ps.req[0] = amplify_bits(p.req[0], s.cs[CS_RS * s.stride + i]);
  if (lane < NVW) {
    NumaCs cs;
    cs.rcb = false;
    const bool used = lane < 2 || (lane < 2 + n) || (lane >= 2 + NV_MAX && lane < 2 + NV_MAX + n);
    if (rcb && used) {
      if (lane == 1) {
        cs = numa_cs_load(s, i, nf, p);
      } else {
        const uint64_t* pr = lane == 0 ? w.pref[NV_MAX] : lane < 2 + NV_MAX ? w.pref[lane - 2] : w.rpref[lane - 2 - NV_MAX];
        const int64_t c0 = s.cs[CS_CNT * s.stride + i];
        int64_t cnt, z6[6];
        cs_fill(s.cpu + i * CPU_SLOTS, cs_cpc(c0), cs_max_ref(c0), s_scr[lane], &cnt, z6, pr);
        cs = numa_cs_words(cnt, z6, nf, p);
      }
    }
    s_cs[lane] = cs;
    NumaNode base;
    numa_load(s, i, base);
    NumaNode o;
    int64_t al[2][8];
    if (lane == 0) {
      numa_view_reuse(s, i, base, w.entry, w.hint, w.hint_keys, o, al);
      if (cs.rcb) numa_trim(o, cs);
      s_v[0] = o;
    } else if (lane == 1) {
      o = base;
      if (cs.rcb) numa_trim(o, cs);
      s_v[1] = o;
      for (int r = 0; r < 2; r++)
        for (int z = 0; z < 8; z++) s_al[NV_MAX][r][z] = numa_al(s, i, base, z, r);
    } else if (lane < 2 + n) {
      const int q = lane - 2;
      numa_view_reuse(s, i, base, w.entry, w.reuse[q], w.keys[q], o, al);
      if (cs.rcb) numa_trim(o, cs);
      s_v[lane] = o;
      for (int r = 0; r < 2; r++)
        for (int z = 0; z < 8; z++) s_al[q][r][z] = al[r][z];
    } else if (lane >= 2 + NV_MAX && lane < 2 + NV_MAX + n) {
      // the Restricted trial's second Allocate: requiredResources when the reserve pod holds NUMA amounts, else the
      // trial's own reusable view; trimmed by the remainedCPUs' availability
      const int q = lane - 2 - NV_MAX;
      if (w.has_req[q]) numa_view_req(base, w.req[q], w.req_keys[q], o);
      else numa_view_reuse(s, i, base, w.entry, w.reuse[q], w.keys[q], o, al);
      if (cs.rcb) numa_trim(o, cs);
      s_v[lane] = o;
    }
  }
  if (lane < 8) reinterpret_cast<unsigned long long*>(s_L)[lane] = 0ull;
  __syncthreads();
  auto fits = [&](int v, uint32_t m) -> bool {  // Allocate on view v with the hint m (a binding pod: counts, §4e)
    if (!rcb) return numa_fits(s_v[v], m, p);
    return m ? numa_fits<true>(s_v[v], m, p, &s_cs[v]) : s_cs[v].total >= s_cs[v].num;
  };
  // tryAllocateFromReservation's trial q with the hint m: Allocate on its view; a Restricted one's
  // numCPUsNeeded <= |remainedCPUs| (a binding pod) and second Allocate
  auto trial = [&](int q, uint32_t m) -> bool {
    if (!fits(2 + q, m)) return false;
    if (!w.restricted[q]) return true;
    if (rcb && s_cs[2 + NV_MAX + q].num > w.rem_cpus[q]) return false;
    return (!w.has_req[q] && !rcb) || fits(2 + NV_MAX + q, m);
  };
  auto allocate = [&](uint32_t m) -> bool {  // Plugin.Allocate / the hint pass's check on mask m (0: no hint)
    if (!m && !rcb) return true;
    for (int q = 0; q < n; q++)
      if (trial(q, m)) return true;
    return !w.required && fits(1, m);
  };
  const NumaNode& hv = s_v[0];
  const uint32_t all = hv.zm;
  bool present[2];
  uint32_t lack[2];
  numa_present_lack(hv, p, present, lack);
  for (int e = lane; e < 255; e += 64) {  // generateResourceHints: the feasible masks per resource
    const uint32_t m = NUMA_ORDER[e];
    if (m & ~all) continue;
    const bool in0 = present[0] && !(m & lack[0]), in1 = present[1] && !(m & lack[1]);
    if ((!in0 && !in1) || !allocate(m)) continue;
    const unsigned long long bit = 1ull << (m & 63u);
    if (in0) atomicOr(&s_L[0][m >> 6], bit);
    if (in1) atomicOr(&s_L[1][m >> 6], bit);
  }
  __syncthreads();
  if (lane == 0) {
    const int policy = pf_numa_policy(p.flags) ? pf_numa_policy(p.flags) : nf_numa_policy(nf);
    const bool excl = (p.flags & PF_NUMA_EXCL_REQ) != 0;
    const bool single = policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE, restricted = policy == KE_NUMA_POLICY_RESTRICTED;
    int st = KE_CODE_SUCCESS, reason = KE_REASON_NONE;
    uint32_t aff = 0;
    uint64_t L[2][4];
    for (int r = 0; r < 2; r++)
      for (int q = 0; q < 4; q++) L[r][q] = s_L[r][q];
    const int R = (int)present[0] + (int)present[1];
    if (all == 0) {  // topology_hint.go:31-41
      st = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, reason = KE_REASON_NUMA_MISSING_RESOURCES;
    } else if (nf & NF_NUMA_OPT_ERR) {
      st = KE_CODE_UNSCHEDULABLE, reason = KE_REASON_NUMA_HINT_UNALIGNED;
    } else if (R == 0) {  // one preferred any-NUMA hint per provider
      if (policy != KE_NUMA_POLICY_BEST_EFFORT && !exclusive_ok(hv, all, excl))
        st = KE_CODE_UNSCHEDULABLE, reason = KE_REASON_NUMA_HINT_UNALIGNED;
      else
        aff = single ? 0u : all;
    } else {
      int minr[2] = {9, 9};
      for (int e = 0; e < 255; e++) {
        const uint32_t m = NUMA_ORDER[e];
        for (int r = 0; r < 2; r++)
          if (present[r] && bit256(L[r], m)) minr[r] = min(minr[r], __popc(m));
      }
      const bool empty0 = present[0] && minr[0] == 9, empty1 = present[1] && minr[1] == 9;
      uint32_t best = all;
      int32_t bsc = 0;
      bool found = false;
      if (!empty0 && !empty1)
        for (int e = 0; e < 255; e++) {  // the preferred merged hints, IterateBitMasks order
          const uint32_t m = NUMA_ORDER[e];
          if ((m & ~all) || (single && __popc(m) != 1)) continue;
          bool cand = true;
          for (int r = 0; r < 2; r++)
            if (present[r]) cand = cand && bit256(L[r], m) && (restricted || (int)__popc(m) == minr[r]);
          if (!cand || !exclusive_ok(hv, m, excl)) continue;
          const int32_t sc = R * numa_hint_score(s, i, hv, m, ps, k);
          if (!found || narrower(m, best) || (__popc(m) == __popc(best) && sc > bsc)) best = m, bsc = sc, found = true;
        }
      if (found) {
        aff = (single && best == all) ? 0u : best;
      } else if (policy != KE_NUMA_POLICY_BEST_EFFORT) {
        st = KE_CODE_UNSCHEDULABLE, reason = KE_REASON_NUMA_HINT_UNALIGNED;
      } else {  // mergeFilteredHints over every permutation of the lists
        MergeLists ml;
        ml.n = 0;
        for (int r = 0; r < 2; r++) {
          if (!present[r]) continue;
          int c = 0;
          if (minr[r] == 9) {
            ml.m[ml.n][0] = 0, c = 1, ml.unsat[ml.n] = 1;
          } else {
            for (int e = 0; e < 255; e++)
              if (bit256(L[r], NUMA_ORDER[e])) ml.m[ml.n][c++] = NUMA_ORDER[e];
            ml.unsat[ml.n] = 0;
          }
          ml.len[ml.n] = c;
          ml.ds[ml.n] = 0;
          ml.n++;
        }
        DsHints dh;
        dh.status = 0;
        dh.none = true;
        dh.copies = 0;
        aff = merge_all_permutations(s, i, hv, ps, k, ml, dh, excl);
      }
    }
    if (st == KE_CODE_SUCCESS && !allocate(aff)) {
      st = KE_CODE_UNSCHEDULABLE;
      reason = w.required ? KE_REASON_RSV_INSUFFICIENT_NUMA : KE_REASON_NUMA_INSUFFICIENT_RESOURCES;
    }
    s_aff = aff;
    s_st = st;
    s_reason = reason;
  }
  __syncthreads();
  const uint32_t aff = s_aff;
  // per trial (lane q < n) and the node's own (lane NV_MAX): the allocation on the affinity and the Score with the
  // options it used -- NUMA-scope allocatable / requested of the zones it touches, else the node's
  bool ok = false;
  if (lane < n || lane == NV_MAX) {
    const int q = lane;
    int64_t d[2][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0}};
    uint32_t got[2] = {0, 0};
    const int vv = q < n ? ((w.restricted[q] && (w.has_req[q] || rcb)) ? 2 + NV_MAX + q : 2 + q) : 1;
    ok = (!aff && !rcb) || (q < n ? trial(q, aff) : fits(1, aff));
    if (ok && aff) {
      if (rcb) numa_distribute<true, true>(s_v[vv], aff, p, got, d, &s_cs[vv]);
      else numa_distribute<true>(s_v[vv], aff, p, got, d);
    }
    const uint32_t zs = got[0] | got[1];
    int64_t req[2] = {nr.nreq[0], nr.nreq[1]}, alloc[2] = {nr.nalloc[0], nr.nalloc[1]};
    if (zs) {
      req[0] = req[1] = alloc[0] = alloc[1] = 0;
      for (int z = 0; z < 8; z++)
        if ((zs >> z) & 1u)
          for (int r = 0; r < 2; r++) {
            alloc[r] += numa_cap(s, i, z, r);
            req[r] += s_al[q < n ? q : NV_MAX][r][z];
          }
    }
    const int oq = q < n ? q : NV_MAX;
    // a binding pod: requested cpu = Amplify(the node's allocated CPUs * 1000) (scoring.go:179-185) -- the node's own
    // here; a trial's gives its preferredCPUs back but for the pod's cpuset (the cpuset pass)
    if (rcb) req[0] = amplify_bits(nr.csm, s.cs[CS_RS * s.stride + i]);
    out[blockIdx.x].score[oq] = ok ? numa_scope_score((k.flags & AF_NUMA_MOST) != 0, req, alloc, rcb ? ps : p, k) : 0;
    out[blockIdx.x].sreq1[oq] = req[1];
    out[blockIdx.x].salloc[oq][0] = alloc[0];
    out[blockIdx.x].salloc[oq][1] = alloc[1];
    for (int z = 0; z < 8; z++)
      for (int r = 0; r < 2; r++) out[blockIdx.x].dist[oq][2 * z + r] = ok ? d[r][z] : 0;
  }
  const uint64_t okm = __ballot(ok);
  if (lane == 0) {
    out[blockIdx.x].st = s_st;
    out[blockIdx.x].reason = s_reason;
    out[blockIdx.x].aff = aff;
    out[blockIdx.x].ok = (uint32_t)(okm & ((1ull << n) - 1ull)) | (((okm >> NV_MAX) & 1ull) ? 1u << NV_MAX : 0u);
  }
}

// A singleton batch of a pod that may bind CPUs, after k_select: selectHost's node, then Reserve in
// profile order — LoadAware, NodeNUMAResource (the NUMA allocation on the affinity Admit picks and the
// cpuset; a failed Allocate fails Reserve and the pod stays unplaced), DeviceShare.  One thread: the
// accumulator is sequential (sorted lists, greedy takes).  NUMA: nodes may carry NUMA policies.
template <bool DS, bool NUMA>
__global__ __launch_bounds__(64) void k_cpuset_reserve(SoA s, const DevPod* __restrict__ pods, const int32_t* __restrict__ batch_base,
                                                       KArgs k, const uint32_t* __restrict__ cand,
                                                       const int32_t* __restrict__ cand_cnt, int32_t* __restrict__ chosen,
                                                       int32_t* __restrict__ chosen_score, int32_t global_offset,
                                                       uint64_t* __restrict__ stamps, uint64_t* __restrict__ pstamps,
                                                       int batch_index, uint64_t* __restrict__ dev_alloc,
                                                       int64_t* __restrict__ numa_alloc, uint64_t* __restrict__ cpusets,
                                                       const uint8_t* __restrict__ aff_in, int eval_lo, int eval_hi) {
  __shared__ AccLds a;
  __shared__ uint32_t s_w;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int base = *batch_base;
  {  // selectHost's key (wave max over the candidates), then the node's CPU records into LDS (all lanes)
    const int cnt = min(cand_cnt[0], KMAX);
    const uint32_t mine = (int)threadIdx.x < cnt ? cand[threadIdx.x] : 0u;
    const uint32_t wmax = wave_max_u32(mine);
    if (threadIdx.x == 0) s_w = wmax;
    __syncthreads();
    if (s_w && s.cpu) {
      // the records, the table's bounds (highest CPU id / NUMA id + 1) and the zeroed per-CPU byte
      // arrays the accumulator's loops stop short of
      const CpuRec* recs = s.cpu + (int64_t)key_node(s_w) * CPU_SLOTS;
      int top_cpu = 0, top_numa = 0;
      for (int c = threadIdx.x; c < CPU_SLOTS; c += 64) {
        const CpuRec r = recs[c];
        a.cpu[c] = r;
        a.alloc[c] = a.res[c] = a.base[c] = a.uni[c] = a.mark[c] = a.pref[c] = 0;
        if (r.flags & CR_VALID) top_cpu = c + 1, top_numa = max(top_numa, (int)r.numa + 1);
      }
      top_cpu = (int)wave_max_u32((uint32_t)top_cpu);
      top_numa = (int)wave_max_u32((uint32_t)top_numa);
      if (threadIdx.x == 0) a.n_cpu = top_cpu, a.n_numa = top_numa, a.has_pref = 0;
    }
    __syncthreads();
  }
  // Thread 0 selects, admits and runs the accumulator; the wave commits the cpuset and re-derives the
  // node's availability words (cs_fill) in parallel; thread 0 then patches the NUMA zones and devices.
  __shared__ CsrShared sh;
  const int lane = threadIdx.x;
  RPROF_DECL
  const DevPod pod = pods[base];
  int64_t qreq[2] = {0, 0};  // ElasticQuota PreFilter: a refused pod is placed nowhere
  const bool quota = (k.flags & AF_QUOTA) && pod.quota;
  uint32_t w = 0;
  int32_t out_node = -1, out_score = -1;
  uint64_t alloc = 0;
  int64_t* out16 = numa_alloc ? numa_alloc + (int64_t)base * 16 : nullptr;
  int64_t node = 0;
  uint32_t nf = 0;
  bool rcb = false, nsoa = false, ok = false, ds_here = false, stored = false;
  NumaNode v;
  v.zm = 0;
  uint32_t got[2] = {0, 0}, aff = 0;
  int64_t dist[2][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0}};
  if (lane == 0) {
    sh.cs_pass = 0;
    sh.commit = 0;
    sh.take = 0;
    sh.numa_ovr = 0;
    for (int q = 0; q < 4; q++) sh.set[q] = 0;
    for (int z = 0; z < 8; z++) sh.cs_old[z] = sh.cs_add[z] = sh.used[z] = 0;
    for (int z = 0; z < 24; z++) sh.zc[z] = 0;
    sh.allocated = sh.all = 0;
    w = (!quota || quota_admit_g(s, pod, k, qreq)) ? s_w : 0u;
    if (out16)
      for (int t = 0; t < 16; t++) out16[t] = 0;
  }
  if (lane == 0 && w) {
    node = key_node(w);
    nf = s.flags[node];
    rcb = !(pod.flags & PF_NUMA_SKIP) &&
          ((pod.flags & PF_CPU_RCB) || (pod.req[0] != 0 && nf_cpu_bind(nf) != KE_NODE_CPU_BIND_NONE && (pod.flags & PF_CPU_INT)));
    const int pol = pf_numa_policy(pod.flags) ? pf_numa_policy(pod.flags) : nf_numa_policy(nf);
    nsoa = NUMA && s.nm != nullptr;  // the node's zones (if any) live in the NUMA SoA
    const bool npol = nsoa && !(pod.flags & PF_NUMA_SKIP) && pol != KE_NUMA_POLICY_NONE;
    ok = !rcb || (nf & NF_CPUS_VALID);
    if (nsoa) numa_load(s, node, v);
    // DeviceShare's hints join the Admit of a pod with device requests (topology_hint.go:38-58)
    ds_here = DS && (pod.flags & PF_DS) && (nf & NF_DS_CACHE);
    const RsvOvr* nro = (ok && npol && (nf & NF_RSV_CS)) ? rsv_ovr_of(s, node) : nullptr;
    sh.numa_ovr = 0;
    if (nro && nro->numa_on) {  // a reservation-matched pod: the allocation k_numa_views chose (RsvOvr.numa_dist)
      sh.numa_ovr = 1;  // (a binding pod: its cpuset from the nominated reservation, RsvOvr.reserve / cpus)
      aff = nro->numa_aff;
      for (int z = 0; z < 8; z++)
        for (int r = 0; r < 2; r++) {
          dist[r][z] = nro->numa_dist[2 * z + r];
          if (dist[r][z] != 0) got[r] |= 1u << z;
        }
      stored = true;
    } else if (ok && npol) {  // the affinity the Filter's Admit stored and the allocation on it
      // this rank evaluated the node: its eval stored the affinity (a feasible node admitted, binding pods);
      // else (a node of another shard, a DeviceShare pod) Admit runs here
      const bool have = node >= eval_lo && node < eval_hi && !ds_here;
      NumaPick pk{KE_CODE_SUCCESS, KE_REASON_NONE, have ? (uint32_t)aff_in[node] : 0u};
      DsHints dh;
      dh.status = 0;
      dh.none = true;
      if (ds_here) ds_numa_hints<true>(s, node, pod, k, dh);
      const DsHints* dhp = ds_here ? &dh : nullptr;
      if (rcb) {
        const NumaCs cs = numa_cs_load(s, node, nf, pod);
        DevPod ps = pod;
        ps.req[0] = amplify_bits(pod.req[0], s.cs[CS_RS * s.stride + node]);
        NumaNode tv = v;
        numa_trim(tv, cs);
        if (!have) pk = numa_admit<false, false, true>(s, node, nf, pol, tv, pod, k, 0u, &cs, &ps, dhp);
        if (pk.status == KE_CODE_SUCCESS && pk.aff) numa_distribute<true, true>(tv, pk.aff, pod, got, dist, &cs);
        ok = pk.status == KE_CODE_SUCCESS;
      } else {
        if (!have) pk = numa_admit<false>(s, node, nf, pol, v, pod, k, 0u, nullptr, nullptr, dhp);
        if (pk.status == KE_CODE_SUCCESS && pk.aff) numa_distribute<true>(v, pk.aff, pod, got, dist);
      }
      stored = pk.status == KE_CODE_SUCCESS;
      aff = pk.aff;
    }
    RPROF(0)
    // DeviceShare Reserve allocates on the stored affinity unless the alignment is disabled (plugin.go:452-466);
    // with the alignment disabled nothing checked the devices of a NUMA-admitted node (Filter skipped,
    // Allocate a no-op), so the allocation may fail: Reserve fails and every Reserve of the pod is undone
    if (ok && ds_here && stored && (k.flags & AF_DS_NO_NUMA)) {  // elsewhere the Filter / Admit checked it
      int why = 0;
      ok = ds_try_allocate<true>(s, node, pod, k, DsAff{false, 0u}, nullptr, &why) == KE_CODE_SUCCESS;  // Reserve: no affinity
    }
    RPROF(1)
    if (ok && ds_here && (pod.flags & PF_DS_HINT)) {  // a hinted pod's Reserve-phase allocation must succeed
      int why = 0;
      uint32_t o3[3];
      int8_t v2[2][DS_MINORS];
      ok = hint_allocate(s, node, pod, k, DsAff{stored && aff != 0 && !(k.flags & AF_DS_NO_NUMA), aff}, true, true, o3, v2,
                         &why) == KE_CODE_SUCCESS;
    }
    sh.take = ok && rcb;
    if (sh.take) {
      sh.node = node;
      sh.nf = nf;
      sh.zmask = got[0] | got[1];
      for (int z = 0; z < 8; z++) sh.zcpu[z] = dist[0][z];
    }
  }
  __syncthreads();
  // a KE_RSV_MATCHED pod on a node without a NUMA policy: NodeNUMAResource Reserve allocates from the nominated
  // reservation first (allocateWithNominatedReservation, reservation.go:492-522), as k_rsv_views computed it
  const RsvOvr* ro = (sh.take && (sh.zmask == 0 || sh.numa_ovr) && (sh.nf & NF_RSV_CS)) ? rsv_ovr_of(s, sh.node) : nullptr;
  if (ro && ro->reserve != 0) {
    for (int c = lane; c < CPU_SLOTS; c += 64) a.res[c] = (ro->cpus[c >> 6] >> (c & 63)) & 1;
    __syncthreads();
    if (lane == 0) ok = ro->reserve == 1;
  } else if (sh.take) {  // the accumulator on the whole wave
    const bool took = cpuset_allocate(s, sh.node, sh.nf, pod, a, sh.zmask, sh.zcpu);
    if (lane == 0) ok = took;
  }
  if (lane == 0 && w) {
    RPROF(2)
    if (ok) {
      reserve_row(s, node, nf, pod);
      if (k.flags & AF_EXT) ext_reserve(s, node, pod, k);
      {  // the node's replay record follows its patched row
        NodeRegs nr;
        load_row(s, node, nr);
        prepare_row(nr);
        int64_t wr[NUM_RW];
        rec_from_regs(nr, k, wr);
        for (int u = 0; u < NUM_RW; u++) s.rec[node * NUM_RW + u] = wr[u];
      }
      sh.cs_pass = nsoa && v.zm && s.cpu;  // allocated CPUs per NUMA id before the pod
      sh.commit = rcb;
      if (rcb) {
        const int64_t cnt = s.cs[CS_CNT * s.stride + node];
        sh.node = node;
        sh.excl = (pod.flags & PF_CPU_RCB) ? pf_cpu_excl(pod.flags) : KE_CPU_EXCL_NONE;
        sh.cpc = cs_cpc(cnt);
        sh.max_ref = cs_max_ref(cnt);
      }
    }
    RPROF(3)
  }
  __syncthreads();
  if (sh.cs_pass) {
    for (int c = lane; c < CPU_SLOTS; c += 64) {
      const CpuRec r = a.cpu[c];
      if ((r.flags & CR_VALID) && r.ref > 0 && r.numa < 8) atomicAdd(&sh.cs_old[r.numa], 1);
    }
    __syncthreads();
  }
  if (sh.commit) cpuset_commit_wave(s, a, sh, lane);
  if (lane == 0) {
    RPROF(4)
    if (ok) {
      uint32_t used = sh.used[0] & 0xFFu;
      int n_used = 0;
      for (int q = 0; q < 8; q++) n_used += __popc(sh.used[q]);
      int cs_old[8], cs_new[8];
      for (int z = 0; z < 8; z++) cs_old[z] = sh.cs_old[z], cs_new[z] = sh.cs_old[z] + sh.cs_add[z];
      if (nsoa && v.zm) numa_reserve_cs(s, node, nf, v, got, dist, cs_old, cs_new, used, n_used, out16);
      RPROF(5)
      if (ds_here)
        alloc = ds_reserve<true>(s, node, pod, k, DsAff{stored && aff != 0 && !(k.flags & AF_DS_NO_NUMA), aff},
                           s.vfo ? s.vfo + (int64_t)base * 2 * DS_MINORS : nullptr,
                           (nf & NF_RSV_CS) ? rsv_ovr_of(s, node) : nullptr);
      out_node = (int32_t)node + global_offset;
      out_score = key_score(w);
      if (quota) quota_reserve_g(s, pod, qreq);  // ElasticQuota Reserve
    }
    RPROF(6)
    RPROF_FLUSH(2, 1)
    chosen[base] = out_node;
    chosen_score[base] = out_score;
    dev_alloc[base] = alloc;
    for (int q = 0; q < 4; q++) cpusets[(int64_t)base * 4 + q] = sh.set[q];
    for (int u = 0; u < 6; u++) pstamps[PST * batch_index + u] = t0;  // no prologue: all "replay"
    pstamps[PST * batch_index + 6] = 1;
    pstamps[PST * batch_index + 7] = out_node >= 0;
    stamps[batch_index + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void k_stamp(uint64_t* stamps) { stamps[0] = __builtin_amdgcn_s_memrealtime(); }
// start of a batch on its eval stream: the eval-start stamp, and the zeroed atomicMax targets of a
// DeviceShare batch (NormalizeScore's max) and of a one-pod argmax (one launch instead of three)
__global__ void k_batch_begin(uint64_t* stamp, uint32_t* dsb, uint32_t* argmax) {  // 64 threads
  const int t = threadIdx.x;
  if (t == 0) stamp[0] = __builtin_amdgcn_s_memrealtime();
  if (dsb) {
    dsb[DSB_MAX + t] = 0;
    dsb[DSB_CNT + t] = 0;
    if (t == 0) dsb[DSB_CUT] = 0xFFFFFFFFu;
  }
  if (argmax && t == 0) argmax[0] = 0;
}

// ---------------------------------------------------------------------------------------------
// device state
// ---------------------------------------------------------------------------------------------
// Page-locked host array: the async copies of a ke_schedule call to / from it neither stage nor block the
// host thread (a pageable destination makes hipMemcpyAsync wait for the stream: every readback copy of a call
// would then sit on its critical path one after another).
template <typename T>
struct PinnedVec {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  PinnedVec() = default;
  PinnedVec(const PinnedVec&) = delete;
  PinnedVec& operator=(const PinnedVec&) = delete;
  ~PinnedVec() {
    if (p) (void)hipHostFree(p);
  }
  bool resize(size_t m) {  // contents not kept when it grows
    if (m > cap) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      cap = 0;
      if (hipHostMalloc((void**)&p, sizeof(T) * std::max<size_t>(m, 1), hipHostMallocDefault) != hipSuccess) {
        p = nullptr;
        n = 0;
        return false;
      }
      cap = m;
    }
    n = m;
    return true;
  }
  T* data() { return p; }
  const T* data() const { return p; }
  size_t size() const { return n; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  T* begin() { return p; }
  T* end() { return p + n; }
  void swap(PinnedVec& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
  }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
};

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
  DevPodHint* d_ph = nullptr;  // the hinted pods' records of the current call
  int64_t ph_cap = 0;
  int8_t* d_vfo = nullptr;     // [n_pods][2][DS_MINORS] VF ranks of the Reserves
  int64_t vfo_cap = 0;
  // batch buffers
  uint16_t* d_scores = nullptr;  // [MAX_BATCH][capacity]
  uint32_t* d_cand = nullptr;    // [MAX_BATCH][KMAX]
  int32_t* d_cand_cnt = nullptr;
  int32_t* d_batch_base = nullptr;  // a zero word (batch base of the parity / bench launches)
  int32_t* d_sched = nullptr;       // ke_schedule bookkeeping: batch bases, hand-off flags, fixup stamps
  int64_t sched_cap = 0;            // bytes
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
  // node sharding (ke_shard_init): this rank evaluates/selects nodes shard_range(rank); the per-shard
  // candidate lists meet in d_gath through an RCCL all-gather (or, loopback, all shards run here)
  int world = 1, rank = 0;
  bool loopback = false;
  ncclComm_t comm = nullptr;
  // ke_shard_init_host: the caller's host collective carries the all-gather / all-reduces instead of RCCL
  ke_host_collective host_fn = nullptr;
  void* host_user = nullptr;
  uint32_t* d_gath = nullptr;  // [world][GATH_WORDS]
  uint32_t* d_split = nullptr; // [MAX_WORLD][GATH_WORDS]: the part lists of a split k_select (unsharded)
  // DeviceShare
  bool ds_alloc = false;         // soa.ds / soa.dsm allocated
  size_t pt_words = 0;           // soa.pt capacity (uint64 words)
  uint16_t* d_dsraw = nullptr;   // [capacity] raw DeviceShare score + 1 of the batch's DeviceShare pod
  uint32_t* d_dsmax = nullptr;   // 1 + max raw score over the feasible nodes of the batch's pod
  uint64_t* d_devalloc = nullptr;  // [n_pods] device minors allocated per pod
  int64_t* d_dsrows = nullptr;   // staging for DeviceShare row uploads
  int64_t ds_staging_cap = 0;
  PinnedVec<DevPod> host_pods;    // the last uploaded queue (batch segmentation), page-locked
  PinnedVec<uint8_t> h_out;       // ke_schedule's readback staging (placements, allocations, stamps)
  PinnedVec<int64_t> h_refresh[2];  // device_refresh's row staging (every table's rows + indices), two in turn
  PinnedVec<uint8_t> h_rsv;       // a matched pod's RsvPair / RsvOvr uploads
  PinnedVec<int32_t> h_rsv_out;   // k_rsv_pick's result words, read back by the call's own copies
  PinnedVec<int32_t> h_cut;       // a DeviceShare batch's cut word (async read-back, the next batch enqueued behind)
  std::vector<DevPodHint> host_ph;  // its hinted pods' records (the async upload reads them)
  // NUMA topology
  bool numa_alloc = false;         // soa.nf / soa.nm allocated
  int64_t* d_numaalloc = nullptr;  // [n_pods][16] per-zone allocation of each pod (ke_schedule)
  int64_t* d_numarows = nullptr;   // staging for NUMA row uploads
  int64_t numa_staging_cap = 0;
  bool ext_alloc = false;          // soa.xf / soa.xm allocated (NodeResourcesFitPlus / ScarceResourceAvoidance)
  int64_t* d_xrows = nullptr;      // staging for ext row uploads
  int64_t ext_staging_cap = 0;
  uint64_t* d_defer = nullptr;     // deferred BestEffort pairs of one eval launch (k_numa_fallback)
  int64_t defer_cap = 0;           // bytes
  uint32_t* d_defer_cnt = nullptr; // one counter per batch of a ke_schedule (or the ke_eval launch)
  int64_t defer_cnt_cap = 0;       // bytes
  // CPU tables (cpuset pods)
  bool cpu_alloc = false;          // soa.cs / soa.cpu allocated
  int64_t* d_cpurows = nullptr;    // staging for CPU table uploads
  int64_t cpu_staging_cap = 0;     // nodes
  uint64_t* d_cpusets = nullptr;   // [n_pods][4] cpuset of each pod (ke_schedule)
  int64_t cpusets_cap = 0;         // bytes
  uint8_t* d_aff = nullptr;        // [capacity] NUMA affinity per node of a singleton batch's eval
  // pipelined schedule: eval + select run on `estream` one batch ahead of the Reserve chain on `stream`
  hipStream_t estream = nullptr;
  // a call's staging copies (pod upload, bookkeeping words) and read-back run on `cstream`: the next call's uploads
  // proceed while this one still runs, and the Reserve stream goes from one call's Reserve kernel to the next.
  // Opt-in (KOORDEVAL_STAGING_STREAM=1): on the C3 bench it measured 78-85 G against 92 G with everything on `stream`
  // (tools/_ab.sh, one box, alternated), so by default the staging work stays on `stream` (nullptr here)
  hipStream_t cstream = nullptr;
  hipEvent_t ev_setup = nullptr, ev_rend = nullptr;
  // a second eval stream with its own score matrix / part lists: consecutive batches of a stale-list run
  // alternate between the two, so batch b+1's eval overlaps batch b's select (nullptr: clusters too large to
  // double the score matrix)
  hipStream_t estream2 = nullptr;
  hipEvent_t ev_sel2 = nullptr;
  std::vector<hipEvent_t> tev;  // device_schedule's events (pool): span, the call's end per stream, samples
  // the other call's buffers of two in flight (ke_schedule_submit): swapped with the fields of the same name
  struct CallBufs {
    PinnedVec<DevPod> host_pods;
    DevPod* d_pods = nullptr;
    int64_t pods_cap = 0;
    int32_t *d_chosen = nullptr, *d_chosen_score = nullptr;
    uint64_t* d_stamps = nullptr;
    uint64_t* d_devalloc = nullptr;
    int64_t* d_numaalloc = nullptr;
    int64_t out_cap = 0;
    uint64_t* d_cpusets = nullptr;
    int64_t cpusets_cap = 0;
    int32_t* d_sched = nullptr;
    int64_t sched_cap = 0;
    PinnedVec<uint8_t> h_out;
    std::vector<hipEvent_t> tev;
  } alt;
  uint16_t* d_scores2 = nullptr;
  uint32_t* d_split2 = nullptr;
  uint32_t* d_stale = nullptr;      // [2][MAX_BATCH][KSTALE] stale-snapshot candidate lists
  uint32_t* d_pre = nullptr;        // [2][MAX_BATCH][KSTALE2] select-ahead lists before k_fixlist (+ counts after)
  uint32_t* d_chg = nullptr;        // changed-node bitmap of the replay when node ids exceed its LDS copy
  int64_t* d_trows = nullptr;       // [MAX_BATCH][NUM_RW] records the last resolved batch changed (node in RW_PAD)
  int32_t* d_tcnt = nullptr;        // their count
  int32_t* d_parts_done = nullptr;  // [MAX_BATCH] parts of each pod a split k_select finished (zero between launches)
  int32_t* d_stale_cnt = nullptr;   // [2][MAX_BATCH]
  static constexpr int EV_RING = 8;
  hipEvent_t ev_res[EV_RING] = {};  // a batch's Reserve done (stream)
  hipEvent_t ev_sel[EV_RING] = {};  // a batch's candidate lists done (estream)
  hipEvent_t ev_start = nullptr;
  // device_refresh's copies + scatters (no host wait since round 6): the next refresh waits on it before it reuses the
  // staging; every reader of the rows runs on `stream` behind them or waits for an event recorded there after them
  hipEvent_t ev_refresh[2] = {};  // the copies out of h_refresh[i] done
  bool refresh_pending[2] = {};
  int refresh_cur = 0;
  std::vector<std::function<void(const int32_t*)>> deferred;  // device_refresh(defer): its scatters, gated
  int32_t* d_rsv_gate = nullptr;    // k_rsv_check's word: a fused matched pod's speculation failed (1)
  bool refresh_sync = false;        // KOORDEVAL_REFRESH_SYNC=1: the host waits for every refresh (A/B)
  bool pipeline = true;             // ke_set_pipeline
  bool pipe_fixup = false;          // ke_set_pipeline(2): exact lists from k_fixup for every run (else quota runs only)
  // dynamic LDS of the eval streams' LDS-free kernels: more than what a Reserve workgroup (ResLds) leaves free of
  // the CU's LDS, from the device's per-CU LDS at device_create (EXCL_LDS at the 160 KB of gfx950)
  unsigned excl_lds = EXCL_LDS;
  bool eval_patch = true;           // two eval streams: evals wait for batch b-3, k_patch adds b-2 (KOORDEVAL_EVAL_PATCH)
  bool select_ahead = true;         // ... and the select follows the eval at once, k_fixlist adds b-2 to the lists
  bool fix_merge = true;            // ... a split select leaves its parts unmerged, k_fixlist<PARTS> merges them first
                                    // (KOORDEVAL_SELECT_AHEAD; 0: k_patch before the select)
  int t_helpers = 4;                // T-row helper workgroups of a stale-list run (THelp; KOORDEVAL_T_HELPERS)
  int t_help_ignore = 0;            // test hook (KOORDEVAL_T_HELPERS_IGNORE): the replay's own T rows every batch
  // the Reservation plugin of a singleton batch (k_rsv_pick): its pairs and result words
  RsvPair* d_rsv = nullptr;
  int64_t rsv_cap = 0;              // bytes
  void* d_rsv_views = nullptr;      // k_rsv_views: views, outputs, the pod
  int64_t rsv_views_cap = 0;
  void* d_ds_views = nullptr;       // k_ds_views: views, outputs, the pod
  int64_t ds_views_cap = 0;
  void* d_numa_views = nullptr;     // k_numa_views: views, outputs, the pod
  int64_t numa_views_cap = 0;
  RsvOvr* d_rovr = nullptr;         // the segment's allocate-from-reservation decisions (SoA::rovr)
  int64_t rovr_cap = 0;
  int32_t* d_rsv_out = nullptr;     // [4]
  RsvPickSt* d_rsv_st = nullptr;    // k_rsv_stage's words (node-sharded contexts)
};

// Contiguous node range of shard `rank`: 512-aligned chunks (k_select's 16-B loads stay aligned).
void shard_range(int n_nodes, int rank, int world, int* lo, int* hi) {
  const int chunk = ((n_nodes + world - 1) / world + 511) & ~511;
  *lo = std::min(rank * chunk, n_nodes);
  *hi = std::min(*lo + chunk, n_nodes);
}

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
  int cu_lds = 0;  // the Reserve kernels' ResLds fills a CU_LDS_BYTES CU; the exclusion of co-resident eval waves
  HIP_OK(hipDeviceGetAttribute(&cu_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, d->device));
  if (cu_lds < (int)sizeof(ResLds))
    return fail(KE_ERR_UNSUPPORTED, "device LDS per CU below the Reserve kernels' ResLds (built for gfx950's 160 KB)");
  d->excl_lds = std::max<unsigned>(EXCL_LDS, (unsigned)(cu_lds - (int)sizeof(ResLds)) + 1024u);
  int prio_lo = 0, prio_hi = 0;  // the Reserve chain gets the higher queue priority
  HIP_OK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  if (const char* e = std::getenv("KOORDEVAL_T_HELPERS")) d->t_helpers = std::max(0, std::min(8, std::atoi(e)));
  if (const char* e = std::getenv("KOORDEVAL_EVAL_PATCH")) d->eval_patch = std::atoi(e) != 0;
  if (const char* e = std::getenv("KOORDEVAL_SELECT_AHEAD")) d->select_ahead = std::atoi(e) != 0;
  if (const char* e = std::getenv("KOORDEVAL_FIX_MERGE")) d->fix_merge = std::atoi(e) != 0;
  if (const char* e = std::getenv("KOORDEVAL_REFRESH_SYNC")) d->refresh_sync = std::atoi(e) != 0;
  if (const char* e = std::getenv("KOORDEVAL_T_HELPERS_IGNORE")) d->t_help_ignore = std::atoi(e) != 0;
  HIP_OK(hipStreamCreateWithPriority(&d->stream, hipStreamNonBlocking, prio_hi));
  HIP_OK(hipStreamCreateWithPriority(&d->estream, hipStreamNonBlocking, prio_lo));
  if (const char* e = std::getenv("KOORDEVAL_STAGING_STREAM"); e && std::atoi(e) != 0)
    HIP_OK(hipStreamCreateWithPriority(&d->cstream, hipStreamNonBlocking, prio_lo));
  HIP_OK(hipEventCreateWithFlags(&d->ev_setup, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&d->ev_rend, hipEventDisableTiming));
  for (int e = 0; e < DeviceState::EV_RING; e++) {
    HIP_OK(hipEventCreateWithFlags(&d->ev_res[e], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&d->ev_sel[e], hipEventDisableTiming));
  }
  HIP_OK(hipEventCreateWithFlags(&d->ev_start, hipEventDisableTiming));
  for (hipEvent_t& e : d->ev_refresh) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  d->capacity = ((int64_t)ctx->cfg.node_capacity + 255) & ~255LL;
  d->soa.stride = d->capacity;
  HIP_OK(hipMalloc(&d->soa.f, sizeof(int64_t) * NUM_I64_FIELDS * d->capacity));
  HIP_OK(hipMalloc(&d->soa.flags, sizeof(uint32_t) * d->capacity));
  HIP_OK(hipMemsetAsync(d->soa.f, 0, sizeof(int64_t) * NUM_I64_FIELDS * d->capacity, d->stream));
  HIP_OK(hipMemsetAsync(d->soa.flags, 0, sizeof(uint32_t) * d->capacity, d->stream));
  HIP_OK(hipMalloc(&d->d_scores, sizeof(uint16_t) * MAX_BATCH * d->capacity));
  if (d->capacity <= (1 << 20)) {  // <= 128 MB for the second score matrix
    HIP_OK(hipStreamCreateWithPriority(&d->estream2, hipStreamNonBlocking, prio_lo));
    HIP_OK(hipEventCreateWithFlags(&d->ev_sel2, hipEventDisableTiming));
    HIP_OK(hipMalloc(&d->d_scores2, sizeof(uint16_t) * MAX_BATCH * d->capacity));
    HIP_OK(hipMalloc(&d->d_split2, sizeof(uint32_t) * GATH_WORDS_MAX * MAX_WORLD));
  }
  HIP_OK(hipMalloc(&d->d_cand, sizeof(uint32_t) * MAX_BATCH * KMAX));
  HIP_OK(hipMalloc(&d->d_cand_cnt, sizeof(int32_t) * MAX_BATCH));
  HIP_OK(hipMalloc(&d->d_batch_base, sizeof(int32_t)));
  HIP_OK(hipMemsetAsync(d->d_batch_base, 0, sizeof(int32_t), d->stream));
  HIP_OK(hipMalloc(&d->d_stale, sizeof(uint32_t) * 2 * MAX_BATCH * KSTALE));
  HIP_OK(hipMalloc(&d->d_pre, sizeof(uint32_t) * 2 * MAX_BATCH * (KSTALE2 + 1)));
  HIP_OK(hipMalloc(&d->d_stale_cnt, sizeof(int32_t) * 2 * MAX_BATCH));
  HIP_OK(hipMalloc(&d->d_trows, sizeof(int64_t) * MAX_BATCH * NUM_RW));
  HIP_OK(hipMalloc(&d->soa.rec, sizeof(int64_t) * NUM_RW * d->capacity));
  HIP_OK(hipMalloc(&d->soa.kerr, sizeof(int32_t)));
  HIP_OK(hipMemsetAsync(d->soa.kerr, 0, sizeof(int32_t), d->stream));
  HIP_OK(hipMemsetAsync(d->soa.rec, 0, sizeof(int64_t) * NUM_RW * d->capacity, d->stream));
  HIP_OK(hipMalloc(&d->d_tcnt, sizeof(int32_t)));
  HIP_OK(hipMalloc(&d->d_parts_done, sizeof(int32_t) * 2 * MAX_BATCH));  // (one half per eval stream)
  HIP_OK(hipMemset(d->d_parts_done, 0, sizeof(int32_t) * 2 * MAX_BATCH));
  if (d->capacity > (int64_t)CHG_LDS_WORDS * 32) {  // zero between batches (each replay clears its bits)
    HIP_OK(hipMalloc(&d->d_chg, sizeof(uint32_t) * (d->capacity + 31) / 32));
    HIP_OK(hipMemsetAsync(d->d_chg, 0, sizeof(uint32_t) * (d->capacity + 31) / 32, d->stream));
  }
  HIP_OK(hipMalloc(&d->d_dsraw, sizeof(uint16_t) * MAX_BATCH * d->capacity));  // per pod of a DeviceShare batch
  HIP_OK(hipMalloc(&d->d_dsmax, sizeof(uint32_t) * DSB_WORDS));
  d->soa.dsb = d->d_dsmax;
  d->soa.dsraw = d->d_dsraw;
  HIP_OK(hipMalloc(&d->d_aff, d->capacity));
  HIP_OK(hipMalloc(&d->d_split, sizeof(uint32_t) * GATH_WORDS_MAX * MAX_WORLD));
  HIP_OK(hipMalloc(&d->d_rsv_out, sizeof(int32_t) * 4));
  HIP_OK(hipMalloc(&d->d_rsv_st, sizeof(RsvPickSt)));
  HIP_OK(hipStreamSynchronize(d->stream));
  return KE_OK;
}

int device_refresh(Context* ctx, int64_t now, bool defer = false);
int device_refresh_flush(Context* ctx, const int32_t* gate);
// k_rsv_views for one KE_RSV_MATCHED pod: the allocate-from-reservation trials `views` on the current device
// state (synchronous; the segment's device_schedule follows)
static KArgs make_kargs(const Context* ctx, int64_t now);
int device_rsv_views(Context* ctx, const ke_pod& pod, int64_t now, const std::vector<RsvView>& views,
                     std::vector<RsvViewOut>& out) {
  DeviceState* d = ctx->dev;
  out.assign(views.size(), RsvViewOut{});
  if (views.empty()) return KE_OK;
  HIP_OK(hipSetDevice(d->device));
  int rc = device_refresh(ctx, now);  // the rows / CPU tables as the segment will see them
  if (rc) return rc;
  for (const RsvView& v : views)
    if (v.node < 0 || v.node >= ctx->n_nodes) return fail(KE_ERR_DEVICE, "reservation view node out of range");
  const DevPod dp = make_dev_pod(ctx->cfg, pod, pod_hints(*ctx, pod), &ctx->tmpl);
  const KArgs k = make_kargs(ctx, now);
  const size_t vb = sizeof(RsvView) * views.size(), ob = sizeof(RsvViewOut) * views.size();
  rc = ensure((void**)&d->d_rsv_views, &d->rsv_views_cap, (int64_t)(vb + ob + sizeof(DevPod)));
  if (rc) return rc;
  uint8_t* base = (uint8_t*)d->d_rsv_views;
  HIP_OK(hipMemcpyAsync(base, views.data(), vb, hipMemcpyHostToDevice, d->stream));
  HIP_OK(hipMemcpyAsync(base + vb + ob, &dp, sizeof(DevPod), hipMemcpyHostToDevice, d->stream));
  hipLaunchKernelGGL(k_rsv_views, dim3((unsigned)views.size()), dim3(64), 0, d->stream, d->soa,
                     (const DevPod*)(base + vb + ob), (const RsvView*)base, (RsvViewOut*)(base + vb), k);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(out.data(), base + vb, ob, hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  return KE_OK;
}

// k_ds_views for one reservation-matched / -ignored DeviceShare pod: its views on the current device state
// (synchronous, like device_rsv_views)
int device_ds_views(Context* ctx, const ke_pod& pod, int64_t now, const std::vector<DsView>& views,
                    std::vector<DsViewOut>& out) {
  DeviceState* d = ctx->dev;
  out.assign(views.size(), DsViewOut{});
  if (views.empty()) return KE_OK;
  HIP_OK(hipSetDevice(d->device));
  int rc = device_refresh(ctx, now);  // the rows as the segment will see them
  if (rc) return rc;
  if (!d->soa.ds) return fail(KE_ERR_DEVICE, "DeviceShare views without a device SoA");
  for (const DsView& v : views)
    if (v.node < 0 || v.node >= ctx->n_nodes) return fail(KE_ERR_DEVICE, "DeviceShare view node out of range");
  const DevPod dp = make_dev_pod(ctx->cfg, pod, pod_hints(*ctx, pod), &ctx->tmpl);
  const KArgs k = make_kargs(ctx, now);
  const size_t vb = sizeof(DsView) * views.size(), ob = sizeof(DsViewOut) * views.size();
  rc = ensure((void**)&d->d_ds_views, &d->ds_views_cap, (int64_t)(vb + ob + sizeof(DevPod)));
  if (rc) return rc;
  uint8_t* base = (uint8_t*)d->d_ds_views;
  HIP_OK(hipMemcpyAsync(base, views.data(), vb, hipMemcpyHostToDevice, d->stream));
  HIP_OK(hipMemcpyAsync(base + vb + ob, &dp, sizeof(DevPod), hipMemcpyHostToDevice, d->stream));
  hipLaunchKernelGGL(k_ds_views, dim3((unsigned)views.size()), dim3(64), 0, d->stream, d->soa,
                     (const DevPod*)(base + vb + ob), (const DsView*)base, (DsViewOut*)(base + vb), k);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(out.data(), base + vb, ob, hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  return KE_OK;
}

int device_numa_views(Context* ctx, const ke_pod& pod, int64_t now, const std::vector<NumaRsvView>& views,
                      std::vector<NumaRsvOut>& out) {
  DeviceState* d = ctx->dev;
  out.assign(views.size(), NumaRsvOut{});
  if (views.empty()) return KE_OK;
  HIP_OK(hipSetDevice(d->device));
  int rc = device_refresh(ctx, now);  // the rows as the segment will see them
  if (rc) return rc;
  if (!d->soa.nf) return fail(KE_ERR_DEVICE, "NUMA views without a NUMA SoA");
  for (const NumaRsvView& v : views)
    if (v.node < 0 || v.node >= ctx->n_nodes || v.n < 0 || v.n > NV_MAX)
      return fail(KE_ERR_DEVICE, "NUMA view node / trial count out of range");
  const DevPod dp = make_dev_pod(ctx->cfg, pod, pod_hints(*ctx, pod), &ctx->tmpl);
  const KArgs k = make_kargs(ctx, now);
  const size_t vb = sizeof(NumaRsvView) * views.size(), ob = sizeof(NumaRsvOut) * views.size();
  rc = ensure((void**)&d->d_numa_views, &d->numa_views_cap, (int64_t)(vb + ob + sizeof(DevPod)));
  if (rc) return rc;
  uint8_t* base = (uint8_t*)d->d_numa_views;
  HIP_OK(hipMemcpyAsync(base, views.data(), vb, hipMemcpyHostToDevice, d->stream));
  HIP_OK(hipMemcpyAsync(base + vb + ob, &dp, sizeof(DevPod), hipMemcpyHostToDevice, d->stream));
  hipLaunchKernelGGL(k_numa_views, dim3((unsigned)views.size()), dim3(64), 0, d->stream, d->soa,
                     (const DevPod*)(base + vb + ob), (const NumaRsvView*)base, (NumaRsvOut*)(base + vb), k);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(out.data(), base + vb, ob, hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  return KE_OK;
}

// k_rsv_pick's result of the last device_schedule (a segment of one KE_RSV_MATCHED pod)
int device_rsv_result(Context* ctx, int32_t* out4) {
  DeviceState* d = ctx->dev;
  // copied after k_rsv_pick on its stream, complete with the call (device_schedule waited for every stream)
  if (d->h_rsv_out.size() < 4) return fail(KE_ERR_DEVICE, "no k_rsv_pick result staged");
  for (int i = 0; i < 4; i++) out4[i] = d->h_rsv_out[i];
  return KE_OK;
}

// the fused matched pod's gate after its call: 1 = a plain pod of the call took a node of its reservations
int device_rsv_gate(const Context* ctx) {
  const DeviceState* d = ctx->dev;
  return d->h_rsv_out.size() >= 5 ? d->h_rsv_out[4] : 0;
}

void device_destroy(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->stream) (void)hipStreamSynchronize(d->stream);
  if (d->comm) (void)ncclCommDestroy(d->comm);
  void* ptrs[] = {d->soa.f,     d->soa.flags, d->d_rows,      d->d_idx,          d->d_pods,   d->d_scores,
                  d->d_cand,    d->d_cand_cnt, d->d_batch_base, d->d_chosen,     d->d_chosen_score,
                  d->d_stamps,  d->d_parity, d->d_best,       d->d_gath,    d->d_split,         d->soa.ds,   d->soa.dsm,
                  d->d_dsraw,   d->d_dsmax,  d->d_devalloc,   d->d_dsrows,       d->soa.nf,   d->soa.nm,
                  d->d_numaalloc, d->d_numarows, d->d_defer, d->d_defer_cnt, d->soa.cs, d->soa.cpu,
                  d->d_cpurows, d->d_cpusets, d->d_aff, d->soa.qt, d->soa.qm, d->d_sched, d->d_stale,
                  d->d_stale_cnt, d->d_pre, d->d_trows, d->d_tcnt, d->d_parts_done, d->d_scores2, d->d_split2, d->d_chg, d->soa.rec, d->soa.pt, d->soa.kerr,
                  d->soa.xf, d->soa.xm, d->d_xrows, d->soa.dsx, d->d_ph, d->d_vfo, d->d_rsv, d->d_rsv_out, d->d_rsv_st,
                  d->d_rsv_views, d->d_ds_views, d->d_numa_views, d->d_rovr, d->d_rsv_gate};
  if (d->estream) (void)hipStreamSynchronize(d->estream);
  if (d->estream2) (void)hipStreamSynchronize(d->estream2);
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (int e = 0; e < DeviceState::EV_RING; e++) {
    if (d->ev_res[e]) (void)hipEventDestroy(d->ev_res[e]);
    if (d->ev_sel[e]) (void)hipEventDestroy(d->ev_sel[e]);
  }
  if (d->ev_start) (void)hipEventDestroy(d->ev_start);
  for (hipEvent_t e : d->ev_refresh)
    if (e) (void)hipEventDestroy(e);
  if (d->estream) (void)hipStreamDestroy(d->estream);
  if (d->cstream) (void)hipStreamDestroy(d->cstream);
  if (d->ev_setup) (void)hipEventDestroy(d->ev_setup);
  if (d->ev_rend) (void)hipEventDestroy(d->ev_rend);
  if (d->estream2) (void)hipStreamDestroy(d->estream2);
  if (d->ev_sel2) (void)hipEventDestroy(d->ev_sel2);
  for (auto& e : d->tev) (void)hipEventDestroy(e);
  for (auto& e : d->alt.tev) (void)hipEventDestroy(e);
  for (void* p : {(void*)d->alt.d_pods, (void*)d->alt.d_chosen, (void*)d->alt.d_chosen_score, (void*)d->alt.d_stamps,
                  (void*)d->alt.d_devalloc, (void*)d->alt.d_numaalloc, (void*)d->alt.d_cpusets, (void*)d->alt.d_sched})
    if (p) (void)hipFree(p);
  if (d->stream) (void)hipStreamDestroy(d->stream);
  delete d;
  ctx->dev = nullptr;
}

// ElasticQuota table -> device (when the host tree changed since the last upload)
static int device_quota_upload(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (!d->soa.qt) {
    HIP_OK(hipMalloc(&d->soa.qt, sizeof(int64_t) * NUM_QF * QT_STRIDE));
    HIP_OK(hipMalloc(&d->soa.qm, sizeof(int32_t) * QT_STRIDE));
  }
  std::vector<int64_t> t((size_t)NUM_QF * QT_STRIDE, 0);
  std::vector<int32_t> m(QT_STRIDE, 0xFFFF);  // parent -1, no keys
  for (size_t i = 0; i < ctx->quotas.size(); i++) {
    const ke_quota& q = ctx->quotas[i];
    uint32_t w = (uint32_t)(uint16_t)(int16_t)q.parent;
    for (int r = 0; r < KE_NRES; r++) {
      t[(QF_LIM + r) * QT_STRIDE + i] = ctx->qlimit[i * KE_NRES + r];
      t[(QF_MIN + r) * QT_STRIDE + i] = q.has_min[r] ? q.min[r] : 0;
      t[(QF_USED + r) * QT_STRIDE + i] = q.used[r];
      t[(QF_NP + r) * QT_STRIDE + i] = q.non_preemptible_used[r];
      w |= (uint32_t)(ctx->qlimit_has[i * KE_NRES + r] != 0) << (16 + r);
      w |= (uint32_t)(q.has_min[r] != 0) << (18 + r);
      w |= (uint32_t)(q.has_max[r] != 0) << (20 + r);
    }
    m[i] = (int32_t)w;
  }
  HIP_OK(hipStreamSynchronize(d->stream));
  HIP_OK(hipMemcpy(d->soa.qt, t.data(), sizeof(int64_t) * t.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d->soa.qm, m.data(), sizeof(int32_t) * m.size(), hipMemcpyHostToDevice));
  ctx->quota_dirty = false;
  ctx->quota_on_device = true;
  return KE_OK;
}

// device used / non-preemptible used -> the host objects (ke_quota_state)
int device_quota_sync(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (!ctx->quota_on_device || !d || !d->soa.qt) return KE_OK;
  HIP_OK(hipSetDevice(d->device));
  std::vector<int64_t> t((size_t)4 * QT_STRIDE);
  HIP_OK(hipStreamSynchronize(d->stream));
  HIP_OK(hipMemcpy(t.data(), d->soa.qt + (size_t)QF_USED * QT_STRIDE, sizeof(int64_t) * t.size(), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < ctx->quotas.size(); i++)
    for (int r = 0; r < KE_NRES; r++) {
      ctx->quotas[i].used[r] = t[(size_t)r * QT_STRIDE + i];
      ctx->quotas[i].non_preemptible_used[r] = t[(size_t)(2 + r) * QT_STRIDE + i];
    }
  return KE_OK;
}

#define RCCL_OK(expr)                                                               \
  do {                                                                              \
    ncclResult_t _r = (expr);                                                       \
    if (_r != ncclSuccess) return fail(KE_ERR_DEVICE, std::string(#expr ": ") + ncclGetErrorString(_r)); \
  } while (0)

int device_comm_unique_id(uint8_t* id) {
  ncclUniqueId u;
  RCCL_OK(ncclGetUniqueId(&u));
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return KE_OK;
}

// Collective over `world` ranks (every rank calls it with the same id); id == nullptr = loopback.
int device_shard_init(Context* ctx, int rank, int world, const uint8_t* id) {
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  if (world < 1 || world > MAX_WORLD || rank < 0 || rank >= world)
    return fail(KE_ERR_INVALID, "ke_shard_init: need 1 <= world <= 8 and 0 <= rank < world");
  if (d->comm) {
    RCCL_OK(ncclCommDestroy(d->comm));
    d->comm = nullptr;
  }
  d->host_fn = nullptr;
  d->host_user = nullptr;
  if (!d->d_gath) HIP_OK(hipMalloc(&d->d_gath, sizeof(uint32_t) * GATH_WORDS_MAX * MAX_WORLD));
  HIP_OK(hipMemsetAsync(d->d_gath, 0, sizeof(uint32_t) * GATH_WORDS_MAX * MAX_WORLD, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  d->world = world;
  d->rank = rank;
  d->loopback = id == nullptr && world > 1;
  if (id) {  // world == 1 with an id: a 1-rank communicator through the sharded path (tests)
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    RCCL_OK(ncclCommInitRank(&d->comm, world, u, rank));
  }
  return KE_OK;
}

// ke_shard_init_host: the same sharded path, its collectives through the caller's host function (e.g. gloo)
int device_shard_init_host(Context* ctx, int rank, int world, ke_host_collective fn, void* user) {
  if (!fn) return fail(KE_ERR_INVALID, "ke_shard_init_host: null collective");
  int rc = device_shard_init(ctx, rank, world, nullptr);
  if (rc) return rc;
  DeviceState* d = ctx->dev;
  d->loopback = false;
  d->host_fn = fn;
  d->host_user = user;
  return KE_OK;
}

// The shard collectives on the eval stream `es`: RCCL, or the host collective (the stream's work so far completes,
// the words go through host memory and back before the next launch on `es`)
static int coll_all_gather(DeviceState* d, uint32_t* mine, uint32_t* all, size_t count, hipStream_t es) {
  if (d->host_fn) {
    std::vector<uint32_t> snd(count), rcv(count * (size_t)d->world);
    HIP_OK(hipStreamSynchronize(es));
    HIP_OK(hipMemcpy(snd.data(), mine, sizeof(uint32_t) * count, hipMemcpyDeviceToHost));
    if (d->host_fn(d->host_user, KE_COLL_ALL_GATHER, KE_COLL_U32, snd.data(), rcv.data(), (int64_t)count))
      return fail(KE_ERR_DEVICE, "host all-gather failed");
    HIP_OK(hipMemcpy(all, rcv.data(), sizeof(uint32_t) * rcv.size(), hipMemcpyHostToDevice));
    return KE_OK;
  }
  RCCL_OK(ncclAllGather(mine, all, count, ncclUint32, d->comm, es));
  return KE_OK;
}
static int coll_all_reduce(DeviceState* d, void* buf, size_t count, int dt, int op, hipStream_t es) {
  const size_t w = (dt == KE_COLL_I64 || dt == KE_COLL_U64) ? 8 : 4;
  if (d->host_fn) {
    std::vector<uint8_t> snd(w * count), rcv(w * count);
    HIP_OK(hipStreamSynchronize(es));
    HIP_OK(hipMemcpy(snd.data(), buf, w * count, hipMemcpyDeviceToHost));
    if (d->host_fn(d->host_user, op, dt, snd.data(), rcv.data(), (int64_t)count))
      return fail(KE_ERR_DEVICE, "host all-reduce failed");
    HIP_OK(hipMemcpy(buf, rcv.data(), w * count, hipMemcpyHostToDevice));
    return KE_OK;
  }
  const ncclDataType_t t = dt == KE_COLL_U32 ? ncclUint32 : dt == KE_COLL_I32 ? ncclInt32 : dt == KE_COLL_I64 ? ncclInt64 : ncclUint64;
  RCCL_OK(ncclAllReduce(buf, buf, count, t, op == KE_COLL_MAX ? ncclMax : ncclMin, d->comm, es));
  return KE_OK;
}

bool device_sharded(const Context* ctx) {
  return ctx->dev && (ctx->dev->world > 1 || ctx->dev->comm || ctx->dev->host_fn);
}

int device_shard_range(Context* ctx, int* lo, int* hi) {
  DeviceState* d = ctx->dev;
  shard_range(ctx->n_nodes, d->rank, d->world, lo, hi);
  return KE_OK;
}

static KArgs make_kargs(const Context* ctx, int64_t now) {
  KArgs k = ctx->kargs_template;
  k.now = now;
  return k;
}

constexpr int DS_ROW_WORDS = NUM_DS_FIELDS + NUM_DS_MASKS + NUM_DSX;  // device fields, masks, hint words
__global__ void k_scatter_ds(SoA s, const int64_t* __restrict__ rows, const int32_t* __restrict__ idx, int n,
                             const int32_t* __restrict__ gate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n || (gate && *gate)) return;
  const int64_t i = idx[t];
  const int64_t* r = rows + (int64_t)t * DS_ROW_WORDS;
  for (int f = 0; f < NUM_DS_FIELDS; f++) s.ds[f * s.stride + i] = r[f];
  for (int w = 0; w < NUM_DS_MASKS; w++) s.dsm[w * s.stride + i] = (uint64_t)r[NUM_DS_FIELDS + w];
  for (int w = 0; w < NUM_DSX; w++) s.dsx[w * s.stride + i] = r[NUM_DS_FIELDS + NUM_DS_MASKS + w];
}

static int ensure_ds(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (d->ds_alloc || !ctx->ds_enabled) return KE_OK;
  HIP_OK(hipMalloc(&d->soa.ds, sizeof(int64_t) * NUM_DS_FIELDS * d->capacity));
  HIP_OK(hipMalloc(&d->soa.dsm, sizeof(uint64_t) * NUM_DS_MASKS * d->capacity));
  HIP_OK(hipMemsetAsync(d->soa.ds, 0, sizeof(int64_t) * NUM_DS_FIELDS * d->capacity, d->stream));
  HIP_OK(hipMemsetAsync(d->soa.dsm, 0, sizeof(uint64_t) * NUM_DS_MASKS * d->capacity, d->stream));
  HIP_OK(hipMalloc(&d->soa.dsx, sizeof(int64_t) * NUM_DSX * d->capacity));
  HIP_OK(hipMemsetAsync(d->soa.dsx, 0, sizeof(int64_t) * NUM_DSX * d->capacity, d->stream));
  d->ds_alloc = true;
  return KE_OK;
}

constexpr int NUMA_ROW_WORDS = NUM_NUMA_FIELDS + 1;  // int64 fields + the mask word

__global__ void k_scatter_numa(SoA s, const int64_t* __restrict__ rows, const int32_t* __restrict__ idx, int n,
                             const int32_t* __restrict__ gate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n || (gate && *gate)) return;
  const int64_t i = idx[t];
  const int64_t* r = rows + (int64_t)t * NUMA_ROW_WORDS;
  for (int f = 0; f < NUM_NUMA_FIELDS; f++) s.nf[f * s.stride + i] = r[f];
  s.nm[i] = (uint64_t)r[NUM_NUMA_FIELDS];
}

static int ensure_numa(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (d->numa_alloc || !ctx->numa_enabled) return KE_OK;
  HIP_OK(hipMalloc(&d->soa.nf, sizeof(int64_t) * NUM_NUMA_FIELDS * d->capacity));
  HIP_OK(hipMalloc(&d->soa.nm, sizeof(uint64_t) * d->capacity));
  HIP_OK(hipMemsetAsync(d->soa.nf, 0, sizeof(int64_t) * NUM_NUMA_FIELDS * d->capacity, d->stream));
  HIP_OK(hipMemsetAsync(d->soa.nm, 0, sizeof(uint64_t) * d->capacity, d->stream));
  d->numa_alloc = true;
  for (int32_t i = 0; i < ctx->n_nodes; i++)  // rows derived before the NUMA SoA existed
    if (!ctx->nodes[i].zones.empty()) ctx->nodes[i].dirty = true;
  return KE_OK;
}

constexpr int XROW_WORDS = NUM_XF + 1;  // ext row: NUM_XF int64 + the mask

__global__ void k_scatter_ext(SoA s, const int64_t* __restrict__ rows, const int32_t* __restrict__ idx, int n,
                             const int32_t* __restrict__ gate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n || (gate && *gate)) return;
  const int64_t i = idx[t];
  const int64_t* r = rows + (int64_t)t * XROW_WORDS;
  for (int f = 0; f < NUM_XF; f++) s.xf[f * s.stride + i] = r[f];
  s.xm[i] = (uint64_t)r[NUM_XF];
}

static int ensure_ext(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (d->ext_alloc || !ctx->ext_enabled) return KE_OK;
  HIP_OK(hipMalloc(&d->soa.xf, sizeof(int64_t) * NUM_XF * d->capacity));
  HIP_OK(hipMalloc(&d->soa.xm, sizeof(uint64_t) * d->capacity));
  HIP_OK(hipMemsetAsync(d->soa.xf, 0, sizeof(int64_t) * NUM_XF * d->capacity, d->stream));
  HIP_OK(hipMemsetAsync(d->soa.xm, 0, sizeof(uint64_t) * d->capacity, d->stream));
  d->ext_alloc = true;
  for (int32_t i = 0; i < ctx->n_nodes; i++) ctx->nodes[i].dirty = true;
  return KE_OK;
}

constexpr int CPU_ROW_WORDS = CPU_SLOTS + NUM_CS_FIELDS;  // records (one int64 each) + summary

__global__ void k_scatter_cpu(SoA s, const int64_t* __restrict__ rows, const int32_t* __restrict__ idx, int n,
                              const int32_t* __restrict__ gate) {
  const int t = blockIdx.x;
  if (t >= n || (gate && *gate)) return;
  const int64_t i = idx[t];
  const int64_t* r = rows + (int64_t)t * CPU_ROW_WORDS;
  reinterpret_cast<int64_t*>(s.cpu + i * CPU_SLOTS)[threadIdx.x] = r[threadIdx.x];
  if (threadIdx.x < NUM_CS_FIELDS) s.cs[threadIdx.x * s.stride + i] = r[CPU_SLOTS + threadIdx.x];
}

// The CPU SoA: every node needs its summary words once a cpuset pod is evaluated (the amplified-cpu
// filter of a binding pod reads the node's ratio even without a CPU table).
static int ensure_cpu(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (d->cpu_alloc || !ctx->cpu_enabled) return KE_OK;
  HIP_OK(hipMalloc(&d->soa.cs, sizeof(int64_t) * NUM_CS_FIELDS * d->capacity));
  HIP_OK(hipMalloc(&d->soa.cpu, sizeof(CpuRec) * CPU_SLOTS * d->capacity));
  HIP_OK(hipMemsetAsync(d->soa.cs, 0, sizeof(int64_t) * NUM_CS_FIELDS * d->capacity, d->stream));
  HIP_OK(hipMemsetAsync(d->soa.cpu, 0, sizeof(CpuRec) * CPU_SLOTS * d->capacity, d->stream));
  d->cpu_alloc = true;
  for (int32_t i = 0; i < ctx->n_nodes; i++)
    if (ctx->nodes[i].valid) ctx->nodes[i].dirty = true;
  return KE_OK;
}

// Re-derive rows of dirty / time-expired nodes and scatter them into the SoA.
int device_refresh(Context* ctx, int64_t now, bool defer) {
  DeviceState* d = ctx->dev;
  d->deferred.clear();
  int rc = ensure_ds(ctx);  // (first use marks the nodes dirty: before the checks below)
  if (rc) return rc;
  rc = ensure_numa(ctx);
  if (rc) return rc;
  rc = ensure_cpu(ctx);
  if (rc) return rc;
  rc = ensure_ext(ctx);
  if (rc) return rc;
  // nothing marked dirty since every row was last clean, and no row expired: no scan over the nodes; no row
  // expired and the same nodes: only the dirty list (the nodes marked since)
  const bool no_expiry = now < ctx->min_valid_until && ctx->n_nodes == ctx->clean_n_nodes;
  const bool all_clean = no_expiry && g_dirty_epoch.load(std::memory_order_relaxed) == ctx->clean_epoch;
  const bool incremental = !all_clean && no_expiry;
  if (!all_clean) mirror_join(*ctx);  // a row may be derived: the host mirror on its thread first
  if (!all_clean && !ctx->pending.empty()) {  // a row to derive needs the deferred host mirror first
    bool any = false;
    if (incremental)
      for (int32_t i : ctx->dirty_list) any = any || (i < ctx->n_nodes && ctx->nodes[i].dirty);
    else
      for (int32_t i = 0; i < ctx->n_nodes && !any; i++) any = ctx->nodes[i].dirty || now >= ctx->nodes[i].valid_until;
    if (any) flush_mirror(*ctx);
  }
  if (ctx->ptab_dirty) {  // GPU partition tables (ke_node_gpu_partitions); the pool only grows
    if (d->pt_words < ctx->ptab.size()) {
      if (d->soa.pt) HIP_OK(hipFree(d->soa.pt));
      const size_t cap = std::max(ctx->ptab.size(), (size_t)16 * PT_WORDS);
      HIP_OK(hipMalloc(&d->soa.pt, sizeof(uint64_t) * cap));
      d->pt_words = cap;
    }
    HIP_OK(hipMemcpyAsync(d->soa.pt, ctx->ptab.data(), sizeof(uint64_t) * ctx->ptab.size(), hipMemcpyHostToDevice,
                          d->stream));
    HIP_OK(hipStreamSynchronize(d->stream));
    ctx->ptab_dirty = false;
  }
  std::vector<int64_t> crows;  // CPU tables + summaries of the dirty nodes
  std::vector<int32_t> cidx;
  std::vector<Row> rows;
  std::vector<int32_t> idx;
  std::vector<int64_t> dsrows;  // DeviceShare rows of the dirty nodes (the device state is not time-dependent)
  std::vector<int32_t> dsidx;
  std::vector<int64_t> nrows;  // NUMA rows of the dirty nodes
  std::vector<int32_t> nidx;
  std::vector<int64_t> xrows;  // ext rows of the dirty nodes
  std::vector<int32_t> xidx;
  int64_t mvu = incremental ? ctx->min_valid_until : INT64_MAX;
  std::vector<int32_t> visit;
  if (incremental) {
    visit.swap(ctx->dirty_list);  // (flush_mirror above may have appended; a repeated node is clean the 2nd time)
  }
  const int32_t n_visit = all_clean ? 0 : incremental ? (int32_t)visit.size() : ctx->n_nodes;
  for (int32_t v = 0; v < n_visit; v++) {
    const int32_t i = incremental ? visit[(size_t)v] : v;
    if (i >= ctx->n_nodes) continue;
    NodeState& ns = ctx->nodes[i];
    if (!ns.dirty && now < ns.valid_until) {
      mvu = std::min(mvu, ns.valid_until);
      continue;
    }
    Row r;
    int64_t vu;
    derive_row(ctx->cfg, ns, now, &r, &vu);
    if (ns.dirty && d->ds_alloc) {
      const size_t o = dsrows.size();
      dsrows.resize(o + DS_ROW_WORDS);
      derive_ds_row(ns, &dsrows[o], reinterpret_cast<uint64_t*>(&dsrows[o + NUM_DS_FIELDS]));
      derive_dsx_row(ns, &dsrows[o + NUM_DS_FIELDS + NUM_DS_MASKS]);
      dsidx.push_back(i);
    }
    if (ns.dirty && d->numa_alloc) {
      const size_t o = nrows.size();
      nrows.resize(o + NUMA_ROW_WORDS);
      uint64_t mask;
      derive_numa_row(ns, &nrows[o], &mask);
      nrows[o + NUM_NUMA_FIELDS] = (int64_t)mask;
      nidx.push_back(i);
    }
    if (ns.dirty && d->ext_alloc) {
      const size_t o = xrows.size();
      xrows.resize(o + XROW_WORDS);
      uint64_t mask;
      derive_ext_row(ctx->cfg, ns, &xrows[o], &mask);
      xrows[o + NUM_XF] = (int64_t)mask;
      xidx.push_back(i);
    }
    if (ns.dirty && d->cpu_alloc) {
      const size_t o = crows.size();
      crows.resize(o + CPU_ROW_WORDS);
      derive_cpu_rows(ns, reinterpret_cast<CpuRec*>(&crows[o]), &crows[o + CPU_SLOTS]);
      cidx.push_back(i);
    }
    ns.valid_until = vu;
    ns.dirty = false;
    mvu = std::min(mvu, vu);
    rows.push_back(r);
    idx.push_back(i);
  }
  if (!all_clean) {
    ctx->clean_epoch = g_dirty_epoch.load(std::memory_order_relaxed);
    ctx->min_valid_until = mvu;
    ctx->clean_n_nodes = ctx->n_nodes;
    ctx->dirty_list.clear();  // every node < n_nodes is clean now
  }
  // every table's rows and indices go through one page-locked staging area: async copies and scatters on the
  // stream, one synchronisation at the end (the staging is reused by the next refresh)
  static_assert(sizeof(Row) % sizeof(int64_t) == 0, "Row staged in int64 words");
  auto words = [](size_t bytes) { return (bytes + sizeof(int64_t) - 1) / sizeof(int64_t); };
  const size_t total = dsrows.size() + words(sizeof(int32_t) * dsidx.size()) + nrows.size() +
                       words(sizeof(int32_t) * nidx.size()) + xrows.size() + words(sizeof(int32_t) * xidx.size()) +
                       crows.size() + words(sizeof(int32_t) * cidx.size()) + words(sizeof(Row) * rows.size()) +
                       words(sizeof(int32_t) * idx.size());
  if (total == 0) return KE_OK;
  // the staging of the refresh before the previous one: its copies are done before it is reused (two refreshes in a
  // row -- a fused matched pod's -- do not wait for each other)
  const int cur = d->refresh_cur ^= 1;
  if (d->refresh_pending[cur]) {
    HIP_OK(hipEventSynchronize(d->ev_refresh[cur]));
    d->refresh_pending[cur] = false;
  }
  PinnedVec<int64_t>& hstage = d->h_refresh[cur];
  if (!hstage.resize(total)) return fail(KE_ERR_DEVICE, "hipHostMalloc of the row staging");
  size_t at = 0;
  auto stage = [&](const void* src, size_t bytes) {  // -> the staged copy
    void* dst = hstage.data() + at;
    if (bytes) std::memcpy(dst, src, bytes);
    at += words(bytes);
    return dst;
  };
  // one table: rows (row_words int64 per node) + indices into its device staging buffer, then its scatter
  auto table = [&](int64_t** dbuf, int64_t* cap, const std::vector<int64_t>& hrows, const std::vector<int32_t>& hidx,
                   int64_t row_words, int32_t** didx) -> int {
    const int64_t n = (int64_t)hidx.size();
    if (*cap < n) {
      if (*dbuf) HIP_OK(hipFree(*dbuf));
      HIP_OK(hipMalloc(dbuf, sizeof(int64_t) * row_words * n + sizeof(int32_t) * n));
      *cap = n;
    }
    *didx = reinterpret_cast<int32_t*>(*dbuf + row_words * n);
    HIP_OK(hipMemcpyAsync(*dbuf, stage(hrows.data(), sizeof(int64_t) * hrows.size()), sizeof(int64_t) * hrows.size(),
                          hipMemcpyHostToDevice, d->stream));
    HIP_OK(hipMemcpyAsync(*didx, stage(hidx.data(), sizeof(int32_t) * n), sizeof(int32_t) * n, hipMemcpyHostToDevice,
                          d->stream));
    return KE_OK;
  };
  int32_t* didx = nullptr;
  if (!dsidx.empty()) {
    const int n = (int)dsidx.size();
    rc = table(&d->d_dsrows, &d->ds_staging_cap, dsrows, dsidx, DS_ROW_WORDS, &didx);
    if (rc) return rc;
    const int64_t* rows = d->d_dsrows;
    d->deferred.push_back([=](const int32_t* gate) {
      hipLaunchKernelGGL(k_scatter_ds, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, d->stream, d->soa, rows, didx, n, gate);
    });
  }
  if (!nidx.empty()) {
    const int n = (int)nidx.size();
    rc = table(&d->d_numarows, &d->numa_staging_cap, nrows, nidx, NUMA_ROW_WORDS, &didx);
    if (rc) return rc;
    const int64_t* rows = d->d_numarows;
    d->deferred.push_back([=](const int32_t* gate) {
      hipLaunchKernelGGL(k_scatter_numa, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, d->stream, d->soa, rows, didx, n, gate);
    });
  }
  if (!xidx.empty()) {
    const int n = (int)xidx.size();
    rc = table(&d->d_xrows, &d->ext_staging_cap, xrows, xidx, XROW_WORDS, &didx);
    if (rc) return rc;
    const int64_t* rows = d->d_xrows;
    d->deferred.push_back([=](const int32_t* gate) {
      hipLaunchKernelGGL(k_scatter_ext, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, d->stream, d->soa, rows, didx, n, gate);
    });
  }
  if (!cidx.empty()) {
    const int n = (int)cidx.size();
    rc = table(&d->d_cpurows, &d->cpu_staging_cap, crows, cidx, CPU_ROW_WORDS, &didx);
    if (rc) return rc;
    const int64_t* rows = d->d_cpurows;
    d->deferred.push_back([=](const int32_t* gate) {
      hipLaunchKernelGGL(k_scatter_cpu, dim3((unsigned)n), dim3(CPU_SLOTS), 0, d->stream, d->soa, rows, didx, n, gate);
    });
  }
  if (!rows.empty()) {
    HIP_OK(hipSetDevice(d->device));
    const int64_t n = (int64_t)rows.size();
    if (d->staging_cap < n) {
      if (d->d_rows) HIP_OK(hipFree(d->d_rows));
      if (d->d_idx) HIP_OK(hipFree(d->d_idx));
      HIP_OK(hipMalloc(&d->d_rows, sizeof(Row) * n));
      HIP_OK(hipMalloc(&d->d_idx, sizeof(int32_t) * n));
      d->staging_cap = n;
    }
    HIP_OK(hipMemcpyAsync(d->d_rows, stage(rows.data(), sizeof(Row) * n), sizeof(Row) * n, hipMemcpyHostToDevice,
                          d->stream));
    HIP_OK(hipMemcpyAsync(d->d_idx, stage(idx.data(), sizeof(int32_t) * n), sizeof(int32_t) * n, hipMemcpyHostToDevice,
                          d->stream));
    const Row* rows_d = d->d_rows;
    const int32_t* idx_d = d->d_idx;
    const KArgs ka = make_kargs(ctx, now);
    const int nn = (int)n;
    d->deferred.push_back([=](const int32_t* gate) {
      hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, d->stream, d->soa, rows_d, idx_d,
                         nn, ka, gate);
    });
  }
  // defer (a fused reservation-matched pod): the copies are on the stream, the scatters wait for
  // device_refresh_flush -- behind the segment's plain pods, gated by their k_rsv_check
  if (defer) return KE_OK;
  return device_refresh_flush(ctx, nullptr);
}

int device_refresh_flush(Context* ctx, const int32_t* gate) {
  DeviceState* d = ctx->dev;
  if (d->deferred.empty()) return KE_OK;
  for (auto& f : d->deferred) f(gate);
  d->deferred.clear();
  HIP_OK(hipGetLastError());
  // no host wait: the staging is reused only after ev_refresh (above), and the kernels reading the rows run on
  // `stream` after the scatters or wait for an event recorded there after them (device_schedule_enqueue's ev_start)
  if (d->refresh_sync) {
    HIP_OK(hipStreamSynchronize(d->stream));
  } else {
    HIP_OK(hipEventRecord(d->ev_refresh[d->refresh_cur], d->stream));
    d->refresh_pending[d->refresh_cur] = true;
  }
  return KE_OK;
}

static int upload_pods(Context* ctx, int32_t n_pods, const ke_pod* pods, hipStream_t ustream = nullptr) {
  DeviceState* d = ctx->dev;
  if (!ustream) ustream = d->stream;
  PinnedVec<DevPod>& dp = d->host_pods;
  if (!dp.resize((size_t)n_pods)) return fail(KE_ERR_DEVICE, "hipHostMalloc of the pod staging buffer");
  std::vector<DevPodHint>& ph = d->host_ph;  // the hinted pods' records; DevPod::ring_bw = slot
  ph.clear();
  // the argument checks of this call staged the records (check_cpuset); pods may be a segment of them
  const bool staged = ctx->staged_src && pods >= ctx->staged_src &&
                      pods + n_pods <= ctx->staged_src + (int64_t)ctx->staged.size();
  const DevPod* st = staged ? ctx->staged.data() + (pods - ctx->staged_src) : nullptr;
  for (int32_t p = 0; p < n_pods; p++) {
    const ke_pod_device_hints* h = pod_hints(*ctx, pods[p]);
    dp[p] = st ? st[p] : make_dev_pod(ctx->cfg, pods[p], h, &ctx->tmpl);
    if (ctx->n_bind_nodes > 0 && dp[p].req[0] > 0) dp[p].flags |= PF_CPUSET;  // a node policy may bind it
    if (dp[p].flags & PF_DS_HINT) {  // hints, or a pod allocated by GPU shared resource template
      static const ke_pod_device_hints none{};
      ph.push_back(make_pod_hint(*ctx, pods[p], dp[p], h ? *h : none));
      dp[p].ring_bw = (int64_t)ph.size() - 1;
    }
  }
  int rc = ensure((void**)&d->d_pods, &d->pods_cap, sizeof(DevPod) * (int64_t)std::max(n_pods, 1));
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(d->d_pods, dp.data(), sizeof(DevPod) * n_pods, hipMemcpyHostToDevice, ustream));
  if (!ph.empty()) {
    rc = ensure((void**)&d->d_ph, &d->ph_cap, sizeof(DevPodHint) * (int64_t)ph.size());
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(d->d_ph, ph.data(), sizeof(DevPodHint) * ph.size(), hipMemcpyHostToDevice, ustream));
  }
  d->soa.ph = d->d_ph;
  // no host wait: the kernels run on d->stream after the copies, and the eval stream waits for ev_start,
  // recorded on d->stream after them; dp / ph stay untouched until the call's final synchronisation
  return KE_OK;
}

int device_eval(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, uint8_t* status, uint8_t* reason,
                int16_t* la, int16_t* numa, int16_t* ds, int16_t* total, int32_t* best) {
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  int rc = device_refresh(ctx, now);
  if (rc) return rc;
  if (n_pods == 0) return KE_OK;
  rc = upload_pods(ctx, n_pods, pods);
  if (rc) return rc;
  const int64_t N = ctx->n_nodes, P = n_pods, M = N * P;
  // parity buffers: status u8, reason u8, la / numa / ds / total i16 = 10 B per pair
  rc = ensure(&d->d_parity, &d->parity_cap, std::max<int64_t>(M, 1) * 10 + 16);
  if (rc) return rc;
  rc = ensure((void**)&d->d_best, &d->best_cap, sizeof(uint32_t) * 2 * P);  // best key + dsmax per pod
  if (rc) return rc;
  uint8_t* d_status = (uint8_t*)d->d_parity;
  uint8_t* d_reason = d_status + M;
  int16_t* d_la = (int16_t*)(d_reason + M + (M & 1));
  int16_t* d_numa = d_la + M;
  int16_t* d_ds = d_numa + M;
  int16_t* d_total = d_ds + M;
  uint32_t* d_dsmax = d->d_best + P;
  HIP_OK(hipMemsetAsync(d->d_best, 0, sizeof(uint32_t) * 2 * P, d->stream));
  HIP_OK(hipMemsetAsync(d->soa.kerr, 0, sizeof(int32_t), d->stream));
  const KArgs k = make_kargs(ctx, now);
  const int ppb = EVAL_PPB;
  bool cpu = false;
  for (const DevPod& q : d->host_pods) cpu = cpu || (q.flags & PF_CPUSET);
  if (cpu && !d->cpu_alloc) return fail(KE_ERR_DEVICE, "cpuset pod without the CPU SoA");
  if (N > 0) {
    dim3 grid((unsigned)((N + EVAL_BLOCK - 1) / EVAL_BLOCK), (unsigned)((P + ppb - 1) / ppb));
    if (d->numa_alloc) {
      rc = ensure((void**)&d->d_defer, &d->defer_cap, (sizeof(uint64_t) + sizeof(uint32_t)) * M);  // pairs, merges
      if (rc) return rc;
      rc = ensure((void**)&d->d_defer_cnt, &d->defer_cnt_cap, sizeof(uint32_t));
      if (rc) return rc;
      HIP_OK(hipMemsetAsync(d->d_defer_cnt, 0, sizeof(uint32_t), d->stream));
      hipLaunchKernelGGL((cpu ? k_eval_parity<true, true> : k_eval_parity<true, false>), grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, (int)N, d->d_pods, (int)P,
                         ppb, k, d_status, d_reason, d_la, d_numa, d_ds, d_total, d_dsmax, d->d_defer, d->d_defer_cnt);
      HIP_OK(hipGetLastError());
      uint32_t* fb = reinterpret_cast<uint32_t*>(d->d_defer + M);
      hipLaunchKernelGGL((cpu ? k_numa_fallback<true, true> : k_numa_fallback<true, false>), dim3(FALLBACK_BLOCKS),
                         dim3(64), 0, d->stream, d->soa, d->d_pods,
                         d->d_batch_base, k, d->d_defer, d->d_defer_cnt, d->d_scores, d->capacity, (int)N, d_status,
                         d_reason, d_la, d_numa, d_ds, d_total, d_dsmax, nullptr, nullptr, fb);
      hipLaunchKernelGGL((cpu ? k_numa_finish<true, true> : k_numa_finish<true, false>), dim3(FINISH_BLOCKS),
                         dim3(64), 0, d->stream, d->soa, d->d_pods,
                         d->d_batch_base, k, d->d_defer, d->d_defer_cnt, d->d_scores, d->capacity, (int)N, d_status,
                         d_reason, d_la, d_numa, d_ds, d_total, d_dsmax, nullptr, nullptr, fb);
    } else {
      hipLaunchKernelGGL((cpu ? k_eval_parity<false, true> : k_eval_parity<false, false>), grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, (int)N, d->d_pods, (int)P,
                         ppb, k, d_status, d_reason, d_la, d_numa, d_ds, d_total, d_dsmax, nullptr, nullptr);
    }
    HIP_OK(hipGetLastError());
    dim3 grid2((unsigned)((N + EVAL_BLOCK - 1) / EVAL_BLOCK), (unsigned)P);
    hipLaunchKernelGGL(k_parity_finalize, grid2, dim3(EVAL_BLOCK), 0, d->stream, (int)N, k, d_ds, d_total, d_dsmax,
                       d->d_best);
    HIP_OK(hipGetLastError());
  }
  if (status) HIP_OK(hipMemcpyAsync(status, d_status, M, hipMemcpyDeviceToHost, d->stream));
  if (reason) HIP_OK(hipMemcpyAsync(reason, d_reason, M, hipMemcpyDeviceToHost, d->stream));
  if (la) HIP_OK(hipMemcpyAsync(la, d_la, M * 2, hipMemcpyDeviceToHost, d->stream));
  if (numa) HIP_OK(hipMemcpyAsync(numa, d_numa, M * 2, hipMemcpyDeviceToHost, d->stream));
  if (ds) HIP_OK(hipMemcpyAsync(ds, d_ds, M * 2, hipMemcpyDeviceToHost, d->stream));
  if (total) HIP_OK(hipMemcpyAsync(total, d_total, M * 2, hipMemcpyDeviceToHost, d->stream));
  std::vector<uint32_t> bk((size_t)P);
  HIP_OK(hipMemcpyAsync(bk.data(), d->d_best, sizeof(uint32_t) * P, hipMemcpyDeviceToHost, d->stream));
  uint32_t deferred = 0;
  if (d->numa_alloc && N > 0)
    HIP_OK(hipMemcpyAsync(&deferred, d->d_defer_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, d->stream));
  int32_t kerr = 0;
  HIP_OK(hipMemcpyAsync(&kerr, d->soa.kerr, sizeof(int32_t), hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  if (kerr & KERR_HINT_ROUTE) return fail(KE_ERR_DEVICE, "internal: a hinted pod reached a kernel without the hint path");
  ctx->kstat_numa_deferred = deferred;
  if (best)
    for (int64_t p = 0; p < P; p++) best[p] = bk[p] ? key_node(bk[p]) + ctx->cfg.global_node_offset : -1;
  return KE_OK;
}

// The other call's buffers become this context's (ke_schedule_submit with a call in flight; host_pods, the pods,
// outputs, stamps, hand-off words, readback staging and events are per call).
void device_swap_call_buffers(Context* ctx) {
  DeviceState* d = ctx->dev;
  DeviceState::CallBufs& a = d->alt;
  d->host_pods.swap(a.host_pods);
  std::swap(d->d_pods, a.d_pods);
  std::swap(d->pods_cap, a.pods_cap);
  std::swap(d->d_chosen, a.d_chosen);
  std::swap(d->d_chosen_score, a.d_chosen_score);
  std::swap(d->d_stamps, a.d_stamps);
  std::swap(d->d_devalloc, a.d_devalloc);
  std::swap(d->d_numaalloc, a.d_numaalloc);
  std::swap(d->out_cap, a.out_cap);
  std::swap(d->d_cpusets, a.d_cpusets);
  std::swap(d->cpusets_cap, a.cpusets_cap);
  std::swap(d->d_sched, a.d_sched);
  std::swap(d->sched_cap, a.sched_cap);
  d->h_out.swap(a.h_out);
  d->tev.swap(a.tev);
}

// a failed enqueue may have left part of its launches on the streams: wait for every stream of the context
void device_quiesce(Context* ctx) {
  DeviceState* d = ctx->dev;
  if (!d) return;
  (void)hipSetDevice(d->device);
  (void)hipDeviceSynchronize();
}

// whether the next call's device_refresh would upload rows (derived from the host state, which lacks the Reserves
// of a call still in flight) or change a device table
bool device_refresh_pending(const Context* ctx, int64_t now) {
  if (ctx->ptab_dirty || !(now < ctx->min_valid_until && ctx->n_nodes == ctx->clean_n_nodes)) return true;
  if (g_dirty_epoch.load(std::memory_order_relaxed) == ctx->clean_epoch) return false;
  for (int32_t i : ctx->dirty_list)  // (the incremental refresh visits these; a clean one derives nothing)
    if (i < ctx->n_nodes && ctx->nodes[(size_t)i].dirty) return true;
  return false;
}

// a plain queue (no DeviceShare / cpuset / hinted pod, no NUMA or quota state, unsharded, pipelined) runs without a
// host round trip between its launches: it may be submitted behind a call in flight
bool device_async_ok(const Context* ctx, int32_t n_pods) {
  const DeviceState* d = ctx->dev;
  if (!d || d->world > 1 || d->comm || d->host_fn || !d->pipeline || d->numa_alloc || !ctx->quotas.empty() || ctx->n_nodes <= 0)
    return false;
  if (ctx->n_bind_nodes > 0 || !ctx->rsv_pairs.empty() || ctx->rsv_affinity || !ctx->rsv_ovr.empty()) return false;
  if ((int64_t)ctx->staged.size() != n_pods) return false;
  for (const DevPod& q : ctx->staged)
    if (q.flags & (PF_DS | PF_CPUSET | PF_DS_HINT)) return false;
  return true;
}

int device_schedule(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, int32_t* chosen, int32_t* score) {
  DevFinish fin;
  const int rc = device_schedule_enqueue(ctx, n_pods, pods, now, score != nullptr, &fin);
  if (rc || !fin) return rc;
  return fin(chosen, score);
}

int device_schedule_enqueue(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, bool want_score,
                            DevFinish* fin) {
  DeviceState* d = ctx->dev;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  auto tp = clk::now();
  HIP_OK(hipSetDevice(d->device));
  const bool fused = ctx->rsv_fused;  // the last pod: a matched pod behind plain ones (its rows' scatters deferred)
  int rc = device_refresh(ctx, now, fused);
  if (rc) return rc;
  ctx->host_ms[1] = ms_since(tp);
  ctx->last_batch_ms.clear();
  ctx->last_dev_alloc.clear();
  ctx->last_total_ms = 0;
  ctx->last_pod_lat.clear();
  if (n_pods == 0) return KE_OK;
  tp = clk::now();
  hipStream_t const cs = d->cstream ? d->cstream : d->stream;  // the call's staging stream
  rc = upload_pods(ctx, n_pods, pods, cs);
  if (rc) return rc;
  ctx->host_ms[2] = ms_since(tp);
  tp = clk::now();
  // Batches: runs of up to B pods without DeviceShare requests (exact speculative batching, DESIGN.md
  // §4), and every DeviceShare pod alone: its NormalizeScore needs the max over all feasible nodes of
  // the current state.
  // A pod that may bind CPUs is alone in its batch too: its Reserve runs the CPU accumulator
  // (k_cpuset_reserve) and may fail, and later pods read the CPU table it patches.
  const int B = ctx->cfg.pod_batch;
  struct Batch {
    int pods;
    bool ds, cpu;  // DeviceShare-capable batch (its pods' NormalizeScore) / singleton of a pod that may bind CPUs
    bool cut;      // a DeviceShare batch with DeviceShare pods: the replay may stop early
    bool hint;     // singleton of a pod with device hints: its eval kernel carries the hint path (H)
  };
  std::vector<Batch> batches;
  // DeviceShare pods share batches (exact: the replay checks each pod's normalisation max and stops the
  // batch where it may have moved) unless the nodes are sharded or carry NUMA policies (then
  // each is a singleton batch)
  const bool ds_batch = !(d->world > 1 || d->comm || d->host_fn) && !d->numa_alloc && ctx->n_nodes > 0;
  ctx->last_ds_cuts = 0;
  for (int32_t p = 0; p < n_pods;) {
    const uint32_t f = d->host_pods[p].flags;
    if ((f & PF_CPUSET) || ((f & PF_DS) && !ds_batch) || (f & PF_DS_HINT) || (fused && p == n_pods - 1)) {
      // hinted pods and a fused matched pod: singletons
      batches.push_back({1, (f & PF_DS) != 0, (f & PF_CPUSET) != 0, false, (f & PF_DS_HINT) != 0});
      p++;
      continue;
    }
    int bp = 0;
    bool has_ds = false, ds_pods = false;
    while (p + bp < n_pods && bp < B && !(fused && p + bp == n_pods - 1)) {
      const uint32_t g = d->host_pods[p + bp].flags;
      if ((g & PF_CPUSET) || ((g & PF_DS) && !ds_batch) || (g & PF_DS_HINT)) break;
      has_ds = has_ds || (g & PF_DS);
      ds_pods = ds_pods || (g & PF_DS);
      bp++;
    }
    batches.push_back({bp, has_ds, false, ds_pods && bp > 1, false});
    p += bp;
  }
  bool any_cpu = false;
  for (const Batch& b : batches) any_cpu = any_cpu || b.cpu;
  if (any_cpu && !d->cpu_alloc) return fail(KE_ERR_DEVICE, "cpuset pod without the CPU SoA");
  const int n_batches = (int)batches.size();
  const int64_t out_bytes = sizeof(int32_t) * (int64_t)n_pods;
  if (d->out_cap < n_pods) {
    if (d->d_chosen) HIP_OK(hipFree(d->d_chosen));
    if (d->d_chosen_score) HIP_OK(hipFree(d->d_chosen_score));
    if (d->d_stamps) HIP_OK(hipFree(d->d_stamps));
    if (d->d_devalloc) HIP_OK(hipFree(d->d_devalloc));
    if (d->d_numaalloc) HIP_OK(hipFree(d->d_numaalloc));
    d->d_numaalloc = nullptr;
    HIP_OK(hipMalloc(&d->d_chosen, out_bytes));
    HIP_OK(hipMalloc(&d->d_chosen_score, out_bytes));
    HIP_OK(hipMalloc(&d->d_stamps, sizeof(uint64_t) * (PST + 2) * ((int64_t)n_pods + 2)));
    HIP_OK(hipMalloc(&d->d_devalloc, sizeof(uint64_t) * n_pods));
    d->out_cap = n_pods;
  }
  rc = ensure((void**)&d->d_cpusets, &d->cpusets_cap, sizeof(uint64_t) * 4 * (int64_t)n_pods);
  if (rc) return rc;
  HIP_OK(hipMemsetAsync(d->d_cpusets, 0, sizeof(uint64_t) * 4 * n_pods, cs));
  bool any_hint = false;
  for (const DevPod& q : d->host_pods) any_hint = any_hint || (q.flags & PF_DS_HINT);
  d->soa.vfo = nullptr;
  if (any_hint) {  // the VF ranks the hinted pods' Reserves take
    rc = ensure((void**)&d->d_vfo, &d->vfo_cap, 2 * DS_MINORS * (int64_t)n_pods);
    if (rc) return rc;
    HIP_OK(hipMemsetAsync(d->d_vfo, 0xFF, 2 * DS_MINORS * (size_t)n_pods, d->stream));
    d->soa.vfo = d->d_vfo;
  }
  const bool numa = d->numa_alloc;
  if (numa && !d->d_numaalloc) HIP_OK(hipMalloc(&d->d_numaalloc, sizeof(int64_t) * 16 * d->out_cap));
  if (numa) {  // deferred-pair list of one batch (reused) + a counter per batch
    rc = ensure((void**)&d->d_defer, &d->defer_cap, (sizeof(uint64_t) + sizeof(uint32_t)) * MAX_BATCH * d->capacity);
    if (rc) return rc;
    rc = ensure((void**)&d->d_defer_cnt, &d->defer_cnt_cap, sizeof(uint32_t) * n_batches);
    if (rc) return rc;
    HIP_OK(hipMemsetAsync(d->d_defer_cnt, 0, sizeof(uint32_t) * n_batches, d->stream));
  }
  KArgs k = make_kargs(ctx, now);
  if (ctx->rsv_affinity) k.flags |= AF_RSV_ONLY;  // the Reservation Filter: RsvOvr.rfilter of the pod's nodes
  if (!ctx->rsv_pairs.empty() || ctx->rsv_affinity) {  // one matched pod (ke_schedule's segment of its own)
    if (n_pods != 1 && !fused) return fail(KE_ERR_UNSUPPORTED, "matched reservations need a singleton segment");
    for (const RsvPair& q : ctx->rsv_pairs)
      if (q.node < 0 || q.node >= ctx->n_nodes) return fail(KE_ERR_DEVICE, "reservation pair node out of range");
    rc = ensure((void**)&d->d_rsv, &d->rsv_cap, (int64_t)sizeof(RsvPair) * (int64_t)ctx->rsv_pairs.size());
    if (rc) return rc;
  }
  if (fused || !ctx->rsv_pairs.empty() || ctx->rsv_affinity) {
    if (!d->h_rsv_out.resize(5)) return fail(KE_ERR_DEVICE, "hipHostMalloc of the reservation staging");
    for (int i = 0; i < 4; i++) d->h_rsv_out[i] = -1;
    d->h_rsv_out[4] = 0;  // the fused pod's gate (k_rsv_check)
  }
  if (fused && !d->d_rsv_gate) HIP_OK(hipMalloc(&d->d_rsv_gate, sizeof(int32_t)));
  // the matched pod's pairs and allocate-from-reservation decisions, staged page-locked (the previous call's copies
  // from this buffer completed with that call)
  const size_t rsv_bytes = sizeof(RsvPair) * ctx->rsv_pairs.size(), ovr_bytes = sizeof(RsvOvr) * ctx->rsv_ovr.size();
  if (rsv_bytes + ovr_bytes && !d->h_rsv.resize(rsv_bytes + ovr_bytes))
    return fail(KE_ERR_DEVICE, "hipHostMalloc of the reservation staging");
  if (!ctx->rsv_pairs.empty() || ctx->rsv_affinity) {
    if (rsv_bytes) {
      std::memcpy(d->h_rsv.data(), ctx->rsv_pairs.data(), rsv_bytes);
      HIP_OK(hipMemcpyAsync(d->d_rsv, d->h_rsv.data(), rsv_bytes, hipMemcpyHostToDevice, d->stream));
    }
    HIP_OK(hipMemsetAsync(d->d_rsv_out, 0xFF, sizeof(int32_t) * 4, d->stream));
  }
  d->soa.n_rovr = 0;  // a matched pod's allocate-from-reservation decisions (NF_RSV_CS rows read them)
  if (!ctx->rsv_ovr.empty()) {
    rc = ensure((void**)&d->d_rovr, &d->rovr_cap, (int64_t)sizeof(RsvOvr) * (int64_t)ctx->rsv_ovr.size());
    if (rc) return rc;
    std::memcpy(d->h_rsv.data() + rsv_bytes, ctx->rsv_ovr.data(), ovr_bytes);
    HIP_OK(hipMemcpyAsync(d->d_rovr, d->h_rsv.data() + rsv_bytes, ovr_bytes, hipMemcpyHostToDevice, d->stream));
    d->soa.rovr = d->d_rovr;
    d->soa.n_rovr = (int32_t)ctx->rsv_ovr.size();
  }
  const bool quota = !ctx->quotas.empty();  // ElasticQuota admission + Reserve in the Reserve kernels
  if (quota) {
    if (ctx->quota_dirty) {
      rc = device_quota_upload(ctx);
      if (rc) return rc;
    }
    k.flags |= AF_QUOTA | (ctx->qargs.enable_check_parent_quota ? AF_QUOTA_PARENT : 0u);
  }
  const int N = ctx->n_nodes;
  const int ppb = EVAL_PPB;
  // first pod of every batch and the end (the kernels' batch base pointer is d_bases + b)
  std::vector<int32_t> bases((size_t)n_batches + 1);
  for (int b = 0, p = 0; b <= n_batches; b++) {
    bases[b] = p;
    if (b < n_batches) p += batches[b].pods;
  }
  // pipelined runs: maximal stretches of plain batches (no DeviceShare / cpuset pod) in a
  // context without NUMA policies; run_end[b] > 0 marks the first batch of a run and holds its end
  // (a lone plain batch between singletons gains nothing from the second stream: it runs serially)
  auto eligible = [&](int b) {
    return d->pipeline && N > 0 && !numa && !batches[b].ds && !batches[b].cpu && !(fused && b == n_batches - 1);
  };
  std::vector<int> run_end((size_t)n_batches, 0);
  for (int b = 0; b < n_batches;) {
    if (!eligible(b)) {
      b++;
      continue;
    }
    int e = b;
    while (e < n_batches && eligible(e)) e++;
    if (e - b >= 2) run_end[b] = e;
    b = e;
  }
  // device: bases [n+1], ready [n], done [n], error word, T-helper counts [n], select-started counts [n], the
  // Reserve kernels' residency flags [n] (by run start); fixup stamps [2n]; the T helpers' lists and maxima (THelp)
  const int64_t sched_words = 6 * ((int64_t)n_batches + 1) + 1;
  constexpr int64_t THELP_WORDS = 2 * (1 + MAX_BATCH) + 2 * MAX_BATCH;
  rc = ensure((void**)&d->d_sched, &d->sched_cap,
              sizeof(int32_t) * sched_words + sizeof(uint64_t) * 2 * n_batches + 8 + sizeof(int32_t) * THELP_WORDS);
  if (rc) return rc;
  int32_t* d_bases = d->d_sched;
  int32_t* d_ready = d_bases + n_batches + 1;
  int32_t* d_done = d_ready + n_batches + 1;
  int32_t* d_err = d_done + n_batches + 1;
  int32_t* d_tready = d_err + 1;
  int32_t* d_sstart = d_tready + n_batches + 1;
  int32_t* d_rres = d_sstart + n_batches + 1;
  uint64_t* d_fst = reinterpret_cast<uint64_t*>(d->d_sched + ((sched_words + 1) & ~1LL));
  int32_t* d_tlist = reinterpret_cast<int32_t*>(d_fst + 2 * n_batches);
  uint32_t* d_tmx = reinterpret_cast<uint32_t*>(d_tlist + 2 * (1 + MAX_BATCH));
  // (the call's own words, on its staging stream; the error word and the split selects' counters stay zero
  // between calls -- an aborted call resets them)
  HIP_OK(hipMemcpyAsync(d_bases, bases.data(), sizeof(int32_t) * (n_batches + 1), hipMemcpyHostToDevice, cs));
  HIP_OK(hipMemsetAsync(d_ready, 0, sizeof(int32_t) * (sched_words - n_batches - 1), cs));
  HIP_OK(hipMemsetAsync(d_fst, 0, sizeof(uint64_t) * 2 * n_batches, cs));
  HIP_OK(hipEventRecord(d->ev_setup, cs));
  // sampled per-kernel HIP event pairs (ke_set_profiling) on the eval stream: eval, select
  constexpr int PE = 4;  // eval start, eval end, select end, select start (after k_patch and its wait)
  const int every = d->profile_every;
  // the call's timing events (the whole span, the samples) come from the context's pool: creating them per call
  // cost the host ~3 us an event
  const size_t n_tev = 5 + (every > 0 ? (size_t)((n_batches + every - 1) / every) * PE : 0);
  while (d->tev.size() < n_tev) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    d->tev.push_back(e);
  }
  hipEvent_t e0 = d->tev[0], e1 = d->tev[1];
  const hipEvent_t done_ev[3] = {d->tev[2], d->tev[3], d->tev[4]};  // the call's end on each stream
  std::vector<hipEvent_t> ev(d->tev.begin() + 5, d->tev.begin() + (long)n_tev);
  HIP_OK(hipStreamWaitEvent(d->stream, d->ev_setup, 0));
  HIP_OK(hipEventRecord(e0, d->stream));
  hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, d->stream, d->d_stamps);
  HIP_OK(hipEventRecord(d->ev_start, d->stream));
  HIP_OK(hipStreamWaitEvent(d->estream, d->ev_start, 0));
  const bool sharded = d->world > 1 || d->comm || d->host_fn;
  uint64_t* estamps = d->d_stamps + (PST + 1) * ((int64_t)n_pods + 2);  // eval start of each batch
  constexpr int R = DeviceState::EV_RING;
  int n_pipelined = 0;
  // Batch b's eval + candidate lists on stream `es`.  pipe: stale top-(k_j + KMAX) lists into the run's
  // stale buffer (k_fixup makes them exact); else the exact top-k_j lists straight into d_cand.
  bool rerun = false;  // the current serial batch is the remainder of a DeviceShare batch that stopped early
  int pre_b = -1;      // a serial batch whose eval + select is already enqueued (behind a DeviceShare cut check)
  // dwait (pipelined, stale lists): the eval first waits for that done flag -- in k_eval_plain itself, else a
  // k_handoff ahead of it; rpub: the select publishes the lists to the running Reserve kernel itself when it
  // can (split or one-workgroup select, unsharded) -- *published tells the caller
  bool published = false;
  auto eval_select = [&](int b, bool pipe, hipStream_t es, const int32_t* dwait = nullptr,
                         int32_t* rpub = nullptr, bool alt = false, const int32_t* pwait = nullptr,
                         const int32_t* ptl = nullptr, int32_t* sstart = nullptr, int32_t dwant = 1,
                         bool pre = false) -> int {
    published = false;
    uint16_t* const scores = alt ? d->d_scores2 : d->d_scores;  // (the second eval stream's buffers)
    uint32_t* const split = alt ? d->d_split2 : d->d_split;
    int32_t* const pdone = d->d_parts_done + (alt ? MAX_BATCH : 0);
    const int bp = batches[b].pods;
    const bool ds = batches[b].ds, cpu = batches[b].cpu;
    const bool prof = every > 0 && b % every == 0;
    hipEvent_t* pe = prof ? &ev[(size_t)(b / every) * PE] : nullptr;
    const int32_t* bbase = d_bases + b;
    const bool argmax1 = !sharded && bp == 1 && !pipe && N > 0;  // selectHost of one pod: a grid-wide argmax
    // this rank's node range (unsharded and loopback: every node)
    int lo = 0, hi = N;
    if (N > 0 && sharded && !d->loopback) shard_range(N, d->rank, d->world, &lo, &hi);
    // a plain batch with nodes to evaluate: k_eval_batch writes the eval-start stamp itself (one launch
    // less on the eval stream); else k_batch_begin — a re-run remainder keeps its batch's first dequeue
    // stamp (latency counts from there)
    const bool fold_begin = !ds && !argmax1 && !rerun && hi > lo;
    if (!fold_begin)
      hipLaunchKernelGGL(k_batch_begin, dim3(1), dim3(MAX_BATCH), 0, es, estamps + (rerun ? n_pods + 1 : b), ds ? d->d_dsmax : nullptr,
                         argmax1 ? d->d_cand : nullptr);
    // (with two eval streams the wait is a one-wave kernel ahead of the eval, outside its timing: an eval grid
    // spinning on the flag would hold the CUs the other stream's select needs)
    const bool plain_rec = !cpu && !ds && !numa && use_record_eval(bp);
    const bool wait_kernel = dwait && (!plain_rec || alt || (d->estream2 != nullptr && !sharded) || hi <= lo);
    if (wait_kernel) hipLaunchKernelGGL(k_handoff, dim3(1), dim3(64), d->excl_lds, es, nullptr, 0, dwait, d_err, nullptr, dwant);
    if (prof) HIP_OK(hipEventRecord(pe[0], es));
    // (select-ahead: top-(k_j + 2 KMAX) into the pre-fix buffer, k_fixlist makes the Reserve kernel's lists)
    const int L = pre ? KSTALE2 : pipe ? KSTALE : KMAX, kext = pre ? 2 * KMAX : pipe ? KMAX : 0;
    uint32_t* lists = pre ? d->d_pre + (size_t)(b & 1) * MAX_BATCH * KSTALE2
                          : pipe ? d->d_stale + (size_t)(b & 1) * MAX_BATCH * KSTALE : d->d_cand;
    int32_t* lists_cnt = pre ? reinterpret_cast<int32_t*>(d->d_pre + (size_t)2 * MAX_BATCH * KSTALE2) + (b & 1) * MAX_BATCH
                             : pipe ? d->d_stale_cnt + (b & 1) * MAX_BATCH : d->d_cand_cnt;
    if (N > 0) {
      const bool single = bp == 1;
      if (hi > lo) {
        // a singleton batch has one pod's worth of lanes: single-wave blocks spread it over every CU
        const int eb = single ? 64 : EVAL_BLOCK;
        const dim3 grid = eval_grid(hi - lo, eb, bp, ppb);
        auto eval = (ds && batches[b].hint)
                        ? (cpu ? (numa ? k_eval_batch<true, true, true, false, true> : k_eval_batch<true, false, true, false, true>)
                               : (numa ? k_eval_batch<true, true, false, false, true> : k_eval_batch<true, false, false, false, true>))
                  : cpu ? (ds ? (numa ? k_eval_batch<true, true, true> : k_eval_batch<true, false, true>)
                              : (numa ? k_eval_batch<false, true, true> : k_eval_batch<false, false, true>))
                        : ds ? (numa ? k_eval_batch<true, true, false> : k_eval_batch<true, false, false>)
                             : (numa ? k_eval_batch<false, true, false>
                                     : ((k.flags & AF_EXT) ? k_eval_batch<false, false, false, true>
                                                           : k_eval_batch<false, false, false>));
        uint32_t* dcnt = numa ? d->d_defer_cnt + b : nullptr;
        if (plain_rec)  // plain batch: the record-based evaluation
          hipLaunchKernelGGL(((k.flags & AF_EXT) ? k_eval_plain<true> : k_eval_plain<false>), grid, dim3(eb), 0, es, d->soa,
                             lo, hi, d->d_pods, bbase, bp, k, scores, d->capacity, fold_begin ? estamps + b : nullptr,
                             wait_kernel ? nullptr : dwait, d_err);
        else
          hipLaunchKernelGGL(eval, grid, dim3(eb), 0, es, d->soa, lo, hi, d->d_pods, bbase, bp,
                             ppb, k, scores, d->capacity, d->d_dsraw, d->d_defer, dcnt, d->d_aff, d->d_dsmax,
                             fold_begin ? estamps + b : nullptr);
        if (numa) {  // a DeviceShare pod defers only on nodes without a device cache (no DeviceShare hints there)
          uint32_t* fb = reinterpret_cast<uint32_t*>(d->d_defer + (int64_t)MAX_BATCH * d->capacity);
          hipLaunchKernelGGL((cpu ? k_numa_fallback<false, true> : k_numa_fallback<false, false>), dim3(FALLBACK_BLOCKS),
                             dim3(64), 0, es, d->soa, d->d_pods,
                             bbase, k, d->d_defer, dcnt, scores, d->capacity, 0, nullptr, nullptr,
                             nullptr, nullptr, nullptr, nullptr, ds ? d->d_dsmax : nullptr, cpu ? d->d_aff : nullptr,
                             ds ? d->d_dsraw : nullptr, fb);
          hipLaunchKernelGGL((cpu ? k_numa_finish<false, true> : k_numa_finish<false, false>), dim3(FINISH_BLOCKS),
                             dim3(64), 0, es, d->soa, d->d_pods,
                             bbase, k, d->d_defer, dcnt, scores, d->capacity, 0, nullptr, nullptr,
                             nullptr, nullptr, nullptr, nullptr, ds ? d->d_dsmax : nullptr, cpu ? d->d_aff : nullptr,
                             ds ? d->d_dsraw : nullptr, fb);
        }
      }
      if (prof) HIP_OK(hipEventRecord(pe[1], es));
      // a plain batch over many nodes: its pods' selections split over several workgroups each (>= 256
      // workgroups in all, parts of >= 4096 nodes), merged by k_merge
      const int parts = ds ? 1 : select_parts(N, bp, L);
      // the nodes batch b-2 changed, once it is done (k_patch waits for the flag; folding it into the split select
      // was measured slower: 256 select workgroups spinning on the flag)
      if (pwait)
        hipLaunchKernelGGL(((k.flags & AF_EXT) ? k_patch<true> : k_patch<false>), dim3((unsigned)bp), dim3(64), d->excl_lds, es,
                           d->soa, d->d_pods, bbase, k, ptl, scores, d->capacity, pwait, d_err);
      if (ds && sharded && !d->loopback) {  // DefaultNormalizeScore's max over the feasible nodes of all ranks
        const int crc = coll_all_reduce(d, d->d_dsmax, 1, KE_COLL_U32, KE_COLL_MAX, es);
        if (crc) return crc;
      }
      if (prof) HIP_OK(hipEventRecord(pe[3], es));
      auto select = [&](int slo, int shi, uint32_t* cand, int32_t* cnt, int32_t* pub) {
        // register-resident when a wave's segment fits SEL_RC steps, else streamed
        const bool rc = select_seg(slo, shi) <= SEL_RC * 512;
        auto sel = ds ? (rc ? k_select<true, SEL_RC> : k_select<true, 0>) : (rc ? k_select<false, SEL_RC> : k_select<false, 0>);
        hipLaunchKernelGGL(sel, dim3((unsigned)bp), dim3(SELECT_BLOCK), 0, es, scores, d->capacity, slo, shi, cand,
                           cnt, d->d_dsraw, d->d_dsmax, k.wp_ds, kext, L, (int64_t)0, nullptr, nullptr, nullptr, pub, sstart);
      };
      if (argmax1) {  // d_cand[0] zeroed by k_batch_begin
        hipLaunchKernelGGL((ds ? k_argmax1<true> : k_argmax1<false>), dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                           es, scores, 0, N, d->d_dsraw, d->d_dsmax, k.wp_ds, d->d_cand, d->d_cand_cnt);
        if ((!ctx->rsv_pairs.empty() || ctx->rsv_affinity) && (!fused || b == n_batches - 1)) {
          // the pod's matched reservations: the Reservation plugin
          hipLaunchKernelGGL(k_rsv_pick, dim3(1), dim3(64), 0, es, scores, d->d_rsv, (int)ctx->rsv_pairs.size(),
                             (int64_t)ctx->cfg.weight_reservation, (int)ctx->rsv_affinity, d->d_cand, d->d_rsv_out,
                             ds ? d->d_dsraw : nullptr, d->d_dsmax, k.wp_ds);
          HIP_OK(hipMemcpyAsync(d->h_rsv_out.data(), d->d_rsv_out, sizeof(int32_t) * 4, hipMemcpyDeviceToHost, es));
        }
      } else if (!sharded && parts > 1) {
        const int gw = gath_words(L);
        const bool rc = select_seg(0, select_part(0, N, parts)) <= SEL_RC * 512;
        // (select-ahead: no parts_done -- the parts stay sorted in `split` and k_fixlist<PARTS> merges them)
        hipLaunchKernelGGL((rc ? k_select<false, SEL_RC> : k_select<false, 0>), dim3((unsigned)bp, (unsigned)parts),
                           dim3(SELECT_BLOCK), 0, es, scores, d->capacity, 0, (int)N, split,
                           reinterpret_cast<int32_t*>(split + MAX_BATCH * L), d->d_dsraw, d->d_dsmax, k.wp_ds,
                           kext, L, (int64_t)gw, lists, lists_cnt, (pre && d->fix_merge) ? nullptr : pdone, rpub,
                           sstart);  // the last part merges
        published = rpub != nullptr;
      } else if (!sharded) {
        select(0, N, lists, lists_cnt, ds ? nullptr : rpub);
        published = rpub != nullptr && !ds;
      } else {
        // node-sharded: per-shard top-k_j, all-gather, merge
        const int gw = gath_words(L);
        for (int r = 0; r < d->world; r++) {
          if (!d->loopback && r != d->rank) continue;
          int slo, shi;
          shard_range(N, r, d->world, &slo, &shi);
          uint32_t* blk = d->d_gath + (int64_t)r * gw;
          select(slo, shi, blk, reinterpret_cast<int32_t*>(blk + MAX_BATCH * L), nullptr);
        }
        if (!d->loopback) {
          uint32_t* mine = d->d_gath + (int64_t)d->rank * gw;  // in place: send = own block of recv
          const int crc = coll_all_gather(d, mine, d->d_gath, (size_t)gw, es);
          if (crc) return crc;
        }
        hipLaunchKernelGGL(k_merge, dim3((unsigned)bp), dim3(MERGE_BLOCK), 0, es, d->d_gath, d->world, L, kext,
                           lists, lists_cnt);
        if (!ctx->rsv_pairs.empty() || ctx->rsv_affinity) {  // a matched singleton: the Reservation plugin in stages
          int rlo = 0, rhi = N;
          if (!d->loopback) shard_range(N, d->rank, d->world, &rlo, &rhi);
          const int K = (int)ctx->rsv_pairs.size();
          const int64_t wr = (int64_t)ctx->cfg.weight_reservation;
          const int aff = (int)ctx->rsv_affinity;
          RsvPickSt* st = d->d_rsv_st;
          const uint16_t* rds = ds ? d->d_dsraw : nullptr;
          const bool coll = !d->loopback && (d->comm || d->host_fn);
          int crc = 0;
          hipLaunchKernelGGL(k_rsv_stage<0>, dim3(1), dim3(64), 0, es, scores, d->d_rsv, K, rlo, rhi, wr, aff, lists, st, d->d_rsv_out, rds, d->d_dsmax, k.wp_ds);
          if (coll && (crc = coll_all_reduce(d, &st->order, 1, KE_COLL_I64, KE_COLL_MIN, es))) return crc;
          hipLaunchKernelGGL(k_rsv_stage<1>, dim3(1), dim3(64), 0, es, scores, d->d_rsv, K, rlo, rhi, wr, aff, lists, st, d->d_rsv_out, rds, d->d_dsmax, k.wp_ds);
          if (coll && (crc = coll_all_reduce(d, &st->node, 1, KE_COLL_I32, KE_COLL_MIN, es))) return crc;
          hipLaunchKernelGGL(k_rsv_stage<2>, dim3(1), dim3(64), 0, es, scores, d->d_rsv, K, rlo, rhi, wr, aff, lists, st, d->d_rsv_out, rds, d->d_dsmax, k.wp_ds);
          if (coll && (crc = coll_all_reduce(d, &st->mx, 1, KE_COLL_I32, KE_COLL_MAX, es))) return crc;
          hipLaunchKernelGGL(k_rsv_stage<3>, dim3(1), dim3(64), 0, es, scores, d->d_rsv, K, rlo, rhi, wr, aff, lists, st, d->d_rsv_out, rds, d->d_dsmax, k.wp_ds);
          if (coll && (crc = coll_all_reduce(d, &st->best, 1, KE_COLL_U64, KE_COLL_MAX, es))) return crc;
          hipLaunchKernelGGL(k_rsv_stage<4>, dim3(1), dim3(64), 0, es, scores, d->d_rsv, K, rlo, rhi, wr, aff, lists, st, d->d_rsv_out, rds, d->d_dsmax, k.wp_ds);
          if (coll && (crc = coll_all_reduce(d, &st->wt, 2, KE_COLL_I32, KE_COLL_MAX, es))) return crc;  // wt, nw
          hipLaunchKernelGGL(k_rsv_stage<5>, dim3(1), dim3(64), 0, es, scores, d->d_rsv, K, rlo, rhi, wr, aff, lists, st, d->d_rsv_out, rds, d->d_dsmax, k.wp_ds);
          HIP_OK(hipMemcpyAsync(d->h_rsv_out.data(), d->d_rsv_out, sizeof(int32_t) * 4, hipMemcpyDeviceToHost, es));
        }
      }
    } else {
      if (prof) HIP_OK(hipEventRecord(pe[1], es));
      if (prof) HIP_OK(hipEventRecord(pe[3], es));
      HIP_OK(hipMemsetAsync(lists_cnt, 0, sizeof(int32_t) * MAX_BATCH, es));
    }
    if (prof) HIP_OK(hipEventRecord(pe[2], es));
    return KE_OK;
  };
  // Two streams (pipelining).  A run of plain batches: one persistent k_resolve_run on
  // `stream` resolves them all; on `estream` batch b's eval + select run while batch b-1 is being
  // resolved (they see the Reserves of batches <= b-2), and k_fixup waits for batch b-1's done flag,
  // re-evaluates the nodes it chose and publishes the exact lists.  Any other batch (DeviceShare /
  // cpuset singletons, NUMA-policy contexts, pipeline off) is serial: its eval waits for the previous
  // batch's Reserve (HIP events), its lists are exact, its Reserve kernel waits for its lists.
  // the candidate lists of batches [b0, e) are in descending key order: they come out of a merge (split or
  // node-sharded select), not straight out of one k_select workgroup (unordered)
  auto run_sorted = [&](int b0, int e) {
    for (int b = b0; b < e; b++) {
      const int bp = batches[b].pods;
      if (N <= 0 || batches[b].ds) return false;
      if (sharded) continue;
      if (select_parts(N, bp) <= 1) return false;
    }
    return true;
  };
  ctx->host_ms[3] = ms_since(tp);
  const auto host_t0 = std::chrono::steady_clock::now();
  for (int b = 0; b < n_batches;) {
    if (run_end[b] > 0) {
      const int r0 = b, e = run_end[b];
      const bool ext = (k.flags & AF_EXT) != 0;
      const bool fixup = quota || d->pipe_fixup;  // the replay_batch path (quota) needs exact lists
      const THelp th{d_tlist, d_tmx, d_tready, fixup ? 0 : d->t_helpers, d->t_help_ignore, d_rres + r0};
      // batches alternate between the eval streams -- unsharded only: a node-sharded batch's all-gather must run
      // in the same order on every rank's communicator, which two streams of one rank would not guarantee
      const bool two_es = !fixup && d->estream2 != nullptr && !sharded;
      const bool ahead = two_es && d->eval_patch && d->select_ahead;  // (k_fixlist's lists: descending)
      hipLaunchKernelGGL((quota ? (ext ? k_resolve_run<true, true> : k_resolve_run<true, false>)
                                : (ext ? k_resolve_run<false, true> : k_resolve_run<false, false>)), dim3(1 + th.H), dim3(res_threads<false>()), 0,
                         d->stream, d->soa, d->d_pods, d_bases, r0, e - r0, k, d->d_cand, d->d_cand_cnt, d->d_chosen,
                         d->d_chosen_score, ctx->cfg.global_node_offset, d->d_stamps, d->d_stamps + (n_pods + 2),
                         d->d_devalloc, d_ready, d_done, d_err, d->d_trows, d->d_tcnt, d->d_chg, N,
                         fixup ? nullptr : d->d_stale, fixup ? nullptr : d->d_stale_cnt, (int)(ahead || run_sorted(r0, e)), th);
      if (r0 > 0) HIP_OK(hipStreamWaitEvent(d->estream, d->ev_res[(r0 - 1) % R], 0));
      if (two_es) HIP_OK(hipStreamWaitEvent(d->estream2, r0 > 0 ? d->ev_res[(r0 - 1) % R] : d->ev_start, 0));
      for (int q = r0; q < e; q++) {
        const bool first = q == r0;
        if (!fixup) {  // the stale lists go to the replay as they are; batch q's eval waits for batch q-2's done
          const bool alt = two_es && ((q - r0) & 1);
          hipStream_t es = alt ? d->estream2 : d->estream;
          if (ahead) {
            // select-ahead: batch q's eval waits for batch q-3 (the first two of the run for the Reserve kernel's
            // residency: k_fixlist workgroups spinning on a done flag must never keep it off the CUs), its select
            // follows at once, and k_fixlist brings in batch q-2's changed nodes and publishes the lists
            const int32_t* ew = q - 3 >= r0 ? d_done + (q - 3) : q - 2 < r0 ? d_rres + r0 : nullptr;
            rc = eval_select(q, true, es, ew, nullptr, alt, nullptr, nullptr, nullptr, 1, true);
            if (rc) return rc;
            const uint32_t* pre = d->d_pre + (size_t)(q & 1) * MAX_BATCH * KSTALE2;
            const int32_t* pre_cnt = reinterpret_cast<const int32_t*>(d->d_pre + (size_t)2 * MAX_BATCH * KSTALE2) + (q & 1) * MAX_BATCH;
            const int sp = N > 0 && !batches[q].ds ? select_parts(N, batches[q].pods, KSTALE2) : 1;
            if (d->fix_merge && sp > 1)  // the select left its parts unmerged in the split buffer: the fix merges them
              hipLaunchKernelGGL((ext ? k_fixlist<true, true> : k_fixlist<false, true>), dim3((unsigned)batches[q].pods),
                                 dim3(FIXL_PARTS_BLOCK), 0, es, d->soa, d->d_pods, d_bases + q, k,
                                 alt ? d->d_split2 : d->d_split, nullptr, d_tlist + ((q - 2) & 1) * (1 + MAX_BATCH),
                                 q - 2 >= r0 ? d_done + (q - 2) : nullptr,
                                 d->d_stale + (size_t)(q & 1) * MAX_BATCH * KSTALE, d->d_stale_cnt + (q & 1) * MAX_BATCH,
                                 d_ready + q, d_err, (int64_t)gath_words(KSTALE2), sp);
            else
              hipLaunchKernelGGL((ext ? k_fixlist<true> : k_fixlist<false>), dim3((unsigned)batches[q].pods), dim3(FIXL_BLOCK),
                                 0, es, d->soa, d->d_pods, d_bases + q, k, pre, pre_cnt,
                                 d_tlist + ((q - 2) & 1) * (1 + MAX_BATCH), q - 2 >= r0 ? d_done + (q - 2) : nullptr,
                                 d->d_stale + (size_t)(q & 1) * MAX_BATCH * KSTALE, d->d_stale_cnt + (q & 1) * MAX_BATCH,
                                 d_ready + q, d_err, (int64_t)0, 1);
            continue;
          }
          // two eval streams: batch q's eval waits only for batch q-3, k_patch brings in batch q-2's changed nodes
          const bool patch = two_es && d->eval_patch && q - 2 >= r0;
          // with k_patch, batch q's eval waits for batch q-1's select to start (it followed k_patch(q-1), which
          // waited for done[q-3]): the select's workgroups are resident before this eval's grid takes the CUs
          const bool after_sel = two_es && d->eval_patch;
          const int32_t* ew = after_sel ? (q - 1 >= r0 ? d_sstart + (q - 1) : d_rres + r0)
                                        : (q - 2 >= r0 ? d_done + (q - 2) : nullptr);
          // (every workgroup of batch q-1's select counts itself in sstart[q-1])
          const int32_t want = after_sel && q - 1 >= r0 ? batches[q - 1].pods * std::max(1, select_parts(N, batches[q - 1].pods)) : 1;
          rc = eval_select(q, true, es, ew, d_ready + q, alt, patch ? d_done + (q - 2) : nullptr,
                           d_tlist + ((q - 2) & 1) * (1 + MAX_BATCH), after_sel ? d_sstart + q : nullptr, want);
          if (rc) return rc;
          if (!published)
            hipLaunchKernelGGL(k_handoff, dim3(1), dim3(64), d->excl_lds, es, d_ready + q, (int32_t)batches[q].pods, nullptr,
                               d_err, nullptr, 1);
          continue;
        }
        rc = eval_select(q, true, d->estream);
        if (rc) return rc;
        hipLaunchKernelGGL((ext ? k_fixup<true> : k_fixup<false>), dim3((unsigned)batches[q].pods), dim3(FIX_BLOCK), 0, d->estream, d->soa, d->d_pods,
                           d_bases + q, k, d->d_stale + (size_t)(q & 1) * MAX_BATCH * KSTALE,
                           d->d_stale_cnt + (q & 1) * MAX_BATCH, d->d_trows, d->d_tcnt, d->d_cand, d->d_cand_cnt,
                           d_done, first ? -1 : q - 1, d_ready + q, d_err, d_fst + 2 * q);
      }
      HIP_OK(hipEventRecord(d->ev_res[(e - 1) % R], d->stream));
      HIP_OK(hipEventRecord(d->ev_sel[(e - 1) % R], d->estream));
      if (two_es) HIP_OK(hipEventRecord(d->ev_sel2, d->estream2));
      n_pipelined += e - r0;
      b = e;
      if (b < n_batches && run_end[b] == 0) {  // a serial batch next: the run's eval streams drain first
        HIP_OK(hipStreamWaitEvent(d->stream, d->ev_sel[(e - 1) % R], 0));
        if (two_es) HIP_OK(hipStreamWaitEvent(d->stream, d->ev_sel2, 0));
      }
      continue;
    }
    // serial batch: eval, select and Reserve in order on one stream (no cross-stream hand-off)
    const int bp = batches[b].pods;
    const bool ds = batches[b].ds, cpu = batches[b].cpu;
    const int32_t* bbase = d_bases + b;
    const bool fused_b = fused && b == n_batches - 1;
    if (fused_b) {  // the fused matched pod: the speculation check, then its rows (gated) before its eval
      hipLaunchKernelGGL(k_rsv_check, dim3(1), dim3(256), 0, d->stream, d->d_chosen, bases[b], d->d_rsv,
                         (int)ctx->rsv_pairs.size(), ctx->cfg.global_node_offset, d->d_rsv_gate);
      rc = device_refresh_flush(ctx, d->d_rsv_gate);
      if (rc) return rc;
    }
    if (pre_b != b) rc = eval_select(b, false, d->stream);
    pre_b = -1;
    if (rc) return rc;
    if (fused_b) {
      hipLaunchKernelGGL(k_rsv_gate_apply, dim3(1), dim3(64), 0, d->stream, d->d_rsv_gate, d->d_cand_cnt);
      HIP_OK(hipMemcpyAsync(d->h_rsv_out.data() + 4, d->d_rsv_gate, sizeof(int32_t), hipMemcpyDeviceToHost, d->stream));
    }
    if (bp == 1) {  // one pod: the single-node Reserve (cpuset accumulator when it binds)
      int elo = 0, ehi = 0;  // nodes whose affinities this batch's eval stored in d_aff (binding batches)
      if (cpu && numa) {
        ehi = N;
        if (sharded && !d->loopback) shard_range(N, d->rank, d->world, &elo, &ehi);
      }
      hipLaunchKernelGGL((ds ? (numa ? k_cpuset_reserve<true, true> : k_cpuset_reserve<true, false>)
                             : (numa ? k_cpuset_reserve<false, true> : k_cpuset_reserve<false, false>)),
                         dim3(1), dim3(64), 0, d->stream, d->soa,
                         d->d_pods, bbase, k, d->d_cand, d->d_cand_cnt, d->d_chosen, d->d_chosen_score,
                         ctx->cfg.global_node_offset, d->d_stamps, d->d_stamps + (n_pods + 2), b, d->d_devalloc,
                         numa ? d->d_numaalloc : nullptr, d->d_cpusets,
                         d->d_aff, elo, ehi);
    } else {
      auto resolve = quota ? (ds ? (numa ? k_resolve<true, true, true> : k_resolve<true, false, true>)
                                 : (numa ? k_resolve<false, true, true> : k_resolve<false, false, true>))
                           : (ds ? (numa ? k_resolve<true, true, false> : k_resolve<true, false, false>)
                                 : (numa ? k_resolve<false, true, false> : k_resolve<false, false, false>));
      hipLaunchKernelGGL(resolve, dim3(1), dim3(numa ? res_threads<true>() : res_threads<false>()), 0, d->stream, d->soa, d->d_pods, bbase, bp, k,
                         d->d_cand, d->d_cand_cnt, d->d_chosen, d->d_chosen_score, ctx->cfg.global_node_offset,
                         d->d_stamps, d->d_stamps + (n_pods + 2), b, d->d_devalloc, d->d_numaalloc, d->d_chg, N,
                         (int)run_sorted(b, b + 1));
      if (batches[b].cut) {  // a DeviceShare batch may stop early: re-run its remaining pods as batch b
        if (!d->h_cut.resize(1)) return fail(KE_ERR_DEVICE, "hipHostMalloc of the cut word");
        HIP_OK(hipMemcpyAsync(d->h_cut.data(), d->d_dsmax + DSB_CUT, sizeof(int32_t), hipMemcpyDeviceToHost, d->stream));
        // the next serial batch's eval + select go in behind the read-back, so the device keeps working while the
        // host waits for the cut (without one they stand; with one the re-run batch overwrites what they wrote)
        if (b + 1 < n_batches && run_end[b + 1] == 0 && !(fused && b + 1 == n_batches - 1)) {
          const bool keep = rerun;
          rerun = false;
          rc = eval_select(b + 1, false, d->stream);
          rerun = keep;
          if (rc) return rc;
          pre_b = b + 1;
        }
        HIP_OK(hipStreamSynchronize(d->stream));
        const int32_t cut = d->h_cut[0];
        if (cut >= 0) {
          pre_b = -1;
          if (cut <= bases[b] || cut >= bases[b] + bp) return fail(KE_ERR_DEVICE, "DeviceShare batch cut out of range");
          batches[b].pods = bases[b] + bp - cut;
          bases[b] = cut;
          HIP_OK(hipMemcpyAsync(d_bases + b, &bases[b], sizeof(int32_t), hipMemcpyHostToDevice, d->stream));
          ctx->last_ds_cuts++;
          rerun = true;
          continue;
        }
      }
      rerun = false;
    }
    if (b + 1 < n_batches && run_end[b + 1] > 0)  // the next run's eval stream waits for this Reserve
      HIP_OK(hipEventRecord(d->ev_res[b % R], d->stream));
    b++;
  }
  HIP_OK(hipGetLastError());
  ctx->last_enqueue_ms = ctx->host_ms[4] = ms_since(host_t0);
  tp = clk::now();
  const auto t_fl = clk::now();
  flush_mirror_async(*ctx);  // the earlier calls' deferred host mirror, on a host thread while the device works
  const double flush_ms = ms_since(t_fl);
  HIP_OK(hipEventRecord(e1, d->stream));
  HIP_OK(hipEventRecord(d->ev_rend, d->stream));  // the read-back on the staging stream after the Reserve chain
  HIP_OK(hipStreamWaitEvent(cs, d->ev_rend, 0));
  // The call's outputs go to one page-locked staging area (async copies, no host wait) and are copied out after
  // the synchronisation; allocations none of the call's batches can make are not read back (zero).
  bool any_ds = false;
  for (const Batch& bt : batches) any_ds = any_ds || bt.ds || bt.hint;
  const bool vf_out = d->soa.vfo != nullptr;
  const size_t np = (size_t)n_pods, nb = (size_t)n_batches;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = (off + bytes + 15) & ~(size_t)15;
    return o;
  };
  const size_t o_chosen = take((size_t)out_bytes), o_score = take(want_score ? (size_t)out_bytes : 0),
               o_dev = take(any_ds ? 8 * np : 0), o_cs = take(any_cpu ? 32 * np : 0),
               o_vf = take(vf_out ? 2 * DS_MINORS * np : 0), o_numa = take(numa ? 8 * 16 * np : 0), o_err = take(8),
               o_fst = take(16 * nb), o_dcnt = take(numa ? 4 * nb : 0), o_st = take(8 * (nb + 1)),
               o_pst = take(8 * PST * nb), o_est = take(8 * nb);
  if (!d->h_out.resize(off)) return fail(KE_ERR_DEVICE, "hipHostMalloc of the readback staging buffer");
  uint8_t* const h = d->h_out.data();
  auto d2h = [&](size_t o, const void* src, size_t bytes) -> int {
    if (bytes) HIP_OK(hipMemcpyAsync(h + o, src, bytes, hipMemcpyDeviceToHost, cs));
    return KE_OK;
  };
  if ((rc = d2h(o_chosen, d->d_chosen, (size_t)out_bytes))) return rc;
  if (want_score && (rc = d2h(o_score, d->d_chosen_score, (size_t)out_bytes))) return rc;
  if (any_ds && (rc = d2h(o_dev, d->d_devalloc, 8 * np))) return rc;
  if (any_cpu && (rc = d2h(o_cs, d->d_cpusets, 32 * np))) return rc;
  if (vf_out && (rc = d2h(o_vf, d->d_vfo, 2 * DS_MINORS * np))) return rc;
  if (numa && (rc = d2h(o_numa, d->d_numaalloc, 8 * 16 * np))) return rc;
  if ((rc = d2h(o_err, d_err, 4)) || (rc = d2h(o_err + 4, d->soa.kerr, 4))) return rc;
  if ((rc = d2h(o_fst, d_fst, 16 * nb))) return rc;
  if (numa && (rc = d2h(o_dcnt, d->d_defer_cnt, 4 * nb))) return rc;
  if ((rc = d2h(o_st, d->d_stamps, 8 * (nb + 1))) || (rc = d2h(o_pst, d->d_stamps + (n_pods + 2), 8 * PST * nb)) ||
      (rc = d2h(o_est, estamps, 8 * nb)))
    return rc;
  // the call's end on every stream: its completion waits for these events, not for the streams (a submission
  // behind it may already be queued on them)
  HIP_OK(hipEventRecord(done_ev[0], cs));
  HIP_OK(hipEventRecord(done_ev[1], d->estream));
  if (d->estream2) HIP_OK(hipEventRecord(done_ev[2], d->estream2));
  double enq_ms[5];
  for (int i = 0; i < 5; i++) enq_ms[i] = ctx->host_ms[i];
  const auto entry = ctx->call_entry;
  *fin = [=, batches = std::move(batches), bases = std::move(bases), run_end = std::move(run_end),
          ev = std::move(ev)](int32_t* chosen, int32_t* score) mutable -> int {
  HIP_OK(hipSetDevice(d->device));
  auto tp = clk::now();
  for (int i = 0; i < 5; i++) ctx->host_ms[i] = enq_ms[i];
  ctx->host_ms[7] = flush_ms;  // (ke_schedule adds its own part of the mirror)
  std::vector<uint64_t> st(nb + 1), pst(PST * nb), est(nb), fst(2 * nb);
  std::vector<uint32_t> dcnt(numa ? nb : 0);
  int32_t herr = 0, kerr = 0;
  // while the device runs: the host copies of the segment's pods for the deferred mirror (flush_mirror;
  // ke_schedule records which of them were placed)
  ctx->pending_base = (int64_t)ctx->pending_pods.size();
  ctx->pending_pods.insert(ctx->pending_pods.end(), pods, pods + n_pods);
  HIP_OK(hipEventSynchronize(done_ev[0]));
  HIP_OK(hipEventSynchronize(done_ev[1]));
  if (d->estream2) HIP_OK(hipEventSynchronize(done_ev[2]));
  const auto t_sync = clk::now();
  std::memcpy(chosen, h + o_chosen, (size_t)out_bytes);
  if (score && want_score) std::memcpy(score, h + o_score, (size_t)out_bytes);
  if (any_ds) {
    ctx->last_dev_alloc.resize(np);
    std::memcpy(ctx->last_dev_alloc.data(), h + o_dev, 8 * np);
  } else {
    ctx->last_dev_alloc.clear();  // (readers take absent entries as zero)
  }
  if (any_cpu) {
    ctx->last_cpusets.resize(4 * np);
    std::memcpy(ctx->last_cpusets.data(), h + o_cs, 32 * np);
  } else {
    ctx->last_cpusets.clear();
  }
  ctx->last_vf.clear();
  if (vf_out) {
    ctx->last_vf.resize(2 * DS_MINORS * np);
    std::memcpy(ctx->last_vf.data(), h + o_vf, 2 * DS_MINORS * np);
  }
  ctx->last_numa_alloc.clear();
  if (numa) {
    ctx->last_numa_alloc.resize(16 * np);
    std::memcpy(ctx->last_numa_alloc.data(), h + o_numa, 8 * 16 * np);
    std::memcpy(dcnt.data(), h + o_dcnt, 4 * nb);
  }
  std::memcpy(&herr, h + o_err, 4);
  std::memcpy(&kerr, h + o_err + 4, 4);
  std::memcpy(fst.data(), h + o_fst, 16 * nb);
  std::memcpy(st.data(), h + o_st, 8 * (nb + 1));
  std::memcpy(pst.data(), h + o_pst, 8 * PST * nb);
  std::memcpy(est.data(), h + o_est, 8 * nb);
  ctx->host_ms[5] = ms_since(tp);
  tp = clk::now();
  if (herr) {
    if (d->d_chg)  // an abandoned replay may have left bits set
      (void)hipMemset(d->d_chg, 0, sizeof(uint32_t) * (d->capacity + 31) / 32);
    (void)hipMemset(d->d_parts_done, 0, sizeof(int32_t) * 2 * MAX_BATCH);  // (an aborted launch's counts)
    return fail(KE_ERR_DEVICE, "pipelined schedule: a device-side hand-off timed out (placements invalid)");
  }
  if (kerr & (KERR_HINT_ROUTE | KERR_LDS_WAIT)) {  // internal errors: the placements are not the reference's
    return fail(KE_ERR_DEVICE, (kerr & KERR_LDS_WAIT) ? "internal: a replay LDS wait expired (placements invalid)"
                                                      : "internal: a hinted pod reached a kernel without the hint path");
  }
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  ctx->last_total_ms = ms;
  ctx->last_pipelined = n_pipelined;
  // s_memrealtime ticks -> ms, calibrated against the event-timed span of the whole queue
  const double span = (double)(st[n_batches] - st[0]);
  const double ms_per_tick = span > 0 ? ms / span : 1e-5;
  // a batch's device service time: from its eval start to the end of its Reserve
  ctx->last_batch_ms.resize(n_batches);
  for (int b = 0; b < n_batches; b++) {
    const uint64_t t0 = std::max(std::min(est[b], st[b + 1]), st[0]);
    ctx->last_batch_ms[b] = (double)(st[b + 1] - t0) * ms_per_tick;
  }
  // a pod's latency: from the ke_schedule call's entry (its dequeue) to its batch's Reserve end,
  // the device stamps placed on the host clock by aligning the last one with the return of the final
  // synchronisation (later than the true end: an upper bound)
  {
    const double sync_ms = std::chrono::duration<double, std::milli>(t_sync - entry).count();
    ctx->last_pod_lat.resize((size_t)n_pods);
    for (int b = 0, p0 = 0; b < n_batches; b++) {  // (a DeviceShare batch cut and re-run covers its first part too)
      const double lat = sync_ms - (double)(st[n_batches] - st[b + 1]) * ms_per_tick;
      const int p1 = bases[b] + batches[b].pods;
      for (int p = p0; p < p1; p++) ctx->last_pod_lat[(size_t)p] = lat;
      p0 = p1;
    }
  }
  double pro = 0, loop = 0;  // resolve kernel: prologue (candidate/row staging) vs sequential replay
  // phases: prologue, then the speculative replay's first round (P, R + S, V), its later rounds, and the
  // write-back (the one-wave replay of other batches counts entirely as write-back)
  double ph[6] = {0, 0, 0, 0, 0, 0};
  for (int b = 0; b < n_batches; b++) {
    const uint64_t* p = &pst[PST * (size_t)b];
    pro += (double)(p[4] - p[0]) * ms_per_tick;
    loop += (double)(st[b + 1] - p[4]) * ms_per_tick;
    const bool spec = p[1] > p[4];
    ph[0] += (double)(p[4] - p[0]);
    ph[1] += spec ? (double)(p[1] - p[4]) : 0.0;
    ph[2] += spec ? (double)(p[2] - p[1]) : 0.0;
    ph[3] += spec ? (double)(p[3] - p[2]) : 0.0;
    ph[4] += spec ? (double)(p[5] - p[3]) : 0.0;
    ph[5] += (double)(st[b + 1] - (spec ? p[5] : p[4]));
  }
  ctx->kstat_resolve_prologue_ms = pro / n_batches;
  ctx->kstat_resolve_loop_ms = loop / n_batches;
  for (int i = 0; i < 6; i++) ctx->kstat_resolve_phase_ms[i] = ph[i] * ms_per_tick / n_batches;
  std::vector<char> in_run((size_t)n_batches, 0);  // a pipelined batch after the first of its run
  for (int b = 0; b < n_batches; b++)
    if (run_end[b] > 0)
      for (int q = b + 1; q < run_end[b]; q++) in_run[(size_t)q] = 1;
  std::vector<char> in_run_t(in_run);  // ... with T maxima the helpers may deliver
  if (quota || d->pipe_fixup || d->t_helpers == 0) std::fill(in_run_t.begin(), in_run_t.end(), 0);
  {  // the speculative replay's first round in detail: T set-up, the prediction loop, wave 1's T
     // rows (concurrent with the loop), wave 0's R
    double sub[4] = {0, 0, 0, 0};
    int ns = 0, nt = 0, hits = 0;
    for (int b = 0; b < n_batches; b++) {
      const uint64_t* p = &pst[PST * (size_t)b];
      if (!(p[1] > p[4])) continue;
      ns++;
      sub[0] += (double)(p[8] - p[4]);
      sub[1] += (double)(p[9] > p[8] ? p[9] - p[8] : 0);
      sub[2] += (double)(p[10] > p[8] ? p[10] - p[8] : 0);
      sub[3] += (double)(p[11] > p[1] ? p[11] - p[1] : 0);
      if (in_run_t[(size_t)b]) nt++, hits += p[12] == 1;
    }
    for (int i = 0; i < 4; i++) ctx->kstat_resolve_sub_ms[i] = ns ? sub[i] * ms_per_tick / ns : 0;
    ctx->kstat_resolve_sub_ms[4] = nt ? (double)hits / nt : 0;
    // the progressive S of wave 1 (batches with helper T maxima): its polls, record loads + Reserves, rows, and
    // its end after the T set-up
    double wv[4] = {0, 0, 0, 0};
    int nw = 0;
    for (int b = 0; b < n_batches; b++) {
      const uint64_t* p = &pst[PST * (size_t)b];
      if (!(p[1] > p[4]) || !in_run_t[(size_t)b] || p[15] <= p[8]) continue;
      nw++;
      wv[0] += (double)p[13];
      wv[1] += (double)(p[14] & 0xffffffffu);
      wv[2] += (double)(p[14] >> 32);
      wv[3] += (double)(p[15] - p[8]);
    }
    for (int i = 0; i < 4; i++) ctx->kstat_resolve_wave1_ms[i] = nw ? wv[i] * ms_per_tick / nw : 0;
  }
  ctx->kstat_numa_deferred = 0;
  for (uint32_t c : dcnt) ctx->kstat_numa_deferred += c;
  // per-batch Reserve time from the in-kernel stamps (start of the batch's prologue -> end of its
  // replay); hand-off = end of batch b-1's replay -> start of batch b (run batches after the first);
  // fixup = k_fixup's workgroup 0 from its wait to its publish
  double res_sum = 0, ho_sum = 0, fx_sum = 0;
  int ho_n = 0, fx_n = 0;
  for (int b = 0; b < n_batches; b++) {
    res_sum += (double)(st[b + 1] - pst[PST * (size_t)b]) * ms_per_tick;
    if (fst[2 * b + 1] > fst[2 * b]) {
      fx_sum += (double)(fst[2 * b + 1] - fst[2 * b]) * ms_per_tick;
      fx_n++;
    }
    if (in_run[(size_t)b] && pst[PST * (size_t)b] > st[b]) {
      ho_sum += (double)(pst[PST * (size_t)b] - st[b]) * ms_per_tick;
      ho_n++;
    }
  }
  ctx->kstat_resolve_ms = n_batches ? res_sum / n_batches : 0;
  double rows_fetched = 0, rows_changed = 0;
  double spec_rounds = 0;
  for (int b = 0; b < n_batches; b++) {
    rows_fetched += (double)(pst[PST * (size_t)b + 6] & 0xFFFFFFFFull);
    spec_rounds += (double)(pst[PST * (size_t)b + 6] >> 32);
    rows_changed += (double)pst[PST * (size_t)b + 7];
  }
  ctx->kstat_spec_failed = n_batches ? spec_rounds / n_batches : 0;
  ctx->kstat_rows_fetched = n_batches ? rows_fetched / n_batches : 0;
  ctx->kstat_rows_changed = n_batches ? rows_changed / n_batches : 0;
  ctx->kstat_fixup_ms = fx_n ? fx_sum / fx_n : 0;
  ctx->kstat_handoff_ms = ho_n ? ho_sum / ho_n : 0;
  ctx->kstat_samples = 0;
  ctx->kstat_eval_ms = ctx->kstat_select_ms = 0;
  for (size_t s = 0; s + PE - 1 < ev.size(); s += PE) {
    float a = 0, b = 0;
    HIP_OK(hipEventElapsedTime(&a, ev[s], ev[s + 1]));
    HIP_OK(hipEventElapsedTime(&b, ev[s + 3], ev[s + 2]));
    ctx->kstat_eval_ms += a;
    ctx->kstat_select_ms += b;
    ctx->kstat_samples++;
  }
  if (ctx->kstat_samples) {
    ctx->kstat_eval_ms /= ctx->kstat_samples;
    ctx->kstat_select_ms /= ctx->kstat_samples;
  }
  ctx->host_ms[6] = ms_since(tp);
  return KE_OK;
  };
  return KE_OK;
}

// cycles per unit of each phase of kernel `which` (0 k_resolve per pod, 1 k_numa_fallback per deferred pair,
// 2 k_cpuset_reserve per pod) since its last read (diagnostic build only; zeros otherwise)
int device_replay_phases(Context* ctx, int which, double* cyc8) {
#ifdef KE_PROF_REPLAY
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  HIP_OK(hipDeviceSynchronize());
  unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const size_t off = sizeof(v) * (size_t)which;
  HIP_OK(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_rprof), sizeof(v), off));
  const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_rprof), z, sizeof(z), off));
  for (int i = 0; i < 7; i++) cyc8[i] = v[7] ? (double)v[i] / (double)v[7] : 0.0;
  cyc8[7] = (double)v[7];
#else
  (void)ctx;
  (void)which;
  for (int i = 0; i < 8; i++) cyc8[i] = 0.0;
#endif
  return KE_OK;
}

int device_set_pipeline(Context* ctx, int32_t on) {
  if (on < 0 || on > 2) return fail(KE_ERR_INVALID, "ke_set_pipeline: 0, 1 or 2");
  ctx->dev->pipeline = on != 0;
  ctx->dev->pipe_fixup = on == 2;
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
  const int ppb = EVAL_PPB;
  HIP_OK(hipMemsetAsync(d->d_batch_base, 0, sizeof(int32_t), d->stream));
  const dim3 grid = eval_grid(N, EVAL_BLOCK, n_pods, ppb);
  // the kernel ke_schedule runs for a plain batch of n_pods
  auto launch = [&]() {
    if (use_record_eval(n_pods))
      hipLaunchKernelGGL((k_eval_plain<false>), grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, 0, N, d->d_pods,
                         d->d_batch_base, n_pods, k, d->d_scores, d->capacity, nullptr, nullptr, nullptr);
    else
      hipLaunchKernelGGL((k_eval_batch<false, false, false>), grid, dim3(EVAL_BLOCK), 0, d->stream, d->soa, 0, N,
                         d->d_pods, d->d_batch_base, n_pods, ppb, k, d->d_scores, d->capacity, d->d_dsraw, d->d_defer,
                         nullptr, d->d_aff, d->d_dsmax, nullptr);
  };
  launch();  // warm
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, d->stream));
  for (int it = 0; it < iters; it++) launch();
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

// every node's replay record against one derived from its current SoA row (test of the record upkeep)
__global__ void k_check_records(SoA s, int n, KArgs k, unsigned long long* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  NodeRegs nr;
  load_row(s, i, nr);
  prepare_row(nr);
  int64_t w[NUM_RW];
  rec_from_regs(nr, k, w);
  int miss = 0;
  for (int u = 0; u < NUM_RW; u++) miss += (u != RW_PAD) & (s.rec[(int64_t)i * NUM_RW + u] != w[u]);
  if (miss) atomicAdd(bad, 1ull);
}

int device_check_records(Context* ctx, int64_t now, int64_t* bad) {
  DeviceState* d = ctx->dev;
  HIP_OK(hipSetDevice(d->device));
  int rc = device_refresh(ctx, now);
  if (rc) return rc;
  unsigned long long* dbad = nullptr;
  HIP_OK(hipMalloc(&dbad, sizeof(unsigned long long)));
  HIP_OK(hipMemsetAsync(dbad, 0, sizeof(unsigned long long), d->stream));
  const int N = ctx->n_nodes;
  if (N > 0)
    hipLaunchKernelGGL(k_check_records, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, d->stream, d->soa, N,
                       make_kargs(ctx, now), dbad);
  unsigned long long h = 0;
  HIP_OK(hipMemcpyAsync(&h, dbad, sizeof(h), hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  HIP_OK(hipFree(dbad));
  *bad = (int64_t)h;
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
