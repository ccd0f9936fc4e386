// ke_types.h — layout of the GPU-resident node state (struct of arrays) and of the per-pod
// parameters, shared by the host-side derivation (ke_host.cpp) and the HIP kernels (ke_kernels.hip).
//
// One node row holds everything the fused LoadAware + NodeNUMAResource Filter/Score needs, already
// folded on the host so that the per-(pod,node) work is pure int64 arithmetic:
//   * LoadAware usage thresholds: int64(math.Round(float64(used)/float64(total)*100)) <= thr
//     (load_aware.go:299) is monotone in `used`, so it is folded into the exact integer bound
//     U*(total,thr) = max{used : round(used/total*100) <= thr}; the kernel tests
//     pod_est <= fh = U* - node_term.  No float64 reaches the device for the filter.
//   * node_term = GetEstimatedUsed minus the pod's own estimate (load_aware.go:251-288), per variant
//     (non-prod / prod) — the assign cache and the NodeMetric enter only through it.
//   * LoadAware score: leastUsedScore(est + term, cap) = (sa - est)*100/cap with sa = cap - term.
//   * NodeNUMAResource: NodeInfo.Requested/Allocatable + the cpuset amplification pieces.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define KE_HD __host__ __device__
#else
#define KE_HD
#endif

namespace ke {

// int64 SoA fields of a node row (index into the field table)
enum RowField : int {
  F_UT = 0,       // NodeMetric.Status.UpdateTime (ns)
  F_FH = 1,       // 4 fields: filter headroom [variant][res]  (variant 0 = non-prod, 1 = prod)
  F_SA = 5,       // 4 fields: score  sa = cap - term_score [variant][res]
  F_CAP = 9,      // 2 fields: EstimateNode allocatable (cpu milli, memory)
  F_NALLOC = 11,  // 2 fields: NodeInfo.Allocatable (cpu milli, memory)
  F_NREQ = 13,    // 2 fields: NodeInfo.Requested
  F_CSM = 15,     // allocated cpuset CPUs * 1000
  F_CSAF = 16,    // Amplify(cpuset milli, filter ratio)
  F_CSAS = 17,    // Amplify(cpuset milli, score ratio)
  NUM_I64_FIELDS = 18
};

// node flags (u32 SoA field)
enum NodeFlag : uint32_t {
  NF_VALID = 1u << 0,          // slot holds a node
  NF_HAS_METRIC = 1u << 1,     // nodeMetricLister.Get succeeded
  NF_HAS_UT = 1u << 2,         // Status.UpdateTime != nil
  NF_NM_NIL = 1u << 3,         // Status.NodeMetric == nil
  NF_HAS_PROD_THR = 1u << 4,   // len(filterProfile.ProdUsageThresholds) > 0
  NF_FILTER_AGG = 1u << 5,     // filterProfile.AggregatedUsage != nil (reason string)
  NF_FH_ON0 = 1u << 6,         // 4 bits: threshold active for [variant][res] -> bit 6 + 2*v + r
  NF_NUMA_AMP_ERR = 1u << 10,  // ratio annotation unparsable -> Filter UnschedulableAndUnresolvable
  NF_NUMA_RATIO_F = 1u << 11,  // filter ratio > 1
  NF_NUMA_TOPO_INVALID = 1u << 12,
  NF_NUMA_RATIO_S = 1u << 13,  // score ratio > 1
  NF_NUMA_SCORE_ZERO = 1u << 14,  // getResourceOptions error -> Score 0
  NF_DS_CACHE = 1u << 15,         // nodeDeviceCache has an entry for the node (DeviceShare runs)
  NF_NUMA_POLICY0 = 1u << 16,     // 2 bits: the node's NUMA topology policy (KE_NUMA_POLICY_*)
  NF_NUMA_OPT_ERR = 1u << 18,     // getResourceOptions fails (amplification annotation unparsable)
  NF_NUMA_AL_AMP = 1u << 19,      // the cpu amplification ratio in force is > 1: every allocation entry has a cpu key
  NF_CPU_BIND0 = 1u << 20,        // 2 bits: the node's CPU bind policy (KE_NODE_CPU_BIND_*)
  NF_CPUS_VALID = 1u << 22,       // the node has a valid CPU topology table (cpuset pods can bind)
  NF_CPU_NUMA_MOST = 1u << 23,    // GetNUMAAllocateStrategy == MostAllocated (cpu accumulator order)
  NF_RSV_CS = 1u << 24,           // the current KE_RSV_MATCHED / IGNORED pod's allocate-from-reservation outcome on
                                  // this node is in SoA::rovr (RsvOvr): it replaces the cpuset trial / allocation,
                                  // DeviceShare's Filter / Score / Reserve, or carries the Reservation Filter
};
// A KE_RSV_MATCHED pod's allocate-from-reservation trial on one node (k_rsv_views): takePreferredCPUs with
// preferredCPUs `pref` (getAvailableCPUs(preferred): RefCount-- on each, nodenumaresource/reservation.go:303-339),
// and for a Restricted reservation a second allocation with `pref2` = its remainedCPUs (:340-417).
// zmask / zcpu (round 6, a pod binding CPUs under a NUMA policy, k_numa_views' allocation): allocateCPUSet per NUMA id
// of the allocation (zmask: ids, zcpu: their cpu amounts) instead of over the node; with score_on the NodeNUMAResource
// Score of the result (scoring.go:101-119, 180-185): requested cpu = Amplify(the node's allocated CPUs with `pref`'s
// RefCount given back, but for the pod's own, x 1000), requested memory / allocatable = sreq1 / salloc (the zones' or
// the node's, from k_numa_views).
struct RsvView {
  int32_t node;
  int32_t restricted;  // 1: Restricted (numCPUsNeeded <= |pref2|, a second allocation on pref2)
  uint64_t pref[4];
  uint64_t pref2[4];
  int32_t zmask, score_on;
  int64_t zcpu[8];
  int64_t sreq1, salloc[2];
};
struct RsvViewOut {
  int32_t ok, score;
  uint64_t cpus[4];
};
// The decisions the host takes from them per node (ke_host.cpp resv_prepare): the Filter's trial allocation
// (0 = the node's own, 1 = satisfied from a reservation, 2 = "Reservation(s) ..." Unschedulable) and Reserve's
// (0 = the node's own allocation, 1 = `cpus` from the nominated reservation, 2 = Reserve fails).
// DeviceShare (k_ds_views): ds_on = the Filter status / reason and raw Score below replace the node's own
// (tryAllocateFromReservation / scoreWithNominatedReservation, deviceshare/plugin.go:350-364, scoring.go:83-102);
// ds_res = Reserve's devices: 0 the node's own allocation, 1 `ds_minors` (bit 16*type + minor), 2 Reserve fails.
// rfilter (a reservation affinity, AF_RSV_ONLY): 1 the Reservation Filter passes on the node (else it fails).
// NodeNUMAResource under a NUMA policy (k_numa_views, a pod binding no CPUs): numa_on = the Filter's status / reason /
// affinity and the Score below replace the node's own (the hints over the allocate-from-reservation trials and the
// nominated reservation's allocation, nodenumaresource/reservation.go:270-424, scoring.go:101-119); Reserve adds
// numa_dist ([2*id + r]) to the zones.
struct RsvOvr {
  int32_t node;
  int8_t filter, reserve;
  int8_t ds_on, ds_res;
  uint8_t ds_st, ds_reason;
  int8_t rfilter, numa_on;
  int16_t ds_raw, numa_score;
  uint8_t numa_st, numa_reason, numa_aff, pad;
  int32_t pad2;
  uint64_t ds_minors;
  uint64_t cpus[4];
  int64_t numa_dist[16];
};
// The NodeNUMAResource allocate-from-reservation views of a node for a reservation-matched pod binding no CPUs under a
// NUMA policy (k_numa_views; nodenumaresource/reservation.go:270-424, resource_manager.go:130-138, 195-254): beyond
// the node's row (its unmatched restore applied), per NUMA id with an allocation entry (`entry`) the reusable amounts
// [2*id + r] (keys: bit 2*id + r) of the hint view (mergedMatchedAllocatable) and of each trial q < n over
// RestoreReservation's matched set in index order (mergedMatchedAllocated + its remained); a Restricted trial's
// requiredResources (its remained, signed; has_req = the reserve pod holds NUMA amounts).
constexpr int NV_MAX = 31;  // k_numa_views: 2 + 2 x NV_MAX lanes (hint, node, trials, their requiredResources) = the wave
// A pod binding CPUs adds preferredCPUs: the hint view's mergedMatchedRemainCPUs (pref[NV_MAX]), each trial's
// mergedMatchedAllocatedCPUs ∪ its remainedCPUs (pref[q]) and a Restricted trial's remainedCPUs (rpref[q], rem_cpus[q]
// of them) -- getAvailableCPUs with RefCount given back, the per-NUMA-id counts of the CPUs allocateCPUSet may take
// (cs_fill) and trimNUMANodeResources under a required bind policy.
struct NumaRsvView {
  int32_t node, n;
  int32_t required;  // a reservation affinity: no allocation from the node itself
  uint32_t entry;
  uint32_t hint_keys;
  uint32_t keys[NV_MAX], req_keys[NV_MAX];
  uint8_t restricted[NV_MAX], has_req[NV_MAX];
  int32_t rem_cpus[NV_MAX];
  int64_t hint[16];
  int64_t reuse[NV_MAX][16];
  int64_t req[NV_MAX][16];
  uint64_t pref[NV_MAX + 1][4];
  uint64_t rpref[NV_MAX][4];
};
// its outcome: the Filter (status, reason, the merged affinity -- 0 nil), and on that affinity per trial q (bit q of
// ok; bit NV_MAX: the node's own) the allocation and the Score with the options it used (a binding pod's Score needs
// its cpuset: sreq1 / salloc are calculateAllocatableAndRequested's memory requested and allocatable, the cpuset pass
// -- k_rsv_views -- adds the cpu)
struct NumaRsvOut {
  int32_t st, reason;
  uint32_t aff, ok;
  int32_t score[NV_MAX + 1];
  int32_t pad;
  int64_t dist[NV_MAX + 1][16];
  int64_t sreq1[NV_MAX + 1];
  int64_t salloc[NV_MAX + 1][2];
};
// One DeviceShare allocate-from-reservation view of a node (k_ds_views): the allocator's arguments a
// reservation-matched (or -ignored) pod sees beyond the node's row (AutopilotAllocator with preemptible /
// requiredDeviceResources / required + preferred minors, deviceshare/reservation.go:207-366):
//   pre:  the preemptible beyond the node's unmatched restore (already in the row's used), per instance and key
//         (bit 16*type + minor in pre_in, keys in pre_keys[k]): the row's used becomes max(0, used - pre);
//   cap:  requiredDeviceResources of a Restricted reservation: per type with cap_in bits only those instances,
//         free = MinResourceList(free, cap) (keys of both);
//   pref / rreq: defaultAllocateDevices' preferred minors (ordered first) and required minors (only these).
struct DsView {
  int32_t node;
  int32_t pad;
  uint16_t pref[3], rreq[3], cap_in[3];
  uint16_t pad2;
  uint64_t pre_in;
  uint64_t pre_keys[3], cap_keys[3];
  int64_t pre[3][16][3];
  int64_t cap[3][16][3];
};
// its outcome: the Filter's allocation without a scorer (status, reason), AutopilotAllocator.score (raw) and the
// Reserve-phase allocation with the plugin's scorer (minors, 0 when it fails)
struct DsViewOut {
  int32_t st, reason;
  int64_t raw;
  uint64_t minors;
};
KE_HD inline int nf_cpu_bind(uint32_t f) { return (int)((f >> 20) & 3u); }
KE_HD inline int nf_numa_policy(uint32_t f) { return (int)((f >> 16) & 3u); }
KE_HD inline int pf_numa_policy(uint32_t f) { return (int)((f >> 9) & 3u); }

// ---- NUMA topology state (a third SoA, allocated when the first node with a NUMA policy appears) ----
// int64 fields indexed by NUMA id z (0..7) and resource r (cpu milli, memory):
//   NUMA_CAP + 2z + r: TopologyOptions.NUMANodeResources after amplifyNUMANodeResources
//   NUMA_AL  + 2z + r: the zone's allocated resources, cpu adjusted for amplified cpusets
//                      (getAvailableNUMANodeResources before its non-negative clamp)
// uint64 mask (bit = NUMA id): zone present (bits 0-7), capacity cpu / memory key (NUMA_M_CAP + 8r),
// allocated cpu / memory key (NUMA_M_AL + 8r; cpu set for every entry when a ratio > 1 adjusts it)
// NUMANodeSharedStatus of NUMA ids 0..n_zones-1 (GetAllNUMANodeStatus): single (NUMA_M_ST),
// shared (NUMA_M_ST + 8)
constexpr int NUMA_M_CAP = 8;
constexpr int NUMA_M_AL = 24;
constexpr int NUMA_M_ST = 40;
constexpr int NUMA_CAP = 0;
constexpr int NUMA_AL = 16;
constexpr int NUM_NUMA_FIELDS = 32;
KE_HD constexpr uint32_t nf_fh_on(int v, int r) { return NF_FH_ON0 << (2 * v + r); }

// pod flags
enum PodFlag : uint32_t {
  PF_DAEMONSET = 1u << 0,
  PF_PROD = 1u << 1,           // GetPodPriorityClassWithDefault == koord-prod
  PF_NUMA_SKIP = 1u << 2,      // PodRequests all zero -> NodeNUMAResource skip
  PF_LA_SCORE_PROD = 1u << 3,  // prod && ScoreAccordingProdUsage
  PF_DS = 1u << 4,             // DeviceShare PreFilter succeeded and did not Skip: Filter/Score run
  PF_DS_INVALID = 1u << 5,     // DeviceShare PreFilter failed (UnschedulableAndUnresolvable everywhere)
  PF_DS_H_CORE = 1u << 6,      // per-GPU request has gpu-core
  PF_DS_H_MEM = 1u << 7,       // per-GPU request has gpu-memory (fill: bytes -> ratio)
  PF_DS_H_RATIO = 1u << 8,     // per-GPU request has gpu-memory-ratio (fill: ratio -> bytes)
  PF_NUMA_POLICY0 = 1u << 9,   // 2 bits: the pod's NUMATopologySpec policy (KE_NUMA_POLICY_*)
  PF_NUMA_EXCL_REQ = 1u << 11, // SingleNUMANodeExclusive Required (explicit, or defaulted by a pod policy)
  // NodeNUMAResource PreFilter cpuset state (plugin.go:251-312)
  PF_CPU_INVALID = 1u << 12,   // non-integer cpuset request: UnschedulableAndUnresolvable everywhere
  PF_CPU_RCB = 1u << 13,       // state.requestCPUBind
  PF_CPU_INT = 1u << 14,       // cpu request is whole CPUs (a node CPU bind policy may force binding)
  PF_CPU_REQ0 = 1u << 15,      // 2 bits: state.requiredCPUBindPolicy (XB_NONE / XB_FULL / XB_SPREAD)
  PF_CPU_PREF0 = 1u << 17,     // 2 bits: state.preferredCPUBindPolicy
  PF_CPU_EXCL0 = 1u << 19,     // 2 bits: state.preferredCPUExclusivePolicy (KE_CPU_EXCL_*)
  PF_CPUSET = 1u << 21,        // the pod may bind CPUs on some node: singleton batch, cpuset Reserve
  PF_QUOTA_NP = 1u << 22,      // ElasticQuota: IsPodNonPreemptible (checked against Min, counted in non-preemptible used)
  PF_GPU_SHARED = 1u << 23,    // GPURequirements.gpuShared (devicehandler_gpu.go:84-93)
  PF_GPU_SCOPE0 = 1u << 24,    // 3 bits: requiredTopologyScope (KE_SCOPE_*)
  PF_GPU_PART_SPEC = 1u << 27, // GPUPartitionSpec present: honorGPUPartition
  PF_GPU_PART_RESTRICTED = 1u << 28,  // GPUPartitionSpec.AllocatePolicy Restricted
  PF_GPU_RING_BW = 1u << 29,   // GPUPartitionSpec.RingBusBandwidth set (DevPod::ring_bw)
  PF_DS_HINT = 1u << 30,       // DeviceAllocateHints / DeviceJointAllocate: DevPod::ring_bw = the DevPodHint slot
};
KE_HD inline int pf_cpu_required(uint32_t f) { return (int)((f >> 15) & 3u); }
KE_HD inline int pf_cpu_preferred(uint32_t f) { return (int)((f >> 17) & 3u); }
KE_HD inline int pf_cpu_excl(uint32_t f) { return (int)((f >> 19) & 3u); }

// ---- CPU topology + cpuset allocation state (allocated when the first node CPU table appears) ----
// Per node CPU_SLOTS records indexed by CPU id (node-major: 2 KiB per node), plus a summary SoA the
// evaluation reads: CS_RF / CS_RS = the filter / score cpu amplification ratios (IEEE double bits),
// CS_CNT = packed counts (cs_* accessors) of the CPUs available to a new cpuset.
constexpr int CPU_SLOTS = 256;  // == KE_MAX_CPUS
enum : uint8_t { CR_VALID = 1, CR_RESERVED = 2 };
enum { XB_NONE = 0, XB_FULL = 1, XB_SPREAD = 2 };  // bind policies as the cpu accumulator sees them
struct CpuRec {  // one logical CPU: ranks of the reference core / socket ids, the NUMA id as given
  uint8_t core, numa, socket, ref, excl, flags, pad0, pad1;
};
static_assert(sizeof(CpuRec) == 8, "CpuRec layout");
constexpr int CS_RF = 0, CS_RS = 1, CS_CNT = 2, CS_TOPO = 3;
constexpr int CS_ZALL = 4, CS_ZFULL = 6, CS_ZSPREAD = 8;  // 2 words each: 16-bit counts per NUMA id 0..7
constexpr int NUM_CS_FIELDS = 10;
// CS_CNT: CPUs in fully available cores (bits 0-15), cores with an available CPU (16-31), CPUs per
// core (32-39), MaxRefCount (40-47), available CPUs (48-63).  CS_TOPO: CPUTopology's NumCPUs /
// NumCores / NumNodes / NumSockets (cpu_topology.go:45-105) in 16-bit lanes.  CS_Z*: the same three
// availabilities per NUMA id (the CPUs allocateCPUSet may take in a zone without / under a required
// FullPCPUs / SpreadByPCPUs policy).
KE_HD inline int64_t cs_pack(int full, int spread, int cpc, int max_ref, int all) {
  return (int64_t)full | ((int64_t)spread << 16) | ((int64_t)cpc << 32) | ((int64_t)max_ref << 40) |
         ((int64_t)all << 48);
}
KE_HD inline int cs_full(int64_t c) { return (int)(c & 0xffff); }
KE_HD inline int cs_spread(int64_t c) { return (int)((c >> 16) & 0xffff); }
KE_HD inline int cs_cpc(int64_t c) { return (int)((c >> 32) & 0xff); }
KE_HD inline int cs_max_ref(int64_t c) { return (int)((c >> 40) & 0xff); }
KE_HD inline int cs_all(int64_t c) { return (int)((c >> 48) & 0xffff); }
KE_HD inline int cs_zone(int64_t lo, int64_t hi, int z) { return (int)(((z < 4 ? lo : hi) >> (16 * (z & 3))) & 0xffff); }
// NodeAllocation.getAvailableCPUs (node_allocation.go:192-219): not reserved, RefCount < MaxRefCount
KE_HD inline bool cpu_available(const CpuRec& r, int max_ref) {
  return (r.flags & CR_VALID) && !(r.flags & CR_RESERVED) && !(r.ref > 0 && r.ref >= max_ref);
}
// CS_CNT and the six CS_Z* words over one node's records; `core_n` is CPU_SLOTS bytes of scratch.  `pref`: a
// view's preferredCPUs given back first (getAvailableCPUs(preferred): RefCount-- on each, node_allocation.go:192-219)
KE_HD inline void cs_fill(const CpuRec* recs, int cpc, int max_ref, uint8_t* core_n, int64_t* cnt, int64_t* z6,
                          const uint64_t* pref = nullptr) {
  auto avail = [&](int c) {
    CpuRec r = recs[c];
    if (pref && ((pref[c >> 6] >> (c & 63)) & 1) && r.ref > 0) r.ref--;
    return cpu_available(r, max_ref);
  };
  for (int k = 0; k < CPU_SLOTS; k++) core_n[k] = 0;
  int all = 0;
  for (int c = 0; c < CPU_SLOTS; c++)
    if (avail(c)) core_n[recs[c].core]++, all++;
  int full = 0, spread = 0;
  for (int k = 0; k < CPU_SLOTS; k++) {
    if (core_n[k] == cpc && cpc > 0) full += cpc;
    if (core_n[k] > 0) spread++;
  }
  *cnt = cs_pack(full, spread, cpc, max_ref, all);
  for (int w = 0; w < 6; w++) z6[w] = 0;
  for (int c = 0; c < CPU_SLOTS; c++) {  // ascending ids: a core's first available CPU is its lowest
    if (!avail(c) || recs[c].numa >= 8) continue;
    const int z = recs[c].numa, sh = 16 * (z & 3), hi = z >> 2;
    uint8_t& n = core_n[recs[c].core];
    z6[0 + hi] += (int64_t)1 << sh;                                  // available
    if ((n & 0x7f) == cpc) z6[2 + hi] += (int64_t)1 << sh;          // in a fully available core
    if (!(n & 0x80)) z6[4 + hi] += (int64_t)1 << sh, n |= 0x80;     // the core's lowest available CPU
  }
}

// host-side packed row (staging for uploads, debug readback)
struct Row {
  int64_t f[NUM_I64_FIELDS];
  uint32_t flags;
  uint32_t pad;
};
static_assert(sizeof(Row) == 152, "Row layout");
// Bytes of one node row the eval kernel reads per pass (18 int64 fields + u32 flags).
constexpr int ROW_BYTES = NUM_I64_FIELDS * 8 + 4;

// ElasticQuota device table: int64 fields x QT_STRIDE quotas, and a meta word per quota
constexpr int QT_STRIDE = 256;
enum QuotaField : int { QF_LIM = 0, QF_MIN = 2, QF_USED = 4, QF_NP = 6, NUM_QF = 8 };  // + resource
// meta: parent index (int16, -1 = root) | used-limit keys << 16 | Min keys << 18 | Max keys << 20
KE_HD inline int qm_parent(int32_t m) { return (int)(int16_t)(m & 0xFFFF); }
KE_HD inline bool qm_lim(int32_t m, int r) { return (m >> (16 + r)) & 1; }
KE_HD inline bool qm_min(int32_t m, int r) { return (m >> (18 + r)) & 1; }
KE_HD inline bool qm_max(int32_t m, int r) { return (m >> (20 + r)) & 1; }

struct DevPod {
  int64_t est[2];  // LoadAware EstimatePod (cpu milli, memory); 0 for a resource without weight
  int64_t req[2];  // PodRequests cpu milli, memory (NodeNUMAResource, NodeInfo.Requested patch)
  uint32_t flags;
  uint8_t ds_cnt[3];  // DeviceShare: desired device count per type (GPU, RDMA, FPGA), 0 = not requested
  uint8_t quota;      // ElasticQuota: 0 = none, else 1 + quota index (ke_pod.quota)
  int64_t ds_req[5];  // DeviceShare per-instance request: gpu-core, gpu-memory, gpu-memory-ratio, rdma, fpga
  int64_t ring_bw;    // GPUPartitionSpec.RingBusBandwidth (PF_GPU_RING_BW)
  // ext slots (KArgs::xs_id: NodeResourcesFitPlus / NodeResourcesFit resources): the pod's request of each slot's
  // resource (ke_pod.xres_value: calculatePodResourceRequest -- cpu / memory with the non-zero defaults --, a
  // scalar's PodRequests), and the ids of its requested resource names (PodRequests > 0)
  int64_t xreq[8];
  uint64_t xmask;
};
static_assert(sizeof(DevPod) == 160, "DevPod layout");
// DevPod::ds_cnt of an ApplyForAll type: the desired count is the node's devices of the type matching the Selector
constexpr uint8_t DS_CNT_ALL = 255;

// ---- DeviceShare hints: one record per hinted pod of a call, indexed by DevPod::ring_bw --------
// Label sets (of devices and VF groups) are interned per context into ids 0..255 (0 = no labels); a selector
// becomes the 256-bit set of label-set ids it matches.  GPU template model keys likewise (ids 1..255).
enum PodHintFlag : uint32_t {
  PH_SEL0 = 1u << 0,     // 3 bits: the type has a Selector (filterNodeDevice keeps the matching devices)
  PH_FILTER = 1u << 3,   // state.hasSelectors: the filtered nodeDevice view
  PH_VF0 = 1u << 4,      // 3 bits: mustAllocateVF for the type
  PH_TMPL = 1u << 8,     // enforceGPUSharedResourceTemplate
  PH_JOINT_PCIE = 1u << 9,      // DeviceJointAllocate RequiredScope SamePCIe
  PH_FITS_WELL_PLANNED = 1u << 10,  // podFitsSecondaryDeviceWellPlanned
};
struct DevPodHint {
  uint64_t sel[3][4];    // label-set ids the type's Selector matches (all ones without one)
  uint64_t vfsel[3][4];  // label-set ids the type's VFSelector matches
  uint64_t tmpl1[4];     // model key ids with exactly one candidate template
  uint64_t tmplm[4];     // model key ids with two or more
  int64_t ring_bw;       // GPUPartitionSpec.RingBusBandwidth (PF_GPU_RING_BW)
  uint32_t flags;        // PH_*
  uint8_t joint_n;       // DeviceJointAllocate types (primary first)
  int8_t joint[3];
};
static_assert(sizeof(DevPodHint) == 272, "DevPodHint layout");
// Per node DeviceShare hint state (a third device SoA, field-major, allocated with the device SoA):
constexpr int DSX_LBL = 0;     // 6 words: label-set id of (type, minor), 8 bits, word 2*type + minor/8
constexpr int DSX_PCIE = 6;    // 6 words: PCIe rank of (type, minor) (ke_device.pcie_rank), 0xFF = no topology
constexpr int DSX_NODE = 12;   // bit 0 secondary well planned, bits 1-2: the node has VFs of RDMA / FPGA,
                               // bits 8-15: GPU template model key id (0 = none)
constexpr int DSX_VFFREE = 13; // 32 words: VF ranks not held, of (type 1..2, minor): word 16*(type-1) + minor
constexpr int DSX_VFG = 45;    // 128 words: group g's VF ranks of (type, minor): DSX_VFG + 4*(16*(type-1)+minor) + g
constexpr int DSX_VFL = 173;   // 16 words: the 4 groups' label-set ids of (type, minor), 8 bits each, 2 devices a word
constexpr int NUM_DSX = 189;
KE_HD inline int pod_scope(uint32_t flags) { return (int)((flags >> 24) & 7u); }
KE_HD inline int scope_level(int scope) { return scope >= 1 && scope <= 4 ? scope : 0; }

// ---- DeviceShare device state (a second SoA, allocated when the first node device cache appears) ----
// int64 fields: total / used per (type, minor, key); key count 3 for GPU, 1 for RDMA/FPGA.
constexpr int DS_MINORS = 16;  // == KE_MAX_MINORS
constexpr int DS_NK[3] = {3, 1, 1};
constexpr int DS_TBASE[3] = {0, 96, 128};  // total[t][m][k] = DS_TBASE[t] + m*DS_NK[t] + k
constexpr int DS_UBASE[3] = {48, 112, 144};
constexpr int NUM_DS_FIELDS = 160;
// uint64 mask words: exists (bit 16t+m) and the key presence of total / used
enum DsMask : int {
  DSM_EXISTS = 0,  // device instance (t, m) is in the cache (bits 0-47); node GPU flags DSX_* (48-63)
  DSM_GPU_HT = 1,  // GPU total has key k: bit 16k+m (empty for unhealthy devices)
  DSM_GPU_HU = 2,  // GPU used has key k:  bit 16k+m
  DSM_RF = 3,      // RDMA total 0-15, RDMA used 16-31, FPGA total 32-47, FPGA used 48-63
  DSM_TOPO = 4,    // GPU topology tree: 4 bits per minor m at 4m = NUMA scope rank (scopes ascending by NodeID)
  DSM_PCIE = 5,    // 4 bits per minor m at 4m = PCIe scope rank (DFS order: NUMA rank, then PCIEID)
  DSM_DNUMA = 6,   // 3 words (per type): 4 bits per minor m at 4m = the device's NUMA code (DN_*)
  NUM_DS_MASKS = 9
};
// device NUMA codes (DeviceInfo.Topology): 0 = no topology, 1 + NodeID for NodeID 0..7, DN_ANY = NodeID -1
constexpr uint32_t DN_ANY = 9;
// DSM_EXISTS high bits: GPU allocator state of the node (allocator_gpu.go:72-133)
constexpr uint64_t DSX_TOPO = 1ull << 48;   // GetGPUTopologyScope != nil
constexpr uint64_t DSX_HONOR = 1ull << 49;  // nodeHonorGPUPartition
constexpr uint64_t DSX_TABLE = 1ull << 50;  // gpuPartitionIndexer != nil
constexpr int DSX_TABLE_SHIFT = 52;         // 12 bits: partition table id in the table pool
constexpr int MAX_PTABLES = 4096;
// One partition table in the pool: PT_SLOTS entries ordered by (number_of_gpus, allocation score group, table
// order), then the ring bus bandwidths.  Entry: minors (bits 0-15) | number_of_gpus << 16 | group << 24 |
// (uint32)allocation_score << 32; number_of_gpus 0 ends the table.
constexpr int PT_SLOTS = 64;                // == KE_MAX_GPU_PARTITIONS
constexpr int PT_WORDS = 2 * PT_SLOTS;      // entries + ring bandwidths (int64, KE_ABSENT = nil)
KE_HD inline uint32_t pt_minors(uint64_t e) { return (uint32_t)(e & 0xFFFFu); }
KE_HD inline int pt_gpus(uint64_t e) { return (int)((e >> 16) & 0xFFu); }
KE_HD inline int pt_group(uint64_t e) { return (int)((e >> 24) & 0xFFu); }
KE_HD inline int32_t pt_score(uint64_t e) { return (int32_t)(uint32_t)(e >> 32); }
KE_HD inline int ds_ht_word(int t) { return t == 0 ? DSM_GPU_HT : DSM_RF; }
KE_HD inline int ds_hu_word(int t) { return t == 0 ? DSM_GPU_HU : DSM_RF; }
KE_HD inline int ds_ht_bit(int t, int m, int k) { return t == 0 ? 16 * k + m : (t == 1 ? m : 32 + m); }
KE_HD inline int ds_hu_bit(int t, int m, int k) { return t == 0 ? 16 * k + m : (t == 1 ? 16 + m : 48 + m); }
// DeviceShare score weight index of (type, key) (KE_DSW_*), -1 = none
KE_HD inline int ds_weight_index(int t, int k) { return t == 0 ? (k == 2 ? 0 : (k == 1 ? 1 : -1)) : (t == 1 ? 2 : 3); }
// pod per-instance request slot of (type, key)
KE_HD inline int ds_req_slot(int t, int k) { return t == 0 ? k : 2 + t; }

// kernel-uniform arguments
enum ArgFlag : uint32_t {
  AF_FILTER_EXPIRED = 1u << 0,      // args.FilterExpiredNodeMetrics
  AF_ENABLE_WHEN_EXPIRED = 1u << 1, // args.EnableScheduleWhenNodeMetricsExpired
  AF_EXP_PRESENT = 1u << 2,         // args.NodeMetricExpirationSeconds != nil
  AF_NUMA_MOST = 1u << 3,           // NodeNUMAResource MostAllocated
  AF_DS_MOST = 1u << 4,             // DeviceShare MostAllocated
  AF_NUMA_HINT_MOST = 1u << 5,      // NodeNUMAResource NUMAScoringStrategy MostAllocated (hint scores)
  AF_QUOTA = 1u << 6,               // an ElasticQuota tree is loaded: PreFilter admission + Reserve
  AF_QUOTA_PARENT = 1u << 7,        // ElasticQuotaArgs.EnableCheckParentQuota
  AF_DS_NO_NUMA = 1u << 8,          // DeviceShareArgs.DisableDeviceNUMATopologyAlignment
  AF_EXT = 1u << 9,                 // NodeResourcesFitPlus / ScarceResourceAvoidance / NodeResourcesFit (ext SoA)
  AF_FIT_FILTER = 1u << 10,         // NodeResourcesFit's Filter in the profile
  AF_FIT_MOST = 1u << 11,           // NodeResourcesFit ScoringStrategy MostAllocated
  AF_RSV_ONLY = 1u << 12,           // a reservation-affinity pod: only NF_RSV_CS nodes whose RsvOvr.rfilter is 1 pass
};
constexpr int NUM_XS = 8;  // ext slots: the resource ids NodeResourcesFitPlus / NodeResourcesFit read
struct KArgs {
  int64_t now;
  int64_t exp_s;       // NodeMetricExpirationSeconds
  int32_t w_la[2];     // LoadAware resourceWeights (0 = absent)
  int32_t w_numa[2];   // NodeNUMAResource ScoringStrategy weights (0 = absent)
  int32_t wsum_la, wsum_numa;
  int32_t wp_la, wp_numa;  // plugin weights in the profile
  uint32_t flags;
  int32_t wp_ds;           // DeviceShare plugin weight
  int32_t w_ds[4];         // DeviceShare ScoringStrategy weights (KE_DSW_*), -1 = absent
  // ext slots q < xs_n (resource id xs_id[q]): NodeResourcesFitPlus scores the slots of fp_mask (weight fp_w[q],
  // MostAllocated bit in fp_most), NodeResourcesFit scores those of fit_mask (weight fit_w[q]) and its Filter
  // checks the scalar slots of fit_scalar; ScarceResourceAvoidance reads the id masks
  int32_t wp_fp, wp_sra, wp_fit;  // plugin weights (0 = not in the profile)
  int32_t xs_n;
  uint32_t fp_mask, fp_most, fit_mask, fit_scalar;
  int32_t xs_id[NUM_XS];
  int64_t fp_w[NUM_XS];
  int64_t fit_w[NUM_XS];
  uint64_t sra_mask;       // ScarceResourceAvoidanceArgs.Resources (resource ids)
};
// ext SoA: XF_ALLOC + q / XF_REQ + q = NodeInfo.Allocatable / what calculateResourceAllocatableRequest reads
// (NonZeroRequested for cpu / memory, Requested for a scalar) of slot q; XF_PODS = AllowedPodNumber - len(Pods);
// plus a uint64 mask per node of the resource ids with Allocatable > 0
constexpr int XF_ALLOC = 0, XF_REQ = NUM_XS, XF_PODS = 2 * NUM_XS, NUM_XF = 2 * NUM_XS + 1;

// Packed candidate key: higher is better.  (score+1) in the top 10 bits, inverted node index in the
// low 22 bits, so max(key) == selectHost with ties resolved to the lowest node index.
constexpr uint32_t KEY_IDX_BITS = 22;
constexpr uint32_t KEY_IDX_MASK = (1u << KEY_IDX_BITS) - 1;
constexpr int MAX_SHARD_NODES = (1 << KEY_IDX_BITS) - 1;
constexpr int MAX_TOTAL_SCORE = 1022;  // (score+1) must fit in 10 bits: Σ plugin weight * 100 <= 1022
constexpr int MAX_DS_RAW = 300;       // DeviceShare raw score: <= 100 per device type
KE_HD inline uint32_t make_key(int32_t total, int32_t idx) {
  return total < 0 ? 0u : ((uint32_t)(total + 1) << KEY_IDX_BITS) | (KEY_IDX_MASK - (uint32_t)idx);
}
KE_HD inline int32_t key_node(uint32_t key) { return (int32_t)(KEY_IDX_MASK - (key & KEY_IDX_MASK)); }
KE_HD inline int32_t key_score(uint32_t key) { return (int32_t)(key >> KEY_IDX_BITS) - 1; }

constexpr int MAX_BATCH = 64;  // pods per speculative batch (== max candidates per pod)

}  // namespace ke
