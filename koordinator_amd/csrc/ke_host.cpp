// ke_host.cpp — folding of the informer-fed object state into GPU node rows.
//
// The reference recomputes GetEstimatedUsed (load_aware.go:251-288) from the NodeMetric and the
// podAssignCache on every Filter and every Score call.  Everything in it except the pod's own
// estimate is a function of the node alone, so here it is computed once per node state change and
// stored as a per-variant "term"; the pod enters the device arithmetic only through its estimate.
#include "ke_host.h"

#include <algorithm>
#include <climits>
#include <cstddef>
#include <cmath>
#include <cstring>
#include <map>
#include <unordered_map>

namespace ke {

static thread_local std::string g_error;
void set_error(const std::string& msg) { g_error = msg; }
int fail(int code, const std::string& msg) {
  g_error = msg;
  return code;
}
const char* last_error_cstr() { return g_error.c_str(); }

constexpr int64_t NS = 1000000000LL;
constexpr int64_t DEFAULT_MILLI_CPU = 250;                 // default_estimator.go:36
constexpr int64_t DEFAULT_MEMORY = 200LL * 1024 * 1024;    // default_estimator.go:38
constexpr int64_t DEFAULT_REPORT_INTERVAL_NS = 60 * NS;    // load_aware.go:58
constexpr int64_t USED_DOMAIN = 1LL << 53;                 // threshold folding is exact for |used| <= 2^53

// ---------------------------------------------------------------------------------------------
// validation
// ---------------------------------------------------------------------------------------------
int validate_config(const ke_config& cfg) {
  if (cfg.abi_version != KE_ABI_VERSION) return fail(KE_ERR_INVALID, "ke_config.abi_version mismatch");
  if (cfg.node_capacity <= 0 || cfg.node_capacity > MAX_SHARD_NODES)
    return fail(KE_ERR_INVALID, "node_capacity out of range (1 .. 2^22-1 per shard)");
  if (cfg.pod_batch < 1 || cfg.pod_batch > MAX_BATCH) return fail(KE_ERR_INVALID, "pod_batch out of range (1..64)");
  const ke_ext_args& x = cfg.ext;
  if (cfg.weight_reservation < 0) return fail(KE_ERR_INVALID, "negative Reservation weight");
  if (cfg.weight_reservation > (1 << 20)) return fail(KE_ERR_UNSUPPORTED, "Reservation weight above 2^20");
  if (cfg.weight_loadaware < 0 || cfg.weight_numa < 0 || cfg.weight_deviceshare < 0 || x.weight_fitplus < 0 ||
      x.weight_sra < 0 || cfg.fit.weight < 0 ||
      (cfg.weight_loadaware + cfg.weight_numa + cfg.weight_deviceshare + x.weight_fitplus + x.weight_sra +
       cfg.fit.weight) * 100 > MAX_TOTAL_SCORE)
    return fail(KE_ERR_UNSUPPORTED, "plugin weights: (sum of the Score plugin weights) * 100 must be <= 1022");
  if (x.n_fitplus < 0 || x.n_fitplus > KE_MAX_FITPLUS)
    return fail(KE_ERR_UNSUPPORTED, "NodeResourcesFitPlusArgs.Resources: at most 4 resources");
  const ke_fit_args& fa = cfg.fit;
  if (fa.weight < 0 || fa.weight > (1 << 20)) return fail(KE_ERR_UNSUPPORTED, "NodeResourcesFit weight out of range");
  if (fa.has_ignored)
    return fail(KE_ERR_UNSUPPORTED, "NodeResourcesFit ignored resources / groups or RequestedToCapacityRatio");
  if (fa.strategy != KE_STRATEGY_LEAST_ALLOCATED && fa.strategy != KE_STRATEGY_MOST_ALLOCATED)
    return fail(KE_ERR_INVALID, "NodeResourcesFit scoring strategy");
  if (fa.n_resources < 0 || fa.n_resources > KE_MAX_FITPLUS || fa.n_scalars < 0 || fa.n_scalars > 8)
    return fail(KE_ERR_UNSUPPORTED, "NodeResourcesFit: at most 4 scored resources and 8 filtered scalars");
  for (int q = 0; q < fa.n_resources; q++) {
    const ke_fitplus_resource& e = fa.resources[q];
    if (e.id < 0 || e.id >= KE_MAX_XRES) return fail(KE_ERR_INVALID, "NodeResourcesFit resource id out of range");
    if (e.weight < 0 || e.weight > (1 << 20)) return fail(KE_ERR_UNSUPPORTED, "NodeResourcesFit resource weight out of range");
    for (int r = 0; r < q; r++)
      if (fa.resources[r].id == e.id) return fail(KE_ERR_INVALID, "NodeResourcesFit resource listed twice");
  }
  for (int q = 0; q < fa.n_scalars; q++)
    if (fa.scalars[q] < 2 || fa.scalars[q] >= KE_MAX_XRES)
      return fail(KE_ERR_INVALID, "NodeResourcesFit scalar id out of range (cpu / memory are not scalars)");
  {
    int32_t ids[2 * NUM_XS + KE_MAX_FITPLUS];
    if (ext_slots(cfg, ids) > NUM_XS)
      return fail(KE_ERR_UNSUPPORTED, "NodeResourcesFitPlus + NodeResourcesFit read more than 8 distinct resources");
  }
  for (int q = 0; q < x.n_fitplus; q++) {
    const ke_fitplus_resource& e = x.fitplus[q];
    if (e.id < 0 || e.id >= KE_MAX_XRES) return fail(KE_ERR_INVALID, "NodeResourcesFitPlus resource id out of range");
    if (e.type != KE_STRATEGY_LEAST_ALLOCATED && e.type != KE_STRATEGY_MOST_ALLOCATED)
      return fail(KE_ERR_INVALID, "NodeResourcesFitPlus resource type");
    if (e.weight < 0 || e.weight > (1 << 20)) return fail(KE_ERR_UNSUPPORTED, "NodeResourcesFitPlus weight out of range");
    for (int r = 0; r < q; r++)
      if (x.fitplus[r].id == e.id) return fail(KE_ERR_INVALID, "NodeResourcesFitPlus resource listed twice");
  }
  for (int i = 0; i < 4; i++) {
    const int64_t w = cfg.deviceshare.weights[i];
    if (w != KE_ABSENT && (w < 0 || w > (1 << 20))) return fail(KE_ERR_UNSUPPORTED, "deviceshare weight out of range");
  }
  if (cfg.deviceshare.strategy != KE_STRATEGY_LEAST_ALLOCATED && cfg.deviceshare.strategy != KE_STRATEGY_MOST_ALLOCATED)
    return fail(KE_ERR_INVALID, "deviceshare scoring strategy");
  for (int r = 0; r < KE_NRES; r++) {
    int64_t w = cfg.loadaware.resource_weights[r];
    if (w != KE_ABSENT && (w < 0 || w > (1 << 20))) return fail(KE_ERR_UNSUPPORTED, "loadaware weight out of range");
    w = cfg.numa.weights[r];
    if (w != KE_ABSENT && (w < 0 || w > (1 << 20))) return fail(KE_ERR_UNSUPPORTED, "numa weight out of range");
  }
  if (cfg.numa.strategy != KE_STRATEGY_LEAST_ALLOCATED && cfg.numa.strategy != KE_STRATEGY_MOST_ALLOCATED)
    return fail(KE_ERR_INVALID, "numa scoring strategy");
  if (cfg.loadaware.has_other_keys)
    return fail(KE_ERR_UNSUPPORTED, "LoadAwareSchedulingArgs maps with keys other than cpu/memory");
  if (cfg.numa.has_other_keys)
    return fail(KE_ERR_UNSUPPORTED, "NodeNUMAResource ScoringStrategy resources other than cpu/memory");
  if (cfg.deviceshare.has_other_keys)
    return fail(KE_ERR_UNSUPPORTED, "DeviceShare ScoringStrategy resources other than gpu-memory(-ratio)/rdma/fpga");
  if (cfg.deviceshare.template_matched_keys & ~7u) return fail(KE_ERR_INVALID, "template_matched_keys");
  const auto& a = cfg.loadaware;
  if (a.agg_usage_type < 0 || a.agg_usage_type >= KE_AGG_TYPES || a.agg_score_type < 0 || a.agg_score_type >= KE_AGG_TYPES)
    return fail(KE_ERR_INVALID, "aggregation type");
  return KE_OK;
}

int validate_node(const ke_node& n) {
  for (int r = 0; r < KE_NRES; r++) {
    if (n.allocatable[r] < 0 || (n.raw_allocatable[r] < 0 && n.raw_allocatable[r] != KE_ABSENT))
      return fail(KE_ERR_INVALID, "negative allocatable");
  }
  if (n.numa_topology_policy < KE_NUMA_POLICY_NONE || n.numa_topology_policy > KE_NUMA_POLICY_SINGLE_NUMA_NODE)
    return fail(KE_ERR_INVALID, "NUMA topology policy");
  if (n.cpu_bind_policy < KE_NODE_CPU_BIND_NONE || n.cpu_bind_policy > KE_NODE_CPU_BIND_SPREAD_BY_PCPUS)
    return fail(KE_ERR_INVALID, "node CPU bind policy");
  if (n.numa_allocate_strategy > KE_NUMA_ALLOCATE_LEAST) return fail(KE_ERR_INVALID, "NUMA allocate strategy");
  if (n.custom_agg_type < 0 || n.custom_agg_type >= KE_AGG_TYPES) return fail(KE_ERR_INVALID, "aggregation type");
  return KE_OK;
}

int validate_devices(int32_t n, const ke_device* devs) {
  if (n < 0 || n > KE_DEV_TYPES * KE_MAX_MINORS || (n > 0 && !devs)) return fail(KE_ERR_INVALID, "device count");
  uint64_t seen = 0;
  for (int32_t i = 0; i < n; i++) {
    const ke_device& d = devs[i];
    if (d.type < 0 || d.type >= KE_DEV_TYPES || d.minor < 0 || d.minor >= KE_MAX_MINORS)
      return fail(KE_ERR_INVALID, "device type / minor out of range");
    const uint64_t bit = 1ull << (16 * d.type + d.minor);
    if (seen & bit) return fail(KE_ERR_INVALID, "duplicate device minor");
    seen |= bit;
    for (int k = DS_NK[d.type]; k < KE_DKEYS; k++)
      if (d.has_total[k] || d.has_used[k]) return fail(KE_ERR_UNSUPPORTED, "resource key outside the device type");
    for (int k = 0; k < KE_DKEYS; k++)
      if ((d.has_total[k] && d.total[k] < 0) || (d.has_used[k] && d.used[k] < 0))
        return fail(KE_ERR_INVALID, "negative device quantity");
    if (d.has_topology && (d.pcie_rank < 0 || d.pcie_rank >= KE_DEV_TYPES * KE_MAX_MINORS))
      return fail(KE_ERR_INVALID, "device pcie_rank out of range");
    if (d.has_topology && (d.numa_node < -1 || d.numa_node >= KE_MAX_NUMA))
      return fail(KE_ERR_UNSUPPORTED, "device NUMA node outside -1 .. KE_MAX_NUMA-1");
    // fillGPUTotalMem divides by the instance's gpu-memory (devicehandler_gpu.go:110-125)
    if (d.type == KE_DEV_GPU && d.health && !(d.has_total[KE_DKEY_GPU_MEMORY] && d.total[KE_DKEY_GPU_MEMORY] > 0))
      return fail(KE_ERR_UNSUPPORTED, "healthy GPU device without a positive gpu-memory total");
    if (d.labels.n < 0 || d.labels.n > KE_MAX_LABELS || d.n_vf_groups < 0 || d.n_vf_groups > KE_MAX_VF_GROUPS)
      return fail(KE_ERR_INVALID, "device label / VF group count");
    for (int g = 0; g < d.n_vf_groups; g++)
      if (d.vf_groups[g].labels.n < 0 || d.vf_groups[g].labels.n > KE_MAX_LABELS)
        return fail(KE_ERR_INVALID, "VF group label count");
  }
  return KE_OK;
}

// ---- DeviceShare hints -------------------------------------------------------------
static std::vector<std::pair<int32_t, int32_t>> label_pairs(const ke_labels& l) {
  std::vector<std::pair<int32_t, int32_t>> v;
  for (int k = 0; k < l.n && k < KE_MAX_LABELS; k++) v.emplace_back(l.key[k], l.value[k]);
  std::sort(v.begin(), v.end());
  return v;
}
static int intern_set(Context& c, const ke_labels& l) {
  auto v = label_pairs(l);
  auto it = c.label_set_ids.find(v);
  if (it != c.label_set_ids.end()) return it->second;
  if (c.label_sets.size() >= 256) return fail(KE_ERR_UNSUPPORTED, "more than 256 distinct device / VF-group label sets");
  const int id = (int)c.label_sets.size();
  c.label_sets.push_back(v);
  c.label_set_ids.emplace(std::move(v), id);
  return id;
}
int intern_device_labels(Context& c, NodeState& ns) {
  ns.dev_lbl.assign(ns.devs.size() * 5, 0);
  for (size_t i = 0; i < ns.devs.size(); i++) {
    const ke_device& d = ns.devs[i];
    int id = intern_set(c, d.labels);
    if (id < 0) return id;
    ns.dev_lbl[i * 5] = (uint8_t)id;
    for (int g = 0; g < d.n_vf_groups && g < KE_MAX_VF_GROUPS; g++) {
      id = intern_set(c, d.vf_groups[g].labels);
      if (id < 0) return id;
      ns.dev_lbl[i * 5 + 1 + g] = (uint8_t)id;
    }
  }
  return KE_OK;
}
int intern_model_key(Context& c, int32_t key) {
  if (key == 0) return 0;
  for (size_t i = 1; i < c.model_keys.size(); i++)
    if (c.model_keys[i] == key) return (int)i;
  if (c.model_keys.size() >= 256) return fail(KE_ERR_UNSUPPORTED, "more than 255 GPU template model keys");
  c.model_keys.push_back(key);
  return (int)c.model_keys.size() - 1;
}

bool selector_matches(const ke_label_selector& sel, const std::vector<std::pair<int32_t, int32_t>>& labels) {
  for (int r = 0; r < sel.n && r < KE_MAX_SEL_REQS; r++) {  // apimachinery labels.Requirement.Matches
    const ke_label_requirement& q = sel.req[r];
    const auto it = std::find_if(labels.begin(), labels.end(), [&](const auto& kv) { return kv.first == q.key; });
    const bool has = it != labels.end();
    bool listed = false;
    for (int v = 0; v < q.n_values && v < KE_MAX_SEL_VALUES; v++) listed = listed || (has && q.values[v] == it->second);
    bool ok;
    switch (q.op) {
      case KE_SEL_IN: ok = has && listed; break;
      case KE_SEL_NOT_IN: ok = !has || !listed; break;
      case KE_SEL_EXISTS: ok = has; break;
      default: ok = !has; break;
    }
    if (!ok) return false;
  }
  return true;
}

// DeviceJointAllocate.DeviceTypes as parsePodDeviceShareExtensions keeps them (utils.go:430-442): the requested
// types without an ApplyForAll hint, in annotation order
static int joint_list(const ke_pod_device_hints& h, const ke_pod& p, int* out) {
  bool req[KE_DEV_TYPES] = {false, p.device_requests[KE_PDR_RDMA] > 0, p.device_requests[KE_PDR_FPGA] > 0};
  for (int i = 0; i < KE_PDR_COUNT; i++)
    req[KE_DEV_GPU] = req[KE_DEV_GPU] || (i != KE_PDR_RDMA && i != KE_PDR_FPGA && p.device_requests[i] > 0);
  int n = 0;
  for (int j = 0; j < h.joint_n && j < KE_DEV_TYPES; j++) {
    const int t = h.joint_types[j];
    if (t < 0 || t >= KE_DEV_TYPES || !req[t] || h.hint[t].strategy == KE_DSTRATEGY_APPLY_FOR_ALL) continue;
    bool dup = false;
    for (int q = 0; q < n; q++) dup = dup || out[q] == t;
    if (!dup) out[n++] = t;
  }
  return n;
}

const ke_pod_device_hints* pod_hints(const Context& c, const ke_pod& p) {
  return p.device_hint > 0 && p.device_hint <= (int32_t)c.hints.size() ? &c.hints[(size_t)p.device_hint - 1] : nullptr;
}

int validate_pod_hints(const Context& c, const ke_pod& p) {
  if (p.device_hint < 0 || p.device_hint > (int32_t)c.hints.size())
    return fail(KE_ERR_INVALID, "ke_pod.device_hint outside the ke_set_pod_device_hints table");
  const ke_pod_device_hints* h = pod_hints(c, p);
  if (!h) return KE_OK;
  if (h->hint[KE_DEV_GPU].vf_selector.present)  // generalAllocate's defaultAllocateDevices with GPU VFs
    return fail(KE_ERR_UNSUPPORTED, "a VFSelector on the gpu device type is not implemented");
  if (h->joint_n < 0 || h->joint_n > KE_DEV_TYPES) return fail(KE_ERR_INVALID, "joint_n");
  for (int j = 0; j < h->joint_n; j++)
    if (h->joint_types[j] < 0 || h->joint_types[j] >= KE_DEV_TYPES) return fail(KE_ERR_INVALID, "joint device type");
  int jl[KE_DEV_TYPES];
  const int jn = joint_list(*h, p, jl);
  for (int j = 1; j < jn; j++)
    if (jl[j] == KE_DEV_GPU)  // GPUAllocator with a preferred PCIe set / maxDesiredCount
      return fail(KE_ERR_UNSUPPORTED, "DeviceJointAllocate with the gpu type after the primary is not implemented");
  if (jn == 3)  // a secondary type outside requestsPerInstance allocates a nil request
    return fail(KE_ERR_UNSUPPORTED, "DeviceJointAllocate over three device types is not implemented");
  for (int t = 0; t < KE_DEV_TYPES; t++)
    for (const ke_label_selector* sel : {&h->hint[t].selector, &h->hint[t].vf_selector})
      if (sel->n < 0 || sel->n > KE_MAX_SEL_REQS) return fail(KE_ERR_INVALID, "selector requirement count");
  return KE_OK;
}

static void set256(uint64_t (&b)[4], int x) { b[x >> 6] |= 1ull << (x & 63); }

DevPodHint make_pod_hint(const Context& c, const ke_pod& pod, const DevPod& dp, const ke_pod_device_hints& h) {
  DevPodHint r{};
  r.ring_bw = (dp.flags & PF_GPU_RING_BW) ? pod.gpu_ring_bus_bandwidth : KE_ABSENT;
  if (h.has_selectors) r.flags |= PH_FILTER;
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    const ke_device_hint& dh = h.hint[t];
    for (int w = 0; w < 4; w++) r.sel[t][w] = ~0ull;
    if (dh.selector.present) {
      r.flags |= PH_SEL0 << t;
      for (int w = 0; w < 4; w++) r.sel[t][w] = 0;
      for (size_t id = 0; id < c.label_sets.size(); id++)
        if (selector_matches(dh.selector, c.label_sets[id])) set256(r.sel[t], (int)id);
    }
    if (dh.vf_selector.present) {
      r.flags |= PH_VF0 << t;
      for (size_t id = 0; id < c.label_sets.size(); id++)
        if (selector_matches(dh.vf_selector, c.label_sets[id])) set256(r.vfsel[t], (int)id);
    }
  }
  int jl[KE_DEV_TYPES];
  const int jn = joint_list(h, pod, jl);
  r.joint_n = (uint8_t)jn;
  for (int j = 0; j < KE_DEV_TYPES; j++) r.joint[j] = (int8_t)(j < jn ? jl[j] : -1);
  if (h.joint_same_pcie) r.flags |= PH_JOINT_PCIE;
  if (dp.ds_cnt[KE_DEV_GPU] && !(dp.flags & PF_GPU_SHARED)) r.flags |= PH_FITS_WELL_PLANNED;
  // enforceGPUSharedResourceTemplate: candidates per model key (gpu_shared_resource_templates_cache.go:41-62)
  const uint32_t keys = c.cfg.deviceshare.template_matched_keys;
  uint32_t named = 0;
  if (dp.flags & PF_DS_H_CORE) named |= KE_TEMPLATE_KEY_CORE;
  if (dp.flags & PF_DS_H_RATIO) named |= KE_TEMPLATE_KEY_MEMORY_RATIO;
  else if (dp.flags & PF_DS_H_MEM) named |= KE_TEMPLATE_KEY_MEMORY;
  if (dp.ds_cnt[KE_DEV_GPU] && (dp.flags & PF_GPU_SHARED) && (named & keys)) {
    r.flags |= PH_TMPL;
    for (size_t id = 1; id < c.model_keys.size(); id++) {
      int n = 0;
      for (const ke_gpu_template& t : c.tmpl)
        if (t.model_key == c.model_keys[id] && t.has[0] == ((named & KE_TEMPLATE_KEY_CORE) != 0) &&
            t.has[1] == ((named & KE_TEMPLATE_KEY_MEMORY) != 0) && t.has[2] == ((named & KE_TEMPLATE_KEY_MEMORY_RATIO) != 0) &&
            (!t.has[0] || t.value[0] == dp.ds_req[0]) && (!t.has[1] || t.value[1] == dp.ds_req[1]) &&
            (!t.has[2] || t.value[2] == dp.ds_req[2]))
          n++;
      if (n == 1) set256(r.tmpl1, (int)id);
      if (n >= 2) set256(r.tmplm, (int)id);
    }
  }
  return r;
}

void derive_dsx_row(const NodeState& ns, int64_t* w) {
  for (int i = 0; i < NUM_DSX; i++) w[i] = 0;
  for (int i = DSX_PCIE; i < DSX_PCIE + 6; i++) w[i] = -1;  // 0xFF: no topology
  uint64_t node = ns.secondary_well_planned ? 1u : 0u;
  node |= (uint64_t)(ns.gpu_model_id & 0xFF) << 8;
  for (size_t x = 0; x < ns.devs.size(); x++) {
    const ke_device& d = ns.devs[x];
    const int t = d.type, m = d.minor, sh = 8 * (m & 7);
    const uint64_t lbl = x * 5 < ns.dev_lbl.size() ? ns.dev_lbl[x * 5] : 0;
    w[DSX_LBL + 2 * t + (m >> 3)] |= (int64_t)(lbl << sh);
    if (d.has_topology)
      w[DSX_PCIE + 2 * t + (m >> 3)] &= (int64_t)~((uint64_t)(0xFFu & ~(uint32_t)d.pcie_rank) << sh);
    if (t == KE_DEV_GPU || d.n_vf_groups <= 0) continue;
    node |= 1ull << t;  // hasVirtualFunctions
    const int dv = 16 * (t - 1) + m;
    uint64_t all = 0;
    for (int g = 0; g < d.n_vf_groups && g < KE_MAX_VF_GROUPS; g++) {
      w[DSX_VFG + 4 * dv + g] = (int64_t)d.vf_groups[g].vfs;
      all |= d.vf_groups[g].vfs;
      const uint64_t gl = x * 5 + 1 + (size_t)g < ns.dev_lbl.size() ? ns.dev_lbl[x * 5 + 1 + (size_t)g] : 0;
      w[DSX_VFL + (dv >> 1)] |= (int64_t)(gl << (32 * (dv & 1) + 8 * g));
    }
    w[DSX_VFFREE + dv] = (int64_t)(all & ~d.vf_allocated);
  }
  w[DSX_NODE] = (int64_t)node;
}

// GetGPUTopologyScope (allocator_gpu_helper.go:202-263) as per-minor scope ranks: NUMA scopes ascending by
// NodeID, PCIe scopes in depth-first order (NUMA rank, then PCIEID).  Returns false for a nil tree.
static bool gpu_topology_ranks(const NodeState& ns, uint64_t* topo, uint64_t* pcie) {
  std::vector<int32_t> numa;
  std::vector<std::pair<int32_t, int32_t>> pc;  // (numa rank, pcie rank)
  int n_gpu = 0;
  for (const ke_device& d : ns.devs) {
    if (d.type != KE_DEV_GPU) continue;
    if (!d.has_topology) return false;
    n_gpu++;
    numa.push_back(d.numa_node);
  }
  if (n_gpu == 0) return false;
  std::sort(numa.begin(), numa.end());
  numa.erase(std::unique(numa.begin(), numa.end()), numa.end());
  auto numa_rank = [&](int32_t id) { return (int32_t)(std::lower_bound(numa.begin(), numa.end(), id) - numa.begin()); };
  for (const ke_device& d : ns.devs)
    if (d.type == KE_DEV_GPU) pc.emplace_back(numa_rank(d.numa_node), d.pcie_rank);
  std::sort(pc.begin(), pc.end());
  pc.erase(std::unique(pc.begin(), pc.end()), pc.end());
  *topo = *pcie = 0;
  for (const ke_device& d : ns.devs) {
    if (d.type != KE_DEV_GPU) continue;
    const int32_t nr = numa_rank(d.numa_node);
    const int32_t pr = (int32_t)(std::lower_bound(pc.begin(), pc.end(), std::make_pair(nr, d.pcie_rank)) - pc.begin());
    *topo |= (uint64_t)nr << (4 * d.minor);
    *pcie |= (uint64_t)pr << (4 * d.minor);
  }
  return true;
}

void derive_ds_row(const NodeState& ns, int64_t* f, uint64_t* m) {
  for (int i = 0; i < NUM_DS_FIELDS; i++) f[i] = 0;
  for (int i = 0; i < NUM_DS_MASKS; i++) m[i] = 0;
  if (!ns.has_dev_cache) return;
  if (gpu_topology_ranks(ns, &m[DSM_TOPO], &m[DSM_PCIE])) m[DSM_EXISTS] |= DSX_TOPO;
  for (const ke_device& d : ns.devs)  // DeviceShare's NUMA hints group devices by Topology.NodeID
    if (d.has_topology)
      m[DSM_DNUMA + d.type] |= (uint64_t)(d.numa_node < 0 ? DN_ANY : 1u + (uint32_t)d.numa_node) << (4 * d.minor);
  if (ns.gpu_honor) m[DSM_EXISTS] |= DSX_HONOR;
  if (ns.ptable >= 0) m[DSM_EXISTS] |= DSX_TABLE | ((uint64_t)ns.ptable << DSX_TABLE_SHIFT);
  for (const ke_device& d : ns.devs) {
    const int t = d.type, mi = d.minor;
    m[DSM_EXISTS] |= 1ull << (16 * t + mi);
    for (int k = 0; k < DS_NK[t]; k++) {
      if (d.health && d.has_total[k]) {  // unhealthy: empty total (device_cache.go:558-560)
        m[ds_ht_word(t)] |= 1ull << ds_ht_bit(t, mi, k);
        f[DS_TBASE[t] + mi * DS_NK[t] + k] = d.total[k];
      }
      // calcFreeWithPreemptible (device_cache.go:327-336) with the unmatched reservations' owners' part
      // (resv_plugin_restore) as preemptible: used = SubtractWithNonNegativeResult(used, preemptible[minor]) --
      // the free it leaves is the filtered view's (an instance left with nothing free is free of nothing either way)
      const uint64_t rbit = 1ull << (16 * t + mi);
      const bool rv = (ns.rv_dev_minors & rbit) != 0;
      if (d.has_used[k] || (rv && (ns.rv_dev_keys[k] & rbit))) {
        m[ds_hu_word(t)] |= 1ull << ds_hu_bit(t, mi, k);
        int64_t u = d.has_used[k] ? d.used[k] : 0;
        if (rv) u = std::max<int64_t>(0, u - ns.rv_dev[t][mi][k]);
        f[DS_UBASE[t] + mi * DS_NK[t] + k] = u;
      }
    }
  }
}

int ptable_intern(Context& c, int32_t n, const ke_gpu_partition* parts) {
  if (n < 0 || n > KE_MAX_GPU_PARTITIONS || (n > 0 && !parts)) return fail(KE_ERR_INVALID, "partition count");
  std::vector<int> order((size_t)n);
  for (int i = 0; i < n; i++) {
    const ke_gpu_partition& q = parts[i];
    if (q.minors == 0 || (q.minors >> KE_MAX_MINORS)) return fail(KE_ERR_INVALID, "partition minors (non-empty, 0..15)");
    if (q.number_of_gpus < 1 || q.number_of_gpus > 255) return fail(KE_ERR_INVALID, "partition number_of_gpus");
    if (q.ring_bus_bandwidth < 0 && q.ring_bus_bandwidth != KE_ABSENT) return fail(KE_ERR_INVALID, "ring bus bandwidth");
    order[(size_t)i] = i;
  }
  // GetGPUPartitionIndexer (allocator_gpu_helper.go:165-200): per number of GPUs, groups of equal
  // AllocationScore ascending, table order inside a group
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    if (parts[a].number_of_gpus != parts[b].number_of_gpus) return parts[a].number_of_gpus < parts[b].number_of_gpus;
    return parts[a].allocation_score < parts[b].allocation_score;
  });
  std::vector<uint64_t> t((size_t)PT_WORDS, 0);
  int group = -1, in_group = 0;
  for (int k = 0; k < n; k++) {
    const ke_gpu_partition& q = parts[order[(size_t)k]];
    const bool same_n = k > 0 && parts[order[(size_t)k - 1]].number_of_gpus == q.number_of_gpus;
    if (!same_n) group = -1;
    if (!same_n || parts[order[(size_t)k - 1]].allocation_score != q.allocation_score) {
      group++;
      in_group = 0;
    }
    // selectPartitionByBinPack sorts the feasible partitions of one group with sort.Slice, which is a
    // stable insertion sort only up to 12 elements (Go pdqsort)
    if (++in_group > 12) return fail(KE_ERR_UNSUPPORTED, "more than 12 GPU partitions with one (number_of_gpus, allocation_score)");
    if (group > 255) return fail(KE_ERR_UNSUPPORTED, "partition groups");
    t[(size_t)k] = (uint64_t)q.minors | (uint64_t)q.number_of_gpus << 16 | (uint64_t)group << 24 |
                   (uint64_t)(uint32_t)q.allocation_score << 32;
    t[(size_t)(PT_SLOTS + k)] = (uint64_t)q.ring_bus_bandwidth;
  }
  const size_t n_tab = c.ptab.size() / PT_WORDS;
  for (size_t id = 0; id < n_tab; id++)
    if (std::equal(t.begin(), t.end(), c.ptab.begin() + (std::ptrdiff_t)(id * PT_WORDS))) return (int)id;
  if (n_tab >= (size_t)MAX_PTABLES) return fail(KE_ERR_UNSUPPORTED, "more than 4096 distinct GPU partition tables");
  c.ptab.insert(c.ptab.end(), t.begin(), t.end());
  c.ptab_dirty = true;
  return (int)n_tab;
}

// the amounts a pod's Reserve puts on one of its instances (fillGPUTotalMem + the per-instance request)
void ds_instance_amounts(const ke_device& d, const DevPod& dp, int64_t* alloc, bool* has) {
  const int t = d.type;
  for (int k = 0; k < KE_DKEYS; k++) alloc[k] = 0, has[k] = false;
  if (t == KE_DEV_GPU) {
    const int64_t tm = d.health && d.has_total[KE_DKEY_GPU_MEMORY] ? d.total[KE_DKEY_GPU_MEMORY] : 0;
    if (dp.flags & PF_DS_H_CORE) has[0] = true, alloc[0] = dp.ds_req[0];
    if (dp.flags & PF_DS_H_RATIO) {  // memoryRatioToBytes
      has[2] = true, alloc[2] = dp.ds_req[2];
      has[1] = true, alloc[1] = dp.ds_req[2] * tm / 100;
    } else if (dp.flags & PF_DS_H_MEM) {  // memoryBytesToRatio
      has[1] = true, alloc[1] = dp.ds_req[1];
      has[2] = true, alloc[2] = (int64_t)((double)dp.ds_req[1] / (double)tm * 100.0);
    }
  } else {
    has[0] = true, alloc[0] = dp.ds_req[2 + t];
  }
}

void host_ds_reserve(const ke_config& cfg, NodeState& ns, const DevPod& dp, uint64_t mask, const int8_t* vf) {
  (void)cfg;
  for (ke_device& d : ns.devs) {
    if (!(mask & (1ull << (16 * d.type + d.minor)))) continue;
    const int t = d.type;
    if (vf && t > 0 && vf[(t - 1) * KE_MAX_MINORS + d.minor] >= 0)  // updateVFAllocations
      d.vf_allocated |= 1ull << vf[(t - 1) * KE_MAX_MINORS + d.minor];
    int64_t alloc[KE_DKEYS];
    bool has[KE_DKEYS];
    ds_instance_amounts(d, dp, alloc, has);
    for (int k = 0; k < DS_NK[t]; k++)
      if (has[k]) {  // quotav1.Add
        d.used[k] = (d.has_used[k] ? d.used[k] : 0) + alloc[k];
        d.has_used[k] = 1;
      }
  }
}

int validate_pod(const ke_pod& p) {
  if (p.has_resource_spec)  // PreFilter returns the unmarshal error (plugin.go:276-280)
    return fail(KE_ERR_UNSUPPORTED, "pods whose ResourceSpec annotation fails to unmarshal");
  if (p.cpu_bind_required < KE_CPU_BIND_UNSET || p.cpu_bind_required > KE_CPU_BIND_CONSTRAINED_BURST ||
      p.cpu_bind_preferred < KE_CPU_BIND_UNSET || p.cpu_bind_preferred > KE_CPU_BIND_CONSTRAINED_BURST ||
      p.cpu_exclusive < KE_CPU_EXCL_NONE || p.cpu_exclusive > KE_CPU_EXCL_NUMA_NODE_LEVEL)
    return fail(KE_ERR_INVALID, "pod CPU bind / exclusive policy");
  if (p.priority_class < 0 || p.priority_class > KE_PRIORITY_FREE) return fail(KE_ERR_INVALID, "priority class");
  if (p.has_unsupported_device_requests)
    return fail(KE_ERR_UNSUPPORTED, "Huawei NPU device requests are not implemented");
  for (int i = 0; i < KE_PDR_COUNT; i++)
    if (p.device_requests[i] < 0) return fail(KE_ERR_INVALID, "negative device request");
  if (p.numa_topology_policy < KE_NUMA_POLICY_NONE || p.numa_topology_policy > KE_NUMA_POLICY_SINGLE_NUMA_NODE)
    return fail(KE_ERR_INVALID, "pod NUMA topology policy");
  if (p.numa_exclusive < KE_NUMA_EXCLUSIVE_NONE || p.numa_exclusive > KE_NUMA_EXCLUSIVE_REQUIRED)
    return fail(KE_ERR_INVALID, "pod NUMA exclusive policy");
  if (p.gpu_required_topology_scope < KE_SCOPE_NONE || p.gpu_required_topology_scope > KE_SCOPE_UNKNOWN)
    return fail(KE_ERR_INVALID, "pod GPU required topology scope");
  if (p.device_hints & KE_DHINT_GPU_VF)  // generalAllocate's defaultAllocateDevices with GPU VFs
    return fail(KE_ERR_UNSUPPORTED, "a VFSelector on the gpu device type is not implemented");
  if (p.device_hints) return fail(KE_ERR_INVALID, "unknown device hint bits");
  if (p.n_xres < 0 || p.n_xres > KE_MAX_POD_XRES) return fail(KE_ERR_INVALID, "pod n_xres out of range (0..8)");
  for (int e = 0; e < p.n_xres; e++) {
    if (p.xres_id[e] < 0 || p.xres_id[e] >= KE_MAX_XRES) return fail(KE_ERR_INVALID, "pod xres id out of range");
    if (p.xres_value[e] < 0) return fail(KE_ERR_INVALID, "negative pod xres value");
    for (int f = 0; f < e; f++)
      if (p.xres_id[f] == p.xres_id[e]) return fail(KE_ERR_INVALID, "pod xres id listed twice");
  }
  return KE_OK;
}

int validate_node_resources(int32_t n, const ke_node_resource* r) {
  if (n < 0 || n > KE_MAX_XRES || (n > 0 && !r)) return fail(KE_ERR_INVALID, "node resources: n out of range (0..64)");
  uint64_t seen = 0;
  for (int32_t e = 0; e < n; e++) {
    if (r[e].id < 0 || r[e].id >= KE_MAX_XRES) return fail(KE_ERR_INVALID, "node resource id out of range");
    if (seen >> r[e].id & 1) return fail(KE_ERR_INVALID, "node resource id listed twice");
    seen |= 1ull << r[e].id;
    if (r[e].allocatable < 0 || r[e].requested < 0) return fail(KE_ERR_INVALID, "negative node resource quantity");
  }
  return KE_OK;
}

int ext_slots(const ke_config& cfg, int32_t* ids) {
  int n = 0;
  auto add = [&](int32_t id) {
    for (int q = 0; q < n; q++)
      if (ids[q] == id) return;
    ids[n++] = id;
  };
  for (int q = 0; q < cfg.ext.n_fitplus && q < KE_MAX_FITPLUS; q++) ids[n++] = cfg.ext.fitplus[q].id;  // slot q = FitPlus q
  for (int q = 0; q < cfg.fit.n_resources && q < KE_MAX_FITPLUS; q++) add(cfg.fit.resources[q].id);
  for (int q = 0; q < cfg.fit.n_scalars && q < 8; q++) add(cfg.fit.scalars[q]);
  return n;
}

// ext row: per slot Allocatable / (NonZero)Requested (0 for a resource the node does not list), the pod room of
// NodeResourcesFit's Filter (AllowedPodNumber - len(Pods), the matched reservations' reserve pods removed), and the
// mask of ids with Allocatable > 0
void derive_ext_row(const ke_config& cfg, const NodeState& ns, int64_t* f, uint64_t* mask) {
  for (int w = 0; w < NUM_XF; w++) f[w] = 0;
  int32_t ids[2 * NUM_XS + KE_MAX_FITPLUS];
  const int nxs = std::min(ext_slots(cfg, ids), NUM_XS);
  uint64_t m = 0;
  for (const ke_node_resource& r : ns.xres) {
    if (r.allocatable > 0) m |= 1ull << r.id;
    for (int q = 0; q < nxs; q++)
      if (ids[q] == r.id) f[XF_ALLOC + q] = r.allocatable, f[XF_REQ + q] = xres_requested(ns, r);
  }
  f[XF_PODS] = (int64_t)ns.node.allowed_pods - ((int64_t)ns.node.pod_count + ns.rv_pods);
  *mask = m;
}

std::atomic<uint64_t> g_dirty_epoch{0};

int64_t xres_requested(const NodeState& ns, const ke_node_resource& r) {
  // cpu / memory rows carry NonZeroRequested: the reservation restore moves it too; scalars move with
  // NodeInfo.Requested.ScalarResources (updateNodeInfoRequested, transformer.go:491-504)
  return r.requested + (r.id == KE_RES_CPU || r.id == KE_RES_MEMORY ? ns.rv_nz[r.id] : rv_x_of(ns, r.id));
}

int64_t rv_x_of(const NodeState& ns, int32_t id) {
  for (const auto& e : ns.rv_x)
    if (e.first == id) return e.second;
  return 0;
}

int64_t pod_request_of(const ke_pod& pod, int32_t id) {
  if (id == KE_XRES_CPU) return pod.requests[KE_RES_CPU];
  if (id == KE_XRES_MEMORY) return pod.requests[KE_RES_MEMORY];
  for (int e = 0; e < pod.n_xres && e < KE_MAX_POD_XRES; e++)
    if (pod.xres_id[e] == id) return pod.xres_value[e];
  return 0;
}

using XDelta = std::vector<std::pair<int32_t, int64_t>>;
static void x_add(XDelta* x, int32_t id, int64_t d) {
  if (!x) return;
  for (auto& e : *x)
    if (e.first == id) {
      e.second += d;
      return;
    }
  x->push_back({id, d});
}
static int64_t x_get(const XDelta& x, int32_t id) {
  for (const auto& e : x)
    if (e.first == id) return e.second;
  return 0;
}
// reservation i's entries beyond cpu / memory (none without ke_reservations_load_full)
static const std::vector<ke_reservation_resource>& resv_entries(const Context& c, int32_t i) {
  static const std::vector<ke_reservation_resource> none;
  return (size_t)i < c.resv_res.size() ? c.resv_res[(size_t)i] : none;
}

// The reservation cache's NodeInfo restore (BeforePreFilter, transformer.go:147-300).  A reservation that is
// available and not AllocateOnce with allocated pods takes part (transformer.go:181-190); for a pod that does
// not match it, it is "unmatched" when it has allocated pods and restoreUnmatchedReservations
// (transformer.go:447-473) removes its reserve pod (requests = allocatable) from NodeInfo and adds back a pod
// requesting SubtractWithNonNegativeResult(allocatable, allocated) when that is not zero; for a pod that
// matches it, restoreMatchedReservation (:422-445) removes the reserve pod.  updateNodeInfoRequested /
// NodeInfo.RemovePod move NonZeroRequested with the 100m / 200Mi defaults of a zero cpu / memory request
// (the reserve pod taken as one container).
static int64_t resv_non0(int k, int64_t v) { return v != 0 ? v : (k == KE_RES_CPU ? 100 : 200LL << 20); }
bool resv_usable(const ke_reservation& r) { return r.available && !(r.allocate_once && r.allocated_pods > 0); }

// node's Requested / NonZeroRequested deltas with `matched` (by reservation index, nullptr = none) matched; `x`:
// the NodeInfo.Requested.ScalarResources deltas by resource id of their entries beyond cpu / memory
static void resv_delta(const Context& c, int32_t node, const std::vector<char>* matched, bool with_matched,
                       int64_t* req, int64_t* nz, int32_t* pods = nullptr, XDelta* x = nullptr) {
  for (int k = 0; k < KE_NRES; k++) req[k] = nz[k] = 0;
  if (pods) *pods = 0;
  if (x) x->clear();
  for (int32_t i : c.resv_by_node[(size_t)node]) {
    const ke_reservation& r = c.resv[(size_t)i];
    if (!resv_usable(r)) continue;
    const std::vector<ke_reservation_resource>& ex = resv_entries(c, i);
    if (matched && (*matched)[(size_t)i]) {
      if (!with_matched) continue;
      if (pods) --*pods;  // NodeInfo.RemovePod(reservePod)
      for (int k = 0; k < KE_NRES; k++) {
        req[k] -= r.allocatable[k];
        nz[k] -= resv_non0(k, r.allocatable[k]);
      }
      for (const ke_reservation_resource& e : ex)
        if (e.id != KE_RSV_RES_PODS) x_add(x, e.id, -e.allocatable);
      continue;
    }
    if (r.allocated_pods == 0) continue;
    int64_t rem[KE_NRES];
    bool rem_nz = false;  // quotav1.IsZero(SubtractWithNonNegativeResult(Allocatable, Allocated)) over every name
    for (int k = 0; k < KE_NRES; k++) {
      rem[k] = r.allocatable[k] > r.allocated[k] ? r.allocatable[k] - r.allocated[k] : 0;
      rem_nz = rem_nz || rem[k] != 0;
    }
    for (const ke_reservation_resource& e : ex) rem_nz = rem_nz || e.allocatable > e.allocated;
    for (int k = 0; k < KE_NRES; k++) {
      req[k] += -r.allocatable[k] + rem[k];
      nz[k] += -resv_non0(k, r.allocatable[k]) + (rem_nz ? resv_non0(k, rem[k]) : 0);
    }
    for (const ke_reservation_resource& e : ex)
      if (e.id != KE_RSV_RES_PODS)
        x_add(x, e.id, -e.allocatable + (e.allocatable > e.allocated ? e.allocatable - e.allocated : 0));
  }
}

// The NodeNUMAResource / DeviceShare restore states of the reservations holding allocations that a pod does not
// match: mergedUnmatchedUsed (nodenumaresource/reservation.go:111-120, deviceshare/reservation.go:99-108) over the
// node's unmatched reservations with allocated pods (transformer.go:195-199), each one's
//   used = subtractAllocated(copy(allocatable), remained, true),  remained = allocatable - allocated
// which per NUMA id / device instance and key is the owners' amount where the reserve pod holds that key (keys of
// both lists kept, the ResourceList arithmetic of quotav1) -- the part the node allocation counts twice.
// ignored: a reservation-ignored pod's rows (every reservation matchedOrIgnored) -- NodeNUMAResource's reusable
// resources are then mergedMatchedAllocatable, the reserve pods' whole NUMA allocations: the hint view
// (GetTopologyHints, resource_manager.go:130-138) and tryAllocateIgnoreReservation's mergedMatchedAllocated + Σ
// remained (nodenumaresource/reservation.go:437-490), equal in value
static void resv_plugin_restore(const Context& c, int32_t node, const std::vector<char>* matched, NodeState& ns,
                                bool ignored = false) {
  std::memset(ns.rv_numa, 0, sizeof ns.rv_numa);
  std::memset(ns.rv_dev, 0, sizeof ns.rv_dev);
  ns.rv_numa_keys = 0;
  ns.rv_numa_zones = 0;
  ns.rv_dev_minors = 0;
  for (int k = 0; k < KE_DKEYS; k++) ns.rv_dev_keys[k] = 0;
  if (c.resv_alloc.empty()) return;
  for (int32_t i : c.resv_by_node[(size_t)node]) {
    const ke_reservation& r = c.resv[(size_t)i];
    if (ignored && resv_usable(r)) {
      const ke_reservation_alloc& a = c.resv_alloc[(size_t)i];
      for (int id = 0; id < KE_MAX_NUMA; id++)
        for (int q = 0; q < KE_NRES; q++) {
          const int j = 2 * id + q;
          if (a.numa[j] == 0) continue;
          ns.rv_numa_zones |= (uint8_t)(1u << id);
          ns.rv_numa_keys |= 1u << j;
          ns.rv_numa[j] += a.numa[j];
        }
      continue;
    }
    if (!resv_usable(r) || (matched && (*matched)[(size_t)i]) || r.allocated_pods == 0) continue;
    const ke_reservation_alloc& a = c.resv_alloc[(size_t)i];
    // NodeNUMAResource (RestoreReservation, reservation.go:196-209): only with the reserve pod's NUMA resources
    bool any = false;
    for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++) any = any || a.numa[j] != 0;
    if (any)
      for (int id = 0; id < KE_MAX_NUMA; id++) {
        const bool in_a = a.numa[2 * id] != 0 || a.numa[2 * id + 1] != 0;
        const bool in_b = a.owner_numa[2 * id] != 0 || a.owner_numa[2 * id + 1] != 0;
        if (!in_a && !in_b) continue;
        ns.rv_numa_zones |= (uint8_t)(1u << id);
        for (int r = 0; r < KE_NRES; r++) {
          const int j = 2 * id + r;
          if (a.numa[j] == 0 && a.owner_numa[j] == 0) continue;
          ns.rv_numa_keys |= 1u << j;
          // used = SubtractWithNonNegativeResult(allocatable, allocatable - allocated) = the owners' amount, also
          // on ids / keys the reserve pod does not hold (an owner allocated from the node, assumed into it)
          if (a.owner_numa[j] > 0) ns.rv_numa[j] += a.owner_numa[j];
        }
      }
    // DeviceShare (RestoreReservation, deviceshare/reservation.go:157-172): the owners' usage on the reserve pod's
    // instances (appendAllocatedByHints); an instance whose used is zero leaves the map (deviceResources.subtract)
    for (int t = 0; t < KE_DEV_TYPES; t++)
      for (int m = 0; m < KE_MAX_MINORS; m++) {
        const uint64_t bit = 1ull << (16 * t + m);
        if (!(a.device_minors & bit)) continue;
        bool nz = false;
        for (int k = 0; k < KE_DKEYS; k++) nz = nz || (a.device[t][m][k] != 0 && a.owner_device[t][m][k] > 0);
        if (!nz) continue;
        ns.rv_dev_minors |= bit;
        for (int k = 0; k < KE_DKEYS; k++) {
          if (a.device[t][m][k] == 0 && a.owner_device[t][m][k] == 0) continue;
          ns.rv_dev_keys[k] |= bit;
          if (a.device[t][m][k] != 0 && a.owner_device[t][m][k] > 0) ns.rv_dev[t][m][k] += a.owner_device[t][m][k];
        }
      }
  }
}

void resv_node_restore(Context& c, int32_t node) {
  NodeState& ns = c.nodes[(size_t)node];
  resv_delta(c, node, nullptr, false, ns.rv_req, ns.rv_nz, &ns.rv_pods, &ns.rv_x);
  resv_plugin_restore(c, node, nullptr, ns);
  ns.dirty = true;
}

// KE_RSV_HOLDS_* of a holdings record
uint8_t resv_holds_of(const ke_reservation_alloc& a) {
  uint8_t h = 0;
  for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++) h |= a.numa[j] != 0 ? KE_RSV_HOLDS_NUMA : 0;
  for (int w = 0; w < 4; w++) h |= a.cpuset[w] ? KE_RSV_HOLDS_CPUSET : 0;
  if (a.device_minors) h |= KE_RSV_HOLDS_DEVICES;
  return h;
}

int load_reservations(Context& c, int32_t n, const ke_reservation* rs, const ke_reservation_alloc* allocs,
                      const int32_t* res_off, const ke_reservation_resource* res) {
  if (n < 0 || (n > 0 && !rs)) return fail(KE_ERR_INVALID, "reservations");
  if (res_off && res_off[0] != 0) return fail(KE_ERR_INVALID, "reservation resource offsets");
  for (int32_t i = 0; i < n; i++) {
    const ke_reservation& r = rs[i];
    if (r.node < 0 || r.node >= c.n_nodes) return fail(KE_ERR_NOT_FOUND, "reservation node index");
    if (r.allocated_pods < 0) return fail(KE_ERR_INVALID, "negative reservation allocated pods");
    if (r.allocate_policy > KE_RSV_POLICY_RESTRICTED) return fail(KE_ERR_INVALID, "reservation allocate policy");
    for (int k = 0; k < KE_NRES; k++)
      if (r.allocatable[k] < 0 || r.allocated[k] < 0 || r.reserved[k] < 0)
        return fail(KE_ERR_INVALID, "negative reservation quantity");
    if (r.names_excluded & ~3u) return fail(KE_ERR_INVALID, "ke_reservation.names_excluded");
    // the holdings come with the record (ke_reservations_load_ex); a holds bit without one has nothing to restore
    // from: refused rather than scheduled around without the NUMA / cpuset / device restore (koord_eval.h)
    const uint8_t held = allocs ? resv_holds_of(allocs[i]) : 0;
    const uint8_t said = r.holds & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET | KE_RSV_HOLDS_DEVICES);
    if (!allocs && said)
      return fail(KE_ERR_UNSUPPORTED, "a reservation holding NUMA / cpuset / device allocations without its "
                                      "ke_reservation_alloc (ke_reservations_load_ex)");
    if (allocs && said != held) return fail(KE_ERR_INVALID, "ke_reservation.holds disagrees with its ke_reservation_alloc");
    if (allocs) {
      const ke_reservation_alloc& a = allocs[i];
      for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++)
        if (a.numa[j] < 0 || a.owner_numa[j] < 0) return fail(KE_ERR_INVALID, "negative reservation NUMA amount");
      for (int t = 0; t < KE_DEV_TYPES; t++)
        for (int m = 0; m < KE_MAX_MINORS; m++)
          for (int k = 0; k < KE_DKEYS; k++) {
            const int64_t v = a.device[t][m][k], o = a.owner_device[t][m][k];
            if (v < 0 || o < 0) return fail(KE_ERR_INVALID, "negative reservation device amount");
            if (k >= (t == KE_DEV_GPU ? 3 : 1) && (v || o)) return fail(KE_ERR_INVALID, "reservation device key of another type");
            if (v && !(a.device_minors >> (16 * t + m) & 1)) return fail(KE_ERR_INVALID, "reservation device amount off its minors");
            if (o && !(a.owner_device_minors >> (16 * t + m) & 1))
              return fail(KE_ERR_INVALID, "reservation owner device amount off its minors");
          }
      if ((a.device_minors | a.owner_device_minors) & ~0x0000FFFFFFFFFFFFull)
        return fail(KE_ERR_INVALID, "reservation device minors beyond the three types");
    }
    // the allocatable names beyond cpu / memory: with their entries (ke_reservations_load_full), else refused
    const int32_t ne = res_off ? res_off[i + 1] - res_off[i] : 0;
    if (ne < 0 || (ne > 0 && !res)) return fail(KE_ERR_INVALID, "reservation resource offsets");
    if (!res_off && (r.holds & KE_RSV_OTHER_ALLOCATABLE))
      return fail(KE_ERR_UNSUPPORTED, "a reservation whose allocatable names resources other than cpu / memory, "
                                      "without its resource entries (ke_reservations_load_full)");
    if (res_off && ((r.holds & KE_RSV_OTHER_ALLOCATABLE) != 0) != (ne > 0))
      return fail(KE_ERR_INVALID, "KE_RSV_OTHER_ALLOCATABLE disagrees with the reservation's resource entries");
    uint64_t seen = 0;
    bool pods_seen = false;
    for (int32_t j = 0; j < ne; j++) {
      const ke_reservation_resource& e = res[res_off[i] + j];
      if (e.id == KE_RSV_RES_PODS) {
        if (pods_seen) return fail(KE_ERR_INVALID, "duplicate reservation resource id");
        pods_seen = true;
      } else {
        if (e.id == KE_XRES_CPU || e.id == KE_XRES_MEMORY || e.id < 0 || e.id >= KE_MAX_XRES)
          return fail(KE_ERR_INVALID, "reservation resource id (cpu / memory go in ke_reservation)");
        if (seen >> e.id & 1) return fail(KE_ERR_INVALID, "duplicate reservation resource id");
        seen |= 1ull << e.id;
      }
      if (e.allocatable <= 0 || e.allocated < 0 || e.reserved < 0) return fail(KE_ERR_INVALID, "reservation resource quantity");
      if (e.excluded > 1) return fail(KE_ERR_INVALID, "ke_reservation_resource.excluded");
    }
    if (r.holds & ~15u) return fail(KE_ERR_INVALID, "unknown ke_reservation.holds bits");
  }
  std::vector<int32_t> old;
  for (const ke_reservation& r : c.resv) old.push_back(r.node);
  c.resv.assign(rs, rs + n);
  if (allocs) c.resv_alloc.assign(allocs, allocs + n);
  else c.resv_alloc.clear();
  c.resv_res.assign((size_t)n, {});
  for (int32_t i = 0; res_off && i < n; i++) c.resv_res[(size_t)i].assign(res + res_off[i], res + res_off[i + 1]);
  c.resv_cpu_cnt.clear();
  c.resv_holds.assign((size_t)n, 0);
  for (int32_t i = 0; allocs && i < n; i++) c.resv_holds[(size_t)i] = resv_holds_of(allocs[i]);
  c.resv_by_node.assign(c.nodes.size(), {});
  for (int32_t i = 0; i < n; i++) c.resv_by_node[(size_t)rs[i].node].push_back(i);
  for (int32_t node : old) resv_node_restore(c, node);  // the old restore leaves
  for (const ke_reservation& r : c.resv) resv_node_restore(c, r.node);
  c.last_resv.clear();  // release records of earlier calls no longer name these reservations
  c.resv_gen++;
  return KE_OK;
}

// FilterNominateReservation -> filterWithReservations(..., requiredFromReservation = true) for one matched
// reservation (plugin.go:351-442, 707-738): a resource name of rInfo.ResourceNames shared with the pod, fitsNode
// over the restored NodeInfo (plugin.go:447-497; preemptible empty) and, for Restricted, fitsReservation
// (plugin.go:499-569).  podRequested = Requested after the unmatched restore only (`ureq`, `ux`: its scalar part's
// restore delta), allRAllocated = Σ allocated of the node's matched reservations (`all_alloc`, `all_x`).
// With a reservation affinity the name check is skipped (the pod may use any matched reservation, :373).
// The pod-count check of fitsNode (plugin.go:450-453) reads len(NodeInfo.Pods) of the snapshot NodeInfo, which
// the BeforePreFilter restore already left without the matched reserve pods (restoreMatchedReservation ->
// RemovePod, transformer.go:440), and subtracts len(matchedOrIgnored) once more: `pods_restored` is the former.
// rInfo.GetAvailable() = SubtractWithNonNegativeResult(Allocatable - Allocated, Reserved) (reservation_info.go:484-488).
static bool resv_nominable(const Context& c, int32_t ri, const ke_pod& pod, const NodeState& ns,
                           const int64_t* pod_requested, const XDelta& ux, const int64_t* all_allocated,
                           const XDelta& all_x, bool affinity, int64_t pods_restored, int64_t n_matched,
                           int64_t allowed_pods) {
  const ke_reservation& r = c.resv[(size_t)ri];
  const std::vector<ke_reservation_resource>& ex = resv_entries(c, ri);
  bool shared = false;  // quotav1.Intersection(rInfo.ResourceNames, ResourceNames(podRequests))
  for (int k = 0; k < KE_NRES; k++)
    shared = shared || (r.allocatable[k] != 0 && !(r.names_excluded >> k & 1) && pod.requests[k] != 0);
  for (const ke_reservation_resource& e : ex)
    shared = shared || (!e.excluded && e.id != KE_RSV_RES_PODS && pod_request_of(pod, e.id) != 0);
  if (!shared && !affinity) return false;
  bool node_fits = pods_restored - n_matched + 1 <= allowed_pods;
  bool other = false;  // ephemeral storage / scalar requests (framework.Resource.ScalarResources): ke_pod.xres
  for (int e = 0; e < pod.n_xres; e++)
    other = other || (pod.xres_id[e] != KE_XRES_CPU && pod.xres_id[e] != KE_XRES_MEMORY && pod.xres_value[e] != 0);
  auto avail = [](int64_t a, int64_t al, int64_t rs) { return a - al - rs > 0 ? a - al - rs : 0; };
  if (pod.requests[KE_RES_CPU] != 0 || pod.requests[KE_RES_MEMORY] != 0 || other) {  // else pods only (:455-460)
    const int64_t* alloc = ns.node.allocatable;
    for (int k = 0; k < KE_NRES; k++) {
      const int64_t remained = avail(r.allocatable[k], r.allocated[k], r.reserved[k]);
      if (pod.requests[k] > alloc[k] - (pod_requested[k] - remained - all_allocated[k])) node_fits = false;
    }
    for (int e = 0; e < pod.n_xres; e++) {  // (plugin.go:487-495)
      const int32_t id = pod.xres_id[e];
      if (id == KE_XRES_CPU || id == KE_XRES_MEMORY || pod.xres_value[e] == 0) continue;
      int64_t a = 0, q = x_get(ux, id), remained = 0;
      for (const ke_node_resource& x : ns.xres)
        if (x.id == id) a = x.allocatable, q += x.requested;
      for (const ke_reservation_resource& re : ex)
        if (re.id == id) remained = avail(re.allocatable, re.allocated, re.reserved);
      if (pod.xres_value[e] > a - (q - remained - x_get(all_x, id))) node_fits = false;
    }
  }
  bool resv_fits = node_fits;
  if (r.allocate_policy == KE_RSV_POLICY_RESTRICTED) {
    resv_fits = true;
    for (const ke_reservation_resource& e : ex)  // "pods" reserved explicitly: one more assigned pod fits (:511-527)
      if (e.id == KE_RSV_RES_PODS && (int64_t)r.allocated_pods + 1 > e.allocatable) resv_fits = false;
    // Mask(podRequests, ResourceNames), zero requests skipped: requested <= capacity - reserved - allocated
    for (int k = 0; k < KE_NRES; k++)
      if (r.allocatable[k] != 0 && !(r.names_excluded >> k & 1) && pod.requests[k] != 0 &&
          pod.requests[k] > r.allocatable[k] - r.reserved[k] - r.allocated[k])
        resv_fits = false;
    for (const ke_reservation_resource& e : ex) {
      if (e.excluded || e.id == KE_RSV_RES_PODS) continue;
      const int64_t q = pod_request_of(pod, e.id);
      if (q != 0 && q > e.allocatable - e.reserved - e.allocated) resv_fits = false;
    }
  }
  return node_fits && resv_fits;
}

// scoreReservation (scoring.go:191-210): MostAllocated of (pod requests + allocated) over the reservation's
// non-zero allocatable (every name, "pods" too), MaxNodeScore * req.MilliValue() / capacity.MilliValue() per
// resource that fits, averaged over all of them (exact in 128-bit: Go's int64 product wraps only beyond ~9.2e13
// bytes of a non-cpu resource)
int32_t resv_score(const Context& c, int32_t i, const ke_pod& pod) {
  const ke_reservation& r = c.resv[(size_t)i];
  int64_t s = 0, w = 0;
  auto term = [&](int64_t req, int64_t cap, bool milli) {
    w++;
    if (req <= cap) {
      const __int128 m = milli ? 1 : 1000;
      s += (int64_t)((__int128)100 * req * m / ((__int128)cap * m));
    }
  };
  for (int k = 0; k < KE_NRES; k++)
    if (r.allocatable[k] != 0) term(pod.requests[k] + r.allocated[k], r.allocatable[k], k == KE_RES_CPU);
  for (const ke_reservation_resource& e : resv_entries(c, i))
    term((e.id == KE_RSV_RES_PODS ? 0 : pod_request_of(pod, e.id)) + e.allocated, e.allocatable, false);
  return w ? (int32_t)(s / w) : 0;
}

int resv_check(const Context& c, const int32_t* ids, int32_t n_ids) {
  for (int32_t j = 0; j < n_ids; j++) {
    if (ids[j] < 0 || ids[j] >= (int32_t)c.resv.size()) return fail(KE_ERR_NOT_FOUND, "matched reservation index");
  }
  return KE_OK;
}

// A reservation-ignored pod (apis/extension/reservation.go:97-99) takes every available reservation of every node
// as matchedOrIgnored (transformer.go:101-106, 181-199): restoreMatchedReservation removes each reserve pod from
// NodeInfo and no unmatched restore is left; the Reservation plugin's Filter passes (filterWithReservations without
// an affinity, plugin.go:350-353), PreScore / Score skip it (scoring.go:48-50) and Reserve assumes it into no
// reservation (plugin.go:755-761).  NodeNUMAResource / DeviceShare allocate it from the node and the ignored
// reservations' unallocated remainder (tryAllocateIgnoreReservation, nodenumaresource/reservation.go:437-490,
// deviceshare/reservation.go:290-310): for a pod binding CPUs on a node without a NUMA policy that remainder is
// the held CPUs, tried as the preferred CPUs of one allocation (resv_ignore_views); for a pod binding no CPUs the
// held NUMA amounts are reusable resources (resv_plugin_restore, ignored); for a DeviceShare pod the held devices
// are views (resv_ds_views).  Refused: a binding pod with its own NUMA policy while a reservation holds NUMA
// resources or CPUs, a binding pod while one of those sits on a NUMA-policy node (its hints over the held CPUs),
// a DeviceShare pod with hints or a NUMA policy (pod or node) beside held devices.
int resv_ignore_check(const Context& c, const ke_pod& pod, uint32_t pod_flags) {
  // a pod binding no CPUs reads held NUMA amounts only as reusable resources, which its rows carry
  // (resv_plugin_restore, ignored); a binding one's NUMA hints would trim them by the held CPUs (not restated)
  const bool binds = (pod_flags & PF_CPUSET) || (c.n_bind_nodes > 0 && pod.requests[KE_RES_CPU] > 0);
  bool dev = false, numa_cpu = false, on_policy_node = false;
  for (size_t i = 0; i < c.resv_holds.size(); i++) {
    const uint8_t h = c.resv_holds[i];
    dev = dev || (h & KE_RSV_HOLDS_DEVICES);
    if (h & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)) {
      numa_cpu = true;
      on_policy_node = on_policy_node || c.nodes[(size_t)c.resv[i].node].node.numa_topology_policy != KE_NUMA_POLICY_NONE;
    }
  }
  // a DeviceShare pod allocates from the held devices (resv_ds_views' ignore view) -- not with device hints, nor in
  // NUMA hints (its own NUMA policy, or a device-holding reservation on a NUMA-policy node)
  bool dev_on_policy = false;
  for (size_t i = 0; i < c.resv_holds.size(); i++)
    if (c.resv_holds[i] & KE_RSV_HOLDS_DEVICES)
      dev_on_policy = dev_on_policy || c.nodes[(size_t)c.resv[i].node].node.numa_topology_policy != KE_NUMA_POLICY_NONE;
  const bool ds = (pod_flags & (PF_DS | PF_DS_HINT)) != 0;
  // a binding pod under a NUMA policy beside held NUMA resources / CPUs: tryAllocateIgnoreReservation in its hints
  // (k_numa_views, resv_ignore_views) -- not with fractional CPUs or a required FullPCPUs binding (the pod's, or a
  // FullPCPUsOnly node's among the holding ones: preferredCPUs taken first may split cores)
  const int preq = pf_cpu_required(pod_flags);
  bool full_req = preq == XB_FULL;
  for (size_t i = 0; preq == XB_NONE && i < c.resv_holds.size(); i++)
    if ((c.resv_holds[i] & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)) &&
        c.nodes[(size_t)c.resv[i].node].node.cpu_bind_policy == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY)
      full_req = true;
  const bool pol_here = (numa_cpu && pod.numa_topology_policy != KE_NUMA_POLICY_NONE) || on_policy_node;
  if ((dev && ds && ((pod_flags & PF_DS_HINT) || pod.numa_topology_policy != KE_NUMA_POLICY_NONE || dev_on_policy)) ||
      (binds && pol_here && (!(pod_flags & PF_CPU_INT) || full_req)))
    return fail(KE_ERR_UNSUPPORTED, "a reservation-ignored pod reading resources a reservation holds "
                                    "(tryAllocateIgnoreReservation's remainder)");
  return KE_OK;
}

void resv_ignore_begin(Context& c) {
  const std::vector<char> all(c.resv.size(), 1);
  for (size_t node = 0; node < c.resv_by_node.size(); node++) {
    if (c.resv_by_node[node].empty()) continue;
    NodeState& ns = c.nodes[node];
    resv_delta(c, (int32_t)node, &all, true, ns.rv_req, ns.rv_nz, &ns.rv_pods, &ns.rv_x);
    resv_plugin_restore(c, (int32_t)node, &all, ns, true);
    ns.dirty = true;
  }
}

void resv_ignore_end(Context& c) {
  for (const RsvOvr& o : c.rsv_ovr) c.nodes[(size_t)o.node].rsv_ovr = false;
  c.rsv_ovr.clear();
  c.rsv_views.clear();
  c.rsv_view_resv.clear();
  c.rsv_view_out.clear();
  c.ds_views.clear();
  c.ds_view_resv.clear();
  c.ds_view_out.clear();
  c.numa_views.clear();
  c.numa_view_ids.clear();
  c.numa_view_out.clear();
  c.numa_cs_views.clear();
  c.numa_cs_ovr.clear();
  c.numa_cs_pair.clear();
  c.numa_cs_out.clear();
  for (size_t node = 0; node < c.resv_by_node.size(); node++)
    if (!c.resv_by_node[node].empty()) resv_node_restore(c, (int32_t)node);
}

static bool resv_holds_cpu(const Context& c, int32_t i);
static bool pod_binds_on(const DevPod& dp, const NodeState& ns);

bool resv_ignore_needs_views(const Context& c, const ke_pod& pod, uint32_t pod_flags) {
  const bool binds = (pod_flags & PF_CPUSET) || (c.n_bind_nodes > 0 && pod.requests[KE_RES_CPU] > 0);
  const bool ds = (pod_flags & PF_DS) && !(pod_flags & PF_DS_INVALID);
  for (size_t i = 0; i < c.resv_holds.size(); i++) {
    if (binds && (c.resv_holds[i] & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET))) return true;
    if (ds && (c.resv_holds[i] & KE_RSV_HOLDS_DEVICES)) return true;
  }
  return false;
}

// tryAllocateIgnoreReservation for a reservation-ignored pod binding CPUs (nodenumaresource/reservation.go:437-490):
// on every node without a NUMA policy whose usable reservations hold NUMA resources or CPUs (RestoreReservation's
// matched set), one allocation with reservedCPUsFromIgnored = their allocatable CPUs (mergedMatchedAllocatedCPUs,
// the remainedCPUs inside them) preferred and no required resources
// Under a NUMA policy (the pod's or the node's) the same allocation is every mask's Allocate of its hints: one
// k_numa_views set per such node (resv_ignore_ovr: the Filter, and the cpuset pass for Score / Reserve) -- the trial
// prefers reservedCPUsFromIgnored, the hint view mergedMatchedRemainCPUs, and the reusable amounts are the rows' own
// (the ignored restore, resv_plugin_restore).
void resv_ignore_views(Context& c, const ke_pod& pod) {
  c.rsv_views.clear();
  c.rsv_view_resv.clear();
  c.rsv_view_out.clear();
  c.numa_views.clear();
  c.numa_view_ids.clear();
  c.numa_view_out.clear();
  if (c.resv_alloc.empty()) return;
  const DevPod dp = make_dev_pod(c.cfg, pod, pod_hints(c, pod), &c.tmpl);
  for (size_t node = 0; node < c.resv_by_node.size(); node++) {
    if (c.resv_by_node[node].empty()) continue;
    const NodeState& ns = c.nodes[node];
    if (!pod_binds_on(dp, ns) || !cpus_valid(ns)) continue;
    if (ns.node.numa_topology_policy != KE_NUMA_POLICY_NONE || pod.numa_topology_policy != KE_NUMA_POLICY_NONE) {
      std::vector<int32_t> mine;
      for (int32_t i : c.resv_by_node[node])
        if (resv_usable(c.resv[(size_t)i]) && resv_holds_cpu(c, i)) mine.push_back(i);
      if (mine.empty()) continue;
      c.numa_views.emplace_back();
      NumaRsvView& v = c.numa_views.back();
      std::memset(&v, 0, sizeof v);
      v.node = (int32_t)node;
      v.n = 1;
      v.required = 1;  // tryAllocateIgnoreReservation's status: no allocation from the node besides it
      for (const ke_numa_zone& z : ns.zones)
        if (z.id >= 0 && z.id < KE_MAX_NUMA && (z.has_allocated & KE_NUMA_ALLOC_ENTRY)) v.entry |= 1u << z.id;
      for (int32_t i : mine)
        for (int w = 0; w < 4; w++) {
          const ke_reservation_alloc& a = c.resv_alloc[(size_t)i];
          v.pref[NV_MAX][w] |= a.cpuset[w] & ~a.owner_cpuset[w];  // mergedMatchedRemainCPUs
          v.pref[0][w] |= a.cpuset[w];                            // reservedCPUsFromIgnored
        }
      c.numa_view_ids.push_back({-2});
      continue;
    }
    RsvView v{};
    bool any = false;
    for (int32_t i : c.resv_by_node[node])
      if (resv_usable(c.resv[(size_t)i]) && resv_holds_cpu(c, i)) {
        any = true;
        for (int w = 0; w < 4; w++) v.pref[w] |= c.resv_alloc[(size_t)i].cpuset[w];
      }
    if (!any) continue;
    v.node = (int32_t)node;
    c.rsv_views.push_back(v);
    c.rsv_view_resv.push_back(-1);
  }
}

// the trials' outcome as the Filter's and Reserve's decisions (a failed allocation fails both: the status is
// returned, plugin.go:384-387 and :554-558)
// DeviceShare (resv_ds_views with every reservation matchedOrIgnored): Filter and Reserve from the ignore view (-2,
// tryAllocateIgnoreReservation, reservation.go:221-223, 381-385), Score from the node's own (-1: no nominated
// reservation, scoring.go:96-102)
void resv_ignore_ovr(Context& c) {
  c.rsv_ovr.clear();
  auto ovr_of = [&](int32_t node) -> RsvOvr& {
    for (RsvOvr& o : c.rsv_ovr)
      if (o.node == node) return o;
    c.rsv_ovr.emplace_back();
    RsvOvr& o = c.rsv_ovr.back();
    std::memset(&o, 0, sizeof o);
    o.node = node;
    NodeState& ns = c.nodes[(size_t)node];
    ns.rsv_ovr = true;
    ns.dirty = true;
    return o;
  };
  for (size_t q = 0; q < c.rsv_views.size(); q++) {
    RsvOvr& o = ovr_of(c.rsv_views[q].node);
    const bool ok = c.rsv_view_out.size() > q && c.rsv_view_out[q].ok;
    o.filter = o.reserve = (int8_t)(ok ? 1 : 2);
    if (ok)
      for (int w = 0; w < 4; w++) o.cpus[w] = c.rsv_view_out[q].cpus[w];
  }
  // NodeNUMAResource under a NUMA policy: the Filter's outcome over tryAllocateIgnoreReservation, then the cpuset pass
  // (k_rsv_views over the allocation's zones) for Reserve's cpuset and the Score (resv_numa_cs_apply)
  c.numa_cs_views.clear();
  c.numa_cs_ovr.clear();
  c.numa_cs_pair.clear();
  c.numa_cs_out.clear();
  for (size_t q = 0; q < c.numa_views.size() && q < c.numa_view_out.size(); q++) {
    const NumaRsvOut& r = c.numa_view_out[q];
    const NumaRsvView& nv = c.numa_views[q];
    RsvOvr& o = ovr_of(nv.node);
    o.numa_on = 1;
    o.numa_st = (uint8_t)r.st;
    o.numa_reason = (uint8_t)r.reason;
    o.numa_aff = (uint8_t)r.aff;
    std::memcpy(o.numa_dist, r.dist[0], sizeof o.numa_dist);
    if (r.st != KE_CODE_SUCCESS) continue;
    if (!(r.ok & 1u)) {  // (the Filter's Allocate on the affinity succeeded: not reached)
      o.numa_st = KE_CODE_UNSCHEDULABLE;
      o.numa_reason = KE_REASON_NUMA_INSUFFICIENT_CPUS;
      continue;
    }
    RsvView v{};
    v.node = nv.node;
    for (int w = 0; w < 4; w++) v.pref[w] = v.pref2[w] = nv.pref[0][w];
    for (int z = 0; z < 8; z++)
      if (r.dist[0][2 * z] != 0 || r.dist[0][2 * z + 1] != 0) {
        v.zmask |= 1 << z;
        v.zcpu[z] = r.dist[0][2 * z];
      }
    v.score_on = 1;
    v.sreq1 = r.sreq1[0];
    v.salloc[0] = r.salloc[0][0];
    v.salloc[1] = r.salloc[0][1];
    c.numa_cs_views.push_back(v);
    c.numa_cs_ovr.push_back((int32_t)(&o - c.rsv_ovr.data()));
    c.numa_cs_pair.push_back(-1);
  }
  for (size_t q = 0; q < c.ds_views.size() && q < c.ds_view_out.size(); q++) {
    RsvOvr& o = ovr_of(c.ds_views[q].node);
    const DsViewOut& v = c.ds_view_out[q];
    o.ds_on = 1;
    if (c.ds_view_resv[q] == -1) {
      o.ds_raw = (int16_t)v.raw;
    } else {
      o.ds_st = (uint8_t)v.st;
      o.ds_reason = (uint8_t)v.reason;
      o.ds_res = (int8_t)(v.st == KE_CODE_SUCCESS && v.minors ? 1 : 2);
      o.ds_minors = v.minors;
    }
  }
}

// requestCPUBind of the pod on the node (util.go:121-138): its own cpuset state, else a node CPU bind policy
// binding a whole-CPU request
static bool pod_binds_on(const DevPod& dp, const NodeState& ns) {
  if (dp.flags & PF_NUMA_SKIP) return false;
  if (dp.flags & PF_CPU_RCB) return true;
  return dp.req[0] != 0 && ns.node.cpu_bind_policy != KE_NODE_CPU_BIND_NONE && (dp.flags & PF_CPU_INT);
}
static bool resv_holds_cpu(const Context& c, int32_t i) {
  return !c.resv_holds.empty() && (c.resv_holds[(size_t)i] & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET));
}

void resv_views(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids) {
  c.rsv_views.clear();
  c.rsv_view_resv.clear();
  c.rsv_view_out.clear();
  if (c.resv_alloc.empty()) return;
  const DevPod dp = make_dev_pod(c.cfg, pod, pod_hints(c, pod), &c.tmpl);
  std::vector<char> m(c.resv.size(), 0);
  for (int32_t j = 0; j < n_ids; j++)
    if (resv_usable(c.resv[(size_t)ids[j]])) m[(size_t)ids[j]] = 1;
  std::vector<int32_t> nodes;
  for (int32_t j = 0; j < n_ids; j++)
    if (m[(size_t)ids[j]] && resv_holds_cpu(c, ids[j])) nodes.push_back(c.resv[(size_t)ids[j]].node);
  std::sort(nodes.begin(), nodes.end());
  nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
  for (int32_t node : nodes) {
    const NodeState& ns = c.nodes[(size_t)node];
    // under a NUMA policy (the pod's or the node's) the trials are k_numa_views'; a pod binding no CPUs there
    // allocates no cpuset
    if (ns.node.numa_topology_policy != KE_NUMA_POLICY_NONE || pod.numa_topology_policy != KE_NUMA_POLICY_NONE ||
        !pod_binds_on(dp, ns) || !cpus_valid(ns))
      continue;
    uint64_t merged[4] = {0, 0, 0, 0};  // mergedMatchedAllocatedCPUs: the matched ones' allocatable CPUs
    for (int32_t i : c.resv_by_node[(size_t)node])
      if (m[(size_t)i] && resv_holds_cpu(c, i))
        for (int w = 0; w < 4; w++) merged[w] |= c.resv_alloc[(size_t)i].cpuset[w];
    for (int32_t i : c.resv_by_node[(size_t)node]) {
      if (!m[(size_t)i] || !resv_holds_cpu(c, i)) continue;
      const ke_reservation_alloc& a = c.resv_alloc[(size_t)i];
      RsvView v{};
      v.node = node;
      v.restricted = c.resv[(size_t)i].allocate_policy == KE_RSV_POLICY_RESTRICTED;
      for (int w = 0; w < 4; w++) {
        v.pref2[w] = a.cpuset[w] & ~a.owner_cpuset[w];  // remainedCPUs
        v.pref[w] = merged[w] | v.pref2[w];
      }
      c.rsv_views.push_back(v);
      c.rsv_view_resv.push_back(i);
    }
  }
}

// ---- DeviceShare allocate-from-reservation views (deviceshare/reservation.go:99-366) ------------------------------
// A deviceResources map of one reservation part: per instance (bit 16*type + minor in `in`) the keys present
// (bit in keys[k]) and their values -- the quotav1 ResourceList arithmetic of the reference, keys kept by union.
struct HDres {
  uint64_t in = 0;
  uint64_t keys[KE_DKEYS] = {0, 0, 0};
  int64_t v[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS] = {};
};
// deviceResources.append of one instance: util.AddResourceList (keys of both, summed)
static void hd_add(HDres& d, int t, int m, const int64_t* val, uint32_t kb) {
  const uint64_t bit = 1ull << (16 * t + m);
  const bool had = (d.in & bit) != 0;
  d.in |= bit;
  for (int k = 0; k < KE_DKEYS; k++) {
    if (!((kb >> k) & 1u)) continue;
    d.v[t][m][k] = (had && (d.keys[k] & bit) ? d.v[t][m][k] : 0) + val[k];
    d.keys[k] |= bit;
  }
}
static void hd_append(HDres& d, const HDres& src) {  // appendAllocated (device_resources.go:116-132)
  for (int t = 0; t < KE_DEV_TYPES; t++)
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      const uint64_t bit = 1ull << (16 * t + m);
      if (!(src.in & bit)) continue;
      uint32_t kb = 0;
      for (int k = 0; k < KE_DKEYS; k++) kb |= (uint32_t)((src.keys[k] & bit) != 0) << k;
      hd_add(d, t, m, src.v[t][m], kb);
    }
}
// RestoreReservation's parts of one reservation (reservation.go:157-172): allocatable = the reserve pod's instances
// (keys with a non-zero amount), allocated = the owners' usage on them (appendAllocatedByHints), remained =
// subtractAllocated(copy(allocatable), allocated, false) -- quotav1.Subtract per allocated instance, deleted IsZero
static void hd_parts(const ke_reservation_alloc& a, HDres& al, HDres& ow, HDres& rem) {
  al = HDres{};
  ow = HDres{};
  for (int t = 0; t < KE_DEV_TYPES; t++)
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      const uint64_t bit = 1ull << (16 * t + m);
      if (!(a.device_minors & bit)) continue;
      uint32_t ka = 0, ko = 0;
      for (int k = 0; k < KE_DKEYS; k++) {
        ka |= (uint32_t)(a.device[t][m][k] != 0) << k;
        ko |= (uint32_t)(a.owner_device[t][m][k] != 0) << k;
      }
      hd_add(al, t, m, a.device[t][m], ka);
      if ((a.owner_device_minors & bit) && ko) hd_add(ow, t, m, a.owner_device[t][m], ko);
    }
  rem = al;
  for (int t = 0; t < KE_DEV_TYPES; t++)
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      const uint64_t bit = 1ull << (16 * t + m);
      if (!(ow.in & bit)) continue;
      bool zero = true;
      for (int k = 0; k < KE_DKEYS; k++) {
        const bool hr = (rem.in & bit) && (rem.keys[k] & bit), ho = (ow.keys[k] & bit) != 0;
        if (!hr && !ho) continue;
        rem.v[t][m][k] = (hr ? rem.v[t][m][k] : 0) - (ho ? ow.v[t][m][k] : 0);
        rem.keys[k] |= bit;
        zero = zero && rem.v[t][m][k] == 0;
      }
      if (zero) {  // the instance leaves the map
        rem.in &= ~bit;
        for (int k = 0; k < KE_DKEYS; k++) rem.keys[k] &= ~bit, rem.v[t][m][k] = 0;
      } else {
        rem.in |= bit;
      }
    }
}
static void hd_to_pre(const HDres& x, DsView& v) {
  v.pre_in = x.in;
  for (int k = 0; k < KE_DKEYS; k++) v.pre_keys[k] = x.keys[k];
  std::memcpy(v.pre, x.v, sizeof v.pre);
}

void resv_ds_views(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids) {
  c.ds_views.clear();
  c.ds_view_resv.clear();
  c.ds_view_out.clear();
  if (c.resv_alloc.empty() || !c.ds_enabled) return;
  const DevPod dp = make_dev_pod(c.cfg, pod, pod_hints(c, pod), &c.tmpl);
  if (!(dp.flags & PF_DS) || (dp.flags & PF_DS_INVALID)) return;
  const bool ignored = ids == nullptr;
  std::vector<char> m(c.resv.size(), ignored ? 1 : 0);
  for (int32_t j = 0; !ignored && j < n_ids; j++) m[(size_t)ids[j]] = 1;
  flush_mirror(c);  // the rows re-derived below carry every earlier placement
  for (size_t node = 0; node < c.resv_by_node.size(); node++) {
    NodeState& ns = c.nodes[node];
    if (c.resv_by_node[node].empty() || !ns.has_dev_cache) continue;
    // RestoreReservation's matched list: the usable matched reservations holding devices, in index order
    // (at most 32, as the restatement keeps them)
    std::vector<int32_t> mine;
    for (int32_t i : c.resv_by_node[node])
      if (m[(size_t)i] && resv_usable(c.resv[(size_t)i]) && c.resv_alloc[(size_t)i].device_minors && mine.size() < 32)
        mine.push_back(i);
    if (mine.empty()) continue;
    if (!ignored) {  // the rows this pod sees: its matched restore (resv_prepare applies the same)
      resv_delta(c, (int32_t)node, &m, true, ns.rv_req, ns.rv_nz, &ns.rv_pods, &ns.rv_x);
      resv_plugin_restore(c, (int32_t)node, &m, ns);
      ns.dirty = true;
    }
    std::vector<HDres> al(mine.size()), ow(mine.size()), rem(mine.size());
    HDres m_alloc, m_allocd, sum_rem;
    for (size_t q = 0; q < mine.size(); q++) {
      hd_parts(c.resv_alloc[(size_t)mine[q]], al[q], ow[q], rem[q]);
      hd_append(m_alloc, al[q]);
      hd_append(m_allocd, ow[q]);
      hd_append(sum_rem, rem[q]);
    }
    auto push = [&](const HDres& extra, int32_t r) -> DsView& {
      c.ds_views.emplace_back();
      DsView& v = c.ds_views.back();
      std::memset(&v, 0, sizeof v);
      v.node = (int32_t)node;
      hd_to_pre(extra, v);
      c.ds_view_resv.push_back(r);
      return v;
    };
    if (!ignored)
      for (size_t q = 0; q < mine.size(); q++) {  // tryAllocateFromReservation's trial of each (reservation.go:229-280)
        HDres extra = m_allocd;  // basicPreemptible (in the row) + mergedMatchedAllocated + remained
        hd_append(extra, rem[q]);
        DsView& v = push(extra, mine[q]);
        const bool restricted = c.resv[(size_t)mine[q]].allocate_policy == KE_RSV_POLICY_RESTRICTED;
        bool any = false;
        for (int t = 0; t < KE_DEV_TYPES; t++) {
          const uint16_t ain = (uint16_t)((al[q].in >> (16 * t)) & 0xFFFF);
          v.pref[t] = ain;  // preferred = the reservation's minors
          if (!restricted) continue;
          v.rreq[t] = ain;  // required = preferred
          v.cap_in[t] = ain ? (uint16_t)((rem[q].in >> (16 * t)) & ain) : 0;  // calcRequiredDeviceResources
          any = any || v.cap_in[t] != 0;
        }
        if (restricted) {
          if (any) {
            for (int k = 0; k < KE_DKEYS; k++) {
              uint64_t cb = 0;
              for (int t = 0; t < KE_DEV_TYPES; t++) cb |= (uint64_t)v.cap_in[t] << (16 * t);
              v.cap_keys[k] = rem[q].keys[k] & cb;
            }
            std::memcpy(v.cap, rem[q].v, sizeof v.cap);
          } else {  // nothing remained: every reservation minor with an empty list
            for (int t = 0; t < KE_DEV_TYPES; t++) v.cap_in[t] = v.rreq[t];
          }
        }
      }
    push(m_alloc, -1);  // the node's own allocation: basicPreemptible + mergedMatchedAllocatable (plugin.go:358-364)
    if (ignored) {      // tryAllocateIgnoreReservation (reservation.go:290-310): Σ remained + mergedMatchedAllocated
      HDres extra = sum_rem;
      hd_append(extra, m_allocd);
      push(extra, -2);
    }
  }
}

// ---- NodeNUMAResource allocate-from-reservation views under a NUMA policy (nodenumaresource/reservation.go:270-424) ----
// Per node of the pod's matched reservations holding NUMA resources / CPUs where the pod's or the node's NUMA policy
// applies (the pod binds no CPUs: check_matches), RestoreReservation's matched set there (index order) and:
//   the hint view (GetTopologyHints, resource_manager.go:136-138): reusable += mergedMatchedAllocatable;
//   trial q (tryAllocateFromReservation, reservation.go:293-311): reusable += mergedMatchedAllocated + its remained;
//   a Restricted trial's requiredResources (:353-357): its remained (quotav1.Subtract: signed, keys of both).
void resv_numa_views(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids) {
  c.numa_views.clear();
  c.numa_view_ids.clear();
  c.numa_view_out.clear();
  if (c.resv_alloc.empty()) return;
  const DevPod dp = make_dev_pod(c.cfg, pod, pod_hints(c, pod), &c.tmpl);
  if (dp.flags & PF_NUMA_SKIP) return;
  std::vector<char> m(c.resv.size(), 0);
  for (int32_t j = 0; j < n_ids; j++)
    if (resv_usable(c.resv[(size_t)ids[j]])) m[(size_t)ids[j]] = 1;
  std::vector<int32_t> nodes;
  for (int32_t j = 0; j < n_ids; j++)
    if (m[(size_t)ids[j]] && resv_holds_cpu(c, ids[j])) nodes.push_back(c.resv[(size_t)ids[j]].node);
  std::sort(nodes.begin(), nodes.end());
  nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
  auto any_numa = [](const int64_t* v) {
    for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++)
      if (v[j]) return true;
    return false;
  };
  for (int32_t node : nodes) {
    NodeState& ns = c.nodes[(size_t)node];
    if (pod.numa_topology_policy == KE_NUMA_POLICY_NONE && ns.node.numa_topology_policy == KE_NUMA_POLICY_NONE) continue;
    std::vector<int32_t> mine;
    for (int32_t i : c.resv_by_node[(size_t)node])
      if (m[(size_t)i] && resv_holds_cpu(c, i) && mine.size() < (size_t)NV_MAX) mine.push_back(i);
    if (mine.empty()) continue;
    // the rows this pod sees: its matched restore (resv_prepare applies the same)
    resv_delta(c, node, &m, true, ns.rv_req, ns.rv_nz, &ns.rv_pods, &ns.rv_x);
    resv_plugin_restore(c, node, &m, ns);
    ns.dirty = true;
    c.numa_views.emplace_back();
    NumaRsvView& v = c.numa_views.back();
    std::memset(&v, 0, sizeof v);
    v.node = node;
    v.n = (int32_t)mine.size();
    v.required = pod.reservation_matched == KE_RSV_AFFINITY;
    for (const ke_numa_zone& z : ns.zones)
      if (z.id >= 0 && z.id < KE_MAX_NUMA && (z.has_allocated & KE_NUMA_ALLOC_ENTRY)) v.entry |= 1u << z.id;
    int64_t m_allocd[KE_MAX_NUMA * KE_NRES] = {};
    uint32_t m_allocd_keys = 0;
    for (int32_t i : mine) {
      const ke_reservation_alloc& a = c.resv_alloc[(size_t)i];
      for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++)
        if (a.numa[j] != 0) v.hint_keys |= 1u << j, v.hint[j] += a.numa[j];  // mergedMatchedAllocatable
      if (!any_numa(a.numa)) continue;
      for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++)
        if (a.owner_numa[j] != 0) m_allocd_keys |= 1u << j, m_allocd[j] += a.owner_numa[j];  // mergedMatchedAllocated
    }
    for (size_t q = 0; q < mine.size(); q++) {
      const ke_reservation_alloc& a = c.resv_alloc[(size_t)mine[q]];
      v.keys[q] = m_allocd_keys;
      std::memcpy(v.reuse[q], m_allocd, sizeof m_allocd);
      v.restricted[q] = c.resv[(size_t)mine[q]].allocate_policy == KE_RSV_POLICY_RESTRICTED;
      v.has_req[q] = any_numa(a.numa);
      if (!v.has_req[q]) continue;
      for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++)
        if (a.numa[j] != 0 || a.owner_numa[j] != 0) {  // remained = allocatable - allocated
          v.req_keys[q] |= 1u << j;
          v.req[q][j] = a.numa[j] - a.owner_numa[j];
          v.keys[q] |= 1u << j;
          v.reuse[q][j] += v.req[q][j];
        }
    }
    if (pod_binds_on(dp, ns) && cpus_valid(ns)) {  // the views' preferredCPUs (reservation.go:293-311, 340-357)
      uint64_t allocd[4] = {0, 0, 0, 0};          // mergedMatchedAllocatedCPUs: the reserve pods' CPUs
      for (int32_t i : mine)
        for (int w = 0; w < 4; w++) allocd[w] |= c.resv_alloc[(size_t)i].cpuset[w];
      for (size_t q = 0; q < mine.size(); q++) {
        const ke_reservation_alloc& a = c.resv_alloc[(size_t)mine[q]];
        int rem = 0;
        for (int w = 0; w < 4; w++) {
          const uint64_t rc = a.cpuset[w] & ~a.owner_cpuset[w];  // remainedCPUs
          v.pref[NV_MAX][w] |= rc;                                // mergedMatchedRemainCPUs (the hint view)
          v.pref[q][w] = allocd[w] | rc;
          v.rpref[q][w] = rc;
          rem += __builtin_popcountll(rc);
        }
        v.rem_cpus[q] = rem;
      }
    }
    c.numa_view_ids.push_back(mine);
  }
}

void resv_numa_cs_apply(Context& c) {
  for (size_t j = 0; j < c.numa_cs_views.size(); j++) {
    RsvOvr& o = c.rsv_ovr[(size_t)c.numa_cs_ovr[j]];
    const bool ok = j < c.numa_cs_out.size() && c.numa_cs_out[j].ok;
    if (ok) {
      o.reserve = 1;
      o.numa_score = (int16_t)c.numa_cs_out[j].score;
      for (int w = 0; w < 4; w++) o.cpus[w] = c.numa_cs_out[j].cpus[w];
    } else {  // (the Filter's counts admitted the trial: not reached while they agree with allocateCPUSet)
      o.reserve = 2;
      if (c.numa_cs_pair[j] < 0) o.numa_st = KE_CODE_UNSCHEDULABLE, o.numa_reason = KE_REASON_NUMA_INSUFFICIENT_CPUS;
      else if (o.numa_st == KE_CODE_SUCCESS) c.rsv_pairs[(size_t)c.numa_cs_pair[j]].allowed |= RSV_PAIR_SCORE_ERROR;
    }
  }
  c.numa_cs_views.clear();
  c.numa_cs_ovr.clear();
  c.numa_cs_pair.clear();
  c.numa_cs_out.clear();
}

int resv_prepare(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids, bool affinity) {
  int rc = resv_check(c, ids, n_ids);  // (ke_schedule's argument checks ran it already: nothing below fails)
  if (rc) return rc;
  c.rsv_affinity = affinity;
  c.rsv_pairs.clear();
  c.rsv_nominated.clear();
  c.rsv_nodes.clear();
  c.rsv_ovr.clear();
  const DevPod dp = make_dev_pod(c.cfg, pod, pod_hints(c, pod), &c.tmpl);
  std::vector<char> m(c.resv.size(), 0);
  for (int32_t j = 0; j < n_ids; j++)
    if (resv_usable(c.resv[(size_t)ids[j]])) m[(size_t)ids[j]] = 1;
  for (int32_t j = 0; j < n_ids; j++)
    if (m[(size_t)ids[j]]) c.rsv_nodes.push_back(c.resv[(size_t)ids[j]].node);
  std::sort(c.rsv_nodes.begin(), c.rsv_nodes.end());
  c.rsv_nodes.erase(std::unique(c.rsv_nodes.begin(), c.rsv_nodes.end()), c.rsv_nodes.end());
  flush_mirror(c);  // NodeInfo.Requested with every earlier placement
  for (int32_t node : c.rsv_nodes) {
    NodeState& ns = c.nodes[(size_t)node];
    int64_t ureq[KE_NRES], unz[KE_NRES], pod_requested[KE_NRES], all_alloc[KE_NRES] = {0, 0};
    XDelta ux, all_x;
    resv_delta(c, node, &m, false, ureq, unz, nullptr, &ux);
    for (int k = 0; k < KE_NRES; k++) pod_requested[k] = ns.node.requested[k] + ureq[k];
    std::vector<int32_t> mine;
    int64_t order = 0;  // findMostPreferredReservationByOrder over all matched (scoring.go:170-189)
    for (int32_t i : c.resv_by_node[(size_t)node])
      if (m[(size_t)i]) {
        mine.push_back(i);
        for (int k = 0; k < KE_NRES; k++) all_alloc[k] += c.resv[(size_t)i].allocated[k];
        for (const ke_reservation_resource& e : resv_entries(c, i))
          if (e.id != KE_RSV_RES_PODS) x_add(&all_x, e.id, e.allocated);
        const int64_t o = c.resv[(size_t)i].order;
        if (o != 0 && (order == 0 || o < order)) order = o;
      }
    int64_t mreq[KE_NRES], mnz[KE_NRES];
    int32_t mpods = 0;  // the snapshot's len(Pods) delta with this pod's matched reserve pods removed
    resv_delta(c, node, &m, true, mreq, mnz, &mpods);
    const int64_t pods_restored = (int64_t)ns.node.pod_count + mpods;
    // NodeNUMAResource's FilterNominateReservation (plugin.go:448-504): a binding pod needs a valid CPU topology;
    // under a reservation affinity a reservation holding a cpuset / NUMA resources needs its trial (k_rsv_views)
    const bool binds = pod_binds_on(dp, ns);
    auto view_of = [&](int32_t i) -> int {  // the trial of reservation i here: 1 ok, 0 failed, -1 none
      for (size_t q = 0; q < c.rsv_views.size(); q++)
        if (c.rsv_view_resv[q] == i && c.rsv_views[q].node == node) return c.rsv_view_out.size() > q ? c.rsv_view_out[q].ok : 0;
      return -1;
    };
    // under a NUMA policy (k_numa_views): with an affinity a reservation of the trials needs its allocation on the
    // stored affinity; one outside RestoreReservation's matched set passes
    int nvi = -1;
    for (size_t q = 0; q < c.numa_views.size(); q++)
      if (c.numa_views[q].node == node) nvi = (int)q;
    const NumaRsvOut* nvo = nvi >= 0 && (size_t)nvi < c.numa_view_out.size() ? &c.numa_view_out[(size_t)nvi] : nullptr;
    auto numa_trial = [&](int32_t i) -> int {  // the trial index of reservation i in the node's view set, or -1
      if (nvi < 0) return -1;
      const std::vector<int32_t>& t = c.numa_view_ids[(size_t)nvi];
      for (size_t q = 0; q < t.size(); q++)
        if (t[q] == i) return (int)q;
      return -1;
    };
    auto numa_nominable = [&](int32_t i) {
      if (nvo) {
        const int q = numa_trial(i);
        return !(affinity && q >= 0 && !((nvo->ok >> q) & 1u));
      }
      if (!binds) return true;
      if (!cpus_valid(ns)) return false;
      return !(affinity && view_of(i) == 0);
    };
    // DeviceShare (a pod with device requests on a node with a cache entry and matched reservations holding devices):
    // the k_ds_views outcomes of its trials -- per reservation (tryAllocateFromReservation over it alone) and the
    // node's own (-1)
    auto ds_view = [&](int32_t r) -> const DsViewOut* {
      for (size_t q = 0; q < c.ds_views.size(); q++)
        if (c.ds_view_resv[q] == r && c.ds_views[q].node == node) return c.ds_view_out.size() > q ? &c.ds_view_out[q] : nullptr;
      return nullptr;
    };
    const DsViewOut* ds_own = ds_view(-1);
    std::vector<int32_t> ok;
    std::vector<int64_t> ok_ds;
    bool fits_one = false;  // the Reservation Filter with a reservation affinity (plugin.go:316-318, 351-442): a
                            // node without matched reservations fails, one with them passes when one of them fits
    for (int32_t i : mine)
      if (resv_nominable(c, i, pod, ns, pod_requested, ux, all_alloc, all_x, affinity, pods_restored,
                         (int64_t)mine.size(), ns.node.allowed_pods)) {
        fits_one = true;
        if (!numa_nominable(i)) continue;
        // DeviceShare's FilterNominateReservation (plugin.go:371-426): a reservation holding devices satisfies the pod
        const DsViewOut* dv = ds_own ? ds_view(i) : nullptr;
        if (dv && dv->st != KE_CODE_SUCCESS) continue;
        ok.push_back(i);
        ok_ds.push_back(dv ? dv->raw : 0);
      }
    const bool allowed = !affinity || fits_one;
    // NominateReservation (nominator.go:223-277): with an affinity and one matched reservation that one, else
    // the survivors: the only one, else the smallest order, else the best Σ ScoreReservation -- the Reservation
    // plugin's raw and DeviceShare's normalized (DefaultReservationNormalizeScore over the list) -- ties to the
    // lowest index (sort.Slice's insertion sort keeps them below 13 elements)
    int32_t nom = -1;
    if (ok.size() == 1) nom = ok[0];
    if (ok.size() > 1) {
      int64_t bo = 0;
      for (int32_t i : ok) {
        const int64_t o = c.resv[(size_t)i].order;
        if (o != 0 && (bo == 0 || o < bo)) {
          bo = o;
          nom = i;
        }
      }
      if (nom < 0) {
        int64_t mx = 0, bs = -1;
        for (int64_t x : ok_ds) mx = std::max(mx, x);
        for (size_t q = 0; q < ok.size(); q++) {
          const int64_t sc = resv_score(c, ok[q], pod) + (mx > 0 ? 100 * ok_ds[q] / mx : ok_ds[q]);
          if (sc > bs) {
            bs = sc;
            nom = ok[q];
          }
        }
      }
    }
    if (affinity && mine.size() == 1) nom = mine[0];
    RsvOvr o{};
    o.node = node;
    bool any_ovr = false;
    // DeviceShare's Filter (tryAllocateFromReservation over the matched list: a satisfied reservation passes, none
    // under an affinity fails, else the node's own), Score (the nominated reservation's view, else the node's own)
    // and Reserve (the nominated one's allocation when it succeeds, else the node's own; failing: not placed)
    bool reserve_fails = false;
    if (ds_own) {
      o.ds_on = 1;
      const DsViewOut* pass = nullptr;
      for (int32_t i : mine) {
        const DsViewOut* dv = ds_view(i);
        if (dv && dv->st == KE_CODE_SUCCESS) {
          pass = dv;
          break;
        }
      }
      if (pass) {
        o.ds_st = KE_CODE_SUCCESS;
      } else if (affinity) {
        o.ds_st = KE_CODE_UNSCHEDULABLE;
        o.ds_reason = KE_REASON_RSV_INSUFFICIENT_DEVICES;
      } else {
        o.ds_st = (uint8_t)ds_own->st;
        o.ds_reason = (uint8_t)ds_own->reason;
      }
      const DsViewOut* nv = nom >= 0 ? ds_view(nom) : nullptr;
      o.ds_raw = (int16_t)(nv ? nv->raw : ds_own->raw);
      const DsViewOut* rv = (nv && nv->st == KE_CODE_SUCCESS && nv->minors) ? nv : ds_own;
      if (rv->st == KE_CODE_SUCCESS && rv->minors) {
        o.ds_res = 1;
        o.ds_minors = rv->minors;
      } else {
        o.ds_res = 2;
        reserve_fails = o.ds_st == KE_CODE_SUCCESS;
      }
      any_ovr = true;
    }
    if (affinity) {
      o.rfilter = (int8_t)(allowed ? 1 : 2);
      any_ovr = true;
    }
    // NodeNUMAResource under a NUMA policy (k_numa_views): the Filter's outcome; Score and Reserve from the
    // nominated reservation's allocation on the affinity (allocateWithNominatedReservation), else the node's own
    // (tryAllocateFromNode); an error status there is a Score error (scoring.go:105-115)
    bool score_err = false;
    if (nvo) {
      o.numa_on = 1;
      o.numa_st = (uint8_t)nvo->st;
      o.numa_reason = (uint8_t)nvo->reason;
      o.numa_aff = (uint8_t)nvo->aff;
      int use = -1;  // the trial, NV_MAX = the node's own
      const int qn = nom >= 0 ? numa_trial(nom) : -1;
      if (nom < 0 && affinity) score_err = true;  // "no nominated reservation"
      else if (qn >= 0 && ((nvo->ok >> qn) & 1u)) use = qn;
      else if (qn >= 0 && affinity) score_err = true;
      else if ((nvo->ok >> NV_MAX) & 1u) use = NV_MAX;
      else score_err = true;
      if (nvo->st != KE_CODE_SUCCESS) score_err = false;  // (an infeasible node is not scored)
      if (use >= 0) {
        o.numa_score = (int16_t)nvo->score[use];
        std::memcpy(o.numa_dist, nvo->dist[use], sizeof o.numa_dist);
      }
      if (use >= 0 && use < NV_MAX && binds && cpus_valid(ns)) {
        // a binding pod: the cpuset of the nominated reservation's allocation and the Score it gives (k_rsv_views
        // with the allocation's zones, resv_numa_cs_apply) -- a Restricted one's from its remainedCPUs
        const NumaRsvView& nv = c.numa_views[(size_t)nvi];
        RsvView v{};
        v.node = node;
        for (int w = 0; w < 4; w++) {
          v.pref[w] = nv.restricted[use] ? nv.rpref[use][w] : nv.pref[use][w];
          v.pref2[w] = nv.pref[use][w];
        }
        for (int z = 0; z < 8; z++)
          if (nvo->dist[use][2 * z] != 0 || nvo->dist[use][2 * z + 1] != 0) {
            v.zmask |= 1 << z;
            v.zcpu[z] = nvo->dist[use][2 * z];
          }
        v.score_on = 1;
        v.sreq1 = nvo->sreq1[use];
        v.salloc[0] = nvo->salloc[use][0];
        v.salloc[1] = nvo->salloc[use][1];
        c.numa_cs_views.push_back(v);
        c.numa_cs_ovr.push_back((int32_t)c.rsv_ovr.size());
        c.numa_cs_pair.push_back((int32_t)c.rsv_pairs.size());
      }
      any_ovr = true;
    }
    c.rsv_pairs.push_back({node, (int16_t)(nom >= 0 ? resv_score(c, nom, pod) : 0),
                           (int16_t)((allowed ? RSV_PAIR_ALLOWED : 0) | (reserve_fails ? RSV_PAIR_RESERVE_FAILS : 0) |
                                     (score_err ? RSV_PAIR_SCORE_ERROR : 0)),
                           order});
    c.rsv_nominated.push_back(nom);
    // NodeNUMAResource with the matched reservations first (plugin.go:381-397, 553-563): the Filter's trial
    // (one satisfied; else "Reservation(s) ..." under an affinity, else the node's own) and Reserve's allocation
    // (the nominated reservation's when it holds one and is satisfied; failing under an affinity)
    if (binds && ns.node.numa_topology_policy == KE_NUMA_POLICY_NONE && !nvo) {
      bool any_view = false, any_ok = false;
      for (size_t q = 0; q < c.rsv_views.size(); q++)
        if (c.rsv_views[q].node == node) {
          any_view = true;
          any_ok = any_ok || (c.rsv_view_out.size() > q && c.rsv_view_out[q].ok);
        }
      o.filter = (int8_t)(any_ok ? 1 : (any_view && affinity) ? 2 : 0);
      const int nv = nom >= 0 ? view_of(nom) : -1;
      if (nom < 0) o.reserve = (int8_t)(affinity ? 2 : 0);  // "no nominated reservation"
      else if (nv == 1) {
        o.reserve = 1;
        for (size_t q = 0; q < c.rsv_views.size(); q++)
          if (c.rsv_view_resv[q] == nom && c.rsv_views[q].node == node)
            for (int w = 0; w < 4; w++) o.cpus[w] = c.rsv_view_out[q].cpus[w];
      } else {
        o.reserve = (int8_t)(nv == 0 && affinity ? 2 : 0);
      }
      any_ovr = any_ovr || o.filter || o.reserve;
    }
    if (any_ovr) {
      c.rsv_ovr.push_back(o);
      ns.rsv_ovr = true;
    }
    // the rows this pod sees: its matched reservations restored too, and left out of the plugins' unmatched states
    resv_delta(c, node, &m, true, ns.rv_req, ns.rv_nz, &ns.rv_pods, &ns.rv_x);
    resv_plugin_restore(c, node, &m, ns);
    ns.dirty = true;
  }
  return KE_OK;
}

// An owner pod's allocations enter (sign +1) or leave (-1) its reservation's owner part: the resource manager /
// device cache entries RestoreReservation reads by the reservation's AssignedPods (reservation.go:201-226,
// deviceshare/reservation.go:165-170).  CPUs are counted per owner (the owners' union is what the record shows).
void resv_owner_update(Context& c, int32_t idx, const ke_pod& pod, const uint64_t* cpuset, const int64_t* numa,
                       uint64_t dev_minors, int sign) {
  if (c.resv_alloc.empty() || idx < 0 || idx >= (int32_t)c.resv_alloc.size()) return;
  ke_reservation_alloc& a = c.resv_alloc[(size_t)idx];
  if (c.resv_cpu_cnt.size() != c.resv_alloc.size()) c.resv_cpu_cnt.assign(c.resv_alloc.size(), {});
  std::vector<uint8_t>& cnt = c.resv_cpu_cnt[(size_t)idx];
  if (cnt.empty()) {
    cnt.assign(KE_MAX_CPUS, 0);
    for (int cpu = 0; cpu < KE_MAX_CPUS; cpu++) cnt[(size_t)cpu] = a.owner_cpuset[cpu >> 6] >> (cpu & 63) & 1;
  }
  for (int cpu = 0; cpuset && cpu < KE_MAX_CPUS; cpu++)
    if (cpuset[cpu >> 6] >> (cpu & 63) & 1) {
      uint8_t& k = cnt[(size_t)cpu];
      k = (uint8_t)(sign > 0 ? std::min(255, k + 1) : std::max(0, k - 1));
      if (k) a.owner_cpuset[cpu >> 6] |= 1ull << (cpu & 63);
      else a.owner_cpuset[cpu >> 6] &= ~(1ull << (cpu & 63));
    }
  for (int j = 0; numa && j < KE_MAX_NUMA * KE_NRES; j++)
    a.owner_numa[j] = std::max<int64_t>(0, a.owner_numa[j] + sign * numa[j]);
  if (dev_minors) {
    const NodeState& ns = c.nodes[(size_t)c.resv[(size_t)idx].node];
    const DevPod dp = make_dev_pod(c.cfg, pod, pod_hints(c, pod), &c.tmpl);
    for (const ke_device& d : ns.devs) {
      const uint64_t bit = 1ull << (16 * d.type + d.minor);
      if (!(dev_minors & bit)) continue;
      int64_t amt[KE_DKEYS];
      bool has[KE_DKEYS];
      ds_instance_amounts(d, dp, amt, has);
      bool any = false;
      for (int k = 0; k < KE_DKEYS; k++) {
        int64_t& o = a.owner_device[d.type][d.minor][k];
        if (has[k]) o = std::max<int64_t>(0, o + sign * amt[k]);
        any = any || o != 0;
      }
      if (any) a.owner_device_minors |= bit;
      else a.owner_device_minors &= ~bit;
    }
  }
  c.resv_holds[(size_t)idx] = resv_holds_of(a);
}

void resv_finish(Context& c, int32_t chosen_local, const ke_pod& pod, int32_t* assumed, const uint64_t* cpuset,
                 const int64_t* numa, uint64_t dev_minors) {
  *assumed = 0;
  for (size_t j = 0; j < c.rsv_nodes.size(); j++)
    if (c.rsv_nodes[j] == chosen_local && c.rsv_nominated[j] >= 0) {
      // assumePod -> AddAssignedPod (reservation_info.go:458-468): Mask(requests, ResourceNames)
      ke_reservation& r = c.resv[(size_t)c.rsv_nominated[j]];
      for (int k = 0; k < KE_NRES; k++)
        if (r.allocatable[k] != 0 && !(r.names_excluded >> k & 1)) r.allocated[k] += pod.requests[k];
      if ((size_t)c.rsv_nominated[j] < c.resv_res.size())
        for (ke_reservation_resource& e : c.resv_res[(size_t)c.rsv_nominated[j]])
          if (!e.excluded && e.id != KE_RSV_RES_PODS) e.allocated += pod_request_of(pod, e.id);
      r.allocated_pods++;
      *assumed = 1 + c.rsv_nominated[j];
      resv_owner_update(c, c.rsv_nominated[j], pod, cpuset, numa, dev_minors, +1);
    }
  for (int32_t node : c.rsv_nodes) {
    c.nodes[(size_t)node].rsv_ovr = false;
    resv_node_restore(c, node);
  }
  c.rsv_affinity = false;
  c.rsv_pairs.clear();
  c.rsv_nominated.clear();
  c.rsv_nodes.clear();
  c.rsv_ovr.clear();
  c.rsv_views.clear();
  c.rsv_view_resv.clear();
  c.rsv_view_out.clear();
  c.ds_views.clear();
  c.ds_view_resv.clear();
  c.ds_view_out.clear();
  c.numa_views.clear();
  c.numa_view_ids.clear();
  c.numa_view_out.clear();
  c.numa_cs_views.clear();
  c.numa_cs_ovr.clear();
  c.numa_cs_pair.clear();
  c.numa_cs_out.clear();
}

// forgetPod -> RemoveAssignedPod (reservation_info.go:470-482)
void resv_forget(Context& c, int32_t idx, const ke_pod& pod, const ke_pod_allocation* a) {
  if (idx < 0 || idx >= (int32_t)c.resv.size()) return;
  ke_reservation& r = c.resv[(size_t)idx];
  for (int k = 0; k < KE_NRES; k++)
    if (r.allocatable[k] != 0 && !(r.names_excluded >> k & 1)) r.allocated[k] = std::max<int64_t>(0, r.allocated[k] - pod.requests[k]);
  if ((size_t)idx < c.resv_res.size())
    for (ke_reservation_resource& e : c.resv_res[(size_t)idx])
      if (!e.excluded && e.id != KE_RSV_RES_PODS) e.allocated = std::max<int64_t>(0, e.allocated - pod_request_of(pod, e.id));
  if (r.allocated_pods > 0) r.allocated_pods--;
  if (a) resv_owner_update(c, idx, pod, a->cpuset, a->numa, a->device_minors, -1);
  resv_node_restore(c, r.node);
}

// host mirror of a placement's ext Reserve: NodeInfo (NonZero)Requested += the pod's requests by id
void host_ext_reserve(NodeState& ns, const ke_pod& pod) {
  for (int e = 0; e < pod.n_xres; e++) {
    bool found = false;
    for (ke_node_resource& r : ns.xres)
      if (r.id == pod.xres_id[e]) r.requested += pod.xres_value[e], found = true;
    if (!found && pod.xres_value[e] != 0) ns.xres.push_back(ke_node_resource{pod.xres_id[e], 0, 0, pod.xres_value[e]});
  }
}

// ---------------------------------------------------------------------------------------------
// arithmetic helpers (IEEE double, no contraction: built with -ffp-contract=off)
// ---------------------------------------------------------------------------------------------
int64_t usage_percent(int64_t used, int64_t total) {
  double q = (double)used / (double)total;  // float64(used) / float64(total)
  double p = q * 100.0;                     // * 100
  return (int64_t)std::round(p);            // int64(math.Round(...)): half away from zero
}

int64_t max_used_within(int64_t total, int64_t thr) {
  // usage_percent is monotone non-decreasing in `used` (each of int64->float64, /total, *100, round
  // is), so {used : pct(used) <= thr} is a prefix of the domain; binary-search its last element.
  int64_t lo = -USED_DOMAIN, hi = USED_DOMAIN;
  if (usage_percent(hi, total) <= thr) return hi;
  if (usage_percent(lo, total) > thr) return lo - 1;
  // the boundary is near (thr + 0.5) * total / 100: step from there to the u with pct(u) <= thr < pct(u + 1),
  // the same element the search below finds (the predicate is monotone); the search when that does not land
  if (total > 0) {
    const double g = std::floor(((double)thr + 0.5) * (double)total / 100.0);
    if (g > (double)(-USED_DOMAIN + 8) && g < (double)(USED_DOMAIN - 8)) {
      int64_t u = (int64_t)g;
      for (int s = 0; s < 8; s++) {
        if (usage_percent(u, total) > thr) u--;
        else if (usage_percent(u + 1, total) <= thr) u++;
        else return u;
      }
    }
  }
  while (hi - lo > 1) {  // pct(lo) <= thr < pct(hi)
    int64_t mid = lo + (hi - lo) / 2;
    if (usage_percent(mid, total) <= thr) lo = mid;
    else hi = mid;
  }
  return lo;
}

static int64_t amplify(int64_t origin, double ratio) {  // node_resource_amplification.go:170-175
  if (ratio <= 1.0) return origin;
  return (int64_t)std::ceil((double)origin * ratio);
}

// ---------------------------------------------------------------------------------------------
// estimator
// ---------------------------------------------------------------------------------------------
static int translated_resource(int32_t priority, int r) {  // apis/extension/resource.go:53-58
  if (priority == KE_PRIORITY_PROD || priority == KE_PRIORITY_NONE) return r;
  if (priority == KE_PRIORITY_BATCH) return r == KE_RES_CPU ? KE_RES_BATCH_CPU : KE_RES_BATCH_MEMORY;
  if (priority == KE_PRIORITY_MID) return r == KE_RES_CPU ? KE_RES_MID_CPU : KE_RES_MID_MEMORY;
  return -1;  // koord-free: no translation entry -> empty resource name
}

static int64_t estimate_resource(const ke_pod& pod, int name, int64_t factor) {  // default_estimator.go:88-122
  const int64_t lim = name >= 0 ? pod.limits[name] : 0;
  const int64_t req = name >= 0 ? pod.requests[name] : 0;
  const int64_t q = lim > req ? lim : req;
  if (q == 0) {
    if (name == KE_RES_CPU || name == KE_RES_BATCH_CPU) return DEFAULT_MILLI_CPU;
    if (name == KE_RES_MEMORY || name == KE_RES_BATCH_MEMORY) return DEFAULT_MEMORY;
    return 0;
  }
  const double prod = (double)q * (double)factor;
  int64_t est = (int64_t)std::round(prod / 100.0);
  if (lim > 0 && est > lim) est = lim;
  return est;
}

void estimate_pod(const ke_loadaware_args& a, const ke_pod& pod, int64_t* est, uint8_t* present) {
  const bool custom = a.allow_customize_estimation && pod.has_custom_scaling_factors;
  for (int r = 0; r < KE_NRES; r++) {
    int64_t f = custom ? pod.custom_scaling_factors[r] : KE_ABSENT;
    if (f == KE_ABSENT) f = a.estimated_scaling_factors[r];
    if (f == KE_ABSENT) f = 0;
    present[r] = a.resource_weights[r] != KE_ABSENT;
    est[r] = present[r] ? estimate_resource(pod, translated_resource(pod.priority_class, r), f) : 0;
  }
}

// DeviceShare PreFilter for one pod: GetPodDeviceRequests -> ValidateDeviceRequest ->
// ConvertDeviceRequest (deviceshare/utils.go:304-342,392-412), calcDesiredRequestsAndCountForGPU
// (devicehandler_gpu.go:53-96) and DefaultDeviceHandler.CalcDesiredRequestsAndCount
// (devicehandler_default.go:44-93, no hint).  Returns false when the request is invalid.
static bool percentage_ok(int64_t q) { return !(q > 100 && q % 100 != 0); }  // ValidatePercentageResource

static bool ds_prepare(const ke_pod& pod, DevPod& d, const ke_pod_device_hints* h) {
  const int64_t* q = pod.device_requests;
  // NvidiaGPU / AMDGPU / HygonDCU: whole devices, ConvertDeviceRequest's x100 (utils.go:190-212)
  bool nv = q[KE_PDR_NVIDIA_GPU] > 0, amd = q[KE_PDR_AMD_GPU] > 0, dcu = q[KE_PDR_HYGON_DCU] > 0, kg = q[KE_PDR_KOORD_GPU] > 0;
  bool sh = q[KE_PDR_GPU_SHARED] > 0, co = q[KE_PDR_GPU_CORE] > 0, me = q[KE_PDR_GPU_MEMORY] > 0,
       ra = q[KE_PDR_GPU_MEMORY_RATIO] > 0;
  const int kinds = nv + amd + dcu + kg + (sh || co || me || ra);
  if (kinds > 1) return false;  // no ValidDeviceResourceCombinations entry mixes these
  int64_t core = 0, mem = 0, ratio = 0;
  bool h_core = false, h_mem = false, h_ratio = false, any_gpu = true;
  int64_t n = 1;
  if (nv || amd || dcu) {
    core = ratio = 100 * q[nv ? KE_PDR_NVIDIA_GPU : amd ? KE_PDR_AMD_GPU : KE_PDR_HYGON_DCU];
    h_core = h_ratio = true;
  } else if (kg) {
    if (!percentage_ok(q[KE_PDR_KOORD_GPU])) return false;
    core = ratio = q[KE_PDR_KOORD_GPU];
    h_core = h_ratio = true;
  } else if (sh) {  // GPUShared | {GPUMemory | GPUMemoryRatio} [| GPUCore]
    if (me == ra) return false;
    const int64_t s = q[KE_PDR_GPU_SHARED];
    if (co && (q[KE_PDR_GPU_CORE] % s != 0 || q[KE_PDR_GPU_CORE] / s > 100)) return false;
    if (ra && (q[KE_PDR_GPU_MEMORY_RATIO] % s != 0 || q[KE_PDR_GPU_MEMORY_RATIO] / s > 100)) return false;
    n = s;
    core = q[KE_PDR_GPU_CORE], mem = q[KE_PDR_GPU_MEMORY], ratio = q[KE_PDR_GPU_MEMORY_RATIO];
    h_core = co, h_mem = me, h_ratio = ra;
  } else if (co || me || ra) {  // GPUMemory | GPUMemoryRatio | GPUCore+either (percentage checks)
    if (me == ra) return false;
    if (co && !percentage_ok(q[KE_PDR_GPU_CORE])) return false;
    if (ra && !percentage_ok(q[KE_PDR_GPU_MEMORY_RATIO])) return false;
    core = q[KE_PDR_GPU_CORE], mem = q[KE_PDR_GPU_MEMORY], ratio = q[KE_PDR_GPU_MEMORY_RATIO];
    h_core = co, h_mem = me, h_ratio = ra;
  } else {
    any_gpu = false;
  }
  if (any_gpu) {
    if (!sh && h_ratio && ratio > 100 && ratio % 100 == 0) n = ratio / 100;
    if (n > 255) return false;
    d.ds_cnt[KE_DEV_GPU] = (uint8_t)n;
    if (h_core) {
      d.flags |= PF_DS_H_CORE;
      d.ds_req[0] = core / n;
    }
    if (h_ratio) {  // ratio wins over memory (devicehandler_gpu.go:83-92)
      d.flags |= PF_DS_H_RATIO;
      d.ds_req[2] = ratio / n;
      if (ratio / n < 100) d.flags |= PF_GPU_SHARED;  // isShared
    } else if (h_mem) {
      d.flags |= PF_DS_H_MEM | PF_GPU_SHARED;
      d.ds_req[1] = mem / n;
    }
  }
  const int pdr[2] = {KE_PDR_RDMA, KE_PDR_FPGA};
  for (int i = 0; i < 2; i++) {
    const int64_t v = q[pdr[i]];
    if (v <= 0) continue;
    if (!percentage_ok(v)) return false;
    int64_t c = 1, per = v;
    const ke_device_hint* ht = h ? &h->hint[1 + i] : nullptr;  // DefaultDeviceHandler (devicehandler_default.go:53-91)
    if (v > 100 && v % 100 == 0) {
      c = v / 100;
      per = v / c;
    } else if (ht && ht->strategy == KE_DSTRATEGY_APPLY_FOR_ALL) {
      c = DS_CNT_ALL;  // the node's devices (matching the Selector): decided per node
    } else if (ht && ht->strategy == KE_DSTRATEGY_REQUESTS_AS_COUNT) {
      c = v < DS_CNT_ALL ? v : DS_CNT_ALL - 1;  // more than KE_MAX_MINORS never fits: the cap keeps that
      per = ht->exclusive == KE_DEXCL_DEVICE_LEVEL ? 100 : 1;
    }
    if (c > 255) return false;
    d.ds_cnt[1 + i] = (uint8_t)c;
    d.ds_req[3 + i] = per;
  }
  return true;
}

DevPod make_dev_pod(const ke_config& cfg, const ke_pod& pod, const ke_pod_device_hints* hints,
                    const std::vector<ke_gpu_template>* tmpl) {
  DevPod d{};
  d.quota = (uint8_t)pod.quota;  // range-checked against the loaded tree by ke_schedule
  uint8_t present[KE_NRES];
  estimate_pod(cfg.loadaware, pod, d.est, present);
  d.req[0] = pod.requests[KE_RES_CPU];
  d.req[1] = pod.requests[KE_RES_MEMORY];
  bool zero = !pod.has_other_requests;  // quotav1.IsZero(PodRequests)
  for (int r = 0; r < KE_RES_COUNT; r++) zero = zero && pod.requests[r] == 0;
  uint32_t f = 0;
  if (pod.is_daemonset) f |= PF_DAEMONSET;
  if (pod.priority_class == KE_PRIORITY_PROD) f |= PF_PROD;
  if (zero) f |= PF_NUMA_SKIP;
  if (pod.priority_class == KE_PRIORITY_PROD && cfg.loadaware.score_according_prod_usage) f |= PF_LA_SCORE_PROD;
  // NUMATopologySpec: the pod's policy; SingleNUMANodeExclusive defaults to Required with a policy
  f |= (uint32_t)pod.numa_topology_policy * PF_NUMA_POLICY0;
  if (pod.numa_exclusive == KE_NUMA_EXCLUSIVE_REQUIRED ||
      (pod.numa_exclusive == KE_NUMA_EXCLUSIVE_NONE && pod.numa_topology_policy != KE_NUMA_POLICY_NONE))
    f |= PF_NUMA_EXCL_REQ;
  // NodeNUMAResource PreFilter (plugin.go:251-312): AllowUseCPUSet (util.go:49-56) and a FullPCPUs /
  // SpreadByPCPUs bind policy from the ResourceSpec, the args' default standing in for "Default"
  const int64_t cpu = pod.requests[KE_RES_CPU];
  if (cpu % 1000 == 0) f |= PF_CPU_INT;
  if ((pod.qos_class == KE_QOS_LSE || pod.qos_class == KE_QOS_LSR) && pod.priority_class == KE_PRIORITY_PROD) {
    const int dflt = cfg.numa.default_cpu_bind_policy;
    int bind = pod.cpu_bind_preferred;
    if (bind == KE_CPU_BIND_UNSET || bind == KE_CPU_BIND_DEFAULT) bind = dflt;
    int required = pod.cpu_bind_required;
    if (required == KE_CPU_BIND_DEFAULT) required = dflt;
    if (required != KE_CPU_BIND_UNSET) bind = required;
    auto xb = [](int b) {
      return b == KE_CPU_BIND_FULL_PCPUS ? XB_FULL : b == KE_CPU_BIND_SPREAD_BY_PCPUS ? XB_SPREAD : XB_NONE;
    };
    if (bind == KE_CPU_BIND_FULL_PCPUS || bind == KE_CPU_BIND_SPREAD_BY_PCPUS) {
      if (cpu % 1000 != 0) {
        f |= PF_CPU_INVALID | PF_CPUSET;  // "the requested CPUs must be integer"
      } else if (cpu > 0) {
        f |= PF_CPU_RCB | PF_CPUSET;
        f |= (uint32_t)xb(required) * PF_CPU_REQ0 | (uint32_t)xb(bind) * PF_CPU_PREF0;
        f |= (uint32_t)pod.cpu_exclusive * PF_CPU_EXCL0;
      }
    }
  }
  d.flags = f;
  int invalid = 0;  // the PreFilter failure's reason (PF_DS_INVALID; DevPod::ds_req[0] carries it)
  if (!ds_prepare(pod, d, hints)) invalid = KE_REASON_DS_INVALID_REQUEST;
  const bool requests = d.ds_cnt[0] || d.ds_cnt[1] || d.ds_cnt[2];
  bool tmpl_pod = false;  // enforceGPUSharedResourceTemplate: the hinted path allocates it (DevPodHint PH_TMPL)
  if (!invalid && requests) {
    if (hints && hints->invalid) invalid = KE_REASON_DS_INVALID_HINT;  // newHintSelectors (utils.go:420-423)
    // parseGPURequirements: no template of any GPU model equal to the request (utils.go:508-515)
    const uint32_t keys = cfg.deviceshare.template_matched_keys;
    uint32_t named = 0;
    if (d.flags & PF_DS_H_CORE) named |= KE_TEMPLATE_KEY_CORE;
    if (d.flags & PF_DS_H_RATIO) named |= KE_TEMPLATE_KEY_MEMORY_RATIO;
    else if (d.flags & PF_DS_H_MEM) named |= KE_TEMPLATE_KEY_MEMORY;
    if (!invalid && d.ds_cnt[KE_DEV_GPU] && (d.flags & PF_GPU_SHARED) && (named & keys)) {
      tmpl_pod = true;
      bool any = false;
      for (const ke_gpu_template& t : tmpl ? *tmpl : std::vector<ke_gpu_template>{})
        any = any || (t.has[0] == ((named & KE_TEMPLATE_KEY_CORE) != 0) && t.has[1] == ((named & KE_TEMPLATE_KEY_MEMORY) != 0) &&
                      t.has[2] == ((named & KE_TEMPLATE_KEY_MEMORY_RATIO) != 0) && (!t.has[0] || t.value[0] == d.ds_req[0]) &&
                      (!t.has[1] || t.value[1] == d.ds_req[1]) && (!t.has[2] || t.value[2] == d.ds_req[2]));
      if (tmpl && !any) invalid = KE_REASON_DS_NO_MATCHED_TEMPLATE;  // (release records: no check)
    }
  }
  if (invalid) {
    for (int t = 0; t < 3; t++) d.ds_cnt[t] = 0;
    for (int i = 0; i < 5; i++) d.ds_req[i] = 0;
    d.ds_req[0] = invalid;
    d.flags = f | PF_DS_INVALID;
  } else if (requests) {
    d.flags |= PF_DS;
    if (hints || tmpl_pod) d.flags |= PF_DS_HINT;  // DevPod::ring_bw becomes the hint slot at upload
  }
  if (pod.quota_non_preemptible) d.flags |= PF_QUOTA_NP;
  // NodeResourcesFitPlus / ScarceResourceAvoidance PreScore: requested names and the FitPlus requests by slot
  d.xmask = pod.xres_request_mask;
  int32_t ids[2 * NUM_XS + KE_MAX_FITPLUS];
  const int nxs = std::min(ext_slots(cfg, ids), NUM_XS);
  for (int q = 0; q < NUM_XS; q++) {
    d.xreq[q] = 0;
    for (int e = 0; q < nxs && e < pod.n_xres; e++)
      if (pod.xres_id[e] == ids[q]) d.xreq[q] = pod.xres_value[e];
  }
  // parseGPURequirements (utils.go:487-513): GPUPartitionSpec and the GPU hint's required topology scope
  d.flags |= (uint32_t)pod.gpu_required_topology_scope * PF_GPU_SCOPE0;
  d.ring_bw = KE_ABSENT;
  if (pod.gpu_partition_spec) {
    d.flags |= PF_GPU_PART_SPEC;
    if (pod.gpu_partition_restricted) d.flags |= PF_GPU_PART_RESTRICTED;
    if (pod.gpu_ring_bus_bandwidth != KE_ABSENT) {
      d.flags |= PF_GPU_RING_BW;
      d.ring_bw = pod.gpu_ring_bus_bandwidth;
    }
  }
  return d;
}

// ---------------------------------------------------------------------------------------------
// NodeMetric views (helper.go)
// ---------------------------------------------------------------------------------------------
static const ke_resource_map* target_aggregated(const NodeState& ns, int64_t dur, int32_t type) {  // helper.go:57-95
  if (!ns.nm.has_node_metric || ns.agg.empty()) return nullptr;
  if (dur == 0) {
    int best = -1;
    int64_t best_dur = 0;
    for (size_t i = 0; i < ns.agg.size(); i++) {
      if (ns.agg[i].usage[type].n_keys > 0 && ns.agg[i].duration_ns > best_dur) {
        best_dur = ns.agg[i].duration_ns;
        best = (int)i;
      }
    }
    if (best >= 0) return &ns.agg[best].usage[type];
    return ns.nm.node_usage.n_keys > 0 ? &ns.nm.node_usage : nullptr;
  }
  for (const auto& a : ns.agg)
    if (a.duration_ns == dur && a.usage[type].n_keys > 0) return &a.usage[type];
  return nullptr;
}

static bool any_present(const int64_t* v) { return v[0] != KE_ABSENT || v[1] != KE_ABSENT; }

struct Profile {  // generateUsageThresholdsFilterProfile (helper.go:107-145)
  int64_t usage[KE_NRES], prod[KE_NRES], agg_thr[KE_NRES];
  bool has_agg = false;
  int32_t agg_type = 0;
  int64_t agg_dur = 0;
};

static Profile filter_profile(const ke_loadaware_args& a, const ke_node& n) {
  Profile p;
  const bool args_agg = a.has_aggregated && any_present(a.agg_usage_thresholds) && a.agg_usage_type != KE_AGG_NONE;
  auto use_args_agg = [&]() {
    p.has_agg = true;
    std::memcpy(p.agg_thr, a.agg_usage_thresholds, sizeof p.agg_thr);
    p.agg_type = a.agg_usage_type;
    p.agg_dur = a.agg_usage_duration_ns;
  };
  if (n.custom_thresholds_error) {
    std::memcpy(p.usage, a.usage_thresholds, sizeof p.usage);
    std::memcpy(p.prod, a.prod_usage_thresholds, sizeof p.prod);
    if (args_agg) use_args_agg();
    return p;
  }
  const bool c = n.has_custom_thresholds;
  if (c && any_present(n.custom_usage_thresholds)) std::memcpy(p.usage, n.custom_usage_thresholds, sizeof p.usage);
  else std::memcpy(p.usage, a.usage_thresholds, sizeof p.usage);
  if (c && any_present(n.custom_prod_usage_thresholds)) std::memcpy(p.prod, n.custom_prod_usage_thresholds, sizeof p.prod);
  else std::memcpy(p.prod, a.prod_usage_thresholds, sizeof p.prod);
  if (c && n.has_custom_agg && any_present(n.custom_agg_thresholds) && n.custom_agg_type != KE_AGG_NONE) {
    p.has_agg = true;
    std::memcpy(p.agg_thr, n.custom_agg_thresholds, sizeof p.agg_thr);
    p.agg_type = n.custom_agg_type;
    p.agg_dur = n.custom_agg_duration_ns;
  } else if (args_agg) {
    use_args_agg();
  }
  return p;
}

// ---------------------------------------------------------------------------------------------
// per-variant node terms (GetEstimatedUsed without the pod's own estimate)
// ---------------------------------------------------------------------------------------------
struct Terms {
  int64_t assigned[KE_NRES] = {0, 0};     // Σ max(est, actual) of estimated assigned pods
  int64_t est_actual[KE_NRES] = {0, 0};   // Σ actual usage of estimated pods (pod metric map)
  int64_t other_actual[KE_NRES] = {0, 0}; // Σ actual usage of the other pods in the metric map
};

// Time from which shouldEstimatePodByConfig (load_aware.go:360-385) flips for this pod, or INT64_MAX.
static int64_t estimate_window_end(const ke_loadaware_args& a, const AssignedPod& info, int64_t now) {
  int64_t after_sched = -1, after_init = -1;
  if (a.allow_customize_estimation) {
    after_sched = info.pod.custom_seconds_after_scheduled;
    after_init = info.pod.custom_seconds_after_initialized;
  }
  if (a.estimated_seconds_after_pod_scheduled != KE_ABSENT && after_sched < 0) after_sched = a.estimated_seconds_after_pod_scheduled;
  if (a.estimated_seconds_after_initialized != KE_ABSENT && after_init < 0) after_init = a.estimated_seconds_after_initialized;
  if (after_init > 0 && info.pod.has_initialized) {
    int64_t t = info.pod.initialized_transition_ns + after_init * NS;
    return t > now ? t : INT64_MAX;
  }
  if (after_sched > 0) {
    int64_t t = info.ts + after_sched * NS;
    return t > now ? t : INT64_MAX;
  }
  return INT64_MAX;
}

static bool should_estimate(const ke_loadaware_args& a, const AssignedPod& info, int64_t now) {
  int64_t after_sched = -1, after_init = -1;
  if (a.allow_customize_estimation) {
    after_sched = info.pod.custom_seconds_after_scheduled;
    after_init = info.pod.custom_seconds_after_initialized;
  }
  if (a.estimated_seconds_after_pod_scheduled != KE_ABSENT && after_sched < 0) after_sched = a.estimated_seconds_after_pod_scheduled;
  if (a.estimated_seconds_after_initialized != KE_ABSENT && after_init < 0) after_init = a.estimated_seconds_after_initialized;
  if (after_init > 0 && info.pod.has_initialized) return info.pod.initialized_transition_ns + after_init * NS > now;
  return after_sched > 0 && info.ts + after_sched * NS > now;
}

static Terms compute_terms(const ke_loadaware_args& a, const NodeState& ns, bool prod, int64_t now, int64_t* valid_until) {
  Terms t;
  if (ns.asg.empty() && ns.pm.empty()) return t;
  // buildPodMetricMap(nodeMetric, prod): name -> last PodMetricInfo (helper.go:154-170), as a key-sorted index
  // (the last entry of a repeated key kept); `est` marks the estimatedPods among them
  struct MetricRef {
    int64_t key;
    int32_t idx;
  };
  thread_local std::vector<MetricRef> metrics;
  thread_local std::vector<uint8_t> est;
  metrics.clear();
  for (size_t i = 0; i < ns.pm.size(); i++) {
    if (prod && ns.pm[i].priority_class != KE_PRIORITY_PROD) continue;
    metrics.push_back({ns.pm[i].pod_key, (int32_t)i});
  }
  std::stable_sort(metrics.begin(), metrics.end(), [](const MetricRef& x, const MetricRef& y) { return x.key < y.key; });
  size_t w = 0;
  for (size_t i = 0; i < metrics.size(); i++)
    if (i + 1 == metrics.size() || metrics[i + 1].key != metrics[i].key) metrics[w++] = metrics[i];
  metrics.resize(w);
  est.assign(w, 0);
  auto find_metric = [&](int64_t key) -> int64_t {
    auto it = std::lower_bound(metrics.begin(), metrics.end(), key, [](const MetricRef& x, int64_t k) { return x.key < k; });
    return it != metrics.end() && it->key == key ? it - metrics.begin() : -1;
  };
  const bool has_ut = ns.nm.has_update_time;
  const int64_t ut = ns.nm.update_time_ns;
  const int64_t interval = ns.nm.report_interval_seconds != KE_ABSENT ? ns.nm.report_interval_seconds * NS : DEFAULT_REPORT_INTERVAL_NS;
  const bool score_agg = a.has_aggregated && a.agg_score_type != KE_AGG_NONE;
  const bool score_agg_missing = score_agg && target_aggregated(ns, a.agg_score_duration_ns, a.agg_score_type) == nullptr;
  for (const auto& info : ns.asg) {  // estimatedAssignedPodUsed (load_aware.go:315-358)
    if (prod && info.pod.priority_class != KE_PRIORITY_PROD) continue;
    const int64_t j = find_metric(info.pod.pod_key);
    const ke_pod_metric* m = j < 0 ? nullptr : &ns.pm[(size_t)metrics[(size_t)j].idx];
    const bool static_cond = (m == nullptr || m->usage.n_keys == 0) || (has_ut ? info.ts > ut : true) ||
                             (has_ut && info.ts < ut && ut - info.ts < interval) || score_agg_missing;
    if (!static_cond) {
      int64_t w = estimate_window_end(a, info, now);
      if (w < *valid_until) *valid_until = w;
    }
    if (static_cond || should_estimate(a, info, now)) {
      if (!info.has_est) continue;
      for (int r = 0; r < KE_NRES; r++) {
        if (!info.est_present[r]) continue;
        int64_t v = info.est[r];
        if (m && m->usage.present[r] && m->usage.value[r] > v) v = m->usage.value[r];
        t.assigned[r] += v;
      }
      if (j >= 0) est[(size_t)j] = 1;  // estimatedPods (only its members with a metric are read below)
    }
  }
  for (size_t j = 0; j < metrics.size(); j++) {  // sumPodUsages (helper.go:172-186)
    const ke_pod_metric& m = ns.pm[(size_t)metrics[j].idx];
    for (int r = 0; r < KE_NRES; r++) {
      if (!m.usage.present[r]) continue;
      (est[j] ? t.est_actual : t.other_actual)[r] += m.usage.value[r];
    }
  }
  return t;
}

// non-prod usage contribution: nodeUsage minus the estimated pods' actual usage when covered
// (load_aware.go:271-283)
static void add_usage(const ke_resource_map* usage, const Terms& t, int64_t* term) {
  if (!usage) return;
  for (int r = 0; r < KE_NRES; r++) {
    if (!usage->present[r]) continue;
    int64_t q = usage->value[r];
    if (t.est_actual[r] != 0 && q >= t.est_actual[r]) q -= t.est_actual[r];
    term[r] += q;
  }
}

void derive_row(const ke_config& cfg, const NodeState& ns, int64_t now, Row* row, int64_t* valid_until) {
  std::memset(row, 0, sizeof(Row));
  *valid_until = INT64_MAX;
  if (!ns.valid) return;
  const ke_loadaware_args& a = cfg.loadaware;
  const ke_node& n = ns.node;
  uint32_t flags = NF_VALID;

  // ---- LoadAwareScheduling
  int64_t cap[KE_NRES];  // EstimateNode (default_estimator.go:124-143)
  for (int r = 0; r < KE_NRES; r++) cap[r] = n.raw_allocatable[r] != KE_ABSENT ? n.raw_allocatable[r] : n.allocatable[r];
  for (int r = 0; r < KE_NRES; r++) row->f[F_CAP + r] = cap[r];
  if (ns.has_metric) {
    flags |= NF_HAS_METRIC;
    if (ns.nm.has_update_time) flags |= NF_HAS_UT;
    row->f[F_UT] = ns.nm.update_time_ns;
    if (!ns.nm.has_node_metric) flags |= NF_NM_NIL;
  }
  if (ns.has_metric && ns.nm.has_node_metric) {
    const Profile prof = filter_profile(a, n);
    if (any_present(prof.prod)) flags |= NF_HAS_PROD_THR;
    if (prof.has_agg) flags |= NF_FILTER_AGG;
    const Terms tnp = compute_terms(a, ns, false, now, valid_until);
    const Terms tp = compute_terms(a, ns, true, now, valid_until);
    // filter terms
    int64_t term_f[2][KE_NRES], term_s[2][KE_NRES];
    for (int r = 0; r < KE_NRES; r++) {
      term_f[0][r] = term_s[0][r] = tnp.assigned[r];
      term_f[1][r] = term_s[1][r] = tp.assigned[r] + tp.other_actual[r];
    }
    add_usage(prof.has_agg ? target_aggregated(ns, prof.agg_dur, prof.agg_type) : &ns.nm.node_usage, tnp, term_f[0]);
    const bool score_agg = a.has_aggregated && a.agg_score_type != KE_AGG_NONE;
    add_usage(score_agg ? target_aggregated(ns, a.agg_score_duration_ns, a.agg_score_type) : &ns.nm.node_usage, tnp, term_s[0]);
    const int64_t* thr[2] = {prof.has_agg ? prof.agg_thr : prof.usage, prof.prod};
    for (int v = 0; v < 2; v++) {
      for (int r = 0; r < KE_NRES; r++) {
        const int64_t th = thr[v][r];
        const bool on = th != KE_ABSENT && th != 0 && cap[r] != 0;
        if (on) {
          flags |= nf_fh_on(v, r);
          row->f[F_FH + 2 * v + r] = max_used_within(cap[r], th) - term_f[v][r];
        }
        row->f[F_SA + 2 * v + r] = cap[r] - term_s[v][r];
      }
    }
  }

  // ---- NodeNUMAResource (policy None, non-cpuset pods)
  for (int r = 0; r < KE_NRES; r++) {
    row->f[F_NALLOC + r] = n.allocatable[r];
    row->f[F_NREQ + r] = n.requested[r] + ns.rv_req[r];  // NodeInfo.Requested after the reservation restore
  }
  const int64_t cs_milli = cpus_allocated(ns) * 1000;
  row->f[F_CSM] = cs_milli;
  if (n.amplification_error) flags |= NF_NUMA_AMP_ERR;
  if (n.cpu_topology_invalid) flags |= NF_NUMA_TOPO_INVALID;
  const double ratio_f = n.cpu_amplification_ratio;  // filterAmplifiedCPUs reads the annotation (plugin.go:420-427)
  if (ratio_f > 1.0) flags |= NF_NUMA_RATIO_F;
  row->f[F_CSAF] = amplify(cs_milli, ratio_f);
  double ratio_s;  // Score: TopologyOptions ratios, else the annotation (util.go:78-87)
  if (n.nrt_cpu_amplification_ratio > -1.5) {
    ratio_s = n.nrt_cpu_amplification_ratio < 0 ? 0.0 : n.nrt_cpu_amplification_ratio;
  } else {
    if (n.amplification_error) flags |= NF_NUMA_SCORE_ZERO;
    ratio_s = n.cpu_amplification_ratio < 0 ? 0.0 : n.cpu_amplification_ratio;
  }
  if (ratio_s > 1.0) flags |= NF_NUMA_RATIO_S;
  row->f[F_CSAS] = amplify(cs_milli, ratio_s);
  if (ns.has_dev_cache) flags |= NF_DS_CACHE;
  flags |= (uint32_t)n.numa_topology_policy * NF_NUMA_POLICY0;
  flags |= (uint32_t)n.cpu_bind_policy * NF_CPU_BIND0;
  if (cpus_valid(ns)) flags |= NF_CPUS_VALID;
  if (ns.rsv_ovr) flags |= NF_RSV_CS;
  // GetNUMAAllocateStrategy (util.go:33-47): the node label, else NUMAScoringStrategy's type
  if (n.numa_allocate_strategy == KE_NUMA_ALLOCATE_MOST ||
      (n.numa_allocate_strategy == KE_NUMA_ALLOCATE_DEFAULT && cfg.numa.numa_strategy == KE_STRATEGY_MOST_ALLOCATED))
    flags |= NF_CPU_NUMA_MOST;
  if (n.nrt_cpu_amplification_ratio <= -1.5 && n.amplification_error) flags |= NF_NUMA_OPT_ERR;
  {  // TopologyOptions.AmplificationRatios[cpu]: the NRT's ratios, else the node annotation's
    const double r = n.nrt_cpu_amplification_ratio > -1.5 ? n.nrt_cpu_amplification_ratio : n.cpu_amplification_ratio;
    if (r > 1.0) flags |= NF_NUMA_AL_AMP;
  }
  row->flags = flags;
}

int validate_zones(int32_t n, const ke_numa_zone* zones) {
  if (n < 0 || n > KE_MAX_NUMA || (n > 0 && !zones)) return fail(KE_ERR_INVALID, "NUMA zone count");
  for (int32_t i = 0; i < n; i++) {
    if (zones[i].id < 0 || zones[i].id >= KE_MAX_NUMA) return fail(KE_ERR_INVALID, "NUMA zone id out of range");
    if (i > 0 && zones[i].id <= zones[i - 1].id) return fail(KE_ERR_INVALID, "NUMA zones must ascend by id");
    for (int r = 0; r < KE_NRES; r++)
      if (zones[i].capacity[r] < 0 || zones[i].cpuset_cpus < 0) return fail(KE_ERR_INVALID, "negative NUMA quantity");
    if (zones[i].cpuset_cpus > 0 && !(zones[i].has_allocated & KE_NUMA_ALLOC_ENTRY))
      return fail(KE_ERR_INVALID, "cpuset CPUs allocated in a zone without an allocation entry");
    if (zones[i].has_allocated > 7 || (zones[i].has_allocated && !(zones[i].has_allocated & KE_NUMA_ALLOC_ENTRY)))
      return fail(KE_ERR_INVALID, "NUMA allocation keys without an allocation entry");
    if (zones[i].numa_status > KE_NUMA_STATUS_SHARED) return fail(KE_ERR_INVALID, "NUMA node status");
    if (zones[i].single_pods < 0 || zones[i].shared_pods < 0) return fail(KE_ERR_INVALID, "negative NUMA pod count");
    if ((zones[i].single_pods || zones[i].shared_pods) && zones[i].numa_status != zone_status(zones[i]))
      return fail(KE_ERR_INVALID, "NUMA node status disagrees with its single / shared pod counts");
  }
  return KE_OK;
}

uint8_t zone_status(const ke_numa_zone& z) {
  if (z.shared_pods > 0) return KE_NUMA_STATUS_SHARED;
  return z.single_pods > 0 ? KE_NUMA_STATUS_SINGLE : KE_NUMA_STATUS_IDLE;
}

void normalize_zone(ke_numa_zone& z) {
  if (z.single_pods || z.shared_pods) return;
  if (z.numa_status == KE_NUMA_STATUS_SINGLE) z.single_pods = 1;
  if (z.numa_status == KE_NUMA_STATUS_SHARED) z.shared_pods = 1;
}

// getResourceOptions -> amplifyNUMANodeResources (util.go:78-98): the NUMA zones' cpu is amplified with
// the node annotation's ratio unless the NRT reported ratios; getAvailableNUMANodeResources
// (node_allocation.go:221-243) adjusts the allocated cpu of amplified cpusets.
void derive_numa_row(const NodeState& ns, int64_t* f, uint64_t* mask) {
  for (int i = 0; i < NUM_NUMA_FIELDS; i++) f[i] = 0;
  *mask = 0;
  const ke_node& n = ns.node;
  double ratio;
  bool amplify_caps = false;
  if (n.nrt_cpu_amplification_ratio > -1.5) {
    ratio = n.nrt_cpu_amplification_ratio < 0 ? 0.0 : n.nrt_cpu_amplification_ratio;
  } else {
    ratio = n.cpu_amplification_ratio < 0 ? 0.0 : n.cpu_amplification_ratio;
    amplify_caps = true;
  }
  for (const ke_numa_zone& z : ns.zones) {
    const int id = z.id;
    *mask |= 1ull << id;
    if (id < (int)ns.zones.size()) {  // GetAllNUMANodeStatus(len(numaNodes)) covers ids 0..n-1
      if (zone_status(z) == KE_NUMA_STATUS_SINGLE) *mask |= 1ull << (NUMA_M_ST + id);
      if (zone_status(z) == KE_NUMA_STATUS_SHARED) *mask |= 1ull << (NUMA_M_ST + 8 + id);
    }
    for (int r = 0; r < KE_NRES; r++) {
      if (z.has[r]) {
        *mask |= 1ull << (NUMA_M_CAP + 8 * r + id);
        int64_t c = z.capacity[r];
        if (r == KE_RES_CPU && amplify_caps && ratio > 1.0 && c != 0) c = amplify(c, ratio);
        f[NUMA_CAP + 2 * id + r] = c;
      }
    }
    if (z.has_allocated & KE_NUMA_ALLOC_ENTRY) {
      for (int r = 0; r < KE_NRES; r++)
        if (z.has_allocated & (r == KE_RES_CPU ? KE_NUMA_ALLOC_CPU : KE_NUMA_ALLOC_MEMORY)) {
          *mask |= 1ull << (NUMA_M_AL + 8 * r + id);
          f[NUMA_AL + 2 * id + r] = z.allocated[r];
        }
      if (ratio > 1.0) {  // the cpu key is (re)written even when the entry had none
        int64_t cs = (int64_t)z.cpuset_cpus * 1000;  // allocatedCPUs.CPUsInNUMANodes(id).Size()
        if (!ns.cpus.empty()) {
          cs = 0;
          for (const ke_cpu& c : ns.cpus) cs += (c.ref_count > 0 && c.numa_id == id) ? 1000 : 0;
        }
        f[NUMA_AL + 2 * id] = f[NUMA_AL + 2 * id] - cs + amplify(cs, ratio);
        *mask |= 1ull << (NUMA_M_AL + id);
      }
      // allocatedRes = SubtractWithNonNegativeResult(allocatedRes, reusableResources[id]) (node_allocation.go:237):
      // the unmatched reservations' owners' part (resv_plugin_restore); keys of both lists
      if (ns.rv_numa_zones >> id & 1)
        for (int r = 0; r < KE_NRES; r++) {
          const bool key = ns.rv_numa_keys >> (2 * id + r) & 1;
          const bool had = *mask >> (NUMA_M_AL + 8 * r + id) & 1;
          if (!key && !had) continue;
          const int64_t v = (had ? f[NUMA_AL + 2 * id + r] : 0) - ns.rv_numa[2 * id + r];
          f[NUMA_AL + 2 * id + r] = v > 0 ? v : 0;
          *mask |= 1ull << (NUMA_M_AL + 8 * r + id);
        }
    }
  }
}

void host_numa_reserve(NodeState& ns, const int64_t* delta) {
  // resourceManager.Update records nothing on a node without a valid CPU topology (resource_manager.go:461-466)
  if (!cpus_valid(ns)) return;
  for (ke_numa_zone& z : ns.zones) {
    const int64_t d[KE_NRES] = {delta[2 * z.id], delta[2 * z.id + 1]};
    if (d[0] == 0 && d[1] == 0) continue;
    for (int r = 0; r < KE_NRES; r++) {  // quotav1.Add(entry, allocation): keys with a non-zero amount
      const uint8_t key = r == KE_RES_CPU ? KE_NUMA_ALLOC_CPU : KE_NUMA_ALLOC_MEMORY;
      if (!(z.has_allocated & key)) z.allocated[r] = 0;
      if (d[r] != 0) z.has_allocated |= key;
      z.allocated[r] += d[r];
    }
    z.has_allocated |= KE_NUMA_ALLOC_ENTRY;
  }
}

// ---------------------------------------------------------------------------------------------
// CPU topology (cpu_topology.go:24-105) and cpuset allocations (node_allocation.go:33-156)
// ---------------------------------------------------------------------------------------------
// The device accumulator keeps per CPU its core / socket rank and NUMA id in a byte each and reduces
// the required-policy Filter to counts, which needs a regular topology: every core
// in one socket and NUMA node with the same number (<= 8) of logical CPUs.
int validate_cpus(int32_t n, const ke_cpu* cpus, int32_t max_ref) {
  if (n < 0 || n > KE_MAX_CPUS || (n > 0 && !cpus)) return fail(KE_ERR_INVALID, "CPU count");
  if (n == 0) return KE_OK;
  if (max_ref < 1 || max_ref > 255) return fail(KE_ERR_INVALID, "MaxRefCount must be in 1..255");
  bool seen[KE_MAX_CPUS] = {};
  for (int32_t i = 0; i < n; i++) {
    const ke_cpu& c = cpus[i];
    if (c.cpu_id < 0 || c.cpu_id >= KE_MAX_CPUS || seen[c.cpu_id]) return fail(KE_ERR_INVALID, "CPU id out of range or repeated");
    seen[c.cpu_id] = true;
    if (c.core_id < 0 || c.socket_id < 0 || c.numa_id < 0 || c.numa_id > 255)
      return fail(KE_ERR_INVALID, "CPU core / socket / NUMA id");
    if (c.ref_count < 0 || c.ref_count > 255 || c.exclusive > KE_CPU_EXCL_NUMA_NODE_LEVEL || c.reserved > 1)
      return fail(KE_ERR_INVALID, "CPU allocation state");
  }
  std::map<int32_t, std::pair<int32_t, int32_t>> where;  // core id -> (socket, NUMA node)
  std::map<int32_t, int> per_core;
  for (int32_t i = 0; i < n; i++) {
    auto it = where.find(cpus[i].core_id);
    if (it == where.end()) where[cpus[i].core_id] = {cpus[i].socket_id, cpus[i].numa_id};
    else if (it->second != std::make_pair(cpus[i].socket_id, cpus[i].numa_id))
      return fail(KE_ERR_UNSUPPORTED, "a core id spanning sockets / NUMA nodes");
    per_core[cpus[i].core_id]++;
  }
  const int cpc = per_core.begin()->second;
  for (const auto& kv : per_core)
    if (kv.second != cpc) return fail(KE_ERR_UNSUPPORTED, "cores with different numbers of logical CPUs");
  if (cpc > 8) return fail(KE_ERR_UNSUPPORTED, "more than 8 logical CPUs per core");
  return KE_OK;
}

bool cpus_valid(const NodeState& ns) { return !ns.cpus.empty() && !ns.node.cpu_topology_invalid; }

int64_t cpus_allocated(const NodeState& ns) {
  if (ns.cpus.empty()) return ns.node.cpuset_allocated_cpus;
  int64_t k = 0;
  for (const ke_cpu& c : ns.cpus) k += c.ref_count > 0;
  return k;
}

void derive_cpu_rows(const NodeState& ns, CpuRec* recs, int64_t* cs) {
  std::memset(recs, 0, sizeof(CpuRec) * CPU_SLOTS);
  const ke_node& n = ns.node;
  const double ratio_f = n.cpu_amplification_ratio;
  const double ratio_s = n.nrt_cpu_amplification_ratio > -1.5
                             ? (n.nrt_cpu_amplification_ratio < 0 ? 0.0 : n.nrt_cpu_amplification_ratio)
                             : (n.cpu_amplification_ratio < 0 ? 0.0 : n.cpu_amplification_ratio);
  std::memcpy(&cs[CS_RF], &ratio_f, 8);
  std::memcpy(&cs[CS_RS], &ratio_s, 8);
  for (int f = CS_CNT; f < NUM_CS_FIELDS; f++) cs[f] = 0;
  if (ns.cpus.empty()) return;
  std::vector<int32_t> cores, sockets;
  for (const ke_cpu& c : ns.cpus) cores.push_back(c.core_id), sockets.push_back(c.socket_id);
  std::sort(cores.begin(), cores.end());
  cores.erase(std::unique(cores.begin(), cores.end()), cores.end());
  std::sort(sockets.begin(), sockets.end());
  sockets.erase(std::unique(sockets.begin(), sockets.end()), sockets.end());
  for (const ke_cpu& c : ns.cpus) {
    CpuRec& r = recs[c.cpu_id];
    r.core = (uint8_t)(std::lower_bound(cores.begin(), cores.end(), c.core_id) - cores.begin());
    r.socket = (uint8_t)(std::lower_bound(sockets.begin(), sockets.end(), c.socket_id) - sockets.begin());
    r.numa = (uint8_t)c.numa_id;
    r.ref = (uint8_t)c.ref_count;
    r.excl = c.ref_count > 0 ? c.exclusive : 0;
    r.flags = (uint8_t)(CR_VALID | (c.reserved ? CR_RESERVED : 0));
  }
  const int cpc = (int)(ns.cpus.size() / cores.size());
  uint8_t scratch[CPU_SLOTS];
  cs_fill(recs, cpc, ns.cpu_max_ref, scratch, &cs[CS_CNT], &cs[CS_ZALL]);
  std::vector<std::pair<int32_t, int32_t>> nodes;  // (socket, NUMA node) pairs
  for (const ke_cpu& c : ns.cpus) nodes.push_back({c.socket_id, c.numa_id});
  std::sort(nodes.begin(), nodes.end());
  nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
  cs[CS_TOPO] = (int64_t)ns.cpus.size() | ((int64_t)cores.size() << 16) | ((int64_t)nodes.size() << 32) |
                ((int64_t)sockets.size() << 48);
}

void host_cpuset_reserve(NodeState& ns, const DevPod& dp, const uint64_t* set) {
  const int excl = (dp.flags & PF_CPU_RCB) ? pf_cpu_excl(dp.flags) : KE_CPU_EXCL_NONE;
  uint32_t used = 0;  // NUMA ids < 32 of the new cpuset (zones carry ids < KE_MAX_NUMA)
  int n_used = 0;
  std::vector<int> ids;
  for (ke_cpu& c : ns.cpus) {
    if (!(set[c.cpu_id >> 6] >> (c.cpu_id & 63) & 1)) continue;
    c.ref_count++;
    c.exclusive = (uint8_t)excl;
    if (std::find(ids.begin(), ids.end(), c.numa_id) == ids.end()) ids.push_back(c.numa_id);
  }
  n_used = (int)ids.size();
  for (int id : ids)
    if (id < 32) used |= 1u << id;
  for (ke_numa_zone& z : ns.zones)  // sharedNode / singleNUMANode after addPodAllocation
    if (z.id < 32 && (used >> z.id & 1)) {
      if (n_used > 1) z.shared_pods++;
      else z.single_pods++;
      z.numa_status = zone_status(z);
    }
  ns.dirty = true;
}

void host_release_node(const ke_config& cfg, bool ext, NodeState& ns, const ke_pod& pod, const ke_pod_allocation& a,
                       const ke_pod_device_hints* h) {
  // LoadAware podAssignCache.unAssign (pod_assign_cache.go:126-136)
  for (size_t i = 0; i < ns.asg_uid.size(); i++)
    if (ns.asg_uid[i] == pod.uid) {
      ns.asg.erase(ns.asg.begin() + (long)i);
      ns.asg_uid.erase(ns.asg_uid.begin() + (long)i);
      break;
    }
  // framework NodeInfo.RemovePod: Requested and (NonZero)Requested by resource id (read by FitPlus -- whose device
  // rows follow when `ext` -- and by the Reservation plugin's fitsNode)
  (void)ext;
  ns.node.requested[KE_RES_CPU] -= pod.requests[KE_RES_CPU];
  ns.node.requested[KE_RES_MEMORY] -= pod.requests[KE_RES_MEMORY];
  ns.node.pod_count--;
  for (int e = 0; e < pod.n_xres; e++)
    for (ke_node_resource& r : ns.xres)
      if (r.id == pod.xres_id[e]) r.requested -= pod.xres_value[e];
  // NodeNUMAResource resourceManager.Release -> NodeAllocation.release (node_allocation.go:158-190); only a
  // node with a valid CPU topology recorded the allocation (Update, resource_manager.go:461-466).  While the
  // NRT is deleted the NodeAllocation lives on in the parked tables (ke_node_topology_delete).
  const bool parked = ns.cpus.empty() && !ns.kept_cpus.empty();
  if (cpus_valid(ns) || parked) {
    std::vector<ke_cpu>& cpus = parked ? ns.kept_cpus : ns.cpus;
    std::vector<ke_numa_zone>& zones = parked ? ns.kept_zones : ns.zones;
    std::vector<int> ids;
    for (ke_cpu& c : cpus) {
      if (!(a.cpuset[c.cpu_id >> 6] >> (c.cpu_id & 63) & 1) || c.ref_count <= 0) continue;
      if (--c.ref_count == 0) c.exclusive = KE_CPU_EXCL_NONE;  // the CPU leaves allocatedCPUs
      if (std::find(ids.begin(), ids.end(), c.numa_id) == ids.end()) ids.push_back(c.numa_id);
    }
    for (ke_numa_zone& z : zones) {
      if (std::find(ids.begin(), ids.end(), z.id) != ids.end()) {  // delete(sharedNode / singleNUMANode[id], uid)
        int16_t& k = ids.size() > 1 ? z.shared_pods : z.single_pods;
        if (k > 0) k--;
        z.numa_status = zone_status(z);
      }
      if (!(z.has_allocated & KE_NUMA_ALLOC_ENTRY)) continue;  // allocatedResources[id] == nil
      for (int r = 0; r < KE_NRES; r++) {  // quotav1.SubtractWithNonNegativeResult: keys of both, floor 0
        const int64_t b = a.numa[2 * z.id + r];
        if (b == 0) continue;
        const uint8_t key = r == KE_RES_CPU ? KE_NUMA_ALLOC_CPU : KE_NUMA_ALLOC_MEMORY;
        const int64_t v = ((z.has_allocated & key) ? z.allocated[r] : 0) - b;
        z.allocated[r] = v > 0 ? v : 0;
        z.has_allocated |= key;
      }
    }
  }
  // DeviceShare updateCacheUsed(allocation, pod, false) -> updateDeviceUsed (device_cache.go:184-209)
  if (ns.has_dev_cache && a.device_minors) {
    const DevPod dp = make_dev_pod(cfg, pod, h);
    for (ke_device& d : ns.devs) {
      if (!(a.device_minors & (1ull << (16 * d.type + d.minor)))) continue;
      if (d.type > 0 && a.vf_rank[d.type - 1][d.minor] >= 0)  // removeVFAllocations (device_cache.go:283-300)
        d.vf_allocated &= ~(1ull << a.vf_rank[d.type - 1][d.minor]);
      const int t = d.type;
      int64_t alloc[KE_DKEYS] = {0, 0, 0};
      bool has[KE_DKEYS] = {false, false, false};
      if (t == KE_DEV_GPU) {  // the amounts Reserve added (fillGPUTotalMem, host_ds_reserve)
        const int64_t tm = d.health && d.has_total[KE_DKEY_GPU_MEMORY] ? d.total[KE_DKEY_GPU_MEMORY] : 0;
        if (dp.flags & PF_DS_H_CORE) has[0] = true, alloc[0] = dp.ds_req[0];
        if (dp.flags & PF_DS_H_RATIO) {
          has[2] = true, alloc[2] = dp.ds_req[2];
          has[1] = true, alloc[1] = dp.ds_req[2] * tm / 100;
        } else if (dp.flags & PF_DS_H_MEM) {
          has[1] = true, alloc[1] = dp.ds_req[1];
          has[2] = true, alloc[2] = (int64_t)((double)dp.ds_req[1] / (double)tm * 100.0);
        }
      } else {
        has[0] = true, alloc[0] = dp.ds_req[2 + t];
      }
      bool zero = true;
      for (int k = 0; k < DS_NK[t]; k++) {  // SubtractWithNonNegativeResult over the keys of both
        if (has[k]) {
          const int64_t v = (d.has_used[k] ? d.used[k] : 0) - alloc[k];
          d.used[k] = v > 0 ? v : 0;
          d.has_used[k] = 1;
        } else if (d.has_used[k] && d.used[k] < 0) {
          d.used[k] = 0;
        }
        zero = zero && (!d.has_used[k] || d.used[k] == 0);
      }
      if (zero)  // quotav1.IsZero(used): the minor's used entry is deleted
        for (int k = 0; k < KE_DKEYS; k++) d.has_used[k] = 0, d.used[k] = 0;
    }
  }
  ns.dirty = true;
}

// the mirror of placements (node, timestamp, pods[idx]) onto the host node state: LoadAware assign cache and
// NodeInfo.Requested / pod count (+ FitPlus requests).  The device rows already carry these Reserves: the nodes'
// dirty flags stay as they are.  Random nodes: cache-miss bound, so the node records (vector headers) are
// prefetched 16 entries ahead and their arrays 8 ahead.
static void apply_mirror(Context& c, const std::vector<Context::PendingAssign>& pending, const std::vector<ke_pod>& pods) {
  const size_t n = pending.size();
  for (size_t k = 0; k < n; k++) {
    if (k + 16 < n) __builtin_prefetch(&c.nodes[pending[k + 16].node].asg, 1);
    if (k + 8 < n) {
      const NodeState& q = c.nodes[pending[k + 8].node];
      __builtin_prefetch(q.asg_uid.data(), 0);
      __builtin_prefetch(q.asg.data() + q.asg.size(), 1);
      __builtin_prefetch(&q.node.requested[0], 1);
    }
    const Context::PendingAssign& a = pending[k];
    NodeState& ns = c.nodes[a.node];
    const ke_pod& pod = pods[(size_t)a.idx];
    host_assign(c.cfg, ns, pod, a.ts, false);
    ns.node.requested[KE_RES_CPU] += pod.requests[KE_RES_CPU];
    ns.node.requested[KE_RES_MEMORY] += pod.requests[KE_RES_MEMORY];
    ns.node.pod_count++;  // NodeInfo.AddPod
    host_ext_reserve(ns, pod);  // NodeInfo.Requested.ScalarResources (FitPlus and the Reservation plugin read them)
  }
}

void mirror_join(Context& c) {
  if (c.mirror_thread.joinable()) c.mirror_thread.join();
}

void flush_mirror(Context& c) {
  mirror_join(c);
  apply_mirror(c, c.pending, c.pending_pods);
  c.pending.clear();
  c.pending_pods.clear();
}

// The queued mirror on a host thread (the lists move to it; later placements queue anew).  It writes only the
// nodes' assign caches, requested amounts and pod counts -- never a dirty flag or list -- and every reader of those
// joins it first.  A worker per node residue was measured slower than this one thread (the allocator's locks).
void flush_mirror_async(Context& c) {
  mirror_join(c);
  if (c.pending.empty()) return;
  auto* pend = new std::vector<Context::PendingAssign>(std::move(c.pending));
  auto* pods = new std::vector<ke_pod>(std::move(c.pending_pods));
  c.pending.clear();
  c.pending_pods.clear();
  c.mirror_thread = std::thread([&c, pend, pods]() {
    apply_mirror(c, *pend, *pods);
    delete pend;
    delete pods;
  });
}

void host_assign(const ke_config& cfg, NodeState& ns, const ke_pod& pod, int64_t timestamp_ns, bool mark_dirty) {
  if (pod.is_terminated) return;  // pod_assign_cache.go:90
  AssignedPod info{};
  info.pod.pod_key = pod.pod_key;
  info.pod.custom_seconds_after_scheduled = pod.custom_seconds_after_scheduled;
  info.pod.custom_seconds_after_initialized = pod.custom_seconds_after_initialized;
  info.pod.initialized_transition_ns = pod.initialized_transition_ns;
  info.pod.priority_class = pod.priority_class;
  info.pod.has_initialized = pod.has_initialized;
  estimate_pod(cfg.loadaware, pod, info.est, info.est_present);
  info.has_est = info.est_present[0] || info.est_present[1];
  for (size_t i = 0; i < ns.asg_uid.size(); i++) {
    if (ns.asg_uid[i] == pod.uid) {  // existing entry: refresh pod + estimate, keep timestamp
      info.ts = ns.asg[i].ts;
      ns.asg[i] = info;
      if (mark_dirty) ns.dirty = true;
      return;
    }
  }
  info.ts = pod.has_scheduled ? pod.scheduled_transition_ns : timestamp_ns;
  ns.asg.push_back(info);
  ns.asg_uid.push_back(pod.uid);
  if (mark_dirty) ns.dirty = true;
}

}  // namespace ke

namespace ke {

// ---------------------------------------------------------------------------------------------
// ElasticQuota runtime (pkg/scheduler/plugins/elasticquota/core).  Requests are fixed for a
// ke_schedule call, so the incremental GroupQuotaManager state reduces to one pass per resource:
// limited requests bottom-up (recursiveUpdateGroupTreeWithDeltaRequest, group_quota_manager.go:196-239;
// getLimitRequestNoLock, quota_info.go:217-228), then each parent's RuntimeQuotaCalculator shares its
// runtime among its children top-down (refreshRuntimeNoLock :286-353; quotaTree.redistribution /
// iterationForRedistribution, runtime_quota_calculator.go:117-189).  System / default quotas
// (limit_is_max) stay out of the sharing; their limit is Max.
// ---------------------------------------------------------------------------------------------
namespace {
struct QuotaShare {
  int64_t weight, request, min;
  bool lent;
  int64_t runtime;
};

// one calculator: `total` shared among `kids` (min first, then sharedWeight water-filling)
void share_runtime(int64_t total, std::vector<QuotaShare*>& kids) {
  std::vector<QuotaShare*> open;
  int64_t left = total, wsum = 0;
  for (QuotaShare* c : kids) {
    if (c->request > c->min) {  // wants more than its min: starts at min, joins the sharing
      c->runtime = c->min;
      open.push_back(c);
      wsum += c->weight;
    } else {
      c->runtime = c->lent ? c->request : c->min;
    }
    left -= c->runtime;
  }
  if (left <= 0) return;
  while (wsum > 0 && !open.empty()) {
    std::vector<QuotaShare*> still;
    int64_t spare = 0, still_w = 0;
    for (QuotaShare* c : open) {
      // int64(float64(sharedWeight)*float64(totalRes)/float64(totalSharedWeight) + 0.5)
      const double share = static_cast<double>(c->weight) * static_cast<double>(left) / static_cast<double>(wsum) + 0.5;
      c->runtime += static_cast<int64_t>(share);
      if (c->runtime < c->request) {
        still.push_back(c);
        still_w += c->weight;
      } else {
        spare += c->runtime - c->request;
        c->runtime = c->request;
      }
    }
    if (spare <= 0) break;
    open.swap(still);
    left = spare;
    wsum = still_w;
  }
}
}  // namespace

int host_quota_release(Context& c, const ke_pod& pod, bool assigned, bool del) {
  if (pod.quota <= 0 || pod.quota > (int32_t)c.quotas.size()) return KE_OK;
  const int qi = pod.quota - 1;
  int64_t req[KE_NRES];  // quotav1.Mask(PodRequests, ResourceNames(Max)) of the pod's own quota
  for (int r = 0; r < KE_NRES; r++)
    req[r] = c.quotas[(size_t)qi].has_max[r] ? pod.requests[r == 0 ? KE_RES_CPU : KE_RES_MEMORY] : 0;
  bool refresh = false;
  if (assigned) {  // updateGroupDeltaUsedNoLock with -request: the quota and every ancestor, floor 0 each
    int64_t before[KE_NRES];
    for (int r = 0; r < KE_NRES; r++) before[r] = c.quotas[(size_t)qi].used[r];
    for (int q = qi; q >= 0; q = c.quotas[(size_t)q].parent)
      for (int r = 0; r < KE_NRES; r++) {
        ke_quota& x = c.quotas[(size_t)q];
        x.used[r] = std::max<int64_t>(0, x.used[r] - req[r]);
        if (pod.quota_non_preemptible) x.non_preemptible_used[r] = std::max<int64_t>(0, x.non_preemptible_used[r] - req[r]);
      }
    // a system / default quota's used shrank: totalResourceExceptSystemAndDefaultUsed grows by as much
    // (updateClusterTotalResourceNoLock, group_quota_manager.go:127-151,268-271)
    if (c.quotas[(size_t)qi].limit_is_max && c.qargs.enable_runtime_quota) {
      for (int r = 0; r < KE_NRES; r++) c.qargs.total[r] += before[r] - c.quotas[(size_t)qi].used[r];
      refresh = true;
    }
  }
  if (del) {  // updatePodRequestNoLock(quota, pod, nil): SelfRequest, floor 0 (quota_info.go:238-258)
    for (int r = 0; r < KE_NRES; r++)
      c.quotas[(size_t)qi].self_request[r] = std::max<int64_t>(0, c.quotas[(size_t)qi].self_request[r] - req[r]);
    refresh = true;
  }
  if (refresh) {
    const int rc = quota_compute_limits(c.qargs, c.quotas, c.qlimit, c.qlimit_has);
    if (rc) return rc;
  }
  c.quota_dirty = true;
  c.quota_on_device = false;  // the host tree is now the current one
  return KE_OK;
}

int quota_compute_limits(const ke_quota_args& args, const std::vector<ke_quota>& q, std::vector<int64_t>& limit,
                         std::vector<uint8_t>& has) {
  const int n = (int)q.size();
  std::vector<std::vector<int>> kids(n + 1);  // kids[n] = children of the root quota
  std::vector<int> order;                     // parents before children
  for (int i = 0; i < n; i++) {
    if (q[i].parent < -1 || q[i].parent >= n) return fail(KE_ERR_INVALID, "ke_quota.parent out of range");
    kids[q[i].parent < 0 ? n : q[i].parent].push_back(i);
  }
  std::vector<int> stack{n};
  while (!stack.empty()) {
    const int p = stack.back();
    stack.pop_back();
    if (p != n) order.push_back(p);
    for (int c : kids[p]) stack.push_back(c);
  }
  if ((int)order.size() != n) return fail(KE_ERR_INVALID, "ke_quota parents form a cycle");
  limit.assign((size_t)n * KE_NRES, 0);
  has.assign((size_t)n * KE_NRES, 0);
  for (int r = 0; r < KE_NRES; r++) {
    std::vector<QuotaShare> sh(n);
    std::vector<int64_t> child_req(n, 0);
    bool tree_key = false;
    for (int i = 0; i < n; i++) tree_key = tree_key || q[i].has_max[r];
    for (int t = n - 1; t >= 0; t--) {  // children before parents
      const int i = order[t];
      const ke_quota& x = q[i];
      int64_t req = child_req[i] + x.self_request[r];
      if (!x.allow_lent_resource && x.has_min[r] && x.min[r] > req) req = x.min[r];
      const int64_t lim = (x.has_max[r] && req > x.max[r]) ? x.max[r] : req;
      sh[i] = QuotaShare{x.shared_weight[r], lim, x.has_min[r] ? x.min[r] : 0, x.allow_lent_resource != 0, 0};
      if (x.parent >= 0) child_req[x.parent] += lim;
    }
    auto share_children = [&](int p, int64_t total) {
      std::vector<QuotaShare*> ks;
      int64_t min_sum = 0;
      for (int c : kids[p])
        if (!q[c].limit_is_max) {
          ks.push_back(&sh[c]);
          min_sum += sh[c].min;
        }
      if (ks.empty()) return;
      // scale-min (scale_minquota_when_over_root_res.go:129-184): the children's Min sum exceeds what
      // the parent shares -> the calculator's AutoScaleMin is each Min's share of `total`
      if (!args.disable_scale_min_quota && total < min_sum)
        for (QuotaShare* c : ks)
          c->min = total <= 0 ? 0
                              : static_cast<int64_t>(static_cast<double>(total) * static_cast<double>(c->min) /
                                                     static_cast<double>(min_sum));
      share_runtime(total, ks);
    };
    share_children(n, args.total[r]);
    for (int i : order) share_children(i, sh[i].runtime);
    for (int i = 0; i < n; i++) {
      const bool use_max = !args.enable_runtime_quota || q[i].limit_is_max;
      has[(size_t)i * KE_NRES + r] = use_max ? q[i].has_max[r] : (uint8_t)tree_key;
      limit[(size_t)i * KE_NRES + r] = use_max ? q[i].max[r] : sh[i].runtime;
    }
  }
  return KE_OK;
}

}  // namespace ke
