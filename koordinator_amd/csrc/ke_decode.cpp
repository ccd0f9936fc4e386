// ke_decode.cpp — SURVEY.md §8f rank 1: the informer objects' wire format (the JSON the apiserver serves) to
// the boundary structs, as the reference's listers and apis/extension helpers read them per call.  Host-only
// C++; a Go caller would instead fill the structs from its typed objects.
//
//   ke_decode_node         Node: status.allocatable, the raw-allocatable / amplification-ratio / usage-thresholds
//                          annotations (apis/extension/node_resource_amplification.go:45-124, load_aware.go:42-72)
//                          and the NUMA / CPU bind / NUMA allocate labels (numa_aware.go:54-59,354-369;
//                          nodenumaresource/util.go:41-47)
//   ke_decode_node_metric  NodeMetric CRD (apis/slo/v1alpha1/nodemetric_types.go:38-136)
//   ke_decode_pod          Pod: resourceapi.PodRequests / PodLimits (k8s v1.28), priority / QoS classes
//                          (apis/extension/priority_utils.go:37-58, qos_utils.go:32-68), the LoadAware estimation
//                          annotations (load_aware.go:75-100), conditions (loadaware/pod_assign_cache.go:89-124,
//                          load_aware.go:360-385), ResourceSpec / NUMATopologySpec (numa_aware.go:62-80,217-243),
//                          the DeviceShare annotations (device_share.go:32-40) and the FitPlus / SRA request names
//   ke_decode_device       Device CRD (apis/scheduling/v1alpha1/device_types.go:32-67) as nodeDeviceCache builds
//                          it (deviceshare/device_cache.go:518-568), plus its GPU partition table and policy
//                          (device_share.go:196-226,355-380)
#include <algorithm>
#include <climits>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/koord_eval.h"
#include "ke_host.h"
#include "ke_json.h"

using namespace ke;
using json::Value;

namespace {

int bad(const std::string& m) { return fail(KE_ERR_INVALID, m); }
int unsup(const std::string& m) { return fail(KE_ERR_UNSUPPORTED, m); }

int parse_doc(const char* js, int64_t len, Value& v, const char* what) {
  if (!js || len < 0) return bad(std::string(what) + ": null input");
  std::string err;
  if (!json::parse(js, (size_t)len, v, err)) return bad(std::string(what) + ": malformed JSON: " + err);
  if (!v.is_obj()) return bad(std::string(what) + ": not a JSON object");
  return KE_OK;
}

// map[string]string (labels / annotations): a non-string value is a malformed object
int string_map(const Value* m, std::map<std::string, std::string>& out, const char* what) {
  out.clear();
  if (!m || m->is_null()) return KE_OK;
  if (!m->is_obj()) return bad(std::string(what) + " is not an object");
  for (const auto& kv : m->o) {
    if (kv.second.t != Value::STR) return bad(std::string(what) + " value is not a string");
    out[kv.first] = kv.second.s;
  }
  return KE_OK;
}

const std::string* lookup(const std::map<std::string, std::string>& m, const char* k) {
  auto it = m.find(k);
  return it == m.end() ? nullptr : &it->second;
}

// corev1.ResourceList: name -> exact quantity (nanos); false on a malformed list / quantity
struct RL {
  std::map<std::string, __int128> q;
  bool overflow = false;
};
bool resource_list(const Value* v, RL& out) {
  out.q.clear();
  out.overflow = false;
  if (!v || v->is_null()) return true;
  if (!v->is_obj()) return false;
  for (const auto& kv : v->o) {
    __int128 n;
    bool ov;
    if (!quantity_json_nanos(kv.second, &n, &ov)) {
      out.overflow |= ov;
      return false;
    }
    out.q[kv.first] = n;
  }
  return true;
}
// getResourceValue (loadaware/helper.go:147-152): cpu MilliValue, everything else Value
bool rl_value(const RL& rl, const std::string& name, int64_t* out) {
  auto it = rl.q.find(name);
  if (it == rl.q.end()) return false;
  int64_t v, m;
  if (!nanos_value(it->second, &v, &m)) return false;
  *out = name == "cpu" ? m : v;
  return true;
}

// map[ResourceName]int64 of cpu / memory (thresholds, scaling factors); other keys -> *other
bool int_map(const Value* v, int64_t (&out)[KE_NRES], bool* other, size_t* n_keys) {
  out[0] = out[1] = KE_ABSENT;
  *other = false;
  if (n_keys) *n_keys = 0;
  if (!v || v->is_null()) return true;
  if (!v->is_obj()) return false;
  bool ok = true;
  std::map<std::string, int64_t> m;
  for (const auto& kv : v->o) {
    int64_t x;
    if (!json::as_int64(kv.second, &x)) ok = false;
    else m[kv.first] = x;
  }
  if (!ok) return false;
  for (const auto& kv : m) {
    if (kv.first == "cpu") out[0] = kv.second;
    else if (kv.first == "memory") out[1] = kv.second;
    else *other = true;
  }
  if (n_keys) *n_keys = m.size();
  return true;
}

const char* str_or_empty(const Value* v) { return v && v->t == Value::STR ? v->s.c_str() : ""; }

int agg_type(const std::string& s, int32_t* out) {
  static const char* names[] = {"", "avg", "p50", "p90", "p95", "p99"};
  for (int i = 0; i < KE_AGG_TYPES; i++)
    if (s == names[i]) {
      *out = i;
      return KE_OK;
    }
  return unsup("aggregation type \"" + s + "\" outside avg/p50/p90/p95/p99");
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

}  // namespace

extern "C" {

int ke_quantity_parse(const char* s, int64_t* value, int64_t* milli_value) {
  if (!s || !value || !milli_value) return bad("ke_quantity_parse arguments");
  bool ov;
  if (!parse_quantity(s, value, milli_value, &ov))
    return ov ? unsup(std::string("quantity out of the int64 range: ") + s) : bad(std::string("malformed quantity: ") + s);
  return KE_OK;
}

// the process-wide label string table (ke_label_id): ids from 1, stable for the process
int32_t ke_label_id(const char* str) {
  if (!str || !*str) return 0;
  static std::mutex mu;
  static std::map<std::string, int32_t> ids;
  std::lock_guard<std::mutex> g(mu);
  auto it = ids.find(str);
  if (it != ids.end()) return it->second;
  const int32_t id = (int32_t)ids.size() + 1;
  ids.emplace(str, id);
  return id;
}

int64_t ke_pod_key(const char* ns, const char* name) {
  return (int64_t)(fnv1a(std::string(ns ? ns : "") + "/" + (name ? name : "")) & (uint64_t)INT64_MAX);
}

int ke_decode_node(const char* js, int64_t len, ke_node* out) {
  if (!out) return bad("ke_decode_node: null output");
  Value doc;
  int rc = parse_doc(js, len, doc, "Node");
  if (rc) return rc;
  ke_node n{};
  n.raw_allocatable[0] = n.raw_allocatable[1] = KE_ABSENT;
  for (int r = 0; r < KE_NRES; r++)
    n.custom_usage_thresholds[r] = n.custom_prod_usage_thresholds[r] = n.custom_agg_thresholds[r] = KE_ABSENT;
  n.cpu_amplification_ratio = -1.0;
  n.nrt_cpu_amplification_ratio = -2.0;  // no NodeResourceTopology in this object
  const Value* meta = doc.field("metadata");
  const Value* status = doc.field("status");
  std::map<std::string, std::string> ann, lab;
  if ((rc = string_map(meta ? meta->field("annotations") : nullptr, ann, "metadata.annotations"))) return rc;
  if ((rc = string_map(meta ? meta->field("labels") : nullptr, lab, "metadata.labels"))) return rc;
  RL alloc;
  if (!resource_list(status ? status->field("allocatable") : nullptr, alloc))
    return alloc.overflow ? unsup("Node allocatable out of range") : bad("Node status.allocatable");
  rl_value(alloc, "cpu", &n.allocatable[0]);
  rl_value(alloc, "memory", &n.allocatable[1]);
  {  // NodeInfo.Allocatable.AllowedPodNumber = int(pods.Value()) (framework.Resource.Add, k8s v1.28.7)
    int64_t pods = 0;
    if (rl_value(alloc, "pods", &pods)) n.allowed_pods = pods > INT32_MAX ? INT32_MAX : (int32_t)pods;
  }
  // raw allocatable (EstimateNode, default_estimator.go:124-143): an unmarshal error falls back to Allocatable
  if (const std::string* s = lookup(ann, "node.koordinator.sh/raw-allocatable")) {
    Value v;
    std::string err;
    RL raw;
    if (json::parse(s->data(), s->size(), v, err) && resource_list(&v, raw)) {
      int64_t x;
      if (rl_value(raw, "cpu", &x)) n.raw_allocatable[0] = x;
      if (rl_value(raw, "memory", &x)) n.raw_allocatable[1] = x;
    }
  }
  // GetNodeResourceAmplificationRatio(annotations, cpu): -1 when unset, an error when unparsable
  if (const std::string* s = lookup(ann, "node.koordinator.sh/resource-amplification-ratio")) {
    Value v;
    std::string err;
    bool ok = json::parse(s->data(), s->size(), v, err) && (v.is_null() || v.is_obj());
    double cpu = -1.0;
    if (ok && v.is_obj())
      for (const auto& kv : v.o) {
        double d;
        if (!json::as_float64(kv.second, &d)) ok = false;
        else if (kv.first == "cpu") cpu = d;
      }
    if (ok) n.cpu_amplification_ratio = cpu;
    else n.amplification_error = 1;
  }
  // CustomUsageThresholds (GetCustomUsageThresholds): present + valid, or present + unmarshal error
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/usage-thresholds")) {
    Value v;
    std::string err;
    bool ok = json::parse(s->data(), s->size(), v, err) && (v.is_null() || v.is_obj());
    bool other = false, o2;
    int64_t u[KE_NRES], pu[KE_NRES], au[KE_NRES];
    u[0] = u[1] = pu[0] = pu[1] = au[0] = au[1] = KE_ABSENT;
    bool has_agg = false;
    int32_t atype = KE_AGG_NONE;
    int64_t adur = 0;
    if (ok && v.is_obj()) {
      ok = int_map(v.field("usageThresholds"), u, &o2, nullptr);
      other |= o2;
      ok = int_map(v.field("prodUsageThresholds"), pu, &o2, nullptr) && ok;
      other |= o2;
      const Value* ag = v.field("aggregatedUsage");
      if (ag && !ag->is_null()) {
        if (!ag->is_obj()) {
          ok = false;
        } else {
          has_agg = true;
          ok = int_map(ag->field("usageThresholds"), au, &o2, nullptr) && ok;
          other |= o2;
          const Value* t = ag->field("usageAggregationType");
          if (t && !t->is_null()) {
            if (t->t != Value::STR) ok = false;
            else if ((rc = agg_type(t->s, &atype))) return rc;
          }
          const Value* d = ag->field("usageAggregatedDuration");
          if (d && !d->is_null() && (d->t != Value::STR || !parse_duration(d->s, &adur))) ok = false;
        }
      }
    }
    if (!ok) {
      n.custom_thresholds_error = 1;
    } else {
      if (other) return unsup("usage-thresholds annotation with resources other than cpu/memory");
      n.has_custom_thresholds = 1;
      for (int r = 0; r < KE_NRES; r++) {
        n.custom_usage_thresholds[r] = u[r];
        n.custom_prod_usage_thresholds[r] = pu[r];
        n.custom_agg_thresholds[r] = au[r];
      }
      n.has_custom_agg = has_agg;
      n.custom_agg_type = atype;
      n.custom_agg_duration_ns = adur;
    }
  }
  // labels
  if (const std::string* s = lookup(lab, "node.koordinator.sh/numa-topology-policy")) {
    if (*s == "") n.numa_topology_policy = KE_NUMA_POLICY_NONE;
    else if (*s == "BestEffort") n.numa_topology_policy = KE_NUMA_POLICY_BEST_EFFORT;
    else if (*s == "Restricted") n.numa_topology_policy = KE_NUMA_POLICY_RESTRICTED;
    else if (*s == "SingleNUMANode") n.numa_topology_policy = KE_NUMA_POLICY_SINGLE_NUMA_NODE;
    else return unsup("NUMA topology policy label \"" + *s + "\"");
  }
  if (const std::string* s = lookup(lab, "node.koordinator.sh/cpu-bind-policy")) {
    if (*s == "FullPCPUsOnly") n.cpu_bind_policy = KE_NODE_CPU_BIND_FULL_PCPUS_ONLY;
    else if (*s == "SpreadByPCPUs") n.cpu_bind_policy = KE_NODE_CPU_BIND_SPREAD_BY_PCPUS;
  }
  if (const std::string* s = lookup(lab, "node.koordinator.sh/numa-allocate-strategy")) {
    if (*s == "MostAllocated") n.numa_allocate_strategy = KE_NUMA_ALLOCATE_MOST;
    else if (*s == "LeastAllocated") n.numa_allocate_strategy = KE_NUMA_ALLOCATE_LEAST;
    else if (*s != "") return unsup("NUMA allocate strategy label \"" + *s + "\"");
  }
  *out = n;
  return KE_OK;
}

// slo/v1alpha1 ResourceMap {resources: ResourceList} -> ke_resource_map (len() of the list kept)
static bool resource_map(const Value* rm, ke_resource_map* out) {
  std::memset(out, 0, sizeof *out);
  if (!rm || rm->is_null()) return true;
  if (!rm->is_obj()) return false;
  RL rl;
  if (!resource_list(rm->field("resources"), rl)) return false;
  for (int r = 0; r < KE_NRES; r++) {
    int64_t x;
    if (rl_value(rl, r == 0 ? "cpu" : "memory", &x)) out->value[r] = x, out->present[r] = 1;
  }
  out->n_keys = (int32_t)rl.q.size();
  return true;
}

int ke_decode_node_metric(const char* js, int64_t len, ke_node_metric* nm, int32_t pm_cap, ke_pod_metric* pm,
                          int32_t* n_pm, int32_t agg_cap, ke_aggregated_usage* agg, int32_t* n_agg) {
  if (!nm || !n_pm || !n_agg || pm_cap < 0 || agg_cap < 0 || (pm_cap && !pm) || (agg_cap && !agg))
    return bad("ke_decode_node_metric arguments");
  Value doc;
  int rc = parse_doc(js, len, doc, "NodeMetric");
  if (rc) return rc;
  ke_node_metric h{};
  h.report_interval_seconds = KE_ABSENT;
  const Value* spec = doc.field("spec");
  const Value* cp = spec ? spec->field("metricCollectPolicy") : nullptr;
  const Value* ri = cp ? cp->field("reportIntervalSeconds") : nullptr;
  if (ri && !ri->is_null() && !json::as_int64(*ri, &h.report_interval_seconds)) return bad("reportIntervalSeconds");
  const Value* st = doc.field("status");
  const Value* ut = st ? st->field("updateTime") : nullptr;
  if (ut && !ut->is_null()) {
    if (ut->t != Value::STR || !parse_rfc3339(ut->s, &h.update_time_ns)) return bad("status.updateTime");
    h.has_update_time = 1;
  }
  const Value* info = st ? st->field("nodeMetric") : nullptr;
  *n_pm = *n_agg = 0;
  if (info && !info->is_null()) {
    h.has_node_metric = 1;
    if (!resource_map(info->field("nodeUsage"), &h.node_usage)) return bad("nodeMetric.nodeUsage");
    const Value* aggs = info->field("aggregatedNodeUsages");
    if (aggs && !aggs->is_null()) {
      if (aggs->t != Value::ARR) return bad("aggregatedNodeUsages");
      if ((int64_t)aggs->a.size() > agg_cap) return bad("aggregatedNodeUsages: more entries than agg_cap");
      for (const Value& a : aggs->a) {
        ke_aggregated_usage u{};
        const Value* d = a.field("duration");
        if (d && !d->is_null() && (d->t != Value::STR || !parse_duration(d->s, &u.duration_ns))) return bad("duration");
        const Value* usage = a.field("usage");
        if (usage && !usage->is_null()) {
          if (!usage->is_obj()) return bad("aggregated usage");
          for (const auto& kv : usage->o) {
            int32_t t;
            if ((rc = agg_type(kv.first, &t))) return rc;
            if (!resource_map(&kv.second, &u.usage[t])) return bad("aggregated usage resources");
          }
        }
        agg[(*n_agg)++] = u;
      }
    }
  }
  const Value* pods = st ? st->field("podsMetric") : nullptr;
  if (pods && !pods->is_null()) {
    if (pods->t != Value::ARR) return bad("podsMetric");
    if ((int64_t)pods->a.size() > pm_cap) return bad("podsMetric: more entries than pm_cap");
    for (const Value& p : pods->a) {
      if (p.is_null()) continue;  // []*PodMetricInfo: a nil entry
      ke_pod_metric m{};
      m.pod_key = ke_pod_key(str_or_empty(p.field("namespace")), str_or_empty(p.field("name")));
      const std::string pr = str_or_empty(p.field("priority"));
      m.priority_class = pr == "koord-prod"    ? KE_PRIORITY_PROD
                         : pr == "koord-mid"   ? KE_PRIORITY_MID
                         : pr == "koord-batch" ? KE_PRIORITY_BATCH
                         : pr == "koord-free"  ? KE_PRIORITY_FREE
                                               : KE_PRIORITY_NONE;
      if (!resource_map(p.field("podUsage"), &m.usage)) return bad("podUsage");
      pm[(*n_pm)++] = m;
    }
  }
  *nm = h;
  return KE_OK;
}

}  // extern "C"

// ---- Pod ---------------------------------------------------------------------------------------------------
namespace {
const char* const KE_RES_NAMES[KE_RES_COUNT] = {"cpu", "memory", "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory",
                                                "kubernetes.io/mid-cpu", "kubernetes.io/mid-memory"};
const char* const PDR_NAMES[KE_PDR_COUNT] = {"nvidia.com/gpu", "amd.com/gpu", "koordinator.sh/gpu",
                                             "koordinator.sh/gpu.shared", "koordinator.sh/gpu-core",
                                             "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio",
                                             "koordinator.sh/rdma", "koordinator.sh/fpga", "dcu.com/gpu"};
const char* const UNSUPPORTED_DEVICE[] = {"huawei.com/npu-core", "huawei.com/npu-cpu", "huawei.com/npu-dvpp"};

struct Container {
  RL req, lim;
};

int containers(const Value* arr, std::vector<Container>& out, const char* what) {
  out.clear();
  if (!arr || arr->is_null()) return KE_OK;
  if (arr->t != Value::ARR) return bad(std::string(what) + " is not an array");
  for (const Value& c : arr->a) {
    Container k;
    const Value* res = c.field("resources");
    if (!resource_list(res ? res->field("requests") : nullptr, k.req) ||
        !resource_list(res ? res->field("limits") : nullptr, k.lim))
      return k.req.overflow || k.lim.overflow ? unsup(std::string(what) + " quantity out of range")
                                              : bad(std::string(what) + " resources");
    const Value* rp = c.field("restartPolicy");
    if (rp && rp->t == Value::STR && rp->s == "Always")
      return unsup("restartable init containers (sidecars) in PodRequests are not modelled");
    out.push_back(std::move(k));
  }
  return KE_OK;
}

// resourceapi.PodRequests / PodLimits (k8s v1.28): Σ containers, max with each init container, + overhead
// (PodLimits adds the overhead only to the resources that already have a limit)
std::map<std::string, __int128> pod_total(const std::vector<Container>& cs, const std::vector<Container>& ics,
                                          const RL& overhead, bool limits) {
  std::map<std::string, __int128> t;
  for (const Container& c : cs)
    for (const auto& kv : (limits ? c.lim : c.req).q) t[kv.first] += kv.second;
  for (const Container& c : ics)
    for (const auto& kv : (limits ? c.lim : c.req).q) t[kv.first] = std::max(t[kv.first], kv.second);
  for (const auto& kv : overhead.q)
    if (!limits || t.count(kv.first)) t[kv.first] += kv.second;
  return t;
}

bool total_value(const std::map<std::string, __int128>& t, const std::string& name, int64_t* out) {
  auto it = t.find(name);
  if (it == t.end()) return false;
  int64_t v, m;
  if (!nanos_value(it->second, &v, &m)) return false;
  *out = name == "cpu" ? m : v;
  return true;
}

// schedutil.IsScalarResourceName (k8s v1.28 pkg/apis/core/v1/helper): an extended resource (a qualified name
// with a domain outside kubernetes.io, not "requests."-prefixed), a hugepages-* resource, a kubernetes.io/
// prefixed native resource or an attachable-volumes-* resource
bool scalar_resource_name(const std::string& n) {
  if (n.rfind("hugepages-", 0) == 0 || n.rfind("attachable-volumes-", 0) == 0) return true;
  if (n.find("kubernetes.io/") != std::string::npos) return true;
  const size_t slash = n.find('/');
  return slash != std::string::npos && slash > 0 && slash + 1 < n.size() && n.rfind("requests.", 0) != 0;
}

// k8s GetPodQOS (pkg/apis/core/v1/helper/qos, v1.28) over cpu / memory of containers + init containers
int kube_qos(const std::vector<Container>& cs, const std::vector<Container>& ics) {  // 0 Guaranteed 1 Burstable 2 BE
  std::map<std::string, __int128> req, lim;
  bool guaranteed = true;
  auto scan = [&](const Container& c) {
    for (const auto& kv : c.req.q)
      if ((kv.first == "cpu" || kv.first == "memory") && kv.second != 0) req[kv.first] += kv.second;
    int found = 0;
    for (const auto& kv : c.lim.q)
      if ((kv.first == "cpu" || kv.first == "memory") && kv.second != 0) lim[kv.first] += kv.second, found++;
    if (found < 2) guaranteed = false;
  };
  for (const Container& c : cs) scan(c);
  for (const Container& c : ics) scan(c);
  if (req.empty() && lim.empty()) return 2;
  if (guaranteed)
    for (const auto& kv : req)
      if (!lim.count(kv.first) || lim[kv.first] != kv.second) guaranteed = false;
  return guaranteed && req.size() == lim.size() ? 0 : 1;
}

int cpu_bind(const Value* v, int32_t* out) {
  const std::string s = str_or_empty(v);
  if (s == "") *out = KE_CPU_BIND_UNSET;
  else if (s == "Default") *out = KE_CPU_BIND_DEFAULT;
  else if (s == "FullPCPUs") *out = KE_CPU_BIND_FULL_PCPUS;
  else if (s == "SpreadByPCPUs") *out = KE_CPU_BIND_SPREAD_BY_PCPUS;
  else if (s == "ConstrainedBurst") *out = KE_CPU_BIND_CONSTRAINED_BURST;
  else return unsup("CPU bind policy \"" + s + "\"");
  return KE_OK;
}

// time of the first condition of `type` with status True (podutil.GetPodCondition); false if none / zero time
bool condition_time(const Value* conds, const char* type, int64_t* ns, int* rc) {
  *rc = KE_OK;
  if (!conds || conds->t != Value::ARR) return false;
  for (const Value& c : conds->a) {
    if (std::string(str_or_empty(c.field("type"))) != type) continue;
    if (std::string(str_or_empty(c.field("status"))) != "True") return false;
    const Value* t = c.field("lastTransitionTime");
    if (!t || t->is_null()) return false;
    if (t->t != Value::STR || !parse_rfc3339(t->s, ns)) {
      *rc = bad(std::string(type) + " lastTransitionTime");
      return false;
    }
    return true;
  }
  return false;
}
}  // namespace

extern "C" {

int ke_decode_pod(const char* js, int64_t len, int32_t n_names, const char* const* xres_names, ke_pod* out) {
  if (!out || n_names < 0 || n_names > KE_MAX_XRES || (n_names && !xres_names)) return bad("ke_decode_pod arguments");
  Value doc;
  int rc = parse_doc(js, len, doc, "Pod");
  if (rc) return rc;
  ke_pod p{};
  const Value* meta = doc.field("metadata");
  const Value* spec = doc.field("spec");
  const Value* status = doc.field("status");
  std::map<std::string, std::string> ann, lab;
  if ((rc = string_map(meta ? meta->field("annotations") : nullptr, ann, "metadata.annotations"))) return rc;
  if ((rc = string_map(meta ? meta->field("labels") : nullptr, lab, "metadata.labels"))) return rc;
  const std::string ns = str_or_empty(meta ? meta->field("namespace") : nullptr),
                    name = str_or_empty(meta ? meta->field("name") : nullptr),
                    uid = str_or_empty(meta ? meta->field("uid") : nullptr);
  p.pod_key = ke_pod_key(ns.c_str(), name.c_str());
  p.uid = uid.empty() ? p.pod_key : (int64_t)(fnv1a(uid) & (uint64_t)INT64_MAX);
  // requests / limits
  std::vector<Container> cs, ics;
  if ((rc = containers(spec ? spec->field("containers") : nullptr, cs, "spec.containers"))) return rc;
  if ((rc = containers(spec ? spec->field("initContainers") : nullptr, ics, "spec.initContainers"))) return rc;
  RL overhead;
  if (!resource_list(spec ? spec->field("overhead") : nullptr, overhead)) return bad("spec.overhead");
  const auto reqs = pod_total(cs, ics, overhead, false), lims = pod_total(cs, ics, overhead, true);
  for (int r = 0; r < KE_RES_COUNT; r++) {
    if (reqs.count(KE_RES_NAMES[r]) && !total_value(reqs, KE_RES_NAMES[r], &p.requests[r]))
      return unsup("pod request out of range");
    if (lims.count(KE_RES_NAMES[r]) && !total_value(lims, KE_RES_NAMES[r], &p.limits[r]))
      return unsup("pod limit out of range");
  }
  for (const auto& kv : reqs) {
    if (kv.second == 0) continue;
    bool known = false, named = false;
    for (const char* n : KE_RES_NAMES) known |= kv.first == n;
    for (int32_t id = 0; id < n_names && !named; id++) named = xres_names[id] && kv.first == xres_names[id];
    // 1: every other name has a resource id (its request is in ke_pod.xres); 2: some name has none
    if (!known) p.has_other_requests = std::max<uint8_t>(p.has_other_requests, named ? 1 : 2);
    for (int d = 0; d < KE_PDR_COUNT; d++)
      if (kv.first == PDR_NAMES[d] && !total_value(reqs, kv.first, &p.device_requests[d]))
        return unsup("device request out of range");
    for (const char* u : UNSUPPORTED_DEVICE)
      if (kv.first == u) p.has_unsupported_device_requests = 1;
  }
  // NodeResourcesFitPlus / ScarceResourceAvoidance: requested names (> 0) and calculatePodResourceRequest
  p.xres_request_mask = 0;
  for (int32_t id = 0; id < n_names; id++) {
    const std::string nm = xres_names[id] ? xres_names[id] : "";
    auto it = reqs.find(nm);
    if (it == reqs.end() || it->second <= 0) continue;
    p.xres_request_mask |= 1ull << id;
    if (p.n_xres >= KE_MAX_POD_XRES) return unsup("more than 8 requested resource names");
    // calculatePodResourceRequest adds Spec.Overhead[name].Value() behind the PodOverhead feature gate
    // (node_resource_fit_plus_utils.go:157-162), which k8s v1.28 no longer registers: not modelled
    if (overhead.q.count(nm)) return unsup("spec.overhead on a NodeResourcesFitPlus / ScarceResourceAvoidance resource");
    // GetNonzeroRequestForResource per container, each rounded as Quantity.MilliValue() (cpu) / Value() before
    // the sum (node_resource_fit_plus_utils.go:140-203): 100m cpu / 200Mi memory for a container without the
    // key, 0 for a name that is not a scalar resource (schedutil.IsScalarResourceName)
    const bool scalar = nm == "cpu" || nm == "memory" || nm == "ephemeral-storage" || scalar_resource_name(nm);
    bool range_ok = true;
    auto nz = [&](const Container& c) -> int64_t {
      auto f = c.req.q.find(nm);
      if (f == c.req.q.end()) return nm == "cpu" ? 100 : nm == "memory" ? 200LL * 1048576 : 0;
      int64_t v, m;
      if (!nanos_value(f->second, &v, &m)) range_ok = false;
      return nm == "cpu" ? m : v;
    };
    int64_t s = 0;
    if (scalar) {
      for (const Container& c : cs)
        if (__builtin_add_overflow(s, nz(c), &s)) range_ok = false;
      for (const Container& c : ics) s = std::max(s, nz(c));
    }
    if (!range_ok) return unsup("pod request out of range");
    p.xres_id[p.n_xres] = id;
    p.xres_value[p.n_xres++] = s;
  }
  // classes (GetPodPriorityClassWithDefault, GetPodQoSClassRaw)
  static const char* QOS[] = {"", "LSE", "LSR", "LS", "BE", "SYSTEM"};
  if (const std::string* q = lookup(lab, "koordinator.sh/qosClass"))
    for (int i = 1; i < 6; i++)
      if (*q == QOS[i]) p.qos_class = i;
  int pc = KE_PRIORITY_NONE;
  if (const std::string* s = lookup(lab, "koordinator.sh/priority-class")) {
    pc = *s == "koord-prod" ? KE_PRIORITY_PROD : *s == "koord-mid" ? KE_PRIORITY_MID : *s == "koord-batch" ? KE_PRIORITY_BATCH
         : *s == "koord-free" ? KE_PRIORITY_FREE : KE_PRIORITY_NONE;
  } else if (const Value* pr = spec ? spec->field("priority") : nullptr; pr && !pr->is_null()) {
    int64_t v;
    if (!json::as_int64(*pr, &v)) return bad("spec.priority");
    pc = (v >= 9000 && v <= 9999) ? KE_PRIORITY_PROD : (v >= 7000 && v <= 7999) ? KE_PRIORITY_MID
         : (v >= 5000 && v <= 5999) ? KE_PRIORITY_BATCH : (v >= 3000 && v <= 3999) ? KE_PRIORITY_FREE : KE_PRIORITY_NONE;
  }
  if (pc == KE_PRIORITY_NONE) {  // GetPodQoSClassWithKubeQoS -> priority by QoS
    int q = p.qos_class;
    static const int BY_KUBE_QOS[3] = {KE_QOS_LSR, KE_QOS_LS, KE_QOS_BE};  // Guaranteed / Burstable / BestEffort
    if (q == KE_QOS_NONE) {  // GetKubeQosClass: Status.QOSClass when set, else computed (qos_utils.go:72-78)
      const std::string sq = str_or_empty(status ? status->field("qosClass") : nullptr);
      int kq = -1;
      if (sq == "Guaranteed") kq = 0;
      else if (sq == "Burstable") kq = 1;
      else if (sq == "BestEffort") kq = 2;
      else if (!sq.empty()) return unsup("status.qosClass \"" + sq + "\"");
      q = BY_KUBE_QOS[kq >= 0 ? kq : kube_qos(cs, ics)];
    }
    pc = (q == KE_QOS_SYSTEM || q == KE_QOS_LSE || q == KE_QOS_LSR || q == KE_QOS_LS) ? KE_PRIORITY_PROD
         : q == KE_QOS_BE ? KE_PRIORITY_BATCH : KE_PRIORITY_NONE;
  }
  p.priority_class = pc;
  // owner, phase, conditions
  const Value* owners = meta ? meta->field("ownerReferences") : nullptr;
  if (owners && owners->t == Value::ARR)
    for (const Value& o : owners->a)
      if (std::string(str_or_empty(o.field("kind"))) == "DaemonSet") p.is_daemonset = 1;
  const std::string phase = str_or_empty(status ? status->field("phase") : nullptr);
  p.is_terminated = phase == "Succeeded" || phase == "Failed";
  const Value* conds = status ? status->field("conditions") : nullptr;
  p.has_scheduled = condition_time(conds, "PodScheduled", &p.scheduled_transition_ns, &rc);
  if (rc) return rc;
  p.has_initialized = condition_time(conds, "Initialized", &p.initialized_transition_ns, &rc);
  if (rc) return rc;
  // LoadAware estimation annotations (load_aware.go:75-100)
  p.custom_scaling_factors[0] = p.custom_scaling_factors[1] = KE_ABSENT;
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/load-estimated-scaling-factors"); s && !s->empty()) {
    Value v;
    std::string err;
    int64_t f[KE_NRES];
    bool other;
    size_t nk = 0;
    if (json::parse(s->data(), s->size(), v, err) && int_map(&v, f, &other, &nk) && nk > 0) {
      p.has_custom_scaling_factors = 1;
      p.custom_scaling_factors[0] = f[0];
      p.custom_scaling_factors[1] = f[1];
    }
  }
  p.custom_seconds_after_scheduled = p.custom_seconds_after_initialized = KE_ABSENT;
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/load-estimated-seconds-after-pod-scheduled"))
    if (!parse_int64(*s, &p.custom_seconds_after_scheduled)) p.custom_seconds_after_scheduled = KE_ABSENT;
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/load-estimated-seconds-after-initialized"))
    if (!parse_int64(*s, &p.custom_seconds_after_initialized)) p.custom_seconds_after_initialized = KE_ABSENT;
  // ResourceSpec (an unmarshal error is PreFilter's error: has_resource_spec)
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/resource-spec")) {
    Value v;
    std::string err;
    const bool ok = json::parse(s->data(), s->size(), v, err) && (v.is_null() || v.is_obj());
    const Value *rq = ok ? v.field("requiredCPUBindPolicy") : nullptr, *pf = ok ? v.field("preferredCPUBindPolicy") : nullptr,
                *ex = ok ? v.field("preferredCPUExclusivePolicy") : nullptr;
    auto strish = [](const Value* x) { return !x || x->is_null() || x->t == Value::STR; };
    if (!ok || !strish(rq) || !strish(pf) || !strish(ex)) {
      p.has_resource_spec = 1;
    } else {
      if ((rc = cpu_bind(rq, &p.cpu_bind_required)) || (rc = cpu_bind(pf, &p.cpu_bind_preferred))) return rc;
      const std::string e = str_or_empty(ex);
      if (e == "" || e == "None") p.cpu_exclusive = KE_CPU_EXCL_NONE;
      else if (e == "PCPULevel") p.cpu_exclusive = KE_CPU_EXCL_PCPU_LEVEL;
      else if (e == "NUMANodeLevel") p.cpu_exclusive = KE_CPU_EXCL_NUMA_NODE_LEVEL;
      else return unsup("CPU exclusive policy \"" + e + "\"");
    }
  }
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/numa-topology-spec")) {
    Value v;
    std::string err;
    if (!json::parse(s->data(), s->size(), v, err) || !(v.is_null() || v.is_obj()))
      return unsup("numa-topology-spec annotation that fails to unmarshal");
    const std::string pol = str_or_empty(v.field("numaTopologyPolicy")), ex = str_or_empty(v.field("singleNUMANodeExclusive"));
    if (pol == "") p.numa_topology_policy = KE_NUMA_POLICY_NONE;
    else if (pol == "BestEffort") p.numa_topology_policy = KE_NUMA_POLICY_BEST_EFFORT;
    else if (pol == "Restricted") p.numa_topology_policy = KE_NUMA_POLICY_RESTRICTED;
    else if (pol == "SingleNUMANode") p.numa_topology_policy = KE_NUMA_POLICY_SINGLE_NUMA_NODE;
    else return unsup("NUMA topology policy \"" + pol + "\"");
    if (ex == "") p.numa_exclusive = KE_NUMA_EXCLUSIVE_NONE;
    else if (ex == "Preferred") p.numa_exclusive = KE_NUMA_EXCLUSIVE_PREFERRED;
    else if (ex == "Required") p.numa_exclusive = KE_NUMA_EXCLUSIVE_REQUIRED;
    else return unsup("SingleNUMANodeExclusive \"" + ex + "\"");
  }
  // ElasticQuota: the quota name -> index mapping is the caller's (ke_quotas_load order); preemptible label
  const std::string* pre = lookup(lab, "quota.scheduling.koordinator.sh/preemptible");
  p.quota_non_preemptible = pre && *pre == "false";
  // DeviceShare annotations (utils.go:355-513)
  p.gpu_ring_bus_bandwidth = KE_ABSENT;
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/gpu-partition-spec")) {
    Value v;
    std::string err;
    if (!json::parse(s->data(), s->size(), v, err) || !(v.is_null() || v.is_obj()))
      return unsup("gpu-partition-spec annotation that fails to unmarshal");
    p.gpu_partition_spec = 1;
    p.gpu_partition_restricted = std::string(str_or_empty(v.field("allocatePolicy"))) == "Restricted";
    const Value* bw = v.field("ringBusBandwidth");
    if (bw && !bw->is_null()) {
      int64_t val, milli;
      bool ov;
      if (!quantity_json(*bw, &val, &milli, &ov)) return unsup("ringBusBandwidth");
      p.gpu_ring_bus_bandwidth = val;
    }
  }
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/device-allocate-hint")) {
    Value v;
    std::string err;
    if (!json::parse(s->data(), s->size(), v, err) || !(v.is_null() || v.is_obj()))
      return unsup("device-allocate-hint annotation that fails to unmarshal");
    uint8_t bits = 0;
    if (v.is_obj())
      for (const auto& kv : v.o) {
        const Value& h = kv.second;
        if (!h.is_obj()) continue;
        auto set = [&](const char* f) { const Value* x = h.field(f); return x && !x->is_null(); };
        // the hints themselves come from ke_decode_pod_device_hints; a gpu VFSelector is not modelled
        if (kv.first == "gpu" && set("vfSelector")) bits |= KE_DHINT_GPU_VF;
        const std::string sc = str_or_empty(h.field("requiredTopologyScope"));
        if (kv.first == "gpu" && !sc.empty())
          p.gpu_required_topology_scope = sc == "Node" ? KE_SCOPE_NODE : sc == "NUMANode" ? KE_SCOPE_NUMA
                                          : sc == "PCIe" ? KE_SCOPE_PCIE : sc == "Device" ? KE_SCOPE_DEVICE : KE_SCOPE_UNKNOWN;
      }
    p.device_hints = bits;
  }
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/device-joint-allocate")) {
    Value v, hints;
    std::string err;
    if (!json::parse(s->data(), s->size(), v, err) || !(v.is_null() || v.is_obj()))
      return unsup("device-joint-allocate annotation that fails to unmarshal");
    const std::string* hs = lookup(ann, "scheduling.koordinator.sh/device-allocate-hint");
    if (hs) json::parse(hs->data(), hs->size(), hints, err);
    bool gpu = false;
    for (int d = 0; d < KE_PDR_COUNT; d++) gpu |= d != KE_PDR_RDMA && d != KE_PDR_FPGA && p.device_requests[d] > 0;
    const Value* types = v.field("deviceTypes");
    if (types && types->t == Value::ARR)
      for (const Value& t : types->a) {
        const std::string ty = t.t == Value::STR ? t.s : "";
        const bool req = (ty == "gpu" && gpu) || (ty == "rdma" && p.device_requests[KE_PDR_RDMA] > 0) ||
                         (ty == "fpga" && p.device_requests[KE_PDR_FPGA] > 0);
        const Value* h = hints.is_obj() ? hints.key(ty.c_str()) : nullptr;
        const bool apply_all = h && std::string(str_or_empty(h->field("allocateStrategy"))) == "ApplyForAll";
        if (req && !apply_all) p.device_joint_allocate = 1;
      }
  }
  *out = p;
  return KE_OK;
}

// a string map of labels into (key, value) ids (Go map order is irrelevant: matching is by key)
static bool labels_of(const Value* v, ke_labels& out) {
  out = ke_labels{};
  if (!v || v->is_null()) return true;
  if (!v->is_obj()) return false;
  for (const auto& kv : v->o) {
    if (kv.second.t != Value::STR || out.n >= KE_MAX_LABELS) return false;
    out.key[out.n] = ke_label_id(kv.first.c_str());
    out.value[out.n] = ke_label_id(kv.second.s.c_str());
    out.n++;
  }
  return true;
}

// metav1.LabelSelector -> labels.Selector (util.GetFastLabelSelector, pkg/util/selector.go:24-32; apimachinery
// LabelSelectorAsSelector): matchLabels entries become In requirements with one value, matchExpressions keep
// their operator (In / NotIn need values, Exists / DoesNotExist take none; anything else is an error)
static bool selector_of(const Value* v, ke_label_selector& out, bool* invalid) {
  out = ke_label_selector{};
  if (!v || v->is_null()) return true;
  if (!v->is_obj()) return false;
  out.present = 1;
  const Value* ml = v->field("matchLabels");
  if (ml && ml->is_obj())
    for (const auto& kv : ml->o) {
      if (kv.second.t != Value::STR || out.n >= KE_MAX_SEL_REQS) return false;
      ke_label_requirement& r = out.req[out.n++];
      r.key = ke_label_id(kv.first.c_str());
      r.op = KE_SEL_IN;
      r.n_values = 1;
      r.values[0] = ke_label_id(kv.second.s.c_str());
    }
  const Value* me = v->field("matchExpressions");
  if (me && me->t == Value::ARR)
    for (const Value& e : me->a) {
      if (out.n >= KE_MAX_SEL_REQS) return false;
      ke_label_requirement& r = out.req[out.n++];
      r.key = ke_label_id(str_or_empty(e.field("key")));
      const std::string op = str_or_empty(e.field("operator"));
      const Value* vals = e.field("values");
      const size_t nv = vals && vals->t == Value::ARR ? vals->a.size() : 0;
      if (nv > KE_MAX_SEL_VALUES) return false;
      for (size_t q = 0; q < nv; q++) {
        if (vals->a[q].t != Value::STR) return false;
        r.values[q] = ke_label_id(vals->a[q].s.c_str());
      }
      r.n_values = (int32_t)nv;
      if (op == "In" || op == "NotIn") {
        r.op = op == "In" ? KE_SEL_IN : KE_SEL_NOT_IN;
        if (nv == 0) *invalid = true;
      } else if (op == "Exists" || op == "DoesNotExist") {
        r.op = op == "Exists" ? KE_SEL_EXISTS : KE_SEL_DOES_NOT_EXIST;
        if (nv != 0) *invalid = true;
      } else {
        *invalid = true;
      }
    }
  return true;
}

// ---- Device ------------------------------------------------------------------------------------------------
int ke_decode_device(const char* js, int64_t len, int32_t cap, ke_device* out, int32_t* n, int32_t part_cap,
                     ke_gpu_partition* parts, int32_t* n_parts, int32_t* has_table, int32_t* honor) {
  if (!n || cap < 0 || (cap && !out) || part_cap < 0 || (part_cap && !parts) || !n_parts || !has_table || !honor)
    return bad("ke_decode_device arguments");
  Value doc;
  int rc = parse_doc(js, len, doc, "Device");
  if (rc) return rc;
  const Value* meta = doc.field("metadata");
  const Value* spec = doc.field("spec");
  std::map<std::string, std::string> ann, lab;
  if ((rc = string_map(meta ? meta->field("annotations") : nullptr, ann, "metadata.annotations"))) return rc;
  if ((rc = string_map(meta ? meta->field("labels") : nullptr, lab, "metadata.labels"))) return rc;
  const Value* devs = spec ? spec->field("devices") : nullptr;
  std::vector<ke_device> out_v;
  std::vector<std::string> pcie;  // per output device: its PCIe id ("" without a topology)
  if (devs && !devs->is_null()) {
    if (devs->t != Value::ARR) return bad("spec.devices");
    for (const Value& d : devs->a) {
      const std::string type = str_or_empty(d.field("type"));
      ke_device k{};
      if (type == "gpu") k.type = KE_DEV_GPU;
      else if (type == "rdma") k.type = KE_DEV_RDMA;
      else if (type == "fpga") k.type = KE_DEV_FPGA;
      else return unsup("device type \"" + type + "\" (not gpu / rdma / fpga)");
      const Value* mi = d.field("minor");
      int64_t minor;
      if (!mi || mi->is_null() || !json::as_int64(*mi, &minor)) return bad("device without a minor");
      if (minor < 0 || minor >= KE_MAX_MINORS) return unsup("device minor outside 0..15");
      k.minor = (int32_t)minor;
      const Value* h = d.field("health");
      k.health = h && h->t == Value::BOOL && h->b;
      RL res;
      if (!resource_list(d.field("resources"), res)) return bad("device resources");
      if (k.health) {  // buildDeviceResources: an unhealthy device has an empty ResourceList
        static const char* GPU_KEYS[KE_DKEYS] = {"koordinator.sh/gpu-core", "koordinator.sh/gpu-memory",
                                                 "koordinator.sh/gpu-memory-ratio"};
        const char* key0 = k.type == KE_DEV_GPU ? nullptr : (k.type == KE_DEV_RDMA ? "koordinator.sh/rdma" : "koordinator.sh/fpga");
        for (const auto& kv : res.q) {
          int slot = -1;
          if (k.type == KE_DEV_GPU) {
            for (int s = 0; s < KE_DKEYS; s++)
              if (kv.first == GPU_KEYS[s]) slot = s;
          } else if (kv.first == key0) {
            slot = 0;
          }
          if (slot < 0) return unsup("device resource \"" + kv.first + "\" outside the device type's keys");
          int64_t v, m;
          if (!nanos_value(kv.second, &v, &m)) return unsup("device resource out of range");
          k.has_total[slot] = 1;
          k.total[slot] = v;
        }
      }
      // DeviceInfo.Labels and VFGroups (VF ranks: the device's VFs in BusID string order over all its groups)
      if (!labels_of(d.field("labels"), k.labels)) return unsup("device labels (more than 8, or not strings)");
      const Value* vg = d.field("vfGroups");
      if (vg && !vg->is_null()) {
        if (vg->t != Value::ARR) return bad("vfGroups");
        if (vg->a.size() > KE_MAX_VF_GROUPS) return unsup("more than 4 VF groups on a device");
        std::vector<std::pair<std::string, int>> vfs;  // (BusID, group)
        for (size_t g = 0; g < vg->a.size(); g++) {
          const Value& grp = vg->a[g];
          if (!labels_of(grp.field("labels"), k.vf_groups[g].labels)) return unsup("VF group labels");
          const Value* list = grp.field("vfs");
          if (list && list->t == Value::ARR)
            for (const Value& vf : list->a) vfs.emplace_back(str_or_empty(vf.field("busID")), (int)g);
        }
        if (vfs.size() > 64) return unsup("more than 64 VFs on a device");
        std::stable_sort(vfs.begin(), vfs.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
        for (size_t r = 0; r < vfs.size(); r++) k.vf_groups[vfs[r].second].vfs |= 1ull << r;
        k.n_vf_groups = (int32_t)vg->a.size();
        if (k.type == KE_DEV_GPU) k.n_vf_groups = 0;  // GPU VFs are not modelled (a GPU VFSelector is refused)
      }
      const Value* topo = d.field("topology");
      std::string pid;
      if (topo && !topo->is_null()) {
        int64_t node = 0;
        const Value* nid = topo->field("nodeID");
        if (nid && !nid->is_null() && !json::as_int64(*nid, &node)) return bad("topology.nodeID");
        k.has_topology = 1;
        k.numa_node = (int32_t)node;
        pid = str_or_empty(topo->field("pcieID"));
      }
      out_v.push_back(k);
      pcie.push_back(pid);
    }
  }
  // PCIe id rank among the node's distinct ids in Go string order (bytewise)
  std::vector<std::string> ids;
  for (size_t i = 0; i < out_v.size(); i++)
    if (out_v[i].has_topology) ids.push_back(pcie[i]);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  for (size_t i = 0; i < out_v.size(); i++)
    if (out_v[i].has_topology)
      out_v[i].pcie_rank = (int32_t)(std::lower_bound(ids.begin(), ids.end(), pcie[i]) - ids.begin());
  if ((int64_t)out_v.size() > cap) return bad("more devices than cap");
  std::copy(out_v.begin(), out_v.end(), out);
  *n = (int32_t)out_v.size();
  // GPU partition table (GetGPUPartitionTable) and policy label (GetGPUPartitionPolicy)
  *n_parts = 0;
  *has_table = 0;
  const std::string* pol = lookup(lab, "node.koordinator.sh/gpu-partition-policy");
  *honor = pol && *pol == "Honor";
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/gpu-partitions"); s && !s->empty()) {
    Value v;
    std::string err;
    if (!json::parse(s->data(), s->size(), v, err) || !(v.is_null() || v.is_obj()))
      return unsup("gpu-partitions annotation that fails to unmarshal (the cache keeps a nil indexer)");
    if (v.is_obj()) {
      *has_table = 1;
      std::vector<std::pair<int64_t, const Value*>> keys;  // map[int][]GPUPartition: ascending by key
      for (const auto& kv : v.o) {
        int64_t k;
        if (!parse_int64(kv.first, &k)) return unsup("gpu-partitions key");
        keys.emplace_back(k, &kv.second);
      }
      std::stable_sort(keys.begin(), keys.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
      for (const auto& kv : keys) {
        if (kv.second->t != Value::ARR) return unsup("gpu-partitions entry");
        for (const Value& g : kv.second->a) {
          ke_gpu_partition q{};
          q.number_of_gpus = (int32_t)kv.first;
          q.ring_bus_bandwidth = KE_ABSENT;
          const Value* mn = g.field("minors");
          if (!mn || mn->t != Value::ARR) return unsup("gpu partition without minors");
          for (const Value& m : mn->a) {
            int64_t x;
            if (!json::as_int64(m, &x) || x < 0 || x >= KE_MAX_MINORS) return unsup("gpu partition minor");
            q.minors |= 1u << x;
          }
          int64_t sc = 0;
          const Value* as = g.field("allocationScore");
          if (as && !as->is_null() && !json::as_int64(*as, &sc)) return unsup("allocationScore");
          q.allocation_score = (int32_t)sc;
          const Value* bw = g.field("ringBusBandwidth");
          if (bw && !bw->is_null()) {
            int64_t val, milli;
            bool ov;
            if (!quantity_json(*bw, &val, &milli, &ov)) return unsup("ringBusBandwidth");
            q.ring_bus_bandwidth = val;
          }
          if (*n_parts >= part_cap) return bad("more partitions than part_cap");
          parts[(*n_parts)++] = q;
        }
      }
    }
  }
  return KE_OK;
}

}  // extern "C"

// ---- DeviceShare pod hints (parsePodDeviceShareExtensions, deviceshare/utils.go:414-482) ---------------------
int ke_decode_pod_device_hints(const char* js, int64_t len, ke_pod_device_hints* out, int32_t* present) {
  if (!out || !present) return bad("ke_decode_pod_device_hints arguments");
  Value doc;
  int rc = parse_doc(js, len, doc, "Pod");
  if (rc) return rc;
  ke_pod_device_hints h{};
  *present = 0;
  const Value* meta = doc.field("metadata");
  std::map<std::string, std::string> ann;
  if ((rc = string_map(meta ? meta->field("annotations") : nullptr, ann, "metadata.annotations"))) return rc;
  auto type_of = [](const std::string& t) { return t == "gpu" ? KE_DEV_GPU : t == "rdma" ? KE_DEV_RDMA : t == "fpga" ? KE_DEV_FPGA : -1; };
  Value hints;
  std::string err;
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/device-allocate-hint")) {
    if (!json::parse(s->data(), s->size(), hints, err) || !(hints.is_null() || hints.is_obj()))
      return unsup("device-allocate-hint annotation that fails to unmarshal");
    *present = 1;
    if (hints.is_obj())
      for (const auto& kv : hints.o) {
        const Value& hv = kv.second;
        if (!hv.is_obj()) continue;
        bool invalid = false;
        ke_label_selector sel, vfsel;
        if (!selector_of(hv.field("selector"), sel, &invalid) || !selector_of(hv.field("vfSelector"), vfsel, &invalid))
          return unsup("a device hint selector beyond 4 requirements / 4 values");
        if (invalid) h.invalid = 1;
        if (sel.present) h.has_selectors = 1;  // any device type, modelled or not (utils.go:446-452)
        const int t = type_of(kv.first);
        if (t < 0) continue;
        ke_device_hint& d = h.hint[t];
        d.selector = sel;
        d.vf_selector = vfsel;
        const std::string st = str_or_empty(hv.field("allocateStrategy"));
        d.strategy = st == "ApplyForAll" ? KE_DSTRATEGY_APPLY_FOR_ALL
                     : st == "RequestsAsCount" ? KE_DSTRATEGY_REQUESTS_AS_COUNT : KE_DSTRATEGY_NONE;
        const std::string ex = str_or_empty(hv.field("exclusivePolicy"));
        d.exclusive = ex == "DeviceLevel" ? KE_DEXCL_DEVICE_LEVEL : ex == "PCIeLevel" ? KE_DEXCL_PCIE_LEVEL : KE_DEXCL_NONE;
      }
  }
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/device-joint-allocate")) {
    Value v;
    if (!json::parse(s->data(), s->size(), v, err) || !(v.is_null() || v.is_obj()))
      return unsup("device-joint-allocate annotation that fails to unmarshal");
    *present = 1;
    // the requested, non-ApplyForAll types in annotation order (utils.go:430-442): the caller's ke_pod tells
    // which types are requested; here every listed gpu / rdma / fpga type is kept and ke_schedule's PreFilter
    // drops the unrequested ones (decode the pod with ke_decode_pod for them)
    const Value* types = v.field("deviceTypes");
    if (types && types->t == Value::ARR)
      for (const Value& tv : types->a) {
        const int t = type_of(tv.t == Value::STR ? tv.s : "");
        if (t < 0 || h.hint[t].strategy == KE_DSTRATEGY_APPLY_FOR_ALL) continue;
        bool dup = false;
        for (int j = 0; j < h.joint_n; j++) dup = dup || h.joint_types[j] == t;
        if (!dup && h.joint_n < KE_DEV_TYPES) h.joint_types[h.joint_n++] = t;
      }
    h.joint_same_pcie = std::string(str_or_empty(v.field("requiredScope"))) == "SamePCIe";
  }
  *out = h;
  return KE_OK;
}

int ke_decode_device_flags(const char* device_json, int64_t device_len, const char* node_json, int64_t node_len,
                           int32_t* secondary_well_planned, int32_t* gpu_model_key) {
  if (!secondary_well_planned || !gpu_model_key) return bad("ke_decode_device_flags arguments");
  *secondary_well_planned = 0;
  *gpu_model_key = 0;
  Value doc;
  int rc;
  if (device_json) {
    if ((rc = parse_doc(device_json, device_len, doc, "Device"))) return rc;
    const Value* meta = doc.field("metadata");
    std::map<std::string, std::string> lab;
    if ((rc = string_map(meta ? meta->field("labels") : nullptr, lab, "metadata.labels"))) return rc;
    const std::string* w = lookup(lab, "node.koordinator.sh/secondary-device-well-planned");
    *secondary_well_planned = w && *w == "true";
  }
  if (node_json) {
    if ((rc = parse_doc(node_json, node_len, doc, "Node"))) return rc;
    const Value* meta = doc.field("metadata");
    std::map<std::string, std::string> lab;
    if ((rc = string_map(meta ? meta->field("labels") : nullptr, lab, "metadata.labels"))) return rc;
    const std::string* vendor = lookup(lab, "node.koordinator.sh/gpu-vendor");
    const std::string* model = lookup(lab, "node.koordinator.sh/gpu-model");
    const std::string key = (vendor ? *vendor : std::string()) + "-" + (model ? *model : std::string());  // buildGPUSharedResourceTemplatesKey
    *gpu_model_key = ke_label_id(key.c_str());
  }
  return KE_OK;
}

// ---- NodeResourceTopology (nodenumaresource/topology_options.go:90-236) -----------------------------------
namespace {
// k8s cpuset.Parse ("0-3,8"); false on a malformed list (the reference then logs and uses the empty set)
bool parse_cpuset(const std::string& s, std::vector<int>& out) {
  out.clear();
  if (s.empty()) return true;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string part = s.substr(i, j - i);
    const size_t dash = part.find('-');
    int64_t a, b;
    if (dash == std::string::npos) {
      if (!parse_int64(part, &a) || a < 0) return false;
      b = a;
    } else if (!parse_int64(part.substr(0, dash), &a) || !parse_int64(part.substr(dash + 1), &b) || a < 0 || b < a) {
      return false;
    }
    if (b - a > 4096) return false;
    for (int64_t c = a; c <= b; c++) out.push_back((int)c);
    i = j + 1;
  }
  return true;
}
}  // namespace

extern "C" {

int ke_decode_nrt(const char* js, int64_t len, ke_node* node, int32_t zone_cap, ke_numa_zone* zones, int32_t* n_zones,
                  int32_t cpu_cap, ke_cpu* cpus, int32_t* n_cpus) {
  if (!node || !n_zones || !n_cpus || zone_cap < 0 || cpu_cap < 0 || (zone_cap && !zones) || (cpu_cap && !cpus))
    return bad("ke_decode_nrt arguments");
  Value doc;
  int rc = parse_doc(js, len, doc, "NodeResourceTopology");
  if (rc) return rc;
  const Value* meta = doc.field("metadata");
  std::map<std::string, std::string> ann;
  if ((rc = string_map(meta ? meta->field("annotations") : nullptr, ann, "metadata.annotations"))) return rc;
  auto parse_ann = [&](const char* key, Value& v) {  // the annotation's JSON, false when absent / unparsable
    const std::string* s = lookup(ann, key);
    std::string err;
    return s && json::parse(s->data(), s->size(), v, err);
  };
  // CPU topology (GetCPUTopology + convertCPUTopology: core id = socket << 16 | core)
  struct Cpu {
    int id, core, node, socket;
  };
  std::map<int, Cpu> topo;
  Value v;
  if (lookup(ann, "node.koordinator.sh/cpu-topology")) {
    if (!parse_ann("node.koordinator.sh/cpu-topology", v) || !(v.is_null() || v.is_obj()))
      return unsup("cpu-topology annotation that fails to unmarshal");
    const Value* det = v.is_obj() ? v.field("detail") : nullptr;
    if (det && det->t == Value::ARR)
      for (const Value& c : det->a) {
        int64_t id = 0, core = 0, sock = 0, nd = 0;
        for (auto f : {std::make_pair("id", &id), std::make_pair("core", &core), std::make_pair("socket", &sock),
                       std::make_pair("node", &nd)}) {
          const Value* x = c.field(f.first);
          if (x && !x->is_null() && !json::as_int64(*x, f.second)) return unsup("cpu-topology entry");
        }
        if (id < 0 || id >= KE_MAX_CPUS || core < 0 || core > 0xFFFF || sock < 0 || sock > 0x7FFF || nd < 0 || nd > 0x7FFF)
          return unsup("cpu-topology ids outside the modelled range (CPU ids 0..255)");
        topo[(int)id] = Cpu{(int)id, (int)(sock << 16 | core), (int)nd, (int)sock};
      }
  }
  // reserved CPUs = pod-cpu-allocs (kubelet-managed) + kubelet reserved + node reservation + exclusive system QoS
  std::vector<int> reserved, tmp;
  if (parse_ann("node.koordinator.sh/pod-cpu-allocs", v) && v.t == Value::ARR)
    for (const Value& a : v.a) {
      const Value* mk = a.field("managedByKubelet");
      if (!(mk && mk->t == Value::BOOL && mk->b) || !*str_or_empty(a.field("uid"))) continue;
      if (parse_cpuset(str_or_empty(a.field("cpuset")), tmp)) reserved.insert(reserved.end(), tmp.begin(), tmp.end());
    }
  bool kubelet_full = false;
  if (parse_ann("kubelet.koordinator.sh/cpu-manager-policy", v) && v.is_obj()) {
    if (parse_cpuset(str_or_empty(v.field("reservedCPUs")), tmp)) reserved.insert(reserved.end(), tmp.begin(), tmp.end());
    const Value* opts = v.field("options");
    const Value* full = opts && opts->is_obj() ? opts->key("full-pcpus-only") : nullptr;
    kubelet_full = std::string(str_or_empty(v.field("policy"))) == "static" && full && full->t == Value::STR &&
                   full->s == "true";
  }
  if (const std::string* s = lookup(ann, "node.koordinator.sh/reservation"); s && !s->empty()) {
    std::string err;
    if (json::parse(s->data(), s->size(), v, err) && v.is_obj() &&
        parse_cpuset(str_or_empty(v.field("reservedCPUs")), tmp))
      reserved.insert(reserved.end(), tmp.begin(), tmp.end());
  }
  if (parse_ann("node.koordinator.sh/system-qos-resource", v) && v.is_obj()) {
    const Value* ex = v.field("cpusetExclusive");
    const bool exclusive = !ex || ex->is_null() || (ex->t == Value::BOOL && ex->b);
    if (exclusive && parse_cpuset(str_or_empty(v.field("cpuset")), tmp))
      reserved.insert(reserved.end(), tmp.begin(), tmp.end());
  }
  std::sort(reserved.begin(), reserved.end());
  reserved.erase(std::unique(reserved.begin(), reserved.end()), reserved.end());
  auto is_reserved = [&](int c) { return std::binary_search(reserved.begin(), reserved.end(), c); };
  // zones: type Node, name node-<id>, Allocatable per resource; cpu minus 1000 per reserved CPU of the NUMA node
  std::vector<ke_numa_zone> zs;
  const Value* zarr = doc.field("zones");
  if (zarr && zarr->t == Value::ARR)
    for (const Value& z : zarr->a) {
      if (std::string(str_or_empty(z.field("type"))) != "Node") continue;
      const std::string name = str_or_empty(z.field("name"));
      if (name.compare(0, 5, "node-") != 0 || name.find("node-", 5) != std::string::npos) continue;
      int64_t id;
      if (!parse_int64(name.substr(5), &id)) continue;  // strconv.Atoi error: the zone is skipped
      if (id < 0 || id >= KE_MAX_NUMA) return unsup("NUMA node id outside 0..7");
      ke_numa_zone k{};
      k.id = (int32_t)id;
      const Value* res = z.field("resources");
      if (res && res->t == Value::ARR)
        for (const Value& r : res->a) {
          const std::string rn = str_or_empty(r.field("name"));
          const int slot = rn == "cpu" ? 0 : rn == "memory" ? 1 : -1;
          if (slot < 0) continue;
          const Value* al = r.field("allocatable");
          int64_t val = 0, milli = 0;
          bool ov;
          if (al && !al->is_null() && !quantity_json(*al, &val, &milli, &ov)) return bad("zone allocatable");
          k.has[slot] = 1;
          k.capacity[slot] = slot == 0 ? milli : val;
        }
      if (k.has[0] && k.capacity[0] != 0) {
        int in_node = 0;
        for (const auto& kv : topo) in_node += kv.second.node == id && is_reserved(kv.first);
        k.capacity[0] -= 1000LL * in_node;
      }
      zs.push_back(k);
    }
  std::stable_sort(zs.begin(), zs.end(), [](const ke_numa_zone& a, const ke_numa_zone& b) { return a.id < b.id; });
  for (size_t i = 1; i < zs.size(); i++)
    if (zs[i].id == zs[i - 1].id) return unsup("two zones with one NUMA node id");
  if ((int64_t)zs.size() > zone_cap || (int64_t)topo.size() > cpu_cap) return bad("zone_cap / cpu_cap too small");
  std::copy(zs.begin(), zs.end(), zones);
  *n_zones = (int32_t)zs.size();
  int32_t nc = 0;
  for (const auto& kv : topo) {
    ke_cpu c{};
    c.cpu_id = kv.second.id;
    c.core_id = kv.second.core;
    c.numa_id = kv.second.node;
    c.socket_id = kv.second.socket;
    c.reserved = is_reserved(kv.first);
    cpus[nc++] = c;
  }
  *n_cpus = nc;
  // node-level fields the NRT carries (getNUMATopologyPolicy, GetNodeCPUBindPolicy, TopologyOptions ratios)
  if (node->numa_topology_policy == KE_NUMA_POLICY_NONE) {
    const Value* pols = doc.field("topologyPolicies");
    if (pols && pols->t == Value::ARR)
      for (const Value& p : pols->a) {
        const std::string s = p.t == Value::STR ? p.s : "";
        const int pol = s == "BestEffort" ? KE_NUMA_POLICY_BEST_EFFORT : s == "Restricted" ? KE_NUMA_POLICY_RESTRICTED
                        : s == "SingleNUMANodePodLevel" ? KE_NUMA_POLICY_SINGLE_NUMA_NODE : KE_NUMA_POLICY_NONE;
        if (pol != KE_NUMA_POLICY_NONE) {
          node->numa_topology_policy = pol;
          break;
        }
      }
  }
  if (kubelet_full) node->cpu_bind_policy = KE_NODE_CPU_BIND_FULL_PCPUS_ONLY;
  node->nrt_cpu_amplification_ratio = -2.0;
  if (lookup(ann, "node.koordinator.sh/resource-amplification-ratio")) {
    bool ok = parse_ann("node.koordinator.sh/resource-amplification-ratio", v) && (v.is_null() || v.is_obj());
    double cpu = 0.0;  // a ratio map without cpu: the Go zero value (no amplification)
    if (ok && v.is_obj())
      for (const auto& kv : v.o) {
        double d;
        if (!json::as_float64(kv.second, &d)) ok = false;
        else if (kv.first == "cpu") cpu = d;
      }
    if (ok && v.is_obj()) node->nrt_cpu_amplification_ratio = cpu;
  }
  node->cpu_topology_invalid = topo.empty();  // convertCPUTopology of no detail: !IsValid()
  return KE_OK;
}

}  // extern "C"

// ---- Reservation (apis/scheduling/v1alpha1/reservation_types.go) --------------------------------------------
namespace {
// a ResourceList's value by name as the reservation cache reads it: cpu MilliValue, every other name Value
bool rl_get(const RL& rl, const std::string& name, int64_t* out) {
  *out = 0;
  auto it = rl.q.find(name);
  if (it == rl.q.end()) return true;
  int64_t v, m;
  if (!nanos_value(it->second, &v, &m)) return false;
  *out = name == "cpu" ? m : v;
  return true;
}
const char* const DEV_TYPE_NAMES[KE_DEV_TYPES] = {"gpu", "rdma", "fpga"};
const char* const DEV_KEY_NAMES[KE_DEV_TYPES][KE_DKEYS] = {
    {"koordinator.sh/gpu-core", "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio"},
    {"koordinator.sh/rdma", nullptr, nullptr},
    {"koordinator.sh/fpga", nullptr, nullptr}};
}  // namespace

extern "C" {

int ke_decode_reservation(const char* js, int64_t len, int32_t n_names, const char* const* xres_names, ke_reservation* out,
                          ke_reservation_alloc* alloc, int32_t res_cap, ke_reservation_resource* res, int32_t* n_res,
                          char* node_name, int32_t name_cap) {
  if (!out || !n_res || res_cap < 0 || (res_cap && !res) || n_names < 0 || n_names > KE_MAX_XRES ||
      (n_names && !xres_names) || name_cap < 0 || (name_cap && !node_name))
    return bad("ke_decode_reservation arguments");
  Value doc;
  int rc = parse_doc(js, len, doc, "Reservation");
  if (rc) return rc;
  ke_reservation r{};
  ke_reservation_alloc a{};
  const Value* meta = doc.field("metadata");
  const Value* spec = doc.field("spec");
  const Value* status = doc.field("status");
  std::map<std::string, std::string> ann, lab;
  if ((rc = string_map(meta ? meta->field("annotations") : nullptr, ann, "metadata.annotations"))) return rc;
  if ((rc = string_map(meta ? meta->field("labels") : nullptr, lab, "metadata.labels"))) return rc;
  r.node = -1;
  const std::string uid = str_or_empty(meta ? meta->field("uid") : nullptr);
  r.uid = uid.empty() ? 0 : (int64_t)(fnv1a(uid) & (uint64_t)INT64_MAX);
  // GetReservationNodeName = status.nodeName; IsReservationAvailable: scheduled and phase Available
  // (util/reservation/reservation.go:238-240,263-265)
  const std::string node = str_or_empty(status ? status->field("nodeName") : nullptr);
  const std::string phase = str_or_empty(status ? status->field("phase") : nullptr);
  bool available = !node.empty() && phase == "Available";
  if (name_cap) {
    if ((int64_t)node.size() + 1 > name_cap) return bad("status.nodeName longer than node_name");
    std::memcpy(node_name, node.c_str(), node.size() + 1);
  }
  // spec.allocateOnce (default true, apis/extension/reservation.go:133-135), spec.allocatePolicy
  const Value* once = spec ? spec->field("allocateOnce") : nullptr;
  r.allocate_once = (!once || once->is_null()) ? 1 : (once->t == Value::BOOL ? (uint8_t)once->b : 2);
  if (r.allocate_once > 1) return bad("spec.allocateOnce is not a boolean");
  const std::string pol = str_or_empty(spec ? spec->field("allocatePolicy") : nullptr);
  if (pol == "" || pol == "Default") r.allocate_policy = KE_RSV_POLICY_DEFAULT;
  else if (pol == "Aligned") r.allocate_policy = KE_RSV_POLICY_ALIGNED;
  else if (pol == "Restricted") r.allocate_policy = KE_RSV_POLICY_RESTRICTED;
  else return unsup("allocate policy \"" + pol + "\"");
  // the reservation-order label (findMostPreferredReservationByOrder, reservation/scoring.go:169-189): unparsable = none
  if (const std::string* o = lookup(lab, "scheduling.koordinator.sh/reservation-order")) {
    int64_t v;
    if (parse_int64(*o, &v)) r.order = v;
  }
  // ReservationRequests (reservation.go:393-404): status.allocatable when available, else the template pod's
  // PodRequests
  std::map<std::string, __int128> alloc_q;
  if (available) {
    RL st;
    if (!resource_list(status ? status->field("allocatable") : nullptr, st))
      return st.overflow ? unsup("status.allocatable quantity out of range") : bad("status.allocatable");
    alloc_q = st.q;
  } else {
    const Value* tspec = spec && spec->field("template") ? spec->field("template")->field("spec") : nullptr;
    std::vector<Container> cs, ics;
    if ((rc = containers(tspec ? tspec->field("containers") : nullptr, cs, "spec.template.spec.containers"))) return rc;
    if ((rc = containers(tspec ? tspec->field("initContainers") : nullptr, ics, "spec.template.spec.initContainers"))) return rc;
    RL overhead;
    if (!resource_list(tspec ? tspec->field("overhead") : nullptr, overhead)) return bad("spec.template.spec.overhead");
    alloc_q = pod_total(cs, ics, overhead, false);
  }
  RL allocatable, allocated;
  allocatable.q = alloc_q;
  if (!resource_list(status ? status->field("allocated") : nullptr, allocated))
    return allocated.overflow ? unsup("status.allocated quantity out of range") : bad("status.allocated");
  // rInfo.Reserved: the node-reservation annotation's resources, cpu = |reservedCPUs| when set (util/node.go:85-120)
  RL reserved;
  if (const std::string* s = lookup(ann, "node.koordinator.sh/reservation")) {
    Value v;
    std::string err;
    if (!json::parse(s->c_str(), s->size(), v, err) || !v.is_obj()) return bad("node.koordinator.sh/reservation annotation");
    if (!resource_list(v.field("resources"), reserved)) return bad("node.koordinator.sh/reservation resources");
    std::vector<int> cpus;
    const std::string rc_s = str_or_empty(v.field("reservedCPUs"));
    if (!rc_s.empty()) {
      if (!parse_cpuset(rc_s, cpus)) return bad("node.koordinator.sh/reservation reservedCPUs");
      reserved.q["cpu"] = (__int128)cpus.size() * 1000000000;
    }
  }
  // rInfo.ResourceNames: the allocatable's names, for Restricted narrowed by the restricted-options annotation
  // (reservation_info.go:87-96, util/reservation/reservation.go:637-654); a malformed annotation is a ParseError
  std::vector<std::string> keep;
  bool restricted_opts = false;
  if (r.allocate_policy == KE_RSV_POLICY_RESTRICTED) {
    if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/reservation-restricted-options")) {
      Value v;
      std::string err;
      if (!s->empty()) {
        if (!json::parse(s->c_str(), s->size(), v, err) || !v.is_obj()) {
          available = false;  // ParseError: the reservation takes no part
        } else if (const Value* rs = v.field("resources")) {
          if (rs->t == Value::ARR)
            for (const Value& x : rs->a)
              if (x.t == Value::STR) keep.push_back(x.s);
          restricted_opts = true;
        }
      }
    }
  }
  auto excluded = [&](const std::string& name) {
    if (!restricted_opts) return false;
    bool any = false, in = false;  // (an options list matching none of the names keeps them all)
    for (const auto& kv : alloc_q)
      if (kv.second != 0)
        for (const std::string& k : keep) any = any || k == kv.first;
    for (const std::string& k : keep) in = in || k == name;
    return any && !in;
  };
  r.available = available ? 1 : 0;
  int32_t ne = 0;
  for (const auto& kv : alloc_q) {
    if (kv.second == 0) continue;  // a zero quantity: not a resource name of the reservation
    int64_t av, al, rs;
    if (!rl_get(allocatable, kv.first, &av) || !rl_get(allocated, kv.first, &al) || !rl_get(reserved, kv.first, &rs))
      return unsup("reservation quantity out of range");
    if (kv.first == "cpu" || kv.first == "memory") {
      const int k = kv.first == "cpu" ? KE_RES_CPU : KE_RES_MEMORY;
      r.allocatable[k] = av;
      r.allocated[k] = excluded(kv.first) ? 0 : al;
      r.reserved[k] = rs;
      if (excluded(kv.first)) r.names_excluded |= (uint8_t)(1u << k);
      continue;
    }
    int32_t id = kv.first == "pods" ? KE_RSV_RES_PODS : -2;
    for (int32_t q = 0; q < n_names && id == -2; q++)
      if (xres_names[q] && kv.first == xres_names[q]) id = q;
    if (id == -2) return unsup("reservation allocatable \"" + kv.first + "\" without a resource id");
    if (id == KE_XRES_CPU || id == KE_XRES_MEMORY) return bad("xres_names maps cpu / memory");
    if (ne >= res_cap) return bad("more reservation resources than res_cap");
    if (av <= 0) return unsup("reservation allocatable \"" + kv.first + "\" not positive");
    ke_reservation_resource& e = res[ne++];
    e = ke_reservation_resource{};
    e.id = id;
    e.excluded = excluded(kv.first) ? 1 : 0;
    e.allocatable = av;
    e.allocated = e.excluded ? 0 : al;
    e.reserved = rs;
  }
  *n_res = ne;
  // the reserve pod's holdings: its DeviceAllocations (device-allocated annotation, device_share.go:32,246-262) and
  // its ResourceStatus (resource-status annotation: CPUSet + NUMANodeResources, numa_aware.go:83-94,257-268); the
  // owner parts are the owner pods' own annotations (the caller's)
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/device-allocated")) {
    Value v;
    std::string err;
    if (!json::parse(s->c_str(), s->size(), v, err) || !v.is_obj()) return bad("device-allocated annotation");
    for (const auto& kv : v.o) {
      int t = -1;
      for (int q = 0; q < KE_DEV_TYPES; q++)
        if (kv.first == DEV_TYPE_NAMES[q]) t = q;
      if (t < 0) return unsup("device-allocated type \"" + kv.first + "\"");
      if (kv.second.t != Value::ARR) return bad("device-allocated list");
      for (const Value& d : kv.second.a) {
        int64_t minor;
        const Value* mv = d.field("minor");
        if (!mv || !json::as_int64(*mv, &minor)) return bad("device-allocated minor");
        if (minor < 0 || minor >= KE_MAX_MINORS) return unsup("device-allocated minor beyond 15");
        RL rl;
        if (!resource_list(d.field("resources"), rl)) return bad("device-allocated resources");
        a.device_minors |= 1ull << (16 * t + minor);
        for (int k = 0; k < KE_DKEYS; k++) {
          if (!DEV_KEY_NAMES[t][k]) continue;
          int64_t x;
          if (!rl_get(rl, DEV_KEY_NAMES[t][k], &x)) return unsup("device-allocated quantity out of range");
          a.device[t][minor][k] += x;
        }
      }
    }
  }
  if (const std::string* s = lookup(ann, "scheduling.koordinator.sh/resource-status")) {
    Value v;
    std::string err;
    if (!json::parse(s->c_str(), s->size(), v, err) || !v.is_obj()) return bad("resource-status annotation");
    std::vector<int> cpus;
    if (!parse_cpuset(str_or_empty(v.field("cpuset")), cpus)) return bad("resource-status cpuset");
    for (int c : cpus) {
      if (c >= KE_MAX_CPUS) return unsup("resource-status cpuset beyond the CPU id range");
      a.cpuset[c >> 6] |= 1ull << (c & 63);
    }
    if (const Value* nr = v.field("numaNodeResources")) {
      if (nr->t != Value::ARR && !nr->is_null()) return bad("resource-status numaNodeResources");
      for (size_t q = 0; nr->t == Value::ARR && q < nr->a.size(); q++) {
        const Value& z = nr->a[q];
        int64_t id;
        const Value* iv = z.field("node");
        if (!iv || !json::as_int64(*iv, &id)) return bad("numaNodeResources node");
        if (id < 0 || id >= KE_MAX_NUMA) return unsup("numaNodeResources node beyond the NUMA id range");
        RL rl;
        if (!resource_list(z.field("resources"), rl)) return bad("numaNodeResources resources");
        int64_t cpu, mem;
        if (!rl_get(rl, "cpu", &cpu) || !rl_get(rl, "memory", &mem)) return unsup("numaNodeResources quantity out of range");
        a.numa[2 * id + KE_RES_CPU] += cpu;
        a.numa[2 * id + KE_RES_MEMORY] += mem;
      }
    }
  }
  r.holds = (uint8_t)(resv_holds_of(a) | (ne > 0 ? KE_RSV_OTHER_ALLOCATABLE : 0u));
  // allocated pods: status.currentOwners (the cache counts the assigned pods it tracks)
  if (const Value* owners = status ? status->field("currentOwners") : nullptr)
    if (owners->t == Value::ARR) r.allocated_pods = (int32_t)owners->a.size();
  *out = r;
  if (alloc) *alloc = a;
  return KE_OK;
}

}  // extern "C"
