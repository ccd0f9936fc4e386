// ke_capi.cpp — the extern "C" boundary (include/koord_eval.h) over the host state (ke_host.cpp)
// and the device evaluator (ke_kernels.hip).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>
#include <new>

#include "ke_host.h"

namespace ke {
const char* last_error_cstr();
int device_available();
int device_create(Context* ctx);
void device_destroy(Context* ctx);
int device_eval(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, uint8_t* status, uint8_t* reason,
                int16_t* la, int16_t* numa, int16_t* ds, int16_t* total, int32_t* best);
int device_schedule(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, int32_t* chosen, int32_t* score);
int device_rsv_result(Context* ctx, int32_t* out4);
int device_rsv_gate(const Context* ctx);
int device_refresh(Context* ctx, int64_t now, bool defer);
int device_ds_views(Context* ctx, const ke_pod& pod, int64_t now, const std::vector<DsView>& views,
                    std::vector<DsViewOut>& out);
int device_rsv_views(Context* ctx, const ke_pod& pod, int64_t now, const std::vector<RsvView>& views,
                     std::vector<RsvViewOut>& out);
int device_numa_views(Context* ctx, const ke_pod& pod, int64_t now, const std::vector<NumaRsvView>& views,
                      std::vector<NumaRsvOut>& out);
int device_quota_sync(Context* ctx);
int device_debug_rows(Context* ctx, int32_t n, Row* out);
int device_set_profiling(Context* ctx, int32_t every);
int device_set_pipeline(Context* ctx, int32_t on);
int device_replay_phases(Context* ctx, int which, double* cyc8);
int device_check_records(Context* ctx, int64_t now, int64_t* bad);
int device_bench_eval(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, int32_t iters, double* avg_ms);
int device_comm_unique_id(uint8_t* id);
int device_shard_init(Context* ctx, int rank, int world, const uint8_t* id);
int device_shard_init_host(Context* ctx, int rank, int world, ke_host_collective fn, void* user);
int device_shard_range(Context* ctx, int* lo, int* hi);
bool device_sharded(const Context* ctx);
}  // namespace ke

using namespace ke;

// KOORDEVAL_RSV_FUSE=0: every reservation-matched pod is a segment of its own (the fused path's A/B)
static const bool kFuseMatched = [] {
  const char* e = std::getenv("KOORDEVAL_RSV_FUSE");
  return !e || std::atoi(e) != 0;
}();

// The release records of one completed call (ke_last_allocations / ke_unreserve read them from the Context):
// taken when the call completes, restored when ke_schedule_wait collects it, so a wait on an earlier ticket
// never pairs that call's nodes with a later call's cpusets / NUMA amounts / device minors.
struct CallRecords {
  std::vector<int32_t> chosen, resv;
  std::vector<int64_t> uid, numa;
  std::vector<uint8_t> quota;
  std::vector<uint64_t> cpusets, dev;
  std::vector<int8_t> vf;
  int32_t resv_gen = 0;  // the reservation set `resv` indexes
  void save(const Context& c) {
    chosen = c.last_chosen, resv = c.last_resv, uid = c.last_uid, numa = c.last_numa_alloc, quota = c.last_quota;
    cpusets = c.last_cpusets, dev = c.last_dev_alloc, vf = c.last_vf;
    resv_gen = c.resv_gen;
  }
  void restore(Context& c) {
    c.last_chosen.swap(chosen), c.last_uid.swap(uid), c.last_numa_alloc.swap(numa), c.last_quota.swap(quota);
    c.last_cpusets.swap(cpusets), c.last_dev_alloc.swap(dev), c.last_vf.swap(vf);
    // a reservation set loaded since names other reservations: as load_reservations does, the records drop them
    if (resv_gen == c.resv_gen) c.last_resv.swap(resv);
    else c.last_resv.assign(c.last_chosen.size(), 0);
  }
};

// A ke_schedule_submit call: its device work in flight (`fin` set), or completed with its outputs kept until
// ke_schedule_wait collects them.
struct AsyncCall {
  int64_t ticket = 0;
  int32_t n = 0;
  const ke_pod* pods = nullptr;  // the caller's array (valid until its ke_schedule_wait)
  int64_t now = 0;
  bool device = false;  // enqueued by ke_schedule_submit (its release records are set when it is collected)
  DevFinish fin;
  int rc = KE_OK;
  std::string msg;
  std::vector<int32_t> chosen, score;
  CallRecords rec;  // its release records (set when it completes)
};

struct ke_ctx {
  Context c;
  std::deque<AsyncCall> async;  // submitted, not yet collected (ticket order)
  int64_t next_ticket = 1;
};

// A submitted call's completion (in submission order): waits for its device work, takes its outputs and statistics,
// and queues its host mirror (the deferred LoadAware assign / NodeInfo.Requested of its placed pods).
static void async_finish(ke_ctx* ctx, AsyncCall& a) {
  if (!a.fin) return;
  DevFinish f = std::move(a.fin);
  a.fin = nullptr;
  a.chosen.assign((size_t)a.n, -1);
  a.score.assign((size_t)a.n, 0);
  a.rc = f(a.chosen.data(), a.score.data());
  if (a.rc) {
    a.msg = last_error_cstr();
    return;
  }
  Context& c = ctx->c;
  // the completion wrote this call's device / cpuset / VF / NUMA records into the Context; a plain queue assumes
  // no reservation and no quota
  c.last_chosen = a.chosen;
  c.last_uid.resize((size_t)a.n);
  for (int32_t p = 0; p < a.n; p++) c.last_uid[(size_t)p] = a.pods[p].uid;
  c.last_quota.assign((size_t)a.n, 0);
  c.last_resv.assign((size_t)a.n, 0);
  a.rec.save(c);
  const int32_t off = c.cfg.global_node_offset;
  const int64_t base = c.pending_base;  // the completion copied the pods there
  c.pending.reserve(c.pending.size() + (size_t)a.n);
  for (int32_t i = 0; i < a.n; i++) {
    const int32_t node = a.chosen[(size_t)i] - off;
    if (a.chosen[(size_t)i] < 0 || node < 0 || node >= c.n_nodes) continue;
    c.pending.push_back({node, a.now, base + i});
  }
}

// Every call in flight completes (an entry point that reads or changes the state the submitted calls work on).
static void async_drain(ke_ctx* ctx) {
  for (AsyncCall& a : ctx->async) async_finish(ctx, a);
  mirror_join(ctx->c);
}

static int check_node(ke_ctx* ctx, int32_t node) {
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  if (node < 0 || node >= ctx->c.cfg.node_capacity) return fail(KE_ERR_NOT_FOUND, "node index out of range");
  return KE_OK;
}

static int check_pods(const ke_pod* pods, int32_t n, const Context* c = nullptr, bool matched_ok = false) {
  if (n < 0 || (n > 0 && !pods)) return fail(KE_ERR_INVALID, "pods");
  for (int32_t p = 0; p < n; p++) {
    int rc = validate_pod(pods[p]);
    if (rc) return rc;
    const uint8_t rm = pods[p].reservation_matched;
    if (rm > KE_RSV_IGNORED) return fail(KE_ERR_INVALID, "ke_pod.reservation_matched");
    if (rm != KE_RSV_NONE && !matched_ok)
      return fail(KE_ERR_UNSUPPORTED, "a pod matching / ignoring reservations outside ke_schedule");
    if (c) rc = validate_pod_hints(*c, pods[p]);
    else if (pods[p].device_hint) rc = fail(KE_ERR_INVALID, "ke_pod.device_hint without a context");
    if (rc) return rc;
    if (c && c->cfg.fit.filter)  // NodeResourcesFit's Filter checks every requested scalar: it must have a slot
      for (int e = 0; e < pods[p].n_xres; e++) {
        const int32_t id = pods[p].xres_id[e];
        bool known = id == KE_XRES_CPU || id == KE_XRES_MEMORY || pods[p].xres_value[e] == 0;
        for (int q = 0; q < c->cfg.fit.n_scalars && !known; q++) known = c->cfg.fit.scalars[q] == id;
        if (!known) return fail(KE_ERR_UNSUPPORTED, "a pod requesting a scalar resource outside ke_fit_args.scalars");
      }
  }
  return KE_OK;
}

static int require_device(ke_ctx* ctx) {
  if (!ctx->c.dev) return fail(KE_ERR_NO_DEVICE, "evaluation needs the gfx950 device; this context has none");
  return KE_OK;
}

// A pod with its own NUMA topology policy switches the NUMA path on for every node (DeviceShare pods on
// NUMA-policy nodes take part in the topology manager's Admit as a second hint provider).
static int check_numa_deviceshare(ke_ctx* ctx, const ke_pod* pods, int32_t n) {
  for (int32_t p = 0; p < n; p++)
    if (pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE) ctx->c.numa_enabled = true;
  return KE_OK;
}

// A pod that may bind CPUs (a cpuset pod, or any cpu request while a node forces CPU binding) reads the
// CPU SoA during evaluation: make sure it exists.
// The pods' DevPod records are staged for upload_pods (built once per call).
static int check_cpuset(ke_ctx* ctx, const ke_pod* pods, int32_t n) {
  Context& c = ctx->c;
  c.staged.resize((size_t)n);
  c.staged_src = pods;
  for (int32_t p = 0; p < n; p++) {
    c.staged[p] = make_dev_pod(c.cfg, pods[p], pod_hints(c, pods[p]), &c.tmpl);
    const uint32_t f = c.staged[p].flags;
    if ((f & PF_CPUSET) || (c.n_bind_nodes > 0 && pods[p].requests[KE_RES_CPU] > 0)) c.cpu_enabled = true;
  }
  return KE_OK;
}

// ke_pod_reservations lists of a ke_schedule call (consumed by it): shape, and the KE_RSV_MATCHED pods the
// nominated-reservation path supports.  Every refusal of that path is raised here, before the
// call schedules any pod: a refusal after earlier segments ran would leave their Reserves applied.
static int check_matches(Context& c, const ke_pod* pods, int32_t n) {
  const bool staged = !c.match_off.empty();
  if (staged && (int32_t)c.match_off.size() != n + 1) {
    c.match_off.clear();
    c.match_ids.clear();
    return fail(KE_ERR_INVALID, "ke_pod_reservations lists for a different number of pods");
  }
  for (int32_t p = 0; p < n; p++) {
    const int32_t cnt = staged ? c.match_off[(size_t)p + 1] - c.match_off[(size_t)p] : 0;
    const uint8_t rm = pods[p].reservation_matched;
    if (rm != KE_RSV_MATCHED && rm != KE_RSV_AFFINITY) {
      if (cnt) return fail(KE_ERR_INVALID, "reservations listed for a pod that is not KE_RSV_MATCHED / AFFINITY");
      if (rm == KE_RSV_IGNORED) {
        const int rc = resv_ignore_check(c, pods[p], c.staged[(size_t)p].flags);
        if (rc) return rc;
      }
      continue;
    }
    if (!staged) return fail(KE_ERR_INVALID, "a KE_RSV_MATCHED / AFFINITY pod without ke_pod_reservations");
    const uint32_t f = c.staged[(size_t)p].flags;
    // (the Reservation plugin reads the pod's requests by name: every name other than cpu / memory through its
    // ke_pod.xres entry -- batch / mid resources and device resources included -- so a requested name without a
    // resource id is refused)
    if (pods[p].has_other_requests > 1 || pods[p].has_unsupported_device_requests)
      return fail(KE_ERR_UNSUPPORTED, "a pod matching reservations with unnamed resources");
    // a DeviceShare pod allocates from its matched reservations' devices (resv_ds_views) -- not with device hints /
    // joint allocation, nor in NUMA hints (a pod with a NUMA policy, or a NUMA-policy node, beside a matched
    // reservation holding devices)
    if ((f & (PF_DS | PF_DS_HINT)) && !c.resv_holds.empty())
      for (int32_t j = c.match_off[(size_t)p]; j < c.match_off[(size_t)p + 1]; j++) {
        const int32_t r = c.match_ids[(size_t)j];
        if (r < 0 || r >= (int32_t)c.resv.size() || !resv_usable(c.resv[(size_t)r]) ||
            !(c.resv_holds[(size_t)r] & KE_RSV_HOLDS_DEVICES))
          continue;
        if ((f & PF_DS_HINT) || pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE ||
            c.nodes[(size_t)c.resv[(size_t)r].node].node.numa_topology_policy != KE_NUMA_POLICY_NONE)
          return fail(KE_ERR_UNSUPPORTED, "a DeviceShare pod with device hints or NUMA hints matching a reservation "
                                          "that holds devices");
      }
    // under a NUMA policy (the pod's or the node's) a matched reservation holding NUMA resources or CPUs enters the
    // hints through its allocate-from-reservation trials (k_numa_views) for a pod without device requests -- one
    // binding CPUs too (whole CPUs, not under a required FullPCPUs policy: preferredCPUs taken first may split cores,
    // which the per-view counts do not see); a DeviceShare pod's joint hints there are not restated, nor more than
    // NV_MAX such reservations of the pod on one node
    if (!c.resv_holds.empty()) {
      const bool binds = (f & PF_CPUSET) || (c.n_bind_nodes > 0 && pods[p].requests[KE_RES_CPU] > 0);
      const bool dev = (f & (PF_DS | PF_DS_HINT)) != 0;
      std::vector<std::pair<int32_t, int32_t>> per_node;
      for (int32_t j = c.match_off[(size_t)p]; j < c.match_off[(size_t)p + 1]; j++) {
        const int32_t r = c.match_ids[(size_t)j];
        if (r < 0 || r >= (int32_t)c.resv.size() || !resv_usable(c.resv[(size_t)r]) ||
            !(c.resv_holds[(size_t)r] & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)))
          continue;
        const int32_t node = c.resv[(size_t)r].node;
        const bool pol = pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE ||
                         c.nodes[(size_t)node].node.numa_topology_policy != KE_NUMA_POLICY_NONE;
        const int preq = pf_cpu_required(f);
        const bool full_req = preq == XB_FULL || (preq == XB_NONE && c.nodes[(size_t)node].node.cpu_bind_policy ==
                                                                         KE_NODE_CPU_BIND_FULL_PCPUS_ONLY);
        if (pol && (dev || (binds && (!(f & PF_CPU_INT) || full_req))))
          return fail(KE_ERR_UNSUPPORTED, "a pod requesting devices, fractional CPUs or a required FullPCPUs binding "
                                          "under a NUMA topology policy matching a reservation that holds NUMA "
                                          "resources or CPUs");
        bool seen = false;
        for (auto& e : per_node)
          if (e.first == node) seen = true, e.second++;
        if (!seen) per_node.emplace_back(node, 1);
      }
      for (auto& e : per_node)
        if (e.second > NV_MAX)
          return fail(KE_ERR_UNSUPPORTED, "more matched reservations holding NUMA resources / CPUs on a node than "
                                          "NV_MAX");
    }
    const int rc = resv_check(c, c.match_ids.data() + c.match_off[(size_t)p], cnt);
    if (rc) return rc;
  }
  return KE_OK;
}

extern "C" {

int ke_abi_version(void) { return KE_ABI_VERSION; }
int ke_abi_struct_sizes(int32_t* sizes, int32_t n) {
  const int32_t all[] = {(int32_t)sizeof(ke_config),       (int32_t)sizeof(ke_node),
                         (int32_t)sizeof(ke_node_metric),  (int32_t)sizeof(ke_pod_metric),
                         (int32_t)sizeof(ke_aggregated_usage), (int32_t)sizeof(ke_pod),
                         (int32_t)sizeof(ke_resource_map), (int32_t)sizeof(ke_loadaware_args),
                         (int32_t)sizeof(ke_numa_args), (int32_t)sizeof(ke_deviceshare_args),
                         (int32_t)sizeof(ke_device),       (int32_t)sizeof(ke_numa_zone),
                         (int32_t)sizeof(ke_cpu),          (int32_t)sizeof(ke_quota_args),
                         (int32_t)sizeof(ke_quota),        (int32_t)sizeof(ke_gpu_partition),
                         (int32_t)sizeof(ke_ext_args),     (int32_t)sizeof(ke_node_resource),
                         (int32_t)sizeof(ke_pod_allocation), (int32_t)sizeof(ke_pod_device_hints),
                         (int32_t)sizeof(ke_gpu_template),   (int32_t)sizeof(ke_reservation),
                         (int32_t)sizeof(ke_reservation_alloc), (int32_t)sizeof(ke_reservation_resource)};
  const int32_t m = (int32_t)(sizeof(all) / sizeof(all[0]));
  for (int32_t i = 0; i < n && i < m; i++) sizes[i] = all[i];
  return m;
}
const char* ke_last_error(void) { return last_error_cstr(); }
int ke_device_available(void) { return device_available(); }
int ke_row_bytes(void) { return ROW_BYTES; }
int ke_pod_record_bytes(void) { return (int)sizeof(DevPod); }

int ke_create(const ke_config* cfg, ke_ctx** out) {
  if (!cfg || !out) return fail(KE_ERR_INVALID, "null argument");
  *out = nullptr;
  int rc = validate_config(*cfg);
  if (rc) return rc;
  ke_ctx* ctx = new (std::nothrow) ke_ctx();
  if (!ctx) return fail(KE_ERR_INVALID, "out of memory");
  Context& c = ctx->c;
  c.cfg = *cfg;
  c.nodes.resize((size_t)cfg->node_capacity);
  for (int32_t i = 0; i < cfg->node_capacity; i++) c.nodes[(size_t)i].dirty.bind(i, &c.dirty_list);
  KArgs& k = c.kargs_template;
  const ke_loadaware_args& a = cfg->loadaware;
  k.exp_s = a.node_metric_expiration_seconds;
  uint32_t f = 0;
  if (a.filter_expired_node_metrics) f |= AF_FILTER_EXPIRED;
  if (a.enable_schedule_when_node_metrics_expired) f |= AF_ENABLE_WHEN_EXPIRED;
  if (a.node_metric_expiration_seconds != KE_ABSENT) f |= AF_EXP_PRESENT;
  if (cfg->numa.strategy == KE_STRATEGY_MOST_ALLOCATED) f |= AF_NUMA_MOST;
  if (cfg->deviceshare.strategy == KE_STRATEGY_MOST_ALLOCATED) f |= AF_DS_MOST;
  if (cfg->deviceshare.disable_numa_alignment) f |= AF_DS_NO_NUMA;
  if (cfg->numa.numa_strategy == KE_STRATEGY_MOST_ALLOCATED) f |= AF_NUMA_HINT_MOST;
  k.flags = f;
  k.wsum_la = k.wsum_numa = 0;
  for (int r = 0; r < KE_NRES; r++) {
    k.w_la[r] = a.resource_weights[r] == KE_ABSENT ? 0 : (int32_t)a.resource_weights[r];
    k.w_numa[r] = cfg->numa.weights[r] == KE_ABSENT ? 0 : (int32_t)cfg->numa.weights[r];
    k.wsum_la += k.w_la[r];
    k.wsum_numa += k.w_numa[r];
  }
  k.wp_la = (int32_t)cfg->weight_loadaware;
  k.wp_numa = (int32_t)cfg->weight_numa;
  k.wp_ds = (int32_t)cfg->weight_deviceshare;
  for (int i = 0; i < 4; i++)
    k.w_ds[i] = cfg->deviceshare.weights[i] == KE_ABSENT ? -1 : (int32_t)cfg->deviceshare.weights[i];
  // NodeResourcesFitPlus / ScarceResourceAvoidance: their Score joins every evaluation path (eval_pair,
  // lite_total, and the fast replay's fast_total from the node's ext words)
  // and NodeResourcesFit: ext slots (ext_slots: FitPlus resources first, then Fit's resources and scalars)
  const ke_ext_args& x = cfg->ext;
  const ke_fit_args& fa = cfg->fit;
  k.wp_fp = (int32_t)x.weight_fitplus;
  k.wp_sra = (int32_t)x.weight_sra;
  k.wp_fit = (int32_t)fa.weight;
  k.sra_mask = x.sra_resources;
  int32_t ids[2 * NUM_XS + KE_MAX_FITPLUS];
  k.xs_n = ext_slots(*cfg, ids);
  k.fp_mask = k.fp_most = k.fit_mask = k.fit_scalar = 0;
  for (int q = 0; q < NUM_XS; q++) {
    k.xs_id[q] = q < k.xs_n ? ids[q] : 0;
    k.fp_w[q] = k.fit_w[q] = 0;
  }
  for (int q = 0; q < x.n_fitplus; q++) {  // FitPlus resource q is slot q
    k.fp_mask |= 1u << q;
    k.fp_w[q] = x.fitplus[q].weight;
    if (x.fitplus[q].type == KE_STRATEGY_MOST_ALLOCATED) k.fp_most |= 1u << q;
  }
  for (int q = 0; q < k.xs_n; q++) {
    for (int r = 0; r < fa.n_resources; r++)
      if (fa.resources[r].id == k.xs_id[q]) k.fit_mask |= 1u << q, k.fit_w[q] = fa.resources[r].weight;
    for (int r = 0; r < fa.n_scalars; r++)
      if (fa.scalars[r] == k.xs_id[q]) k.fit_scalar |= 1u << q;
  }
  if (fa.filter) k.flags |= AF_FIT_FILTER;
  if (fa.strategy == KE_STRATEGY_MOST_ALLOCATED) k.flags |= AF_FIT_MOST;
  if (x.weight_fitplus > 0 || x.weight_sra > 0 || fa.weight > 0 || fa.filter) {
    k.flags |= AF_EXT;
    c.ext_enabled = true;
  }
  if (device_available()) {
    rc = device_create(&c);
    if (rc) {
      device_destroy(&c);
      delete ctx;
      return rc;
    }
  }
  *out = ctx;
  return KE_OK;
}

void ke_destroy(ke_ctx* ctx) {
  if (!ctx) return;
  async_drain(ctx);
  device_destroy(&ctx->c);
  delete ctx;
}

int32_t ke_num_nodes(ke_ctx* ctx) { return ctx ? ctx->c.n_nodes : 0; }

int ke_node_resources_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_node_resource* res) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  rc = validate_node_resources(n, res);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.xres.assign(res, res + n);
  ns.dirty = true;
  ctx->c.n_nodes = std::max(ctx->c.n_nodes, node + 1);
  return KE_OK;
}

int ke_node_resources_get(ke_ctx* ctx, int32_t node, int32_t cap, ke_node_resource* res, int32_t* n) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  if (!n || cap < 0 || (cap > 0 && !res)) return fail(KE_ERR_INVALID, "ke_node_resources_get arguments");
  const NodeState& ns = ctx->c.nodes[node];
  *n = (int32_t)ns.xres.size();
  for (int32_t e = 0; e < cap && e < *n; e++) res[e] = ns.xres[e];
  return KE_OK;
}

int ke_debug_rsv_fused(ke_ctx* ctx, int64_t* out2) {
  if (!ctx || !out2) return fail(KE_ERR_INVALID, "ke_debug_rsv_fused arguments");
  out2[0] = ctx->c.last_rsv_fused;
  out2[1] = ctx->c.last_rsv_fused_gated;
  return KE_OK;
}

int ke_debug_ds_cuts(ke_ctx* ctx, int32_t* cuts) {
  if (!ctx || !cuts) return fail(KE_ERR_INVALID, "ke_debug_ds_cuts arguments");
  *cuts = ctx->c.last_ds_cuts;
  return KE_OK;
}

int ke_node_upsert(ke_ctx* ctx, int32_t node, const ke_node* n) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  if (!n) return fail(KE_ERR_INVALID, "null node");
  rc = validate_node(*n);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  if (ns.valid) {
    ctx->c.n_bind_nodes -= ns.node.cpu_bind_policy != KE_NODE_CPU_BIND_NONE;
    ctx->c.n_policy_nodes -= ns.node.numa_topology_policy != KE_NUMA_POLICY_NONE;
  }
  ns.valid = true;
  ns.known = true;
  ns.node = *n;
  ns.dirty = true;
  ctx->c.n_bind_nodes += n->cpu_bind_policy != KE_NODE_CPU_BIND_NONE;
  ctx->c.n_policy_nodes += n->numa_topology_policy != KE_NUMA_POLICY_NONE;
  if (n->numa_topology_policy != KE_NUMA_POLICY_NONE) ctx->c.numa_enabled = true;
  ctx->c.n_nodes = std::max(ctx->c.n_nodes, node + 1);
  return KE_OK;
}

int ke_node_delete(ke_ctx* ctx, int32_t node) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);  // pending Reserves on it first: the object state stays (koord_eval.h)
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  if (!ns.valid) return KE_OK;
  ctx->c.n_bind_nodes -= ns.node.cpu_bind_policy != KE_NODE_CPU_BIND_NONE;
  ctx->c.n_policy_nodes -= ns.node.numa_topology_policy != KE_NUMA_POLICY_NONE;
  ns.valid = false;  // derive_row: no NF_VALID -> every Filter path fails the node
  ns.dirty = true;
  return KE_OK;
}

int ke_node_topology_delete(ke_ctx* ctx, int32_t node) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  // the NodeAllocation stays (resource_manager.go keeps nodeAllocations[node] until the Node itself goes)
  if (!ns.cpus.empty()) ns.kept_cpus = ns.cpus;
  if (!ns.zones.empty()) ns.kept_zones = ns.zones;
  ns.zones.clear();
  ns.cpus.clear();
  ns.cpu_max_ref = 1;
  ns.node.cpuset_allocated_cpus = 0;        // GetAvailableCPUs without a CPU topology: no allocated CPUs
  ns.node.nrt_cpu_amplification_ratio = -2;  // no NRT ratio map
  ns.node.cpu_topology_invalid = 0;
  ns.dirty = true;
  return KE_OK;
}

int ke_nodes_load(ke_ctx* ctx, int32_t n, const ke_node* nodes) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || (n > 0 && !nodes)) return fail(KE_ERR_INVALID, "ke_nodes_load arguments");
  if (ctx) flush_mirror(ctx->c);
  if (n > ctx->c.cfg.node_capacity) return fail(KE_ERR_INVALID, "more nodes than node_capacity");
  for (int32_t i = 0; i < n; i++) {
    int rc = ke_node_upsert(ctx, i, &nodes[i]);
    if (rc) return rc;
  }
  return KE_OK;
}

int ke_node_devices_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_device* devices) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  rc = validate_devices(n, devices);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.has_dev_cache = true;
  ns.devs.assign(devices, devices + n);
  rc = intern_device_labels(ctx->c, ns);
  if (rc) return rc;
  ns.dirty = true;
  ctx->c.ds_enabled = true;
  return KE_OK;
}

int ke_node_device_flags(ke_ctx* ctx, int32_t node, int32_t secondary_well_planned, int32_t gpu_model_key) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  const int id = intern_model_key(ctx->c, gpu_model_key);
  if (id < 0) return id;
  NodeState& ns = ctx->c.nodes[node];
  ns.secondary_well_planned = secondary_well_planned != 0;
  ns.gpu_model_id = id;
  ns.dirty = true;
  return KE_OK;
}

int ke_set_pod_device_hints(ke_ctx* ctx, int32_t n, const ke_pod_device_hints* hints) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || (n > 0 && !hints)) return fail(KE_ERR_INVALID, "ke_set_pod_device_hints arguments");
  ctx->c.hints.assign(hints, hints + n);
  return KE_OK;
}

int ke_gpu_templates_load(ke_ctx* ctx, int32_t n, const ke_gpu_template* templates) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || (n > 0 && !templates)) return fail(KE_ERR_INVALID, "ke_gpu_templates_load arguments");
  for (int32_t i = 0; i < n; i++) {
    const int id = intern_model_key(ctx->c, templates[i].model_key);
    if (id < 0) return id;
  }
  ctx->c.tmpl.assign(templates, templates + n);
  return KE_OK;
}

int ke_reservations_load(ke_ctx* ctx, int32_t n, const ke_reservation* reservations) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  flush_mirror(ctx->c);
  return load_reservations(ctx->c, n, reservations);
}

int ke_reservations_load_ex(ke_ctx* ctx, int32_t n, const ke_reservation* reservations,
                            const ke_reservation_alloc* allocs) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  flush_mirror(ctx->c);
  return load_reservations(ctx->c, n, reservations, allocs);
}

int ke_reservations_load_full(ke_ctx* ctx, int32_t n, const ke_reservation* reservations,
                              const ke_reservation_alloc* allocs, const int32_t* res_offsets,
                              const ke_reservation_resource* res) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  if (!res_offsets) return fail(KE_ERR_INVALID, "ke_reservations_load_full: res_offsets");
  flush_mirror(ctx->c);
  return load_reservations(ctx->c, n, reservations, allocs, res_offsets, res);
}

int ke_reservation_resources_get(ke_ctx* ctx, int32_t r, int32_t cap, ke_reservation_resource* out, int32_t* n) {
  if (ctx) async_drain(ctx);
  if (!ctx || !n || cap < 0 || (cap > 0 && !out) || r < 0 || r >= (int32_t)ctx->c.resv.size())
    return fail(KE_ERR_INVALID, "ke_reservation_resources_get arguments");
  const auto& e = (size_t)r < ctx->c.resv_res.size() ? ctx->c.resv_res[(size_t)r] : std::vector<ke_reservation_resource>{};
  *n = (int32_t)e.size();
  for (int32_t i = 0; i < cap && i < *n; i++) out[i] = e[(size_t)i];
  return KE_OK;
}

int ke_reservation_allocs_get(ke_ctx* ctx, int32_t n, ke_reservation_alloc* out) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || (n > 0 && !out) || n > (int32_t)ctx->c.resv.size())
    return fail(KE_ERR_INVALID, "ke_reservation_allocs_get arguments");
  for (int32_t i = 0; i < n; i++)
    out[i] = ctx->c.resv_alloc.empty() ? ke_reservation_alloc{} : ctx->c.resv_alloc[(size_t)i];
  return KE_OK;
}

int32_t ke_reservations_generation(ke_ctx* ctx) { return ctx ? ctx->c.resv_gen : 0; }

int ke_reservations_get(ke_ctx* ctx, int32_t n, ke_reservation* out) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || (n > 0 && !out) || n > (int32_t)ctx->c.resv.size()) return fail(KE_ERR_INVALID, "ke_reservations_get arguments");
  std::copy(ctx->c.resv.begin(), ctx->c.resv.begin() + n, out);
  return KE_OK;
}

int ke_pod_reservations(ke_ctx* ctx, int32_t n_pods, const int32_t* offsets, const int32_t* ids) {
  if (ctx) async_drain(ctx);
  if (!ctx || n_pods < 0 || !offsets) return fail(KE_ERR_INVALID, "ke_pod_reservations arguments");
  Context& c = ctx->c;
  if (offsets[0] != 0) return fail(KE_ERR_INVALID, "ke_pod_reservations offsets[0] != 0");
  for (int32_t p = 0; p < n_pods; p++)
    if (offsets[p + 1] < offsets[p]) return fail(KE_ERR_INVALID, "ke_pod_reservations offsets decrease");
  if (offsets[n_pods] > 0 && !ids) return fail(KE_ERR_INVALID, "ke_pod_reservations ids");
  for (int32_t j = 0; j < offsets[n_pods]; j++)
    if (ids[j] < 0 || ids[j] >= (int32_t)c.resv.size()) return fail(KE_ERR_NOT_FOUND, "ke_pod_reservations: reservation index");
  c.match_off.assign(offsets, offsets + n_pods + 1);
  c.match_ids.assign(ids, ids + offsets[n_pods]);
  return KE_OK;
}

int ke_node_info_requested(ke_ctx* ctx, int32_t node, int64_t* requested, int64_t* non_zero) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (rc) return rc;
  if (!requested || !non_zero) return fail(KE_ERR_INVALID, "ke_node_info_requested outputs");
  flush_mirror(ctx->c);
  const NodeState& ns = ctx->c.nodes[node];
  for (int k = 0; k < KE_NRES; k++) {
    requested[k] = ns.node.requested[k] + ns.rv_req[k];
    non_zero[k] = KE_ABSENT;  // NonZeroRequested is known from the node's ke_node_resources_set rows
    for (const ke_node_resource& r : ns.xres)
      if (r.id == k) non_zero[k] = xres_requested(ns, r);
  }
  return KE_OK;
}

int ke_node_gpu_partitions(ke_ctx* ctx, int32_t node, int32_t has_table, int32_t honor, int32_t n,
                           const ke_gpu_partition* partitions) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  if (n > 0 && !has_table) return fail(KE_ERR_INVALID, "partitions without a table");
  int id = -1;
  if (has_table) {
    id = ptable_intern(ctx->c, n, partitions);
    if (id < 0) return id;
  }
  NodeState& ns = ctx->c.nodes[node];
  ns.ptable = id;
  ns.gpu_honor = honor != 0;
  ns.dirty = true;
  return KE_OK;
}

int ke_node_devices_delete(ke_ctx* ctx, int32_t node) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.has_dev_cache = false;
  ns.devs.clear();
  ns.ptable = -1;
  ns.gpu_honor = false;
  ns.dirty = true;
  return KE_OK;
}

int ke_node_numa_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_numa_zone* zones) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  rc = validate_zones(n, zones);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.zones.assign(zones, zones + n);
  for (ke_numa_zone& z : ns.zones) normalize_zone(z);
  bool bare = true;  // an NRT without the resource manager's allocation: the parked one comes back
  for (const ke_numa_zone& z : ns.zones)
    bare = bare && !z.has_allocated && !z.single_pods && !z.shared_pods && !z.cpuset_cpus;
  if (bare)
    for (ke_numa_zone& z : ns.zones)
      for (const ke_numa_zone& k : ns.kept_zones)
        if (k.id == z.id) {
          z.has_allocated = k.has_allocated;
          for (int r = 0; r < KE_NRES; r++) z.allocated[r] = k.allocated[r];
          z.cpuset_cpus = k.cpuset_cpus;
          z.single_pods = k.single_pods;
          z.shared_pods = k.shared_pods;
          z.numa_status = zone_status(z);
        }
  if (n > 0) ns.kept_zones.clear();
  ns.dirty = true;
  ctx->c.numa_enabled = true;
  return KE_OK;
}

int ke_node_cpus_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_cpu* cpus, int32_t max_ref_count) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  rc = validate_cpus(n, cpus, max_ref_count);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.cpus.assign(cpus, cpus + n);
  ns.cpu_max_ref = n > 0 ? max_ref_count : 1;
  bool bare = true;  // a topology without allocatedCPUs: the parked NodeAllocation comes back by CPU id
  for (const ke_cpu& c : ns.cpus) bare = bare && c.ref_count == 0;
  if (bare)
    for (ke_cpu& c : ns.cpus)
      for (const ke_cpu& k : ns.kept_cpus)
        if (k.cpu_id == c.cpu_id) c.ref_count = k.ref_count, c.exclusive = k.exclusive;
  if (n > 0) ns.kept_cpus.clear();
  ns.dirty = true;
  if (n > 0) ctx->c.cpu_enabled = true;
  return KE_OK;
}

int ke_quotas_load(ke_ctx* ctx, const ke_quota_args* args, const ke_quota* quotas, int32_t n) {
  if (ctx) async_drain(ctx);
  if (!ctx || !args || n < 0 || n > KE_MAX_QUOTAS || (n > 0 && !quotas)) return fail(KE_ERR_INVALID, "ke_quotas_load arguments");
  if (args->n_hook_plugins) return fail(KE_ERR_UNSUPPORTED, "ElasticQuotaArgs.HookPlugins are not supported");
  if (args->enable_guarantee_usage) return fail(KE_ERR_UNSUPPORTED, "ElasticQuotaGuaranteeUsage is not supported");
  for (int r = 0; r < KE_NRES; r++)
    if (args->total[r] < 0) return fail(KE_ERR_INVALID, "ke_quota_args.total must be >= 0");
  std::vector<ke_quota> q(quotas, quotas + n);
  for (const ke_quota& x : q)
    for (int r = 0; r < KE_NRES; r++)
      if (x.max[r] < 0 || x.min[r] < 0 || x.shared_weight[r] < 0 || x.self_request[r] < 0 || x.used[r] < 0 ||
          x.non_preemptible_used[r] < 0)
        return fail(KE_ERR_INVALID, "ke_quota values must be >= 0");
  std::vector<int64_t> lim;
  std::vector<uint8_t> has;
  const int rc = quota_compute_limits(*args, q, lim, has);
  if (rc) return rc;
  Context& c = ctx->c;
  c.qargs = *args;
  c.quotas.swap(q);
  c.qlimit.swap(lim);
  c.qlimit_has.swap(has);
  c.quota_dirty = true;
  c.quota_on_device = false;
  return KE_OK;
}

int ke_quota_state(ke_ctx* ctx, int32_t q, int64_t* limit, uint8_t* limit_has, int64_t* used, int64_t* np_used) {
  if (ctx) async_drain(ctx);
  if (!ctx || q < 0 || q >= (int32_t)ctx->c.quotas.size()) return fail(KE_ERR_NOT_FOUND, "ke_quota_state: no such quota");
  const int rc = device_quota_sync(&ctx->c);
  if (rc) return rc;
  const ke_quota& x = ctx->c.quotas[q];
  for (int r = 0; r < KE_NRES; r++) {
    if (limit) limit[r] = ctx->c.qlimit[(size_t)q * KE_NRES + r];
    if (limit_has) limit_has[r] = ctx->c.qlimit_has[(size_t)q * KE_NRES + r];
    if (used) used[r] = x.used[r];
    if (np_used) np_used[r] = x.non_preemptible_used[r];
  }
  return KE_OK;
}

int ke_last_cpusets(ke_ctx* ctx, int32_t n, uint64_t* out) {
  if (!ctx || n < 0 || (n > 0 && !out)) return fail(KE_ERR_INVALID, "ke_last_cpusets arguments");
  const auto& a = ctx->c.last_cpusets;
  for (int64_t i = 0; i < (int64_t)n * 4; i++) out[i] = i < (int64_t)a.size() ? a[i] : 0;
  return KE_OK;
}

int ke_last_numa_allocations(ke_ctx* ctx, int32_t n, int64_t* out) {
  if (!ctx || n < 0 || (n > 0 && !out)) return fail(KE_ERR_INVALID, "ke_last_numa_allocations arguments");
  const auto& a = ctx->c.last_numa_alloc;
  constexpr int W = KE_MAX_NUMA * KE_NRES;
  for (int64_t i = 0; i < (int64_t)n * W; i++) out[i] = i < (int64_t)a.size() ? a[i] : 0;
  return KE_OK;
}

int ke_last_device_allocations(ke_ctx* ctx, int32_t n, uint64_t* minors) {
  if (!ctx || n < 0 || (n > 0 && !minors)) return fail(KE_ERR_INVALID, "ke_last_device_allocations arguments");
  const auto& a = ctx->c.last_dev_alloc;
  for (int32_t i = 0; i < n; i++) minors[i] = i < (int32_t)a.size() ? a[i] : 0;
  return KE_OK;
}

int ke_node_set_requested(ke_ctx* ctx, int32_t node, int64_t milli_cpu, int64_t memory) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.node.requested[KE_RES_CPU] = milli_cpu;
  ns.node.requested[KE_RES_MEMORY] = memory;
  ns.dirty = true;
  return KE_OK;
}

int ke_node_set_cpuset_allocated(ke_ctx* ctx, int32_t node, int64_t cpus) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.node.cpuset_allocated_cpus = cpus;
  ns.dirty = true;
  return KE_OK;
}

int ke_nodemetric_upsert(ke_ctx* ctx, int32_t node, const ke_node_metric* nm, int32_t n_pm, const ke_pod_metric* pm,
                         int32_t n_agg, const ke_aggregated_usage* agg) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  if (!nm || n_pm < 0 || n_agg < 0 || (n_pm && !pm) || (n_agg && !agg)) return fail(KE_ERR_INVALID, "nodemetric");
  NodeState& ns = ctx->c.nodes[node];
  ns.has_metric = true;
  ns.nm = *nm;
  ns.pm.assign(pm, pm + n_pm);
  ns.agg.assign(agg, agg + n_agg);
  ns.dirty = true;
  return KE_OK;
}

int ke_nodemetrics_load(ke_ctx* ctx, int32_t n, const ke_node_metric* nms, const int64_t* pm_offsets,
                        const ke_pod_metric* pod_metrics, const int64_t* agg_offsets, const ke_aggregated_usage* aggregated) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || (n > 0 && (!nms || !pm_offsets || !agg_offsets))) return fail(KE_ERR_INVALID, "nodemetrics_load");
  if (ctx) flush_mirror(ctx->c);
  for (int32_t i = 0; i < n; i++) {
    const int64_t p0 = pm_offsets[i], p1 = pm_offsets[i + 1], a0 = agg_offsets[i], a1 = agg_offsets[i + 1];
    if (p1 < p0 || a1 < a0) return fail(KE_ERR_INVALID, "offsets must be non-decreasing");
    int rc = ke_nodemetric_upsert(ctx, i, &nms[i], (int32_t)(p1 - p0), pod_metrics ? pod_metrics + p0 : nullptr,
                                  (int32_t)(a1 - a0), aggregated ? aggregated + a0 : nullptr);
    if (rc) return rc;
  }
  return KE_OK;
}

int ke_nodemetric_delete(ke_ctx* ctx, int32_t node) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  ns.has_metric = false;
  ns.nm = ke_node_metric{};
  ns.pm.clear();
  ns.agg.clear();
  ns.dirty = true;
  return KE_OK;
}

int ke_pod_assign(ke_ctx* ctx, int32_t node, const ke_pod* pod, int64_t timestamp_ns) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  if (!pod) return fail(KE_ERR_INVALID, "null pod");
  host_assign(ctx->c.cfg, ctx->c.nodes[node], *pod, timestamp_ns);
  return KE_OK;
}

int ke_pods_assign(ke_ctx* ctx, int32_t n, const int32_t* nodes, const ke_pod* pods, const int64_t* timestamps_ns) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || (n > 0 && (!nodes || !pods || !timestamps_ns))) return fail(KE_ERR_INVALID, "ke_pods_assign");
  if (ctx) flush_mirror(ctx->c);
  for (int32_t i = 0; i < n; i++) {
    int rc = check_node(ctx, nodes[i]);
    if (rc) return rc;
    host_assign(ctx->c.cfg, ctx->c.nodes[nodes[i]], pods[i], timestamps_ns[i]);
  }
  return KE_OK;
}

int ke_pod_unassign(ke_ctx* ctx, int32_t node, int64_t uid) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  NodeState& ns = ctx->c.nodes[node];
  for (size_t i = 0; i < ns.asg_uid.size(); i++) {
    if (ns.asg_uid[i] == uid) {
      ns.asg.erase(ns.asg.begin() + (long)i);
      ns.asg_uid.erase(ns.asg_uid.begin() + (long)i);
      ns.dirty = true;
      break;
    }
  }
  return KE_OK;
}

int ke_estimate_pod(ke_ctx* ctx, const ke_pod* pod, int64_t* est) {
  if (ctx) async_drain(ctx);
  if (!ctx || !pod || !est) return fail(KE_ERR_INVALID, "ke_estimate_pod arguments");
  uint8_t present[KE_NRES];
  estimate_pod(ctx->c.cfg.loadaware, *pod, est, present);
  for (int r = 0; r < KE_NRES; r++)
    if (!present[r]) est[r] = KE_ABSENT;
  return KE_OK;
}

int ke_eval(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns, uint8_t* status, uint8_t* reason,
            int16_t* la_score, int16_t* numa_score, int16_t* ds_score, int16_t* total, int32_t* best) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  if (ctx) flush_mirror(ctx->c);
  int rc = check_pods(pods, n_pods, &ctx->c);
  if (rc) return rc;
  rc = check_numa_deviceshare(ctx, pods, n_pods);
  if (rc) return rc;
  rc = check_cpuset(ctx, pods, n_pods);
  if (rc) return rc;
  rc = require_device(ctx);
  if (rc) return rc;
  return device_eval(&ctx->c, n_pods, pods, now_ns, status, reason, la_score, numa_score, ds_score, total, best);
}

static int schedule_sync(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns, int32_t* chosen, int32_t* score) {
  if (!ctx || (n_pods > 0 && !chosen)) return fail(KE_ERR_INVALID, "ke_schedule arguments");
  using clk = std::chrono::steady_clock;
  auto tp = clk::now();
  ctx->c.call_entry = tp;  // every pod of the call is dequeued now (ke_last_pod_latencies)
  // the staged ke_pod_reservations lists belong to this call, refused or not
  auto refuse = [&](int r) {
    ctx->c.match_off.clear();
    ctx->c.match_ids.clear();
    return r;
  };
  int rc = check_pods(pods, n_pods, &ctx->c, true);
  if (rc) return refuse(rc);
  rc = check_numa_deviceshare(ctx, pods, n_pods);
  if (rc) return refuse(rc);
  rc = check_cpuset(ctx, pods, n_pods);
  if (rc) return refuse(rc);
  for (int32_t p = 0; p < n_pods; p++)
    if (pods[p].quota < 0 || pods[p].quota > (int32_t)ctx->c.quotas.size())
      return refuse(fail(KE_ERR_INVALID, "ke_pod.quota outside the loaded ElasticQuota tree"));
  rc = check_matches(ctx->c, pods, n_pods);
  if (rc) return refuse(rc);
  rc = require_device(ctx);
  if (rc) return refuse(rc);
  ctx->c.host_ms[0] = std::chrono::duration<double, std::milli>(clk::now() - tp).count();
  Context& c = ctx->c;
  // ElasticQuota: a Reserve into the system / default quota (limit_is_max) with runtime quota on
  // shrinks totalResourceExceptSystemAndDefaultUsed (updateClusterTotalResourceNoLock,
  // group_quota_manager.go:268-271, 127-151), and every later pod sees runtime limits refreshed from it.
  // The queue is cut after each such pod; between the segments the host takes the device's used,
  // shrinks the total by the pod's masked request and recomputes the limits (uploaded by the next
  // segment).  Without such pods the queue is one segment.
  auto barrier = [&](int32_t p) {
    if (c.quotas.empty() || !c.qargs.enable_runtime_quota || pods[p].quota <= 0) return false;
    return c.quotas[(size_t)pods[p].quota - 1].limit_is_max != 0;
  };
  std::vector<uint64_t> all_dev, all_cs;
  std::vector<int8_t> all_vf;
  std::vector<int64_t> all_numa;
  std::vector<double> all_batch_ms, all_lat;
  double all_ms = 0;
  bool numa_out = false, multi = false;
  const int32_t off = c.cfg.global_node_offset;
  // A pod with matched reservations (KE_RSV_MATCHED with a non-empty list) is a segment of its own: its
  // rows carry its matched restore and k_rsv_pick adds the Reservation score (resv_prepare / resv_finish).
  std::vector<int32_t> moff, mids;
  moff.swap(c.match_off);  // consumed by this call
  mids.swap(c.match_ids);
  auto matched = [&](int32_t p) {
    return pods[p].reservation_matched == KE_RSV_AFFINITY ||
           (!moff.empty() && moff[(size_t)p + 1] > moff[(size_t)p]);
  };
  // A run of KE_RSV_IGNORED pods is a segment of its own: its rows carry every reservation's matched restore.
  // An ignored pod that may bind CPUs beside CPU-holding reservations is alone too (its trials read the state).
  auto ignored = [&](int32_t p) { return pods[p].reservation_matched == KE_RSV_IGNORED; };
  auto ign_views = [&](int32_t p) { return ignored(p) && resv_ignore_needs_views(c, pods[p], c.staged[(size_t)p].flags); };
  auto alone = [&](int32_t p) { return matched(p) || ign_views(p); };
  std::vector<int32_t> assumed((size_t)n_pods, 0);
  c.last_rsv_fused = c.last_rsv_fused_gated = 0;
  for (int32_t s0 = 0; s0 < n_pods || (n_pods == 0 && s0 == 0);) {
    int32_t s1 = s0;
    const bool ign = s0 < n_pods && ignored(s0);
    while (s1 < n_pods && !barrier(s1) && !alone(s1) && ignored(s1) == ign) s1++;
    // a barrier pod ends its segment; a matched one is alone
    if (s1 < n_pods && (s1 == s0 || (!alone(s1) && barrier(s1) && ignored(s1) == ign))) s1++;
    int32_t len = s1 - s0;
    const bool rsv = len == 1 && matched(s0);
    mirror_join(c);  // (the previous segment's host mirror thread: this one reads the node state)
    if (ign) resv_ignore_begin(c);
    if (ign && len == 1 && ign_views(s0)) {  // its trials on the current state, as the matched pods' below
      flush_mirror(c);
      resv_ignore_views(c, pods[s0]);
      if (!c.rsv_views.empty()) {
        rc = device_rsv_views(&c, pods[s0], now_ns, c.rsv_views, c.rsv_view_out);
        if (rc) return resv_ignore_end(c), rc;
      }
      if (!c.numa_views.empty()) {  // NUMA policies: the hints over tryAllocateIgnoreReservation (k_numa_views)
        rc = device_numa_views(&c, pods[s0], now_ns, c.numa_views, c.numa_view_out);
        if (rc) return resv_ignore_end(c), rc;
      }
      resv_ds_views(c, pods[s0], nullptr, 0);  // DeviceShare's ignore / own views (k_ds_views)
      if (!c.ds_views.empty()) {
        rc = device_ds_views(&c, pods[s0], now_ns, c.ds_views, c.ds_view_out);
        if (rc) return resv_ignore_end(c), rc;
      }
      resv_ignore_ovr(c);
      if (!c.numa_cs_views.empty()) {  // its cpuset and Score on the Filter's affinity
        rc = device_rsv_views(&c, pods[s0], now_ns, c.numa_cs_views, c.numa_cs_out);
        if (rc) return resv_ignore_end(c), rc;
        resv_numa_cs_apply(c);
      }
    }
    if (rsv) {
      const int32_t* ids = mids.data() + moff[(size_t)s0];
      const int32_t n_ids = moff[(size_t)s0 + 1] - moff[(size_t)s0];
      resv_views(c, pods[s0], ids, n_ids);  // allocate-from-reservation trials on the current state first
      if (!c.rsv_views.empty()) {
        rc = device_rsv_views(&c, pods[s0], now_ns, c.rsv_views, c.rsv_view_out);
        if (rc) return rc;
      }
      resv_ds_views(c, pods[s0], ids, n_ids);  // DeviceShare's trials, on the rows with the pod's matched restore
      if (!c.ds_views.empty()) {
        rc = device_ds_views(&c, pods[s0], now_ns, c.ds_views, c.ds_view_out);
        if (rc) {
          for (const DsView& v : c.ds_views) resv_node_restore(c, v.node);
          c.ds_views.clear();
          return rc;
        }
      }
      resv_numa_views(c, pods[s0], ids, n_ids);  // NodeNUMAResource's hints over the trials (NUMA policies)
      if (!c.numa_views.empty()) {
        rc = device_numa_views(&c, pods[s0], now_ns, c.numa_views, c.numa_view_out);
        if (rc) {
          for (const NumaRsvView& v : c.numa_views) resv_node_restore(c, v.node);
          for (const DsView& v : c.ds_views) resv_node_restore(c, v.node);
          c.numa_views.clear();
          c.ds_views.clear();
          return rc;
        }
      }
      rc = resv_prepare(c, pods[s0], ids, n_ids, pods[s0].reservation_matched == KE_RSV_AFFINITY);
      if (rc) return rc;
      if (!c.numa_cs_views.empty()) {  // a binding pod's cpuset of the nominated reservation (NUMA policies)
        rc = device_rsv_views(&c, pods[s0], now_ns, c.numa_cs_views, c.numa_cs_out);
        if (rc) {
          int32_t dummy = 0;
          resv_finish(c, -1, pods[s0], &dummy);
          return rc;
        }
        resv_numa_cs_apply(c);
      }
    }
    // a device failure leaves the pods of earlier segments Reserved on the device and the context's state
    // undefined (KE_ERR_DEVICE: rebuild the context); the matched-restore state is still undone so the
    // reservation's capacity does not stay visible to later calls
    auto undo_rsv = [&]() {
      int32_t dummy = 0;
      if (rsv) resv_finish(c, -1, pods[s0], &dummy);
      if (ign) resv_ignore_end(c);
    };
    // A plain segment followed by a matched pod without allocate-from-reservation views or decisions (DESIGN.md §4k,
    // "fused"): the pod's nomination and rows are taken now, on the state before the segment, and it runs last in the
    // segment's call -- k_rsv_check gates it on the device when a plain pod of the segment took a node of its
    // reservations, and the host then runs it as a segment of its own.
    bool fuse = kFuseMatched && !ign && !rsv && len >= 1 && s1 < n_pods && pods[s1].reservation_matched == KE_RSV_MATCHED &&
                matched(s1) && c.quotas.empty() && !device_sharded(&c) && (size_t)s1 < c.staged.size() &&
                !(c.staged[(size_t)s1].flags & (PF_CPUSET | PF_DS | PF_DS_HINT));
    if (fuse) {
      rc = device_refresh(&c, now_ns, false);  // the segment's rows (no host wait)
      if (rc) return rc;
      const int32_t* ids = mids.data() + moff[(size_t)s1];
      const int32_t n_ids = moff[(size_t)s1 + 1] - moff[(size_t)s1];
      resv_views(c, pods[s1], ids, n_ids);
      fuse = c.rsv_views.empty();
      if (fuse) {
        resv_ds_views(c, pods[s1], ids, n_ids);
        fuse = c.ds_views.empty();
      }
      if (fuse) {
        resv_numa_views(c, pods[s1], ids, n_ids);
        fuse = c.numa_views.empty();
      }
      if (!fuse) {  // its own segment after all: the views' rows back as they were
        for (const DsView& v : c.ds_views) resv_node_restore(c, v.node);
        for (const NumaRsvView& v : c.numa_views) resv_node_restore(c, v.node);
        int32_t dummy = 0;
        resv_finish(c, -1, pods[s1], &dummy);
      } else {
        rc = resv_prepare(c, pods[s1], ids, n_ids, false);
        if (rc) return rc;
        if (!c.rsv_ovr.empty() || !c.numa_cs_views.empty()) {
          int32_t dummy = 0;
          resv_finish(c, -1, pods[s1], &dummy);
          fuse = false;
        }
      }
    }
    c.rsv_fused = fuse;
    rc = device_schedule(&c, fuse ? len + 1 : len, pods + s0, now_ns, chosen + (n_pods ? s0 : 0), score ? score + s0 : nullptr);
    c.rsv_fused = false;
    if (rc && fuse) {
      int32_t dummy = 0;
      resv_finish(c, -1, pods[s1], &dummy);
    }
    if (rc) return undo_rsv(), rc;
    if (ign) resv_ignore_end(c);
    if (fuse && device_rsv_gate(&c)) {
      // a plain pod took a node of the fused pod's reservations: the pod placed nothing; its nomination and rows are
      // undone and it runs next as a segment of its own (the call's per-pod outputs: the segment's only)
      int32_t dummy = 0;
      resv_finish(c, -1, pods[s1], &dummy);
      chosen[s1] = -1;
      auto cut = [&](auto& v, size_t per) {
        if (v.size() > per * (size_t)len) v.resize(per * (size_t)len);
      };
      cut(c.last_dev_alloc, 1);
      cut(c.last_cpusets, 4);
      cut(c.last_vf, 2 * KE_MAX_MINORS);
      cut(c.last_numa_alloc, (size_t)KE_MAX_NUMA * KE_NRES);
      cut(c.last_pod_lat, 1);
      if (!c.last_batch_ms.empty()) c.last_batch_ms.pop_back();
      c.last_rsv_fused_gated++;
      fuse = false;
    } else if (fuse) {  // the Reservation plugin's outcome of the fused pod, as for a matched segment below
      const int32_t local = chosen[s1] < 0 ? -1 : chosen[s1] - off;
      int32_t pick[4] = {local, 0, 0, -1};
      if (!c.rsv_pairs.empty()) rc = device_rsv_result(&c, pick);
      if (!rc && local >= 0 && local != pick[0]) rc = fail(KE_ERR_DEVICE, "k_rsv_pick winner differs from the placement");
      if (rc) {
        int32_t dummy = 0;
        resv_finish(c, -1, pods[s1], &dummy);
        return rc;
      }
      if (local >= 0 && score) score[s1] = (int32_t)((int64_t)score[s1] + c.cfg.weight_reservation * (int64_t)pick[1]);
      const size_t L = (size_t)len;
      resv_finish(c, local, pods[s1], &assumed[(size_t)s1],
                  c.last_cpusets.size() >= 4 * (L + 1) ? c.last_cpusets.data() + 4 * L : nullptr,
                  c.last_numa_alloc.size() >= (L + 1) * KE_MAX_NUMA * KE_NRES ? c.last_numa_alloc.data() + L * KE_MAX_NUMA * KE_NRES : nullptr,
                  c.last_dev_alloc.size() > L ? c.last_dev_alloc[L] : 0);
      c.last_rsv_fused++;
      len++;
      s1++;
    }
    if (rsv) {
      const int32_t local = chosen[s0] < 0 ? -1 : chosen[s0] - off;
      int32_t pick[4] = {local, 0, 0, -1};  // no usable matched reservation: no Reservation score
      if (!c.rsv_pairs.empty() || c.rsv_affinity) rc = device_rsv_result(&c, pick);
      if (rc) return undo_rsv(), rc;
      if (local >= 0 && local != pick[0])
        return undo_rsv(), fail(KE_ERR_DEVICE, "k_rsv_pick winner differs from the placement");
      if (local >= 0 && score) score[s0] = (int32_t)((int64_t)score[s0] + c.cfg.weight_reservation * (int64_t)pick[1]);
      resv_finish(c, local, pods[s0], &assumed[(size_t)s0], c.last_cpusets.size() >= 4 ? c.last_cpusets.data() : nullptr,
                  c.last_numa_alloc.size() >= (size_t)(KE_MAX_NUMA * KE_NRES) ? c.last_numa_alloc.data() : nullptr,
                  c.last_dev_alloc.empty() ? 0 : c.last_dev_alloc[0]);
    }
    if (n_pods == 0) break;
    tp = clk::now();
    // Host mirror of the Reserves the device already applied to its rows: keep the object state
    // (assign cache, NodeInfo.Requested) in step so later re-derivations include these pods.
    c.pending.reserve(c.pending.size() + (size_t)len);
    const int64_t base = c.pending_base;  // device_schedule copied pods[s0 .. s1) there during its wait
    for (int32_t i = 0; i < len; i++) {
      const int32_t p = s0 + i;
      const int32_t node = chosen[p] - off;
      if (chosen[p] < 0 || node < 0 || node >= c.n_nodes) continue;
      // LoadAware assign + NodeInfo.Requested: deferred (flush_mirror), the device rows carry them
      c.pending.push_back({node, now_ns, base + i});
      // the allocations (read back only when the call's batches could make them): the node's state is touched
      // only for a pod that has one
      const bool dev = i < (int32_t)c.last_dev_alloc.size() && c.last_dev_alloc[i];
      const bool numa = (int64_t)c.last_numa_alloc.size() >= (int64_t)(i + 1) * KE_MAX_NUMA * KE_NRES;
      const uint64_t* cs = (int64_t)c.last_cpusets.size() >= (int64_t)(i + 1) * 4 ? &c.last_cpusets[(size_t)i * 4] : nullptr;
      const bool cpus = cs && (cs[0] | cs[1] | cs[2] | cs[3]);
      if (!dev && !numa && !cpus) continue;
      mirror_join(c);  // (the earlier calls' mirror may still be running on its thread)
      NodeState& ns = c.nodes[node];
      const bool was_dirty = ns.dirty;
      if (dev)
        host_ds_reserve(c.cfg, ns, make_dev_pod(c.cfg, pods[p], pod_hints(c, pods[p]), &c.tmpl), c.last_dev_alloc[i],
                        (int64_t)c.last_vf.size() >= (int64_t)(i + 1) * 2 * KE_MAX_MINORS ? &c.last_vf[(size_t)i * 2 * KE_MAX_MINORS] : nullptr);
      if (numa) host_numa_reserve(ns, &c.last_numa_alloc[(size_t)i * KE_MAX_NUMA * KE_NRES]);
      ns.dirty = was_dirty;  // the device rows already carry these Reserves
      // cpuset Reserve: the CPU table (the device one is patched too) and the zones' NUMA status (not
      // patched on the device: re-derived from this mirror)
      if (cpus) host_cpuset_reserve(ns, make_dev_pod(c.cfg, pods[p]), cs);
    }
    c.host_ms[7] += std::chrono::duration<double, std::milli>(clk::now() - tp).count();
    const bool whole = s0 == 0 && s1 == n_pods;  // one segment: the last_* outputs are already whole
    if (!whole) {
      c.last_dev_alloc.resize((size_t)len, 0);  // (a segment without DeviceShare batches reads none back)
      c.last_cpusets.resize((size_t)len * 4, 0);
      all_dev.insert(all_dev.end(), c.last_dev_alloc.begin(), c.last_dev_alloc.end());
      if (c.last_vf.empty()) all_vf.resize(all_vf.size() + (size_t)len * 2 * KE_MAX_MINORS, -1);
      else all_vf.insert(all_vf.end(), c.last_vf.begin(), c.last_vf.end());
      all_cs.insert(all_cs.end(), c.last_cpusets.begin(), c.last_cpusets.end());
      numa_out = numa_out || !c.last_numa_alloc.empty();
      if (c.last_numa_alloc.empty()) all_numa.resize(all_numa.size() + (size_t)len * KE_MAX_NUMA * KE_NRES, 0);
      else all_numa.insert(all_numa.end(), c.last_numa_alloc.begin(), c.last_numa_alloc.end());
      all_batch_ms.insert(all_batch_ms.end(), c.last_batch_ms.begin(), c.last_batch_ms.end());
      all_lat.insert(all_lat.end(), c.last_pod_lat.begin(), c.last_pod_lat.end());
      all_ms += c.last_total_ms;
    }
    // the placed system / default pod (also when it ends the only segment): refresh the runtime
    if (barrier(s1 - 1) && chosen[s1 - 1] >= 0) {
      rc = device_quota_sync(&c);
      if (rc) return rc;
      const ke_quota& q = c.quotas[(size_t)pods[s1 - 1].quota - 1];
      c.qargs.total[0] -= q.has_max[0] ? pods[s1 - 1].requests[KE_RES_CPU] : 0;
      c.qargs.total[1] -= q.has_max[1] ? pods[s1 - 1].requests[KE_RES_MEMORY] : 0;
      rc = quota_compute_limits(c.qargs, c.quotas, c.qlimit, c.qlimit_has);
      if (rc) return rc;
      c.quota_dirty = true;
    }
    if (whole) break;
    s0 = s1;
    multi = true;
  }
  if (multi) {
    c.last_dev_alloc.swap(all_dev);
    c.last_vf.swap(all_vf);
    c.last_cpusets.swap(all_cs);
    if (numa_out) c.last_numa_alloc.swap(all_numa);
    else c.last_numa_alloc.clear();
    c.last_batch_ms.swap(all_batch_ms);
    c.last_pod_lat.swap(all_lat);
    c.last_total_ms = all_ms;
  }
  // release records of this call (ke_last_allocations / ke_unreserve)
  c.last_chosen.assign(chosen, chosen + n_pods);
  c.last_uid.resize((size_t)n_pods);
  c.last_quota.resize((size_t)n_pods);
  c.last_resv.swap(assumed);
  for (int32_t p = 0; p < n_pods; p++) {
    c.last_uid[(size_t)p] = pods[p].uid;
    c.last_quota[(size_t)p] = chosen[p] >= 0 && pods[p].quota > 0 && !c.quotas.empty();
  }
  return KE_OK;
}

int ke_schedule(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns, int32_t* chosen, int32_t* score) {
  if (ctx) async_drain(ctx);
  return schedule_sync(ctx, n_pods, pods, now_ns, chosen, score);
}

int ke_schedule_submit(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns, int64_t* ticket) {
  if (!ctx || n_pods < 0 || (n_pods > 0 && !pods) || !ticket) return fail(KE_ERR_INVALID, "ke_schedule_submit arguments");
  using clk = std::chrono::steady_clock;
  Context& c = ctx->c;
  int in_flight = 0;
  for (const AsyncCall& a : ctx->async) in_flight += a.fin != nullptr;
  // at most one call in flight behind which this one is enqueued (two sets of call buffers)
  for (AsyncCall& a : ctx->async)
    if (in_flight >= 2 && a.fin) async_finish(ctx, a), in_flight--;
  // a plain queue: no reservation-matched, NUMA-policy or quota pod, no staged reservation lists
  bool plain = c.dev && n_pods > 0 && c.match_off.empty() && c.quotas.empty() && !c.numa_enabled;
  for (int32_t p = 0; p < n_pods && plain; p++)
    plain = pods[p].reservation_matched == KE_RSV_NONE && pods[p].numa_topology_policy == KE_NUMA_POLICY_NONE &&
            pods[p].quota == 0;
  if (plain) {
    const auto tp = clk::now();
    int rc = check_pods(pods, n_pods, &c);
    if (rc) return rc;
    rc = check_cpuset(ctx, pods, n_pods);  // (stages the pods' records)
    if (rc) return rc;
    plain = device_async_ok(&c, n_pods);
    if (plain && in_flight > 0 && device_refresh_pending(&c, now_ns)) {
      async_drain(ctx);  // rows to derive from the host state: it must carry the Reserves of the calls in flight
      in_flight = 0;
    }
    if (plain) {
      c.call_entry = tp;
      c.host_ms[0] = std::chrono::duration<double, std::milli>(clk::now() - tp).count();
      if (in_flight > 0) device_swap_call_buffers(&c);  // (the call in flight keeps its own)
      AsyncCall a;
      a.ticket = ctx->next_ticket++;
      a.n = n_pods;
      a.pods = pods;
      a.now = now_ns;
      a.device = true;
      rc = device_schedule_enqueue(&c, n_pods, pods, now_ns, true, &a.fin);
      if (rc) {
        // the call in flight keeps the buffers its completion captured: swap back, and let no partly enqueued
        // launch of this call outlive the error
        if (in_flight > 0) device_swap_call_buffers(&c);
        device_quiesce(&c);
        return rc;
      }
      *ticket = a.ticket;
      ctx->async.push_back(std::move(a));
      return KE_OK;
    }
  }
  // anything else runs now, after every call in flight
  async_drain(ctx);
  AsyncCall a;
  a.ticket = ctx->next_ticket++;
  a.n = n_pods;
  a.pods = pods;
  a.now = now_ns;
  a.chosen.assign((size_t)n_pods, -1);
  a.score.assign((size_t)n_pods, 0);
  const int rc = schedule_sync(ctx, n_pods, pods, now_ns, a.chosen.data(), a.score.data());
  if (rc) return rc;
  a.rec.save(c);
  *ticket = a.ticket;
  ctx->async.push_back(std::move(a));
  return KE_OK;
}

int ke_schedule_wait(ke_ctx* ctx, int64_t ticket, int32_t* chosen, int32_t* score) {
  if (!ctx) return fail(KE_ERR_INVALID, "ke_schedule_wait arguments");
  size_t i = 0;
  while (i < ctx->async.size() && ctx->async[i].ticket != ticket) i++;
  if (i == ctx->async.size()) return fail(KE_ERR_NOT_FOUND, "ke_schedule_wait: no such submitted call");
  if (ctx->async[i].n > 0 && !chosen) return fail(KE_ERR_INVALID, "ke_schedule_wait arguments");
  for (size_t j = 0; j <= i; j++) async_finish(ctx, ctx->async[j]);  // (in submission order)
  AsyncCall a = std::move(ctx->async[i]);
  ctx->async.erase(ctx->async.begin() + (long)i);
  if (a.rc) return fail(a.rc, a.msg);
  std::copy(a.chosen.begin(), a.chosen.end(), chosen);
  if (score) std::copy(a.score.begin(), a.score.end(), score);
  // release records of this call (ke_last_allocations / ke_unreserve): the last collected call, device-enqueued
  // or run at once alike
  a.rec.restore(ctx->c);
  return KE_OK;
}

// the release record of position p of the last ke_schedule
static ke_pod_allocation last_allocation(const Context& c, int32_t p) {
  ke_pod_allocation a{};
  memset(a.vf_rank, -1, sizeof a.vf_rank);
  a.node = p < (int32_t)c.last_chosen.size() ? c.last_chosen[(size_t)p] : -1;
  if (a.node < 0) return a;
  a.reservation = p < (int32_t)c.last_resv.size() ? c.last_resv[(size_t)p] : 0;
  a.reservation_generation = c.resv_gen;
  a.reservation_uid = a.reservation > 0 ? c.resv[(size_t)a.reservation - 1].uid : 0;
  a.quota_assigned = c.last_quota[(size_t)p];
  constexpr int W = KE_MAX_NUMA * KE_NRES;
  for (int q = 0; q < 4; q++)
    a.cpuset[q] = (int64_t)c.last_cpusets.size() >= (int64_t)(p + 1) * 4 ? c.last_cpusets[(size_t)p * 4 + q] : 0;
  for (int w = 0; w < W; w++)
    a.numa[w] = (int64_t)c.last_numa_alloc.size() >= (int64_t)(p + 1) * W ? c.last_numa_alloc[(size_t)p * W + w] : 0;
  a.device_minors = p < (int32_t)c.last_dev_alloc.size() ? c.last_dev_alloc[(size_t)p] : 0;
  for (int k = 0; k < 2 * KE_MAX_MINORS; k++)
    a.vf_rank[k / KE_MAX_MINORS][k % KE_MAX_MINORS] =
        (int64_t)c.last_vf.size() >= (int64_t)(p + 1) * 2 * KE_MAX_MINORS ? c.last_vf[(size_t)p * 2 * KE_MAX_MINORS + k] : (int8_t)-1;
  return a;
}

int ke_last_allocations(ke_ctx* ctx, int32_t n, ke_pod_allocation* out) {
  if (!ctx || n < 0 || (n > 0 && !out)) return fail(KE_ERR_INVALID, "ke_last_allocations arguments");
  for (int32_t p = 0; p < n; p++) out[p] = last_allocation(ctx->c, p);
  return KE_OK;
}

int ke_pod_release(ke_ctx* ctx, const ke_pod* pod, const ke_pod_allocation* alloc, int32_t mode) {
  if (ctx) async_drain(ctx);
  if (!ctx || !pod || !alloc) return fail(KE_ERR_INVALID, "ke_pod_release arguments");
  if (mode != KE_RELEASE_UNRESERVE && mode != KE_RELEASE_DELETE) return fail(KE_ERR_INVALID, "ke_pod_release mode");
  int rc = validate_pod(*pod);
  if (rc) return rc;
  Context& c = ctx->c;
  rc = validate_pod_hints(c, *pod);
  if (rc) return rc;
  flush_mirror(c);  // the pod's own deferred Reserve mirror first
  if (pod->quota < 0 || pod->quota > (int32_t)c.quotas.size())
    return fail(KE_ERR_INVALID, "ke_pod.quota outside the loaded ElasticQuota tree");
  const int32_t node = alloc->node < 0 ? -1 : alloc->node - c.cfg.global_node_offset;
  if (node >= c.cfg.node_capacity) return fail(KE_ERR_NOT_FOUND, "ke_pod_release: node index out of range");
  // the reservation the pod was assumed into: by uid (the set may have been reloaded since), else by an index of
  // the current set
  int32_t ridx = -1;
  if (alloc->reservation > 0 && alloc->reservation_uid != 0) {
    for (size_t i = 0; i < c.resv.size() && ridx < 0; i++)
      if (c.resv[i].uid == alloc->reservation_uid) ridx = (int32_t)i;
  } else if (alloc->reservation > 0) {
    if (alloc->reservation > (int32_t)c.resv.size()) return fail(KE_ERR_NOT_FOUND, "ke_pod_release: reservation index");
    if (alloc->reservation_generation != c.resv_gen)
      return fail(KE_ERR_INVALID, "ke_pod_release: a reservation index of an earlier reservation set (no uid)");
    ridx = alloc->reservation - 1;
  } else if (alloc->reservation < 0) {
    return fail(KE_ERR_NOT_FOUND, "ke_pod_release: reservation index");
  }
  if (node >= 0 && c.nodes[(size_t)node].known)  // (also a deleted node: its caches keep the pod until released)
    host_release_node(c.cfg, c.ext_enabled, c.nodes[(size_t)node], *pod, *alloc, pod_hints(c, *pod));
  if (node >= 0 && ridx >= 0) resv_forget(c, ridx, *pod, alloc);
  const bool assigned = alloc->node >= 0 && alloc->quota_assigned;
  if (pod->quota > 0 && (assigned || mode == KE_RELEASE_DELETE)) {
    if (c.dev) {
      rc = device_quota_sync(&c);  // the device holds the current used after a ke_schedule
      if (rc) return rc;
    }
    rc = host_quota_release(c, *pod, assigned, mode == KE_RELEASE_DELETE);
    if (rc) return rc;
  }
  return KE_OK;
}

int ke_unreserve(ke_ctx* ctx, const ke_pod* pod, int32_t queue_pos) {
  if (ctx) async_drain(ctx);
  if (!ctx || !pod) return fail(KE_ERR_INVALID, "ke_unreserve arguments");
  Context& c = ctx->c;
  if (queue_pos < 0 || queue_pos >= (int32_t)c.last_chosen.size())
    return fail(KE_ERR_NOT_FOUND, "ke_unreserve: no such position in the last ke_schedule");
  if (c.last_uid[(size_t)queue_pos] != pod->uid) return fail(KE_ERR_INVALID, "ke_unreserve: pod uid differs from the queue's");
  if (c.last_chosen[(size_t)queue_pos] < 0) return KE_OK;  // not placed, or already unreserved
  const ke_pod_allocation a = last_allocation(c, queue_pos);
  const int rc = ke_pod_release(ctx, pod, &a, KE_RELEASE_UNRESERVE);
  if (rc) return rc;
  c.last_chosen[(size_t)queue_pos] = -1;
  return KE_OK;
}

int ke_last_pod_latencies(ke_ctx* ctx, int32_t n, double* ms) {
  if (!ctx || n < 0 || (n > 0 && !ms)) return fail(KE_ERR_INVALID, "ke_last_pod_latencies arguments");
  const auto& v = ctx->c.last_pod_lat;
  for (int32_t i = 0; i < n; i++) ms[i] = i < (int32_t)v.size() ? v[(size_t)i] : 0.0;
  return KE_OK;
}

int ke_last_host_stats(ke_ctx* ctx, double* ms8) {
  if (!ctx || !ms8) return fail(KE_ERR_INVALID, "ke_last_host_stats arguments");
  for (int i = 0; i < 8; i++) ms8[i] = ctx->c.host_ms[i];
  return KE_OK;
}

int ke_last_schedule_stats(ke_ctx* ctx, double* total_ms, int32_t* n_batches, double* batch_ms, int32_t batch_ms_cap) {
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  if (total_ms) *total_ms = ctx->c.last_total_ms;
  if (n_batches) *n_batches = (int32_t)ctx->c.last_batch_ms.size();
  if (batch_ms) {
    const int32_t n = std::min<int32_t>(batch_ms_cap, (int32_t)ctx->c.last_batch_ms.size());
    for (int32_t i = 0; i < n; i++) batch_ms[i] = ctx->c.last_batch_ms[i];
  }
  return KE_OK;
}

int ke_set_profiling(ke_ctx* ctx, int32_t sample_every) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  int rc = require_device(ctx);
  if (rc) return rc;
  return device_set_profiling(&ctx->c, sample_every);
}

int ke_last_kernel_stats(ke_ctx* ctx, double* eval_ms, double* select_ms, double* resolve_ms, int32_t* samples) {
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  if (eval_ms) *eval_ms = ctx->c.kstat_eval_ms;
  if (select_ms) *select_ms = ctx->c.kstat_select_ms;
  if (resolve_ms) *resolve_ms = ctx->c.kstat_resolve_ms;
  if (samples) *samples = ctx->c.kstat_samples;
  return KE_OK;
}

int ke_last_kernel_stats_ex(ke_ctx* ctx, double* ms4 /* [8] */, int32_t* samples, int32_t* pipelined_batches) {
  if (!ctx || !ms4) return fail(KE_ERR_INVALID, "ke_last_kernel_stats_ex arguments");
  ms4[0] = ctx->c.kstat_eval_ms;
  ms4[1] = ctx->c.kstat_select_ms;
  ms4[2] = ctx->c.kstat_fixup_ms;
  ms4[3] = ctx->c.kstat_resolve_ms;
  if (samples) *samples = ctx->c.kstat_samples;
  if (pipelined_batches) *pipelined_batches = ctx->c.last_pipelined;
  ms4[4] = ctx->c.last_enqueue_ms;
  ms4[5] = ctx->c.kstat_handoff_ms;
  ms4[6] = ctx->c.kstat_rows_fetched;
  ms4[7] = ctx->c.kstat_rows_changed;
  return KE_OK;
}

int ke_debug_replay_phases(ke_ctx* ctx, double* cyc8) {
  if (ctx) async_drain(ctx);
  if (!ctx || !cyc8) return fail(KE_ERR_INVALID, "ke_debug_replay_phases arguments");
  int rc = require_device(ctx);
  if (rc) return rc;
  return device_replay_phases(&ctx->c, 0, cyc8);
}

int ke_debug_kernel_phases(ke_ctx* ctx, int32_t kernel, double* cyc8) {
  if (ctx) async_drain(ctx);
  if (!ctx || !cyc8 || kernel < 0 || kernel > 3) return fail(KE_ERR_INVALID, "ke_debug_kernel_phases arguments");
  int rc = require_device(ctx);
  if (rc) return rc;
  return device_replay_phases(&ctx->c, kernel, cyc8);
}

int ke_debug_spec_failed(ke_ctx* ctx, double* per_batch) {
  if (!ctx || !per_batch) return fail(KE_ERR_INVALID, "ke_debug_spec_failed arguments");
  *per_batch = ctx->c.kstat_spec_failed;
  return KE_OK;
}

int ke_debug_check_records(ke_ctx* ctx, int64_t now_ns, int64_t* mismatched_nodes) {
  if (ctx) async_drain(ctx);
  if (!ctx || !mismatched_nodes) return fail(KE_ERR_INVALID, "ke_debug_check_records arguments");
  flush_mirror(ctx->c);
  int rc = require_device(ctx);
  if (rc) return rc;
  return device_check_records(&ctx->c, now_ns, mismatched_nodes);
}

int ke_set_pipeline(ke_ctx* ctx, int32_t on) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  int rc = require_device(ctx);
  if (rc) return rc;
  return device_set_pipeline(&ctx->c, on);
}

int ke_last_resolve_split(ke_ctx* ctx, double* prologue_ms, double* replay_ms) {
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  if (prologue_ms) *prologue_ms = ctx->c.kstat_resolve_prologue_ms;
  if (replay_ms) *replay_ms = ctx->c.kstat_resolve_loop_ms;
  return KE_OK;
}

int ke_debug_numa_deferred(ke_ctx* ctx, int64_t* n) {
  if (!ctx || !n) return fail(KE_ERR_INVALID, "ke_debug_numa_deferred arguments");
  *n = ctx->c.kstat_numa_deferred;
  return KE_OK;
}

int ke_debug_resolve_phases(ke_ctx* ctx, double* phases6) {
  if (!ctx || !phases6) return fail(KE_ERR_INVALID, "ke_debug_resolve_phases arguments");
  for (int i = 0; i < 6; i++) phases6[i] = ctx->c.kstat_resolve_phase_ms[i];
  return KE_OK;
}

int ke_debug_resolve_subphases(ke_ctx* ctx, double* sub5) {
  if (!ctx || !sub5) return fail(KE_ERR_INVALID, "ke_debug_resolve_subphases arguments");
  for (int i = 0; i < 5; i++) sub5[i] = ctx->c.kstat_resolve_sub_ms[i];
  return KE_OK;
}

int ke_debug_resolve_wave1(ke_ctx* ctx, double* w4) {
  if (!ctx || !w4) return fail(KE_ERR_INVALID, "ke_debug_resolve_wave1 arguments");
  for (int i = 0; i < 4; i++) w4[i] = ctx->c.kstat_resolve_wave1_ms[i];
  return KE_OK;
}

int ke_bench_eval_kernel(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns, int32_t iters,
                         double* avg_ms) {
  if (ctx) async_drain(ctx);
  if (!ctx || !avg_ms) return fail(KE_ERR_INVALID, "ke_bench_eval_kernel arguments");
  if (ctx) flush_mirror(ctx->c);
  int rc = check_pods(pods, n_pods);
  if (rc) return rc;
  rc = require_device(ctx);
  if (rc) return rc;
  return device_bench_eval(&ctx->c, n_pods, pods, now_ns, iters, avg_ms);
}

int ke_comm_unique_id(uint8_t* id, int32_t id_bytes) {
  if (!id || id_bytes < KE_COMM_ID_BYTES) return fail(KE_ERR_INVALID, "ke_comm_unique_id: need a 128-byte buffer");
  if (!device_available()) return fail(KE_ERR_NO_DEVICE, "ke_comm_unique_id: no HIP device");
  return device_comm_unique_id(id);
}

int ke_shard_init(ke_ctx* ctx, int32_t rank, int32_t world, const uint8_t* id) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  int rc = require_device(ctx);
  if (rc) return rc;
  return device_shard_init(&ctx->c, rank, world, id);
}

int ke_shard_init_host(ke_ctx* ctx, int32_t rank, int32_t world, ke_host_collective fn, void* user) {
  if (ctx) async_drain(ctx);
  if (!ctx) return fail(KE_ERR_INVALID, "null context");
  int rc = require_device(ctx);
  if (rc) return rc;
  return device_shard_init_host(&ctx->c, rank, world, fn, user);
}

int ke_shard_range(ke_ctx* ctx, int32_t* lo, int32_t* hi) {
  if (ctx) async_drain(ctx);
  if (!ctx || !lo || !hi) return fail(KE_ERR_INVALID, "ke_shard_range arguments");
  int rc = require_device(ctx);
  if (rc) return rc;
  int l = 0, h = 0;
  rc = device_shard_range(&ctx->c, &l, &h);
  *lo = l;
  *hi = h;
  return rc;
}

int ke_debug_node_state(ke_ctx* ctx, int32_t node, ke_node* out, int32_t cpu_cap, ke_cpu* cpus, int32_t* n_cpus,
                        int32_t zone_cap, ke_numa_zone* zones, int32_t* n_zones, int32_t dev_cap, ke_device* devs,
                        int32_t* n_devs) {
  if (ctx) async_drain(ctx);
  int rc = check_node(ctx, node);
  if (ctx) flush_mirror(ctx->c);
  if (rc) return rc;
  const NodeState& ns = ctx->c.nodes[(size_t)node];
  if (out) *out = ns.node;
  if (n_cpus) *n_cpus = (int32_t)ns.cpus.size();
  for (int32_t i = 0; cpus && i < cpu_cap && i < (int32_t)ns.cpus.size(); i++) cpus[i] = ns.cpus[(size_t)i];
  if (n_zones) *n_zones = (int32_t)ns.zones.size();
  for (int32_t i = 0; zones && i < zone_cap && i < (int32_t)ns.zones.size(); i++) zones[i] = ns.zones[(size_t)i];
  if (n_devs) *n_devs = (int32_t)ns.devs.size();
  for (int32_t i = 0; devs && i < dev_cap && i < (int32_t)ns.devs.size(); i++) devs[i] = ns.devs[(size_t)i];
  return KE_OK;
}

int64_t ke_debug_usage_bound(int64_t total, int64_t thr) { return total > 0 ? max_used_within(total, thr) : 0; }

int ke_debug_rows(ke_ctx* ctx, int32_t n, int64_t now_ns, void* device_rows, void* host_rows) {
  if (ctx) async_drain(ctx);
  if (!ctx || n < 0 || n > ctx->c.n_nodes) return fail(KE_ERR_INVALID, "ke_debug_rows arguments");
  if (ctx) flush_mirror(ctx->c);
  if (device_rows) {
    int rc = require_device(ctx);
    if (rc) return rc;
    rc = device_debug_rows(&ctx->c, n, (Row*)device_rows);
    if (rc) return rc;
  }
  if (host_rows) {
    Row* out = (Row*)host_rows;
    for (int32_t i = 0; i < n; i++) {
      int64_t vu;
      derive_row(ctx->c.cfg, ctx->c.nodes[i], now_ns, &out[i], &vu);
    }
  }
  return KE_OK;
}

}  // extern "C"
