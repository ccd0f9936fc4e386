// ke_host.h — host side of the evaluator: the informer-fed object state (what the reference keeps in
// its listers, podAssignCache and NodeInfo snapshot) and its folding into GPU rows.
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/koord_eval.h"
#include "ke_types.h"

namespace ke {

// One podAssignCache entry (pkg/scheduler/plugins/loadaware/pod_assign_cache.go:45-49).
// podAssignCache's podAssignInfo (pod_assign_cache.go:41-47): the pod fields estimatedAssignedPodUsed reads
struct AssignedPod {
  struct {
    int64_t pod_key;
    int64_t custom_seconds_after_scheduled, custom_seconds_after_initialized, initialized_transition_ns;
    int32_t priority_class;
    uint8_t has_initialized;
  } pod;
  int64_t ts;
  int64_t est[KE_NRES];
  uint8_t est_present[KE_NRES];
  bool has_est;
};

// A node's "row must be re-derived" flag.  Setting it bumps a process-wide epoch, so device_refresh can skip its
// scan over every node when no flag was set since it last cleaned them all (conservative across contexts), and
// a bound flag (its context's nodes) appends its node to the context's dirty list on a clean -> dirty change, so
// the refresh can visit only those nodes while no row has expired.
extern std::atomic<uint64_t> g_dirty_epoch;
struct DirtyFlag {
  bool v = true;
  int32_t idx = -1;
  std::vector<int32_t>* list = nullptr;
  DirtyFlag() { g_dirty_epoch.fetch_add(1, std::memory_order_relaxed); }  // a new node starts dirty
  // a copy keeps the binding: Context::nodes elements moved by a reallocation still feed their context's dirty
  // list under the same node index (a stray copy pushing its index only costs the refresh one more visit)
  DirtyFlag(const DirtyFlag& o) : v(o.v), idx(o.idx), list(o.list) { g_dirty_epoch.fetch_add(1, std::memory_order_relaxed); }
  DirtyFlag& operator=(const DirtyFlag& o) { return *this = o.v; }
  DirtyFlag& operator=(bool x) {
    if (x) {
      g_dirty_epoch.fetch_add(1, std::memory_order_relaxed);
      if (!v && list) list->push_back(idx);
    }
    v = x;
    return *this;
  }
  void bind(int32_t i, std::vector<int32_t>* l) {
    idx = i;
    list = l;
    if (v) l->push_back(i);
  }
  operator bool() const { return v; }
};

// one node holding reservations a pod matches (k_rsv_pick)
struct RsvPair {
  int32_t node;     // local node index
  int16_t raw;      // ScoreReservation of the nominated reservation (0 = none)
  int16_t allowed;  // RSV_PAIR_* bits
  int64_t order;    // smallest reservation-order label of the matched reservations (0 = none)
};
constexpr int16_t RSV_PAIR_ALLOWED = 1;        // the Reservation plugin's Filter passes (always without an affinity)
constexpr int16_t RSV_PAIR_RESERVE_FAILS = 2;  // DeviceShare's Reserve fails there (the pod is not placed)
constexpr int16_t RSV_PAIR_SCORE_ERROR = 4;    // NodeNUMAResource's Score errs there: feasible, it fails the pod's cycle

struct NodeState {
  bool valid = false;  // in the snapshot (ke_node_upsert .. ke_node_delete)
  bool known = false;  // upserted at least once: the object state below belongs to a node
  ke_node node{};
  bool has_metric = false;
  ke_node_metric nm{};
  std::vector<ke_pod_metric> pm;
  std::vector<ke_aggregated_usage> agg;
  std::vector<AssignedPod> asg;
  std::vector<int64_t> asg_uid;  // asg[i].pod.uid: the uid scans of assign / unassign read 8 B an entry
  // NodeResourceTopology NUMA zones + the resource manager's allocation on them
  std::vector<ke_numa_zone> zones;
  // CPU topology + cpuset allocations (TopologyOptions.CPUTopology / ReservedCPUs / MaxRefCount,
  // NodeAllocation.allocatedCPUs); empty = no CPU topology
  std::vector<ke_cpu> cpus;
  int32_t cpu_max_ref = 1;
  // The resource manager's NodeAllocation outlives the NRT (topologyManager.Delete drops only the
  // TopologyOptions, topology_options.go:84-88): ke_node_topology_delete parks the CPU records and zones here
  // (releases keep applying to them) and the next ke_node_cpus_set / ke_node_numa_set that carries no
  // allocation of its own takes the parked ref counts / zone allocations back by CPU / NUMA id.
  std::vector<ke_cpu> kept_cpus;
  std::vector<ke_numa_zone> kept_zones;
  // DeviceShare node device cache entry (device_cache.go:518-568)
  bool has_dev_cache = false;
  std::vector<ke_device> devs;
  // GPU partition indexer / policy (ke_node_gpu_partitions): table id in Context::ptab, -1 = nil indexer
  int32_t ptable = -1;
  bool gpu_honor = false;
  // DeviceShare hints: interned label-set ids per device (5 per device: its labels, then its 4 VF groups'),
  // the Device's secondary-well-planned label and the node's GPU template model key id (0 = none)
  std::vector<uint8_t> dev_lbl;
  bool secondary_well_planned = false;
  int32_t gpu_model_id = 0;
  // NodeResourcesFitPlus / ScarceResourceAvoidance: NodeInfo Allocatable / (NonZero)Requested by resource id
  std::vector<ke_node_resource> xres;
  // Reservations: the NodeInfo restore every pod sees (restoreUnmatchedReservations), added to
  // Requested / NonZeroRequested (MilliCPU, Memory) when the rows are derived (load_reservations)
  int64_t rv_req[KE_NRES] = {0, 0}, rv_nz[KE_NRES] = {0, 0};
  int32_t rv_pods = 0;  // len(NodeInfo.Pods) delta of the restore (matched reserve pods removed)
  // ... and of NodeInfo.Requested.ScalarResources by resource id (reservations' allocatable beyond cpu / memory)
  std::vector<std::pair<int32_t, int64_t>> rv_x;
  // ... and the plugins' restore states of the reservations holding NUMA / cpuset / device allocations
  // (ke_reservations_load_ex): NodeNUMAResource's reusableResources per zone (mergedUnmatchedUsed; key bits
  // 2*id + r of the ResourceList keys present) and DeviceShare's preemptible per instance
  // (mergedUnmatchedUsed[type][minor]; bit 16*type + minor present), folded into the NUMA / device rows
  int64_t rv_numa[KE_MAX_NUMA * KE_NRES] = {};
  uint32_t rv_numa_keys = 0;
  uint8_t rv_numa_zones = 0;  // NUMA ids with a reusable entry
  int64_t rv_dev[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS] = {};
  uint64_t rv_dev_keys[KE_DKEYS] = {0, 0, 0};  // bit 16*type + minor per key present
  uint64_t rv_dev_minors = 0;
  bool rsv_ovr = false;  // the current KE_RSV_MATCHED segment overrides this node's cpuset trial (NF_RSV_CS)
  // derived
  DirtyFlag dirty;              // row must be re-derived and uploaded
  int64_t valid_until = INT64_MAX;  // derived row is exact for now < valid_until
  // LoadAware U*(total, thr) per [variant][res] (INT64_MAX = no constraint); cached by derive_row
};

struct DeviceState;  // ke_kernels.hip

struct Context {
  ke_config cfg{};
  KArgs kargs_template{};
  std::vector<NodeState> nodes;  // size = node_capacity
  int32_t n_nodes = 0;           // 1 + highest populated index
  bool ds_enabled = false;       // some node has a device cache entry: the device SoA exists
  bool numa_enabled = false;     // some node has a NUMA topology policy: the NUMA SoA exists
  bool cpu_enabled = false;      // some node has a CPU table: the CPU SoA exists
  bool ext_enabled = false;      // NodeResourcesFitPlus / ScarceResourceAvoidance in the profile: the ext SoA exists
  int32_t n_bind_nodes = 0;      // nodes with a CPU bind policy (a cpu request may bind CPUs there)
  int32_t n_policy_nodes = 0;    // nodes with a NUMA topology policy
  std::vector<uint64_t> last_cpusets;    // per pod of the last ke_schedule: 4 words (CPU-id bitset)
  std::vector<int64_t> last_numa_alloc;  // per pod of the last ke_schedule: [KE_MAX_NUMA*KE_NRES]
  std::vector<uint64_t> last_dev_alloc;  // per pod of the last ke_schedule
  // per pod of the last ke_schedule: the chosen node (-1 once unreserved), the pod uid and whether its
  // ElasticQuota Reserve ran (ke_last_allocations / ke_unreserve)
  std::vector<int32_t> last_chosen;
  std::vector<int64_t> last_uid;
  std::vector<uint8_t> last_quota;
  DeviceState* dev = nullptr;
  // last ke_schedule timing
  double last_total_ms = 0.0;
  std::vector<double> last_batch_ms;
  double kstat_eval_ms = 0, kstat_select_ms = 0, kstat_resolve_ms = 0, kstat_fixup_ms = 0, kstat_handoff_ms = 0;
  int32_t last_pipelined = 0;
  int32_t last_ds_cuts = 0;  // DeviceShare batches of the last ke_schedule that stopped early (re-run remainders)
  double kstat_spec_failed = 0;  // per batch: speculative-replay rounds that ended at a failed prediction
  double kstat_rows_fetched = 0, kstat_rows_changed = 0;  // per batch: replay records fetched (best unchanged candidates), rows changed
  double last_enqueue_ms = 0;  // host time spent enqueueing the last ke_schedule's launches
  // host wall ms of the last ke_schedule by phase: argument checks, row refresh, pod upload, launch
  // setup, enqueue, wait for the device, statistics readback, host mirror of the Reserves
  double host_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // batches of the last ke_schedule that ran pipelined (two streams)
  double kstat_resolve_prologue_ms = 0, kstat_resolve_loop_ms = 0;
  double kstat_resolve_phase_ms[6] = {0, 0, 0, 0, 0, 0};
  double kstat_resolve_sub_ms[5] = {0, 0, 0, 0, 0};  // ke_debug_resolve_subphases
  double kstat_resolve_wave1_ms[4] = {0, 0, 0, 0};  // ke_debug_resolve_wave1
  int64_t kstat_numa_deferred = 0;  // BestEffort pairs the last ke_eval / ke_schedule left to k_numa_fallback
  int32_t kstat_samples = 0;
  // Host mirror of the LoadAware / NodeInfo part of the last ke_schedule's Reserves (the device rows
  // already carry them), applied lazily: by the next call that reads or changes host node state, or
  // while the next ke_schedule's launches run (flush_mirror).
  struct PendingAssign {
    int32_t node;
    int64_t ts;
    int64_t idx;  // the pod: pending_pods[idx]
  };
  std::vector<PendingAssign> pending;
  std::vector<ke_pod> pending_pods;  // copies of scheduled pods, taken while the device runs the call
  int64_t pending_base = 0;          // pending_pods index of the current device_schedule segment's first pod
  // flush_mirror_async: the mirror of earlier placements applied on a host thread while this one enqueues and
  // waits; every reader of the host node state joins it first (mirror_join; flush_mirror joins)
  std::thread mirror_thread;
  ~Context() { if (mirror_thread.joinable()) mirror_thread.join(); }
  Context() = default;
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  // The DevPod records of the current call's pods, built once by the argument checks (check_cpuset) and
  // reused by upload_pods
  std::vector<DevPod> staged;
  const ke_pod* staged_src = nullptr;
  // ElasticQuota tree (ke_quotas_load): objects, the used limits computed on the host, and whether the
  // device copy of the table is stale
  ke_quota_args qargs{};
  std::vector<ke_quota> quotas;
  std::vector<int64_t> qlimit;     // [q * KE_NRES + r]
  std::vector<uint8_t> qlimit_has; // [q * KE_NRES + r]
  bool quota_dirty = false;        // host table newer than the device table
  bool quota_on_device = false;    // the device table holds the current used (after a ke_schedule)
  // GPU partition tables, deduplicated: PT_WORDS words per table (ke_types.h), uploaded when ptab_dirty
  std::vector<uint64_t> ptab;
  bool ptab_dirty = false;
  // DeviceShare hints (ke_set_pod_device_hints), GPU shared resource templates (ke_gpu_templates_load), the
  // interned device / VF-group label sets (id -> sorted (key, value) pairs; id 0 = no labels) and template
  // model keys (id -> ke_label_id of "<vendor>-<model>", id 0 = none); the VF ranks of the last ke_schedule
  std::vector<ke_pod_device_hints> hints;
  std::vector<ke_gpu_template> tmpl;
  std::vector<ke_reservation> resv;  // ke_reservations_load (allocated / allocated_pods kept by Reserve)
  std::vector<ke_reservation_alloc> resv_alloc;  // their NUMA / cpuset / device holdings (owner parts kept by Reserve)
  std::vector<uint8_t> resv_holds;   // derived from resv_alloc: KE_RSV_HOLDS_* bits
  // per reservation its allocatable names beyond cpu / memory (ke_reservations_load_full; allocated kept by Reserve)
  std::vector<std::vector<ke_reservation_resource>> resv_res;
  std::vector<std::vector<uint8_t>> resv_cpu_cnt;  // per reservation: owners per CPU id (lazily from owner_cpuset)
  std::vector<std::vector<int32_t>> resv_by_node;  // reservation indices per node
  // ke_pod_reservations staging for the next ke_schedule: CSR over its pods
  std::vector<int32_t> match_off, match_ids;
  // the KE_RSV_MATCHED pod of the current segment: its nodes with matched reservations, their
  // (node, ScoreReservation of the nominated one, smallest order) for the device pick, the nominated index
  std::vector<int32_t> rsv_nodes;
  std::vector<RsvPair> rsv_pairs;
  std::vector<int32_t> rsv_nominated;
  bool rsv_affinity = false;  // the segment's pod has a required reservation affinity
  bool rsv_fused = false;
  int64_t last_rsv_fused = 0, last_rsv_fused_gated = 0;  // fused matched pods placed / gated (statistics)     // the call's last pod is a matched pod fused behind plain pods (ke_schedule)
  std::vector<RsvOvr> rsv_ovr;  // its allocate-from-reservation decisions per node (SoA::rovr)
  // its allocate-from-reservation trials (resv_views -> k_rsv_views): per view the reservation and the outcome
  std::vector<RsvView> rsv_views;
  std::vector<int32_t> rsv_view_resv;
  std::vector<RsvViewOut> rsv_view_out;
  // its DeviceShare allocate-from-reservation views (resv_ds_views -> k_ds_views): per view the reservation (-1: the
  // node's own allocation with the matched reservations' allocatable preemptible, -2: the ignored pod's
  // tryAllocateIgnoreReservation) and the outcome
  std::vector<DsView> ds_views;
  std::vector<int32_t> ds_view_resv;
  std::vector<DsViewOut> ds_view_out;
  // its NodeNUMAResource views under a NUMA policy (resv_numa_views -> k_numa_views): per node view set the
  // reservations of its trials (index order) and the outcome
  std::vector<NumaRsvView> numa_views;
  std::vector<std::vector<int32_t>> numa_view_ids;
  std::vector<NumaRsvOut> numa_view_out;
  // a binding pod's cpuset pass after the nomination (resv_prepare -> k_rsv_views with zones, resv_numa_cs_apply): per
  // view the rsv_ovr / rsv_pairs entries it completes
  std::vector<RsvView> numa_cs_views;
  std::vector<int32_t> numa_cs_ovr, numa_cs_pair;
  std::vector<RsvViewOut> numa_cs_out;
  std::vector<int32_t> last_resv;  // per pod of the last ke_schedule: 1 + the reservation assumed, 0 = none
  int32_t resv_gen = 0;            // ke_reservations_generation: bumped by every load_reservations
  // per-pod latency of the last ke_schedule (ke_last_pod_latencies): the call's entry on the host clock, and
  // per pod the ms from it to its batch's Reserve end
  std::chrono::steady_clock::time_point call_entry{};
  std::vector<double> last_pod_lat;
  // device_refresh: g_dirty_epoch when every row was last clean, and the earliest valid_until then
  uint64_t clean_epoch = UINT64_MAX;
  int64_t min_valid_until = INT64_MIN;
  int32_t clean_n_nodes = -1;         // n_nodes at that scan
  std::vector<int32_t> dirty_list;    // nodes that became dirty since (may repeat or be clean again)
  std::vector<std::vector<std::pair<int32_t, int32_t>>> label_sets{{}};
  std::map<std::vector<std::pair<int32_t, int32_t>>, int> label_set_ids{{{}, 0}};
  std::vector<int32_t> model_keys{0};
  std::vector<int8_t> last_vf;  // [pod][2][KE_MAX_MINORS]
};

// the hint record of a pod (nullptr: none); the index was validated by validate_pod_hints
const ke_pod_device_hints* pod_hints(const Context& c, const ke_pod& p);
int validate_pod_hints(const Context& c, const ke_pod& p);
// intern the label sets of a node's devices into ns.dev_lbl (KE_ERR_UNSUPPORTED beyond 256 distinct sets)
int intern_device_labels(Context& c, NodeState& ns);
int intern_model_key(Context& c, int32_t key);  // id 1..255, or a negative KE_ERR_*
// labels.Selector.Matches of a converted LabelSelector against an interned label set
bool selector_matches(const ke_label_selector& sel, const std::vector<std::pair<int32_t, int32_t>>& labels);
// the device-side record of a hinted pod: the Selector / VFSelector / template candidate sets over the
// current interned ids, flags and the joint types
DevPodHint make_pod_hint(const Context& c, const ke_pod& pod, const DevPod& dp, const ke_pod_device_hints& h);

// Encode a node's partition table (validated) into the pool; returns its id or a negative KE_ERR_*.
int ptable_intern(Context& c, int32_t n, const ke_gpu_partition* parts);

// ElasticQuota used limits of every quota (RuntimeQuotaCalculator over the tree, or Max)
int quota_compute_limits(const ke_quota_args& args, const std::vector<ke_quota>& q, std::vector<int64_t>& limit,
                         std::vector<uint8_t>& has);

// error plumbing (thread-local, read by ke_last_error)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

// validation of objects against the implemented hot path
int validate_config(const ke_config& cfg);
int validate_node(const ke_node& n);
int validate_pod(const ke_pod& p);

// DefaultEstimator.EstimatePod (estimator/default_estimator.go:59-122)
void estimate_pod(const ke_loadaware_args& a, const ke_pod& pod, int64_t* est, uint8_t* present);
// pod -> device parameters
DevPod make_dev_pod(const ke_config& cfg, const ke_pod& pod, const ke_pod_device_hints* hints = nullptr,
                    const std::vector<ke_gpu_template>* tmpl = nullptr);

// Fold a node's object state into its row for evaluation at `now` (valid until *valid_until).
void derive_row(const ke_config& cfg, const NodeState& ns, int64_t now, Row* row, int64_t* valid_until);

// U*(total, thr): the largest used with int64(math.Round(float64(used)/float64(total)*100)) <= thr,
// searched over |used| <= 2^53 (load_aware.go:299).  total > 0.
int64_t max_used_within(int64_t total, int64_t thr);
int64_t usage_percent(int64_t used, int64_t total);

// host mirror of Reserve (podAssignCache.assign + NodeInfo.Requested += requests)
void host_assign(const ke_config& cfg, NodeState& ns, const ke_pod& pod, int64_t timestamp_ns, bool mark_dirty = true);
// apply Context::pending (placements whose device rows are already patched: dirty flags unchanged)
void flush_mirror(Context& c);
void flush_mirror_async(Context& c);
void mirror_join(Context& c);
// ke_schedule_submit / ke_schedule_wait (ke_kernels.hip): a call's enqueue part returns its completion, which waits
// for the call's device work, writes the placements / scores and the call's statistics
using DevFinish = std::function<int(int32_t* chosen, int32_t* score)>;
int device_schedule_enqueue(Context* ctx, int32_t n_pods, const ke_pod* pods, int64_t now, bool want_score, DevFinish* fin);
void device_swap_call_buffers(Context* ctx);
void device_quiesce(Context* ctx);  // wait for every stream of the context (after a failed enqueue)
bool device_refresh_pending(const Context* ctx, int64_t now);
bool device_async_ok(const Context* ctx, int32_t n_pods);

// DeviceShare
int validate_devices(int32_t n, const ke_device* devs);
// the device SoA row of a node: NUM_DS_FIELDS int64 + NUM_DS_MASKS uint64 (zero when no cache entry)
void derive_ds_row(const NodeState& ns, int64_t* f, uint64_t* masks);
// its NUM_DSX hint words (DSX_*: label-set ids, PCIe ranks, node flags, VF state)
void derive_dsx_row(const NodeState& ns, int64_t* w);
// host mirror of DeviceShare Reserve: add the allocation of `pod` on the minors in `mask`
// (bit 16*type+minor) to the node's device cache (fillGPUTotalMem + updateCacheUsed)
void host_ds_reserve(const ke_config& cfg, NodeState& ns, const DevPod& dp, uint64_t mask, const int8_t* vf = nullptr);

// NUMA topology
int validate_zones(int32_t n, const ke_numa_zone* zones);
// NUMANodeSharedStatus (node_allocation.go:60-68) from the zone's single / shared pod counts
uint8_t zone_status(const ke_numa_zone& z);
// a status given without counts stands for one pod of that kind
void normalize_zone(ke_numa_zone& z);
// the NUMA SoA row of a node: NUM_NUMA_FIELDS int64 + the uint32 mask
void derive_numa_row(const NodeState& ns, int64_t* f, uint64_t* mask);
// host mirror of the NUMA allocation the device Reserve made: delta[z][r] per zone id
void host_numa_reserve(NodeState& ns, const int64_t* delta /*[KE_MAX_NUMA*KE_NRES]*/);

// NodeResourcesFitPlus / ScarceResourceAvoidance
int validate_node_resources(int32_t n, const ke_node_resource* r);
// the ext slots' resource ids (FitPlus resources, then NodeResourcesFit's other resources and filtered scalars);
// returns their count (> NUM_XS: refused by validate_config).  `ids` holds 2 * NUM_XS + KE_MAX_FITPLUS entries.
int ext_slots(const ke_config& cfg, int32_t* ids);
// the ext SoA row of a node: NUM_XF int64 + the uint64 mask of resource ids with Allocatable > 0
void derive_ext_row(const ke_config& cfg, const NodeState& ns, int64_t* f, uint64_t* mask);
int load_reservations(Context& c, int32_t n, const ke_reservation* r, const ke_reservation_alloc* allocs = nullptr,
                      const int32_t* res_off = nullptr, const ke_reservation_resource* res = nullptr);
bool resv_usable(const ke_reservation& r);
void resv_node_restore(Context& c, int32_t node);  // the restore every non-matching pod sees
// scoreReservation of reservation i for the pod (reservation/scoring.go:191-210)
int32_t resv_score(const Context& c, int32_t i, const ke_pod& pod);
// the pod's PodRequests of resource id (cpu / memory: ke_pod.requests, others: its ke_pod.xres entry, 0 without)
int64_t pod_request_of(const ke_pod& pod, int32_t id);
// the scalar restore delta of resource id on the node (NodeInfo.Requested.ScalarResources)
int64_t rv_x_of(const NodeState& ns, int32_t id);
// the nominated-reservation path of one KE_RSV_MATCHED pod: rows with its matched restore, rsv_pairs /
// rsv_nominated; resv_finish assumes the pod into the chosen node's nominated reservation (1 + index, 0)
int resv_prepare(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids, bool affinity);
// the allocate-from-reservation trials a KE_RSV_MATCHED pod needs (into c.rsv_views / rsv_view_resv): per node of
// its matched reservations holding a cpuset / NUMA resources where the pod binds CPUs, one per such reservation
void resv_views(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids);
// the DeviceShare views of a reservation-matched DeviceShare pod (ids: its matched reservations) or, ids == nullptr,
// of a reservation-ignored one: per node of its device-holding reservations one per such reservation in index order
// and the node's own (-1); an ignored pod the node's own and the ignore view (-2).  Into c.ds_views / ds_view_resv.
void resv_ds_views(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids);
// the NodeNUMAResource views of a reservation-matched pod (ids: its matched reservations): per node of its
// reservations holding NUMA resources / CPUs where a NUMA policy applies, one view set over them (k_numa_views), with
// the views' preferredCPUs for a pod binding CPUs there.  Into c.numa_views / numa_view_ids; the rows of those nodes
// carry the pod's matched restore.
void resv_numa_views(Context& c, const ke_pod& pod, const int32_t* ids, int32_t n_ids);
// the cpuset pass's outcome (c.numa_cs_out, k_rsv_views over c.numa_cs_views after resv_prepare): Reserve's cpuset and
// the Score of the nominated reservation's allocation; a failed one is a Score error
void resv_numa_cs_apply(Context& c);
// the refusals of resv_prepare, checked for every pod before a ke_schedule call schedules any
int resv_check(const Context& c, const int32_t* ids, int32_t n_ids);
// a run of KE_RSV_IGNORED pods: the rows with every usable reservation matchedOrIgnored (begin) and back to the
// restore every other pod sees (end); resv_ignore_check is the refusal, checked before any segment runs
int resv_ignore_check(const Context& c, const ke_pod& pod, uint32_t pod_flags);
void resv_ignore_begin(Context& c);
void resv_ignore_end(Context& c);
// a reservation-ignored pod that may bind CPUs beside reservations holding NUMA resources / CPUs: a segment of its
// own, its allocate-ignoring-reservation trials (resv_ignore_views -> device_rsv_views) turned into the Filter /
// Reserve decisions of those nodes (resv_ignore_ovr)
bool resv_ignore_needs_views(const Context& c, const ke_pod& pod, uint32_t pod_flags);
void resv_ignore_views(Context& c, const ke_pod& pod);
void resv_ignore_ovr(Context& c);
void resv_finish(Context& c, int32_t chosen_local, const ke_pod& pod, int32_t* assumed, const uint64_t* cpuset = nullptr,
                 const int64_t* numa = nullptr, uint64_t dev_minors = 0);
void resv_forget(Context& c, int32_t idx, const ke_pod& pod, const ke_pod_allocation* a = nullptr);
uint8_t resv_holds_of(const ke_reservation_alloc& a);
void ds_instance_amounts(const ke_device& d, const DevPod& dp, int64_t* alloc, bool* has);
// NodeResourcesFitPlus' (NonZero)Requested of resource `id` on the node, with the reservation restore
int64_t xres_requested(const NodeState& ns, const ke_node_resource& r);
void host_ext_reserve(NodeState& ns, const ke_pod& pod);

// CPU topology / cpuset binding (NodeNUMAResource with NUMA policy None)
int validate_cpus(int32_t n, const ke_cpu* cpus, int32_t max_ref);
bool cpus_valid(const NodeState& ns);  // a CPU table that CPUTopology.IsValid() accepts
int64_t cpus_allocated(const NodeState& ns);  // allocatedCPUs.Size() (else ke_node.cpuset_allocated_cpus)
// the node's CPU records (CPU_SLOTS, by CPU id) and its NUM_CS_FIELDS summary words
void derive_cpu_rows(const NodeState& ns, CpuRec* recs, int64_t* cs);
// host mirror of a cpuset Reserve: RefCount++ / exclusive policy on the CPUs of `set` (4 words), the
// NUMA nodes' single / shared status (node_allocation.go:111-156)
void host_cpuset_reserve(NodeState& ns, const DevPod& dp, const uint64_t* set);

// Release of one placement from its node (ke_pod_release): podAssignCache.unAssign, NodeInfo.RemovePod
// (Requested, the FitPlus requested when `ext`), resourceManager.Release, DeviceShare updateCacheUsed(false)
void host_release_node(const ke_config& cfg, bool ext, NodeState& ns, const ke_pod& pod, const ke_pod_allocation& a,
                       const ke_pod_device_hints* h = nullptr);
// ElasticQuota UnreservePod (assigned) / OnPodDelete (del) on the host tree (used already synced from the
// device); recomputes the runtime limits when the tree total or a request moved
int host_quota_release(Context& c, const ke_pod& pod, bool assigned, bool del);

}  // namespace ke
