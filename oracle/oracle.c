/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain-C restatement of the reference's
 * per-node Filter/Score arithmetic.  Every function cites the Go it follows
 * (paths relative to haoyann/koordinator @ /root/reference):
 *
 *   LoadAwareScheduling  pkg/scheduler/plugins/loadaware/load_aware.go, helper.go,
 *                        estimator/default_estimator.go, pod_assign_cache.go
 *   NodeNUMAResource     pkg/scheduler/plugins/nodenumaresource/plugin.go, scoring.go,
 *                        least_allocated.go, most_allocated.go, util.go
 *   DeviceShare          pkg/scheduler/plugins/deviceshare/plugin.go, utils.go, scoring.go,
 *                        device_allocator.go, allocator_gpu.go, device_cache.go, device_resources.go,
 *                        devicehandler_gpu.go, devicehandler_default.go; k8s.io/apiserver quota/v1
 *   helpers              apis/extension/node_resource_amplification.go, resource.go, load_aware.go
 *   framework            k8s v1.28.7 weighted score sum + selectHost (tie -> lowest node index)
 *
 * Unlike the product it precomputes nothing: GetEstimatedUsed is rebuilt from the NodeMetric and the
 * assign cache on every Filter and every Score call, as the Go plugin does.
 */
#include "oracle.h"
#include "quota.h"
#include "cpu_accumulator.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NS_PER_S 1000000000LL
#define MAX_NODE_SCORE 100 /* framework.MaxNodeScore */
#define DEFAULT_MILLI_CPU 250LL                   /* default_estimator.go:36 */
#define DEFAULT_MEMORY (200LL * 1024 * 1024)      /* default_estimator.go:38 */
#define DEFAULT_REPORT_INTERVAL_NS (60LL * NS_PER_S) /* load_aware.go:58 */

typedef struct or_asg {
  ke_pod pod;
  int64_t ts;
  int64_t est[KE_NRES];
  uint8_t est_present[KE_NRES];
  int has_est; /* estimated != nil */
} or_asg;

typedef struct or_node {
  ke_node node;
  int has_metric;
  ke_node_metric nm;
  ke_pod_metric* pm;
  int32_t n_pm;
  ke_aggregated_usage* agg;
  int32_t n_agg;
  or_asg* asg;
  int32_t n_asg, cap_asg;
  int32_t n_zone; /* TopologyOptions.NUMANodeResources + the resource manager's per-zone allocation */
  ke_numa_zone zone[KE_MAX_NUMA];
  int has_dev_cache; /* nodeDeviceCache.getNodeDevice != nil */
  int32_t n_dev;
  ke_device dev[KE_DEV_TYPES * KE_MAX_MINORS];
  /* GPU partition indexer + policy as GPUAllocator.Allocate resolves them (allocator_gpu.go:77-82) */
  int gpu_has_table, gpu_honor;
  int secondary_well_planned; /* Device label: IsSecondaryDeviceWellPlanned (device_cache.go:546) */
  int32_t gpu_model_key;      /* "<vendor>-<model>" of the node's GPU labels (allocator_gpu.go:140), 0 = none */
  int32_t n_part;
  ke_gpu_partition part[KE_MAX_GPU_PARTITIONS];
  struct or_cpus* cpus; /* CPU topology + allocated CPUs (NULL: no CPU topology) */
  /* the NodeAllocation while the NRT is deleted (topology_options.go:84-88 drops only the TopologyOptions):
   * or_node_topology_delete parks the CPU table / zones, releases apply to them, a bare re-add takes them back */
  struct or_cpus* kept_cpus;
  int32_t n_kept_zone;
  ke_numa_zone kept_zone[KE_MAX_NUMA];
  /* NodeInfo Allocatable / (NonZero)Requested by resource id (NodeResourcesFitPlus, ScarceResourceAvoidance) */
  int32_t n_xres;
  ke_node_resource xres[KE_MAX_XRES];
  /* the reservation cache's NodeInfo restore for a pod that matches no reservation (or_reservations_load) */
  int64_t rv_req[KE_NRES], rv_nz[KE_NRES];
  int32_t rv_pods; /* len(NodeInfo.Pods) delta of the restore: a matched reservation's reserve pod is removed */
  int64_t rv_x[KE_MAX_XRES]; /* ... and of NodeInfo.Requested.ScalarResources by resource id */
  /* the plugins' RestoreReservation states of the pod being evaluated (or_restore): NodeNUMAResource's
   * mergedUnmatchedUsed per NUMA id (ResourceList keys tracked) and DeviceShare's per (type, minor) */
  int rs_numa_has[KE_MAX_NUMA];
  uint8_t rs_numa_key[KE_MAX_NUMA][KE_NRES];
  int64_t rs_numa[KE_MAX_NUMA][KE_NRES];
  int rs_dev_has[KE_DEV_TYPES][KE_MAX_MINORS];
  uint8_t rs_dev_key[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS];
  int64_t rs_dev[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS];
  int deleted; /* Node informer delete: out of the snapshot (every other cache keeps its state) */
} or_node;

/* TopologyOptions.CPUTopology / ReservedCPUs / MaxRefCount + NodeAllocation.allocatedCPUs */
typedef struct or_cpus {
  acc_topo t;
  acc_alloc al; /* present = RefCount > 0 */
  uint8_t reserved[ACC_MAX_CPUS];
  int max_ref;
} or_cpus;

struct or_cluster {
  ke_config cfg;
  int32_t n;
  or_node* nodes;
  or_quotas* quotas; /* ElasticQuota tree (quota.c), NULL until loaded */
  /* ke_set_pod_device_hints table (ke_pod.device_hint = 1 + index) and the GPU shared resource templates */
  ke_pod_device_hints* hints;
  int32_t n_hints;
  ke_gpu_template* tmpl;
  int32_t n_tmpl;
  int8_t* last_vf; /* VF ranks of the last or_schedule: [pod][2][KE_MAX_MINORS] */
  int32_t last_vf_n;
  /* the reservation cache (or_reservations_load; allocated / allocated pods kept by Reserve), the matched
   * lists of the next or_schedule (or_pod_reservations) and 1 + the reservation each pod of the last
   * or_schedule was assumed into */
  ke_reservation* resv;
  ke_reservation_alloc* ralloc; /* the reservations' NUMA / cpuset / device holdings (NULL: none) */
  const char* resv_m;           /* the matched flags of the pod being evaluated (or_resv_begin), NULL = none */
  int ignored;                  /* the pod being evaluated / reserved is reservation-ignored (or_numa_ignored) */
  const int32_t* ds_nom;        /* per node the reservation nominated for the pod being scored / reserved (or NULL) */
  const int32_t* numa_nom;      /* the same for NodeNUMAResource's Score (allocateWithNominatedReservation), or NULL */
  const int8_t* numa_rok;       /* per reservation NodeNUMAResource's FilterNominateReservation under a NUMA policy (or NULL) */
  uint8_t* rcpu;                /* [reservation][cpu] owner counts (or_owner_update), NULL until first needed */
  int32_t n_resv;
  /* each reservation's allocatable entries beyond cpu / memory (or_reservations_load_full): roff[i] .. roff[i+1] */
  int32_t* roff;
  ke_reservation_resource* rres;
  int32_t* moff;
  int32_t* mids;
  int32_t m_pods;
  int32_t* last_resv;
  int32_t last_resv_n;
};

/* ---------------------------------------------------------------------------------------------- */
/* helpers                                                                                          */
/* ---------------------------------------------------------------------------------------------- */

int64_t or_usage_percent(int64_t used, int64_t total) {
  /* int64(math.Round(float64(used) / float64(total) * 100))  load_aware.go:299 */
  double u = (double)used;
  double t = (double)total;
  double q = u / t;
  double p = q * 100.0;
  return (int64_t)round(p);
}

/* extension.Amplify  node_resource_amplification.go:170-175 */
static int64_t amplify(int64_t origin, double ratio) {
  if (ratio <= 1.0) return origin;
  double x = (double)origin * ratio;
  return (int64_t)ceil(x);
}

/* translated resource index for a weighted resource (cpu/memory) and a priority class:
 * extension.TranslateResourceNameByPriorityClass  apis/extension/resource.go:53-58.
 * Returns -1 for the empty resource name (PriorityFree has no mapping). */
static int translate(int32_t priority, int r) {
  switch (priority) {
    case KE_PRIORITY_PROD:
    case KE_PRIORITY_NONE:
      return r;
    case KE_PRIORITY_BATCH:
      return r == KE_RES_CPU ? KE_RES_BATCH_CPU : KE_RES_BATCH_MEMORY;
    case KE_PRIORITY_MID:
      return r == KE_RES_CPU ? KE_RES_MID_CPU : KE_RES_MID_MEMORY;
    default:
      return -1;
  }
}

/* estimatedUsedByResource  default_estimator.go:88-122 */
static int64_t estimated_used_by_resource(const ke_pod* pod, int name, int64_t factor) {
  int64_t lim = name >= 0 ? pod->limits[name] : 0;
  int64_t req = name >= 0 ? pod->requests[name] : 0;
  int64_t q = lim > req ? lim : req;
  if (q == 0) {
    switch (name) {
      case KE_RES_CPU:
      case KE_RES_BATCH_CPU:
        return DEFAULT_MILLI_CPU;
      case KE_RES_MEMORY:
      case KE_RES_BATCH_MEMORY:
        return DEFAULT_MEMORY;
    }
    return 0;
  }
  /* float64(q) * float64(scalingFactor) / 100, cpu in milli, others Value() */
  double x = (double)q * (double)factor;
  int64_t est = (int64_t)round(x / 100.0);
  if (lim > 0 && est > lim) est = lim;
  return est;
}

/* DefaultEstimator.EstimatePod  default_estimator.go:59-85 */
static void estimate_pod(const ke_loadaware_args* a, const ke_pod* pod, int64_t* est, uint8_t* present) {
  int64_t factors[KE_NRES];
  int use_custom = a->allow_customize_estimation && pod->has_custom_scaling_factors;
  for (int r = 0; r < KE_NRES; r++) {
    int64_t f = KE_ABSENT;
    if (use_custom) f = pod->custom_scaling_factors[r];
    if (f == KE_ABSENT) f = a->estimated_scaling_factors[r]; /* fill missing keys from args */
    factors[r] = f == KE_ABSENT ? 0 : f;                    /* scalingFactors[r] of a missing key = 0 */
  }
  for (int r = 0; r < KE_NRES; r++) {
    present[r] = a->resource_weights[r] != KE_ABSENT; /* keys of resourceWeights */
    est[r] = present[r] ? estimated_used_by_resource(pod, translate(pod->priority_class, r), factors[r]) : 0;
  }
}

void or_estimate_pod(const or_cluster* c, const ke_pod* pod, int64_t* est) {
  uint8_t present[KE_NRES];
  estimate_pod(&c->cfg.loadaware, pod, est, present);
  for (int r = 0; r < KE_NRES; r++)
    if (!present[r]) est[r] = -1;
}

/* isNodeMetricExpired  helper.go:35-40 */
static int node_metric_expired(const or_node* n, int64_t exp_s, int64_t now) {
  if (!n->nm.has_update_time) return 1;
  return exp_s > 0 && (now - n->nm.update_time_ns) >= exp_s * NS_PER_S;
}

/* getTargetAggregatedUsage  helper.go:57-95; returns NULL for nil */
static const ke_resource_map* target_aggregated_usage(const or_node* n, int64_t dur, int32_t type) {
  if (!n->nm.has_node_metric || n->n_agg == 0) return NULL;
  if (dur == 0) {
    int64_t max_dur = 0;
    int max_idx = -1;
    for (int i = 0; i < n->n_agg; i++) {
      if (n->agg[i].usage[type].n_keys > 0 && n->agg[i].duration_ns > max_dur) {
        max_dur = n->agg[i].duration_ns;
        max_idx = i;
      }
    }
    if (max_idx == -1) {
      if (n->nm.node_usage.n_keys > 0) return &n->nm.node_usage;
    } else {
      return &n->agg[max_idx].usage[type];
    }
  } else {
    for (int i = 0; i < n->n_agg; i++) {
      if (n->agg[i].duration_ns == dur && n->agg[i].usage[type].n_keys > 0) return &n->agg[i].usage[type];
    }
  }
  return NULL;
}

/* scoreWithAggregation / filterWithAggregation  helper.go:97-103 */
static int score_with_aggregation(const ke_loadaware_args* a) {
  return a->has_aggregated && a->agg_score_type != KE_AGG_NONE;
}
static int filter_with_aggregation(const ke_loadaware_args* a) {
  int any = 0;
  for (int r = 0; r < KE_NRES; r++) any |= a->agg_usage_thresholds[r] != KE_ABSENT;
  return a->has_aggregated && any && a->agg_usage_type != KE_AGG_NONE;
}

static int any_present(const int64_t* v) {
  for (int r = 0; r < KE_NRES; r++)
    if (v[r] != KE_ABSENT) return 1;
  return 0;
}

typedef struct filter_profile {
  int64_t usage[KE_NRES];
  int64_t prod[KE_NRES];
  int has_agg;
  int64_t agg_thr[KE_NRES];
  int32_t agg_type;
  int64_t agg_dur;
} filter_profile;

/* generateUsageThresholdsFilterProfile  helper.go:107-145 */
static void filter_profile_of(const ke_loadaware_args* a, const ke_node* node, filter_profile* p) {
  const int args_agg = filter_with_aggregation(a);
  if (node->custom_thresholds_error) {
    memcpy(p->usage, a->usage_thresholds, sizeof p->usage);
    memcpy(p->prod, a->prod_usage_thresholds, sizeof p->prod);
    p->has_agg = args_agg;
    memcpy(p->agg_thr, a->agg_usage_thresholds, sizeof p->agg_thr);
    p->agg_type = a->agg_usage_type;
    p->agg_dur = a->agg_usage_duration_ns;
    return;
  }
  /* GetCustomUsageThresholds: a missing annotation yields an empty profile */
  int64_t cu[KE_NRES], cp[KE_NRES], ca[KE_NRES];
  for (int r = 0; r < KE_NRES; r++) {
    cu[r] = node->has_custom_thresholds ? node->custom_usage_thresholds[r] : KE_ABSENT;
    cp[r] = node->has_custom_thresholds ? node->custom_prod_usage_thresholds[r] : KE_ABSENT;
    ca[r] = node->has_custom_thresholds ? node->custom_agg_thresholds[r] : KE_ABSENT;
  }
  if (any_present(cu)) memcpy(p->usage, cu, sizeof cu);
  else memcpy(p->usage, a->usage_thresholds, sizeof p->usage);
  if (any_present(cp)) memcpy(p->prod, cp, sizeof cp);
  else memcpy(p->prod, a->prod_usage_thresholds, sizeof p->prod);
  p->has_agg = node->has_custom_thresholds && node->has_custom_agg;
  if (p->has_agg) {
    if (!any_present(ca) || node->custom_agg_type == KE_AGG_NONE) p->has_agg = 0;
    else {
      memcpy(p->agg_thr, ca, sizeof ca);
      p->agg_type = node->custom_agg_type;
      p->agg_dur = node->custom_agg_duration_ns;
    }
  }
  if (!p->has_agg && args_agg) {
    p->has_agg = 1;
    memcpy(p->agg_thr, a->agg_usage_thresholds, sizeof p->agg_thr);
    p->agg_type = a->agg_usage_type;
    p->agg_dur = a->agg_usage_duration_ns;
  }
}

/* DefaultEstimator.EstimateNode  default_estimator.go:124-143 (raw-allocatable override per key) */
static void estimate_node(const ke_node* node, int64_t* alloc) {
  for (int r = 0; r < KE_NRES; r++)
    alloc[r] = node->raw_allocatable[r] != KE_ABSENT ? node->raw_allocatable[r] : node->allocatable[r];
}

/* the PodMetricInfo that buildPodMetricMap (helper.go:154-170) keeps for `key` (last one wins) */
static const ke_pod_metric* pod_metric_lookup(const or_node* n, int64_t key, int prod_only) {
  for (int i = n->n_pm - 1; i >= 0; i--) {
    const ke_pod_metric* m = &n->pm[i];
    if (prod_only && m->priority_class != KE_PRIORITY_PROD) continue;
    if (m->pod_key == key) return m;
  }
  return NULL;
}

/* shouldEstimatePodByConfig  load_aware.go:360-385 */
static int should_estimate_by_config(const ke_loadaware_args* a, const or_asg* info, int64_t now) {
  int64_t after_sched = -1, after_init = -1;
  if (a->allow_customize_estimation) {
    after_sched = info->pod.custom_seconds_after_scheduled;
    after_init = info->pod.custom_seconds_after_initialized;
  }
  if (a->estimated_seconds_after_pod_scheduled != KE_ABSENT && after_sched < 0)
    after_sched = a->estimated_seconds_after_pod_scheduled;
  if (a->estimated_seconds_after_initialized != KE_ABSENT && after_init < 0)
    after_init = a->estimated_seconds_after_initialized;
  if (after_init > 0 && info->pod.has_initialized) {
    return info->pod.initialized_transition_ns + after_init * NS_PER_S > now;
  }
  if (after_sched > 0 && info->ts + after_sched * NS_PER_S > now) return 1;
  return 0;
}

/* Plugin.GetEstimatedUsed  load_aware.go:251-288, with estimatedAssignedPodUsed (:315-358),
 * buildPodMetricMap / sumPodUsages (helper.go:154-186).  used[r] for r in cpu/memory. */
static void get_estimated_used(const ke_loadaware_args* a, const or_node* n, const ke_pod* pod,
                               const ke_resource_map* node_usage, int prod_pod, int64_t now, int64_t* used) {
  int64_t est[KE_NRES];
  uint8_t present[KE_NRES];
  estimate_pod(a, pod, est, present);
  for (int r = 0; r < KE_NRES; r++) used[r] = est[r];

  /* estimatedAssignedPodUsed */
  const int ut_present = n->nm.has_update_time;
  const int64_t ut = n->nm.update_time_ns;
  const int64_t interval = n->nm.report_interval_seconds != KE_ABSENT ? n->nm.report_interval_seconds * NS_PER_S
                                                                      : DEFAULT_REPORT_INTERVAL_NS;
  const int score_agg_missing =
      score_with_aggregation(a) && target_aggregated_usage(n, a->agg_score_duration_ns, a->agg_score_type) == NULL;
  int64_t assigned[KE_NRES] = {0, 0};
  /* estimated pods set, as keys */
  int64_t* est_keys = n->n_asg ? (int64_t*)malloc(sizeof(int64_t) * (size_t)n->n_asg) : NULL;
  int n_est = 0;
  for (int i = 0; i < n->n_asg; i++) {
    const or_asg* info = &n->asg[i];
    if (prod_pod && info->pod.priority_class != KE_PRIORITY_PROD) continue;
    const ke_pod_metric* pm = n->n_pm ? pod_metric_lookup(n, info->pod.pod_key, prod_pod) : NULL;
    const int usage_len = pm ? pm->usage.n_keys : 0;
    const int missed_latest = ut_present ? info->ts > ut : 1;              /* helper.go:49-51 (zero UpdateTime) */
    const int in_interval = ut_present && info->ts < ut && (ut - info->ts) < interval; /* helper.go:53-55 */
    if (usage_len == 0 || missed_latest || in_interval || score_agg_missing ||
        should_estimate_by_config(a, info, now)) {
      if (!info->has_est) continue;
      for (int r = 0; r < KE_NRES; r++) {
        if (!info->est_present[r]) continue;
        int64_t v = info->est[r];
        if (pm && pm->usage.present[r]) {
          int64_t u = pm->usage.value[r];
          if (u > v) v = u;
        }
        assigned[r] += v;
      }
      est_keys[n_est++] = info->pod.pod_key;
    }
  }
  for (int r = 0; r < KE_NRES; r++) used[r] += assigned[r];

  /* sumPodUsages over the deduplicated, (prod-)filtered pod metric map */
  int64_t pod_actual[KE_NRES] = {0, 0}, est_actual[KE_NRES] = {0, 0};
  for (int i = 0; i < n->n_pm; i++) {
    const ke_pod_metric* m = &n->pm[i];
    if (prod_pod && m->priority_class != KE_PRIORITY_PROD) continue;
    int shadowed = 0; /* a later entry with the same name overwrote this one in the map */
    for (int j = i + 1; j < n->n_pm && !shadowed; j++) {
      if (prod_pod && n->pm[j].priority_class != KE_PRIORITY_PROD) continue;
      shadowed = n->pm[j].pod_key == m->pod_key;
    }
    if (shadowed) continue;
    int is_est = 0;
    for (int k = 0; k < n_est && !is_est; k++) is_est = est_keys[k] == m->pod_key;
    for (int r = 0; r < KE_NRES; r++) {
      if (!m->usage.present[r]) continue;
      if (is_est) est_actual[r] += m->usage.value[r];
      else pod_actual[r] += m->usage.value[r];
    }
  }
  free(est_keys);

  if (prod_pod) {
    for (int r = 0; r < KE_NRES; r++) used[r] += pod_actual[r];
  } else if (node_usage != NULL) {
    for (int r = 0; r < KE_NRES; r++) {
      if (!node_usage->present[r]) continue;
      int64_t q = node_usage->value[r];
      int64_t e = est_actual[r];
      if (e != 0 && q >= e) q -= e;
      used[r] += q;
    }
  }
}

/* ---------------------------------------------------------------------------------------------- */
/* unsupported-feature guards (ABI v1 hot path: LoadAware + NodeNUMAResource policy None)           */
/* ---------------------------------------------------------------------------------------------- */

/* AllowUseCPUSet + PreFilter requestCPUBind (nodenumaresource/util.go:49-56, plugin.go:276-301) */
static int pod_is_cpuset(const ke_pod* pod) {
  return (pod->qos_class == KE_QOS_LSE || pod->qos_class == KE_QOS_LSR) && pod->priority_class == KE_PRIORITY_PROD &&
         pod->requests[KE_RES_CPU] > 0;
}
static int pod_unsupported(const ke_pod* pod) {
  /* KE_RSV_MATCHED / AFFINITY / IGNORED pods are checked by or_schedule (or_resv_supported) */
  return pod->has_resource_spec || pod->has_unsupported_device_requests || pod->reservation_matched > KE_RSV_IGNORED;
}
static int node_unsupported(const ke_node* n) {
  return n->numa_topology_policy < 0 || n->numa_topology_policy > KE_NUMA_POLICY_SINGLE_NUMA_NODE ||
         n->cpu_bind_policy < 0 || n->cpu_bind_policy > KE_NODE_CPU_BIND_SPREAD_BY_PCPUS;
}

/* ---- cpuset binding (PreFilter plugin.go:251-312, requestCPUBind util.go:121-138) ----------------- */
typedef struct cpuset_state {
  int rcb;        /* state.requestCPUBind */
  int required;   /* state.requiredCPUBindPolicy */
  int preferred;  /* state.preferredCPUBindPolicy */
  int excl;       /* state.preferredCPUExclusivePolicy */
  int num_cpus;   /* numCPUsNeeded */
  int invalid;    /* PreFilter: non-integer cpuset request -> UnschedulableAndUnresolvable */
} cpuset_state;

static void cpuset_prefilter(const or_cluster* c, const ke_pod* pod, cpuset_state* st) {
  memset(st, 0, sizeof *st);
  const int64_t cpu = pod->requests[KE_RES_CPU];
  st->num_cpus = (int)(cpu / 1000);
  if (!pod_is_cpuset(pod) && !((pod->qos_class == KE_QOS_LSE || pod->qos_class == KE_QOS_LSR) &&
                               pod->priority_class == KE_PRIORITY_PROD))
    return; /* AllowUseCPUSet */
  int bind = pod->cpu_bind_preferred;
  if (bind == KE_CPU_BIND_UNSET || bind == KE_CPU_BIND_DEFAULT) bind = c->cfg.numa.default_cpu_bind_policy;
  int required = pod->cpu_bind_required;
  if (required == KE_CPU_BIND_DEFAULT) required = c->cfg.numa.default_cpu_bind_policy;
  if (required != KE_CPU_BIND_UNSET) bind = required;
  if (bind == KE_CPU_BIND_FULL_PCPUS || bind == KE_CPU_BIND_SPREAD_BY_PCPUS) {
    if (cpu % 1000 != 0) {
      st->invalid = 1;
      return;
    }
    if (cpu > 0) {
      st->rcb = 1;
      st->required = required;
      st->preferred = bind;
      st->excl = pod->cpu_exclusive;
    }
  }
}

/* requestCPUBind (util.go:121-138): -1 = UnschedulableAndUnresolvable (non-integer cpus) */
static int request_cpu_bind(const cpuset_state* st, const ke_pod* pod, int node_bind) {
  if (st->rcb) return 1;
  const int64_t cpu = pod->requests[KE_RES_CPU];
  if (cpu == 0) return 0;
  if (node_bind != KE_NODE_CPU_BIND_NONE) return cpu % 1000 != 0 ? -1 : 1;
  return 0;
}

static int cpus_valid(const or_node* n) {
  return n->cpus && !n->node.cpu_topology_invalid && n->cpus->t.num_sockets && n->cpus->t.num_nodes &&
         n->cpus->t.num_cores && n->cpus->t.num_cpus;
}

/* NodeAllocation.NUMANodeSharedStatus (node_allocation.go:60-68) from the sizes of the zone's
 * singleNUMANode / sharedNode pod sets */
static uint8_t zone_status_of(const ke_numa_zone* z) {
  if (z->shared_pods > 0) return KE_NUMA_STATUS_SHARED;
  return z->single_pods > 0 ? KE_NUMA_STATUS_SINGLE : KE_NUMA_STATUS_IDLE;
}

/* GetAvailableCPUs(node) allocated.CPUs().Size() (resource_manager.go:497-511) */
static int64_t cpus_allocated_count(const or_node* n) {
  if (!n->cpus) return n->node.cpuset_allocated_cpus;
  int64_t k = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) k += n->cpus->al.present[c];
  return k;
}

/* getCPUBindPolicy (util.go:101-119): the policy and whether it is required */
static int cpu_bind_policy_of(const cpuset_state* st, int node_bind, int* required) {
  if (st->required != KE_CPU_BIND_UNSET) {
    *required = 1;
    return st->required;
  }
  *required = 0;
  if (node_bind == KE_NODE_CPU_BIND_SPREAD_BY_PCPUS) {
    *required = 1;
    return KE_CPU_BIND_SPREAD_BY_PCPUS;
  }
  if (node_bind == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY) {
    *required = 1;
    return KE_CPU_BIND_FULL_PCPUS;
  }
  return st->preferred;
}

static int acc_bind(int bind) {
  return bind == KE_CPU_BIND_FULL_PCPUS ? ACC_BIND_FULL_PCPUS
                                        : bind == KE_CPU_BIND_SPREAD_BY_PCPUS ? ACC_BIND_SPREAD_BY_PCPUS : ACC_BIND_NONE;
}

/* GetNUMAAllocateStrategy (util.go:33-47): 1 = NUMAMostAllocated */
static int numa_most_allocated(const or_cluster* c, const or_node* n) {
  if (n->node.numa_allocate_strategy == KE_NUMA_ALLOCATE_MOST) return 1;
  if (n->node.numa_allocate_strategy == KE_NUMA_ALLOCATE_LEAST) return 0;
  return c->cfg.numa.numa_strategy == KE_STRATEGY_MOST_ALLOCATED;
}

/* a node's NUMA zones as getResourceOptions / getAvailableNUMANodeResources see them */
typedef struct numa_view {
  int n;
  int id[KE_MAX_NUMA];
  uint8_t cap_has[KE_MAX_NUMA][KE_NRES];
  int64_t cap[KE_MAX_NUMA][KE_NRES];     /* amplified NUMANodeResources (amplifyNUMANodeResources) */
  uint8_t av_has[KE_MAX_NUMA][KE_NRES];
  int64_t av[KE_MAX_NUMA][KE_NRES];      /* totalAvailable */
  int has_alloc[KE_MAX_NUMA];
  int64_t al[KE_MAX_NUMA][KE_NRES];      /* totalAllocated (cpu adjusted for amplified cpusets) */
  uint8_t al_has[KE_MAX_NUMA][KE_NRES];
  double ratio;                          /* TopologyOptions.AmplificationRatios[cpu] */
} numa_view;

/* The cpuset part of ResourceOptions for a pod that binds CPUs on the node (getResourceOptions
 * plugin.go:629-668, getCPUBindPolicy util.go:101-119) and the CPUs allocateCPUSet may take:
 * GetAvailableCPUs filtered by a required bind policy (resource_manager.go:353-377), per NUMA id. */
typedef struct numa_cs {
  int rcb;             /* requestCPUBind */
  int valid;           /* the node's CPU topology is valid */
  int required, bind;  /* requiredCPUBindPolicy, cpuBindPolicy (KE_CPU_BIND_*) */
  int num_cpus, cpc, excl, numa_most;
  int avail_total;
  int zcnt[KE_MAX_NUMA];
  uint64_t avail[ACC_WORDS];
  /* ResourceOptions.preferredCPUs (reservations) and the allocateInfo getAvailableCPUs returns with them
   * (RefCount-- per preferred CPU, dropped at 0); has_pref = 0: the node's own allocation, no preferred CPUs */
  int has_pref;
  uint64_t pref[ACC_WORDS];
  acc_alloc al;
} numa_cs;

static int exact_cpusets = 0; /* hints / admit run the CPU accumulator itself instead of its counts */
void or_set_exact_cpusets(int on) { exact_cpusets = on; }

static int popcount_set(const uint64_t* s) {
  int n = 0;
  for (int w = 0; w < ACC_WORDS; w++) n += __builtin_popcountll(s[w]);
  return n;
}

static void numa_cs_build_pref(const or_cluster* c, const or_node* n, const ke_pod* pod, numa_cs* cs,
                               const uint64_t* pref);
static void numa_cs_build(const or_cluster* c, const or_node* n, const ke_pod* pod, numa_cs* cs) {
  numa_cs_build_pref(c, n, pod, cs, NULL);
}
/* with ResourceOptions.preferredCPUs: getAvailableCPUs(preferredCPUs) (node_allocation.go:192-219) */
static void numa_cs_build_pref(const or_cluster* c, const or_node* n, const ke_pod* pod, numa_cs* cs,
                               const uint64_t* pref) {
  memset(cs, 0, sizeof *cs);
  cpuset_state st;
  cpuset_prefilter(c, pod, &st);
  if (request_cpu_bind(&st, pod, n->node.cpu_bind_policy) <= 0) return;
  cs->rcb = 1;
  cs->valid = cpus_valid(n);
  cs->num_cpus = st.num_cpus;
  cs->excl = st.excl;
  cs->bind = cpu_bind_policy_of(&st, n->node.cpu_bind_policy, &cs->required);
  cs->numa_most = numa_most_allocated(c, n);
  if (!cs->valid) return;
  const or_cpus* x = n->cpus;
  cs->cpc = acc_cpus_per_core(&x->t);
  cs->al = x->al;
  if (pref) {
    cs->has_pref = 1;
    memcpy(cs->pref, pref, sizeof cs->pref);
    for (int c1 = 0; c1 < ACC_MAX_CPUS; c1++)
      if ((pref[c1 >> 6] >> (c1 & 63) & 1) && cs->al.present[c1] && --cs->al.ref[c1] == 0) {
        cs->al.present[c1] = 0;
        cs->al.excl[c1] = 0;
      }
  }
  memset(cs->avail, 0, sizeof cs->avail);
  for (int c1 = 0; c1 < ACC_MAX_CPUS; c1++)
    if (x->t.valid[c1] && !x->reserved[c1] && !(cs->al.present[c1] && cs->al.ref[c1] >= x->max_ref))
      cs->avail[c1 >> 6] |= 1ull << (c1 & 63);
  if (cs->required) { /* filterCPUsByRequiredCPUBindPolicy (:655-695) */
    uint64_t keep[ACC_WORDS] = {0};
    for (int c1 = 0; c1 < ACC_MAX_CPUS; c1++) {
      if (!(cs->avail[c1 >> 6] >> (c1 & 63) & 1)) continue;
      int in_core = 0, lowest = 1;
      for (int c2 = 0; c2 < ACC_MAX_CPUS; c2++)
        if ((cs->avail[c2 >> 6] >> (c2 & 63) & 1) && x->t.core[c2] == x->t.core[c1]) {
          in_core++;
          if (c2 < c1) lowest = 0;
        }
      if ((cs->bind == KE_CPU_BIND_FULL_PCPUS && in_core == cs->cpc) || (cs->bind == KE_CPU_BIND_SPREAD_BY_PCPUS && lowest) ||
          (cs->bind != KE_CPU_BIND_FULL_PCPUS && cs->bind != KE_CPU_BIND_SPREAD_BY_PCPUS))
        keep[c1 >> 6] |= 1ull << (c1 & 63);
    }
    memcpy(cs->avail, keep, sizeof keep);
  }
  cs->avail_total = popcount_set(cs->avail);
  for (int c1 = 0; c1 < ACC_MAX_CPUS; c1++)
    if ((cs->avail[c1 >> 6] >> (c1 & 63) & 1) && x->t.node[c1] >= 0 && x->t.node[c1] < KE_MAX_NUMA)
      cs->zcnt[x->t.node[c1]]++;
}

/* satisfiedRequiredCPUBindPolicy (:697-718) */
static int cpuset_satisfied(const numa_cs* cs, const or_cpus* x, const uint64_t* result) {
  if (!cs->required) return 1;
  int ncpu = 0, cores[ACC_MAX_CPUS], ncore = 0;
  for (int c1 = 0; c1 < ACC_MAX_CPUS; c1++) {
    if (!(result[c1 >> 6] >> (c1 & 63) & 1)) continue;
    ncpu++;
    int f = 0;
    for (int k = 0; k < ncore && !f; k++) f = cores[k] == x->t.core[c1];
    if (!f) cores[ncore++] = x->t.core[c1];
  }
  if (cs->bind == KE_CPU_BIND_FULL_PCPUS && ncore * cs->cpc != ncpu) return 0;
  if (cs->bind == KE_CPU_BIND_SPREAD_BY_PCPUS && ncore != ncpu) return 0;
  return 1;
}

/* allocateCPUSet (resource_manager.go:353-459): with the pod's NUMA allocation `dist` (zones of the
 * view with a non-zero amount, ascending id) a takePreferredCPUs per zone over its available CPUs,
 * then the remainder over the node.  0 and the cpuset, or -1. */
static int cpuset_allocate_cs(const or_node* n, const numa_cs* cs, const numa_view* v,
                              const int64_t (*dist)[KE_NRES], uint64_t* result) {
  const or_cpus* x = n->cpus;
  memset(result, 0, sizeof(uint64_t) * ACC_WORDS);
  if (cs->avail_total < cs->num_cpus) return -1;
  int needed = cs->num_cpus, any = 0;
  for (int z = 0; dist && z < v->n; z++) {
    if (dist[z][0] == 0 && dist[z][1] == 0) continue;
    any = 1;
    uint64_t az[ACC_WORDS] = {0}, got[ACC_WORDS];
    for (int c1 = 0; c1 < ACC_MAX_CPUS; c1++)
      if ((cs->avail[c1 >> 6] >> (c1 & 63) & 1) && x->t.node[c1] == v->id[z]) az[c1 >> 6] |= 1ull << (c1 & 63);
    int k = popcount_set(az);
    const int want = (int)(dist[z][KE_RES_CPU] / 1000);
    if (want < k) k = want;
    if (acc_take_preferred_cpus(&x->t, x->max_ref, az, cs->has_pref ? cs->pref : NULL, &cs->al, k, acc_bind(cs->bind),
                                cs->excl, cs->numa_most, got) != 0)
      return -1;
    for (int w = 0; w < ACC_WORDS; w++) result[w] |= got[w];
  }
  if (any) {
    needed -= popcount_set(result);
    if (needed != 0) return -1;
  }
  if (needed > 0) {
    uint64_t rest[ACC_WORDS], got[ACC_WORDS];
    for (int w = 0; w < ACC_WORDS; w++) rest[w] = cs->avail[w] & ~result[w];
    if (acc_take_preferred_cpus(&x->t, x->max_ref, rest, cs->has_pref ? cs->pref : NULL, &cs->al, needed,
                                acc_bind(cs->bind), cs->excl, cs->numa_most, got) != 0)
      return -1;
    for (int w = 0; w < ACC_WORDS; w++) result[w] |= got[w];
  }
  return cpuset_satisfied(cs, x, result) ? 0 : -1;
}

/* The same outcome from counts: per zone takeCPUs over k <= |available| CPUs never
 * fails and takes exactly k; a required FullPCPUs result is whole cores iff every zone's k is a
 * multiple of CPUs per core (whole cores are all a zone offers then); SpreadByPCPUs offers one CPU per
 * core.  Verified against cpuset_allocate_cs by tests/test_oracle_cpuset_numa.py. */
static int cpuset_fits_cs(const or_node* n, const numa_cs* cs, const numa_view* v, const int64_t (*dist)[KE_NRES]) {
  if (exact_cpusets || cs->has_pref) {
    uint64_t r[ACC_WORDS];
    return cpuset_allocate_cs(n, cs, v, dist, r) == 0;
  }
  if (cs->avail_total < cs->num_cpus) return 0;
  int taken = 0, any = 0, aligned = 1;
  for (int z = 0; dist && z < v->n; z++) {
    if (dist[z][0] == 0 && dist[z][1] == 0) continue;
    any = 1;
    int k = v->id[z] < KE_MAX_NUMA ? cs->zcnt[v->id[z]] : 0;
    const int want = (int)(dist[z][KE_RES_CPU] / 1000);
    if (want < k) k = want;
    if (k <= 0) continue;
    taken += k;
    if (k % cs->cpc) aligned = 0;
  }
  if (!any) return 1; /* the whole-node take: FullPCPUs is SMT-aligned after Filter */
  if (taken != cs->num_cpus) return 0;
  return !(cs->required && cs->bind == KE_CPU_BIND_FULL_PCPUS && !aligned);
}

/* allocateCPUSet without a NUMA allocation (policy None) */
static int cpuset_allocate(const or_cluster* c, const or_node* n, const ke_pod* pod, uint64_t* result) {
  numa_cs cs;
  numa_cs_build(c, n, pod, &cs);
  return cpuset_allocate_cs(n, &cs, NULL, NULL, result);
}
/* ... with ResourceOptions.preferredCPUs */
static int cpuset_allocate_pref(const or_cluster* c, const or_node* n, const ke_pod* pod, const uint64_t* pref,
                                uint64_t* result) {
  numa_cs cs;
  numa_cs_build_pref(c, n, pod, &cs, pref);
  return cpuset_allocate_cs(n, &cs, NULL, NULL, result);
}

static int or_holds_of_idx(const or_cluster* c, int32_t r);
static int or_resv_usable(const ke_reservation* r);

/* tryAllocateIgnoreReservation for a reservation-ignored binding pod on a node without a NUMA policy
 * (nodenumaresource/reservation.go:437-490; the hint is empty, so the held NUMA amounts do not enter): over
 * RestoreReservation's matched set -- every usable reservation on the node whose reserve pod holds NUMA resources or
 * a cpuset -- one Allocate with reservedCPUsFromIgnored (their allocatable CPUs, the remainedCPUs inside them)
 * preferred and no required resources; its status is the Filter's (plugin.go:384-387) and Reserve's: 1 and the
 * cpuset, or -1.  An empty set gives 0 (tryAllocateFromNode). */
static int or_numa_ignored(const or_cluster* c, const ke_pod* pod, int32_t node, uint64_t* out) {
  const or_node* n = &c->nodes[node];
  uint64_t pref[ACC_WORDS] = {0}, got[ACC_WORDS];
  int any = 0;
  for (int32_t r = 0; c->ralloc && r < c->n_resv; r++) {
    if (c->resv[r].node != node || !or_resv_usable(&c->resv[r]) ||
        !(or_holds_of_idx(c, r) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)))
      continue;
    any = 1;
    for (int w = 0; w < ACC_WORDS; w++) pref[w] |= c->ralloc[r].cpuset[w];
  }
  if (!any) return 0;
  if (cpuset_allocate_pref(c, n, pod, pref, got) != 0) return -1;
  memcpy(out, got, sizeof got);
  return 1;
}

/* NodeNUMAResource's allocate-from-reservation for a binding pod on a node without a NUMA policy
 * (tryAllocateFromReservation, nodenumaresource/reservation.go:270-424; the hint is empty, so Allocate is
 * allocateCPUSet alone and the NUMA restore states do not enter): over RestoreReservation's matched set --
 * the pod's matched reservations (c->resv_m) on the node whose reserve pod holds NUMA resources or a cpuset
 * -- or only reservation `only` (the nominated one, allocateWithNominatedReservation :492-522, and
 * FilterNominateReservation, plugin.go:448-504), each with
 *   preferredCPUs = mergedMatchedAllocatedCPUs (the matched reservations' allocatedCPUs, i.e. their
 *                   allocatable CPUs: or_restore_state) ∪ its remainedCPUs;
 *   Default / Aligned: one Allocate;  Restricted: that Allocate, then numCPUsNeeded <= |remainedCPUs|, then an
 *   Allocate with preferredCPUs = remainedCPUs whose cpuset may not outgrow them.
 * The first satisfied one (ascending index; Go ranges over a map, so only whether one is satisfied is the
 * reference's -- the Filter's question) gives 1 and its cpuset; none: -1 with requiredFromReservation (the
 * Filter's "Reservation(s) ..." Unschedulable), else 0 (nil: the node itself, tryAllocateFromNode).  An empty
 * matched set gives 0 whatever the requirement. */
static int or_numa_from_rsv(const or_cluster* c, const ke_pod* pod, int32_t node, int32_t only, int required,
                            uint64_t* out) {
  const or_node* n = &c->nodes[node];
  uint64_t merged[ACC_WORDS] = {0};
  int any = 0;
  for (int32_t r = 0; c->resv_m && c->ralloc && r < c->n_resv; r++) {
    if (!c->resv_m[r] || c->resv[r].node != node || !(or_holds_of_idx(c, r) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)))
      continue;
    any = 1;
    for (int w = 0; w < ACC_WORDS; w++) merged[w] |= c->ralloc[r].cpuset[w];
  }
  if (!any) return 0;
  if (only >= 0 && !(c->resv_m[only] && c->resv[only].node == node &&
                     (or_holds_of_idx(c, only) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET))))
    return 0; /* "nominated reservation doesn't reserve numa resource or cpuset" */
  for (int32_t r = 0; r < c->n_resv; r++) {
    if (only >= 0 ? r != only : !(c->resv_m[r] && c->resv[r].node == node &&
                                  (or_holds_of_idx(c, r) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET))))
      continue;
    const ke_reservation_alloc* a = &c->ralloc[r];
    uint64_t rem[ACC_WORDS], pref[ACC_WORDS], got[ACC_WORDS];
    for (int w = 0; w < ACC_WORDS; w++) {
      rem[w] = a->cpuset[w] & ~a->owner_cpuset[w];
      pref[w] = merged[w] | rem[w];
    }
    if (cpuset_allocate_pref(c, n, pod, pref, got) != 0) continue;
    if (c->resv[r].allocate_policy == KE_RSV_POLICY_RESTRICTED) {
      cpuset_state st;
      cpuset_prefilter(c, pod, &st);
      const int reserved = popcount_set(rem);
      if (st.num_cpus > reserved) continue; /* numCPUsNeeded > reservedCPUs.Size() */
      if (cpuset_allocate_pref(c, n, pod, rem, got) != 0) continue;
      if (popcount_set(got) > reserved) continue;
    }
    memcpy(out, got, sizeof got);
    return 1;
  }
  return required ? -1 : 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* LoadAwareScheduling                                                                             */
/* ---------------------------------------------------------------------------------------------- */

/* Plugin.Filter  load_aware.go:122-186 and filterNodeUsage :290-313 */
int or_la_filter(const or_cluster* c, const ke_pod* pod, int32_t node, int64_t now, int* reason) {
  const ke_loadaware_args* a = &c->cfg.loadaware;
  const or_node* n = &c->nodes[node];
  *reason = KE_REASON_NONE;
  if (pod->is_daemonset) return KE_CODE_SUCCESS;
  if (!n->has_metric) return KE_CODE_SUCCESS; /* NotFound: skip load-aware */
  if (a->filter_expired_node_metrics && a->node_metric_expiration_seconds != KE_ABSENT &&
      node_metric_expired(n, a->node_metric_expiration_seconds, now)) {
    if (!a->enable_schedule_when_node_metrics_expired) {
      *reason = KE_REASON_LA_NODEMETRIC_EXPIRED;
      return KE_CODE_UNSCHEDULABLE;
    }
    return KE_CODE_SUCCESS;
  }
  if (!n->nm.has_node_metric) return KE_CODE_SUCCESS;

  int64_t alloc[KE_NRES];
  estimate_node(&n->node, alloc);
  filter_profile prof;
  filter_profile_of(a, &n->node, &prof);
  const int prod_pod = any_present(prof.prod) && pod->priority_class == KE_PRIORITY_PROD;
  const ke_resource_map* usage = NULL;
  const int64_t* thr;
  if (prod_pod) {
    thr = prof.prod;
  } else if (prof.has_agg) {
    usage = target_aggregated_usage(n, prof.agg_dur, prof.agg_type);
    thr = prof.agg_thr;
  } else {
    usage = &n->nm.node_usage;
    thr = prof.usage;
  }
  int64_t used[KE_NRES];
  get_estimated_used(a, n, pod, usage, prod_pod, now, used);
  /* Go iterates the threshold map in random order; the first exceeding resource names the reason.
   * Pass/fail is order independent; this restatement reports cpu before memory. */
  for (int r = 0; r < KE_NRES; r++) {
    int64_t v = thr[r];
    if (v == KE_ABSENT || v == 0) continue;
    int64_t total = alloc[r];
    if (total == 0) continue;
    int64_t pct = or_usage_percent(used[r], total);
    if (pct <= v) continue;
    if (!prod_pod && prof.has_agg)
      *reason = r == KE_RES_CPU ? KE_REASON_LA_AGG_USAGE_CPU : KE_REASON_LA_AGG_USAGE_MEMORY;
    else
      *reason = r == KE_RES_CPU ? KE_REASON_LA_USAGE_CPU : KE_REASON_LA_USAGE_MEMORY;
    return KE_CODE_UNSCHEDULABLE;
  }
  return KE_CODE_SUCCESS;
}

/* leastUsedScore  load_aware.go:397-406 */
static int64_t least_used_score(int64_t used, int64_t capacity) {
  if (capacity == 0) return 0;
  if (used > capacity) return 0;
  return ((capacity - used) * MAX_NODE_SCORE) / capacity;
}

/* Plugin.Score  load_aware.go:201-249, loadAwareSchedulingScorer :387-395 */
int64_t or_la_score(const or_cluster* c, const ke_pod* pod, int32_t node, int64_t now) {
  const ke_loadaware_args* a = &c->cfg.loadaware;
  const or_node* n = &c->nodes[node];
  if (!n->has_metric) return 0;
  if (a->node_metric_expiration_seconds != KE_ABSENT && node_metric_expired(n, a->node_metric_expiration_seconds, now))
    return 0;
  if (!n->nm.has_node_metric) return 0;
  const int prod_pod = pod->priority_class == KE_PRIORITY_PROD && a->score_according_prod_usage;
  const ke_resource_map* usage = NULL;
  if (!prod_pod) {
    if (score_with_aggregation(a)) usage = target_aggregated_usage(n, a->agg_score_duration_ns, a->agg_score_type);
    else usage = &n->nm.node_usage;
  }
  int64_t used[KE_NRES], alloc[KE_NRES];
  get_estimated_used(a, n, pod, usage, prod_pod, now, used);
  estimate_node(&n->node, alloc);
  int64_t score = 0, wsum = 0;
  for (int r = 0; r < KE_NRES; r++) {
    int64_t w = a->resource_weights[r];
    if (w == KE_ABSENT) continue;
    score += least_used_score(used[r], alloc[r]) * w;
    wsum += w;
  }
  return wsum ? score / wsum : 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* NodeNUMAResource (NUMA policy None, non-cpuset pods)                                             */
/* ---------------------------------------------------------------------------------------------- */

static int pod_requests_zero(const ke_pod* pod) { /* quotav1.IsZero(PodRequests)  plugin.go:262-268 */
  if (pod->has_other_requests) return 0;
  for (int r = 0; r < KE_RES_COUNT; r++)
    if (pod->requests[r] != 0) return 0;
  return 1;
}

/* Plugin.Filter  plugin.go:318-406 -> filterAmplifiedCPUs :408-442 */
static int numa_filter_amplified(const or_node* n, const ke_pod* pod, int rcb, int* reason);
/* DeviceShare as a NUMA hint provider (defined with DeviceShare below) */
struct numa_hint;
static int ds_numa_hints(const or_cluster* c, const or_node* nd, const ke_pod* pod, struct numa_hint* list, int* n,
                         int* copies, int* none, int* reason);
static int ds_numa_allocate(const or_cluster* c, const or_node* nd, const ke_pod* pod, uint32_t affinity, int* reason);
static int numa_stored_affinity(const or_cluster* c, const ke_pod* pod, int32_t node, uint32_t* aff);
static int numa_admit(const or_cluster* c, const or_node* nd, const ke_pod* pod, int policy, int exclusive,
                      uint32_t* affinity, int* reason, const numa_cs* cs);

/* getNUMATopologyPolicy + mergeTopologyPolicy (util.go:58-74) and the exclusive default of
 * Filter (plugin.go:330-336): -1 on a node / pod policy conflict. */
static int effective_policy(const or_node* n, const ke_pod* pod, int* exclusive) {
  const int np = n->node.numa_topology_policy, pp = pod->numa_topology_policy;
  *exclusive = pod->numa_exclusive;
  if (*exclusive == KE_NUMA_EXCLUSIVE_NONE && pp != KE_NUMA_POLICY_NONE) *exclusive = KE_NUMA_EXCLUSIVE_REQUIRED;
  if (np != KE_NUMA_POLICY_NONE && pp != KE_NUMA_POLICY_NONE && pp != np) return -1;
  return pp != KE_NUMA_POLICY_NONE ? pp : np;
}

/* Filter's path; *stored = topologymanager Admit ran and stored *aff (0 = nil NUMANodeAffinity) */
static int numa_filter_aff(const or_cluster* c, const ke_pod* pod, int32_t node, int* reason, int* stored,
                           uint32_t* aff_out);
int or_numa_filter(const or_cluster* c, const ke_pod* pod, int32_t node, int* reason) {
  int stored;
  uint32_t aff;
  return numa_filter_aff(c, pod, node, reason, &stored, &aff);
}

/* The affinity NodeNUMAResource's Filter stores for the pod on the node (topologymanager Store,
 * manager.go:64-95): 1 when its Filter passes through Admit, *aff = the NUMANodeAffinity (0 = nil). */
static int numa_stored_affinity(const or_cluster* c, const ke_pod* pod, int32_t node, uint32_t* aff) {
  int reason, stored;
  const int code = numa_filter_aff(c, pod, node, &reason, &stored, aff);
  return code == KE_CODE_SUCCESS && stored;
}

static int numa_filter_aff(const or_cluster* c, const ke_pod* pod, int32_t node, int* reason, int* stored,
                           uint32_t* aff_out) {
  const or_node* n = &c->nodes[node];
  *reason = KE_REASON_NONE;
  *stored = 0;
  *aff_out = 0;
  if (pod_requests_zero(pod)) return KE_CODE_SUCCESS; /* state.skip */
  cpuset_state st;
  cpuset_prefilter(c, pod, &st);
  if (st.invalid) { /* PreFilter (plugin.go:296-298) */
    *reason = KE_REASON_NUMA_INVALID_REQUESTED_CPUS;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  int exclusive;
  const int policy = effective_policy(n, pod, &exclusive);
  if (policy < 0) {
    *reason = KE_REASON_NUMA_POLICY_CONFLICT;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  const int rcb = request_cpu_bind(&st, pod, n->node.cpu_bind_policy);
  if (rcb < 0) {
    *reason = KE_REASON_NUMA_INVALID_REQUESTED_CPUS;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  const int code = numa_filter_amplified(n, pod, rcb, reason);
  if (code != KE_CODE_SUCCESS) return code;
  if (rcb) { /* plugin.go:351-398 */
    if (!cpus_valid(n)) {
      *reason = KE_REASON_NUMA_INVALID_CPU_TOPOLOGY;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    int required = st.required;
    if (n->node.cpu_bind_policy == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = KE_CPU_BIND_FULL_PCPUS;
    else if (n->node.cpu_bind_policy == KE_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = KE_CPU_BIND_SPREAD_BY_PCPUS;
    if (st.required != KE_CPU_BIND_UNSET && st.required != required) {
      *reason = KE_REASON_NUMA_CPU_BIND_POLICY_CONFLICT;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    if (required == KE_CPU_BIND_FULL_PCPUS && st.num_cpus % acc_cpus_per_core(&n->cpus->t) != 0) {
      *reason = KE_REASON_NUMA_SMT_ALIGNMENT;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    if (required != KE_CPU_BIND_UNSET && policy == KE_NUMA_POLICY_NONE) { /* trial Allocate */
      uint64_t cs[ACC_WORDS];
      /* from the matched reservations first (plugin.go:381-390), then the node (tryAllocateFromNode) */
      const int fr = c->ignored ? or_numa_ignored(c, pod, node, cs)
                                : or_numa_from_rsv(c, pod, node, -1, pod->reservation_matched == KE_RSV_AFFINITY, cs);
      if (fr < 0) {
        *reason = KE_REASON_RSV_INSUFFICIENT_CPUS;
        return KE_CODE_UNSCHEDULABLE;
      }
      if (fr > 0) return KE_CODE_SUCCESS;
      if (cpuset_allocate(c, n, pod, cs) != 0) {
        *reason = KE_REASON_NUMA_INSUFFICIENT_CPUS;
        return KE_CODE_UNSCHEDULABLE;
      }
      return KE_CODE_SUCCESS;
    }
  }
  if (policy == KE_NUMA_POLICY_NONE) return KE_CODE_SUCCESS;
  if (n->n_zone == 0) { /* FilterByNUMANode  topology_hint.go:31-41 */
    *reason = KE_REASON_NUMA_MISSING_RESOURCES;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  uint32_t aff;
  numa_cs cs;
  numa_cs_build(c, n, pod, &cs);
  const int admit_code = numa_admit(c, n, pod, policy, exclusive, &aff, reason, &cs);
  if (admit_code == KE_CODE_SUCCESS) {
    *stored = 1;
    *aff_out = aff;
  }
  return admit_code;
}

/* filterAmplifiedCPUs  plugin.go:408-442 */
static int numa_filter_amplified(const or_node* n, const ke_pod* pod, int rcb, int* reason) {
  int64_t pod_cpu = pod->requests[KE_RES_CPU];
  if (pod_cpu == 0) return KE_CODE_SUCCESS;
  if (n->node.amplification_error) {
    *reason = KE_REASON_NUMA_INVALID_AMPLIFICATION_RATIO;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  const double ratio = n->node.cpu_amplification_ratio;
  if (ratio <= 1.0) return KE_CODE_SUCCESS;
  if (n->node.cpu_topology_invalid) { /* GetAvailableCPUs error, resource_manager.go:502-504 */
    *reason = KE_REASON_NUMA_INVALID_CPU_TOPOLOGY;
    return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
  }
  if (rcb) pod_cpu = amplify(pod_cpu, ratio);
  const int64_t allocated_milli = cpus_allocated_count(n) * 1000;
  int64_t requested = n->node.requested[KE_RES_CPU] + n->rv_req[KE_RES_CPU]; /* NodeInfo after the restore */
  if (requested >= allocated_milli && allocated_milli > 0) {
    requested = requested - allocated_milli;
    requested += amplify(allocated_milli, ratio);
  }
  if (pod_cpu > n->node.allocatable[KE_RES_CPU] - requested) {
    *reason = KE_REASON_NUMA_INSUFFICIENT_AMPLIFIED_CPU;
    return KE_CODE_UNSCHEDULABLE;
  }
  return KE_CODE_SUCCESS;
}

/* resourceAllocationScorer.score (scoring.go:210-226) with least/mostResourceScorer
 * (least_allocated.go:30-58, most_allocated.go:30-62) over cpu and memory. */
static int64_t numa_resource_score_as(const ke_numa_args* na, int strategy, const int64_t* requested,
                                      const int64_t* allocatable, const int64_t* podreq) {
  int64_t score = 0, wsum = 0;
  for (int r = 0; r < KE_NRES; r++) {
    int64_t w = na->weights[r];
    if (w == KE_ABSENT) continue;
    int64_t alloc = allocatable[r];
    int64_t req = requested[r] + podreq[r];
    if (alloc == 0) continue; /* calculateResourceAllocatableRequest result dropped */
    int64_t s;
    if (strategy == KE_STRATEGY_MOST_ALLOCATED) {
      int64_t rq = req > alloc ? alloc : req;
      s = (rq * MAX_NODE_SCORE) / alloc;
    } else {
      s = req > alloc ? 0 : ((alloc - req) * MAX_NODE_SCORE) / alloc;
    }
    score += s * w;
    wsum += w;
  }
  return wsum ? score / wsum : 0;
}
static int64_t numa_resource_score(const ke_numa_args* na, const int64_t* requested, const int64_t* allocatable,
                                   const int64_t* podreq) {
  return numa_resource_score_as(na, na->strategy, requested, allocatable, podreq);
}

/* ---------------------------------------------------------------------------------------------- */
/* NUMA topology policies for non-cpuset pods: GetPodTopologyHints (topology_hint.go:43-76,          */
/* resource_manager.go:130-192,525-653), topologymanager Admit / Merge (manager.go:64-129,          */
/* policy*.go), Allocate by hint (resource_manager.go:194-330), NUMA-scope Score (scoring.go:141-187) */
/* ---------------------------------------------------------------------------------------------- */




/* allocatedCPUs.CPUsInNUMANodes(id).Size(): from the CPU table when the node has one */
static int zone_cpusets(const or_node* nd, int id, int given) {
  if (!nd->cpus) return given;
  int k = 0;
  for (int c = 0; c < ACC_MAX_CPUS; c++) k += nd->cpus->al.present[c] && nd->cpus->t.node[c] == id;
  return k;
}

/* getResourceOptions -> amplifyNUMANodeResources (util.go:78-98) + getAvailableNUMANodeResources
 * (node_allocation.go:221-243).  Returns -1 on an amplification-ratio annotation error. */
/* ResourceOptions beyond the node's own restore state, for NodeNUMAResource's allocate-from-reservation
 * (nodenumaresource/reservation.go:270-424, resource_manager.go:130-138): reusableResources added to the restore
 * state's (quotav1.Add per NUMA id: keys of both), requiredResources replacing totalAvailable
 * (allocateResourcesByHint, resource_manager.go:226-254), preferredCPUs (numa_cs_build_pref). */
typedef struct numa_opt {
  int64_t reuse[KE_MAX_NUMA][KE_NRES];
  uint8_t reuse_key[KE_MAX_NUMA][KE_NRES];
  int has_req;
  int64_t req[KE_MAX_NUMA][KE_NRES];
  uint8_t req_key[KE_MAX_NUMA][KE_NRES];
  int has_pref;
  uint64_t pref[ACC_WORDS];
} numa_opt;

static int numa_view_build_opt(const or_node* nd, numa_view* v, const numa_cs* cs, const numa_opt* opt);
static int numa_view_build(const or_node* nd, numa_view* v, const numa_cs* cs) {
  return numa_view_build_opt(nd, v, cs, NULL);
}
static int numa_view_build_opt(const or_node* nd, numa_view* v, const numa_cs* cs, const numa_opt* opt) {
  memset(v, 0, sizeof *v);
  double ratio;
  int amplify_caps = 0;
  if (nd->node.nrt_cpu_amplification_ratio > -1.5) { /* TopologyOptions.AmplificationRatios != nil */
    ratio = nd->node.nrt_cpu_amplification_ratio < 0 ? 0.0 : nd->node.nrt_cpu_amplification_ratio;
  } else {
    if (nd->node.amplification_error) return -1;
    ratio = nd->node.cpu_amplification_ratio < 0 ? 0.0 : nd->node.cpu_amplification_ratio;
    amplify_caps = 1;
  }
  v->ratio = ratio;
  v->n = nd->n_zone;
  for (int z = 0; z < nd->n_zone; z++) {
    const ke_numa_zone* zn = &nd->zone[z];
    v->id[z] = zn->id;
    for (int r = 0; r < KE_NRES; r++) {
      v->cap_has[z][r] = zn->has[r];
      v->cap[z][r] = zn->has[r] ? zn->capacity[r] : 0;
    }
    if (amplify_caps && ratio > 1.0 && v->cap_has[z][KE_RES_CPU] && v->cap[z][KE_RES_CPU] != 0)
      v->cap[z][KE_RES_CPU] = amplify(v->cap[z][KE_RES_CPU], ratio);
    v->has_alloc[z] = (zn->has_allocated & KE_NUMA_ALLOC_ENTRY) != 0;
    if (v->has_alloc[z]) {
      int64_t al[KE_NRES];
      uint8_t has[KE_NRES];
      for (int r = 0; r < KE_NRES; r++) {
        has[r] = (zn->has_allocated & (r == KE_RES_CPU ? KE_NUMA_ALLOC_CPU : KE_NUMA_ALLOC_MEMORY)) != 0;
        al[r] = has[r] ? zn->allocated[r] : 0;
      }
      if (ratio > 1.0) { /* the cpu key is (re)written even when the entry had none */
        const int64_t cs = (int64_t)zone_cpusets(nd, zn->id, zn->cpuset_cpus) * 1000;
        al[KE_RES_CPU] = al[KE_RES_CPU] - cs + amplify(cs, ratio);
        has[KE_RES_CPU] = 1;
      }
      /* SubtractWithNonNegativeResult(allocated, reusableResources[id]) (node_allocation.go:237): the pod's
       * restore state (or_restore) -- keys of both, floor 0 */
      const int zid = zn->id >= 0 && zn->id < KE_MAX_NUMA ? zn->id : -1;
      for (int r = 0; r < KE_NRES; r++) {
        const int rk0 = zid >= 0 && nd->rs_numa_has[zid] && nd->rs_numa_key[zid][r];
        const int rk1 = zid >= 0 && opt && opt->reuse_key[zid][r];
        const int64_t reuse = (rk0 ? nd->rs_numa[zid][r] : 0) + (rk1 ? opt->reuse[zid][r] : 0);
        const int64_t q = (has[r] ? al[r] : 0) - reuse;
        v->al_has[z][r] = has[r] || rk0 || rk1;
        v->al[z][r] = v->al_has[z][r] && q > 0 ? q : 0;
      }
    }
    for (int r = 0; r < KE_NRES; r++) { /* SubtractWithNonNegativeResult(capacity, allocated) */
      const int64_t a = v->al_has[z][r] ? v->al[z][r] : 0;
      v->av_has[z][r] = v->cap_has[z][r] || v->al_has[z][r];
      const int64_t q = v->cap_has[z][r] ? v->cap[z][r] - a : -a;
      v->av[z][r] = q > 0 ? q : 0;
    }
    if (opt && opt->has_req) /* totalAvailable = requiredResources: its NUMA ids and keys, signed (quotav1.Subtract) */
      for (int r = 0; r < KE_NRES; r++) {
        const int in = zn->id >= 0 && zn->id < KE_MAX_NUMA && opt->req_key[zn->id][r];
        v->av_has[z][r] = (uint8_t)in;
        v->av[z][r] = in ? opt->req[zn->id][r] : 0;
      }
    /* trimNUMANodeResources (resource_manager.go:166-192): a required bind policy caps a zone's cpu
     * at its CPUs that the policy leaves available */
    if (cs && cs->rcb && cs->required && v->av[z][KE_RES_CPU] != 0 && zn->id < KE_MAX_NUMA &&
        (int64_t)cs->zcnt[zn->id] * 1000 < v->av[z][KE_RES_CPU])
      v->av[z][KE_RES_CPU] = (int64_t)cs->zcnt[zn->id] * 1000;
  }
  return 0;
}

static int zone_of(const numa_view* v, int id) {
  for (int z = 0; z < v->n; z++)
    if (v->id[z] == id) return z;
  return -1;
}

/* the pod's requests as options.requests sees them (PodRequests keys cpu / memory, non-zero) */
static int pod_has_req(const ke_pod* pod, int r) { return pod->requests[r] != 0; }

/* tryBestToDistributeEvenly (resource_manager.go:260-314) over the NUMA ids in `mask`.  The sort of the
 * hint's nodes compares totalAvailable indexed by slice position (a reference quirk, reproduced):
 * Go's sort.Slice on <= 12 elements is an insertion sort.  out[z][r]: allocated per zone. */
/* resource.Quantity.Value() of a cpu amount in milli: rounded up, away from zero */
static int64_t qty_value(int64_t milli) { return milli >= 0 ? (milli + 999) / 1000 : -((-milli + 999) / 1000); }

static int numa_distribute(const numa_view* v, uint32_t mask, const ke_pod* pod, int64_t out[KE_MAX_NUMA][KE_NRES],
                           const numa_cs* cs) {
  memset(out, 0, sizeof(int64_t) * KE_MAX_NUMA * KE_NRES);
  int names[KE_NRES] = {0, 0}; /* resourceNamesByNUMA: keys of any totalAvailable entry */
  for (int z = 0; z < v->n; z++)
    for (int r = 0; r < KE_NRES; r++) names[r] |= v->av_has[z][r];
  int bits[KE_MAX_NUMA], nb = 0;
  for (int b = 0; b < KE_MAX_NUMA; b++)
    if (mask & (1u << b)) bits[nb++] = b;
  int ok = 1;
  for (int r = 0; r < KE_NRES; r++) {
    if (!names[r] || !pod_has_req(pod, r)) continue;
    int sorted[KE_MAX_NUMA];
    for (int i = 0; i < nb; i++) sorted[i] = bits[i];
    for (int i = 1; i < nb; i++) /* insertionSortLessFunc with less(i,j) = avail[pos i] < avail[pos j] */
      for (int j = i; j > 0; j--) {
        const int zj = zone_of(v, j), zj1 = zone_of(v, j - 1);
        const int64_t aj = zj >= 0 && v->av_has[zj][r] ? v->av[zj][r] : 0;
        const int64_t aj1 = zj1 >= 0 && v->av_has[zj1][r] ? v->av[zj1][r] : 0;
        if (!(aj < aj1)) break;
        const int t = sorted[j];
        sorted[j] = sorted[j - 1];
        sorted[j - 1] = t;
      }
    int64_t q = pod->requests[r]; /* requestCPUBind: originalRequests (never amplified) */
    for (int i = 0; i < nb; i++) {
      int64_t split = q / (nb - i); /* splitQuantity (:316-330): cpu milli / memory value */
      if (r == KE_RES_CPU && cs && cs->rcb) { /* whole CPUs; whole cores under a required FullPCPUs */
        if (cs->required && cs->bind == KE_CPU_BIND_FULL_PCPUS)
          split = qty_value(q) / cs->cpc / (nb - i) * cs->cpc * 1000;
        else
          split = qty_value(q) / (nb - i) * 1000;
      }
      const int z = zone_of(v, sorted[i]);
      const int64_t avail = z >= 0 && v->av_has[z][r] ? v->av[z][r] : 0;
      const int64_t got = avail > split ? split : avail; /* allocateRes */
      if (got != 0) {
        out[z][r] += got;
        q -= got;
      }
    }
    if (q != 0) ok = 0;
  }
  return ok;
}

/* ---- NodeNUMAResource's allocate-from-reservation under a NUMA policy (nodenumaresource/reservation.go:270-424) ---- */

/* RestoreReservation's matched set on `node` (reservation.go:185-259): the pod's matched usable reservations there
 * whose reserve pod holds NUMA resources or a cpuset (c->resv_m); ascending index.  Returns the count. */
static int numa_rsv_matched(const or_cluster* c, int32_t node, int32_t* ids) {
  int n = 0;
  for (int32_t r = 0; c->resv_m && c->ralloc && r < c->n_resv; r++)
    if (c->resv_m[r] && c->resv[r].node == node && or_resv_usable(&c->resv[r]) &&
        (or_holds_of_idx(c, r) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)) && n < 64)
      ids[n++] = r;
  return n;
}

/* the set a reservation-ignored pod sees there (every reservation matchedOrIgnored, transformer.go:101-106): the
 * usable reservations on `node` holding NUMA resources or a cpuset, ascending index */
static int numa_rsv_ignored(const or_cluster* c, int32_t node, int32_t* ids) {
  int n = 0;
  for (int32_t r = 0; c->ralloc && r < c->n_resv; r++)
    if (c->resv[r].node == node && or_resv_usable(&c->resv[r]) &&
        (or_holds_of_idx(c, r) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)) && n < 64)
      ids[n++] = r;
  return n;
}

static int numa_any(const int64_t* v16) {
  for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++)
    if (v16[j]) return 1;
  return 0;
}
/* quotav1.Add of a NUMA map into o->reuse (keys of both: a non-zero amount is a key) */
static void numa_opt_add(numa_opt* o, const int64_t* v16, const uint8_t* k16) {
  for (int id = 0; id < KE_MAX_NUMA; id++)
    for (int r = 0; r < KE_NRES; r++)
      if (k16 ? k16[2 * id + r] : v16[2 * id + r] != 0) {
        o->reuse_key[id][r] = 1;
        o->reuse[id][r] += v16[2 * id + r];
      }
}
/* reservationAlloc.allocated (Σ the owner pods' NUMA resources) and remained = quotav1.Subtract(allocatable,
 * allocated) per NUMA id, keys of both; both nil without a NUMA allocation of the reserve pod (reservation.go:195-208) */
static int numa_rsv_remained(const ke_reservation_alloc* a, int64_t* rem16, uint8_t* key16) {
  memset(rem16, 0, sizeof(int64_t) * 2 * KE_MAX_NUMA);
  memset(key16, 0, 2 * KE_MAX_NUMA);
  if (!numa_any(a->numa)) return 0;
  for (int j = 0; j < 2 * KE_MAX_NUMA; j++) {
    key16[j] = a->numa[j] != 0 || a->owner_numa[j] != 0;
    rem16[j] = a->numa[j] - a->owner_numa[j];
  }
  return 1;
}
static void cpus_remained(const ke_reservation_alloc* a, uint64_t* out) {
  for (int w = 0; w < ACC_WORDS; w++) out[w] = a->cpuset[w] & ~a->owner_cpuset[w];
}

/* The views of the hint pass (GetTopologyHints, resource_manager.go:136-138): reusable = mergedUnmatchedUsed (the
 * restore state) + mergedMatchedAllocatable, preferredCPUs = mergedMatchedRemainCPUs */
static void numa_opt_hint(const or_cluster* c, const int32_t* M, int nM, numa_opt* o) {
  memset(o, 0, sizeof *o);
  o->has_pref = 1;
  for (int q = 0; q < nM; q++) {
    const ke_reservation_alloc* a = &c->ralloc[M[q]];
    numa_opt_add(o, a->numa, NULL);
    uint64_t rc[ACC_WORDS];
    cpus_remained(a, rc);
    for (int w = 0; w < ACC_WORDS; w++) o->pref[w] |= rc[w];
  }
}
/* A reservation-ignored pod's options: the hint view's preferredCPUs mergedMatchedRemainCPUs; tryAllocateIgnoreReservation
 * (reservation.go:437-490) prefers reservedCPUsFromIgnored = mergedMatchedAllocatedCPUs (the reserve pods' CPUs) ∪ Σ
 * remainedCPUs.  Their reusable amounts (mergedMatchedAllocatable; mergedMatchedAllocated + Σ remained, equal in value)
 * are the node's restore state already (or_numa_ignored_reusable): none added here. */
static void numa_opt_ign(const or_cluster* c, const int32_t* M, int nM, int hint, numa_opt* o) {
  memset(o, 0, sizeof *o);
  o->has_pref = 1;
  for (int q = 0; q < nM; q++) {
    const ke_reservation_alloc* a = &c->ralloc[M[q]];
    uint64_t rc[ACC_WORDS];
    cpus_remained(a, rc);
    for (int w = 0; w < ACC_WORDS; w++) o->pref[w] |= hint ? rc[w] : (a->cpuset[w] | rc[w]);
  }
}
/* tryAllocateFromReservation's options for reservation r (reservation.go:293-311): reusable = mergedUnmatchedUsed +
 * mergedMatchedAllocated + r's remained, preferredCPUs = mergedMatchedAllocatedCPUs ∪ r's remainedCPUs */
static void numa_opt_rsv(const or_cluster* c, const int32_t* M, int nM, int32_t r, numa_opt* o) {
  memset(o, 0, sizeof *o);
  o->has_pref = 1;
  for (int q = 0; q < nM; q++) {
    const ke_reservation_alloc* a = &c->ralloc[M[q]];
    if (numa_any(a->numa)) numa_opt_add(o, a->owner_numa, NULL);
    for (int w = 0; w < ACC_WORDS; w++) o->pref[w] |= a->cpuset[w]; /* allocatedCPUs = the reserve pod's CPUs */
  }
  int64_t rem[2 * KE_MAX_NUMA];
  uint8_t key[2 * KE_MAX_NUMA];
  if (numa_rsv_remained(&c->ralloc[r], rem, key)) numa_opt_add(o, rem, key);
  uint64_t rc[ACC_WORDS];
  cpus_remained(&c->ralloc[r], rc);
  for (int w = 0; w < ACC_WORDS; w++) o->pref[w] |= rc[w];
}

/* resourceManager.Allocate (resource_manager.go:195-224) with the hint `mask` (0 = nil) and options `o`:
 * allocateResourcesByHint, then allocateCPUSet for a binding pod.  1 and the NUMA allocation (dist16[2*id + r]) and
 * cpuset, or 0. */
static int numa_alloc_try(const or_cluster* c, const or_node* nd, const ke_pod* pod, uint32_t mask, const numa_opt* o,
                          int64_t* dist16, uint64_t* cpus) {
  numa_cs cs;
  numa_cs_build_pref(c, nd, pod, &cs, o && o->has_pref ? o->pref : NULL);
  if (dist16) memset(dist16, 0, sizeof(int64_t) * 2 * KE_MAX_NUMA);
  if (cpus) memset(cpus, 0, sizeof(uint64_t) * ACC_WORDS);
  if (cs.rcb && !cs.valid) return 0;
  numa_view v;
  if (numa_view_build_opt(nd, &v, &cs, o) != 0) return 0;
  int64_t out[KE_MAX_NUMA][KE_NRES];
  memset(out, 0, sizeof out);
  if (mask && !numa_distribute(&v, mask, pod, out, &cs)) return 0;
  if (cs.rcb) {
    uint64_t got[ACC_WORDS];
    if (cpuset_allocate_cs(nd, &cs, &v, mask ? (const int64_t(*)[KE_NRES])out : NULL, got) != 0) return 0;
    if (cpus) memcpy(cpus, got, sizeof got);
  }
  if (dist16)
    for (int z = 0; z < v.n; z++)
      if (v.id[z] >= 0 && v.id[z] < KE_MAX_NUMA)
        for (int r = 0; r < KE_NRES; r++) dist16[2 * v.id[z] + r] = out[z][r];
  return 1;
}

/* tryAllocateFromReservation (reservation.go:270-424) for a pod matching the reservations M[0..nM) of RestoreReservation's
 * matched set on the node, over S[0..nS) (M itself, or the nominated / nominating one), with the hint `mask`:
 * Default / Aligned: one Allocate; Restricted: that Allocate, numCPUsNeeded <= |remainedCPUs| for a binding pod, then an
 * Allocate with requiredResources = remained and preferredCPUs = remainedCPUs whose cpuset may not outgrow them.  The
 * first satisfied one in ascending index (Go ranges over a map: which one is the reference's choice only for one) gives
 * 1, its options (*used) and its allocation; none: -1 under a reservation affinity, else 0 (nil: tryAllocateFromNode). */
static int numa_from_rsv_try(const or_cluster* c, const ke_pod* pod, int32_t node, const int32_t* M, int nM,
                             const int32_t* S, int nS, uint32_t mask, int required, numa_opt* used, int64_t* dist16,
                             uint64_t* cpus) {
  const or_node* nd = &c->nodes[node];
  if (nM == 0) return 0;
  for (int q = 0; q < nS; q++) {
    const int32_t r = S[q];
    numa_opt o1;
    numa_opt_rsv(c, M, nM, r, &o1);
    if (!numa_alloc_try(c, nd, pod, mask, &o1, dist16, cpus)) continue;
    if (c->resv[r].allocate_policy == KE_RSV_POLICY_RESTRICTED) {
      uint64_t rc[ACC_WORDS];
      cpus_remained(&c->ralloc[r], rc);
      const int reserved = popcount_set(rc);
      cpuset_state st;
      cpuset_prefilter(c, pod, &st);
      numa_cs cs0;
      numa_cs_build(c, nd, pod, &cs0);
      if (cs0.rcb && st.num_cpus > reserved) continue;
      numa_opt o2 = o1;
      int64_t rem[2 * KE_MAX_NUMA];
      uint8_t key[2 * KE_MAX_NUMA];
      o2.has_req = numa_rsv_remained(&c->ralloc[r], rem, key);
      for (int id = 0; id < KE_MAX_NUMA; id++)
        for (int k = 0; k < KE_NRES; k++) {
          o2.req[id][k] = rem[2 * id + k];
          o2.req_key[id][k] = key[2 * id + k];
        }
      memcpy(o2.pref, rc, sizeof rc);
      uint64_t got[ACC_WORDS];
      if (!numa_alloc_try(c, nd, pod, mask, &o2, dist16, got)) continue;
      if (popcount_set(got) > reserved) continue; /* (never: the take is numCPUsNeeded <= reserved) */
      if (cpus) memcpy(cpus, got, sizeof got);
    }
    if (used) *used = o1;
    return 1;
  }
  return required ? -1 : 0;
}

/* The Allocate of a matched pod under a NUMA policy on the node with the hint `mask` as Filter's hint generation and
 * Plugin.Allocate run it (resource_manager.go:586-594, topology_hint.go:78-118): from one of the node's matched
 * reservations, else (no reservation affinity) from the node.  1 = a hint / allocation, 0 = none. */
static int numa_matched_alloc_ok(const or_cluster* c, const ke_pod* pod, int32_t node, const int32_t* M, int nM,
                                 uint32_t mask) {
  if (c->ignored) {  /* tryAllocateIgnoreReservation: its status, no fallback (reservation.go:282-284) */
    numa_opt o;
    numa_opt_ign(c, M, nM, 0, &o);
    return numa_alloc_try(c, &c->nodes[node], pod, mask, &o, NULL, NULL);
  }
  const int required = pod->reservation_matched == KE_RSV_AFFINITY;
  const int r = numa_from_rsv_try(c, pod, node, M, nM, M, nM, mask, required, NULL, NULL, NULL);
  if (r != 0) return r > 0;
  return numa_alloc_try(c, &c->nodes[node], pod, mask, NULL, NULL, NULL);
}

/* allocateWithNominatedReservation (reservation.go:492-522) then tryAllocateFromNode (plugin.go:671-689) for a matched
 * pod under a NUMA policy with the stored affinity: the nominated reservation nom (-1: none) -- Score and Reserve.
 * 1 and the allocation (NUMA, cpuset) and the options it used (*used, for calculateAllocatableAndRequested), or 0 = an
 * error status (no nominated reservation under an affinity; the reservation's or the node's Allocate failed). */
static int numa_matched_alloc(const or_cluster* c, const ke_pod* pod, int32_t node, const int32_t* M, int nM,
                              int32_t nom, uint32_t aff, numa_opt* used, int64_t* dist16, uint64_t* cpus) {
  if (c->ignored) {  /* allocateWithNominatedReservation of an ignored pod: tryAllocateIgnoreReservation (:504-506) */
    numa_opt_ign(c, M, nM, 0, used);
    return numa_alloc_try(c, &c->nodes[node], pod, aff, used, dist16, cpus);
  }
  const int required = pod->reservation_matched == KE_RSV_AFFINITY;
  if (nom < 0 && required) return 0; /* "no nominated reservation" */
  int in = 0;
  for (int q = 0; q < nM; q++) in |= M[q] == nom;
  if (nom >= 0 && in) {
    const int r = numa_from_rsv_try(c, pod, node, M, nM, &nom, 1, aff, required, used, dist16, cpus);
    if (r < 0) return 0;
    if (r > 0) return 1;
  }
  memset(used, 0, sizeof *used); /* tryAllocateFromNode: reusable = mergedUnmatchedUsed, no preferred CPUs */
  return numa_alloc_try(c, &c->nodes[node], pod, aff, NULL, dist16, cpus);
}

typedef struct numa_hint {
  uint32_t mask; /* 0 = nil NUMANodeAffinity */
  int preferred, unsatisfied;
  int64_t score;
} numa_hint;

/* A matched pod's hint pass on a node with reservations in RestoreReservation's matched set (numa_admit): every
 * mask's Allocate goes through tryAllocateFromReservation, then tryAllocateFromNode (resource_manager.go:586-594) */
static __thread struct {
  int on;
  int32_t node;
  int nM;
  int32_t M[64];
} g_trial;

/* generateResourceHints (resource_manager.go:525-622) for a non-cpuset pod.  Per resource (cpu,
 * memory): the list of hints in IterateBitMasks order; present[r] = the resource has a list. */
static void numa_generate_hints(const or_cluster* c, const or_node* nd, const numa_view* v, const ke_pod* pod,
                                int policy, numa_hint* lists /*[KE_NRES][255]*/, int* counts, int* present,
                                const numa_cs* cs) {
  /* options.requests: a binding pod's cpu amplified (getResourceOptions, plugin.go:634-640) */
  int64_t podreq[KE_NRES] = {pod->requests[KE_RES_CPU], pod->requests[KE_RES_MEMORY]};
  if (cs && cs->rcb && v->ratio > 1.0) podreq[KE_RES_CPU] = amplify(podreq[KE_RES_CPU], v->ratio);
  int names[KE_NRES] = {0, 0};
  for (int z = 0; z < v->n; z++)
    for (int r = 0; r < KE_NRES; r++) names[r] |= v->cap_has[z][r];
  uint32_t lack[KE_NRES] = {0, 0}; /* numaNodesLackResource */
  for (int r = 0; r < KE_NRES; r++)
    if (names[r])
      for (int z = 0; z < v->n; z++)
        if (!v->av_has[z][r] || v->av[z][r] == 0) lack[r] |= 1u << v->id[z];
  int min_size[KE_NRES] = {v->n, v->n};
  int total_names[KE_NRES] = {0, 0};
  for (int r = 0; r < KE_NRES; r++) counts[r] = 0;
  /* IterateBitMasks: sizes 1..n, combinations of the zone ids in lexicographic order */
  for (int size = 1; size <= v->n; size++) {
    int idx[KE_MAX_NUMA];
    for (int i = 0; i < size; i++) idx[i] = i;
    for (;;) {
      uint32_t mask = 0;
      int64_t avail[KE_NRES] = {0, 0}, total[KE_NRES] = {0, 0};
      int total_has[KE_NRES] = {0, 0};
      for (int i = 0; i < size; i++) {
        const int z = idx[i];
        mask |= 1u << v->id[z];
        for (int r = 0; r < KE_NRES; r++) {
          avail[r] += v->av_has[z][r] ? v->av[z][r] : 0;
          total[r] += v->cap_has[z][r] ? v->cap[z][r] : 0;
          total_has[r] |= v->cap_has[z][r];
        }
      }
      for (int r = 0; r < KE_NRES; r++)
        if (pod_has_req(pod, r) && total_has[r]) total_names[r] = 1;
      /* numaScorer.score(requested = total - available, total, pod) with the NUMA strategy */
      int64_t req[KE_NRES];
      for (int r = 0; r < KE_NRES; r++) req[r] = total[r] - avail[r] > 0 ? total[r] - avail[r] : 0;
      const int64_t score = numa_resource_score_as(&c->cfg.numa, c->cfg.numa.numa_strategy, req, total, podreq);
      int64_t out[KE_MAX_NUMA][KE_NRES];
      /* tryAllocateFromNode with the mask: allocateResourcesByHint, then allocateCPUSet */
      const int fits = g_trial.on ? numa_matched_alloc_ok(c, pod, g_trial.node, g_trial.M, g_trial.nM, mask)
                                  : numa_distribute(v, mask, pod, out, cs) &&
                                        (!cs || !cs->rcb || cpuset_fits_cs(nd, cs, v, (const int64_t(*)[KE_NRES])out));
      if (fits)
        for (int r = 0; r < KE_NRES; r++) { /* generator.generateHints per resource */
          if (!total_names[r]) continue;
          if (mask & lack[r]) continue;
          if (size < min_size[r]) min_size[r] = size;
          numa_hint h = {mask, 0, 0, score};
          lists[r * 255 + counts[r]++] = h;
        }
      int i = size - 1; /* next combination */
      while (i >= 0 && idx[i] == v->n - size + i) i--;
      if (i < 0) break;
      idx[i]++;
      for (int j = i + 1; j < size; j++) idx[j] = idx[j - 1] + 1;
    }
  }
  for (int r = 0; r < KE_NRES; r++) {
    present[r] = total_names[r] && pod_has_req(pod, r);
    for (int i = 0; i < counts[r]; i++)
      lists[r * 255 + i].preferred = __builtin_popcount(lists[r * 255 + i].mask) == min_size[r] ||
                                     policy == KE_NUMA_POLICY_RESTRICTED;
  }
}

/* mergePermutation (policy.go:98-137) */
static numa_hint merge_permutation(uint32_t all, const numa_hint* perm, int n) {
  int preferred = 1, satisfied = 1, maxn = 0, have = 0;
  uint32_t first = 0, merged = all;
  for (int i = 0; i < n; i++) {
    if (perm[i].mask) {
      if (!have) first = perm[i].mask, have = 1;
      if (perm[i].mask != first) preferred = 0;
      if (__builtin_popcount(perm[i].mask) > maxn) maxn = __builtin_popcount(perm[i].mask);
      merged &= perm[i].mask;
    }
    if (!perm[i].preferred) preferred = 0;
    if (perm[i].unsatisfied) satisfied = 0;
  }
  satisfied = (!have || maxn == __builtin_popcount(merged)) && satisfied;
  numa_hint h = {merged, preferred, !satisfied, 0};
  return h;
}

/* checkExclusivePolicy (policy.go:73-93); status[id] = NUMANodeSharedStatus of NUMA id `id` */
static int exclusive_ok(uint32_t mask, int exclusive, const uint8_t* status) {
  if (!mask) return 0;
  if (exclusive == KE_NUMA_EXCLUSIVE_REQUIRED) {
    if (__builtin_popcount(mask) > 1) {
      for (int b = 0; b < KE_MAX_NUMA; b++)
        if ((mask >> b & 1u) && status[b] == KE_NUMA_STATUS_SINGLE) return 0;
    } else if (status[__builtin_ctz(mask)] == KE_NUMA_STATUS_SHARED) {
      return 0;
    }
  }
  return 1;
}

static int narrower(uint32_t a, uint32_t b) { /* bitmask.IsNarrowerThan */
  const int ca = __builtin_popcount(a), cb = __builtin_popcount(b);
  return ca == cb ? a < b : ca < cb;
}

/* mergeFilteredHints (policy.go:198-260) + iterateAllProviderTopologyHints (:282-299) */
static numa_hint merge_filtered(uint32_t all, numa_hint* const* lists, const int* lens, int nl, int exclusive,
                                const uint8_t* status) {
  numa_hint best = {all, 0, 0, 0};
  int idx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < nl; i++)
    if (lens[i] == 0) return best; /* an empty list: no permutation */
  for (;;) {
    numa_hint perm[8];
    for (int i = 0; i < nl; i++) perm[i] = lists[i][idx[i]];
    numa_hint m = merge_permutation(all, perm, nl);
    if (__builtin_popcount(m.mask) != 0) {
      if (!exclusive_ok(m.mask, exclusive, status)) m.preferred = 0;
      for (int i = 0; i < nl; i++)
        if (perm[i].mask && perm[i].mask == m.mask) m.score += perm[i].score;
      if (m.preferred && !best.preferred) {
        best = m;
      } else if (!(!m.preferred && best.preferred)) {
        if (!narrower(m.mask, best.mask)) {
          if (__builtin_popcount(m.mask) == __builtin_popcount(best.mask) && m.score > best.score) best = m;
        } else {
          best = m;
        }
      }
    }
    int i = nl - 1;
    while (i >= 0 && ++idx[i] == lens[i]) idx[i--] = 0;
    if (i < 0) break;
  }
  return best;
}

/* Policy.Merge after filterProvidersHints (policy_best_effort.go:48-60, policy_restricted.go:50-62,
 * policy_single_numa_node.go:52-90).  `lists` are the filtered provider lists (for SingleNUMANode
 * already reduced by filterSingleNumaHints); `reasons` = filterProvidersHints reported an empty list.
 * Returns admit; *best = the merged hint (mask 0 = nil affinity). */
static int policy_merge(int policy, uint32_t all, numa_hint* const* lists, const int* lens, int nl, int reasons,
                        int exclusive, const uint8_t* status, numa_hint* best) {
  if (policy == KE_NUMA_POLICY_BEST_EFFORT) {
    *best = merge_filtered(all, lists, lens, nl, exclusive, status);
    if (best->unsatisfied) *best = (numa_hint){all, 0, 0, 0};
    return 1;
  }
  if (policy == KE_NUMA_POLICY_RESTRICTED) {
    if (reasons) {
      *best = (numa_hint){all, 0, 0, 0};
      return 0;
    }
    *best = merge_filtered(all, lists, lens, nl, exclusive, status);
    return best->preferred;
  }
  if (reasons) { /* SingleNUMANode */
    *best = (numa_hint){0, 0, 0, 0};
    return 0;
  }
  *best = merge_filtered(all, lists, lens, nl, exclusive, status);
  if (best->mask == all) *best = (numa_hint){0, best->preferred, 0, 0};
  return best->preferred;
}

/* Golden-vector entry point: Policy.Merge over raw provider hint lists.  kinds[i]: 0 = a hint list,
 * 1 = nil list / provider without hints (one preferred any-NUMA hint), 2 = empty list (unsatisfied,
 * reason).  Hints are flattened: masks (0 = nil affinity), preferred, scores; lens[i] per list. */
int or_topology_merge(int32_t policy, uint32_t all, int32_t n_lists, const int32_t* kinds, const int32_t* lens,
                      const uint32_t* masks, const uint8_t* preferred, const int64_t* scores, uint32_t* out_mask,
                      uint8_t* out_preferred, uint8_t* out_unsatisfied, int64_t* out_score) {
  static __thread numa_hint buf[16][64];
  numa_hint* lists[16];
  int ln[16], nl = 0, reasons = 0, off = 0;
  if (n_lists > 15) return -1;
  for (int i = 0; i < n_lists; i++) {
    lists[nl] = buf[nl];
    if (kinds[i] == 1) {
      buf[nl][0] = (numa_hint){0, 1, 0, 0};
      ln[nl++] = 1;
      continue;
    }
    if (kinds[i] == 2) {
      buf[nl][0] = (numa_hint){0, 0, 1, 0};
      ln[nl] = policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE ? 0 : 1;
      nl++;
      reasons = 1;
      continue;
    }
    int n = 0;
    for (int j = 0; j < lens[i] && j < 64; j++) {
      numa_hint h = {masks[off + j], preferred[off + j], 0, scores[off + j]};
      if (policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE &&  /* filterSingleNumaHints */
          !((h.mask == 0 && h.preferred) || (h.mask != 0 && __builtin_popcount(h.mask) == 1 && h.preferred)))
        continue;
      buf[nl][n++] = h;
    }
    off += lens[i];
    ln[nl++] = n;
  }
  if (nl == 0) { /* no providers at all */
    buf[0][0] = (numa_hint){0, 1, 0, 0};
    lists[0] = buf[0];
    ln[0] = 1;
    nl = 1;
  }
  numa_hint best;
  static const uint8_t idle[KE_MAX_NUMA] = {0};
  const int admit = policy_merge(policy, all, lists, ln, nl, reasons, KE_NUMA_EXCLUSIVE_NONE, idle, &best);
  *out_mask = best.mask;
  *out_preferred = (uint8_t)best.preferred;
  *out_unsatisfied = (uint8_t)best.unsatisfied;
  *out_score = best.score;
  return admit;
}

/* topologymanager Admit for the pod on the node (manager.go:64-129 with the NodeNUMAResource hint
 * provider; DeviceShare provides no hints for a pod without device requests).  Returns the status
 * code, *affinity (0 = nil) on success. */
static int numa_admit(const or_cluster* c, const or_node* nd, const ke_pod* pod, int policy, int exclusive,
                      uint32_t* affinity, int* reason, const numa_cs* cs) {
  numa_view v;
  uint32_t all = 0;
  for (int z = 0; z < nd->n_zone; z++) all |= 1u << nd->zone[z].id;
  /* GetAllNUMANodeStatus(len(numaNodes)): the statuses of NUMA ids 0..n-1 (a zone id >= n would
   * index past the reference's slice; read as idle here) */
  uint8_t status[KE_MAX_NUMA] = {0};
  for (int z = 0; z < nd->n_zone; z++)
    if (nd->zone[z].id < nd->n_zone) status[nd->zone[z].id] = nd->zone[z].numa_status;
  /* a matched pod on a node of its reservations holding NUMA resources / CPUs: the hint view (mergedMatchedAllocatable
   * reusable, mergedMatchedRemainCPUs preferred) and every mask's Allocate from the reservations first */
  const int32_t node = (int32_t)(nd - c->nodes);
  int32_t M[64];
  /* a reservation-ignored pod binding CPUs: the hint view prefers the held remainedCPUs, every mask's Allocate is
   * tryAllocateIgnoreReservation (a pod binding none reads the held amounts as reusable only: its rows) */
  const int nM = c->resv_m && !c->ignored ? numa_rsv_matched(c, node, M)
                 : c->ignored && cs && cs->rcb ? numa_rsv_ignored(c, node, M) : 0;
  numa_opt oh;
  numa_cs cs_h;
  if (nM > 0) {
    if (c->ignored) numa_opt_ign(c, M, nM, 1, &oh);
    else numa_opt_hint(c, M, nM, &oh);
    numa_cs_build_pref(c, nd, pod, &cs_h, oh.pref);
    cs = &cs_h;
  }
  if (numa_view_build_opt(nd, &v, cs, nM > 0 ? &oh : NULL) != 0) { /* GetPodTopologyHints error -> Unschedulable */
    *reason = KE_REASON_NUMA_HINT_UNALIGNED;
    return KE_CODE_UNSCHEDULABLE;
  }
  static __thread numa_hint store[KE_NRES * 255];
  int counts[KE_NRES], present[KE_NRES];
  if (nM > 0) {
    g_trial.on = 1;
    g_trial.node = node;
    g_trial.nM = nM;
    memcpy(g_trial.M, M, sizeof(int32_t) * (size_t)nM);
  }
  numa_generate_hints(c, nd, &v, pod, policy, store, counts, present, cs);
  g_trial.on = 0;
  /* DeviceShare's hints (topology_hint.go:38-58): a provider error is an Admit reason
   * (accumulateProvidersHints, manager.go:110-125) */
  static __thread numa_hint ds_list[255];
  int ds_n = 0, ds_copies = 0, ds_none = 1;
  const int ds_st = ds_numa_hints(c, nd, pod, ds_list, &ds_n, &ds_copies, &ds_none, reason);
  if (ds_st) return KE_CODE_UNSCHEDULABLE;
  /* filterProvidersHints: the NUMA provider's lists in sorted resource-name order (cpu, memory), then
   * DeviceShare's: nil hints -> one preferred any-NUMA hint, else one (identical) list per requested device
   * type.  Providers in profile order (NodeNUMAResource, DeviceShare); the reference creates plugins from a
   * Go map, so this order is a convention. */
  static __thread numa_hint filt[KE_NRES + 4][255];
  numa_hint* lists[KE_NRES + 4];
  int lens[KE_NRES + 4], nl = 0, reasons = 0;
  int any_present = present[0] || present[1];
  for (int r = 0; r < KE_NRES; r++) {
    if (!present[r]) continue;
    if (counts[r] == 0) { /* no possible affinity for the resource */
      if (policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE) { /* filterSingleNumaHints drops the unsatisfied hint */
        lists[nl] = filt[nl];
        lens[nl++] = 0;
        reasons = 1;
        continue;
      }
      filt[nl][0] = (numa_hint){0, 0, 1, 0};
      lists[nl] = filt[nl];
      lens[nl++] = 1;
      reasons = 1;
      continue;
    }
    int n = 0;
    for (int i = 0; i < counts[r]; i++) {
      const numa_hint h = store[r * 255 + i];
      if (policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE && !(h.preferred && __builtin_popcount(h.mask) == 1)) continue;
      filt[nl][n++] = h;
    }
    lists[nl] = filt[nl];
    lens[nl++] = n;
  }
  if (!any_present) { /* the provider returned an empty map: one preferred any-NUMA hint */
    filt[nl][0] = (numa_hint){0, 1, 0, 0};
    lists[nl] = filt[nl];
    lens[nl++] = 1;
  }
  if (ds_none) {
    filt[nl][0] = (numa_hint){0, 1, 0, 0}; /* DeviceShare: no preference */
    lists[nl] = filt[nl];
    lens[nl++] = 1;
  } else {
    for (int t = 0; t < ds_copies; t++) {
      int n = 0;
      for (int i = 0; i < ds_n; i++) {
        const numa_hint h = ds_list[i];
        if (policy == KE_NUMA_POLICY_SINGLE_NUMA_NODE && !(h.preferred && __builtin_popcount(h.mask) == 1)) continue;
        filt[nl][n++] = h;
      }
      lists[nl] = filt[nl];
      lens[nl++] = n;
    }
  }
  numa_hint best;
  const int admit = policy_merge(policy, all, lists, lens, nl, reasons, exclusive, status, &best);
  if (!admit) {
    *reason = KE_REASON_NUMA_HINT_UNALIGNED;
    return KE_CODE_UNSCHEDULABLE;
  }
  /* allocateResources -> NodeNUMAResource.Allocate -> tryAllocateFromReservation / tryAllocateFromNode with the hint */
  int64_t out[KE_MAX_NUMA][KE_NRES];
  memset(out, 0, sizeof out);
  if (nM > 0) {
    if (!numa_matched_alloc_ok(c, pod, node, M, nM, best.mask)) {
      *reason = pod->reservation_matched == KE_RSV_AFFINITY ? KE_REASON_RSV_INSUFFICIENT_NUMA
                                                            : KE_REASON_NUMA_INSUFFICIENT_RESOURCES;
      return KE_CODE_UNSCHEDULABLE;
    }
  } else if (best.mask && !numa_distribute(&v, best.mask, pod, out, cs)) {
    *reason = KE_REASON_NUMA_INSUFFICIENT_RESOURCES;
    return KE_CODE_UNSCHEDULABLE;
  }
  if (nM == 0 && cs && cs->rcb && !cpuset_fits_cs(nd, cs, &v, (const int64_t(*)[KE_NRES])out)) {
    *reason = KE_REASON_NUMA_INSUFFICIENT_CPUS; /* "not enough cpus available to satisfy request" */
    return KE_CODE_UNSCHEDULABLE;
  }
  /* -> DeviceShare.Allocate with the affinity (topology_hint.go:60-117) */
  const int ds_code = ds_numa_allocate(c, nd, pod, best.mask, reason);
  if (ds_code) return ds_code;
  *affinity = best.mask;
  return KE_CODE_SUCCESS;
}

/* Golden-vector entry points.  tryBestToDistributeEvenly of `pod` on node `node` for the NUMA ids in
 * `mask` (resource_manager.go:260-314): returns 1 when every requested NUMA resource was split;
 * out16[2*id + r] = the amounts. */
int or_numa_distribute(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t mask, int64_t* out16) {
  const or_node* nd = &c->nodes[node];
  numa_view v;
  numa_cs cs;
  numa_cs_build(c, nd, pod, &cs);
  if (numa_view_build(nd, &v, &cs) != 0) return -1;
  int64_t out[KE_MAX_NUMA][KE_NRES];
  const int ok = numa_distribute(&v, mask, pod, out, &cs);
  for (int i = 0; i < 2 * KE_MAX_NUMA; i++) out16[i] = 0;
  for (int z = 0; z < v.n; z++)
    for (int r = 0; r < KE_NRES; r++) out16[2 * v.id[z] + r] = out[z][r];
  return ok;
}

/* generateResourceHints for `pod` on `node` under `policy` (resource_manager.go:525-622): per
 * resource r (cpu, memory) present[r] = the resource has a hint list, counts[r] its length and
 * masks / preferred / scores[r*255 + i] its hints in order. */
int or_numa_hints(const or_cluster* c, int32_t node, const ke_pod* pod, int32_t policy, uint32_t* masks,
                  uint8_t* preferred, int64_t* scores, int32_t* counts, int32_t* present) {
  const or_node* nd = &c->nodes[node];
  numa_view v;
  numa_cs cs;
  numa_cs_build(c, nd, pod, &cs);
  if (numa_view_build(nd, &v, &cs) != 0) return -1;
  static __thread numa_hint store[KE_NRES * 255];
  int cnt[KE_NRES], pres[KE_NRES];
  numa_generate_hints(c, nd, &v, pod, policy, store, cnt, pres, &cs);
  for (int r = 0; r < KE_NRES; r++) {
    counts[r] = cnt[r];
    present[r] = pres[r];
    for (int i = 0; i < cnt[r]; i++) {
      masks[r * 255 + i] = store[r * 255 + i].mask;
      preferred[r * 255 + i] = (uint8_t)store[r * 255 + i].preferred;
      scores[r * 255 + i] = store[r * 255 + i].score;
    }
  }
  return 0;
}

/* CPU accumulator golden-vector entry point (cpu_accumulator_test.go): cpus[i] = {cpu id, core id,
 * NUMA node id, socket id}; alloc_ref / alloc_excl per CPU id (-1 = not allocated); preferred may be
 * NULL.  Returns 0 and `out` (CPU-id bitset) or -1. */
int or_take_cpus(const int32_t* cpus, int32_t n, int32_t max_ref, const uint64_t* available, const int32_t* alloc_ref,
                 const int32_t* alloc_excl, int32_t needed, int32_t bind, int32_t excl, int32_t numa_most,
                 const uint64_t* preferred, uint64_t* out) {
  static __thread acc_topo t;
  static __thread acc_alloc al;
  memset(&t, 0, sizeof t);
  memset(&al, 0, sizeof al);
  for (int i = 0; i < n; i++) {
    const int c = cpus[4 * i];
    if (c < 0 || c >= ACC_MAX_CPUS) return -2;
    t.valid[c] = 1;
    t.core[c] = cpus[4 * i + 1];
    t.node[c] = cpus[4 * i + 2];
    t.socket[c] = cpus[4 * i + 3];
  }
  acc_topo_finish(&t);
  for (int c = 0; c < ACC_MAX_CPUS; c++)
    if (alloc_ref && alloc_ref[c] >= 0) {
      al.present[c] = 1;
      al.ref[c] = alloc_ref[c];
      al.excl[c] = alloc_excl ? alloc_excl[c] : 0;
    }
  return acc_take_preferred_cpus(&t, max_ref, available, preferred, &al, needed, bind, excl, numa_most, out);
}

int or_spread_order(const int32_t* cpus, int32_t n, const uint64_t* available, int32_t numa_most, int32_t* out) {
  static __thread acc_topo t;
  memset(&t, 0, sizeof t);
  for (int i = 0; i < n; i++) {
    const int c = cpus[4 * i];
    t.valid[c] = 1;
    t.core[c] = cpus[4 * i + 1];
    t.node[c] = cpus[4 * i + 2];
    t.socket[c] = cpus[4 * i + 3];
  }
  acc_topo_finish(&t);
  return acc_spread_order(&t, available, numa_most, out);
}

/* checkExclusivePolicy golden-vector entry point: status[i] for NUMA id i, n ids */
int or_numa_exclusive_ok(uint32_t mask, int32_t exclusive, const uint8_t* status, int32_t n) {
  uint8_t st[KE_MAX_NUMA] = {0};
  for (int i = 0; i < n && i < KE_MAX_NUMA; i++) st[i] = status[i];
  return exclusive_ok(mask, exclusive, st);
}

/* the pod's NUMA allocation on its affinity (resourceManager.Allocate -> allocateResourcesByHint) */
static int numa_allocation(const or_node* nd, const ke_pod* pod, uint32_t affinity, numa_view* v,
                           int64_t out[KE_MAX_NUMA][KE_NRES], const numa_cs* cs) {
  memset(out, 0, sizeof(int64_t) * KE_MAX_NUMA * KE_NRES);
  if (numa_view_build(nd, v, cs) != 0) return 0;
  if (!affinity) return 1;
  return numa_distribute(v, affinity, pod, out, cs);
}

/* Plugin.Score  scoring.go:66-120 -> scoreWithAmplifiedCPUs :122-139.  *err (may be NULL): the Score returned an
 * error status (a matched pod's allocateWithNominatedReservation / tryAllocateFromNode failed, scoring.go:105-115) */
static int64_t numa_score_ex(const or_cluster* c, const ke_pod* pod, int32_t node, int* err);
int64_t or_numa_score(const or_cluster* c, const ke_pod* pod, int32_t node) { return numa_score_ex(c, pod, node, NULL); }
static int64_t numa_score_ex(const or_cluster* c, const ke_pod* pod, int32_t node, int* err) {
  const or_node* n = &c->nodes[node];
  if (err) *err = 0;
  if (pod_requests_zero(pod)) return 0; /* state.skip */
  int exclusive;
  const int policy = effective_policy(n, pod, &exclusive);
  if (policy < 0) return 0;
  int32_t M[64];
  numa_cs cs;
  numa_cs_build(c, n, pod, &cs);
  const int nM = policy == KE_NUMA_POLICY_NONE ? 0
                 : c->resv_m && !c->ignored && c->numa_nom ? numa_rsv_matched(c, node, M)
                 : c->ignored && cs.rcb ? numa_rsv_ignored(c, node, M) : 0;
  if (nM > 0) {
    /* a matched pod on a node of its reservations holding NUMA resources / CPUs: the allocation from the nominated
     * reservation (else the node) on the stored affinity, calculateAllocatableAndRequested with the options it used;
     * an ignored binding pod: tryAllocateIgnoreReservation's */
    if (cs.rcb && !cs.valid) return 0;
    uint32_t aff = 0;
    int reason;
    if (n->n_zone == 0 || numa_admit(c, n, pod, policy, exclusive, &aff, &reason, &cs) != KE_CODE_SUCCESS) return 0;
    numa_opt used;
    int64_t dist16[2 * KE_MAX_NUMA];
    uint64_t pcpus[ACC_WORDS];
    if (!numa_matched_alloc(c, pod, node, M, nM, c->ignored ? -1 : c->numa_nom[node], aff, &used, dist16, pcpus)) {
      if (err) *err = 1;
      return 0;
    }
    numa_cs csu;
    numa_cs_build_pref(c, n, pod, &csu, used.has_pref ? used.pref : NULL);
    numa_view v;
    if (numa_view_build_opt(n, &v, &csu, &used) != 0) return 0;
    int64_t alloc[KE_NRES] = {0, 0}, req[KE_NRES] = {0, 0};
    int any = 0;
    for (int z = 0; z < v.n; z++) {
      const int id = v.id[z];
      if (id < 0 || id >= KE_MAX_NUMA || (dist16[2 * id] == 0 && dist16[2 * id + 1] == 0)) continue;
      any = 1;
      for (int r = 0; r < KE_NRES; r++) {
        alloc[r] += v.cap_has[z][r] ? v.cap[z][r] : 0;
        req[r] += v.has_alloc[z] ? v.al[z][r] : 0;
      }
    }
    if (!any) {
      req[0] = n->node.requested[KE_RES_CPU] + n->rv_req[KE_RES_CPU];
      req[1] = n->node.requested[KE_RES_MEMORY] + n->rv_req[KE_RES_MEMORY];
      alloc[0] = n->node.allocatable[KE_RES_CPU];
      alloc[1] = n->node.allocatable[KE_RES_MEMORY];
    }
    int64_t podreq[KE_NRES] = {pod->requests[KE_RES_CPU], pod->requests[KE_RES_MEMORY]};
    if (cs.rcb) { /* the node's allocated CPUs with preferredCPUs minus the pod's own released (scoring.go:180-185) */
      int64_t k = 0;
      for (int c1 = 0; n->cpus && c1 < ACC_MAX_CPUS; c1++) {
        int ref = n->cpus->al.present[c1] ? n->cpus->al.ref[c1] : 0;
        if (ref > 0 && used.has_pref && (used.pref[c1 >> 6] >> (c1 & 63) & 1) && !(pcpus[c1 >> 6] >> (c1 & 63) & 1)) ref--;
        k += ref > 0;
      }
      req[0] = amplify(n->cpus ? k * 1000 : cpus_allocated_count(n) * 1000, v.ratio);
      if (v.ratio > 1.0) podreq[KE_RES_CPU] = amplify(podreq[KE_RES_CPU], v.ratio);
    }
    return numa_resource_score(&c->cfg.numa, req, alloc, podreq);
  }
  if (policy != KE_NUMA_POLICY_NONE) {
    /* the affinity the Filter's Admit stored, the allocation on it, calculateAllocatableAndRequested */
    uint32_t aff = 0;
    int reason;
    numa_cs cs;
    numa_cs_build(c, n, pod, &cs);
    if (cs.rcb && !cs.valid) return 0; /* scoring.go:93-95 */
    if (n->n_zone == 0 || numa_admit(c, n, pod, policy, exclusive, &aff, &reason, &cs) != KE_CODE_SUCCESS) return 0;
    numa_view v;
    int64_t out[KE_MAX_NUMA][KE_NRES];
    if (!numa_allocation(n, pod, aff, &v, out, &cs)) return 0;
    int64_t alloc[KE_NRES] = {0, 0}, req[KE_NRES] = {0, 0};
    int any = 0;
    for (int z = 0; z < v.n; z++) {
      if (out[z][0] == 0 && out[z][1] == 0) continue; /* podAllocation.NUMANodeResources */
      any = 1;
      for (int r = 0; r < KE_NRES; r++) {
        alloc[r] += v.cap_has[z][r] ? v.cap[z][r] : 0;
        req[r] += v.has_alloc[z] ? v.al[z][r] : 0;
      }
    }
    if (!any) {
      req[0] = n->node.requested[KE_RES_CPU] + n->rv_req[KE_RES_CPU];
      req[1] = n->node.requested[KE_RES_MEMORY] + n->rv_req[KE_RES_MEMORY];
      alloc[0] = n->node.allocatable[KE_RES_CPU];
      alloc[1] = n->node.allocatable[KE_RES_MEMORY];
    }
    int64_t podreq[KE_NRES] = {pod->requests[KE_RES_CPU], pod->requests[KE_RES_MEMORY]};
    if (cs.rcb) {
      /* a non-empty pod cpuset: requested cpu = Amplify(all allocated CPUs of the node * 1000)
       * (scoring.go:179-185); options.requests carries the amplified cpu */
      req[0] = amplify(cpus_allocated_count(n) * 1000, v.ratio);
      if (v.ratio > 1.0) podreq[KE_RES_CPU] = amplify(podreq[KE_RES_CPU], v.ratio);
    }
    return numa_resource_score(&c->cfg.numa, req, alloc, podreq);
  }
  /* getResourceOptions -> amplifyNUMANodeResources (util.go:78-87) */
  double ratio;
  if (n->node.nrt_cpu_amplification_ratio > -1.5) {
    ratio = n->node.nrt_cpu_amplification_ratio < 0 ? 0.0 : n->node.nrt_cpu_amplification_ratio;
  } else {
    if (n->node.amplification_error) return 0;
    ratio = n->node.cpu_amplification_ratio < 0 ? 0.0 : n->node.cpu_amplification_ratio;
  }
  /* requestCPUBind (scoring.go:86-92): a cpuset pod scores 0 without a valid CPU topology, and its
   * cpu request is amplified (getResourceOptions, plugin.go:634-640) */
  cpuset_state st;
  cpuset_prefilter(c, pod, &st);
  const int rcb = request_cpu_bind(&st, pod, n->node.cpu_bind_policy);
  if (rcb < 0 || (rcb && !cpus_valid(n))) return 0;
  int64_t podreq[KE_NRES] = {pod->requests[KE_RES_CPU], pod->requests[KE_RES_MEMORY]};
  if (rcb && ratio > 1.0) podreq[KE_RES_CPU] = amplify(podreq[KE_RES_CPU], ratio);
  int64_t requested[KE_NRES] = {n->node.requested[KE_RES_CPU] + n->rv_req[KE_RES_CPU],
                                 n->node.requested[KE_RES_MEMORY] + n->rv_req[KE_RES_MEMORY]};
  if (!(pod->requests[KE_RES_CPU] == 0 || ratio <= 1.0)) {
    if (n->node.cpu_topology_invalid) return 0;
    const int64_t allocated_milli = cpus_allocated_count(n) * 1000;
    requested[KE_RES_CPU] -= allocated_milli;
    requested[KE_RES_CPU] += amplify(allocated_milli, ratio);
  }
  return numa_resource_score(&c->cfg.numa, requested, n->node.allocatable, podreq);
}


/* ---------------------------------------------------------------------------------------------- */
/* DeviceShare (no reservations / preemption / NUMA affinity / hints / joint allocation / templates)  */
/* ---------------------------------------------------------------------------------------------- */

/* A corev1.ResourceList restricted to one device type's keys (GPU: core, memory, memory-ratio;
 * RDMA/FPGA: one key). */
typedef struct rl {
  uint8_t has[KE_DKEYS];
  int64_t v[KE_DKEYS];
} rl;

static int nkeys(int t) { return t == KE_DEV_GPU ? 3 : 1; }
static rl rl_empty(void) {
  rl r;
  memset(&r, 0, sizeof r);
  return r;
}
/* quotav1.SubtractWithNonNegativeResult (k8s.io/apiserver v0.28.7 quota/v1/resources.go) */
static rl rl_sub_nonneg(rl a, rl b, int nk) {
  rl r = rl_empty();
  for (int k = 0; k < nk; k++) {
    if (a.has[k]) {
      int64_t q = a.v[k] - (b.has[k] ? b.v[k] : 0);
      r.has[k] = 1;
      r.v[k] = q > 0 ? q : 0;
    } else if (b.has[k]) { /* a key only in b: zero */
      r.has[k] = 1;
      r.v[k] = 0;
    }
  }
  return r;
}
/* quotav1.IsZero */
static int rl_is_zero(rl a, int nk) {
  for (int k = 0; k < nk; k++)
    if (a.has[k] && a.v[k] != 0) return 0;
  return 1;
}
/* quotav1.LessThanOrEqual(a, b): only the keys of b that a also has are compared */
static int rl_leq(rl a, rl b, int nk) {
  for (int k = 0; k < nk; k++)
    if (b.has[k] && a.has[k] && a.v[k] > b.v[k]) return 0;
  return 1;
}
/* quotav1.Equals: the same keys with equal values */
static int rl_equal(rl a, rl b, int nk) {
  for (int k = 0; k < nk; k++) {
    if (a.has[k] != b.has[k]) return 0;
    if (a.has[k] && a.v[k] != b.v[k]) return 0;
  }
  return 1;
}
/* quotav1.Add */
static rl rl_add(rl a, rl b, int nk) {
  rl r = rl_empty();
  for (int k = 0; k < nk; k++) {
    r.has[k] = a.has[k] || b.has[k];
    r.v[k] = (a.has[k] ? a.v[k] : 0) + (b.has[k] ? b.v[k] : 0);
  }
  return r;
}

/* the request of one device instance + how many, per type (preparePod + CalcDesiredRequestsAndCount) */
typedef struct ds_pod {
  int status; /* PreFilter status: 0 or UnschedulableAndUnresolvable (invalid device requests) */
  int status_reason; /* its reason: KE_REASON_DS_INVALID_REQUEST (0 here) / _INVALID_HINT / _NO_MATCHED_TEMPLATE */
  int skip;   /* no device requests: PreFilter returns Skip */
  int has[KE_DEV_TYPES];
  int count[KE_DEV_TYPES];
  rl req[KE_DEV_TYPES];
  /* GPURequirements (utils.go:487-513) */
  int gpu_shared;       /* calcDesiredRequestsAndCountForGPU isShared */
  int scope;            /* requiredTopologyScope: KE_SCOPE_* */
  int scope_level;      /* DeviceTopologyScopeLevel[requiredTopologyScope] (0 for "" / unknown) */
  int part_spec;        /* honorGPUPartition from the pod's GPUPartitionSpec */
  int part_restricted;  /* restrictedGPUPartition */
  int64_t ring_bw;      /* rindBusBandwidth, KE_ABSENT = nil */
  /* parsePodDeviceShareExtensions (utils.go:414-455): the hints (NULL = none) */
  const ke_pod_device_hints* h;
  int apply_all[KE_DEV_TYPES]; /* ApplyForAll: the desired count is the node's (matching) devices */
  int vf[KE_DEV_TYPES];        /* mustAllocateVF */
  int sel[KE_DEV_TYPES];       /* a Selector for the type */
  int has_selectors;           /* state.hasSelectors: filterNodeDevice runs */
  int joint_n, joint[KE_DEV_TYPES], joint_pcie; /* DeviceJointAllocate after parsing; RequiredScope SamePCIe */
  int fits_well_planned;       /* podFitsSecondaryDeviceWellPlanned (utils.go:381) */
  int tmpl;                    /* enforceGPUSharedResourceTemplate (utils.go:508-515) */
} ds_pod;

static int valid_percentage(int64_t q) { return !(q > 100 && q % 100 != 0); } /* utils.go:222-227 */

/* GetPodDeviceRequests -> ValidateDeviceRequest -> ConvertDeviceRequest (utils.go:304-342,392-412),
 * then calcDesiredRequestsAndCountForGPU (devicehandler_gpu.go:53-96) and
 * DefaultDeviceHandler.CalcDesiredRequestsAndCount (devicehandler_default.go:44-93, no hint). */
static int rl_equal(rl a, rl b, int nk);
static int tmpl_candidates(const or_cluster* c, const ds_pod* d, int32_t key);
static void ds_prepare_pod(const or_cluster* c, const ke_pod* pod, ds_pod* d) {
  memset(d, 0, sizeof *d);
  const ke_pod_device_hints* h = NULL;
  if (pod->device_hint > 0 && c && pod->device_hint <= c->n_hints) h = &c->hints[pod->device_hint - 1];
  const int64_t* q = pod->device_requests;
  /* GPU combination flags (utils.go:38-52) */
  enum { NV = 1, AMD = 2, KGPU = 4, SHARED = 8, CORE = 16, MEM = 32, RATIO = 64, DCU = 128 };
  int comb = 0;
  if (q[KE_PDR_NVIDIA_GPU] > 0) comb |= NV;
  if (q[KE_PDR_AMD_GPU] > 0) comb |= AMD;
  if (q[KE_PDR_HYGON_DCU] > 0) comb |= DCU;
  if (q[KE_PDR_KOORD_GPU] > 0) comb |= KGPU;
  if (q[KE_PDR_GPU_SHARED] > 0) comb |= SHARED;
  if (q[KE_PDR_GPU_CORE] > 0) comb |= CORE;
  if (q[KE_PDR_GPU_MEMORY] > 0) comb |= MEM;
  if (q[KE_PDR_GPU_MEMORY_RATIO] > 0) comb |= RATIO;
  if (comb) {
    int ok = 0;
    const int64_t core = q[KE_PDR_GPU_CORE], ratio = q[KE_PDR_GPU_MEMORY_RATIO], shared = q[KE_PDR_GPU_SHARED];
    if (comb == KGPU) ok = valid_percentage(q[KE_PDR_KOORD_GPU]);
    else if (comb == NV || comb == AMD || comb == DCU) ok = 1; /* ValidDeviceResourceCombinationsDefaultTrue */
    else if (comb == MEM || comb == RATIO || comb == (CORE | MEM) || comb == (CORE | RATIO))
      ok = (!(comb & CORE) || valid_percentage(core)) && (!(comb & RATIO) || valid_percentage(ratio));
    else if (comb == (SHARED | MEM) || comb == (SHARED | RATIO) || comb == (SHARED | CORE | MEM) ||
             comb == (SHARED | CORE | RATIO))
      ok = (!(comb & CORE) || (core % shared == 0 && core / shared <= 100)) &&
           (!(comb & RATIO) || (ratio % shared == 0 && ratio / shared <= 100));
    if (!ok) {
      d->status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      return;
    }
    /* ConvertDeviceRequest: converted keys */
    int64_t c_core = 0, c_mem = 0, c_ratio = 0, c_shared = 0;
    int h_core = 0, h_mem = 0, h_ratio = 0, h_shared = 0;
    if (comb == NV || comb == AMD || comb == DCU) { /* utils.go:190-212 */
      const int64_t n = q[comb == NV ? KE_PDR_NVIDIA_GPU : comb == AMD ? KE_PDR_AMD_GPU : KE_PDR_HYGON_DCU];
      c_core = c_ratio = n * 100;
      h_core = h_ratio = 1;
    } else if (comb == KGPU) {
      c_core = c_ratio = q[KE_PDR_KOORD_GPU];
      h_core = h_ratio = 1;
    } else {
      if (comb & SHARED) { c_shared = shared; h_shared = 1; }
      if (comb & CORE) { c_core = core; h_core = 1; }
      if (comb & MEM) { c_mem = q[KE_PDR_GPU_MEMORY]; h_mem = 1; }
      if (comb & RATIO) { c_ratio = ratio; h_ratio = 1; }
    }
    /* calcDesiredRequestsAndCountForGPU */
    int64_t n = 1;
    if (h_shared && c_shared > 0) n = c_shared;
    else if (h_ratio && c_ratio > 100 && c_ratio % 100 == 0) n = c_ratio / 100;
    rl r = rl_empty();
    if (h_core) { r.has[KE_DKEY_GPU_CORE] = 1; r.v[KE_DKEY_GPU_CORE] = c_core / n; }
    if (h_ratio) { r.has[KE_DKEY_GPU_MEMORY_RATIO] = 1; r.v[KE_DKEY_GPU_MEMORY_RATIO] = c_ratio / n; }
    else if (h_mem) { r.has[KE_DKEY_GPU_MEMORY] = 1; r.v[KE_DKEY_GPU_MEMORY] = c_mem / n; }
    d->gpu_shared = h_ratio ? (c_ratio / n < 100) : h_mem; /* isShared (devicehandler_gpu.go:84-93) */
    d->has[KE_DEV_GPU] = 1;
    d->count[KE_DEV_GPU] = (int)n;
    d->req[KE_DEV_GPU] = r;
  }
  const int pdr[2] = {KE_PDR_RDMA, KE_PDR_FPGA};
  for (int i = 0; i < 2; i++) {
    const int t = i == 0 ? KE_DEV_RDMA : KE_DEV_FPGA;
    const int64_t v = q[pdr[i]];
    if (v <= 0) continue;
    if (!valid_percentage(v)) {
      d->status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      return;
    }
    int64_t n = 1, per = v;
    const ke_device_hint* ht = h ? &h->hint[t] : NULL;
    if (v > 100 && v % 100 == 0) {
      n = v / 100;
      per = v / n;
    } else if (ht && ht->strategy == KE_DSTRATEGY_APPLY_FOR_ALL) { /* devicehandler_default.go:62-80 */
      d->apply_all[t] = 1;
    } else if (ht && ht->strategy == KE_DSTRATEGY_REQUESTS_AS_COUNT) { /* :81-90 */
      n = v;
      per = ht->exclusive == KE_DEXCL_DEVICE_LEVEL ? 100 : 1;
    }
    d->has[t] = 1;
    d->count[t] = (int)n;
    d->req[t] = rl_empty();
    d->req[t].has[0] = 1;
    d->req[t].v[0] = per;
  }
  d->skip = !(d->has[0] || d->has[1] || d->has[2]);
  /* parseGPURequirements (utils.go:487-513): the pod's GPUPartitionSpec and GPU hint */
  d->scope = pod->gpu_required_topology_scope;
  d->scope_level = d->scope >= KE_SCOPE_NODE && d->scope <= KE_SCOPE_DEVICE ? d->scope : 0;
  d->part_spec = pod->gpu_partition_spec != 0;
  d->part_restricted = d->part_spec && pod->gpu_partition_restricted;
  d->ring_bw = d->part_spec ? pod->gpu_ring_bus_bandwidth : KE_ABSENT;
  d->fits_well_planned = d->has[KE_DEV_GPU] && !d->gpu_shared;
  if (d->skip) return;
  d->h = h;
  if (h) {
    if (h->invalid) { /* newHintSelectors error: PreFilter UnschedulableAndUnresolvable */
      d->status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      d->status_reason = KE_REASON_DS_INVALID_HINT;
      return;
    }
    d->has_selectors = h->has_selectors;
    for (int t = 0; t < KE_DEV_TYPES; t++) {
      d->vf[t] = h->hint[t].vf_selector.present != 0;
      d->sel[t] = h->hint[t].selector.present != 0;
    }
    /* DeviceJointAllocate.DeviceTypes kept by parsePodDeviceShareExtensions (utils.go:430-442): requested, no
     * ApplyForAll hint, annotation order */
    for (int i = 0; i < h->joint_n && i < KE_DEV_TYPES; i++) {
      const int t = h->joint_types[i];
      if (t < 0 || t >= KE_DEV_TYPES || !d->has[t] || h->hint[t].strategy == KE_DSTRATEGY_APPLY_FOR_ALL) continue;
      int dup = 0;
      for (int q = 0; q < d->joint_n; q++) dup |= d->joint[q] == t;
      if (!dup) d->joint[d->joint_n++] = t;
    }
    d->joint_pcie = h->joint_same_pcie;
  }
  /* parseGPURequirements: a shared GPU whose per-GPU request names a template-matched resource is allocated by
   * template; no template of any GPU model equal to the request fails PreFilter (utils.go:508-515) */
  if (d->has[KE_DEV_GPU] && d->gpu_shared && c) {
    const uint32_t keys = c->cfg.deviceshare.template_matched_keys;
    int named = 0;
    for (int k = 0; k < KE_DKEYS; k++) named |= d->req[KE_DEV_GPU].has[k] && ((keys >> k) & 1u);
    if (named) {
      d->tmpl = 1;
      if (tmpl_candidates(c, d, -1) == 0) {
        d->status = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
        d->status_reason = KE_REASON_DS_NO_MATCHED_TEMPLATE;
      }
    }
  }
}

/* findMatchedTemplates(requestsPerGPU, strict) (gpu_shared_resource_templates_cache.go:41-62): templates whose
 * resources equal the per-GPU request, of GPU model `key` (-1: any model) */
static int tmpl_candidates(const or_cluster* c, const ds_pod* d, int32_t key) {
  int n = 0;
  for (int i = 0; i < c->n_tmpl; i++) {
    const ke_gpu_template* t = &c->tmpl[i];
    if (key >= 0 && t->model_key != key) continue;
    rl r = rl_empty();
    for (int k = 0; k < KE_DKEYS; k++) {
      r.has[k] = t->has[k];
      r.v[k] = t->has[k] ? t->value[k] : 0;
    }
    if (rl_equal(r, d->req[KE_DEV_GPU], KE_DKEYS)) n++;
  }
  return n;
}

/* labels.Selector.Matches for a converted metav1.LabelSelector (apimachinery labels/selector.go Requirement.Matches):
 * In: the key is present with a listed value; NotIn: absent, or its value not listed; Exists / DoesNotExist. */
static int label_get(const ke_labels* l, int32_t key, int32_t* value) {
  for (int i = 0; i < l->n && i < KE_MAX_LABELS; i++)
    if (l->key[i] == key) {
      *value = l->value[i];
      return 1;
    }
  return 0;
}
static int sel_matches(const ke_label_selector* s, const ke_labels* l) {
  for (int r = 0; r < s->n && r < KE_MAX_SEL_REQS; r++) {
    const ke_label_requirement* q = &s->req[r];
    int32_t v = 0;
    const int has = label_get(l, q->key, &v);
    int listed = 0;
    for (int i = 0; i < q->n_values && i < KE_MAX_SEL_VALUES; i++) listed |= q->values[i] == v;
    int ok = 0;
    switch (q->op) {
      case KE_SEL_IN: ok = has && listed; break;
      case KE_SEL_NOT_IN: ok = !has || !listed; break;
      case KE_SEL_EXISTS: ok = has; break;
      default: ok = !has; break;
    }
    if (!ok) return 0;
  }
  return 1;
}

/* deviceResources of every device type (map[DeviceType]map[minor]ResourceList): in[t] bit m = minor m present */
typedef struct ds_dres {
  uint16_t in[KE_DEV_TYPES];
  rl r[KE_DEV_TYPES][KE_MAX_MINORS];
} ds_dres;
/* The allocator's arguments beyond the node's cache when DeviceShare allocates for a reservation-matched pod
 * (AutopilotAllocator.Allocate / score, device_allocator.go:96-138,469-492): the whole preemptible map
 * (calcFreeWithPreemptible, device_cache.go:322-348), requiredDeviceResources (has_req; per type restricted when the
 * type has minors, :350-362), and defaultAllocateDevices' required / preferred minors (:364-382).  NULL: the plain
 * path (preemptible = the node's mergedUnmatchedUsed, nd->rs_dev). */
typedef struct ds_rview {
  ds_dres pre;
  int has_req;
  ds_dres req;
  uint16_t required[KE_DEV_TYPES], preferred[KE_DEV_TYPES];
} ds_rview;
static __thread const ds_rview* g_rv = NULL;

/* one device type of a node's cache: minors in ascending order */
typedef struct ds_view {
  int n;
  int minor[KE_MAX_MINORS];
  rl total[KE_MAX_MINORS], used[KE_MAX_MINORS], free[KE_MAX_MINORS];
  int present; /* the filtered nodeDevice kept this type (its free is not all zero) */
} ds_view;

static rl dev_total(const ke_device* d, int nk) {
  rl r = rl_empty();
  if (!d->health) return r; /* buildDeviceResources: unhealthy -> empty (device_cache.go:550-568) */
  for (int k = 0; k < nk; k++) {
    r.has[k] = d->has_total[k];
    r.v[k] = d->has_total[k] ? d->total[k] : 0;
  }
  return r;
}
static rl dev_used(const ke_device* d, int nk) {
  rl r = rl_empty();
  for (int k = 0; k < nk; k++) {
    r.has[k] = d->has_used[k];
    r.v[k] = d->has_used[k] ? d->used[k] : 0;
  }
  return r;
}

/* The original cache view (resetDeviceFree, device_cache.go:165-182). */
static void ds_orig_view(const or_node* nd, int t, ds_view* v) {
  memset(v, 0, sizeof *v);
  const int nk = nkeys(t);
  for (int m = 0; m < KE_MAX_MINORS; m++)
    for (int i = 0; i < nd->n_dev; i++)
      if (nd->dev[i].type == t && nd->dev[i].minor == m) {
        v->minor[v->n] = m;
        v->total[v->n] = dev_total(&nd->dev[i], nk);
        v->used[v->n] = dev_used(&nd->dev[i], nk);
        v->free[v->n] = rl_sub_nonneg(v->total[v->n], v->used[v->n], nk);
        v->n++;
      }
}

/* AutopilotAllocator.numaNodes (nil = off): the NUMA affinity the devices are restricted to */
typedef struct ds_aff {
  int on;
  uint32_t mask;
} ds_aff;
static const ds_aff NO_AFF = {0, 0};

/* filterNodeDevice's device choice (device_allocator.go:137-166): with numaNodes set, a device needs a
 * topology whose NodeID is -1 or in the affinity */
static int dev_allowed(const ke_device* dv, ds_aff a) {
  if (!a.on) return 1;
  if (!dv->has_topology) return 0;
  if (dv->numa_node == -1) return 1;
  return dv->numa_node >= 0 && dv->numa_node < 32 && ((a.mask >> dv->numa_node) & 1u);
}

/* AutopilotAllocator.filterNodeDevice -> nodeDevice.filter (device_allocator.go:137-166,
 * device_cache.go:360-415) with no required resources and an empty preemptible map: the type is dropped
 * when its free is all zero (over every instance) or no instance passes the NUMA affinity; otherwise the
 * passing instances with used' = total - free (kept if non-zero) and free' = total - used'. */
static const ke_device* dev_of(const or_node* nd, int t, int minor) {
  for (int j = 0; j < nd->n_dev; j++)
    if (nd->dev[j].type == t && nd->dev[j].minor == minor) return &nd->dev[j];
  return NULL;
}
/* filterNodeDevice's Selector (device_allocator.go:150-161) */
static int dev_selected(const ds_pod* d, int t, const ke_device* dv) {
  return !d || !d->sel[t] || sel_matches(&d->h->hint[t].selector, &dv->labels);
}
static void ds_filtered_view_aff(const or_node* nd, const ds_pod* d, int t, ds_aff a, ds_view* v) {
  ds_orig_view(nd, t, v);
  const int nk = nkeys(t);
  /* calcFreeWithPreemptible (device_cache.go:322-348) with the pod's restore state as preemptible: an instance
   * with a preemptible entry and a non-zero remaining = total - (used - preemptible) frees that instead
   * (mergedFreeDevices; the others keep deviceFree) */
  for (int i = 0; i < v->n; i++) {
    const int m = v->minor[i];
    rl pre = rl_empty();
    if (g_rv) { /* the reservation path's preemptible map replaces the node's */
      if (!((g_rv->pre.in[t] >> m) & 1u)) continue;
      pre = g_rv->pre.r[t][m];
    } else {
      if (!nd->rs_dev_has[t][m]) continue;
      for (int k = 0; k < nk; k++) {
        pre.has[k] = nd->rs_dev_key[t][m][k];
        pre.v[k] = nd->rs_dev[t][m][k];
      }
    }
    const rl remaining = rl_sub_nonneg(v->total[i], rl_sub_nonneg(v->used[i], pre, nk), nk);
    if (!rl_is_zero(remaining, nk)) v->free[i] = remaining;
  }
  /* requiredDeviceResources of the type (a Restricted reservation): only its minors, free = MinResourceList(free,
   * required) -- the keys of both, the smaller value (pkg/util/resource.go:64-78) */
  if (g_rv && g_rv->has_req && g_rv->req.in[t]) {
    int n = 0;
    for (int i = 0; i < v->n; i++) {
      const int m = v->minor[i];
      if (!((g_rv->req.in[t] >> m) & 1u)) continue;
      const rl q = g_rv->req.r[t][m];
      rl f = rl_empty();
      for (int k = 0; k < nk; k++)
        if (v->free[i].has[k] && q.has[k]) {
          f.has[k] = 1;
          f.v[k] = v->free[i].v[k] < q.v[k] ? v->free[i].v[k] : q.v[k];
        }
      v->minor[n] = m;
      v->total[n] = v->total[i];
      v->used[n] = v->used[i];
      v->free[n] = f;
      n++;
    }
    v->n = n;
  }
  int all_zero = 1;
  for (int i = 0; i < v->n; i++)
    if (!rl_is_zero(v->free[i], nk)) all_zero = 0;
  if (a.on || (d && d->has_selectors)) { /* the instances that pass the affinity and the Selector, ascending minors */
    int n = 0;
    for (int i = 0; i < v->n; i++) {
      const ke_device* dv = dev_of(nd, t, v->minor[i]);
      if (!dev_allowed(dv, a) || !dev_selected(d, t, dv)) continue;
      v->minor[n] = v->minor[i];
      v->total[n] = v->total[i];
      v->used[n] = v->used[i];
      v->free[n] = v->free[i];
      n++;
    }
    if (n == 0) all_zero = 1; /* devices[type] not set: the type is absent */
    v->n = n;
  }
  v->present = v->n > 0 && !all_zero;
  if (!v->present) return;
  for (int i = 0; i < v->n; i++) {
    const rl u = rl_sub_nonneg(v->total[i], v->free[i], nk);
    v->free[i] = rl_is_zero(u, nk) ? v->total[i] : rl_sub_nonneg(v->total[i], u, nk);
  }
}

/* resourceAllocationScorer weights keyed by the device type's keys (scoring.go:142-197) */
static int64_t ds_weight(const ke_deviceshare_args* a, int t, int k) {
  if (t == KE_DEV_GPU) {
    if (k == KE_DKEY_GPU_MEMORY_RATIO) return a->weights[KE_DSW_GPU_MEMORY_RATIO];
    if (k == KE_DKEY_GPU_MEMORY) return a->weights[KE_DSW_GPU_MEMORY];
    return KE_ABSENT;
  }
  return a->weights[t == KE_DEV_RDMA ? KE_DSW_RDMA : KE_DSW_FPGA];
}

/* leastRequestedScore / mostRequestedScore (scoring.go:283-322) */
static int64_t ds_resource_score(int strategy, int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (strategy == KE_STRATEGY_MOST_ALLOCATED) {
    if (requested > capacity) requested = capacity;
    return requested * MAX_NODE_SCORE / capacity;
  }
  if (requested > capacity) return 0;
  return (capacity - requested) * MAX_NODE_SCORE / capacity;
}

/* resourceAllocationScorer.scorer over (requested, allocatable) pairs of the keys with a weight and
 * non-zero total: Σ w·score / Σ w (scoring.go:268-297) */
static int64_t ds_weighted(const ke_deviceshare_args* a, int t, const int64_t* req, const int64_t* cap,
                           const int* use, int nk) {
  int64_t s = 0, ws = 0;
  for (int k = 0; k < nk; k++) {
    if (!use[k]) continue;
    const int64_t w = ds_weight(a, t, k);
    s += ds_resource_score(a->strategy, req[k], cap[k]) * w;
    ws += w;
  }
  return ws == 0 ? 0 : s / ws;
}

/* resourceAllocationScorer.scoreNode (scoring.go:227-257) */
static int64_t ds_score_node(const ke_deviceshare_args* a, int t, const rl* podreq, const ds_view* v) {
  const int nk = nkeys(t);
  int64_t req[KE_DKEYS] = {0}, cap[KE_DKEYS] = {0};
  int use[KE_DKEYS] = {0};
  for (int k = 0; k < nk; k++) {
    if (ds_weight(a, t, k) == KE_ABSENT) continue;
    int64_t total = 0, free = 0;
    for (int i = 0; i < v->n; i++) {
      total += v->total[i].has[k] ? v->total[i].v[k] : 0;
      free += v->free[i].has[k] ? v->free[i].v[k] : 0;
    }
    if (total == 0) continue;
    int64_t r = total;
    if (total >= free) r = total - free + (podreq->has[k] ? podreq->v[k] : 0);
    req[k] = r;
    cap[k] = total;
    use[k] = 1;
  }
  return ds_weighted(a, t, req, cap, use, nk);
}

/* resourceAllocationScorer.scoreDevice (scoring.go:200-225) */
static int64_t ds_score_device(const ke_deviceshare_args* a, int t, const rl* podreq, const rl* total,
                               const rl* free) {
  const int nk = nkeys(t);
  int64_t req[KE_DKEYS] = {0}, cap[KE_DKEYS] = {0};
  int use[KE_DKEYS] = {0};
  for (int k = 0; k < nk; k++) {
    if (ds_weight(a, t, k) == KE_ABSENT) continue;
    const int64_t tq = total->has[k] ? total->v[k] : 0;
    if (tq == 0) continue;
    const int64_t fq = free->has[k] ? free->v[k] : 0;
    int64_t r = tq;
    if (tq >= fq) r = tq - fq + (podreq->has[k] ? podreq->v[k] : 0);
    req[k] = r;
    cap[k] = tq;
    use[k] = 1;
  }
  return ds_weighted(a, t, req, cap, use, nk);
}

/* defaultAllocateDevices (device_allocator.go:353-424) on the filtered view: devices in
 * (score desc, minor asc) order (scoreDevices + sortDeviceResourcesByMinor, device_resources.go:171-208),
 * the first `count` with a non-zero free that covers the request.  Returns the number chosen
 * (picked[] = view indices).  scorer == NULL: Filter's allocator (every score 0). */
/* allocateVF (device_allocator.go:426-455): the lowest-BusID VF (rank) of the groups the VFSelector matches that
 * the node's pods do not hold; -1 = none */
static int vf_pick(const ke_device* dv, const ke_label_selector* vsel) {
  if (!dv) return -1;
  uint64_t cand = 0;
  for (int g = 0; g < dv->n_vf_groups && g < KE_MAX_VF_GROUPS; g++)
    if (sel_matches(vsel, &dv->vf_groups[g].labels)) cand |= dv->vf_groups[g].vfs;
  cand &= ~dv->vf_allocated;
  return cand ? __builtin_ctzll(cand) : -1;
}

/* defaultAllocateDevices with the joint-allocation extras: `pref` = preferred PCIe ranks
 * (sortDeviceResourcesByPreferredPCIe, device_resources.go:211-220: preferred first, then score desc, minor
 * asc), up to max_count devices (maxDesiredCount), and for a pod that must allocate VFs one VF per device
 * (vf_out[i] = its rank; nd / d give the device infos and the VFSelector). */
static int ds_allocate_x(const or_node* nd, const ds_pod* d, const ke_deviceshare_args* scorer, int t, const rl* req,
                         int max_count, uint64_t pref, const ds_view* v, int* picked, int* vf_out) {
  const int nk = nkeys(t);
  if (!v->present) return 0;
  int order[KE_MAX_MINORS], pf[KE_MAX_MINORS];
  int64_t sc[KE_MAX_MINORS];
  const uint16_t rpref = g_rv ? g_rv->preferred[t] : 0, rreq = g_rv ? g_rv->required[t] : 0;
  for (int i = 0; i < v->n; i++) {
    order[i] = i;
    sc[i] = scorer ? ds_score_device(scorer, t, req, &v->total[i], &v->free[i]) : 0;
    const ke_device* dv = nd ? dev_of(nd, t, v->minor[i]) : NULL;
    pf[i] = pref && dv && dv->has_topology && dv->pcie_rank >= 0 && dv->pcie_rank < 64 && ((pref >> dv->pcie_rank) & 1);
    /* sortDeviceResourcesByMinor with a non-empty preferred set overwrites the PCIe flags (device_resources.go:187-193) */
    if (rpref) pf[i] = (rpref >> v->minor[i]) & 1u;
  }
  for (int i = 1; i < v->n; i++) /* insertion sort: preferred, score desc, minor asc */
    for (int j = i; j > 0; j--) {
      const int a = order[j - 1], b = order[j];
      const int before = pf[b] != pf[a] ? pf[b] > pf[a] : (sc[b] > sc[a] || (sc[b] == sc[a] && v->minor[b] < v->minor[a]));
      if (!before) break;
      order[j - 1] = b;
      order[j] = a;
    }
  const int vf = d && d->vf[t];
  int n = 0;
  for (int i = 0; i < v->n && n < max_count; i++) {
    const int k = order[i];
    if (rreq && !((rreq >> v->minor[k]) & 1u)) continue; /* required.Len() > 0 && !required.Has(minor) */
    if (rl_is_zero(v->free[k], nk)) continue;
    if (!rl_leq(*req, v->free[k], nk)) continue;
    int r = -1;
    if (vf) {
      r = vf_pick(dev_of(nd, t, v->minor[k]), &d->h->hint[t].vf_selector);
      if (r < 0) continue;
    }
    if (vf_out) vf_out[n] = r;
    picked[n++] = k;
  }
  return n;
}
static int ds_allocate(const ke_deviceshare_args* scorer, int t, const rl* req, int count, const ds_view* v,
                       int* picked) {
  return ds_allocate_x(NULL, NULL, scorer, t, req, count, 0, v, picked, NULL);
}

/* ---- GPUAllocator (allocator_gpu.go) --------------------------------------------------------- */
static int popcount16(uint32_t x) { return __builtin_popcount(x & 0xFFFFu); }

/* AllocateContext (allocator_gpu.go:52-57,83-89) over the filtered view of the node's GPUs */
typedef struct gpu_ctx {
  uint32_t used;   /* deviceUsedMinorsHash = hashDevices(getRealUsed(...)) (:59-70, :239-254) */
  uint32_t total;  /* minors of removeZeroDevice(deviceTotal) (:114-122) */
  int present;     /* the filtered nodeDevice kept the GPU type: deviceFree[GPU] exists */
  rl free[KE_MAX_MINORS];
  rl crd_total[KE_MAX_MINORS]; /* GPUTopologyScope.minorsResources: the cache total of each GPU */
  uint32_t minors; /* every GPU device of the node (DeviceInfos) */
} gpu_ctx;

static void gpu_ctx_init(const or_node* nd, const ds_view* v, gpu_ctx* g) {
  memset(g, 0, sizeof *g);
  g->present = v->present;
  uint32_t refined = 0; /* the refined deviceTotal's minors */
  if (v->present)
    for (int i = 0; i < v->n; i++) refined |= 1u << v->minor[i];
  for (int i = 0; i < nd->n_dev; i++) {
    const ke_device* dv = &nd->dev[i];
    if (dv->type != KE_DEV_GPU) continue;
    g->minors |= 1u << dv->minor;
    g->crd_total[dv->minor] = dev_total(dv, 3);
    /* original used minors not in the refined total (outside the affinity, or the type dropped) */
    if (!(refined >> dv->minor & 1u) && (dv->has_used[0] || dv->has_used[1] || dv->has_used[2]))
      g->used |= 1u << dv->minor;
  }
  if (!v->present) return;
  for (int i = 0; i < v->n; i++) {
    const int m = v->minor[i];
    g->free[m] = v->free[i];
    if (!rl_is_zero(v->total[i], 3)) g->total |= 1u << m;
    /* refined used: total - free' non-zero (nodeDevice.filter keeps used' only when non-zero) */
    if (!rl_is_zero(rl_sub_nonneg(v->total[i], v->free[i], 3), 3)) g->used |= 1u << m;
  }
}

/* selectPartitionByBinPack (allocator_gpu.go:261-296): for each feasible partition, Σ over the 8/4/2-GPU
 * partitions of the lowest allocation-score group that stay free after it, weight 10000/100/1 x their
 * AllocationScore; sort.Slice descending (stable for <= 12 elements, enforced at the boundary). */
static int gpu_binpack(const or_node* nd, uint32_t used, const int* feas, int nf, int want) {
  if (nf == 1) return feas[0];
  static const int cnts[3] = {8, 4, 2}, wts[3] = {10000, 100, 1};
  int best = -1;
  int64_t best_score = 0;
  for (int f = 0; f < nf; f++) {
    const uint32_t alloc = used | nd->part[feas[f]].minors;
    int64_t score = 0;
    for (int c = 0; c < 3; c++) {
      if (cnts[c] < want) continue;
      int lo = -1; /* indexerOfGPUNumber[0]: the lowest allocation score listed for cnts[c] */
      for (int i = 0; i < nd->n_part; i++)
        if (nd->part[i].number_of_gpus == cnts[c] && (lo < 0 || nd->part[i].allocation_score < nd->part[lo].allocation_score))
          lo = i;
      if (lo < 0) continue;
      for (int i = 0; i < nd->n_part; i++) {
        const ke_gpu_partition* q = &nd->part[i];
        if (q->number_of_gpus != cnts[c] || q->allocation_score != nd->part[lo].allocation_score) continue;
        if (q->minors & alloc) continue;
        score += (int64_t)wts[c] * q->allocation_score;
      }
    }
    if (best < 0 || score > best_score) { /* stable descending sort: first of the maxima */
      best = feas[f];
      best_score = score;
    }
  }
  return best;
}

/* allocateByPartition (allocator_gpu.go:177-237).  Returns the status (0 also when !honor swallows a
 * failure); *out = the chosen partition's minors, 0 = none. */
static int gpu_by_partition(const or_node* nd, const ds_pod* d, const gpu_ctx* g, int honor, uint32_t* out,
                            int* reason) {
  *out = 0;
  if (d->gpu_shared) return 0;
  int st = 0;
  const int want = d->count[KE_DEV_GPU];
  if (!nd->gpu_has_table) {
    st = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    *reason = KE_REASON_DS_MISSING_PARTITION_TABLE;
  } else {
    /* indexer[numberOfGPUs]: groups of equal AllocationScore, ascending (GetGPUPartitionIndexer :165-200) */
    int scores[KE_MAX_GPU_PARTITIONS], ng = 0;
    for (int i = 0; i < nd->n_part; i++) {
      if (nd->part[i].number_of_gpus != want) continue;
      const int sc = nd->part[i].allocation_score;
      int j = 0;
      while (j < ng && scores[j] < sc) j++;
      if (j < ng && scores[j] == sc) continue;
      for (int k = ng; k > j; k--) scores[k] = scores[k - 1];
      scores[j] = sc;
      ng++;
    }
    if (ng == 0) {
      st = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      *reason = KE_REASON_DS_UNSUPPORTED_GPU_REQUESTS;
    } else {
      int feas[KE_MAX_GPU_PARTITIONS], nf = 0;
      for (int gi = 0; gi < ng; gi++) {
        for (int i = 0; i < nd->n_part; i++) {
          const ke_gpu_partition* q = &nd->part[i];
          if (q->number_of_gpus != want || q->allocation_score != scores[gi]) continue;
          if (q->minors & g->used) continue;
          if ((g->total & q->minors) != q->minors) continue;
          if (d->ring_bw != KE_ABSENT) {
            if (q->ring_bus_bandwidth == KE_ABSENT) continue;
            if (d->ring_bw > q->ring_bus_bandwidth) continue;
          }
          feas[nf++] = i;
        }
        if (nf > 0 || d->part_restricted) break;
      }
      if (nf == 0) {
        st = KE_CODE_UNSCHEDULABLE;
        *reason = KE_REASON_DS_INSUFFICIENT_PARTITIONED;
      } else {
        *out = nd->part[gpu_binpack(nd, g->used, feas, nf, want)].minors;
        return 0;
      }
    }
  }
  return honor ? st : 0;
}

/* GPUTopologyScope (allocator_gpu.go:298-309) as GetGPUTopologyScope builds it (allocator_gpu_helper.go:202-263) */
typedef struct gscope {
  int level; /* DeviceTopologyScopeLevel: Node 1, NUMANode 2, PCIe 3 */
  uint32_t minors;
  int n_child;
  int child[KE_MAX_MINORS];
} gscope;

/* Scope tree in an array: [0] = Node, then NUMANode scopes by NodeID, each followed by nothing; PCIe
 * scopes after all NUMA scopes.  Returns the scope count, 0 = nil tree. */
static int gpu_scope_tree(const or_node* nd, gscope* sc) {
  int n_gpu = 0;
  for (int i = 0; i < nd->n_dev; i++) {
    if (nd->dev[i].type != KE_DEV_GPU) continue;
    if (!nd->dev[i].has_topology) return 0; /* info.Topology == nil -> nil */
    n_gpu++;
  }
  if (n_gpu == 0) return 0;
  int numa_ids[KE_MAX_MINORS], nn = 0;
  for (int i = 0; i < nd->n_dev; i++) { /* NUMA ids ascending */
    if (nd->dev[i].type != KE_DEV_GPU) continue;
    const int id = nd->dev[i].numa_node;
    int j = 0;
    while (j < nn && numa_ids[j] < id) j++;
    if (j < nn && numa_ids[j] == id) continue;
    for (int k = nn; k > j; k--) numa_ids[k] = numa_ids[k - 1];
    numa_ids[j] = id;
    nn++;
  }
  int ns = 1;
  memset(&sc[0], 0, sizeof sc[0]);
  sc[0].level = 1;
  for (int i = 0; i < nd->n_dev; i++)
    if (nd->dev[i].type == KE_DEV_GPU) sc[0].minors |= 1u << nd->dev[i].minor;
  for (int a = 0; a < nn; a++) {
    const int ni = ns++;
    memset(&sc[ni], 0, sizeof sc[ni]);
    sc[ni].level = 2;
    sc[0].child[sc[0].n_child++] = ni;
    int pcie[KE_MAX_MINORS], np = 0; /* PCIe ranks of this NUMA node, ascending */
    for (int i = 0; i < nd->n_dev; i++) {
      const ke_device* dv = &nd->dev[i];
      if (dv->type != KE_DEV_GPU || dv->numa_node != numa_ids[a]) continue;
      sc[ni].minors |= 1u << dv->minor;
      int j = 0;
      while (j < np && pcie[j] < dv->pcie_rank) j++;
      if (j < np && pcie[j] == dv->pcie_rank) continue;
      for (int k = np; k > j; k--) pcie[k] = pcie[k - 1];
      pcie[j] = dv->pcie_rank;
      np++;
    }
    for (int b = 0; b < np; b++) {
      const int pi = ns++;
      memset(&sc[pi], 0, sizeof sc[pi]);
      sc[pi].level = 3;
      sc[ni].child[sc[ni].n_child++] = pi;
      for (int i = 0; i < nd->n_dev; i++) {
        const ke_device* dv = &nd->dev[i];
        if (dv->type == KE_DEV_GPU && dv->numa_node == numa_ids[a] && dv->pcie_rank == pcie[b])
          sc[pi].minors |= 1u << dv->minor;
      }
    }
  }
  return ns;
}

typedef struct sres { /* ScopeLevelAllocateResult */
  int ok;
  uint32_t minors;
  int cum, depth;
  int64_t score;
} sres;

typedef struct dctx { /* DeviceLevelContext cache, filled on first visit */
  int seen[KE_MAX_MINORS], sat[KE_MAX_MINORS];
  int64_t score[KE_MAX_MINORS];
} dctx;

/* allocateFromScope (allocator_gpu.go:357-451) */
static sres gpu_from_scope(const gscope* sc, int s, const ds_pod* d, const gpu_ctx* g,
                           const ke_deviceshare_args* scorer, int cum, int depth, dctx* dc) {
  sres none;
  memset(&none, 0, sizeof none);
  const int want = d->count[KE_DEV_GPU];
  if (popcount16(sc[s].minors) < want) return none;
  depth++;
  if (sc[s].minors & g->used) cum++;
  sres best = none;
  for (int c = 0; c < sc[s].n_child; c++) {
    const int ch = sc[s].child[c];
    if (popcount16(sc[ch].minors) < want) continue;
    const sres r = gpu_from_scope(sc, ch, d, g, scorer, cum, depth, dc);
    if (!r.ok) continue;
    if (!best.ok) {
      best = r;
      continue;
    }
    if (best.depth < r.depth || (best.depth == r.depth && best.cum < r.cum)) best = r;
    if (d->gpu_shared && best.depth == r.depth && best.cum == r.cum && best.score < r.score) best = r;
  }
  if (best.ok) return best;
  if (d->scope_level > sc[s].level) return none;
  uint32_t cand = 0;
  int n_cand = 0, satisfied = 0, best_minor = -1;
  int64_t best_score = -1;
  for (int m = 0; m < KE_MAX_MINORS; m++) {
    if (!(sc[s].minors & (1u << m))) continue;
    if (!dc->seen[m]) {
      dc->seen[m] = 1;
      const rl empty = rl_empty();
      const rl* fr = g->present ? &g->free[m] : &empty; /* deviceFree[minor] (nil -> empty) */
      dc->sat[m] = rl_leq(d->req[KE_DEV_GPU], *fr, 3) && (g->total & (1u << m));
      dc->score[m] = 0;
      if (dc->sat[m] && d->gpu_shared && scorer)
        dc->score[m] = ds_score_device(scorer, KE_DEV_GPU, &d->req[KE_DEV_GPU], &g->crd_total[m], fr);
    }
    if (!dc->sat[m]) continue;
    if (!d->gpu_shared) {
      cand |= 1u << m;
      if (++n_cand == want) {
        satisfied = 1;
        break;
      }
      continue;
    }
    satisfied = 1;
    if (dc->score[m] > best_score) {
      best_minor = m;
      best_score = dc->score[m];
    }
  }
  if (!satisfied) return none;
  sres r;
  r.ok = 1;
  r.cum = cum;
  r.depth = depth;
  r.score = best_score;
  r.minors = d->gpu_shared ? (1u << best_minor) : cand;
  return r;
}

/* allocateByDeviceTopology (allocator_gpu.go:312-341) */
static int gpu_by_topology(const or_node* nd, const ds_pod* d, const gpu_ctx* g, const ke_deviceshare_args* scorer,
                           uint32_t* out, int* reason) {
  *out = 0;
  const int required = d->scope != KE_SCOPE_NONE;
  gscope sc[1 + 2 * KE_MAX_MINORS];
  const int ns = gpu_scope_tree(nd, sc);
  if (ns == 0) { /* UnschedulableAndUnresolvable, swallowed when not required */
    *reason = KE_REASON_DS_MISSING_TOPOLOGY_TREE;
    return required ? KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE : 0;
  }
  if (d->gpu_shared && d->count[KE_DEV_GPU] > 1) {
    *reason = KE_REASON_DS_MULTI_SHARED_GPU;
    return required ? KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE : 0;
  }
  dctx dc;
  memset(&dc, 0, sizeof dc);
  const sres r = gpu_from_scope(sc, 0, d, g, scorer, 0, 0, &dc);
  if (!r.ok) {
    *reason = required ? KE_REASON_DS_INSUFFICIENT_TOPOLOGY_SCOPED : KE_REASON_DS_INSUFFICIENT_GPU_TOPOLOGY;
    return KE_CODE_UNSCHEDULABLE;
  }
  *out = r.minors;
  return 0;
}

/* GPUAllocator.Allocate (allocator_gpu.go:72-112; allocateByTemplate is refused at the boundary) on the
 * filtered view.  Returns the status; *mask = the minors chosen. */
static int ds_gpu_allocate(const or_cluster* c, const or_node* nd, const ds_pod* d, const ds_view* v,
                           const ke_deviceshare_args* scorer, uint32_t* mask, int* reason) {
  gpu_ctx g;
  gpu_ctx_init(nd, v, &g);
  *mask = 0;
  int general = 0; /* allocateByTemplate (:135-159): one candidate template of the node's GPU model -> generalAllocate */
  if (d->tmpl) {
    const int nc = tmpl_candidates(c, d, nd->gpu_model_key);
    if (nc == 0) {
      *reason = KE_REASON_DS_NO_MATCHED_TEMPLATE;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    general = nc == 1;
  }
  const int honor = d->part_spec || nd->gpu_honor;
  int st = general ? 0 : gpu_by_partition(nd, d, &g, honor, mask, reason);
  if (st || *mask) return st;
  st = gpu_by_topology(nd, d, &g, scorer, mask, reason); /* generalAllocate (:114-126) */
  if (st || *mask) return st;
  int picked[KE_MAX_MINORS];
  const int n = ds_allocate(scorer, KE_DEV_GPU, &d->req[KE_DEV_GPU], d->count[KE_DEV_GPU], v, picked);
  if (n < d->count[KE_DEV_GPU]) {
    *reason = KE_REASON_DS_INSUFFICIENT_GPU;
    return KE_CODE_UNSCHEDULABLE;
  }
  for (int i = 0; i < n; i++) *mask |= 1u << v->minor[picked[i]];
  return 0;
}

static int ds_insufficient_reason(int t) {
  return t == KE_DEV_GPU ? KE_REASON_DS_INSUFFICIENT_GPU
                         : (t == KE_DEV_RDMA ? KE_REASON_DS_INSUFFICIENT_RDMA : KE_REASON_DS_INSUFFICIENT_FPGA);
}

/* AutopilotAllocator.Prepare (device_allocator.go:74-94) on node nd: per requested type whether it is in
 * requestsPerInstance (a secondary type of a joint pod is left out outside Reserve on a node whose secondary
 * devices are well planned, :188-190) and its desired count (ApplyForAll: the node's devices of the type
 * matching the Selector, devicehandler_default.go:62-80); a type without devices, an ApplyForAll matching none,
 * or a VF pod on a node without VFs of the type fail UnschedulableAndUnresolvable (fixed type order GPU, RDMA, FPGA). */
static int ds_node_prepare(const or_node* nd, const ds_pod* d, int reserve, int* inc, int* count, int* reason) {
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    inc[t] = 0;
    count[t] = 0;
    if (!d->has[t]) continue;
    if (d->joint_n > 0 && t != d->joint[0] && d->fits_well_planned && nd->secondary_well_planned && !reserve) continue;
    int n = 0, matched = 0, vfs = 0;
    for (int i = 0; i < nd->n_dev; i++) {
      const ke_device* dv = &nd->dev[i];
      if (dv->type != t) continue;
      n++;
      matched += dev_selected(d, t, dv);
      vfs |= dv->n_vf_groups > 0;
    }
    if (n == 0) {
      *reason = ds_insufficient_reason(t);
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    count[t] = d->apply_all[t] ? (d->sel[t] ? matched : n) : d->count[t];
    if (count[t] == 0) {
      *reason = ds_insufficient_reason(t);
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    inc[t] = 1;
    (void)vfs;
  }
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    if (!inc[t] || !d->vf[t]) continue;
    int vfs = 0;
    for (int i = 0; i < nd->n_dev; i++) vfs |= nd->dev[i].type == t && nd->dev[i].n_vf_groups > 0;
    if (!vfs) { /* hasVirtualFunctions */
      *reason = t == KE_DEV_RDMA ? KE_REASON_DS_INSUFFICIENT_RDMA_VF : KE_REASON_DS_INSUFFICIENT_FPGA_VF;
      return KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
  }
  return 0;
}

/* allocateDevices (device_allocator.go:320-350) of one type: GPUs through GPUAllocator, other types
 * defaultAllocateDevices; desired / maxDesired as that function derives them from the count and the preferred
 * PCIe set.  out = minors, vf[minor] = VF ranks. */
static int ds_alloc_type(const or_cluster* c, const or_node* nd, const ds_pod* d, int t, const rl* req, int desired,
                         uint64_t pref, ds_aff a, const ke_deviceshare_args* scorer, uint32_t* out, int8_t* vf,
                         int* reason) {
  int max_count = desired;
  const int np = __builtin_popcountll(pref);
  if (np > max_count) max_count = np;
  if (desired == 0) desired = 1;
  if (max_count < desired) max_count = desired;
  ds_view v;
  ds_filtered_view_aff(nd, d, t, a, &v);
  *out = 0;
  if (t == KE_DEV_GPU) return ds_gpu_allocate(c, nd, d, &v, scorer, out, reason);
  int picked[KE_MAX_MINORS], vr[KE_MAX_MINORS];
  const int n = ds_allocate_x(nd, d, scorer, t, req, max_count, pref, &v, picked, vr);
  if (n < desired) {
    *reason = ds_insufficient_reason(t);
    return KE_CODE_UNSCHEDULABLE;
  }
  for (int i = 0; i < n; i++) {
    *out |= 1u << v.minor[picked[i]];
    if (vf) vf[v.minor[picked[i]]] = (int8_t)vr[i];
  }
  return 0;
}

/* the PCIe ranks of the devices in `minors` that have a topology (newPreferredPCIes, :456-467) */
static uint64_t pcie_set(const or_node* nd, int t, uint32_t minors) {
  uint64_t r = 0;
  for (int m = 0; m < KE_MAX_MINORS; m++) {
    if (!((minors >> m) & 1u)) continue;
    const ke_device* dv = dev_of(nd, t, m);
    if (dv && dv->has_topology && dv->pcie_rank >= 0 && dv->pcie_rank < 64) r |= 1ull << dv->pcie_rank;
  }
  return r;
}

/* AutopilotAllocator.Allocate (device_allocator.go:96-138) on the devices the NUMA affinity / Selector leave:
 * Prepare, tryJointAllocate (:205-299; primary type first, the secondary types preferring the primary's PCIe
 * switches, SamePCIe validated) when more than one type is requested, then every other requested type in the
 * fixed order GPU, RDMA, FPGA.  scorer NULL: Filter's allocator.  out[type] = minors, vf[type-1][minor] = VF
 * ranks (optional). */
static int ds_autopilot(const or_cluster* c, const or_node* nd, const ds_pod* d, ds_aff a,
                        const ke_deviceshare_args* scorer, int reserve, uint32_t* out, int8_t (*vf)[KE_MAX_MINORS],
                        int* reason) {
  int inc[KE_DEV_TYPES], count[KE_DEV_TYPES], done[KE_DEV_TYPES] = {0, 0, 0};
  for (int t = 0; t < KE_DEV_TYPES; t++) out[t] = 0;
  int st = ds_node_prepare(nd, d, reserve, inc, count, reason);
  if (st) return st;
  const int n_inc = inc[0] + inc[1] + inc[2];
  if (n_inc > 1 && d->joint_n > 0) {
    const int p = d->joint[0];
    st = ds_alloc_type(c, nd, d, p, &d->req[p], count[p], 0, a, scorer, &out[p], p ? vf[p - 1] : NULL, reason);
    if (st) return st;
    if (!out[p]) {
      *reason = KE_REASON_DS_INSUFFICIENT_PRIMARY;
      return KE_CODE_UNSCHEDULABLE;
    }
    done[p] = 1;
    const uint64_t pcie = pcie_set(nd, p, out[p]);
    for (int j = 1; j < d->joint_n; j++) {
      const int t = d->joint[j];
      int desired = count[t];
      if (d->joint_pcie && desired < __builtin_popcountll(pcie)) desired = __builtin_popcountll(pcie);
      const rl empty = rl_empty();
      st = ds_alloc_type(c, nd, d, t, inc[t] ? &d->req[t] : &empty, desired, pcie, a, scorer, &out[t],
                         t ? vf[t - 1] : NULL, reason);
      if (st) return st;
      done[t] = out[t] != 0;
    }
    if (d->joint_pcie)
      for (int j = 1; j < d->joint_n; j++)
        if (pcie_set(nd, d->joint[j], out[d->joint[j]]) != pcie) { /* validateJointAllocation */
          *reason = KE_REASON_DS_JOINT_VIOLATION;
          return KE_CODE_UNSCHEDULABLE;
        }
  }
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    if (!inc[t] || done[t]) continue;
    st = ds_alloc_type(c, nd, d, t, &d->req[t], count[t], 0, a, scorer, &out[t], t ? vf[t - 1] : NULL, reason);
    if (st) return st;
  }
  return 0;
}

/* ---- DeviceShare allocate-from-reservation (deviceshare/reservation.go:35-450) ---------------------------------- */
/* nodeReservationRestoreStateData of one node for the pod being scheduled: RestoreReservation's matched list (the
 * usable matched reservations whose reserve pod holds device instances, in reservation index order), each with
 * allocatable = nd.getUsed(reservePod), allocated = the owners' usage on those instances (appendAllocatedByHints),
 * remained = subtractAllocated(copy(allocatable), allocated, false); mergeReservationAllocations' sums; and the
 * basicPreemptible the plugin starts from (mergedUnmatchedUsed + the node's preemptible of preemption -- the latter
 * only in golden tests). */
#define DS_MAX_MATCHED 32
typedef struct ds_ralloc {
  int32_t r;      /* reservation index (-1 in golden tests) */
  int32_t policy; /* KE_RSV_POLICY_* */
  ds_dres allocatable, allocated, remained;
} ds_ralloc;
typedef struct ds_rstate {
  int n;
  ds_ralloc m[DS_MAX_MATCHED];
  ds_dres basic, matched_allocatable, matched_allocated;
} ds_rstate;

/* deviceResources.append (device_resources.go:47-63) of one instance: util.AddResourceList (keys of both, summed) */
static void dres_add(ds_dres* d, int t, int m, rl x) {
  if ((d->in[t] >> m) & 1u) {
    d->r[t][m] = rl_add(d->r[t][m], x, nkeys(t));
  } else {
    d->in[t] |= (uint16_t)(1u << m);
    d->r[t][m] = x;
  }
}
/* appendAllocated(dst, src) (device_resources.go:116-132) */
static void dres_append(ds_dres* d, const ds_dres* src) {
  for (int t = 0; t < KE_DEV_TYPES; t++)
    for (int m = 0; m < KE_MAX_MINORS; m++)
      if ((src->in[t] >> m) & 1u) dres_add(d, t, m, src->r[t][m]);
}
/* quotav1.Subtract: the keys of both, a - b (may go negative) */
static rl rl_sub(rl a, rl b, int nk) {
  rl r = rl_empty();
  for (int k = 0; k < nk; k++) {
    r.has[k] = a.has[k] || b.has[k];
    r.v[k] = (a.has[k] ? a.v[k] : 0) - (b.has[k] ? b.v[k] : 0);
  }
  return r;
}

/* the preemptible / required / preferred the allocator gets for matched reservation `idx` (tryAllocateFromReservation,
 * reservation.go:229-280 and scoreWithReservation :323-345): preemptible = basicPreemptible + mergedMatchedAllocated +
 * remained (+ preemptibleInRR, empty: no preemption); preferred = the reservation's minors; Restricted: required =
 * preferred and requiredDeviceResources = calcRequiredDeviceResources (:347-366) -- remained by the reservation's
 * minors, or, with nothing remained, every reservation minor with an empty list.  idx = -1: the node's own
 * allocation (Filter / Score / Reserve fallback): basicPreemptible + mergedMatchedAllocatable.  idx = -2:
 * tryAllocateIgnoreReservation (:290-310): Σ remained + basicPreemptible + mergedMatchedAllocated. */
static void ds_view_of(const ds_rstate* st, int idx, ds_rview* v) {
  memset(v, 0, sizeof *v);
  if (idx == -1) {
    dres_append(&v->pre, &st->basic);
    dres_append(&v->pre, &st->matched_allocatable);
    return;
  }
  if (idx == -2) {
    for (int i = 0; i < st->n; i++) dres_append(&v->pre, &st->m[i].remained);
    dres_append(&v->pre, &st->basic);
    dres_append(&v->pre, &st->matched_allocated);
    return;
  }
  const ds_ralloc* a = &st->m[idx];
  dres_append(&v->pre, &st->basic);
  dres_append(&v->pre, &st->matched_allocated);
  dres_append(&v->pre, &a->remained);
  for (int t = 0; t < KE_DEV_TYPES; t++) v->preferred[t] = a->allocatable.in[t];
  if (a->policy == KE_RSV_POLICY_RESTRICTED) {
    v->has_req = 1;
    int any = 0;
    for (int t = 0; t < KE_DEV_TYPES; t++) {
      v->required[t] = a->allocatable.in[t];
      v->req.in[t] = a->allocatable.in[t] ? (uint16_t)(a->remained.in[t] & a->allocatable.in[t]) : 0;
      for (int m = 0; m < KE_MAX_MINORS; m++)
        if ((v->req.in[t] >> m) & 1u) v->req.r[t][m] = a->remained.r[t][m];
      any |= v->req.in[t] != 0;
    }
    if (!any) /* no resources left: every reservation minor with an empty list */
      for (int t = 0; t < KE_DEV_TYPES; t++) {
        v->req.in[t] = a->allocatable.in[t];
        for (int m = 0; m < KE_MAX_MINORS; m++) v->req.r[t][m] = rl_empty();
      }
  }
}

static int or_resv_usable(const ke_reservation* r);
/* the owners' part of reservation alloc a that RestoreReservation reads: the instances the reserve pod holds,
 * each with the keys of a non-zero owner amount */
static void ds_rsv_parts(const ke_reservation_alloc* a, ds_dres* allocatable, ds_dres* allocated) {
  memset(allocatable, 0, sizeof *allocatable);
  memset(allocated, 0, sizeof *allocated);
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    const int nk = nkeys(t);
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      const uint64_t bit = 1ull << (16 * t + m);
      if (!(a->device_minors & bit)) continue;
      rl al = rl_empty(), ow = rl_empty();
      for (int k = 0; k < nk; k++) {
        al.has[k] = a->device[t][m][k] != 0;
        al.v[k] = a->device[t][m][k];
        ow.has[k] = a->owner_device[t][m][k] != 0;
        ow.v[k] = a->owner_device[t][m][k];
      }
      dres_add(allocatable, t, m, al);
      if ((a->owner_device_minors & bit) && !rl_is_zero(ow, nk)) dres_add(allocated, t, m, ow);
    }
  }
}
/* remained = subtractAllocated(copy(allocatable), allocated, false): quotav1.Subtract per allocated instance, an
 * instance deleted when the result IsZero */
static void ds_remained(const ds_dres* allocatable, const ds_dres* allocated, ds_dres* remained) {
  *remained = *allocatable;
  for (int t = 0; t < KE_DEV_TYPES; t++)
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      if (!((allocated->in[t] >> m) & 1u)) continue;
      const rl x = rl_sub(((remained->in[t] >> m) & 1u) ? remained->r[t][m] : rl_empty(), allocated->r[t][m], nkeys(t));
      if (rl_is_zero(x, nkeys(t))) {
        remained->in[t] &= (uint16_t)~(1u << m);
      } else {
        remained->in[t] |= (uint16_t)(1u << m);
        remained->r[t][m] = x;
      }
    }
}
/* the restore state of `node` for a pod whose matched reservations are flagged in m[] (NULL: none) -- from the
 * holdings, as RestoreReservation + mergeReservationAllocations build it (reservation.go:99-195) */
static void ds_rstate_build(const or_cluster* c, int32_t node, const char* mflags, ds_rstate* st) {
  memset(st, 0, sizeof *st);
  if (!c->ralloc) return;
  for (int32_t i = 0; i < c->n_resv; i++) {
    const ke_reservation* r = &c->resv[i];
    if (r->node != node || !or_resv_usable(r) || !c->ralloc[i].device_minors) continue;
    const int matched = mflags && mflags[i];
    if (!matched && r->allocated_pods == 0) continue; /* an unmatched one restores only with allocated pods */
    ds_dres al, ow, rem;
    ds_rsv_parts(&c->ralloc[i], &al, &ow);
    ds_remained(&al, &ow, &rem);
    if (matched) {
      if (st->n >= DS_MAX_MATCHED) continue;
      ds_ralloc* a = &st->m[st->n++];
      a->r = i;
      a->policy = r->allocate_policy;
      a->allocatable = al;
      a->allocated = ow;
      a->remained = rem;
      dres_append(&st->matched_allocatable, &al);
      dres_append(&st->matched_allocated, &ow);
    } else { /* mergedUnmatchedUsed += subtractAllocated(copy(allocatable), remained, true) */
      ds_dres used = al;
      for (int t = 0; t < KE_DEV_TYPES; t++)
        for (int mm = 0; mm < KE_MAX_MINORS; mm++) {
          if (!((rem.in[t] >> mm) & 1u)) continue;
          const rl x = rl_sub_nonneg(((used.in[t] >> mm) & 1u) ? used.r[t][mm] : rl_empty(), rem.r[t][mm], nkeys(t));
          if (rl_is_zero(x, nkeys(t))) used.in[t] &= (uint16_t)~(1u << mm);
          else used.in[t] |= (uint16_t)(1u << mm), used.r[t][mm] = x;
        }
      dres_append(&st->basic, &used);
    }
  }
}
static int ds_rsv_find(const ds_rstate* st, int32_t r) {
  for (int i = 0; i < st->n; i++)
    if (st->m[i].r == r) return i;
  return -1;
}

static int ds_autopilot(const or_cluster* c, const or_node* nd, const ds_pod* d, ds_aff a,
                        const ke_deviceshare_args* scorer, int reserve, uint32_t* out, int8_t (*vf)[KE_MAX_MINORS],
                        int* reason);
/* AutopilotAllocator.Allocate under view v */
static int ds_autopilot_view(const or_cluster* c, const or_node* nd, const ds_pod* d, const ds_rview* v,
                             const ke_deviceshare_args* scorer, int reserve, uint32_t* out, int8_t (*vf)[KE_MAX_MINORS],
                             int* reason) {
  const ds_rview* keep = g_rv;
  g_rv = v;
  const int st = ds_autopilot(c, nd, d, NO_AFF, scorer, reserve, out, vf, reason);
  g_rv = keep;
  return st;
}
/* tryAllocateFromReservation (reservation.go:207-287) over the matched list (only >= 0: that entry alone): 1 = a
 * reservation satisfied the pod (out = the allocation), 0 = none satisfied and not required (nil result), -1 =
 * Unschedulable "Reservation(s) ..." (required).  A reservation-ignored pod: tryAllocateIgnoreReservation's status. */
static int ds_from_rsv(const or_cluster* c, const or_node* nd, const ds_pod* d, const ds_rstate* st, int only,
                       int required, int ignored, const ke_deviceshare_args* scorer, int reserve, uint32_t* out,
                       int8_t (*vf)[KE_MAX_MINORS], int* reason) {
  (void)ignored;
  if (st->n == 0) return 0;
  ds_rview v;
  for (int i = 0; i < st->n; i++) {
    if (only >= 0 && i != only) continue;
    ds_view_of(st, i, &v);
    int why = 0;
    if (ds_autopilot_view(c, nd, d, &v, scorer, reserve, out, vf, &why) == KE_CODE_SUCCESS) return 1;
  }
  for (int t = 0; t < KE_DEV_TYPES; t++) out[t] = 0;
  if (required) {
    *reason = KE_REASON_RSV_INSUFFICIENT_DEVICES;
    return -1;
  }
  return 0;
}
/* AutopilotAllocator.score (device_allocator.go:469-492) under view v: Σ scoreNode over the requested types the
 * filtered nodeDevice keeps; a Prepare error scores 0 */
static int64_t ds_score_view(const or_cluster* c, const or_node* nd, const ds_pod* d, const ds_rview* v) {
  int inc[KE_DEV_TYPES], cnt[KE_DEV_TYPES], why = 0;
  if (ds_node_prepare(nd, d, 0, inc, cnt, &why)) return 0;
  const ds_rview* keep = g_rv;
  g_rv = v;
  int64_t s = 0;
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    if (!inc[t]) continue;
    ds_view dv;
    ds_filtered_view_aff(nd, d, t, NO_AFF, &dv);
    if (dv.present && dv.n > 0) s += ds_score_node(&c->cfg.deviceshare, t, &d->req[t], &dv);
  }
  g_rv = keep;
  return s;
}
/* scoreWithReservation / ScoreReservation of matched entry i (scoring.go:113-153, reservation.go:323-345); -1: the
 * node's own (Score's fallback, scoring.go:96-102) */
static int64_t ds_rsv_score(const or_cluster* c, const or_node* nd, const ds_pod* d, const ds_rstate* st, int i) {
  ds_rview v;
  ds_view_of(st, i, &v);
  return ds_score_view(c, nd, d, &v);
}
/* golden-vector entry point (Test_tryAllocateFromReservation, deviceshare/reservation_test.go:225-888;
 * TestScoreReservation, scoring_test.go:670-1240): the restore state given directly.  Each deviceResources map is
 * packed as 192 int64 [type][minor][4] = key values 0..2 and a flags word (bit k: key k present, bit 3: the minor is
 * in the map); `matched` holds n x 3 of them (allocatable, allocated, remained) with policy[i].
 *   mode 0: tryAllocateFromReservation over the n entries (required: requiredFromReservation; ignored: the pod is
 *           reservation-ignored; scored: with the plugin's scorer) -> 0 success (out3 = minors per type), 1 nil
 *           result, else the status code (Unschedulable "Reservation(s) ...": *reason = KE_REASON_RSV_*)
 *   mode 1: scoreWithReservation of entry 0 -> 0 and *score */
static void dres_unpack(const int64_t* w, ds_dres* d) {
  memset(d, 0, sizeof *d);
  for (int t = 0; t < KE_DEV_TYPES; t++)
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      const int64_t* e = w + (t * KE_MAX_MINORS + m) * 4;
      if (!((e[3] >> 3) & 1)) continue;
      d->in[t] |= (uint16_t)(1u << m);
      for (int k = 0; k < KE_DKEYS; k++) {
        d->r[t][m].has[k] = (uint8_t)((e[3] >> k) & 1);
        d->r[t][m].v[k] = d->r[t][m].has[k] ? e[k] : 0;
      }
    }
}
int32_t or_ds_rsv_direct(or_cluster* c, const ke_pod* pod, int32_t node, int32_t n, const int32_t* policy,
                         const int64_t* matched, const int64_t* basic, const int64_t* m_alloc, const int64_t* m_allocd,
                         int32_t mode, int32_t required, int32_t ignored, int32_t scored, uint32_t* out3,
                         int64_t* score, int32_t* reason) {
  static ds_rstate st;
  memset(&st, 0, sizeof st);
  if (n < 0 || n > DS_MAX_MATCHED) return KE_ERR_INVALID;
  st.n = n;
  for (int i = 0; i < n; i++) {
    st.m[i].r = -1;
    st.m[i].policy = policy[i];
    dres_unpack(matched + (3 * i + 0) * 192, &st.m[i].allocatable);
    dres_unpack(matched + (3 * i + 1) * 192, &st.m[i].allocated);
    dres_unpack(matched + (3 * i + 2) * 192, &st.m[i].remained);
  }
  dres_unpack(basic, &st.basic);
  dres_unpack(m_alloc, &st.matched_allocatable);
  dres_unpack(m_allocd, &st.matched_allocated);
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  const or_node* nd = &c->nodes[node];
  *reason = 0;
  for (int t = 0; t < KE_DEV_TYPES; t++) out3[t] = 0;
  if (mode == 1) {
    *score = n > 0 ? ds_rsv_score(c, nd, &d, &st, 0) : 0;
    return 0;
  }
  int8_t vf[2][KE_MAX_MINORS];
  int why = 0;
  const ke_deviceshare_args* sc = scored ? &c->cfg.deviceshare : NULL;
  if (n == 0) return 1;
  if (ignored) {
    ds_rview v;
    ds_view_of(&st, -2, &v);
    const int code = ds_autopilot_view(c, nd, &d, &v, sc, 0, out3, vf, &why);
    *reason = why;
    return code;
  }
  const int r = ds_from_rsv(c, nd, &d, &st, -1, required, 0, sc, 0, out3, vf, &why);
  *reason = why;
  return r == 1 ? 0 : r == 0 ? 1 : KE_CODE_UNSCHEDULABLE;
}

/* the pod's DeviceShare restore state on `node` when it is a reservation-matched (or ignored) DeviceShare pod: 1 and
 * *st, else 0 (the plain path) */
static int ds_pod_rstate(const or_cluster* c, const ke_pod* pod, const ds_pod* d, int32_t node, ds_rstate* st) {
  if (d->skip || d->status || !c->ralloc) return 0;
  if (c->ignored && pod->reservation_matched == KE_RSV_IGNORED) {
    char* all = (char*)malloc((size_t)c->n_resv);
    memset(all, 1, (size_t)c->n_resv);
    ds_rstate_build(c, node, all, st);
    free(all);
    return st->n > 0;
  }
  if (!c->resv_m || (pod->reservation_matched != KE_RSV_MATCHED && pod->reservation_matched != KE_RSV_AFFINITY)) return 0;
  ds_rstate_build(c, node, c->resv_m, st);
  return st->n > 0;
}

/* Filter's trial allocation: *gpu = the GPU minors */
static int ds_try_allocate(const or_cluster* c, const or_node* nd, const ds_pod* d, ds_aff a, uint32_t* gpu,
                           int* reason) {
  uint32_t out[KE_DEV_TYPES];
  int8_t vf[2][KE_MAX_MINORS];
  const int st = ds_autopilot(c, nd, d, a, NULL, 0, out, vf, reason);
  *gpu = st ? 0 : out[KE_DEV_GPU];
  return st;
}

/* DeviceShare Filter (plugin.go:311-365): skipped when the topology manager stored an affinity for the
 * node (Admit ran DeviceShare.Allocate on it), else AutopilotAllocator.Allocate. */
int or_ds_filter(const or_cluster* c, const ke_pod* pod, int32_t node, int* reason) {
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  if (d.status) {
    *reason = d.status_reason ? d.status_reason : KE_REASON_DS_INVALID_REQUEST;
    return d.status;
  }
  const or_node* nd = &c->nodes[node];
  if (d.skip) return KE_CODE_SUCCESS;
  uint32_t aff;
  if (numa_stored_affinity(c, pod, node, &aff)) return KE_CODE_SUCCESS;
  if (!nd->has_dev_cache) return KE_CODE_SUCCESS;
  uint32_t gpu;
  int why = 0;
  static __thread ds_rstate rs;
  if (ds_pod_rstate(c, pod, &d, node, &rs)) {
    /* tryAllocateFromReservation over the matched list (plugin.go:350-356): a satisfied reservation passes, none
     * under a reservation affinity fails; else the node's own allocation with the matched reservations' allocatable
     * preemptible (:358-364).  A reservation-ignored pod: tryAllocateIgnoreReservation's status. */
    uint32_t out[KE_DEV_TYPES];
    int8_t vf[2][KE_MAX_MINORS];
    if (pod->reservation_matched == KE_RSV_IGNORED) { /* tryAllocateIgnoreReservation (reservation.go:221-223) */
      ds_rview v;
      ds_view_of(&rs, -2, &v);
      const int st = ds_autopilot_view(c, nd, &d, &v, NULL, 0, out, vf, &why);
      if (st) *reason = why;
      return st;
    }
    const int r = ds_from_rsv(c, nd, &d, &rs, -1, pod->reservation_matched == KE_RSV_AFFINITY, 0, NULL, 0, out, vf, &why);
    if (r == 1) return KE_CODE_SUCCESS;
    if (r == -1) {
      *reason = why;
      return KE_CODE_UNSCHEDULABLE;
    }
    ds_rview v;
    ds_view_of(&rs, -1, &v);
    const int st = ds_autopilot_view(c, nd, &d, &v, NULL, 0, out, vf, &why);
    if (st) *reason = why;
    return st;
  }
  const int st = ds_try_allocate(c, nd, &d, NO_AFF, &gpu, &why);
  if (st) *reason = why;
  return st;
}

/* The DeviceShare NUMA hint provider (topology_hint.go:38-58,119-212).  Returns a provider error status
 * (+ *reason) or 0 with: *none = no preference (the provider returned no hints), else the hint list over
 * the device NUMA ids (IterateBitMasks order, preferred = the minimal affinity size, score 500 when the
 * hint's GPU allocation equals the one on all device NUMA nodes) and *copies = one list per requested
 * device type. */
static int ds_numa_hints(const or_cluster* c, const or_node* nd, const ke_pod* pod, numa_hint* list, int* n,
                         int* copies, int* none, int* reason) {
  *n = 0;
  *copies = 0;
  *none = 1;
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  if (d.status || d.skip || !nd->has_dev_cache || c->cfg.deviceshare.disable_numa_alignment) return 0;
  int ids[KE_MAX_NUMA], k = 0; /* numaTopology.nodes: the NodeIDs of devices with a topology, -1 excluded */
  for (int i = 0; i < nd->n_dev; i++) {
    const ke_device* dv = &nd->dev[i];
    if (!dv->has_topology || dv->numa_node < 0) continue;
    int j = 0;
    while (j < k && ids[j] < dv->numa_node) j++;
    if (j < k && ids[j] == dv->numa_node) continue;
    for (int q = k; q > j; q--) ids[q] = ids[q - 1];
    ids[j] = dv->numa_node;
    k++;
  }
  if (k == 0) return 0; /* no mask to iterate: an empty hint map */
  int prep_reason = 0, inc[KE_DEV_TYPES], cnt_t[KE_DEV_TYPES]; /* Prepare fails on every mask alike */
  const int prep = ds_node_prepare(nd, &d, 0, inc, cnt_t, &prep_reason);
  static __thread uint32_t fmask[255], fgpu[255];
  int nf = 0, min_size = -1, full_st = 0, full_reason = 0;
  uint32_t best_gpu = 0;
  for (int size = 1; size <= k; size++) { /* bitmask.IterateBitMasks(numaNodes) */
    int idx[KE_MAX_NUMA];
    for (int i = 0; i < size; i++) idx[i] = i;
    for (;;) {
      uint32_t mask = 0;
      for (int i = 0; i < size; i++) mask |= 1u << ids[idx[i]];
      int st = prep, why = prep_reason;
      uint32_t gpu = 0;
      if (!st) { /* calcTotalDevicesByNUMA: a requested type with devices there but too few */
        for (int t = 0; t < KE_DEV_TYPES && !st; t++) {
          if (!inc[t]) continue;
          int cnt = 0;
          for (int i = 0; i < nd->n_dev; i++) {
            const ke_device* dv = &nd->dev[i];
            if (dv->type == t && dv->has_topology && dv->numa_node >= 0 && ((mask >> dv->numa_node) & 1u)) cnt++;
          }
          if (cnt > 0 && cnt < cnt_t[t]) st = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, why = KE_REASON_DS_INSUFFICIENT_NUMA_SCOPED;
        }
      }
      if (!st) {
        if (min_size < 0) min_size = k;
        st = ds_try_allocate(c, nd, &d, (ds_aff){1, mask}, &gpu, &why);
        if (!st) {
          fmask[nf] = mask;
          fgpu[nf] = gpu;
          nf++;
          if (size < min_size) min_size = size;
        }
      }
      if (size == k) { /* the mask of every device NUMA node: statusUnsatisfied, bestAllocationResult */
        full_st = st;
        full_reason = why;
        best_gpu = st ? 0 : gpu;
      }
      int i = size - 1;
      while (i >= 0 && idx[i] == k - size + i) i--;
      if (i < 0) break;
      idx[i]++;
      for (int j = i + 1; j < size; j++) idx[j] = idx[j - 1] + 1;
    }
  }
  if (full_st) {
    *reason = full_reason;
    return full_st;
  }
  *none = 0;
  for (int t = 0; t < KE_DEV_TYPES; t++) *copies += inc[t]; /* minAffinitySize: the types of requestsPerInstance */
  for (int i = 0; i < nf; i++) {
    numa_hint h = {fmask[i], __builtin_popcount(fmask[i]) == min_size, 0, fgpu[i] == best_gpu ? 500 : 0};
    list[(*n)++] = h;
  }
  return 0;
}

/* DeviceShare.Allocate during Admit (topology_hint.go:60-117): the allocation on the affinity's NUMA
 * nodes (nil affinity: every device) must succeed. */
static int ds_numa_allocate(const or_cluster* c, const or_node* nd, const ke_pod* pod, uint32_t affinity, int* reason) {
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  if (d.status || d.skip || !nd->has_dev_cache || c->cfg.deviceshare.disable_numa_alignment) return KE_CODE_SUCCESS;
  uint32_t gpu;
  int why = 0;
  const int st = ds_try_allocate(c, nd, &d, (ds_aff){affinity != 0, affinity}, &gpu, &why);
  if (st) *reason = why;
  return st;
}

/* Golden-vector entry points for the DeviceShare NUMA hint provider: the hint list (masks, preferred,
 * scores; *copies lists of it, *none = no preference) or the provider's error status; and
 * DeviceShare.Allocate on an affinity (0 = nil). */
int or_ds_numa_hints(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t* masks, uint8_t* preferred,
                     int64_t* scores, int32_t* n, int32_t* copies, int32_t* none, int32_t* reason) {
  static __thread numa_hint list[255];
  int nn = 0, cp = 0, no = 1, why = 0;
  const int st = ds_numa_hints(c, &c->nodes[node], pod, list, &nn, &cp, &no, &why);
  for (int i = 0; i < nn; i++) {
    masks[i] = list[i].mask;
    preferred[i] = (uint8_t)list[i].preferred;
    scores[i] = list[i].score;
  }
  *n = nn;
  *copies = cp;
  *none = no;
  *reason = why;
  return st;
}

int or_ds_numa_allocate(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t affinity, int32_t* reason) {
  int why = 0;
  const int st = ds_numa_allocate(c, &c->nodes[node], pod, affinity, &why);
  *reason = why;
  return st;
}

/* DeviceShare Score before NormalizeScore (scoring.go:45-103 -> AutopilotAllocator.score
 * device_allocator.go:469-492) for a node that passed Filter. */
int64_t or_ds_score(const or_cluster* c, const ke_pod* pod, int32_t node) {
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  const or_node* nd = &c->nodes[node];
  if (d.status || d.skip || !nd->has_dev_cache) return 0;
  uint32_t aff = 0; /* the stored affinity restricts the devices scored (scoring.go:63-73) */
  const ds_aff a = numa_stored_affinity(c, pod, node, &aff) ? (ds_aff){aff != 0, aff} : NO_AFF;
  int inc[KE_DEV_TYPES], cnt[KE_DEV_TYPES], why = 0;
  if (ds_node_prepare(nd, &d, 0, inc, cnt, &why)) return 0; /* Prepare error: Score returns 0 with an error status */
  static __thread ds_rstate rs;
  if (ds_pod_rstate(c, pod, &d, node, &rs)) {
    /* the nominated reservation's scoreWithNominatedReservation, else the node's own (scoring.go:83-102) */
    const int i = c->ds_nom && pod->reservation_matched != KE_RSV_IGNORED ? ds_rsv_find(&rs, c->ds_nom[node]) : -1;
    return ds_rsv_score(c, nd, &d, &rs, i);
  }
  int64_t s = 0;
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    if (!inc[t]) continue;
    ds_view v;
    ds_filtered_view_aff(nd, &d, t, a, &v);
    if (v.present && v.n > 0) s += ds_score_node(&c->cfg.deviceshare, t, &d.req[t], &v);
  }
  return s;
}

/* DeviceShare Reserve (plugin.go:426-492): allocate with the plugin's scorer, fillGPUTotalMem
 * (devicehandler_gpu.go:98-125), updateCacheUsed (device_cache.go:127-141).  Returns the minor mask. */
/* the affinity DeviceShare's Reserve allocates on: the one the Filter's Admit stored (taken before any
 * Reserve of the pod changes the node), none when the alignment is disabled (plugin.go:452-466) */
static ds_aff ds_reserve_affinity(const or_cluster* c, const ke_pod* pod, int32_t node) {
  uint32_t aff = 0;
  return !c->cfg.deviceshare.disable_numa_alignment && numa_stored_affinity(c, pod, node, &aff)
             ? (ds_aff){aff != 0, aff} : NO_AFF;
}

static uint64_t ds_reserve_on(or_cluster* c, const ke_pod* pod, int32_t node, ds_aff a, int8_t (*vf_out)[KE_MAX_MINORS]);

/* fillGPUTotalMem (devicehandler_gpu.go:98-125): the allocated instance's memory / memory ratio from the other
 * and the device's own gpu-memory total */
static void fill_gpu_total_mem(const ke_device* dev, rl* alloc) {
  const int64_t tm = dev->has_total[KE_DKEY_GPU_MEMORY] && dev->health ? dev->total[KE_DKEY_GPU_MEMORY] : 0;
  if (alloc->has[KE_DKEY_GPU_MEMORY]) { /* memoryBytesToRatio */
    alloc->has[KE_DKEY_GPU_MEMORY_RATIO] = 1;
    alloc->v[KE_DKEY_GPU_MEMORY_RATIO] = (int64_t)((double)alloc->v[KE_DKEY_GPU_MEMORY] / (double)tm * 100.0);
  } else { /* memoryRatioToBytes */
    alloc->has[KE_DKEY_GPU_MEMORY] = 1;
    alloc->v[KE_DKEY_GPU_MEMORY] = alloc->v[KE_DKEY_GPU_MEMORY_RATIO] * tm / 100;
  }
}

/* DeviceShare Reserve's allocation (plugin.go:428-496): for a reservation-matched pod the nominated reservation's
 * (allocateWithNominatedReservation, reservation.go:368-415) when it holds devices and satisfies the pod, else the
 * node's own with the matched reservations' allocatable preemptible (plugin.go:482-487); for a reservation-ignored
 * pod tryAllocateIgnoreReservation's (reservation.go:381-385); else on the stored NUMA affinity `a`. */
static int ds_reserve_alloc(const or_cluster* c, const ke_pod* pod, const ds_pod* d, int32_t node, ds_aff a,
                            uint32_t* out, int8_t (*vf)[KE_MAX_MINORS], int* why) {
  const or_node* nd = &c->nodes[node];
  static __thread ds_rstate rs;
  if (ds_pod_rstate(c, pod, d, node, &rs)) {
    ds_rview v;
    if (pod->reservation_matched == KE_RSV_IGNORED) {
      ds_view_of(&rs, -2, &v);
      return ds_autopilot_view(c, nd, d, &v, &c->cfg.deviceshare, 1, out, vf, why);
    }
    const int i = c->ds_nom ? ds_rsv_find(&rs, c->ds_nom[node]) : -1;
    if (i >= 0 && ds_from_rsv(c, nd, d, &rs, i, 0, 0, &c->cfg.deviceshare, 1, out, vf, why) == 1) return KE_CODE_SUCCESS;
    ds_view_of(&rs, -1, &v);
    return ds_autopilot_view(c, nd, d, &v, &c->cfg.deviceshare, 1, out, vf, why);
  }
  return ds_autopilot(c, nd, d, a, &c->cfg.deviceshare, 1, out, vf, why);
}

/* AutopilotAllocator.Allocate in Reserve (plugin.go:459-486) succeeds: with the alignment disabled nothing
 * checked the devices of a node whose NUMA Admit stored an affinity (Filter skipped, Allocate a no-op) */
static int ds_reserve_feasible(const or_cluster* c, const ke_pod* pod, int32_t node, ds_aff a) {
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  const or_node* nd = &c->nodes[node];
  if (d.status || d.skip || !nd->has_dev_cache) return 1;
  uint32_t out[KE_DEV_TYPES];
  int8_t vf[2][KE_MAX_MINORS];
  int why = 0;
  return ds_reserve_alloc(c, pod, &d, node, a, out, vf, &why) == KE_CODE_SUCCESS;
}

uint64_t or_ds_reserve(or_cluster* c, const ke_pod* pod, int32_t node) {
  return ds_reserve_on(c, pod, node, ds_reserve_affinity(c, pod, node), NULL);
}

/* Reserve: AutopilotAllocator.Allocate with the plugin's scorer in the Reserve phase, then updateCacheUsed
 * (device_cache.go:132-209; VF allocations recorded per minor).  vf_out[type-1][minor] = the VF ranks. */
static uint64_t ds_reserve_on(or_cluster* c, const ke_pod* pod, int32_t node, ds_aff a, int8_t (*vf_out)[KE_MAX_MINORS]) {
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  or_node* nd = &c->nodes[node];
  if (d.status || d.skip || !nd->has_dev_cache) return 0;
  uint32_t out[KE_DEV_TYPES];
  int8_t vf[2][KE_MAX_MINORS];
  memset(vf, -1, sizeof vf);
  int why = 0;
  if (ds_reserve_alloc(c, pod, &d, node, a, out, vf, &why)) return 0; /* passed Filter */
  uint64_t mask = 0;
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    const int nk = nkeys(t);
    for (int minor = 0; minor < KE_MAX_MINORS; minor++) {
      if (!((out[t] >> minor) & 1u)) continue;
      /* the allocation's resources: the per-instance request (jointAllocate's secondary type outside
       * requestsPerInstance allocates its nil request) */
      rl alloc = d.has[t] ? d.req[t] : rl_empty();
      ke_device* dev = (ke_device*)dev_of(nd, t, minor);
      if (t == KE_DEV_GPU) fill_gpu_total_mem(dev, &alloc);
      const rl u = rl_add(dev_used(dev, nk), alloc, nk);
      for (int k = 0; k < nk; k++) {
        dev->has_used[k] = u.has[k];
        dev->used[k] = u.v[k];
      }
      if (t > 0 && vf[t - 1][minor] >= 0) dev->vf_allocated |= 1ull << vf[t - 1][minor];
      mask |= 1ull << (16 * t + minor);
    }
  }
  if (vf_out) memcpy(vf_out, vf, sizeof vf);
  return mask;
}

/* AutopilotAllocator.Allocate on `node` (golden-vector entry point: TestAutopilotAllocator calls it outside
 * Reserve without a scorer): the status, the minors per type and the VF ranks ([type-1][minor]) */
int or_ds_allocate(const or_cluster* c, const ke_pod* pod, int32_t node, int32_t reserve, int32_t scored,
                   uint32_t* out3, int8_t* vf32, int32_t* reason) {
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  *reason = 0;
  for (int t = 0; t < KE_DEV_TYPES; t++) out3[t] = 0;
  memset(vf32, -1, 2 * KE_MAX_MINORS);
  if (d.status) {
    *reason = d.status_reason ? d.status_reason : KE_REASON_DS_INVALID_REQUEST;
    return d.status;
  }
  if (d.skip) return 0;
  int why = 0;
  const int st = ds_autopilot(c, &c->nodes[node], &d, NO_AFF, scored ? &c->cfg.deviceshare : NULL, reserve, out3,
                              (int8_t(*)[KE_MAX_MINORS])vf32, &why);
  *reason = why;
  return st;
}

/* preparePod outcome: status, skip, and per type (count, per-instance request [key] / presence) */
int or_ds_prefilter(const or_cluster* c, const ke_pod* pod, int* skip, int32_t* count, int64_t* req, uint8_t* req_has) {
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  *skip = d.skip;
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    count[t] = d.has[t] ? d.count[t] : 0;
    for (int k = 0; k < KE_DKEYS; k++) {
      req[t * KE_DKEYS + k] = d.req[t].v[k];
      req_has[t * KE_DKEYS + k] = d.has[t] ? d.req[t].has[k] : 0;
    }
  }
  return d.status;
}

/* resourceAllocationScorer.scoreDevice for one instance (golden-vector entry point) */
int64_t or_ds_score_device(const or_cluster* c, int32_t type, const int64_t* req, const uint8_t* req_has,
                           const int64_t* total, const uint8_t* total_has, const int64_t* free,
                           const uint8_t* free_has) {
  rl r = rl_empty(), t = rl_empty(), f = rl_empty();
  for (int k = 0; k < KE_DKEYS; k++) {
    r.has[k] = req_has[k]; r.v[k] = req[k];
    t.has[k] = total_has[k]; t.v[k] = total[k];
    f.has[k] = free_has[k]; f.v[k] = free[k];
  }
  return ds_score_device(&c->cfg.deviceshare, type, &r, &t, &f);
}

/* ---------------------------------------------------------------------------------------------- */
/* state                                                                                           */
/* ---------------------------------------------------------------------------------------------- */

or_cluster* or_create(const ke_config* cfg, int32_t n_nodes) {
  if (!cfg || n_nodes < 0) return NULL;
  or_cluster* c = (or_cluster*)calloc(1, sizeof(or_cluster));
  c->cfg = *cfg;
  c->n = n_nodes;
  c->nodes = (or_node*)calloc((size_t)(n_nodes > 0 ? n_nodes : 1), sizeof(or_node));
  return c;
}

void or_destroy(or_cluster* c) {
  if (!c) return;
  free(c->resv);
  free(c->ralloc);
  free(c->rcpu);
  free(c->roff);
  free(c->rres);
  free(c->moff);
  free(c->mids);
  free(c->last_resv);
  for (int i = 0; i < c->n; i++) {
    free(c->nodes[i].pm);
    free(c->nodes[i].agg);
    free(c->nodes[i].asg);
    free(c->nodes[i].cpus);
    free(c->nodes[i].kept_cpus);
  }
  free(c->nodes);
  free(c->quotas);
  free(c->hints);
  free(c->tmpl);
  free(c->last_vf);
  free(c);
}

int or_set_pod_device_hints(or_cluster* c, int32_t n, const ke_pod_device_hints* hints) {
  if (n < 0 || (n > 0 && !hints)) return KE_ERR_INVALID;
  free(c->hints);
  c->hints = (ke_pod_device_hints*)malloc(sizeof(ke_pod_device_hints) * (size_t)(n > 0 ? n : 1));
  if (n) memcpy(c->hints, hints, sizeof(ke_pod_device_hints) * (size_t)n);
  c->n_hints = n;
  return KE_OK;
}

int or_gpu_templates_load(or_cluster* c, int32_t n, const ke_gpu_template* t) {
  if (n < 0 || (n > 0 && !t)) return KE_ERR_INVALID;
  free(c->tmpl);
  c->tmpl = (ke_gpu_template*)malloc(sizeof(ke_gpu_template) * (size_t)(n > 0 ? n : 1));
  if (n) memcpy(c->tmpl, t, sizeof(ke_gpu_template) * (size_t)n);
  c->n_tmpl = n;
  return KE_OK;
}

/* BeforePreFilter's NodeInfo restore (transformer.go:147-300).  forEachAvailableReservationOnNode skips a
 * reservation that is not available or is AllocateOnce with allocated pods (:181-190).  For the scheduling pod
 * the others are matched (checkReservationMatchedOrIgnored) or, with allocated pods, unmatched (:195-199):
 *  - restoreUnmatchedReservations (:447-473) removes the reserve pod (requests = allocatable) and adds a pod
 *    requesting SubtractWithNonNegativeResult(allocatable, allocated) unless that is zero;
 *  - restoreMatchedReservation (:422-445) removes the reserve pod (NodeInfo.RemovePod).
 * updateNodeInfoRequested / RemovePod move NonZeroRequested with the 100m / 200Mi defaults of a zero request
 * (:491-504).  `matched` (by reservation index) may be NULL; with_matched = 0 leaves the matched ones out. */
static const ke_node_resource* node_xres(const or_node* nd, int32_t id);
static int64_t or_non0(int k, int64_t v) { return v != 0 ? v : (k == KE_RES_CPU ? 100 : 200LL << 20); }
static int or_resv_usable(const ke_reservation* r) { return r->available && !(r->allocate_once && r->allocated_pods > 0); }
/* NodeNUMAResource RestoreReservation for one unmatched reservation (nodenumaresource/reservation.go:196-209) and
 * its share of mergeReservationAllocations (:111-120): allocatable = the reserve pod's NUMANodeResources,
 * allocated = Σ owners', remained = subtractAllocated(copy(allocatable), allocated, false) over allocated's NUMA ids
 * (quotav1.Subtract: keys of both), used = subtractAllocated(copy(allocatable), remained, true) over remained's ids
 * (SubtractWithNonNegativeResult: keys of both, floor 0), added into the node's map (quotav1.Add).  A zero
 * amount in ke_reservation_alloc is an absent key. */
static void or_numa_unmatched_used(or_node* nd, const ke_reservation_alloc* a) {
  int any = 0;
  for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++) any |= a->numa[j] != 0;
  if (!any) return; /* GetAllocatedNUMAResource(reservePod) empty: no allocatable, nothing restored */
  for (int id = 0; id < KE_MAX_NUMA; id++) {
    const int in_alloc = a->numa[2 * id] != 0 || a->numa[2 * id + 1] != 0;
    const int in_owned = a->owner_numa[2 * id] != 0 || a->owner_numa[2 * id + 1] != 0;
    /* remained[id]: allocatable (copy) minus allocated where the owners hold the id */
    int rem_has[KE_NRES] = {0, 0}, rem_in = in_alloc || in_owned;
    int64_t rem[KE_NRES] = {0, 0};
    for (int r = 0; r < KE_NRES; r++) {
      const int ha = a->numa[2 * id + r] != 0, hb = in_owned && a->owner_numa[2 * id + r] != 0;
      rem_has[r] = ha || hb;
      rem[r] = (ha ? a->numa[2 * id + r] : 0) - (hb ? a->owner_numa[2 * id + r] : 0);
    }
    if (!rem_in) continue;
    /* used[id] = SubtractWithNonNegativeResult(allocatable[id], remained[id]) */
    nd->rs_numa_has[id] = 1;
    for (int r = 0; r < KE_NRES; r++) {
      const int ha = a->numa[2 * id + r] != 0;
      if (!ha && !rem_has[r]) continue;
      const int64_t u = (ha ? a->numa[2 * id + r] : 0) - (rem_has[r] ? rem[r] : 0);
      nd->rs_numa_key[id][r] = 1;
      nd->rs_numa[id][r] += u > 0 ? u : 0;
    }
  }
}

/* DeviceShare RestoreReservation for one unmatched reservation (deviceshare/reservation.go:157-178): allocatable =
 * nd.getUsed(reservePod), allocated = appendAllocatedByHints(the reserve pod's minors, owners' usage),
 * remained = subtractAllocated(copy(allocatable), allocated, false), used = subtractAllocated(copy(allocatable),
 * remained, true) -- deviceResources.subtract drops an instance whose result IsZero -- then appendAllocated. */
static void or_dev_unmatched_used(or_node* nd, const ke_reservation_alloc* a) {
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    const int nk = t == KE_DEV_GPU ? 3 : 1;
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      if (!(a->device_minors >> (16 * t + m) & 1)) continue;
      rl al = rl_empty(), ow = rl_empty(), rem;
      for (int k = 0; k < nk; k++) {
        al.has[k] = a->device[t][m][k] != 0;
        al.v[k] = a->device[t][m][k];
        ow.has[k] = a->owner_device[t][m][k] != 0;
        ow.v[k] = a->owner_device[t][m][k];
      }
      const int owned = (a->owner_device_minors >> (16 * t + m) & 1) && !rl_is_zero(ow, nk);
      int rem_in = 1;
      if (owned) { /* quotav1.Subtract, deleted when IsZero */
        rem = rl_empty();
        for (int k = 0; k < nk; k++) {
          rem.has[k] = al.has[k] || ow.has[k];
          rem.v[k] = al.v[k] - ow.v[k];
        }
        rem_in = !rl_is_zero(rem, nk);
      } else {
        rem = al;
      }
      rl used = al; /* an instance absent from remained keeps allocatable's list in used */
      if (rem_in) used = rl_sub_nonneg(al, rem, nk);
      if (rl_is_zero(used, nk)) continue; /* deleted */
      nd->rs_dev_has[t][m] = 1;
      for (int k = 0; k < nk; k++)
        if (used.has[k]) {
          nd->rs_dev_key[t][m][k] = 1;
          nd->rs_dev[t][m][k] += used.v[k];
        }
    }
  }
}

/* a reservation-ignored pod's NodeNUMAResource reusable: mergedMatchedAllocatable over every reservation (the hint
 * view, resource_manager.go:130-138), equal in value to tryAllocateIgnoreReservation's mergedMatchedAllocated + Σ
 * remained (nodenumaresource/reservation.go:437-490) */
static void or_numa_ignored_reusable(or_node* nd, const ke_reservation_alloc* a) {
  for (int id = 0; id < KE_MAX_NUMA; id++)
    for (int r = 0; r < KE_NRES; r++) {
      if (a->numa[2 * id + r] == 0) continue;
      nd->rs_numa_has[id] = 1;
      nd->rs_numa_key[id][r] = 1;
      nd->rs_numa[id][r] += a->numa[2 * id + r];
    }
}

/* with_matched 2: a reservation-ignored pod's restore (every reservation matched, the NUMA reusable above) */
static void or_restore(or_cluster* c, const char* matched, int with_matched) {
  for (int32_t i = 0; i < c->n; i++) {
    or_node* nd = &c->nodes[i];
    for (int k = 0; k < KE_NRES; k++) nd->rv_req[k] = nd->rv_nz[k] = 0;
    nd->rv_pods = 0;
    memset(nd->rv_x, 0, sizeof nd->rv_x);
    memset(nd->rs_numa_has, 0, sizeof nd->rs_numa_has);
    memset(nd->rs_numa_key, 0, sizeof nd->rs_numa_key);
    memset(nd->rs_numa, 0, sizeof nd->rs_numa);
    memset(nd->rs_dev_has, 0, sizeof nd->rs_dev_has);
    memset(nd->rs_dev_key, 0, sizeof nd->rs_dev_key);
    memset(nd->rs_dev, 0, sizeof nd->rs_dev);
  }
  /* the plugins' unmatched restore states: the node's unmatched reservations with allocated pods
   * (transformer.go:195-199) */
  for (int32_t i = 0; c->ralloc && i < c->n_resv; i++) {
    const ke_reservation* r = &c->resv[i];
    if (with_matched == 2 && or_resv_usable(r)) or_numa_ignored_reusable(&c->nodes[r->node], &c->ralloc[i]);
    if (!or_resv_usable(r) || (matched && matched[i]) || r->allocated_pods == 0) continue;
    or_numa_unmatched_used(&c->nodes[r->node], &c->ralloc[i]);
    or_dev_unmatched_used(&c->nodes[r->node], &c->ralloc[i]);
  }
  for (int32_t i = 0; i < c->n_resv; i++) {
    const ke_reservation* r = &c->resv[i];
    if (!or_resv_usable(r)) continue;
    or_node* nd = &c->nodes[r->node];
    const ke_reservation_resource* ex = c->rres ? c->rres + c->roff[i] : NULL;
    const int32_t nex = c->rres ? c->roff[i + 1] - c->roff[i] : 0;
    if (matched && matched[i]) {
      if (with_matched) nd->rv_pods--; /* restoreMatchedReservation: NodeInfo.RemovePod(reservePod) */
      if (with_matched) {
        for (int k = 0; k < KE_NRES; k++) {
          nd->rv_req[k] -= r->allocatable[k];
          nd->rv_nz[k] -= or_non0(k, r->allocatable[k]);
        }
        for (int32_t e = 0; e < nex; e++) /* Requested.ScalarResources of the reserve pod's other names */
          if (ex[e].id != KE_RSV_RES_PODS) nd->rv_x[ex[e].id] -= ex[e].allocatable;
      }
      continue;
    }
    if (r->allocated_pods == 0) continue;
    int64_t rem[KE_NRES];
    int rem_nz = 0; /* quotav1.IsZero(SubtractWithNonNegativeResult(Allocatable, Allocated)) over every name */
    for (int k = 0; k < KE_NRES; k++) {
      rem[k] = r->allocatable[k] - r->allocated[k] > 0 ? r->allocatable[k] - r->allocated[k] : 0;
      rem_nz |= rem[k] != 0;
    }
    for (int32_t e = 0; e < nex; e++) rem_nz |= ex[e].allocatable - ex[e].allocated > 0;
    for (int k = 0; k < KE_NRES; k++) {
      nd->rv_req[k] += -r->allocatable[k] + rem[k];
      nd->rv_nz[k] += -or_non0(k, r->allocatable[k]) + (rem_nz ? or_non0(k, rem[k]) : 0);
    }
    for (int32_t e = 0; e < nex; e++)
      if (ex[e].id != KE_RSV_RES_PODS)
        nd->rv_x[ex[e].id] += -ex[e].allocatable + (ex[e].allocatable - ex[e].allocated > 0 ? ex[e].allocatable - ex[e].allocated : 0);
  }
}
/* An owner pod enters (+1) / leaves (-1) the reservation's AssignedPods: its resource manager / device cache entries
 * are what RestoreReservation sums as the owners' (reservation.go:201-226, deviceshare/reservation.go:165-170).
 * CPUs are counted per owner (c->rcpu), the owners' union is the record's owner_cpuset. */
static void or_owner_update(or_cluster* c, int32_t idx, const ke_pod* pod, const uint64_t* cpuset, const int64_t* numa,
                            uint64_t dev_minors, int sign) {
  if (!c->ralloc || idx < 0 || idx >= c->n_resv) return;
  ke_reservation_alloc* a = &c->ralloc[idx];
  if (!c->rcpu) {
    c->rcpu = (uint8_t*)calloc((size_t)c->n_resv * KE_MAX_CPUS, 1);
    for (int32_t i = 0; i < c->n_resv; i++)
      for (int cpu = 0; cpu < KE_MAX_CPUS; cpu++)
        c->rcpu[(size_t)i * KE_MAX_CPUS + cpu] = (uint8_t)(c->ralloc[i].owner_cpuset[cpu >> 6] >> (cpu & 63) & 1);
  }
  uint8_t* cnt = c->rcpu + (size_t)idx * KE_MAX_CPUS;
  for (int cpu = 0; cpuset && cpu < KE_MAX_CPUS; cpu++) {
    if (!(cpuset[cpu >> 6] >> (cpu & 63) & 1)) continue;
    if (sign > 0 && cnt[cpu] < 255) cnt[cpu]++;
    if (sign < 0 && cnt[cpu] > 0) cnt[cpu]--;
    if (cnt[cpu]) a->owner_cpuset[cpu >> 6] |= 1ull << (cpu & 63);
    else a->owner_cpuset[cpu >> 6] &= ~(1ull << (cpu & 63));
  }
  for (int j = 0; numa && j < KE_MAX_NUMA * KE_NRES; j++) {
    const int64_t v = a->owner_numa[j] + sign * numa[j];
    a->owner_numa[j] = v > 0 ? v : 0;
  }
  if (dev_minors) {
    const or_node* nd = &c->nodes[c->resv[idx].node];
    ds_pod d;
    ds_prepare_pod(c, pod, &d);
    for (int i = 0; i < nd->n_dev; i++) {
      const ke_device* dv = &nd->dev[i];
      const uint64_t bit = 1ull << (16 * dv->type + dv->minor);
      if (!(dev_minors & bit)) continue;
      rl amt = d.has[dv->type] ? d.req[dv->type] : rl_empty();
      if (dv->type == KE_DEV_GPU) fill_gpu_total_mem(dv, &amt);
      int any = 0;
      for (int k = 0; k < KE_DKEYS; k++) {
        int64_t* o = &a->owner_device[dv->type][dv->minor][k];
        if (amt.has[k]) {
          const int64_t v = *o + sign * amt.v[k];
          *o = v > 0 ? v : 0;
        }
        any |= *o != 0;
      }
      if (any) a->owner_device_minors |= bit;
      else a->owner_device_minors &= ~bit;
    }
  }
}

/* RestoreReservation's per-reservation state of a matched reservation (nodenumaresource/reservation.go:187-239,
 * deviceshare/reservation.go:148-180), as the allocate-from-reservation paths read it:
 *  - CPUs: allocatableCPUs = the reserve pod's cpuset; allocatedCPUs starts as that same set and only grows by
 *    allocatable ∩ owner CPUs, so it equals allocatableCPUs (the reference's own construction, pinned by
 *    TestRestoreReservation); remainedCPUs = allocatable minus the owners' CPUs;
 *  - NUMA (only with the reserve pod's NUMA resources): allocatable, allocated = Σ owners', remained =
 *    subtractAllocated(copy(allocatable), allocated, false) -- quotav1.Subtract, may go negative;
 *  - devices (only with the reserve pod's instances): allocatable, allocated = the owners' usage on those instances,
 *    remained = subtractAllocated(copy(allocatable), allocated, false) dropping all-zero instances.
 * A zero amount is an absent ResourceList key. */
int or_restore_state(const or_cluster* c, int32_t r, or_rsv_state* out) {
  if (!c->ralloc || r < 0 || r >= c->n_resv) return KE_ERR_NOT_FOUND;
  const ke_reservation_alloc* a = &c->ralloc[r];
  memset(out, 0, sizeof *out);
  for (int w = 0; w < 4; w++) {
    out->allocatable_cpus[w] = a->cpuset[w];
    out->allocated_cpus[w] = a->cpuset[w];
    out->remained_cpus[w] = a->cpuset[w] & ~a->owner_cpuset[w];
  }
  for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++) out->numa_in |= a->numa[j] != 0;
  if (out->numa_in)
    for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++) {
      out->numa_allocatable[j] = a->numa[j];
      out->numa_allocated[j] = a->owner_numa[j];
      out->numa_remained[j] = a->numa[j] - a->owner_numa[j];
      out->numa_remained_has[j] = a->numa[j] != 0 || a->owner_numa[j] != 0;
    }
  for (int t = 0; t < KE_DEV_TYPES; t++) {
    const int nk = t == KE_DEV_GPU ? 3 : 1;
    for (int m = 0; m < KE_MAX_MINORS; m++) {
      const uint64_t bit = 1ull << (16 * t + m);
      if (!(a->device_minors & bit)) continue;
      out->dev_allocatable_minors |= bit;
      int owned = 0, rem_nz = 0;
      for (int k = 0; k < nk; k++) owned |= (a->owner_device_minors & bit) && a->owner_device[t][m][k] != 0;
      for (int k = 0; k < nk; k++) {
        out->dev_allocatable[t][m][k] = a->device[t][m][k];
        out->dev_allocated[t][m][k] = owned ? a->owner_device[t][m][k] : 0;
        out->dev_remained[t][m][k] = a->device[t][m][k] - out->dev_allocated[t][m][k];
        rem_nz |= out->dev_remained[t][m][k] != 0;
      }
      if (owned) out->dev_allocated_minors |= bit;
      if (rem_nz) out->dev_remained_minors |= bit;
    }
  }
  return KE_OK;
}

static uint8_t or_holds_of(const ke_reservation_alloc* a);
static int or_holds_of_idx(const or_cluster* c, int32_t r) { return c->ralloc ? or_holds_of(&c->ralloc[r]) : 0; }
static uint8_t or_holds_of(const ke_reservation_alloc* a) {
  uint8_t h = 0;
  for (int j = 0; j < KE_MAX_NUMA * KE_NRES; j++)
    if (a->numa[j]) h |= KE_RSV_HOLDS_NUMA;
  for (int w = 0; w < 4; w++)
    if (a->cpuset[w]) h |= KE_RSV_HOLDS_CPUSET;
  if (a->device_minors) h |= KE_RSV_HOLDS_DEVICES;
  return h;
}
int or_reservations_load_full(or_cluster* c, int32_t n, const ke_reservation* rs, const ke_reservation_alloc* allocs,
                              const int32_t* roff, const ke_reservation_resource* res) {
  for (int32_t i = 0; i < n; i++) {
    if (rs[i].node < 0 || rs[i].node >= c->n) return KE_ERR_NOT_FOUND;
    const uint8_t said = rs[i].holds & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET | KE_RSV_HOLDS_DEVICES);
    const int32_t ne = roff ? roff[i + 1] - roff[i] : 0;
    if (!roff && (rs[i].holds & KE_RSV_OTHER_ALLOCATABLE)) return KE_ERR_UNSUPPORTED; /* names without entries */
    if (roff && ((rs[i].holds & KE_RSV_OTHER_ALLOCATABLE) != 0) != (ne > 0)) return KE_ERR_INVALID;
    if (!allocs && said) return KE_ERR_UNSUPPORTED;                      /* holdings without their record */
    if (allocs && or_holds_of(&allocs[i]) != said) return KE_ERR_INVALID;
    for (int32_t e = 0; e < ne; e++) {
      const ke_reservation_resource* x = &res[roff[i] + e];
      if (x->id != KE_RSV_RES_PODS && (x->id < 2 || x->id >= KE_MAX_XRES)) return KE_ERR_INVALID;
      if (x->allocatable <= 0 || x->allocated < 0 || x->reserved < 0) return KE_ERR_INVALID;
      for (int32_t f = 0; f < e; f++)
        if (res[roff[i] + f].id == x->id) return KE_ERR_INVALID; /* one entry per name */
    }
  }
  free(c->resv);
  c->resv = (ke_reservation*)malloc(sizeof(ke_reservation) * (size_t)(n > 0 ? n : 1));
  if (n > 0) memcpy(c->resv, rs, sizeof(ke_reservation) * (size_t)n);
  free(c->ralloc);
  c->ralloc = NULL;
  free(c->rcpu);
  c->rcpu = NULL;
  free(c->roff);
  free(c->rres);
  c->roff = NULL;
  c->rres = NULL;
  if (roff) {
    c->roff = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    memcpy(c->roff, roff, sizeof(int32_t) * (size_t)(n + 1));
    c->rres = (ke_reservation_resource*)malloc(sizeof(ke_reservation_resource) * (size_t)(roff[n] > 0 ? roff[n] : 1));
    if (roff[n] > 0) memcpy(c->rres, res, sizeof(ke_reservation_resource) * (size_t)roff[n]);
  }
  if (allocs && n > 0) {
    c->ralloc = (ke_reservation_alloc*)malloc(sizeof(ke_reservation_alloc) * (size_t)n);
    memcpy(c->ralloc, allocs, sizeof(ke_reservation_alloc) * (size_t)n);
  }
  c->n_resv = n;
  or_restore(c, NULL, 0);
  return KE_OK;
}
int or_reservations_load_ex(or_cluster* c, int32_t n, const ke_reservation* rs, const ke_reservation_alloc* allocs) {
  return or_reservations_load_full(c, n, rs, allocs, NULL, NULL);
}
int or_reservations_load(or_cluster* c, int32_t n, const ke_reservation* rs) {
  return or_reservations_load_ex(c, n, rs, NULL);
}
int or_reservation_resources_get(const or_cluster* c, int32_t r, int32_t cap, ke_reservation_resource* out, int32_t* n) {
  if (r < 0 || r >= c->n_resv) return KE_ERR_INVALID;
  *n = c->rres ? c->roff[r + 1] - c->roff[r] : 0;
  for (int32_t e = 0; e < cap && e < *n; e++) out[e] = c->rres[c->roff[r] + e];
  return KE_OK;
}
int or_reservation_allocs_get(const or_cluster* c, int32_t n, ke_reservation_alloc* out) {
  if (n < 0 || n > c->n_resv) return KE_ERR_INVALID;
  for (int32_t i = 0; i < n; i++) {
    if (c->ralloc) out[i] = c->ralloc[i];
    else memset(&out[i], 0, sizeof out[i]);
  }
  return KE_OK;
}
int or_reservations_get(const or_cluster* c, int32_t n, ke_reservation* out) {
  if (n < 0 || n > c->n_resv) return KE_ERR_INVALID;
  if (n > 0) memcpy(out, c->resv, sizeof(ke_reservation) * (size_t)n);
  return KE_OK;
}
int or_pod_reservations(or_cluster* c, int32_t n_pods, const int32_t* offsets, const int32_t* ids) {
  free(c->moff);
  free(c->mids);
  c->moff = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n_pods + 1));
  memcpy(c->moff, offsets, sizeof(int32_t) * (size_t)(n_pods + 1));
  const int32_t m = offsets[n_pods];
  c->mids = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
  if (m > 0) memcpy(c->mids, ids, sizeof(int32_t) * (size_t)m);
  c->m_pods = n_pods;
  for (int32_t j = 0; j < m; j++)
    if (ids[j] < 0 || ids[j] >= c->n_resv) return KE_ERR_NOT_FOUND;
  return KE_OK;
}

/* ScoreReservation -> scoreReservation (reservation/scoring.go:141-164, 191-210): requested = PodRequests +
 * allocated; over RemoveZeros(allocatable) -- every name, "pods" too: MaxNodeScore * req.MilliValue() /
 * capacity.MilliValue() for each resource with req <= capacity, summed, divided by the number of resources.
 * (128-bit products: Go's int64 product wraps only beyond ~9.2e13 of a non-cpu resource.) */
static void or_score_term(int64_t req, int64_t cap, int milli_is_value, int64_t* s, int64_t* w) {
  (*w)++;
  if (req > cap) return;
  const __int128 m = milli_is_value ? 1 : 1000; /* cpu: MilliValue(); others: Value() * 1000 */
  *s += (int64_t)((__int128)MAX_NODE_SCORE * req * m / ((__int128)cap * m));
}
/* the pod's PodRequests of resource id (cpu / memory: requests; others: its ke_pod.xres entry) */
static int64_t pod_xres(const ke_pod* pod, int32_t id);
static int64_t or_pod_request_of(const ke_pod* pod, int32_t id) {
  if (id == KE_XRES_CPU) return pod->requests[KE_RES_CPU];
  if (id == KE_XRES_MEMORY) return pod->requests[KE_RES_MEMORY];
  return pod_xres(pod, id);
}
int64_t or_reservation_score(const ke_reservation* r, const ke_pod* pod) {
  int64_t s = 0, w = 0;
  for (int k = 0; k < KE_NRES; k++)
    if (r->allocatable[k] != 0) or_score_term(pod->requests[k] + r->allocated[k], r->allocatable[k], k == KE_RES_CPU, &s, &w);
  return w ? s / w : 0;
}
static int64_t or_reservation_score_idx(const or_cluster* c, int32_t i, const ke_pod* pod) {
  const ke_reservation* r = &c->resv[i];
  int64_t s = 0, w = 0;
  for (int k = 0; k < KE_NRES; k++)
    if (r->allocatable[k] != 0) or_score_term(pod->requests[k] + r->allocated[k], r->allocatable[k], k == KE_RES_CPU, &s, &w);
  for (int32_t e = c->rres ? c->roff[i] : 0; c->rres && e < c->roff[i + 1]; e++) {
    const ke_reservation_resource* x = &c->rres[e];
    or_score_term((x->id == KE_RSV_RES_PODS ? 0 : or_pod_request_of(pod, x->id)) + x->allocated, x->allocatable, 0, &s, &w);
  }
  return w ? s / w : 0;
}

/* FilterNominateReservation (reservation/plugin.go:707-738) -> filterWithReservations(..., true) on one
 * reservation (:351-442): skipped (not nominable) without a name of rInfo.ResourceNames shared with the pod
 * (:369-375); fitsNode (:447-497; preemptible empty) with podRequested = Requested after the unmatched restore
 * (scalars too), rRemained = GetAvailable = max(0, allocatable - allocated - reserved) per name, allRAllocated =
 * Σ allocated of the node's matched reservations; fitsReservation (:499-569) for the Restricted policy (the "pods"
 * cap, then every requested name of ResourceNames within allocatable - reserved - allocated), else the node fit.
 * The NUMA / DeviceShare FilterNominateReservation pass for pods without cpuset, NUMA policy or devices. */
static int64_t or_rsv_entry(const or_cluster* c, int32_t i, int32_t id, const ke_reservation_resource** out) {
  *out = NULL;
  for (int32_t e = c->rres ? c->roff[i] : 0; c->rres && e < c->roff[i + 1]; e++)
    if (c->rres[e].id == id) *out = &c->rres[e];
  return *out ? 1 : 0;
}
static int64_t or_avail(int64_t a, int64_t al, int64_t rs) { return a - al - rs > 0 ? a - al - rs : 0; }
static int or_resv_nominable(const or_cluster* c, int32_t ri, const ke_pod* pod, int32_t node,
                             const int64_t* pod_requested, const int64_t* all_allocated, int affinity) {
  const ke_reservation* r = &c->resv[ri];
  const int32_t e0 = c->rres ? c->roff[ri] : 0, e1 = c->rres ? c->roff[ri + 1] : 0;
  int shared = 0;
  for (int k = 0; k < KE_NRES; k++)
    if (r->allocatable[k] != 0 && !((r->names_excluded >> k) & 1) && pod->requests[k] != 0) shared = 1;
  for (int32_t e = e0; e < e1; e++)
    if (!c->rres[e].excluded && c->rres[e].id != KE_RSV_RES_PODS && or_pod_request_of(pod, c->rres[e].id) != 0) shared = 1;
  if (!shared && !affinity) return 0; /* plugin.go:373: skipped only without a reservation affinity */
  /* fitsNode's pod count (plugin.go:450-453): len(nodeInfo.Pods) of the snapshot NodeInfo the BeforePreFilter
   * restore left (the matched reserve pods removed: rv_pods after or_restore(m, 1)) minus len(matchedOrIgnored) */
  int32_t n_matched = 0;
  for (int32_t i = 0; i < c->n_resv; i++)
    if (c->resv[i].node == node && or_resv_usable(&c->resv[i]) && c->resv_m && c->resv_m[i]) n_matched++;
  /* (restoreMatchedReservation removed one reserve pod per matched reservation from Pods; the unmatched restore
   * moves only Requested) */
  const int64_t pods_restored = (int64_t)c->nodes[node].node.pod_count - n_matched;
  int node_fits = pods_restored - n_matched + 1 <= (int64_t)c->nodes[node].node.allowed_pods;
  /* the pod's ephemeral storage / scalar resources (ke_pod.xres): Allocatable - (podRequested - rRemained -
   * allRAllocated) per name (plugin.go:487-495); without any request only the pod count is checked (:455-460) */
  int other = 0;
  for (int32_t e = 0; e < pod->n_xres; e++)
    other |= pod->xres_id[e] != KE_XRES_CPU && pod->xres_id[e] != KE_XRES_MEMORY && pod->xres_value[e] != 0;
  if (!(pod->requests[KE_RES_CPU] == 0 && pod->requests[KE_RES_MEMORY] == 0) || other) {
    for (int k = 0; k < KE_NRES; k++) {
      const int64_t remained = or_avail(r->allocatable[k], r->allocated[k], r->reserved[k]);
      const int64_t avail = c->nodes[node].node.allocatable[k] - (pod_requested[k] - remained - all_allocated[k]);
      if (pod->requests[k] > avail) node_fits = 0;
    }
    for (int32_t e = 0; e < pod->n_xres; e++) {
      const int32_t id = pod->xres_id[e];
      if (id == KE_XRES_CPU || id == KE_XRES_MEMORY || pod->xres_value[e] == 0) continue;
      const ke_node_resource* x = node_xres(&c->nodes[node], id);
      /* podRequested: the node's requested with the unmatched restore (its scalar delta: pod_requested[KE_NRES + id],
       * taken by or_resv_begin before the matched restore) */
      const int64_t q = (x ? x->requested : 0) + pod_requested[KE_NRES + id];
      const ke_reservation_resource* re;
      const int64_t remained = or_rsv_entry(c, ri, id, &re) ? or_avail(re->allocatable, re->allocated, re->reserved) : 0;
      if (pod->xres_value[e] > (x ? x->allocatable : 0) - (q - remained - all_allocated[KE_NRES + id])) node_fits = 0;
    }
  }
  int resv_fits = node_fits;
  if (r->allocate_policy == KE_RSV_POLICY_RESTRICTED) {
    resv_fits = 1;
    const ke_reservation_resource* pods_e;
    if (or_rsv_entry(c, ri, KE_RSV_RES_PODS, &pods_e) && (int64_t)r->allocated_pods + 1 > pods_e->allocatable) resv_fits = 0;
    for (int k = 0; k < KE_NRES; k++) {
      if (r->allocatable[k] == 0 || ((r->names_excluded >> k) & 1) || pod->requests[k] == 0) continue; /* Mask; zero skipped */
      if (pod->requests[k] > r->allocatable[k] - r->reserved[k] - r->allocated[k]) resv_fits = 0;
    }
    for (int32_t e = e0; e < e1; e++) {
      const ke_reservation_resource* x = &c->rres[e];
      if (x->excluded || x->id == KE_RSV_RES_PODS) continue;
      const int64_t q = or_pod_request_of(pod, x->id);
      if (q != 0 && q > x->allocatable - x->reserved - x->allocated) resv_fits = 0;
    }
  }
  return node_fits && resv_fits;
}

int or_node_info_requested(const or_cluster* c, int32_t node, int64_t* requested, int64_t* non_zero) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  const or_node* nd = &c->nodes[node];
  for (int k = 0; k < KE_NRES; k++) {
    requested[k] = nd->node.requested[k] + nd->rv_req[k];
    const ke_node_resource* r = node_xres(nd, k);
    non_zero[k] = r ? r->requested + nd->rv_nz[k] : KE_ABSENT;
  }
  return KE_OK;
}

int or_node_device_flags(or_cluster* c, int32_t node, int32_t secondary_well_planned, int32_t gpu_model_key) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  c->nodes[node].secondary_well_planned = secondary_well_planned != 0;
  c->nodes[node].gpu_model_key = gpu_model_key;
  return KE_OK;
}

int or_last_vf_ranks(const or_cluster* c, int32_t n, int8_t* out) {
  for (int32_t p = 0; p < n; p++)
    for (int k = 0; k < 2 * KE_MAX_MINORS; k++)
      out[(int64_t)p * 2 * KE_MAX_MINORS + k] = p < c->last_vf_n && c->last_vf ? c->last_vf[(int64_t)p * 2 * KE_MAX_MINORS + k] : -1;
  return KE_OK;
}

int or_quotas_load(or_cluster* c, const ke_quota_args* args, const ke_quota* q, int32_t n) {
  if (!c->quotas) c->quotas = (or_quotas*)calloc(1, sizeof(or_quotas));
  if (!c->quotas) return KE_ERR_INVALID;
  return orq_load(c->quotas, args, q, n);
}

int or_quota_state(const or_cluster* c, int32_t q, int64_t* limit, uint8_t* limit_has, int64_t* used,
                   int64_t* np_used) {
  if (!c->quotas || q < 0 || q >= c->quotas->n) return KE_ERR_NOT_FOUND;
  for (int r = 0; r < KE_NRES; r++) {
    if (limit) limit[r] = c->quotas->limit[q][r];
    if (limit_has) limit_has[r] = c->quotas->limit_has[q][r];
    if (used) used[r] = c->quotas->q[q].used[r];
    if (np_used) np_used[r] = c->quotas->q[q].non_preemptible_used[r];
  }
  return KE_OK;
}

int or_node_cpus_set(or_cluster* c, int32_t node, int32_t n, const ke_cpu* cpus, int32_t max_ref) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  or_node* nd = &c->nodes[node];
  if (n <= 0) {
    free(nd->cpus);
    nd->cpus = NULL;
    return n < 0 ? KE_ERR_INVALID : KE_OK;
  }
  if (n > ACC_MAX_CPUS || max_ref < 1) return KE_ERR_INVALID;
  or_cpus* x = (or_cpus*)calloc(1, sizeof(or_cpus));
  for (int i = 0; i < n; i++) {
    const int id = cpus[i].cpu_id;
    if (id < 0 || id >= ACC_MAX_CPUS || x->t.valid[id] || cpus[i].ref_count < 0 || cpus[i].exclusive > 2) {
      free(x);
      return KE_ERR_INVALID;
    }
    x->t.valid[id] = 1;
    x->t.core[id] = cpus[i].core_id;
    x->t.node[id] = cpus[i].numa_id;
    x->t.socket[id] = cpus[i].socket_id;
    x->reserved[id] = cpus[i].reserved;
    if (cpus[i].ref_count > 0) {
      x->al.present[id] = 1;
      x->al.ref[id] = cpus[i].ref_count;
      x->al.excl[id] = cpus[i].exclusive;
    }
  }
  acc_topo_finish(&x->t);
  x->max_ref = max_ref;
  int bare = 1; /* no allocatedCPUs given: the parked NodeAllocation comes back by CPU id */
  for (int i = 0; i < ACC_MAX_CPUS; i++) bare = bare && !x->al.present[i];
  if (bare && nd->kept_cpus)
    for (int i = 0; i < ACC_MAX_CPUS; i++)
      if (x->t.valid[i] && nd->kept_cpus->al.present[i]) {
        x->al.present[i] = 1;
        x->al.ref[i] = nd->kept_cpus->al.ref[i];
        x->al.excl[i] = nd->kept_cpus->al.excl[i];
      }
  free(nd->kept_cpus);
  nd->kept_cpus = NULL;
  free(nd->cpus);
  nd->cpus = x;
  return KE_OK;
}

/* NodeNUMAResource Reserve (resourceManager.Allocate with the affinity the Filter stored,
 * resource_manager.go:194-225): the NUMA allocation on a NUMA-policy node and the cpuset of a binding
 * pod, both from the state before the pod.  Returns -1 when Allocate fails (Reserve fails: the pod is
 * not placed). */
typedef struct reserve_plan {
  int64_t dist[KE_MAX_NUMA][KE_NRES]; /* per zone of the node (zone order) */
  uint64_t cpus[ACC_WORDS];
  int excl;
} reserve_plan;

static int or_numa_from_rsv(const or_cluster* c, const ke_pod* pod, int32_t node, int32_t only, int required,
                            uint64_t* out);
/* nom_r: the reservation the Reservation plugin nominated on the node for a KE_RSV_MATCHED pod (-1 = none; the
 * pod's matched flags in c->resv_m): NodeNUMAResource Reserve allocates from it first
 * (allocateWithNominatedReservation, nodenumaresource/reservation.go:492-522) -- a binding pod on a node without
 * a NUMA policy; a binding pod with a reservation affinity and no nominated reservation fails ("no nominated
 * reservation", :508-513) */
static int or_reserve_plan(const or_cluster* c, const ke_pod* pod, int32_t node, reserve_plan* rp, int32_t nom_r) {
  const or_node* n = &c->nodes[node];
  memset(rp, 0, sizeof *rp);
  if (pod_requests_zero(pod)) return 0;
  int exclusive;
  const int policy = effective_policy(n, pod, &exclusive);
  numa_cs cs;
  numa_cs_build(c, n, pod, &cs);
  rp->excl = cs.excl;
  if (cs.rcb && !cs.valid) return -1;
  if (c->ignored && cs.rcb && policy == KE_NUMA_POLICY_NONE) {  /* allocateWithNominatedReservation, ignored */
    const int fr = or_numa_ignored(c, pod, node, rp->cpus);
    if (fr < 0) return -1;
    if (fr > 0) return 0;
  }
  if (c->resv_m && cs.rcb && policy == KE_NUMA_POLICY_NONE) {
    const int required = pod->reservation_matched == KE_RSV_AFFINITY;
    if (nom_r < 0 && required) return -1;
    if (nom_r >= 0) {
      const int fr = or_numa_from_rsv(c, pod, node, nom_r, required, rp->cpus);
      if (fr < 0) return -1;
      if (fr > 0) return 0;
    }
  }
  if (((c->resv_m && !c->ignored) || (c->ignored && cs.rcb)) && policy > KE_NUMA_POLICY_NONE && n->n_zone > 0) {
    /* a matched pod on a node of its reservations holding NUMA resources / CPUs (plugin.go:552-566):
     * allocateWithNominatedReservation, else tryAllocateFromNode, on the stored affinity; an ignored binding pod
     * beside held NUMA resources / CPUs: tryAllocateIgnoreReservation */
    int32_t M[64];
    const int nM = c->ignored ? numa_rsv_ignored(c, node, M) : numa_rsv_matched(c, node, M);
    if (nM > 0) {
      uint32_t aff = 0;
      int reason;
      if (numa_admit(c, n, pod, policy, exclusive, &aff, &reason, &cs) != KE_CODE_SUCCESS) return -1;
      numa_opt used;
      int64_t d16[2 * KE_MAX_NUMA];
      uint64_t pc[ACC_WORDS];
      if (!numa_matched_alloc(c, pod, node, M, nM, nom_r, aff, &used, d16, pc)) return -1;
      for (int z = 0; z < n->n_zone; z++)
        for (int r = 0; r < KE_NRES; r++)
          rp->dist[z][r] = n->zone[z].id >= 0 && n->zone[z].id < KE_MAX_NUMA ? d16[2 * n->zone[z].id + r] : 0;
      if (cs.rcb) memcpy(rp->cpus, pc, sizeof pc);
      return 0;
    }
  }
  numa_view v;
  int have = 0;
  if (policy > KE_NUMA_POLICY_NONE && n->n_zone > 0) {
    uint32_t aff = 0;
    int reason;
    if (numa_admit(c, n, pod, policy, exclusive, &aff, &reason, &cs) != KE_CODE_SUCCESS) return cs.rcb ? -1 : 0;
    if (!numa_allocation(n, pod, aff, &v, rp->dist, &cs)) return cs.rcb ? -1 : 0;
    have = 1;
  }
  if (cs.rcb &&
      cpuset_allocate_cs(n, &cs, have ? &v : NULL, have ? (const int64_t(*)[KE_NRES])rp->dist : NULL, rp->cpus) != 0)
    return -1;
  return 0;
}

/* resourceManager.Update -> NodeAllocation.addPodAllocation (node_allocation.go:111-156): RefCount++
 * and the pod's exclusive policy per CPU, the NUMA nodes' single / shared status, the NUMA allocation
 * added to the zones' entries (quotav1.Add keys). */
static void or_reserve_apply(or_cluster* c, int32_t node, const reserve_plan* rp, int64_t* out16) {
  or_node* n = &c->nodes[node];
  for (int z = 0; z < n->n_zone; z++) /* state.allocation: the pod carries it whatever Update records */
    if (out16)
      for (int r = 0; r < KE_NRES; r++) out16[2 * n->zone[z].id + r] = rp->dist[z][r];
  /* resourceManager.Update returns before recording anything when !CPUTopology.IsValid()
   * (resource_manager.go:461-466) */
  if (!cpus_valid(n)) return;
  if (n->cpus) {
    or_cpus* x = n->cpus;
    int used[ACC_MAX_CPUS], nu = 0;
    for (int cpu = 0; cpu < ACC_MAX_CPUS; cpu++) {
      if (!(rp->cpus[cpu >> 6] >> (cpu & 63) & 1)) continue;
      x->al.present[cpu] = 1;
      x->al.ref[cpu]++;
      x->al.excl[cpu] = rp->excl;
      int f = 0;
      for (int k = 0; k < nu && !f; k++) f = used[k] == x->t.node[cpu];
      if (!f) used[nu++] = x->t.node[cpu];
    }
    for (int k = 0; k < nu; k++) /* the pod joins sharedNode[id] (several NUMA ids) or singleNUMANode[id] */
      for (int z = 0; z < n->n_zone; z++)
        if (n->zone[z].id == used[k]) {
          if (nu > 1) n->zone[z].shared_pods++;
          else n->zone[z].single_pods++;
          n->zone[z].numa_status = zone_status_of(&n->zone[z]);
        }
  }
  for (int z = 0; z < n->n_zone; z++) {
    if (rp->dist[z][0] == 0 && rp->dist[z][1] == 0) continue;
    ke_numa_zone* zn = &n->zone[z];
    for (int r = 0; r < KE_NRES; r++) {
      const uint8_t key = r == KE_RES_CPU ? KE_NUMA_ALLOC_CPU : KE_NUMA_ALLOC_MEMORY;
      if (!(zn->has_allocated & key)) zn->allocated[r] = 0;
      if (rp->dist[z][r] != 0) zn->has_allocated |= key;
      zn->allocated[r] += rp->dist[z][r];
    }
    zn->has_allocated |= KE_NUMA_ALLOC_ENTRY;
  }
}

/* Golden-vector entry point: resourceManager.Allocate for `pod` on `node` with the hint `mask` (0 =
 * nil NUMANodeAffinity), resource_manager.go:194-225.  0 and out16[2*id + r] / cpus, or -1. */
int or_numa_allocate(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t mask, int64_t* out16,
                     uint64_t* cpus) {
  const or_node* nd = &c->nodes[node];
  numa_cs cs;
  numa_cs_build(c, nd, pod, &cs);
  numa_view v;
  int64_t dist[KE_MAX_NUMA][KE_NRES];
  memset(dist, 0, sizeof dist);
  memset(cpus, 0, sizeof(uint64_t) * ACC_WORDS);
  for (int i = 0; i < 2 * KE_MAX_NUMA; i++) out16[i] = 0;
  if (numa_view_build(nd, &v, &cs) != 0) return -1;
  if (mask && !numa_distribute(&v, mask, pod, dist, &cs)) return -1;
  if (cs.rcb && (!cs.valid || cpuset_allocate_cs(nd, &cs, &v, mask ? (const int64_t(*)[KE_NRES])dist : NULL, cpus) != 0))
    return -1;
  for (int z = 0; z < v.n; z++)
    for (int r = 0; r < KE_NRES; r++) out16[2 * v.id[z] + r] = dist[z][r];
  return 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* NodeResourcesFitPlus / ScarceResourceAvoidance                            */
/* ---------------------------------------------------------------------------------------------- */

int or_node_resources_set(or_cluster* c, int32_t node, int32_t n, const ke_node_resource* res) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  if (n < 0 || n > KE_MAX_XRES) return KE_ERR_INVALID;
  c->nodes[node].n_xres = n;
  if (n) memcpy(c->nodes[node].xres, res, sizeof(ke_node_resource) * (size_t)n);
  return KE_OK;
}

static const ke_node_resource* node_xres(const or_node* nd, int32_t id) {
  for (int32_t e = 0; e < nd->n_xres; e++)
    if (nd->xres[e].id == id) return &nd->xres[e];
  return NULL;
}

/* calculatePodResourceRequest (node_resource_fit_plus_utils.go:138-165) as the caller computed it */
static int64_t pod_xres(const ke_pod* pod, int32_t id) {
  for (int32_t e = 0; e < pod->n_xres; e++)
    if (pod->xres_id[e] == id) return pod->xres_value[e];
  return 0;
}

/* Go int64 multiply (wraps) */
static int64_t mul_wrap(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

/* mostRequestedScore / leastRequestedScore (node_resource_fit_plus_utils.go:35-55) */
static int64_t fp_most(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) requested = capacity;
  return mul_wrap(requested, MAX_NODE_SCORE) / capacity;
}
static int64_t fp_least(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return mul_wrap(capacity - requested, MAX_NODE_SCORE) / capacity;
}

/* NodeResourcesFitPlus Score (node_resources_fit_plus.go:75-93 -> getResourceScore -> resourceScorer,
 * node_resource_fit_plus_utils.go:57-103): for every resource name the pod requests (PodRequests > 0,
 * fitsPodRequestName) that the args list, calculateResourceAllocatableRequest gives allocatable and
 * NodeInfo (NonZero)Requested + the pod's request; score = Σ score·weight / Σ weight (MaxNodeScore for a
 * zero weight sum).  The map's iteration order does not matter: integer sums. */
int64_t or_fitplus_score(const or_cluster* c, const ke_pod* pod, int32_t node) {
  const or_node* nd = &c->nodes[node];
  const ke_ext_args* x = &c->cfg.ext;
  int64_t node_score = 0, weight_sum = 0;
  for (int32_t id = 0; id < KE_MAX_XRES; id++) {
    if (!((pod->xres_request_mask >> id) & 1)) continue;
    const ke_fitplus_resource* ra = NULL;
    for (int q = 0; q < x->n_fitplus; q++)
      if (x->fitplus[q].id == id) ra = &x->fitplus[q];
    if (!ra) continue;
    const ke_node_resource* r = node_xres(nd, id);
    const int64_t alloc = r ? r->allocatable : 0;
    /* NonZeroRequested of cpu / memory after the reservation restore */
    const int64_t rv = r && (id == KE_RES_CPU || id == KE_RES_MEMORY) ? nd->rv_nz[id] : (r ? nd->rv_x[id] : 0);
    const int64_t req = (r ? r->requested + rv : 0) + pod_xres(pod, id);
    const int64_t rs = ra->type == KE_STRATEGY_MOST_ALLOCATED ? fp_most(req, alloc) : fp_least(req, alloc);
    node_score += rs * ra->weight;
    weight_sum += ra->weight;
  }
  if (weight_sum == 0) return MAX_NODE_SCORE;
  return node_score / weight_sum;
}

/* NodeResourcesFit (upstream kube-scheduler v1.28.7, pkg/scheduler/framework/plugins/noderesources; not in the
 * reference tree, go.mod:60): PARITY UNPINNED -- restated from the published algorithm, no reference test vector.
 * Filter (fit.go fitsRequest): len(NodeInfo.Pods) + 1 > AllowedPodNumber ("Too many pods"); a pod requesting
 * nothing passes; cpu / memory requests > 0 above Allocatable - Requested; scalar requests > 0 above the scalar's
 * Allocatable - Requested (the first insufficiency in that order; the scalars in args order).  Returns the reason,
 * 0 = fits. */
static int or_fit_filter(const or_cluster* c, const ke_pod* pod, int32_t node) {
  const or_node* nd = &c->nodes[node];
  if ((int64_t)nd->node.pod_count + nd->rv_pods + 1 > nd->node.allowed_pods) return KE_REASON_FIT_TOO_MANY_PODS;
  for (int r = 0; r < KE_NRES; r++) {
    const int64_t q = pod->requests[r];
    if (q > 0 && q > nd->node.allocatable[r] - (nd->node.requested[r] + nd->rv_req[r]))
      return r == KE_RES_CPU ? KE_REASON_FIT_INSUFFICIENT_CPU : KE_REASON_FIT_INSUFFICIENT_MEMORY;
  }
  for (int q = 0; q < c->cfg.fit.n_scalars; q++) {
    const int32_t id = c->cfg.fit.scalars[q];
    const int64_t v = pod_xres(pod, id);
    const ke_node_resource* r = node_xres(nd, id);
    if (v > 0 && v > (r ? r->allocatable : 0) - (r ? r->requested + nd->rv_x[id] : 0)) return KE_REASON_FIT_INSUFFICIENT_SCALAR;
  }
  return 0;
}

/* NodeResourcesFit Score (resource_allocation.go score + calculateResourceAllocatableRequest, least_allocated.go /
 * most_allocated.go): per configured resource, cpu / memory: (Allocatable, NonZeroRequested + the pod's request
 * with the container defaults); a scalar the pod does not request: skipped; else (Allocatable, Requested +
 * request); alloc 0: skipped; Σ weight·score / Σ weight, 0 for a zero weight sum. */
static int64_t or_fit_score(const or_cluster* c, const ke_pod* pod, int32_t node) {
  const or_node* nd = &c->nodes[node];
  const ke_fit_args* a = &c->cfg.fit;
  int64_t node_score = 0, weight_sum = 0;
  for (int q = 0; q < a->n_resources; q++) {
    const int32_t id = a->resources[q].id;
    const int64_t preq = pod_xres(pod, id);
    if (id >= 2 && preq == 0) continue;
    const ke_node_resource* r = node_xres(nd, id);
    const int64_t alloc = r ? r->allocatable : 0;
    if (alloc == 0) continue;
    const int64_t rv = id == KE_RES_CPU || id == KE_RES_MEMORY ? nd->rv_nz[id] : nd->rv_x[id];
    const int64_t req = r->requested + rv + preq;
    const int64_t rs = a->strategy == KE_STRATEGY_MOST_ALLOCATED ? fp_most(req, alloc) : fp_least(req, alloc);
    node_score += rs * a->resources[q].weight;
    weight_sum += a->resources[q].weight;
  }
  return weight_sum == 0 ? 0 : node_score / weight_sum;
}

/* ScarceResourceAvoidance Score (scarce_resource_avoidance.go:70-90): the node's allocatable names (> 0)
 * minus the pod's requested names (quotav1.Difference), intersected with args.Resources; resourceTypesScore
 * (:159-161). */
int64_t or_sra_score(const or_cluster* c, const ke_pod* pod, int32_t node) {
  const or_node* nd = &c->nodes[node];
  int64_t n_diff = 0, n_inter = 0;
  for (int32_t e = 0; e < nd->n_xres; e++) {
    const int32_t id = nd->xres[e].id;
    if (nd->xres[e].allocatable <= 0 || ((pod->xres_request_mask >> id) & 1)) continue;
    n_diff++;
    if ((c->cfg.ext.sra_resources >> id) & 1) n_inter++;
  }
  if (n_diff == 0 || n_inter == 0) return MAX_NODE_SCORE;
  return (n_diff - n_inter) * MAX_NODE_SCORE / n_diff;
}

int or_node_numa_set(or_cluster* c, int32_t node, int32_t n, const ke_numa_zone* zones) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  if (n < 0 || n > KE_MAX_NUMA) return KE_ERR_INVALID;
  for (int32_t i = 0; i < n; i++) { /* same validation as the product (ke_node_numa_set) */
    if (zones[i].id < 0 || zones[i].id >= KE_MAX_NUMA || (i > 0 && zones[i].id <= zones[i - 1].id)) return KE_ERR_INVALID;
    if (zones[i].capacity[0] < 0 || zones[i].capacity[1] < 0 || zones[i].cpuset_cpus < 0) return KE_ERR_INVALID;
    if (zones[i].cpuset_cpus > 0 && !(zones[i].has_allocated & KE_NUMA_ALLOC_ENTRY)) return KE_ERR_INVALID;
    if (zones[i].has_allocated > 7 || (zones[i].has_allocated && !(zones[i].has_allocated & KE_NUMA_ALLOC_ENTRY)))
      return KE_ERR_INVALID;
    if (zones[i].numa_status > KE_NUMA_STATUS_SHARED || zones[i].single_pods < 0 || zones[i].shared_pods < 0)
      return KE_ERR_INVALID;
    if ((zones[i].single_pods || zones[i].shared_pods) && zones[i].numa_status != zone_status_of(&zones[i]))
      return KE_ERR_INVALID;
  }
  c->nodes[node].n_zone = n;
  if (n) memcpy(c->nodes[node].zone, zones, sizeof(ke_numa_zone) * (size_t)n);
  for (int32_t i = 0; i < n; i++) { /* a status without counts: one pod in that set */
    ke_numa_zone* z = &c->nodes[node].zone[i];
    if (!z->single_pods && !z->shared_pods) {
      if (z->numa_status == KE_NUMA_STATUS_SINGLE) z->single_pods = 1;
      if (z->numa_status == KE_NUMA_STATUS_SHARED) z->shared_pods = 1;
    }
  }
  or_node* nd = &c->nodes[node];
  int bare = 1; /* an NRT without the resource manager's allocation: the parked zones' allocation comes back */
  for (int32_t i = 0; i < n; i++)
    bare = bare && !nd->zone[i].has_allocated && !nd->zone[i].single_pods && !nd->zone[i].shared_pods &&
           !nd->zone[i].cpuset_cpus;
  if (bare)
    for (int32_t i = 0; i < n; i++)
      for (int32_t k = 0; k < nd->n_kept_zone; k++)
        if (nd->kept_zone[k].id == nd->zone[i].id) {
          ke_numa_zone* z = &nd->zone[i];
          const ke_numa_zone* kz = &nd->kept_zone[k];
          z->has_allocated = kz->has_allocated;
          for (int r = 0; r < KE_NRES; r++) z->allocated[r] = kz->allocated[r];
          z->cpuset_cpus = kz->cpuset_cpus;
          z->single_pods = kz->single_pods;
          z->shared_pods = kz->shared_pods;
          z->numa_status = zone_status_of(z);
        }
  if (n > 0) nd->n_kept_zone = 0;
  return KE_OK;
}

int or_node_devices_set(or_cluster* c, int32_t node, int32_t n, const ke_device* devs) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  if (n < 0 || n > KE_DEV_TYPES * KE_MAX_MINORS) return KE_ERR_INVALID;
  or_node* nd = &c->nodes[node];
  nd->has_dev_cache = 1;
  nd->n_dev = n;
  if (n) memcpy(nd->dev, devs, sizeof(ke_device) * (size_t)n);
  return KE_OK;
}

int or_node_devices_delete(or_cluster* c, int32_t node) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  c->nodes[node].has_dev_cache = 0;
  c->nodes[node].n_dev = 0;
  c->nodes[node].gpu_has_table = c->nodes[node].gpu_honor = 0;
  c->nodes[node].n_part = 0;
  return KE_OK;
}

int or_node_gpu_partitions(or_cluster* c, int32_t node, int32_t has_table, int32_t honor, int32_t n,
                           const ke_gpu_partition* parts) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  if (n < 0 || n > KE_MAX_GPU_PARTITIONS || (n > 0 && !has_table)) return KE_ERR_INVALID;
  or_node* nd = &c->nodes[node];
  nd->gpu_has_table = has_table != 0;
  nd->gpu_honor = honor != 0;
  nd->n_part = n;
  if (n) memcpy(nd->part, parts, sizeof(ke_gpu_partition) * (size_t)n);
  return KE_OK;
}

int or_node_upsert(or_cluster* c, int32_t node, const ke_node* n) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  c->nodes[node].node = *n;
  c->nodes[node].deleted = 0;
  return KE_OK;
}

/* Node informer delete: the scheduler cache's RemoveNode leaves the NodeInfo out of the snapshot (k8s v1.28.7);
 * NodeMetric, podAssignCache, resource manager, device cache and reservation cache keep their entries */
int or_node_delete(or_cluster* c, int32_t node) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  c->nodes[node].deleted = 1;
  return KE_OK;
}

/* NodeResourceTopology delete (topology_eventhandler.go:82-99): TopologyOptions gone -- no NUMA node resources,
 * no CPU topology (GetAvailableCPUs: nothing allocated), no NRT amplification ratios */
int or_node_topology_delete(or_cluster* c, int32_t node) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  or_node* nd = &c->nodes[node];
  if (nd->n_zone) {
    nd->n_kept_zone = nd->n_zone;
    memcpy(nd->kept_zone, nd->zone, sizeof(ke_numa_zone) * (size_t)nd->n_zone);
  }
  nd->n_zone = 0;
  if (nd->cpus) {
    free(nd->kept_cpus);
    nd->kept_cpus = nd->cpus;
  }
  nd->cpus = NULL;
  nd->node.cpuset_allocated_cpus = 0;
  nd->node.nrt_cpu_amplification_ratio = -2;
  nd->node.cpu_topology_invalid = 0;
  return KE_OK;
}

int or_node_set_requested(or_cluster* c, int32_t node, int64_t milli_cpu, int64_t memory) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  c->nodes[node].node.requested[KE_RES_CPU] = milli_cpu;
  c->nodes[node].node.requested[KE_RES_MEMORY] = memory;
  return KE_OK;
}

int or_node_set_cpuset_allocated(or_cluster* c, int32_t node, int64_t cpus) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  c->nodes[node].node.cpuset_allocated_cpus = cpus;
  return KE_OK;
}

int or_nodemetric_upsert(or_cluster* c, int32_t node, const ke_node_metric* nm, int32_t n_pm,
                         const ke_pod_metric* pm, int32_t n_agg, const ke_aggregated_usage* agg) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  or_node* n = &c->nodes[node];
  free(n->pm);
  free(n->agg);
  n->has_metric = 1;
  n->nm = *nm;
  n->n_pm = n_pm;
  n->pm = n_pm ? (ke_pod_metric*)malloc(sizeof(ke_pod_metric) * (size_t)n_pm) : NULL;
  if (n_pm) memcpy(n->pm, pm, sizeof(ke_pod_metric) * (size_t)n_pm);
  n->n_agg = n_agg;
  n->agg = n_agg ? (ke_aggregated_usage*)malloc(sizeof(ke_aggregated_usage) * (size_t)n_agg) : NULL;
  if (n_agg) memcpy(n->agg, agg, sizeof(ke_aggregated_usage) * (size_t)n_agg);
  return KE_OK;
}

int or_nodemetric_delete(or_cluster* c, int32_t node) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  or_node* n = &c->nodes[node];
  free(n->pm);
  free(n->agg);
  n->pm = NULL;
  n->agg = NULL;
  n->n_pm = n->n_agg = 0;
  n->has_metric = 0;
  return KE_OK;
}

/* podAssignCache.assign  pod_assign_cache.go:89-124 */
int or_pod_assign(or_cluster* c, int32_t node, const ke_pod* pod, int64_t timestamp_ns) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  if (pod->is_terminated) return KE_OK;
  or_node* n = &c->nodes[node];
  int64_t est[KE_NRES];
  uint8_t present[KE_NRES];
  estimate_pod(&c->cfg.loadaware, pod, est, present);
  int has_est = 0;
  for (int r = 0; r < KE_NRES; r++) has_est |= present[r];
  for (int i = 0; i < n->n_asg; i++) {
    if (n->asg[i].pod.uid == pod->uid) { /* existing: keep timestamp, refresh pod + estimate */
      n->asg[i].pod = *pod;
      memcpy(n->asg[i].est, est, sizeof est);
      memcpy(n->asg[i].est_present, present, sizeof present);
      n->asg[i].has_est = has_est;
      return KE_OK;
    }
  }
  if (n->n_asg == n->cap_asg) {
    n->cap_asg = n->cap_asg ? 2 * n->cap_asg : 8;
    n->asg = (or_asg*)realloc(n->asg, sizeof(or_asg) * (size_t)n->cap_asg);
  }
  or_asg* a = &n->asg[n->n_asg++];
  a->pod = *pod;
  a->ts = pod->has_scheduled ? pod->scheduled_transition_ns : timestamp_ns;
  memcpy(a->est, est, sizeof est);
  memcpy(a->est_present, present, sizeof present);
  a->has_est = has_est;
  return KE_OK;
}

int or_pods_assign(or_cluster* c, int32_t n, const int32_t* nodes, const ke_pod* pods, const int64_t* ts) {
  for (int32_t i = 0; i < n; i++) {
    int rc = or_pod_assign(c, nodes[i], &pods[i], ts[i]);
    if (rc) return rc;
  }
  return KE_OK;
}

/* podAssignCache.unAssign  pod_assign_cache.go:126-136 */
int or_pod_unassign(or_cluster* c, int32_t node, int64_t uid) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  or_node* n = &c->nodes[node];
  for (int i = 0; i < n->n_asg; i++) {
    if (n->asg[i].pod.uid == uid) {
      n->asg[i] = n->asg[n->n_asg - 1];
      n->n_asg--;
      return KE_OK;
    }
  }
  return KE_OK;
}

/* ---------------------------------------------------------------------------------------------- */
/* framework                                                                                       */
/* ---------------------------------------------------------------------------------------------- */

typedef struct eval_out {
  uint8_t status, reason;
  int16_t la, numa, ds, total; /* ds: DeviceShare.Score before NormalizeScore */
  int16_t fp, sra, fit;         /* NodeResourcesFitPlus, ScarceResourceAvoidance, NodeResourcesFit */
} eval_out;

/* RunFilterPlugins in profile order LoadAware, NodeNUMAResource, DeviceShare
 * (scheduler-config.yaml:68-73), then the raw Score of each plugin for a feasible node. */
static void eval_pair(const or_cluster* c, const ke_pod* pod, int32_t node, int64_t now, eval_out* o) {
  int reason = 0;
  int code = KE_CODE_SUCCESS;
  if (c->nodes[node].deleted) { /* not in the snapshot: evaluated nowhere (KE_CODE_ERROR, as the product) */
    o->status = KE_CODE_ERROR;
    o->reason = 0;
    o->la = o->numa = o->ds = o->fp = o->sra = o->fit = 0;
    o->total = -1;
    return;
  }
  /* PreFilter failures fail the pod on every node before any Filter runs (profile order
   * NodeNUMAResource, DeviceShare): a cpuset pod with a non-integer cpu request, invalid device requests */
  cpuset_state st;
  cpuset_prefilter(c, pod, &st);
  ds_pod d;
  ds_prepare_pod(c, pod, &d);
  if (!pod_requests_zero(pod) && st.invalid) {
    code = KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    reason = KE_REASON_NUMA_INVALID_REQUESTED_CPUS;
  } else if (d.status) {
    code = d.status;
    reason = d.status_reason ? d.status_reason : KE_REASON_DS_INVALID_REQUEST;
  }
  /* NodeResourcesFit's Filter: a default plugin, ahead of the profile's own Filters */
  if (code == KE_CODE_SUCCESS && c->cfg.fit.filter && (reason = or_fit_filter(c, pod, node)) != 0)
    code = KE_CODE_UNSCHEDULABLE;
  if (code == KE_CODE_SUCCESS) code = or_la_filter(c, pod, node, now, &reason);
  if (code == KE_CODE_SUCCESS) code = or_numa_filter(c, pod, node, &reason);
  if (code == KE_CODE_SUCCESS) code = or_ds_filter(c, pod, node, &reason);
  o->status = (uint8_t)code;
  o->reason = (uint8_t)reason;
  o->la = o->numa = o->ds = o->fp = o->sra = o->fit = 0;
  o->total = -1;
  if (code != KE_CODE_SUCCESS) return;
  if (c->cfg.fit.weight) o->fit = (int16_t)or_fit_score(c, pod, node);
  if (c->cfg.ext.weight_fitplus) o->fp = (int16_t)or_fitplus_score(c, pod, node);
  if (c->cfg.ext.weight_sra) o->sra = (int16_t)or_sra_score(c, pod, node);
  o->la = (int16_t)or_la_score(c, pod, node, now);
  o->numa = (int16_t)or_numa_score(c, pod, node);
  o->ds = (int16_t)or_ds_score(c, pod, node);
}

/* DeviceShare NormalizeScore = DefaultNormalizeScore(MaxNodeScore, false) over the feasible nodes
 * (scoring.go:109-111; k8s pkg/scheduler/framework/plugins/helper/normalize_score.go), then the
 * weighted sum (scheduler-config.yaml:85-94). */
static void normalize_and_total(const or_cluster* c, eval_out* o, int64_t n) {
  int64_t mx = 0;
  for (int64_t i = 0; i < n; i++)
    if (o[i].status == KE_CODE_SUCCESS && o[i].ds > mx) mx = o[i].ds;
  for (int64_t i = 0; i < n; i++) {
    if (o[i].status != KE_CODE_SUCCESS) continue;
    const int64_t ds = mx > 0 ? MAX_NODE_SCORE * o[i].ds / mx : o[i].ds;
    o[i].total = (int16_t)(c->cfg.weight_loadaware * o[i].la + c->cfg.weight_numa * o[i].numa +
                           c->cfg.weight_deviceshare * ds + c->cfg.ext.weight_fitplus * o[i].fp +
                           c->cfg.ext.weight_sra * o[i].sra + c->cfg.fit.weight * o[i].fit);
  }
}

/* DefaultNormalizeScore(MaxNodeScore, reverse=false) on a score list (golden-vector entry point) */
void or_normalize_scores(int64_t* scores, int32_t n) {
  int64_t mx = 0;
  for (int32_t i = 0; i < n; i++)
    if (scores[i] > mx) mx = scores[i];
  if (mx == 0) return;
  for (int32_t i = 0; i < n; i++) scores[i] = MAX_NODE_SCORE * scores[i] / mx;
}

static int check_supported(const or_cluster* c, int32_t n_pods, const ke_pod* pods) {
  int ds = 0, numa = 0, cpuset = 0, node_bind = 0;
  for (int i = 0; i < c->n; i++) node_bind |= c->nodes[i].node.cpu_bind_policy != KE_NODE_CPU_BIND_NONE;
  for (int p = 0; p < n_pods; p++) {
    cpuset_state st;
    cpuset_prefilter(c, &pods[p], &st);
    if (st.rcb || (node_bind && pods[p].requests[KE_RES_CPU] > 0)) {
      cpuset = 1;
      if (pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE) numa = 1;
    }
    if (pod_unsupported(&pods[p])) return KE_ERR_UNSUPPORTED;
    if (pods[p].numa_topology_policy < 0 || pods[p].numa_topology_policy > KE_NUMA_POLICY_SINGLE_NUMA_NODE ||
        pods[p].numa_exclusive < 0 || pods[p].numa_exclusive > KE_NUMA_EXCLUSIVE_REQUIRED)
      return KE_ERR_INVALID;
    ds_pod d;
    ds_prepare_pod(c, &pods[p], &d);
    if (!d.skip && d.status == KE_CODE_SUCCESS) {
      ds = 1;
      if (pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE) numa = 1;
    }
  }
  for (int i = 0; i < c->n; i++) {
    if (node_unsupported(&c->nodes[i].node)) return KE_ERR_UNSUPPORTED;
    if (c->nodes[i].node.numa_topology_policy != KE_NUMA_POLICY_NONE) numa = 1;
  }
  (void)cpuset;
  (void)ds;
  (void)numa;
  return KE_OK;
}

/* One pod against every node: filter + raw scores (parallel over nodes), normalize, selectHost
 * (ties -> lowest node index).  Returns the chosen node or -1. */
static int32_t eval_pod(const or_cluster* c, const ke_pod* pod, int64_t now, eval_out* o, int16_t* best_score) {
  const int64_t N = c->n;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; i++) eval_pair(c, pod, (int32_t)i, now, &o[i]);
  normalize_and_total(c, o, N);
  int32_t b = -1;
  int16_t bs = -1;
  for (int64_t i = 0; i < N; i++)
    if (o[i].total > bs) {
      bs = o[i].total;
      b = (int32_t)i;
    }
  *best_score = bs;
  return bs >= 0 ? b : -1;
}

int or_eval(const or_cluster* c, int32_t n_pods, const ke_pod* pods, int64_t now, uint8_t* status, uint8_t* reason,
            int16_t* la_score, int16_t* numa_score, int16_t* ds_score, int16_t* total, int32_t* best, int n_threads) {
  int rc = check_supported(c, n_pods, pods);
  if (rc) return rc;
  for (int32_t p = 0; p < n_pods; p++)
    if (pods[p].reservation_matched) return KE_ERR_UNSUPPORTED;
  const int64_t N = c->n;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#else
  (void)n_threads;
#endif
  eval_out* o = (eval_out*)malloc(sizeof(eval_out) * (size_t)(N > 0 ? N : 1));
  for (int p = 0; p < n_pods; p++) {
    int16_t bs;
    const int32_t b = eval_pod(c, &pods[p], now, o, &bs);
    for (int64_t i = 0; i < N; i++) {
      const int64_t k = (int64_t)p * N + i;
      if (status) status[k] = o[i].status;
      if (reason) reason[k] = o[i].reason;
      if (la_score) la_score[k] = o[i].la;
      if (numa_score) numa_score[k] = o[i].numa;
      if (ds_score) ds_score[k] = o[i].ds;
      if (total) total[k] = o[i].total;
    }
    if (best) best[p] = b;
  }
  free(o);
  return KE_OK;
}

/* The Reservation plugin's PreScore + Score for a pod whose matched reservations are flagged in m[]
 * (reservation/scoring.go:42-128, nominator.go:207-278): per node the matched reservations in index order, their
 * smallest order, the nominated one (NominateReservation: the FilterNominateReservation survivors; the only one,
 * else the smallest order, else the best ScoreReservation) and its ScoreReservation; preferredNode = the node
 * of `nodes` (feasible[i] != 0, NULL = every node) with the smallest order (first in node order) scores 1000.
 * pod_requested[i*KE_NRES + k]: NodeInfo Requested after the unmatched restore.  raw[i] = Score (before
 * NormalizeScore), nom[i] = the nominated reservation or -1.  Returns preferredNode or -1. */
/* NodeNUMAResource's FilterNominateReservation (plugin.go:448-504): a pod that binds no CPUs on a node without a
 * NUMA policy passes, a binding pod needs a valid CPU topology, a reservation outside RestoreReservation's matched
 * set passes, else tryAllocateFromReservation over it alone -- which fails only under a reservation affinity. */
static int or_numa_nominable(const or_cluster* c, const ke_pod* pod, int32_t node, int32_t r, int affinity) {
  const or_node* n = &c->nodes[node];
  if (pod_requests_zero(pod)) return 1;
  cpuset_state st;
  cpuset_prefilter(c, pod, &st);
  int exclusive;
  const int policy = effective_policy(n, pod, &exclusive);
  const int rcb = request_cpu_bind(&st, pod, n->node.cpu_bind_policy);
  if (rcb < 0) return 0;
  if (!rcb && policy <= KE_NUMA_POLICY_NONE) return 1;
  if (rcb && !cpus_valid(n)) return 0;
  if (policy != KE_NUMA_POLICY_NONE) return !c->numa_rok || c->numa_rok[r] != 0; /* (or_resv_eval's precomputation) */
  uint64_t got[ACC_WORDS];
  return or_numa_from_rsv(c, pod, node, r, affinity, got) >= 0;
}

/* golden entry point: NodeNUMAResource Reserve's allocation from reservation `nom` for a binding pod matching
 * reservations ids[] on `node` (allocateWithNominatedReservation -> tryAllocateFromReservation): 1 and the cpuset,
 * 0 (nil: the node itself), -1 (Unschedulable under a reservation affinity). */
int or_numa_reserve_from_rsv(or_cluster* c, const ke_pod* pod, int32_t node, const int32_t* ids, int32_t n_ids,
                             int32_t nom, int32_t required, uint64_t* cpus) {
  char* m = (char*)calloc((size_t)(c->n_resv > 0 ? c->n_resv : 1), 1);
  for (int32_t j = 0; j < n_ids; j++)
    if (or_resv_usable(&c->resv[ids[j]])) m[ids[j]] = 1;
  c->resv_m = m;
  memset(cpus, 0, sizeof(uint64_t) * ACC_WORDS);
  const int r = or_numa_from_rsv(c, pod, node, nom, required, cpus);
  c->resv_m = NULL;
  free(m);
  return r;
}

/* golden entry point: NodeNUMAResource Reserve under a NUMA policy for a pod matching reservations ids[] on `node`
 * with the stored affinity `aff` (0 = nil) and the nominated reservation `nom` (allocateWithNominatedReservation ->
 * tryAllocateFromReservation, then tryAllocateFromNode; plugin.go:552-566): 1 = from the reservation, 0 = from the
 * node, -1 = Unschedulable; dist16[2*id + r] the NUMA allocation, cpus the cpuset. */
int or_numa_reserve_policy(or_cluster* c, const ke_pod* pod, int32_t node, const int32_t* ids, int32_t n_ids,
                           int32_t nom, int32_t required, uint32_t aff, int64_t* dist16, uint64_t* cpus) {
  char* m = (char*)calloc((size_t)(c->n_resv > 0 ? c->n_resv : 1), 1);
  for (int32_t j = 0; j < n_ids; j++)
    if (or_resv_usable(&c->resv[ids[j]])) m[ids[j]] = 1;
  c->resv_m = m;
  int32_t M[64];
  const int nM = numa_rsv_matched(c, node, M);
  int in = 0;
  for (int q = 0; q < nM; q++) in |= M[q] == nom;
  int rc = in ? numa_from_rsv_try(c, pod, node, M, nM, &nom, 1, aff, required, NULL, dist16, cpus) : 0;
  if (rc == 0) rc = numa_alloc_try(c, &c->nodes[node], pod, aff, NULL, dist16, cpus) ? 0 : -1;
  c->resv_m = NULL;
  free(m);
  return rc;
}

/* golden entry point: NodeNUMAResource Reserve of a reservation-ignored pod on a node without a NUMA policy
 * (tryAllocateIgnoreReservation, reservation.go:437-490): 1 and the cpuset, 0 (no holding reservation: the node), -1 */
int or_numa_reserve_ignored(or_cluster* c, const ke_pod* pod, int32_t node, uint64_t* cpus) {
  memset(cpus, 0, sizeof(uint64_t) * ACC_WORDS);
  return or_numa_ignored(c, pod, node, cpus);
}

/* allRAllocated of node i: Σ allocated of its matched reservations, [cpu, memory, then KE_NRES + resource id] */
#define PRW (KE_NRES + KE_MAX_XRES)
static void or_all_allocated(const or_cluster* c, const char* m, int32_t i, int64_t* all) {
  memset(all, 0, sizeof(int64_t) * PRW);
  for (int32_t r = 0; r < c->n_resv; r++) {
    if (!m[r] || c->resv[r].node != i) continue;
    for (int k = 0; k < KE_NRES; k++) all[k] += c->resv[r].allocated[k];
    for (int32_t e = c->rres ? c->roff[r] : 0; c->rres && e < c->roff[r + 1]; e++)
      if (c->rres[e].id != KE_RSV_RES_PODS) all[KE_NRES + c->rres[e].id] += c->rres[e].allocated;
  }
}
static int32_t or_resv_prescore(const or_cluster* c, const ke_pod* pod, const char* m, const int64_t* pod_requested,
                                const uint8_t* feasible, int affinity, int64_t* raw, int32_t* nom) {
  const int32_t N = c->n;
  int32_t pref = -1;
  int64_t po = 0;
  char* has = (char*)calloc((size_t)(N > 0 ? N : 1), 1); /* nodes holding a matched reservation */
  for (int32_t r = 0; r < c->n_resv; r++)
    if (m[r]) has[c->resv[r].node] = 1;
  for (int32_t i = 0; i < N; i++) {
    nom[i] = -1;
    raw[i] = 0;
    if (!has[i]) continue;
    int64_t all_alloc[PRW], order = 0;
    int any = 0;
    or_all_allocated(c, m, i, all_alloc);
    for (int32_t r = 0; r < c->n_resv; r++)
      if (m[r] && c->resv[r].node == i) {
        any = 1;
        if (c->resv[r].order != 0 && (order == 0 || c->resv[r].order < order)) order = c->resv[r].order;
      }
    if (!any) continue;
    /* DeviceShare's part of the nomination for a DeviceShare pod (FilterNominateReservation, plugin.go:371-426;
     * ScoreReservation, scoring.go:113-153): over the node's matched reservations holding devices */
    ds_pod d;
    ds_prepare_pod(c, pod, &d);
    static __thread ds_rstate rs;
    const int ds_on = c->nodes[i].has_dev_cache && ds_pod_rstate(c, pod, &d, i, &rs);
    int32_t n_ok = 0, first = -1, by_order = -1, n_matched = 0, only = -1;
    int32_t okr[DS_MAX_MATCHED * 4];
    int64_t ok_rs[DS_MAX_MATCHED * 4], ok_ds[DS_MAX_MATCHED * 4];
    int64_t bo = 0;
    for (int32_t r = 0; r < c->n_resv; r++) {
      if (!m[r] || c->resv[r].node != i) continue;
      n_matched++;
      only = r;
      if (!or_resv_nominable(c, r, pod, i, &pod_requested[i * PRW], all_alloc, affinity) ||
          !or_numa_nominable(c, pod, i, r, affinity))
        continue;
      const int di = ds_on ? ds_rsv_find(&rs, r) : -1;
      if (di >= 0) { /* tryAllocateFromReservation over it alone, required */
        uint32_t out[KE_DEV_TYPES];
        int8_t vf[2][KE_MAX_MINORS];
        int why = 0;
        if (ds_from_rsv(c, &c->nodes[i], &d, &rs, di, 1, 0, NULL, 0, out, vf, &why) != 1) continue;
      }
      if (n_ok < DS_MAX_MATCHED * 4) {
        okr[n_ok] = r;
        ok_rs[n_ok] = or_reservation_score_idx(c, r, pod);
        ok_ds[n_ok] = di >= 0 ? ds_rsv_score(c, &c->nodes[i], &d, &rs, di) : 0;
      }
      n_ok++;
      if (first < 0) first = r;
      if (c->resv[r].order != 0 && (bo == 0 || c->resv[r].order < bo)) {
        bo = c->resv[r].order;
        by_order = r;
      }
    }
    /* prioritizeReservations (nominator.go:315-360): Σ of the plugins' ScoreReservation -- the Reservation plugin's
     * raw, DeviceShare's normalized (DefaultReservationNormalizeScore over the list, normalize_score.go:24-52) --
     * sort.Slice by score desc (equal scores keep list order: insertion sort below 13 elements) */
    int32_t by_score = -1;
    {
      int64_t mx = 0, bsc = -1;
      const int32_t n = n_ok < DS_MAX_MATCHED * 4 ? n_ok : DS_MAX_MATCHED * 4;
      for (int32_t q = 0; q < n; q++) mx = ok_ds[q] > mx ? ok_ds[q] : mx;
      for (int32_t q = 0; q < n; q++) {
        const int64_t sc = ok_rs[q] + (mx > 0 ? 100 * ok_ds[q] / mx : ok_ds[q]);
        if (sc > bsc) {
          bsc = sc;
          by_score = okr[q];
        }
      }
    }
    nom[i] = n_ok == 0 ? -1 : n_ok == 1 ? first : by_order >= 0 ? by_order : by_score;
    if (affinity && n_matched == 1) nom[i] = only; /* nominator.go:223-225 */
    raw[i] = nom[i] >= 0 ? or_reservation_score_idx(c, nom[i], pod) : 0;
    if ((!feasible || feasible[i]) && order != 0 && (pref < 0 || order < po)) {
      po = order;
      pref = i;
    }
  }
  if (pref >= 0) raw[pref] = 1000; /* mostPreferredScore */
  free(has);
  return pref;
}

/* The Reservation Filter of a pod with a reservation affinity on node i (plugin.go:316-318, 351-442): a node
 * without matched reservations fails, one with them passes when one fits (fitsNode, and fitsReservation for
 * Restricted; resource names are not required to overlap with an affinity) */
static int or_resv_filter_node(const or_cluster* c, const ke_pod* pod, const char* m, const int64_t* pod_requested,
                               int32_t i) {
  int64_t all_alloc[PRW];
  or_all_allocated(c, m, i, all_alloc);
  for (int32_t r = 0; r < c->n_resv; r++)
    if (m[r] && c->resv[r].node == i && or_resv_nominable(c, r, pod, i, &pod_requested[i * PRW], all_alloc, 1))
      return 1;
  return 0;
}

/* matched flags + fitsNode's podRequested for the listed reservations of a pod; the rows left restored with
 * the matched ones (with_matched) */
static char* or_resv_begin(or_cluster* c, const int32_t* ids, int32_t n_ids, int64_t** pod_requested) {
  const int32_t N = c->n;
  char* m = (char*)calloc((size_t)(c->n_resv > 0 ? c->n_resv : 1), 1);
  for (int32_t j = 0; j < n_ids; j++)
    if (or_resv_usable(&c->resv[ids[j]])) m[ids[j]] = 1;
  c->resv_m = m;
  or_restore(c, m, 0);
  *pod_requested = (int64_t*)malloc(sizeof(int64_t) * PRW * (size_t)(N > 0 ? N : 1));
  for (int32_t i = 0; i < N; i++) {
    for (int k = 0; k < KE_NRES; k++) (*pod_requested)[i * PRW + k] = c->nodes[i].node.requested[k] + c->nodes[i].rv_req[k];
    for (int id = 0; id < KE_MAX_XRES; id++) (*pod_requested)[i * PRW + KE_NRES + id] = c->nodes[i].rv_x[id];
  }
  or_restore(c, m, 1);
  return m;
}

/* golden-vector entry point: the Reservation plugin's Score per node (every node in PreScore's list) */
int32_t or_reservation_prescore(or_cluster* c, const ke_pod* pod, const int32_t* ids, int32_t n_ids, int64_t* raw,
                                int32_t* nom) {
  int64_t* pr;
  char* m = or_resv_begin(c, ids, n_ids, &pr);
  const int32_t pref = or_resv_prescore(c, pod, m, pr, NULL, 0, raw, nom);
  or_restore(c, NULL, 0);
  c->resv_m = NULL;
  free(m);
  free(pr);
  return pref;
}

/* golden-vector entry point: filterWithReservations (reservation/plugin.go:351-442) over reservation r alone on
 * `node`, with the cycle state a test gives directly: pod_requested[PRW] = nodeRState.podRequested (cpu, memory,
 * then [KE_NRES + id] the scalars), r_allocated[PRW] = nodeRState.rAllocated; `required` =
 * requiredFromReservation, `affinity` = state.hasAffinity.  Returns 0 = Success, 1 = Unschedulable with a node
 * insufficiency ("... by node"), 2 = with a reservation reason ("Reservation(s) ..."), 3 = no reservation met. */
int32_t or_rsv_filter_with(or_cluster* c, int32_t r, const ke_pod* pod, int32_t node, const int64_t* pod_requested,
                           const int64_t* r_allocated, int32_t required, int32_t affinity) {
  if (!required) return 0;
  if (r < 0 || r >= c->n_resv || node < 0 || node >= c->n) return -1;
  char* m = (char*)calloc((size_t)c->n_resv, 1);
  m[r] = 1;
  c->resv_m = m;
  const ke_reservation* rv = &c->resv[r];
  int shared = 0;
  for (int k = 0; k < KE_NRES; k++)
    if (rv->allocatable[k] != 0 && !((rv->names_excluded >> k) & 1) && pod->requests[k] != 0) shared = 1;
  for (int32_t e = c->rres ? c->roff[r] : 0; c->rres && e < c->roff[r + 1]; e++)
    if (!c->rres[e].excluded && c->rres[e].id != KE_RSV_RES_PODS && or_pod_request_of(pod, c->rres[e].id) != 0) shared = 1;
  int32_t out = 3;
  if (shared || affinity) {
    /* the node part alone (a Default copy of the reservation), then the whole decision */
    ke_reservation keep = *rv;
    c->resv[r].allocate_policy = KE_RSV_POLICY_DEFAULT;
    const int node_fits = or_resv_nominable(c, r, pod, node, pod_requested, r_allocated, 1);
    c->resv[r] = keep;
    const int fits = or_resv_nominable(c, r, pod, node, pod_requested, r_allocated, 1);
    out = fits ? 0 : !node_fits ? 1 : 2;
  }
  c->resv_m = NULL;
  free(m);
  return out;
}

/* golden-vector entry point: the Reservation Filter with a reservation affinity on `node` (1 = passes) */
int32_t or_reservation_filter(or_cluster* c, const ke_pod* pod, const int32_t* ids, int32_t n_ids, int32_t node) {
  int64_t* pr;
  char* m = or_resv_begin(c, ids, n_ids, &pr);
  const int32_t ok = or_resv_filter_node(c, pod, m, pr, node);
  or_restore(c, NULL, 0);
  c->resv_m = NULL;
  free(m);
  free(pr);
  return ok;
}

/* A KE_RSV_MATCHED pod: BeforePreFilter restore with its matched reservations, Filter / Score of the plugins
 * (eval_pod), the Reservation plugin's PreScore / Score, NormalizeScore (DefaultNormalizeScore over the
 * feasible nodes, scoring.go:134-139) and selectHost over the total with weight_reservation.  Returns the
 * chosen node (-1), its total in *best and the nominated reservation of every node in nom[]. */
static int32_t or_resv_eval(or_cluster* c, const ke_pod* pod, int64_t now, eval_out* o, const int32_t* ids, int32_t n_ids,
                            int affinity, int32_t* best, int32_t* nom) {
  const int32_t N = c->n;
  int64_t* pr;
  char* m = or_resv_begin(c, ids, n_ids, &pr);
  int16_t bs16;
  (void)eval_pod(c, pod, now, o, &bs16);
  /* NodeNUMAResource's FilterNominateReservation under a NUMA policy (plugin.go:448-504) for a pod with a reservation
   * affinity, in the cycle's restore state: tryAllocateFromReservation over the reservation alone on the stored
   * affinity; a reservation outside RestoreReservation's matched set passes */
  int8_t* rok = NULL;
  if (affinity) {
    rok = (int8_t*)malloc((size_t)(c->n_resv > 0 ? c->n_resv : 1));
    memset(rok, 1, (size_t)(c->n_resv > 0 ? c->n_resv : 1));
    for (int32_t r = 0; r < c->n_resv; r++) {
      if (!m[r]) continue;
      const int32_t i = c->resv[r].node;
      int ex;
      const int pol = effective_policy(&c->nodes[i], pod, &ex);
      if (pol <= KE_NUMA_POLICY_NONE || pod_requests_zero(pod) || o[i].status != KE_CODE_SUCCESS) continue;
      int32_t M[64];
      const int nM = numa_rsv_matched(c, i, M);
      int in = 0;
      for (int q = 0; q < nM; q++) in |= M[q] == r;
      if (!in) continue;
      uint32_t aff = 0;
      if (!numa_stored_affinity(c, pod, i, &aff)) aff = 0;
      rok[r] = (int8_t)(numa_from_rsv_try(c, pod, i, M, nM, &r, 1, aff, 1, NULL, NULL, NULL) == 1);
    }
  }
  or_restore(c, NULL, 0);
  uint8_t* feasible = (uint8_t*)malloc((size_t)(N > 0 ? N : 1));
  for (int32_t i = 0; i < N; i++) feasible[i] = o[i].status == KE_CODE_SUCCESS;
  if (affinity) {
    char* has = (char*)calloc((size_t)(N > 0 ? N : 1), 1);
    for (int32_t r = 0; r < c->n_resv; r++)
      if (m[r]) has[c->resv[r].node] = 1;
    for (int32_t i = 0; i < N; i++)
      if (feasible[i]) feasible[i] = (uint8_t)(has[i] && or_resv_filter_node(c, pod, m, pr, i));
    free(has);
  }
  int64_t* raw = (int64_t*)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
  c->numa_rok = rok;
  (void)or_resv_prescore(c, pod, m, pr, feasible, affinity, raw, nom);
  c->numa_rok = NULL;
  free(rok);
  /* NodeNUMAResource's Score of a node with reservations in RestoreReservation's matched set under a NUMA policy reads
   * the nominated reservation (scoring.go:101-119); an error status there fails the pod's cycle (RunScorePlugins) */
  int score_err = 0;
  or_restore(c, m, 1);
  c->numa_nom = nom;
  for (int32_t i = 0; i < N && !score_err; i++) {
    if (!feasible[i]) continue;
    int ex;
    int32_t M[64];
    if (effective_policy(&c->nodes[i], pod, &ex) <= KE_NUMA_POLICY_NONE || numa_rsv_matched(c, i, M) == 0) continue;
    int err = 0;
    o[i].numa = (int16_t)numa_score_ex(c, pod, i, &err);
    score_err |= err;
  }
  c->numa_nom = NULL;
  or_restore(c, NULL, 0);
  /* DeviceShare's Score reads the nominated reservation (scoring.go:83-102), and NormalizeScore runs over the nodes
   * that passed every Filter, the Reservation Filter of a reservation affinity included */
  ds_pod dsp;
  ds_prepare_pod(c, pod, &dsp);
  if (!dsp.skip && !dsp.status) {
    c->ds_nom = nom;
    for (int32_t i = 0; i < N; i++)
      if (feasible[i] && c->nodes[i].has_dev_cache) o[i].ds = (int16_t)or_ds_score(c, pod, i);
    c->ds_nom = NULL;
  }
  for (int32_t i = 0; i < N; i++)
    if (!feasible[i] && o[i].status == KE_CODE_SUCCESS) o[i].status = KE_CODE_UNSCHEDULABLE;
  normalize_and_total(c, o, N);
  int64_t mx = 0;
  for (int32_t i = 0; i < N; i++)
    if (feasible[i] && raw[i] > mx) mx = raw[i];
  int32_t b = -1;
  int64_t bt = -1;
  for (int32_t i = 0; i < N; i++) {
    if (!feasible[i]) continue;
    const int64_t n = mx > 0 ? MAX_NODE_SCORE * raw[i] / mx : 0;
    const int64_t t = o[i].total + c->cfg.weight_reservation * n;
    if (t > bt) {
      bt = t;
      b = i;
    }
  }
  if (score_err) b = -1, bt = -1;
  *best = b >= 0 ? (int32_t)bt : -1;
  c->resv_m = NULL;
  free(m);
  free(pr);
  free(feasible);
  free(raw);
  return b;
}

/* the KE_RSV_MATCHED pods this restatement covers (koord_eval.h ke_pod_reservations) */
static int or_resv_supported(const or_cluster* c, int32_t n_pods, const ke_pod* pods) {
  int node_bind = 0;
  for (int i = 0; i < c->n; i++) node_bind |= c->nodes[i].node.cpu_bind_policy != KE_NODE_CPU_BIND_NONE;
  for (int32_t p = 0; p < n_pods; p++) {
    const int32_t n_ids = c->moff && c->m_pods == n_pods ? c->moff[p + 1] - c->moff[p] : 0;
    if (pods[p].reservation_matched != KE_RSV_MATCHED && pods[p].reservation_matched != KE_RSV_AFFINITY) {
      if (n_ids) return KE_ERR_INVALID;
      /* a reservation-ignored pod: tryAllocateIgnoreReservation's remainder is restated for a pod binding no CPUs
       * (the held NUMA amounts reusable), a pod binding CPUs on nodes without a NUMA policy (the held CPUs) and a
       * DeviceShare pod without hints beside held devices off NUMA-policy nodes; refused: a binding pod with a NUMA
       * policy beside held NUMA resources / CPUs, a binding pod beside those on a NUMA-policy node (its hints over
       * the held CPUs), a DeviceShare pod with hints or a NUMA policy (node or pod) beside held devices */
      if (pods[p].reservation_matched == KE_RSV_IGNORED && c->ralloc) {
        int dev = 0, dev_on_policy = 0, numa_cpu = 0, on_policy = 0;
        for (int32_t r = 0; r < c->n_resv; r++) {
          const int h = or_holds_of(&c->ralloc[r]);
          const int pol = c->nodes[c->resv[r].node].node.numa_topology_policy != KE_NUMA_POLICY_NONE;
          if (h & KE_RSV_HOLDS_DEVICES) dev = 1, dev_on_policy |= pol;
          if (h & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)) {
            numa_cpu = 1;
            on_policy |= pol;
          }
        }
        ds_pod d; /* (a pod binding CPUs allocates from the held CPUs: or_numa_ignored; a DeviceShare pod from the
                     held devices: tryAllocateIgnoreReservation; a pod binding none reads the held NUMA amounts as
                     reusable: or_numa_ignored_reusable) -- the held devices in NUMA hints and a binding pod's NUMA
                     hints over held CPUs are not restated */
        ds_prepare_pod(c, &pods[p], &d);
        const int pod_pol = pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE;
        cpuset_state cst;
        cpuset_prefilter(c, &pods[p], &cst);
        const int binds = cst.rcb || cst.invalid || (node_bind && pods[p].requests[KE_RES_CPU] > 0);
        /* a binding pod under a NUMA policy beside held NUMA resources / CPUs: tryAllocateIgnoreReservation in its
         * hints (numa_admit) -- refused as for matched pods with fractional CPUs or a required FullPCPUs binding
         * (the pod's, or a FullPCPUsOnly node's among those) */
        int full_req = cst.required == KE_CPU_BIND_FULL_PCPUS;
        for (int32_t r = 0; cst.required != KE_CPU_BIND_FULL_PCPUS && cst.required != KE_CPU_BIND_SPREAD_BY_PCPUS &&
                            r < c->n_resv; r++)
          if ((or_holds_of(&c->ralloc[r]) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)) &&
              c->nodes[c->resv[r].node].node.cpu_bind_policy == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY)
            full_req = 1;
        const int pol_here = (numa_cpu && pod_pol) || on_policy;
        if ((dev && !d.skip && (d.h || pod_pol || dev_on_policy)) ||
            (binds && pol_here && (pods[p].requests[KE_RES_CPU] % 1000 != 0 || full_req)))
          return KE_ERR_UNSUPPORTED;
      }
      continue;
    }
    if (!(c->moff && c->m_pods == n_pods)) return KE_ERR_INVALID;
    cpuset_state st;
    cpuset_prefilter(c, &pods[p], &st);
    ds_pod d;
    ds_prepare_pod(c, &pods[p], &d);
    /* every requested name beyond cpu / memory is read through its ke_pod.xres entry: a name without an id is
     * refused (batch / mid resources included); a DeviceShare pod allocates from its matched reservations' devices
     * (deviceshare/reservation.go:207-449) -- not with device hints / joint allocation, nor in NUMA hints (a pod
     * with a NUMA policy, or a NUMA-policy node, beside a matched reservation holding devices) */
    if (pods[p].has_other_requests > 1 || pods[p].has_unsupported_device_requests) return KE_ERR_UNSUPPORTED;
    if (!d.skip && c->ralloc)
      for (int32_t j = c->moff[p]; j < c->moff[p + 1]; j++) {
        const int32_t r = c->mids[j];
        if (!or_resv_usable(&c->resv[r]) || !(or_holds_of(&c->ralloc[r]) & KE_RSV_HOLDS_DEVICES)) continue;
        if (d.h || pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE ||
            c->nodes[c->resv[r].node].node.numa_topology_policy != KE_NUMA_POLICY_NONE)
          return KE_ERR_UNSUPPORTED;
      }
    /* under a NUMA policy (the pod's or the node's) a matched reservation holding NUMA resources / CPUs enters the
     * hints through its allocate-from-reservation trials (numa_admit) for a pod without device requests; refused: a
     * DeviceShare pod's joint hints there, a binding pod with fractional CPUs or under a required FullPCPUs policy (the
     * product counts a view's CPUs; preferredCPUs taken first may split cores there), more than 8 such reservations
     * of the pod on one node (the product's NV_MAX, 31) */
    if (c->ralloc) {
      const int binds = st.rcb || st.invalid || (node_bind && pods[p].requests[KE_RES_CPU] > 0);
      const int dev = !d.skip || d.h;
      for (int32_t j = c->moff[p]; j < c->moff[p + 1]; j++) {
        const int32_t r = c->mids[j];
        if (!or_resv_usable(&c->resv[r]) || !(or_holds_of(&c->ralloc[r]) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET)))
          continue;
        const int32_t node = c->resv[r].node;
        const int rq = st.required == KE_CPU_BIND_FULL_PCPUS ? 1 : st.required == KE_CPU_BIND_SPREAD_BY_PCPUS ? 2 : 0;
        const int full_req = rq == 1 || (rq == 0 && c->nodes[node].node.cpu_bind_policy == KE_NODE_CPU_BIND_FULL_PCPUS_ONLY);
        if ((pods[p].numa_topology_policy != KE_NUMA_POLICY_NONE ||
             c->nodes[node].node.numa_topology_policy != KE_NUMA_POLICY_NONE) &&
            (dev || (binds && (pods[p].requests[KE_RES_CPU] % 1000 != 0 || full_req))))
          return KE_ERR_UNSUPPORTED;
        int same = 0;
        for (int32_t j2 = c->moff[p]; j2 < c->moff[p + 1]; j2++) {
          const int32_t r2 = c->mids[j2];
          same += or_resv_usable(&c->resv[r2]) && c->resv[r2].node == node &&
                  (or_holds_of(&c->ralloc[r2]) & (KE_RSV_HOLDS_NUMA | KE_RSV_HOLDS_CPUSET));
        }
        if (same > 31) return KE_ERR_UNSUPPORTED;
      }
    }
  }
  return KE_OK;
}

int or_schedule(or_cluster* c, int32_t n_pods, const ke_pod* pods, int64_t now, int32_t* chosen, int32_t* score,
                uint64_t* dev_alloc, int64_t* numa_alloc, uint64_t* cpusets, int n_threads) {
  int rc = check_supported(c, n_pods, pods);
  if (rc) return rc;
  rc = or_resv_supported(c, n_pods, pods);
  if (rc) return rc;
  const int64_t N = c->n;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#else
  (void)n_threads;
#endif
  if (numa_alloc) memset(numa_alloc, 0, sizeof(int64_t) * 16 * (size_t)n_pods);
  free(c->last_vf);
  c->last_vf = (int8_t*)malloc((size_t)(n_pods > 0 ? n_pods : 1) * 2 * KE_MAX_MINORS);
  memset(c->last_vf, -1, (size_t)(n_pods > 0 ? n_pods : 1) * 2 * KE_MAX_MINORS);
  c->last_vf_n = n_pods;
  eval_out* o = (eval_out*)malloc(sizeof(eval_out) * (size_t)(N > 0 ? N : 1));
  int32_t* nom = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
  if (c->moff && c->m_pods != n_pods) c->moff = (free(c->moff), NULL); /* lists for another queue: none */
  free(c->last_resv);
  c->last_resv = (int32_t*)calloc((size_t)(n_pods > 0 ? n_pods : 1), sizeof(int32_t));
  c->last_resv_n = n_pods;
  for (int p = 0; p < n_pods; p++) {
    /* ElasticQuota PreFilter (plugin.go:223-275): a refused pod is evaluated nowhere */
    if (c->quotas && orq_admit(c->quotas, &pods[p]) == 0) {
      chosen[p] = -1;
      if (score) score[p] = -1;
      if (cpusets) memset(cpusets + (int64_t)p * ACC_WORDS, 0, sizeof(uint64_t) * ACC_WORDS);
      if (dev_alloc) dev_alloc[p] = 0;
      continue;
    }
    int16_t bs16;
    int32_t bs, b;
    int ign_restored = 0;
    const int affinity = pods[p].reservation_matched == KE_RSV_AFFINITY;
    const int32_t n_ids = c->moff && pods[p].reservation_matched ? c->moff[p + 1] - c->moff[p] : 0;
    if (n_ids > 0 || affinity) {
      b = or_resv_eval(c, &pods[p], now, o, c->moff ? c->mids + c->moff[p] : NULL, n_ids, affinity, &bs, nom);
    } else if (pods[p].reservation_matched == KE_RSV_IGNORED) {
      /* a reservation-ignored pod (transformer.go:101-106, 181-199): every available reservation matchedOrIgnored,
       * restoreMatchedReservation for each; the Reservation plugin filters nothing (plugin.go:350-353), skips
       * PreScore (scoring.go:48-50) and Reserve (plugin.go:755-761) */
      char* all = (char*)malloc((size_t)(c->n_resv > 0 ? c->n_resv : 1));
      memset(all, 1, (size_t)(c->n_resv > 0 ? c->n_resv : 1));
      or_restore(c, all, 2);
      c->ignored = 1;
      b = eval_pod(c, &pods[p], now, o, &bs16);
      bs = bs16;
      ign_restored = 1; /* NodeNUMAResource's Reserve reads the same cycle state (the reusable NUMA view) */
      free(all);
    } else {
      b = eval_pod(c, &pods[p], now, o, &bs16);
      bs = bs16;
    }
    chosen[p] = b;
    if (score) score[p] = b >= 0 ? bs : -1;
    uint64_t mask = 0;
    reserve_plan rp;
    memset(&rp, 0, sizeof rp);
    ds_aff da = NO_AFF; /* the affinity the Filter stored, for DeviceShare's Reserve */
    char* mflags = NULL; /* the matched flags again for NodeNUMAResource's Reserve */
    if (b >= 0 && (n_ids > 0 || affinity)) {
      mflags = (char*)calloc((size_t)(c->n_resv > 0 ? c->n_resv : 1), 1);
      for (int32_t j = c->moff[p]; j < c->moff[p + 1]; j++)
        if (or_resv_usable(&c->resv[c->mids[j]])) mflags[c->mids[j]] = 1;
      c->resv_m = mflags;
    }
    if (mflags) or_restore(c, mflags, 1); /* the cycle's restore state through Reserve (as the Filter saw it) */
    if (b >= 0) da = ds_reserve_affinity(c, &pods[p], b);
    const int plan = b >= 0 ? or_reserve_plan(c, &pods[p], b, &rp, mflags ? nom[b] : -1) : 0;
    if (mflags) or_restore(c, NULL, 0);
    c->ds_nom = mflags ? nom : NULL; /* DeviceShare Reserve: the nominated reservation (with resv_m / ignored) */
    if (b >= 0 && (plan != 0 || !ds_reserve_feasible(c, &pods[p], b, da))) {
      /* Reserve failed (Unreserve undoes the others): not placed */
      chosen[p] = -1;
      if (score) score[p] = -1;
      b = -1;
      memset(&rp, 0, sizeof rp);
    }
    if (cpusets) memcpy(cpusets + (int64_t)p * ACC_WORDS, rp.cpus, sizeof rp.cpus);
    if (b >= 0) {
      /* Reserve in profile order: LoadAware podAssignCache.assign (load_aware.go:192-195) at `now`,
       * NodeNUMAResource (NUMA allocation + cpuset), DeviceShare device allocation (plugin.go:426-492);
       * framework assume: NodeInfo.Requested. */
      or_pod_assign(c, b, &pods[p], now);
      or_reserve_apply(c, b, &rp, numa_alloc ? numa_alloc + (int64_t)p * 16 : NULL);
      mask = ds_reserve_on(c, &pods[p], b, da, (int8_t(*)[KE_MAX_MINORS])(c->last_vf + (int64_t)p * 2 * KE_MAX_MINORS));
      c->resv_m = NULL;
      c->ds_nom = NULL;
      c->ignored = 0;
      c->nodes[b].node.requested[KE_RES_CPU] += pods[p].requests[KE_RES_CPU];
      c->nodes[b].node.requested[KE_RES_MEMORY] += pods[p].requests[KE_RES_MEMORY];
      c->nodes[b].node.pod_count++; /* NodeInfo.AddPod */
      /* NodeInfo (NonZero)Requested of every resource the pod requests (NodeResourcesFitPlus reads them) */
      or_node* nb = &c->nodes[b];
      for (int32_t e = 0; e < pods[p].n_xres; e++) {
        ke_node_resource* r = (ke_node_resource*)node_xres(nb, pods[p].xres_id[e]);
        if (r) r->requested += pods[p].xres_value[e];
        else if (pods[p].xres_value[e] != 0 && nb->n_xres < KE_MAX_XRES) {
          ke_node_resource z = {pods[p].xres_id[e], 0, 0, pods[p].xres_value[e]};
          nb->xres[nb->n_xres++] = z;
        }
      }
      if (c->quotas) orq_reserve(c->quotas, &pods[p]); /* ElasticQuota Reserve */
      if ((n_ids > 0 || affinity) && nom[b] >= 0) {
        /* Reservation Reserve: assumePod -> AddAssignedPod (reservation/plugin.go:783,
         * reservation_info.go:458-468): allocated += Mask(requests, ResourceNames), one more allocated pod */
        ke_reservation* r = &c->resv[nom[b]];
        for (int k = 0; k < KE_NRES; k++)
          if (r->allocatable[k] != 0 && !((r->names_excluded >> k) & 1)) r->allocated[k] += pods[p].requests[k];
        for (int32_t e = c->rres ? c->roff[nom[b]] : 0; c->rres && e < c->roff[nom[b] + 1]; e++)
          if (!c->rres[e].excluded && c->rres[e].id != KE_RSV_RES_PODS) c->rres[e].allocated += or_pod_request_of(&pods[p], c->rres[e].id);
        r->allocated_pods++;
        c->last_resv[p] = 1 + nom[b];
        or_owner_update(c, nom[b], &pods[p], rp.cpus, numa_alloc ? numa_alloc + (int64_t)p * 16 : NULL, mask, +1);
        or_restore(c, NULL, 0);
      }
    }
    if (dev_alloc) dev_alloc[p] = mask;
    c->resv_m = NULL;
    c->ds_nom = NULL;
    c->ignored = 0;
    if (ign_restored) or_restore(c, NULL, 0);
    free(mflags);
  }
  free(o);
  free(nom);
  free(c->moff); /* the lists were for this call */
  c->moff = NULL;
  return KE_OK;
}
int or_last_reservations(const or_cluster* c, int32_t n, int32_t* out) {
  for (int32_t p = 0; p < n; p++) out[p] = p < c->last_resv_n ? c->last_resv[p] : 0;
  return KE_OK;
}

/* ---------------------------------------------------------------------------------------------- */
/* Unreserve / pod delete (ReservePlugin.Unreserve of every plugin, framework ForgetPod)             */
/* ---------------------------------------------------------------------------------------------- */

/* The release of one placement recorded in `a` (see ke_pod_release in koord_eval.h):
 *  - loadaware Unreserve: podAssignCache.unAssign (load_aware.go:197-199, pod_assign_cache.go:126-136)
 *  - framework RemovePod: NodeInfo.Requested and the per-resource requested NodeResourcesFitPlus reads
 *  - nodenumaresource Unreserve: resourceManager.Release -> NodeAllocation.release (plugin.go:569-577,
 *    node_allocation.go:158-190): RefCount-- per CPU (deleted at 0), the pod leaves sharedNode /
 *    singleNUMANode of its CPUs' NUMA ids, allocatedResources[id] = SubtractWithNonNegativeResult;
 *    nothing was recorded on a node without a valid CPU topology (Update, resource_manager.go:461-466)
 *  - deviceshare Unreserve: updateCacheUsed(allocationResult, pod, false) (plugin.go:498-516,
 *    device_cache.go:184-209): used = SubtractWithNonNegativeResult(used, allocation), deleted when zero
 *  - elasticquota Unreserve: UnreservePod (plugin.go:361, group_quota_manager.go:965-981), or OnPodDelete
 *    (:922-941) for an informer delete (quota.c orq_release) */
int or_pod_release(or_cluster* c, const ke_pod* pod, const ke_pod_allocation* a, int32_t mode) {
  const int32_t node = a->node;
  if (node >= c->n) return KE_ERR_NOT_FOUND;
  int32_t ridx = -1; /* the reservation the pod was assumed into: by uid when the record has one */
  if (a->reservation > 0 && a->reservation_uid != 0) {
    for (int32_t i = 0; i < c->n_resv && ridx < 0; i++)
      if (c->resv[i].uid == a->reservation_uid) ridx = i;
  } else if (a->reservation != 0) {
    if (a->reservation < 0 || a->reservation > c->n_resv) return KE_ERR_NOT_FOUND;
    ridx = a->reservation - 1;
  }
  if (node >= 0 && ridx >= 0) {
    /* reservation forgetPod -> RemoveAssignedPod (reservation/plugin.go:815-819, reservation_info.go:470-482):
     * allocated = SubtractWithNonNegativeResult(allocated, Mask(requests, ResourceNames)) */
    ke_reservation* r = &c->resv[ridx];
    for (int k = 0; k < KE_NRES; k++)
      if (r->allocatable[k] != 0 && !((r->names_excluded >> k) & 1))
        r->allocated[k] = r->allocated[k] - pod->requests[k] > 0 ? r->allocated[k] - pod->requests[k] : 0;
    for (int32_t e = c->rres ? c->roff[ridx] : 0; c->rres && e < c->roff[ridx + 1]; e++) {
      ke_reservation_resource* x = &c->rres[e];
      if (x->excluded || x->id == KE_RSV_RES_PODS) continue;
      const int64_t v = x->allocated - or_pod_request_of(pod, x->id);
      x->allocated = v > 0 ? v : 0;
    }
    if (r->allocated_pods > 0) r->allocated_pods--;
    or_owner_update(c, ridx, pod, a->cpuset, a->numa, a->device_minors, -1);
    or_restore(c, NULL, 0);
  }
  if (node >= 0) {
    or_node* n = &c->nodes[node];
    or_pod_unassign(c, node, pod->uid);
    n->node.requested[KE_RES_CPU] -= pod->requests[KE_RES_CPU];
    n->node.requested[KE_RES_MEMORY] -= pod->requests[KE_RES_MEMORY];
    n->node.pod_count--; /* NodeInfo.RemovePod */
    /* NodeInfo.RemovePod: Requested.ScalarResources by resource id, whichever plugins read them */
    for (int32_t e = 0; e < pod->n_xres; e++) {
      ke_node_resource* r = (ke_node_resource*)node_xres(n, pod->xres_id[e]);
      if (r) r->requested -= pod->xres_value[e];
    }
    const int parked = !n->cpus && n->kept_cpus; /* NRT deleted: the NodeAllocation is parked */
    if (cpus_valid(n) || parked) {
      or_cpus* x = parked ? n->kept_cpus : n->cpus;
      ke_numa_zone* zones = parked ? n->kept_zone : n->zone;
      const int32_t nz = parked ? n->n_kept_zone : n->n_zone;
      int used[ACC_MAX_CPUS], nu = 0;
      for (int cpu = 0; cpu < ACC_MAX_CPUS; cpu++) {
        if (!(a->cpuset[cpu >> 6] >> (cpu & 63) & 1) || !x->al.present[cpu]) continue;
        if (--x->al.ref[cpu] == 0) {
          x->al.present[cpu] = 0;
          x->al.excl[cpu] = 0;
        }
        int f = 0;
        for (int k = 0; k < nu && !f; k++) f = used[k] == x->t.node[cpu];
        if (!f) used[nu++] = x->t.node[cpu];
      }
      for (int z = 0; z < nz; z++) {
        ke_numa_zone* zn = &zones[z];
        for (int k = 0; k < nu; k++)
          if (used[k] == zn->id) {
            int16_t* cnt = nu > 1 ? &zn->shared_pods : &zn->single_pods;
            if (*cnt > 0) (*cnt)--;
            zn->numa_status = zone_status_of(zn);
          }
        if (!(zn->has_allocated & KE_NUMA_ALLOC_ENTRY)) continue;
        for (int r = 0; r < KE_NRES; r++) {
          const int64_t b = a->numa[2 * zn->id + r];
          if (b == 0) continue; /* a key of the pod's allocation carries a non-zero amount */
          const uint8_t key = r == KE_RES_CPU ? KE_NUMA_ALLOC_CPU : KE_NUMA_ALLOC_MEMORY;
          const int64_t v = ((zn->has_allocated & key) ? zn->allocated[r] : 0) - b;
          zn->allocated[r] = v > 0 ? v : 0;
          zn->has_allocated |= key;
        }
      }
    }
    if (n->has_dev_cache && a->device_minors) {
      ds_pod d;
      ds_prepare_pod(c, pod, &d);
      for (int i = 0; i < n->n_dev; i++) {
        ke_device* dv = &n->dev[i];
        if (!(a->device_minors >> (16 * dv->type + dv->minor) & 1)) continue;
        const int t = dv->type, nk = nkeys(t);
        if (t > 0 && a->vf_rank[t - 1][dv->minor] >= 0) /* removeVFAllocations */
          dv->vf_allocated &= ~(1ull << a->vf_rank[t - 1][dv->minor]);
        rl alloc = d.has[t] ? d.req[t] : rl_empty();
        if (t == KE_DEV_GPU) fill_gpu_total_mem(dv, &alloc);
        rl used = rl_sub_nonneg(dev_used(dv, nk), alloc, nk);
        if (rl_is_zero(used, nk)) used = rl_empty();
        for (int k = 0; k < nk; k++) {
          dv->has_used[k] = used.has[k];
          dv->used[k] = used.has[k] ? used.v[k] : 0;
        }
      }
    }
  }
  if (c->quotas && pod->quota > 0)
    orq_release(c->quotas, pod, node >= 0 && a->quota_assigned, mode == KE_RELEASE_DELETE);
  return KE_OK;
}

/* The oracle's object state of `node` in the product's introspection layout (ke_debug_node_state). */
int or_debug_node_state(const or_cluster* c, int32_t node, ke_node* out, int32_t cpu_cap, ke_cpu* cpus,
                        int32_t* n_cpus, int32_t zone_cap, ke_numa_zone* zones, int32_t* n_zones, int32_t dev_cap,
                        ke_device* devs, int32_t* n_devs) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  const or_node* n = &c->nodes[node];
  if (out) *out = n->node;
  int32_t k = 0;
  if (n->cpus)
    for (int id = 0; id < ACC_MAX_CPUS; id++) {
      if (!n->cpus->t.valid[id]) continue;
      if (cpus && k < cpu_cap) {
        ke_cpu e;
        memset(&e, 0, sizeof e);
        e.cpu_id = id;
        e.core_id = n->cpus->t.core[id];
        e.numa_id = n->cpus->t.node[id];
        e.socket_id = n->cpus->t.socket[id];
        e.ref_count = n->cpus->al.present[id] ? n->cpus->al.ref[id] : 0;
        e.exclusive = (uint8_t)(n->cpus->al.present[id] ? n->cpus->al.excl[id] : 0);
        e.reserved = n->cpus->reserved[id];
        cpus[k] = e;
      }
      k++;
    }
  if (n_cpus) *n_cpus = k;
  if (n_zones) *n_zones = n->n_zone;
  for (int32_t i = 0; zones && i < zone_cap && i < n->n_zone; i++) zones[i] = n->zone[i];
  if (n_devs) *n_devs = n->n_dev;
  for (int32_t i = 0; devs && i < dev_cap && i < n->n_dev; i++) devs[i] = n->dev[i];
  return KE_OK;
}
