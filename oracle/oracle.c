/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain-C restatement of the reference's
 * per-node Filter/Score arithmetic.  Every function cites the Go it follows
 * (paths relative to haoyann/koordinator @ /root/reference):
 *
 *   LoadAwareScheduling  pkg/scheduler/plugins/loadaware/load_aware.go, helper.go,
 *                        estimator/default_estimator.go, pod_assign_cache.go
 *   NodeNUMAResource     pkg/scheduler/plugins/nodenumaresource/plugin.go, scoring.go,
 *                        least_allocated.go, most_allocated.go, util.go
 *   helpers              apis/extension/node_resource_amplification.go, resource.go, load_aware.go
 *   framework            k8s v1.28.7 weighted score sum + selectHost (tie -> lowest node index)
 *
 * Unlike the product it precomputes nothing: GetEstimatedUsed is rebuilt from the NodeMetric and the
 * assign cache on every Filter and every Score call, as the Go plugin does.
 */
#include "oracle.h"

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
} or_node;

struct or_cluster {
  ke_config cfg;
  int32_t n;
  or_node* nodes;
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
static int pod_unsupported(const ke_pod* pod) { return pod_is_cpuset(pod) || pod->has_resource_spec; }
static int node_unsupported(const ke_node* n) { return n->numa_topology_policy != 0 || n->cpu_bind_policy != 0; }

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
int or_numa_filter(const or_cluster* c, const ke_pod* pod, int32_t node, int* reason) {
  const or_node* n = &c->nodes[node];
  *reason = KE_REASON_NONE;
  if (pod_requests_zero(pod)) return KE_CODE_SUCCESS; /* state.skip */
  const int64_t pod_cpu = pod->requests[KE_RES_CPU];
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
  const int64_t allocated_milli = n->node.cpuset_allocated_cpus * 1000;
  int64_t requested = n->node.requested[KE_RES_CPU];
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
static int64_t numa_resource_score(const ke_numa_args* na, const int64_t* requested, const int64_t* allocatable,
                                   const ke_pod* pod) {
  int64_t score = 0, wsum = 0;
  for (int r = 0; r < KE_NRES; r++) {
    int64_t w = na->weights[r];
    if (w == KE_ABSENT) continue;
    int64_t alloc = allocatable[r];
    int64_t req = requested[r] + pod->requests[r];
    if (alloc == 0) continue; /* calculateResourceAllocatableRequest result dropped */
    int64_t s;
    if (na->strategy == KE_STRATEGY_MOST_ALLOCATED) {
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

/* Plugin.Score  scoring.go:66-120 -> scoreWithAmplifiedCPUs :122-139 */
int64_t or_numa_score(const or_cluster* c, const ke_pod* pod, int32_t node) {
  const or_node* n = &c->nodes[node];
  if (pod_requests_zero(pod)) return 0; /* state.skip */
  /* getResourceOptions -> amplifyNUMANodeResources (util.go:78-87) */
  double ratio;
  if (n->node.nrt_cpu_amplification_ratio > -1.5) {
    ratio = n->node.nrt_cpu_amplification_ratio < 0 ? 0.0 : n->node.nrt_cpu_amplification_ratio;
  } else {
    if (n->node.amplification_error) return 0;
    ratio = n->node.cpu_amplification_ratio < 0 ? 0.0 : n->node.cpu_amplification_ratio;
  }
  int64_t requested[KE_NRES] = {n->node.requested[KE_RES_CPU], n->node.requested[KE_RES_MEMORY]};
  if (!(pod->requests[KE_RES_CPU] == 0 || ratio <= 1.0)) {
    if (n->node.cpu_topology_invalid) return 0;
    const int64_t allocated_milli = n->node.cpuset_allocated_cpus * 1000;
    requested[KE_RES_CPU] -= allocated_milli;
    requested[KE_RES_CPU] += amplify(allocated_milli, ratio);
  }
  return numa_resource_score(&c->cfg.numa, requested, n->node.allocatable, pod);
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
  for (int i = 0; i < c->n; i++) {
    free(c->nodes[i].pm);
    free(c->nodes[i].agg);
    free(c->nodes[i].asg);
  }
  free(c->nodes);
  free(c);
}

int or_node_upsert(or_cluster* c, int32_t node, const ke_node* n) {
  if (node < 0 || node >= c->n) return KE_ERR_NOT_FOUND;
  c->nodes[node].node = *n;
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
  int16_t la, numa, total;
} eval_out;

/* RunFilterPlugins in profile order (scheduler-config.yaml:68-73), then RunScorePlugins with
 * weights (:85-94) for a feasible node. */
static void eval_pair(const or_cluster* c, const ke_pod* pod, int32_t node, int64_t now, eval_out* o) {
  int reason = 0;
  int code = or_la_filter(c, pod, node, now, &reason);
  if (code == KE_CODE_SUCCESS) code = or_numa_filter(c, pod, node, &reason);
  o->status = (uint8_t)code;
  o->reason = (uint8_t)reason;
  if (code != KE_CODE_SUCCESS) {
    o->la = o->numa = 0;
    o->total = -1;
    return;
  }
  int64_t la = or_la_score(c, pod, node, now);
  int64_t nu = or_numa_score(c, pod, node);
  o->la = (int16_t)la;
  o->numa = (int16_t)nu;
  o->total = (int16_t)(c->cfg.weight_loadaware * la + c->cfg.weight_numa * nu);
}

static int check_supported(const or_cluster* c, int32_t n_pods, const ke_pod* pods) {
  for (int p = 0; p < n_pods; p++)
    if (pod_unsupported(&pods[p])) return KE_ERR_UNSUPPORTED;
  for (int i = 0; i < c->n; i++)
    if (node_unsupported(&c->nodes[i].node)) return KE_ERR_UNSUPPORTED;
  return KE_OK;
}

int or_eval(const or_cluster* c, int32_t n_pods, const ke_pod* pods, int64_t now, uint8_t* status, uint8_t* reason,
            int16_t* la_score, int16_t* numa_score, int16_t* total, int32_t* best, int n_threads) {
  int rc = check_supported(c, n_pods, pods);
  if (rc) return rc;
  const int64_t N = c->n;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#else
  (void)n_threads;
#endif
  for (int p = 0; p < n_pods; p++) {
    int32_t b = -1;
    int16_t bs = -1;
#pragma omp parallel
    {
      int32_t lb = -1;
      int16_t ls = -1;
#pragma omp for schedule(static)
      for (int64_t i = 0; i < N; i++) {
        eval_out o;
        eval_pair(c, &pods[p], (int32_t)i, now, &o);
        const int64_t k = (int64_t)p * N + i;
        if (status) status[k] = o.status;
        if (reason) reason[k] = o.reason;
        if (la_score) la_score[k] = o.la;
        if (numa_score) numa_score[k] = o.numa;
        if (total) total[k] = o.total;
        if (o.total > ls) { /* strict: keeps the lowest index of this thread's (ascending) chunk */
          ls = o.total;
          lb = (int32_t)i;
        }
      }
#pragma omp critical
      {
        if (ls > bs || (ls == bs && ls >= 0 && lb < b)) {
          bs = ls;
          b = lb;
        }
      }
    }
    if (best) best[p] = bs >= 0 ? b : -1;
  }
  return KE_OK;
}

int or_schedule(or_cluster* c, int32_t n_pods, const ke_pod* pods, int64_t now, int32_t* chosen, int32_t* score,
                int n_threads) {
  int rc = check_supported(c, n_pods, pods);
  if (rc) return rc;
  const int64_t N = c->n;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#else
  (void)n_threads;
#endif
  for (int p = 0; p < n_pods; p++) {
    int32_t b = -1;
    int16_t bs = -1;
#pragma omp parallel
    {
      int32_t lb = -1;
      int16_t ls = -1;
#pragma omp for schedule(static)
      for (int64_t i = 0; i < N; i++) {
        eval_out o;
        eval_pair(c, &pods[p], (int32_t)i, now, &o);
        if (o.total > ls) {
          ls = o.total;
          lb = (int32_t)i;
        }
      }
#pragma omp critical
      {
        if (ls > bs || (ls == bs && ls >= 0 && lb < b)) {
          bs = ls;
          b = lb;
        }
      }
    }
    if (bs < 0) b = -1;
    chosen[p] = b;
    if (score) score[p] = bs;
    if (b >= 0) {
      /* Reserve: LoadAware podAssignCache.assign (load_aware.go:192-195) at `now`;
       * framework assume: NodeInfo.Requested += pod requests. */
      or_pod_assign(c, b, &pods[p], now);
      c->nodes[b].node.requested[KE_RES_CPU] += pods[p].requests[KE_RES_CPU];
      c->nodes[b].node.requested[KE_RES_MEMORY] += pods[p].requests[KE_RES_MEMORY];
    }
  }
  return KE_OK;
}
