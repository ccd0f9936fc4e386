/* ElasticQuota admission — plain-C restatement of the reference (TEST INFRASTRUCTURE ONLY: the
 * oracle the GPU/host path is checked against; nothing in libkoordeval links or calls it).
 *
 *   runtime quota   pkg/scheduler/plugins/elasticquota/core/runtime_quota_calculator.go:117-189
 *                   (quotaTree.redistribution / iterationForRedistribution)
 *   limited request core/group_quota_manager.go:196-239 (recursiveUpdateGroupTreeWithDeltaRequest),
 *                   core/quota_info.go:217-228 (getLimitRequestNoLock)
 *   refresh         core/group_quota_manager.go:286-353 (refreshRuntimeNoLock, top-down); used limit
 *                   plugin_helper.go:318-323 (GetRuntime, quota_info.go:378-382, or GetMax)
 *   PreFilter       plugin.go:223-275, checkQuotaRecursive plugin_helper.go:281-301
 *   Reserve         core/group_quota_manager.go:700-760,943-963 (used += Mask(PodRequests, Max) on
 *                   the quota and every ancestor)
 * quotav1.LessThanOrEqual(a, b) compares only keys of b also present in a (k8s.io/apiserver v0.28.7
 * quota/v1); with non-negative values a key absent from a compares as 0.  A zero pod request counts
 * as an absent key (ke_pod carries no key set).  A Reserve into the system / default quota (limit_is_max)
 * with runtime quota on shrinks the tree total and refreshes every runtime limit (orq_reserve). */
#include "quota.h"

#include <string.h>

static int64_t pod_req(const ke_quota* q, const ke_pod* p, int r) {
  const int64_t v = r == 0 ? p->requests[KE_RES_CPU] : p->requests[KE_RES_MEMORY];
  return q->has_max[r] ? v : 0; /* quotav1.Mask(PodRequests, ResourceNames(Max)) */
}

/* iterationForRedistribution (runtime_quota_calculator.go:150-189) */
static void iterate(int64_t total, int64_t tw, const int* nodes, int n, const int64_t* w, const int64_t* req,
                    int64_t* rt) {
  if (tw <= 0) return;
  int next[KE_MAX_QUOTAS];
  int nn = 0;
  int64_t to_part = 0, ntw = 0;
  for (int k = 0; k < n; k++) {
    const int i = nodes[k];
    const double d = (double)w[i] * (double)total / (double)tw + 0.5;
    rt[i] += (int64_t)d;
    if (rt[i] < req[i]) {
      next[nn++] = i;
      ntw += w[i];
    } else {
      to_part += rt[i] - req[i];
      rt[i] = req[i];
    }
  }
  if (to_part > 0 && nn > 0) iterate(to_part, ntw, next, nn, w, req, rt);
}

/* redistribution (runtime_quota_calculator.go:117-148) over the children `ids` of one parent */
static void redistribute(int64_t total, const int* ids, int n, const int64_t* w, const int64_t* req,
                         const int64_t* mn, const uint8_t* lent, int64_t* rt) {
  int64_t to_part = total, tw = 0;
  int adj[KE_MAX_QUOTAS];
  int na = 0;
  for (int k = 0; k < n; k++) {
    const int i = ids[k];
    if (req[i] > mn[i]) {
      adj[na++] = i;
      tw += w[i];
      rt[i] = mn[i];
    } else {
      rt[i] = lent[i] ? req[i] : mn[i];
    }
    to_part -= rt[i];
  }
  if (to_part > 0) iterate(to_part, tw, adj, na, w, req, rt);
}

static int depth_of(const ke_quota* q, int n, int i) {
  int d = 0;
  while (q[i].parent >= 0) {
    i = q[i].parent;
    if (++d > n) return -1; /* cycle */
  }
  return d;
}

int orq_load(or_quotas* Q, const ke_quota_args* args, const ke_quota* q, int32_t n) {
  if (n < 0 || n > KE_MAX_QUOTAS) return KE_ERR_INVALID;
  memset(Q, 0, sizeof *Q);
  Q->n = n;
  Q->args = *args;
  memcpy(Q->q, q, sizeof(ke_quota) * (size_t)n);
  int depth[KE_MAX_QUOTAS], maxd = 0;
  for (int i = 0; i < n; i++) {
    if (q[i].parent >= n || q[i].parent < -1) return KE_ERR_INVALID;
    depth[i] = depth_of(q, n, i);
    if (depth[i] < 0) return KE_ERR_INVALID;
    if (depth[i] > maxd) maxd = depth[i];
  }
  for (int r = 0; r < KE_NRES; r++) {
    int64_t child[KE_MAX_QUOTAS], limreq[KE_MAX_QUOTAS], w[KE_MAX_QUOTAS], mn[KE_MAX_QUOTAS], rt[KE_MAX_QUOTAS];
    uint8_t lent[KE_MAX_QUOTAS];
    for (int i = 0; i < n; i++) {
      child[i] = q[i].self_request[r];
      w[i] = q[i].shared_weight[r];
      mn[i] = q[i].has_min[r] ? q[i].min[r] : 0; /* AutoScaleMin = Min until scaled below; guarantee 0 */
      lent[i] = q[i].allow_lent_resource;
      rt[i] = 0;
    }
    /* bottom-up: ChildRequest = Σ children's limited requests; Request = ChildRequest, raised to Min
     * when the quota does not lend; limited request = min(Request, Max) on Max's keys */
    for (int d = maxd; d >= 0; d--)
      for (int i = 0; i < n; i++) {
        if (depth[i] != d) continue;
        int64_t req = child[i];
        if (!q[i].allow_lent_resource && q[i].has_min[r] && q[i].min[r] > req) req = q[i].min[r];
        limreq[i] = (q[i].has_max[r] && req > q[i].max[r]) ? q[i].max[r] : req;
        if (q[i].parent >= 0) child[q[i].parent] += limreq[i];
      }
    /* top-down: the root's children share the tree total, every quota's children its runtime */
    int ids[KE_MAX_QUOTAS];
    for (int d = 0; d <= maxd + 1; d++) {
      for (int p = -1; p < n; p++) {
        if ((p < 0 ? 0 : depth[p] + 1) != d) continue;
        int k = 0;
        int64_t min_sum = 0;
        for (int i = 0; i < n; i++)
          if (q[i].parent == p && !q[i].limit_is_max) {
            ids[k++] = i;
            min_sum += mn[i];
          }
        if (k == 0) continue;
        const int64_t total = p < 0 ? args->total[r] : rt[p];
        /* ScaleMinQuotaManager.getScaledMinQuota (scale_minquota_when_over_root_res.go:129-184), every
         * child scale-enabled (UpdateQuota passes scaleMinQuotaEnabled, group_quota_manager.go:604):
         * total < ΣMin -> AutoScaleMin = int64(float64(total) * float64(Min) / float64(ΣMin)), 0 when
         * total <= 0; refreshRuntimeNoLock applies it before the parent's calculator shares (:320-333) */
        if (!args->disable_scale_min_quota && total < min_sum)
          for (int j = 0; j < k; j++)
            mn[ids[j]] = total <= 0 ? 0 : (int64_t)((double)total * (double)mn[ids[j]] / (double)min_sum);
        redistribute(total, ids, k, w, limreq, mn, lent, rt);
      }
    }
    /* Runtime carries every resource key of the tree (updateOneGroupRuntimeQuota over resourceKeys =
     * the union of the quotas' Max keys), unmasked (quota_info.go:378-382 GetRuntime); Max its own */
    int tree_has = 0;
    for (int i = 0; i < n; i++) tree_has |= q[i].has_max[r];
    for (int i = 0; i < n; i++) {
      const int use_max = !args->enable_runtime_quota || q[i].limit_is_max;
      Q->limit_has[i][r] = (uint8_t)(use_max ? q[i].has_max[r] : tree_has);
      Q->limit[i][r] = use_max ? q[i].max[r] : rt[i];
    }
  }
  return KE_OK;
}

int orq_admit(const or_quotas* Q, const ke_pod* pod) {
  if (pod->quota <= 0 || pod->quota > Q->n) return -1;
  const int qi = pod->quota - 1;
  const ke_quota* q = &Q->q[qi];
  int64_t req[KE_NRES];
  for (int r = 0; r < KE_NRES; r++) req[r] = pod_req(q, pod, r);
  for (int r = 0; r < KE_NRES; r++) /* used + request <= used limit */
    if (Q->limit_has[qi][r] && q->used[r] + req[r] > Q->limit[qi][r]) return 0;
  if (pod->quota_non_preemptible) /* non-preemptible used + request <= Min */
    for (int r = 0; r < KE_NRES; r++)
      if (q->has_min[r] && q->non_preemptible_used[r] + req[r] > q->min[r]) return 0;
  if (Q->args.enable_check_parent_quota) /* every ancestor below the root, on the request's keys */
    for (int a = q->parent; a >= 0; a = Q->q[a].parent)
      for (int r = 0; r < KE_NRES; r++)
        if (req[r] != 0 && Q->limit_has[a][r] && Q->q[a].used[r] + req[r] > Q->limit[a][r]) return 0;
  return 1;
}

void orq_reserve(or_quotas* Q, const ke_pod* pod) {
  if (pod->quota <= 0 || pod->quota > Q->n) return;
  const int qi = pod->quota - 1;
  int64_t req[KE_NRES];
  for (int r = 0; r < KE_NRES; r++) req[r] = pod_req(&Q->q[qi], pod, r);
  for (int a = qi; a >= 0; a = Q->q[a].parent)
    for (int r = 0; r < KE_NRES; r++) {
      Q->q[a].used[r] += req[r];
      if (pod->quota_non_preemptible) Q->q[a].non_preemptible_used[r] += req[r];
    }
  /* the system / default quota's used changed: updateClusterTotalResourceNoLock (group_quota_manager.go:
   * 268-271, 127-151) shrinks totalResourceExceptSystemAndDefaultUsed by it, the root's
   * RuntimeQuotaCalculator takes the new total and every runtime quota is refreshed from it */
  if (Q->q[qi].limit_is_max && Q->args.enable_runtime_quota) {
    ke_quota_args args = Q->args;
    for (int r = 0; r < KE_NRES; r++) args.total[r] -= req[r];
    ke_quota q[KE_MAX_QUOTAS];
    memcpy(q, Q->q, sizeof(ke_quota) * (size_t)Q->n);
    orq_load(Q, &args, q, Q->n);
  }
}

/* Unreserve (UnreservePod, group_quota_manager.go:965-981) of an assigned pod: used / non-preemptible used
 * minus Mask(PodRequests, Max) on the quota and every ancestor, each floored at 0 (addUsedNonNegativeNoLock,
 * quota_info.go:279-299); a system / default quota's smaller used grows the tree total back
 * (updateClusterTotalResourceNoLock, :127-151).  `del` (OnPodDelete, :922-941): the pod's request leaves
 * the quota's SelfRequest too (addRequestNonNegativeNoLock, quota_info.go:238-258) and the runtime is
 * recomputed. */
void orq_release(or_quotas* Q, const ke_pod* pod, int assigned, int del) {
  if (pod->quota <= 0 || pod->quota > Q->n) return;
  const int qi = pod->quota - 1;
  int64_t req[KE_NRES], before[KE_NRES];
  for (int r = 0; r < KE_NRES; r++) req[r] = pod_req(&Q->q[qi], pod, r), before[r] = Q->q[qi].used[r];
  ke_quota_args args = Q->args;
  int refresh = 0;
  if (assigned) {
    for (int a = qi; a >= 0; a = Q->q[a].parent)
      for (int r = 0; r < KE_NRES; r++) {
        int64_t u = Q->q[a].used[r] - req[r];
        Q->q[a].used[r] = u > 0 ? u : 0;
        if (pod->quota_non_preemptible) {
          u = Q->q[a].non_preemptible_used[r] - req[r];
          Q->q[a].non_preemptible_used[r] = u > 0 ? u : 0;
        }
      }
    if (Q->q[qi].limit_is_max && Q->args.enable_runtime_quota) {
      for (int r = 0; r < KE_NRES; r++) args.total[r] += before[r] - Q->q[qi].used[r];
      refresh = 1;
    }
  }
  if (del) {
    for (int r = 0; r < KE_NRES; r++) {
      const int64_t v = Q->q[qi].self_request[r] - req[r];
      Q->q[qi].self_request[r] = v > 0 ? v : 0;
    }
    refresh = 1;
  }
  if (refresh) {
    ke_quota q[KE_MAX_QUOTAS];
    memcpy(q, Q->q, sizeof(ke_quota) * (size_t)Q->n);
    orq_load(Q, &args, q, Q->n);
  }
}
