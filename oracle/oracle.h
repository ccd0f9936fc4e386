/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of koord-scheduler's LoadAwareScheduling,
 * NodeNUMAResource (policy None) and DeviceShare Filter/Score/Reserve and of the framework's
 * NormalizeScore + weighted sum + selectHost.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only
 * as the checker / the timed CPU baseline.  The product (libkoordeval.so) never links or calls it.
 *
 * It works on the same object-level structs as the product boundary (include/koord_eval.h) but keeps
 * its own state and recomputes every per-node quantity on every call, exactly like the Go plugins do.
 */
#ifndef KE_ORACLE_H
#define KE_ORACLE_H
#include <stdint.h>
#include "koord_eval.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_cluster or_cluster;

or_cluster* or_create(const ke_config* cfg, int32_t n_nodes);
void or_destroy(or_cluster* c);
int or_node_upsert(or_cluster* c, int32_t node, const ke_node* n);
int or_node_delete(or_cluster* c, int32_t node);          /* Node informer delete (ke_node_delete) */
int or_node_topology_delete(or_cluster* c, int32_t node); /* NRT delete (ke_node_topology_delete) */
int or_node_set_requested(or_cluster* c, int32_t node, int64_t milli_cpu, int64_t memory);
int or_node_set_cpuset_allocated(or_cluster* c, int32_t node, int64_t cpus);
int or_nodemetric_upsert(or_cluster* c, int32_t node, const ke_node_metric* nm, int32_t n_pm,
                         const ke_pod_metric* pm, int32_t n_agg, const ke_aggregated_usage* agg);
int or_nodemetric_delete(or_cluster* c, int32_t node);
int or_pod_assign(or_cluster* c, int32_t node, const ke_pod* pod, int64_t timestamp_ns);
int or_pod_unassign(or_cluster* c, int32_t node, int64_t uid);
int or_pods_assign(or_cluster* c, int32_t n, const int32_t* nodes, const ke_pod* pods, const int64_t* ts);
int or_node_devices_set(or_cluster* c, int32_t node, int32_t n, const ke_device* devs);
int or_node_numa_set(or_cluster* c, int32_t node, int32_t n, const ke_numa_zone* zones);
int or_node_cpus_set(or_cluster* c, int32_t node, int32_t n, const ke_cpu* cpus, int32_t max_ref);
int or_node_devices_delete(or_cluster* c, int32_t node);
/* NodeResourcesFitPlus / ScarceResourceAvoidance: the node's resources by id, and the two raw scores */
int or_node_resources_set(or_cluster* c, int32_t node, int32_t n, const ke_node_resource* res);
int64_t or_fitplus_score(const or_cluster* c, const ke_pod* pod, int32_t node);
int64_t or_sra_score(const or_cluster* c, const ke_pod* pod, int32_t node);
/* DeviceShare hints / templates / node device flags / VF ranks of the last or_schedule (ke_set_pod_device_hints,
 * ke_gpu_templates_load, ke_node_device_flags, ke_pod_allocation.vf_rank) */
int or_set_pod_device_hints(or_cluster* c, int32_t n, const ke_pod_device_hints* hints);
int or_gpu_templates_load(or_cluster* c, int32_t n, const ke_gpu_template* t);
int or_node_device_flags(or_cluster* c, int32_t node, int32_t secondary_well_planned, int32_t gpu_model_key);
int or_reservations_load(or_cluster* c, int32_t n, const ke_reservation* r);
int or_reservations_load_ex(or_cluster* c, int32_t n, const ke_reservation* r, const ke_reservation_alloc* allocs);
int or_reservations_load_full(or_cluster* c, int32_t n, const ke_reservation* r, const ke_reservation_alloc* allocs,
                              const int32_t* res_offsets, const ke_reservation_resource* res);
int or_reservation_resources_get(const or_cluster* c, int32_t r, int32_t cap, ke_reservation_resource* out, int32_t* n);
int or_reservation_allocs_get(const or_cluster* c, int32_t n, ke_reservation_alloc* out);
/* RestoreReservation's state of reservation r as a matched reservation (golden entry, oracle.c) */
typedef struct or_rsv_state {
  uint64_t allocatable_cpus[4], allocated_cpus[4], remained_cpus[4];
  int32_t numa_in; /* the reserve pod has NUMA resources (allocatable != nil) */
  int32_t pad;
  int64_t numa_allocatable[KE_MAX_NUMA * KE_NRES], numa_allocated[KE_MAX_NUMA * KE_NRES];
  int64_t numa_remained[KE_MAX_NUMA * KE_NRES];
  uint8_t numa_remained_has[KE_MAX_NUMA * KE_NRES];
  uint64_t dev_allocatable_minors, dev_allocated_minors, dev_remained_minors;
  int64_t dev_allocatable[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS];
  int64_t dev_allocated[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS];
  int64_t dev_remained[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS];
} or_rsv_state;
int or_restore_state(const or_cluster* c, int32_t r, or_rsv_state* out);
int32_t or_ds_rsv_direct(or_cluster* c, const ke_pod* pod, int32_t node, int32_t n, const int32_t* policy,
                         const int64_t* matched, const int64_t* basic, const int64_t* m_alloc, const int64_t* m_allocd,
                         int32_t mode, int32_t required, int32_t ignored, int32_t scored, uint32_t* out3,
                         int64_t* score, int32_t* reason);
int or_numa_reserve_from_rsv(or_cluster* c, const ke_pod* pod, int32_t node, const int32_t* ids, int32_t n_ids,
                             int32_t nom, int32_t required, uint64_t* cpus);
int or_numa_reserve_policy(or_cluster* c, const ke_pod* pod, int32_t node, const int32_t* ids, int32_t n_ids,
                           int32_t nom, int32_t required, uint32_t aff, int64_t* dist16, uint64_t* cpus);
int or_numa_reserve_ignored(or_cluster* c, const ke_pod* pod, int32_t node, uint64_t* cpus);
int or_reservations_get(const or_cluster* c, int32_t n, ke_reservation* out);
int or_pod_reservations(or_cluster* c, int32_t n_pods, const int32_t* offsets, const int32_t* ids);
int or_last_reservations(const or_cluster* c, int32_t n, int32_t* out);
int64_t or_reservation_score(const ke_reservation* r, const ke_pod* pod);
int32_t or_reservation_filter(or_cluster* c, const ke_pod* pod, const int32_t* ids, int32_t n_ids, int32_t node);
int32_t or_rsv_filter_with(or_cluster* c, int32_t r, const ke_pod* pod, int32_t node, const int64_t* pod_requested,
                           const int64_t* r_allocated, int32_t required, int32_t affinity);
int32_t or_reservation_prescore(or_cluster* c, const ke_pod* pod, const int32_t* ids, int32_t n_ids, int64_t* raw,
                                int32_t* nom);
int or_node_info_requested(const or_cluster* c, int32_t node, int64_t* requested, int64_t* non_zero);
int or_ds_allocate(const or_cluster* c, const ke_pod* pod, int32_t node, int32_t reserve, int32_t scored,
                   uint32_t* out3, int8_t* vf32, int32_t* reason);
int or_last_vf_ranks(const or_cluster* c, int32_t n, int8_t* out /* [n][2][KE_MAX_MINORS] */);
int or_node_gpu_partitions(or_cluster* c, int32_t node, int32_t has_table, int32_t honor, int32_t n,
                           const ke_gpu_partition* parts);

/* Per-plugin entry points for one (pod, node) pair (golden-vector tests). */
int or_la_filter(const or_cluster* c, const ke_pod* pod, int32_t node, int64_t now_ns, int* reason);
int64_t or_la_score(const or_cluster* c, const ke_pod* pod, int32_t node, int64_t now_ns);
int or_numa_filter(const or_cluster* c, const ke_pod* pod, int32_t node, int* reason);
int64_t or_numa_score(const or_cluster* c, const ke_pod* pod, int32_t node);
/* DeviceShare: PreFilter status (0 or UnschedulableAndUnresolvable) and skip; Filter; raw Score
 * (before NormalizeScore); Reserve (mutates the device cache, returns the minor mask 1<<(16*type+minor)). */
int or_ds_prefilter(const or_cluster* c, const ke_pod* pod, int* skip, int32_t* count /*[3]*/, int64_t* req /*[3][3]*/,
                    uint8_t* req_has /*[3][3]*/);
int64_t or_ds_score_device(const or_cluster* c, int32_t type, const int64_t* req, const uint8_t* req_has,
                           const int64_t* total, const uint8_t* total_has, const int64_t* free,
                           const uint8_t* free_has);
void or_normalize_scores(int64_t* scores, int32_t n);
/* topologymanager Policy.Merge over raw provider hint lists (see oracle.c). Returns admit. */
int or_topology_merge(int32_t policy, uint32_t all, int32_t n_lists, const int32_t* kinds, const int32_t* lens,
                      const uint32_t* masks, const uint8_t* preferred, const int64_t* scores, uint32_t* out_mask,
                      uint8_t* out_preferred, uint8_t* out_unsatisfied, int64_t* out_score);
int or_ds_filter(const or_cluster* c, const ke_pod* pod, int32_t node, int* reason);
int64_t or_ds_score(const or_cluster* c, const ke_pod* pod, int32_t node);
uint64_t or_ds_reserve(or_cluster* c, const ke_pod* pod, int32_t node);
int or_ds_numa_hints(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t* masks /*[255]*/, uint8_t* preferred,
                     int64_t* scores, int32_t* n, int32_t* copies, int32_t* none, int32_t* reason);
int or_ds_numa_allocate(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t affinity, int32_t* reason);
/* DefaultEstimator.EstimatePod (estimator/default_estimator.go:59-85): est[KE_NRES], -1 = key absent */
void or_estimate_pod(const or_cluster* c, const ke_pod* pod, int64_t* est);

/* NUMA golden-vector entry points (tryBestToDistributeEvenly on a forced hint; generateResourceHints) */
int or_numa_distribute(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t mask, int64_t* out16);
int or_numa_allocate(const or_cluster* c, int32_t node, const ke_pod* pod, uint32_t mask, int64_t* out16,
                     uint64_t* cpus);
void or_set_exact_cpusets(int on);
int or_numa_exclusive_ok(uint32_t mask, int32_t exclusive, const uint8_t* status, int32_t n);
int or_numa_hints(const or_cluster* c, int32_t node, const ke_pod* pod, int32_t policy, uint32_t* masks,
                  uint8_t* preferred, int64_t* scores, int32_t* counts, int32_t* present);

/* Matrix evaluation, same layout as ke_eval.  n_threads <= 0: all cores. */
int or_eval(const or_cluster* c, int32_t n_pods, const ke_pod* pods, int64_t now_ns, uint8_t* status,
            uint8_t* reason, int16_t* la_score, int16_t* numa_score, int16_t* ds_score, int16_t* total,
            int32_t* best, int n_threads);
/* Sequential scheduling, same contract as ke_schedule (mutates the oracle's state). */
int or_schedule(or_cluster* c, int32_t n_pods, const ke_pod* pods, int64_t now_ns, int32_t* chosen,
                int32_t* score, uint64_t* dev_alloc, int64_t* numa_alloc, uint64_t* cpusets, int n_threads);

/* filterNodeUsage's usage percentage, exposed for the threshold-folding property tests:
 * int64(math.Round(float64(used)/float64(total)*100)) (load_aware.go:299). */
int64_t or_usage_percent(int64_t used, int64_t total);
/* ElasticQuota (quota.c): tree load (runtime computed) and per-quota used limit / used state */
int or_quotas_load(or_cluster* c, const ke_quota_args* args, const ke_quota* q, int32_t n);
int or_quota_state(const or_cluster* c, int32_t q, int64_t* limit, uint8_t* limit_has, int64_t* used,
                   int64_t* np_used);
/* Unreserve / informer delete of one placement (same contract as ke_pod_release) */
int or_pod_release(or_cluster* c, const ke_pod* pod, const ke_pod_allocation* a, int32_t mode);
int or_debug_node_state(const or_cluster* c, int32_t node, ke_node* out, int32_t cpu_cap, ke_cpu* cpus,
                        int32_t* n_cpus, int32_t zone_cap, ke_numa_zone* zones, int32_t* n_zones, int32_t dev_cap,
                        ke_device* devs, int32_t* n_devs);

#ifdef __cplusplus
}
#endif
#endif
