/*
 * koord_eval.h — C ABI of the MI355X-native koord-scheduler Filter/Score evaluator.
 *
 * This is the drop-in boundary for koord-scheduler's per-pod Filter/Score pass of
 * LoadAwareScheduling, NodeNUMAResource (policy None, non-cpuset pods) and the framework's
 * weighted-sum + selectHost step.  A Go scheduler binds it through cgo;
 * the Python tests and bench bind it through ctypes.  No torch / HIP types cross it:
 * plain structs, pointers and sizes only.
 *
 * What each entry point replaces in the reference (paths relative to haoyann/koordinator):
 *   ke_create / ke_destroy        plugin factories  loadaware.New (pkg/scheduler/plugins/loadaware/load_aware.go:77-108),
 *                                 nodenumaresource.NewWithOptions (pkg/scheduler/plugins/nodenumaresource/plugin.go:104-172),
 *                                 registered through frameworkext.PluginFactoryProxy (pkg/scheduler/frameworkext/framework_extender_factory.go:325-343)
 *   ke_node_upsert                NodeInfo snapshot + node annotations/labels read per call
 *                                 (load_aware.go:155,160; plugin.go:408-442; estimator/default_estimator.go:124-143)
 *   ke_nodemetric_upsert/_delete  nodeMetricLister.Get (load_aware.go:132,210) — NodeMetric informer events
 *   ke_pod_assign / _unassign     podAssignCache.assign/unAssign (pkg/scheduler/plugins/loadaware/pod_assign_cache.go:89-136),
 *                                 i.e. Reserve/Unreserve (load_aware.go:192-199) and pod informer OnAdd/OnUpdate/OnDelete (:138-181)
 *   ke_node_set_requested         framework NodeInfo.Requested accounting (upstream assume/AddPod, k8s v1.28.7)
 *   ke_node_set_cpuset_allocated  resourceManager.GetAvailableCPUs allocated count (nodenumaresource/resource_manager.go:130-164)
 *   ke_eval                       per-node Filter + Score of all three plugins for a batch of pods
 *                                 (load_aware.go:122-186,201-249; nodenumaresource/plugin.go:318-406; scoring.go:66-139);
 *                                 parity mode returns the full pods x nodes status/score matrices
 *   ke_schedule                   findNodesThatFitPod + RunScorePlugins + selectHost + Reserve for a queue of pods,
 *                                 bit-exact with scheduling the pods one at a time (exact speculative batching)
 *
 * Conventions
 *   - Return 0 on success, a negative KE_ERR_* on failure; ke_last_error() is thread-local.
 *   - No pointer passed in is retained after the call returns (cgo rule).  All inputs are copied.
 *   - A context is single-writer: the caller serialises calls on one context.
 *   - Quantities are int64 in the unit the reference reads them in: cpu via Quantity.MilliValue(),
 *     every other resource via Quantity.Value() (loadaware/helper.go:147-152).  Fractional quantities
 *     must already be rounded up the way resource.Quantity does.
 *   - Times are int64 unix nanoseconds; `now` is always passed explicitly.
 *   - "absent" for an optional int64 is KE_ABSENT (-1) unless stated otherwise.
 */
#ifndef KOORD_EVAL_H
#define KOORD_EVAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KE_ABI_VERSION 13
#define KE_ABSENT (-1)

typedef struct ke_ctx ke_ctx; /* one evaluator context (ke_create) */

/* ---- error codes ---------------------------------------------------------------------------- */
#define KE_OK 0
#define KE_ERR_INVALID (-1)      /* bad argument / malformed object                              */
#define KE_ERR_UNSUPPORTED (-2)  /* object uses a feature outside the implemented hot path      */
#define KE_ERR_DEVICE (-3)       /* HIP runtime failure                                          */
#define KE_ERR_NOT_FOUND (-4)    /* node / pod index not known                                   */
#define KE_ERR_NO_DEVICE (-5)    /* evaluation requested but the HIP device/kernels are missing  */

/* ---- framework status codes: k8s.io/kubernetes/pkg/scheduler/framework Code (v1.28.7) -------- */
#define KE_CODE_SUCCESS 0
#define KE_CODE_ERROR 1
#define KE_CODE_UNSCHEDULABLE 2
#define KE_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE 3
#define KE_CODE_SKIP 5

/* ---- filter failure reasons (which plugin / which message) ---------------------------------- */
#define KE_REASON_NONE 0
#define KE_REASON_LA_NODEMETRIC_EXPIRED 1    /* "node(s) nodeMetric expired"                 load_aware.go:46  */
#define KE_REASON_LA_USAGE_CPU 2             /* "node(s) cpu usage exceed threshold"          load_aware.go:47  */
#define KE_REASON_LA_USAGE_MEMORY 3          /* "node(s) memory usage exceed threshold"                         */
#define KE_REASON_LA_AGG_USAGE_CPU 4         /* "node(s) cpu aggregated usage exceed threshold" load_aware.go:48 */
#define KE_REASON_LA_AGG_USAGE_MEMORY 5
#define KE_REASON_NUMA_INSUFFICIENT_AMPLIFIED_CPU 16 /* "Insufficient amplified cpu" nodenumaresource/plugin.go:57 */
#define KE_REASON_NUMA_INVALID_AMPLIFICATION_RATIO 17 /* "node(s) invalid CPU amplification ratio" plugin.go:56 */
#define KE_REASON_NUMA_INVALID_CPU_TOPOLOGY 18 /* "node(s) invalid CPU Topology" plugin.go:52 (GetAvailableCPUs) */
#define KE_REASON_DS_INVALID_REQUEST 32      /* PreFilter: "invalid resource device requests" / unit (deviceshare/utils.go:304-327) */
#define KE_REASON_DS_INSUFFICIENT_GPU 33     /* "Insufficient gpu devices"  (devicehandler_gpu.go:41, device_allocator.go:412) */
#define KE_REASON_DS_INSUFFICIENT_RDMA 34    /* "Insufficient rdma devices" (devicehandler_default.go:46, device_allocator.go:412) */
#define KE_REASON_DS_INSUFFICIENT_FPGA 35    /* "Insufficient fpga devices" */
/* GPUAllocator.Allocate (deviceshare/allocator_gpu.go:72-133): partition and topology-scope outcomes */
#define KE_REASON_DS_MISSING_PARTITION_TABLE 36   /* ErrNodeMissingGPUPartitionTable "node(s) missing GPU Partition Table" */
#define KE_REASON_DS_UNSUPPORTED_GPU_REQUESTS 37  /* ErrUnsupportedGPURequests "node(s) Unsupported number of GPU requests" */
#define KE_REASON_DS_INSUFFICIENT_PARTITIONED 38  /* ErrInsufficientPartitionedDevice "Insufficient Partitioned GPU Devices" */
#define KE_REASON_DS_MISSING_TOPOLOGY_TREE 39     /* ErrNodeMissingGPUDeviceTopologyTree (required scope only) */
#define KE_REASON_DS_MULTI_SHARED_GPU 40          /* ErrUnsupportedMultiSharedGPU (required scope only) */
#define KE_REASON_DS_INSUFFICIENT_TOPOLOGY_SCOPED 41 /* ErrInsufficientTopologyScopedGPUDevices */
#define KE_REASON_DS_INSUFFICIENT_GPU_TOPOLOGY 42 /* ErrInsufficientGPUDevices "Insufficient GPU Devices" (topology tree) */
#define KE_REASON_DS_INSUFFICIENT_NUMA_SCOPED 43  /* ErrInsufficientNUMAScopedDevices (topology_hint.go:32), via Admit */
#define KE_REASON_DS_INVALID_HINT 44              /* PreFilter: "invalid Selector / VFSelector of DeviceHint" (utils.go:457-482) */
#define KE_REASON_DS_INSUFFICIENT_RDMA_VF 45      /* "Insufficient rdma VirtualFunctions" (device_allocator.go:85-89) */
#define KE_REASON_DS_INSUFFICIENT_FPGA_VF 46      /* "Insufficient fpga VirtualFunctions" */
#define KE_REASON_DS_INSUFFICIENT_PRIMARY 47      /* "node(s) Insufficient primary device" (device_allocator.go:264-266) */
#define KE_REASON_DS_JOINT_VIOLATION 48           /* "node(s) Device Joint-Allocate rules violation" (:247-249) */
#define KE_REASON_DS_NO_MATCHED_TEMPLATE 49       /* ErrNoMatchedGPUSharedResourceTemplate (allocator_gpu.go:141-143, utils.go:512-514) */
/* NodeResourcesFit's Filter (upstream k8s v1.28.7 noderesources/fit.go fitsRequest): the first insufficiency in
 * fitsRequest's order (pods, cpu, memory, then the scalar resources -- ranged over a Go map there, here in ext
 * slot order) */
#define KE_REASON_FIT_TOO_MANY_PODS 64            /* "Too many pods" */
#define KE_REASON_FIT_INSUFFICIENT_CPU 65         /* "Insufficient cpu" */
#define KE_REASON_FIT_INSUFFICIENT_MEMORY 66      /* "Insufficient memory" */
#define KE_REASON_FIT_INSUFFICIENT_SCALAR 67      /* "Insufficient <resource name>" */

/* ---- resources (index into per-resource arrays) ---------------------------------------------- */
#define KE_RES_CPU 0          /* "cpu"                         MilliValue */
#define KE_RES_MEMORY 1       /* "memory"                      Value      */
#define KE_RES_BATCH_CPU 2    /* "kubernetes.io/batch-cpu"     Value      */
#define KE_RES_BATCH_MEMORY 3 /* "kubernetes.io/batch-memory"  Value      */
#define KE_RES_MID_CPU 4      /* "kubernetes.io/mid-cpu"       Value      */
#define KE_RES_MID_MEMORY 5   /* "kubernetes.io/mid-memory"    Value      */
#define KE_RES_COUNT 6
#define KE_NRES 2             /* resources the LoadAware/NUMA scorers act on: cpu, memory */

/* ---- koordinator priority / QoS classes (apis/extension/priority.go, qos.go) ----------------- */
#define KE_PRIORITY_NONE 0
#define KE_PRIORITY_PROD 1
#define KE_PRIORITY_MID 2
#define KE_PRIORITY_BATCH 3
#define KE_PRIORITY_FREE 4

#define KE_QOS_NONE 0
#define KE_QOS_LSE 1
#define KE_QOS_LSR 2
#define KE_QOS_LS 3
#define KE_QOS_BE 4
#define KE_QOS_SYSTEM 5

/* ---- NodeMetric aggregation types (apis/extension/constants.go:49-58) ------------------------ */
#define KE_AGG_NONE 0 /* "" */
#define KE_AGG_AVG 1
#define KE_AGG_P50 2
#define KE_AGG_P90 3
#define KE_AGG_P95 4
#define KE_AGG_P99 5
#define KE_AGG_TYPES 6

/* ---- scoring strategies (pkg/scheduler/apis/config/types.go:91-98) --------------------------- */
#define KE_STRATEGY_LEAST_ALLOCATED 0
#define KE_STRATEGY_MOST_ALLOCATED 1

/* A resource map restricted to cpu/memory, with key presence (ResourceList semantics) and the
 * total key count of the original map (len(ResourceList) matters in loadaware/helper.go:68,77,88). */
typedef struct ke_resource_map {
  int64_t value[KE_NRES];
  uint8_t present[KE_NRES];
  uint8_t pad[2];
  int32_t n_keys; /* len() of the original ResourceList, including keys other than cpu/memory */
} ke_resource_map; /* 24 bytes */

/* LoadAwareSchedulingArgs after v1beta3 defaulting (pkg/scheduler/apis/config/types.go:31-87,
 * v1beta3/defaults.go:89-114).  Threshold/weight/factor arrays are indexed by KE_RES_CPU/MEMORY,
 * KE_ABSENT = key absent from the map.  Keys other than cpu/memory are not supported. */
typedef struct ke_loadaware_args {
  int64_t node_metric_expiration_seconds; /* KE_ABSENT = nil                       */
  int64_t resource_weights[KE_NRES];
  int64_t usage_thresholds[KE_NRES];
  int64_t prod_usage_thresholds[KE_NRES];
  int64_t estimated_scaling_factors[KE_NRES];
  int64_t estimated_seconds_after_pod_scheduled; /* KE_ABSENT = nil */
  int64_t estimated_seconds_after_initialized;   /* KE_ABSENT = nil */
  /* Aggregated (nil when both types are KE_AGG_NONE and all thresholds absent) */
  int64_t agg_usage_thresholds[KE_NRES];
  int64_t agg_usage_duration_ns; /* 0 = "max non-empty duration" policy */
  int64_t agg_score_duration_ns;
  int32_t agg_usage_type;        /* KE_AGG_*  */
  int32_t agg_score_type;        /* KE_AGG_*  */
  uint8_t filter_expired_node_metrics;               /* *bool, default true  */
  uint8_t enable_schedule_when_node_metrics_expired; /* *bool, default false */
  uint8_t score_according_prod_usage;
  uint8_t allow_customize_estimation;
  uint8_t has_aggregated; /* args.Aggregated != nil */
  /* Some map of the args (ResourceWeights, UsageThresholds, ProdUsageThresholds, EstimatedScalingFactors,
   * Aggregated.UsageThresholds) has a key other than cpu/memory: not supported (KE_ERR_UNSUPPORTED). */
  uint8_t has_other_keys;
  uint8_t pad[2];
} ke_loadaware_args;

/* NodeNUMAResourceArgs.ScoringStrategy (types.go:114-125, v1beta3/defaults.go:118-153). */
typedef struct ke_numa_args {
  int64_t weights[KE_NRES]; /* KE_ABSENT = resource not in ScoringStrategy.Resources */
  int32_t strategy;         /* KE_STRATEGY_*                                       */
  int32_t numa_strategy;    /* NUMAScoringStrategy.Type (KE_STRATEGY_*); its weights are the node-level
                               ScoringStrategy.Resources (scoring.go:37-52, plugin.go:121-126) */
  int32_t default_cpu_bind_policy; /* DefaultCPUBindPolicy (KE_CPU_BIND_*, v1beta3 default FullPCPUs) */
  uint8_t has_other_keys;  /* ScoringStrategy.Resources names a resource other than cpu/memory (scoring.go
                              217-262 scores scalar resources too): not supported (KE_ERR_UNSUPPORTED) */
  uint8_t pad[3];
} ke_numa_args;

/* ---- cpuset binding (nodenumaresource cpu accumulator) ----------------------------------------- */
#define KE_CPU_BIND_UNSET 0 /* schedulingconfig.CPUBindPolicy: "" */
#define KE_CPU_BIND_DEFAULT 1
#define KE_CPU_BIND_FULL_PCPUS 2
#define KE_CPU_BIND_SPREAD_BY_PCPUS 3
#define KE_CPU_BIND_CONSTRAINED_BURST 4
#define KE_CPU_EXCL_NONE 0 /* CPUExclusivePolicy */
#define KE_CPU_EXCL_PCPU_LEVEL 1
#define KE_CPU_EXCL_NUMA_NODE_LEVEL 2
#define KE_NODE_CPU_BIND_NONE 0 /* node label / kubelet cpu manager policy (numa_aware.go:354-365) */
#define KE_NODE_CPU_BIND_FULL_PCPUS_ONLY 1
#define KE_NODE_CPU_BIND_SPREAD_BY_PCPUS 2
#define KE_NUMA_ALLOCATE_DEFAULT 0 /* node label node.koordinator.sh/numa-allocate-strategy */
#define KE_NUMA_ALLOCATE_MOST 1
#define KE_NUMA_ALLOCATE_LEAST 2
#define KE_MAX_CPUS 256 /* CPU ids 0..255 per node */
#define KE_REASON_NUMA_INVALID_REQUESTED_CPUS 23 /* "the requested CPUs must be integer" (plugin.go:296-298, util.go:131-134) */
#define KE_REASON_NUMA_CPU_BIND_POLICY_CONFLICT 24 /* ErrCPUBindPolicyConflict (plugin.go:365-367) */
#define KE_REASON_NUMA_SMT_ALIGNMENT 25 /* ErrSMTAlignmentError (plugin.go:369-373) */
#define KE_REASON_NUMA_INSUFFICIENT_CPUS 26 /* allocateCPUSet: "not enough cpus available to satisfy request" */
#define KE_REASON_RSV_INSUFFICIENT_CPUS 50 /* a pod with a reservation affinity whose matched reservations holding a
                                              cpuset / NUMA resources satisfy none (tryAllocateFromReservation,
                                              nodenumaresource/reservation.go:420-422: "Reservation(s) ...") */
#define KE_REASON_RSV_INSUFFICIENT_DEVICES 51 /* a DeviceShare pod with a reservation affinity whose matched
                                                 reservations holding devices satisfy none (tryAllocateFromReservation,
                                                 deviceshare/reservation.go:283-285: "Reservation(s) Insufficient ...") */
#define KE_REASON_RSV_AFFINITY 52 /* a pod with a reservation affinity on a node where none of its matched reservations
                                     fits (the Reservation plugin's Filter, reservation/plugin.go:316-318, 351-442) */
#define KE_REASON_RSV_INSUFFICIENT_NUMA 53 /* a pod with a reservation affinity under a NUMA policy whose matched
                                              reservations cannot allocate on the merged affinity: "Reservation(s)
                                              Insufficient NUMA <resource>" (nodenumaresource/reservation.go:420-422) */

/* One logical CPU of a node: CPUTopology.CPUDetails (cpu_topology.go:24-105, built from the NRT's
 * CPU topology, topology_options.go:90-164) + NodeAllocation.allocatedCPUs (node_allocation.go:33-41)
 * + TopologyOptions.ReservedCPUs. */
typedef struct ke_cpu {
  int32_t cpu_id;      /* 0 .. KE_MAX_CPUS-1 */
  int32_t core_id;     /* as the topology holds it (socket<<16 | core for NRT topologies) */
  int32_t numa_id;     /* NUMA node id */
  int32_t socket_id;
  int32_t ref_count;   /* allocatedCPUs[cpu].RefCount, 0 = not allocated */
  uint8_t exclusive;   /* allocatedCPUs[cpu].ExclusivePolicy (KE_CPU_EXCL_*) */
  uint8_t reserved;    /* in TopologyOptions.ReservedCPUs */
  uint8_t pad[2];
} ke_cpu; /* 24 bytes */

/* ---- NUMA topology (nodenumaresource + frameworkext/topologymanager) --------------------------- */
/* NUMA topology policies (apis/extension/numa_aware.go): node label / NRT kubelet topology-manager policy */
#define KE_NUMA_POLICY_NONE 0
#define KE_NUMA_POLICY_BEST_EFFORT 1
#define KE_NUMA_POLICY_RESTRICTED 2
#define KE_NUMA_POLICY_SINGLE_NUMA_NODE 3
#define KE_MAX_NUMA 8
#define KE_NUMA_EXCLUSIVE_NONE 0 /* ke_pod.numa_exclusive: unset (Required when the pod sets a policy) */
#define KE_NUMA_EXCLUSIVE_PREFERRED 1
#define KE_NUMA_EXCLUSIVE_REQUIRED 2
#define KE_NUMA_STATUS_IDLE 0   /* ke_numa_zone.numa_status: NodeAllocation.NUMANodeSharedStatus */
#define KE_NUMA_STATUS_SINGLE 1 /* only single-NUMA cpuset pods use the zone */
#define KE_NUMA_STATUS_SHARED 2 /* some cpuset pod spans several zones including this one */
#define KE_NUMA_ALLOC_ENTRY 1u  /* ke_numa_zone.has_allocated bits */
#define KE_NUMA_ALLOC_CPU 2u
#define KE_NUMA_ALLOC_MEMORY 4u
#define KE_REASON_NUMA_POLICY_CONFLICT 19 /* "node(s) NUMA Topology policy cannot match" (ErrNotMatchNUMATopology) */
#define KE_REASON_NUMA_MISSING_RESOURCES 20 /* "node(s) missing NUMA resources" (topology_hint.go:35-37) */
#define KE_REASON_NUMA_HINT_UNALIGNED 21 /* topologymanager Admit: "Unaligned NUMA Hint ..." / "Unsatisfied NUMA ..." */
#define KE_REASON_NUMA_INSUFFICIENT_RESOURCES 22 /* Allocate: "Insufficient NUMA <resource>" (resource_manager.go:307) */

/* One NUMA node of TopologyOptions.NUMANodeResources (topology_options.go:90-164; reserved CPUs already
 * removed) with the resource manager's allocation on it (node_allocation.go:33-243). */
typedef struct ke_numa_zone {
  int32_t id;                  /* NUMA node id, 0 .. KE_MAX_NUMA-1; zones ascending by id */
  uint8_t has[KE_NRES];        /* cpu / memory key present in the zone's resources */
  uint8_t has_allocated;       /* the resource manager's allocatedResources entry of the zone:
                                  KE_NUMA_ALLOC_ENTRY | KE_NUMA_ALLOC_CPU | KE_NUMA_ALLOC_MEMORY (the keys
                                  its ResourceList holds; 0 = no entry) */
  uint8_t numa_status;         /* KE_NUMA_STATUS_* (node_allocation.go:52-68), from the cpuset pods on it */
  int64_t capacity[KE_NRES];   /* cpu milli, memory bytes (before amplification) */
  int64_t allocated[KE_NRES];  /* Σ NUMANodeResources of the pods allocated on the zone */
  int32_t cpuset_cpus;         /* cpuset CPUs allocated in the zone (allocatedCPUs.CPUsInNUMANodes) */
  /* len(NodeAllocation.singleNUMANode[id]) / len(sharedNode[id]): the cpuset pods whose CPUs lie only in
   * this zone / in several zones including it.  The status is Shared when shared_pods > 0, else Single
   * when single_pods > 0, else Idle (NUMANodeSharedStatus).  Both 0 with numa_status Single / Shared
   * counts as one such pod.  A release (ke_pod_release) of a cpuset pod removes it from these sets. */
  int16_t single_pods;
  int16_t shared_pods;
} ke_numa_zone; /* 48 bytes */

/* ---- DeviceShare (pkg/scheduler/plugins/deviceshare) ------------------------------------------ */
#define KE_DEV_GPU 0  /* schedulingv1alpha1.GPU  */
#define KE_DEV_RDMA 1 /* schedulingv1alpha1.RDMA */
#define KE_DEV_FPGA 2 /* schedulingv1alpha1.FPGA */
#define KE_DEV_TYPES 3
#define KE_MAX_MINORS 16 /* device instances per type per node (minors 0..15) */
/* Resource keys of one device instance.  GPU devices use all three, RDMA/FPGA devices key 0. */
#define KE_DKEY_GPU_CORE 0         /* koordinator.sh/gpu-core          */
#define KE_DKEY_GPU_MEMORY 1       /* koordinator.sh/gpu-memory (bytes) */
#define KE_DKEY_GPU_MEMORY_RATIO 2 /* koordinator.sh/gpu-memory-ratio  */
#define KE_DKEY_RDMA 0             /* koordinator.sh/rdma              */
#define KE_DKEY_FPGA 0             /* koordinator.sh/fpga              */
#define KE_DKEYS 3
/* Pod device requests: PodRequests of the DeviceShare resource names (deviceshare/utils.go:54-69). */
#define KE_PDR_NVIDIA_GPU 0       /* nvidia.com/gpu              */
#define KE_PDR_AMD_GPU 1          /* amd.com/gpu                 */
#define KE_PDR_KOORD_GPU 2        /* koordinator.sh/gpu          */
#define KE_PDR_GPU_SHARED 3       /* koordinator.sh/gpu.shared   */
#define KE_PDR_GPU_CORE 4         /* koordinator.sh/gpu-core     */
#define KE_PDR_GPU_MEMORY 5       /* koordinator.sh/gpu-memory   */
#define KE_PDR_GPU_MEMORY_RATIO 6 /* koordinator.sh/gpu-memory-ratio */
#define KE_PDR_RDMA 7             /* koordinator.sh/rdma         */
#define KE_PDR_FPGA 8             /* koordinator.sh/fpga         */
#define KE_PDR_HYGON_DCU 9        /* dcu.com/gpu (a GPU: ConvertDeviceRequest's x100, utils.go:206-212) */
#define KE_PDR_COUNT 10
/* DeviceShareArgs.ScoringStrategy (types.go:263-275, v1beta3/defaults.go:218-242): weights indexed
 * gpu-memory-ratio, gpu-memory, rdma, fpga; KE_ABSENT = not in Resources. */
#define KE_DSW_GPU_MEMORY_RATIO 0
#define KE_DSW_GPU_MEMORY 1
#define KE_DSW_RDMA 2
#define KE_DSW_FPGA 3
/* KE_DKEY_* bits of DeviceShareArgs.GPUSharedResourceTemplatesMatchedResources (types.go:277-283) */
#define KE_TEMPLATE_KEY_CORE 1u
#define KE_TEMPLATE_KEY_MEMORY 2u
#define KE_TEMPLATE_KEY_MEMORY_RATIO 4u
typedef struct ke_deviceshare_args {
  int64_t weights[4];
  int32_t strategy; /* KE_STRATEGY_* */
  /* GPUSharedResourceTemplatesMatchedResources restricted to the GPU keys (KE_TEMPLATE_KEY_*): a shared-GPU
   * pod whose per-GPU request names one of them would be allocated by template (allocator_gpu.go:135-159,
   * utils.go:508-515), which is not implemented: ke_eval / ke_schedule return KE_ERR_UNSUPPORTED for it. */
  uint8_t template_matched_keys;
  uint8_t has_other_keys; /* ScoringStrategy.Resources names a resource outside KE_DSW_*: not supported */
  uint8_t disable_numa_alignment; /* DisableDeviceNUMATopologyAlignment (types.go:271-272): no device NUMA
                                     hints, no device Allocate in Admit, Reserve ignores the affinity */
  uint8_t pad;
} ke_deviceshare_args;

/* ---- labels and label selectors (DeviceShare hints: apis/extension/device_share.go:151-195) ---------
 * Label keys and values are ids of one process-wide string table (ke_label_id; 0 = no string), so a label
 * set is KE_MAX_LABELS (key, value) id pairs and a selector is metav1.LabelSelector after
 * LabelSelectorAsSelector (util.GetFastLabelSelector, pkg/util/selector.go:24-32): every matchLabels entry is
 * an In requirement with one value; a present selector without requirements matches everything. */
#define KE_MAX_LABELS 8
#define KE_MAX_SEL_REQS 4
#define KE_MAX_SEL_VALUES 4
int32_t ke_label_id(const char* s); /* intern (stable for the process); NULL / "" -> 0 */
typedef struct ke_labels {
  int32_t n;
  int32_t key[KE_MAX_LABELS];
  int32_t value[KE_MAX_LABELS];
} ke_labels; /* 68 bytes */
#define KE_SEL_IN 0             /* also matchLabels k: v */
#define KE_SEL_NOT_IN 1         /* key absent, or its value not listed */
#define KE_SEL_EXISTS 2
#define KE_SEL_DOES_NOT_EXIST 3
typedef struct ke_label_requirement {
  int32_t key;
  int32_t op; /* KE_SEL_* */
  int32_t n_values;
  int32_t values[KE_MAX_SEL_VALUES];
} ke_label_requirement; /* 28 bytes */
typedef struct ke_label_selector {
  int32_t present; /* the *metav1.LabelSelector is not nil */
  int32_t n;
  ke_label_requirement req[KE_MAX_SEL_REQS];
} ke_label_selector; /* 120 bytes */

/* A device's SR-IOV virtual function group (DeviceInfo.VFGroups, apis/scheduling/v1alpha1/device_types.go):
 * its labels and its VFs as a mask over the device's VF ranks (rank r = the r-th VF of the device in BusID
 * string order over all its groups; at most 64 VFs per device). */
#define KE_MAX_VF_GROUPS 4
typedef struct ke_vf_group {
  ke_labels labels;
  int32_t pad;
  uint64_t vfs;
} ke_vf_group; /* 80 bytes */

/* One device instance as koord-scheduler's nodeDeviceCache holds it (device_cache.go:518-568):
 * `total` = DeviceInfo.Resources (left empty by the cache when !Health), `used` = Σ allocations of
 * the pods already on it (updateCacheUsed).  has_* mark the keys present in each ResourceList. */
typedef struct ke_device {
  int32_t type;  /* KE_DEV_* */
  int32_t minor; /* DeviceInfo.Minor, 0 .. KE_MAX_MINORS-1 */
  uint8_t health;
  uint8_t has_total[KE_DKEYS];
  uint8_t has_used[KE_DKEYS];
  uint8_t has_topology; /* DeviceInfo.Topology != nil */
  int64_t total[KE_DKEYS];
  int64_t used[KE_DKEYS];
  /* DeviceInfo.Topology: NodeID (-1 .. KE_MAX_NUMA-1), and the rank of PCIEID among the node's distinct PCIEID
   * strings in Go string order (0 = smallest).  GetGPUTopologyScope (allocator_gpu_helper.go:202-263) builds
   * the GPU scope tree Node > NUMANode (by NodeID) > PCIe (by PCIEID) from them when every GPU device has a
   * topology; DeviceShare's NUMA hints (topology_hint.go) group the devices by NodeID (-1: any NUMA node). */
  int32_t numa_node;
  int32_t pcie_rank;
  ke_labels labels;          /* DeviceInfo.Labels (Selector / ApplyForAll matching)                        */
  int32_t n_vf_groups;       /* DeviceInfo.VFGroups (hasVirtualFunctions, allocateVF); RDMA / FPGA only     */
  ke_vf_group vf_groups[KE_MAX_VF_GROUPS];
  uint64_t vf_allocated;     /* VF ranks held by pods on the node (nodeDevice.vfAllocations[type][minor])   */
} ke_device; /* 472 bytes */

/* One GPUPartition of a node's GPUPartitionTable (apis/extension/device_share.go:196-226): the table is the
 * Device annotation scheduling.koordinator.sh/gpu-partitions, or, when the Device has none, the designated
 * table of the node's GPU model (GetDesignatedGPUPartitionIndexer, allocator_gpu_helper.go:146-162). */
typedef struct ke_gpu_partition {
  uint32_t minors;          /* bit m = minor m (Minors; minors 0 .. KE_MAX_MINORS-1, non-empty)          */
  int32_t number_of_gpus;   /* the table key the partition is listed under                               */
  int32_t allocation_score; /* AllocationScore                                                           */
  int32_t pad;
  int64_t ring_bus_bandwidth; /* RingBusBandwidth.Value(), KE_ABSENT = nil                               */
} ke_gpu_partition; /* 24 bytes */
#define KE_MAX_GPU_PARTITIONS 64 /* partitions per node table */

/* ---- NodeResourcesFitPlus / ScarceResourceAvoidance -------------------------
 * Two Score plugins without Filter or NormalizeScore, fused into the same per-(pod, node) pass:
 *  - NodeResourcesFitPlus (pkg/scheduler/plugins/noderesourcefitplus/node_resources_fit_plus.go:75-93,
 *    node_resource_fit_plus_utils.go:35-89): over the pod's requested resources (PodRequests > 0) that the
 *    args name, Σ weight·{least,most}RequestedScore(NodeInfo (NonZero)Requested + pod request, Allocatable)
 *    / Σ weight, MaxNodeScore when the weight sum is 0;
 *  - ScarceResourceAvoidance (scarceresourceavoidance/scarce_resource_avoidance.go:70-160): diff = the node's
 *    allocatable resource names (> 0) minus the pod's requested names, n = |diff ∩ args.Resources|:
 *    MaxNodeScore when diff or n is empty, else (|diff| - n)·100/|diff|.
 * Resource names are interned by the caller into ids 0 .. KE_MAX_XRES-1 (one table per context, every name
 * a node advertises must have an id); cpu and memory have fixed ids.  Plugin weight 0 = not in the profile. */
#define KE_MAX_XRES 64
#define KE_XRES_CPU 0
#define KE_XRES_MEMORY 1
#define KE_MAX_FITPLUS 4 /* NodeResourcesFitPlusArgs.Resources entries */
#define KE_MAX_POD_XRES 8 /* ke_pod.xres_id / xres_value entries */
typedef struct ke_fitplus_resource {
  int32_t id;     /* resource id */
  int32_t type;   /* KE_STRATEGY_* (ResourcesType.Type: LeastAllocated / MostAllocated) */
  int64_t weight; /* ResourcesType.Weight, >= 0 */
} ke_fitplus_resource; /* 16 bytes */
typedef struct ke_ext_args {
  int64_t weight_fitplus;      /* profile Score weight of NodeResourcesFitPlus (0 = disabled) */
  int64_t weight_sra;          /* profile Score weight of ScarceResourceAvoidance (0 = disabled) */
  uint64_t sra_resources;      /* ScarceResourceAvoidanceArgs.Resources as a mask of resource ids */
  int32_t n_fitplus;           /* entries of NodeResourcesFitPlusArgs.Resources (distinct ids) */
  int32_t pad;
  ke_fitplus_resource fitplus[KE_MAX_FITPLUS];
} ke_ext_args; /* 96 bytes */

/* ---- NodeResourcesFit (upstream kube-scheduler v1.28.7 pkg/scheduler/framework/plugins/noderesources: fit.go,
 * resource_allocation.go, least_allocated.go, most_allocated.go -- not in the reference tree, go.mod:60; restated
 * from the published algorithm, parity unpinned).  The shipped profile runs it by default with LeastAllocated over
 * cpu, memory, kubernetes.io/batch-cpu and kubernetes.io/batch-memory at weight 1 (config/manager/
 * scheduler-config.yaml:17-31):
 *  - Filter (fitsRequest), before every koordinator Filter (default plugins precede the profile's): len(Pods) + 1 >
 *    AllowedPodNumber fails; a pod requesting nothing passes; else cpu / memory requests > 0 above Allocatable -
 *    Requested fail, and so does a scalar request above Allocatable - Requested of its resource.
 *  - Score: per configured resource, alloc / req = calculateResourceAllocatableRequest (cpu / memory: Allocatable,
 *    NonZeroRequested + the pod's request with the 100m / 200Mi container defaults; a scalar the pod does not
 *    request is skipped, else Allocatable, Requested + request), resources with alloc 0 skipped, then
 *    Σ weight·{least,most}RequestedScore / Σ weight (0 when no weight counts).
 * Resource ids as for NodeResourcesFitPlus; cpu / memory come from ke_node (Allocatable, Requested) and from the
 * node's ke_node_resources_set rows (NonZeroRequested), scalars from those rows, the pod's requests from ke_pod.requests
 * (cpu / memory) and ke_pod.xres (scalars; cpu / memory with the defaults for the Score).  Every scalar a pod may
 * request must be listed in `scalars` (a pod listing another scalar id with a non-zero value is refused). */
typedef struct ke_fit_args {
  int64_t weight;          /* profile Score weight (0 = the Score is not in the profile) */
  int32_t strategy;        /* ScoringStrategy.Type: KE_STRATEGY_LEAST_ALLOCATED / MOST_ALLOCATED */
  int32_t n_resources;     /* ScoringStrategy.Resources (<= KE_MAX_FITPLUS; the type field of an entry is unused) */
  ke_fitplus_resource resources[KE_MAX_FITPLUS];
  int32_t n_scalars;       /* scalar resource ids (not cpu / memory) the Filter checks, <= 8 */
  int32_t scalars[8];
  uint8_t filter;          /* the Filter is in the profile */
  uint8_t has_ignored;     /* IgnoredResources / IgnoredResourceGroups set, or RequestedToCapacityRatio:
                              KE_ERR_UNSUPPORTED */
  uint8_t pad[2];
} ke_fit_args; /* 120 bytes */
/* The ext slots NodeResourcesFitPlus and NodeResourcesFit read (their resources and the Filter's scalars,
 * FitPlus's first) are at most 8 distinct ids (KE_ERR_UNSUPPORTED beyond). */

/* Framework profile: score plugin weights (config/manager/scheduler-config.yaml:85-94). */
typedef struct ke_config {
  int32_t abi_version;    /* must be KE_ABI_VERSION                                      */
  int32_t device_ordinal; /* HIP device used by this context (one process per GPU)      */
  int64_t weight_loadaware;
  int64_t weight_numa;
  int64_t weight_deviceshare;
  ke_loadaware_args loadaware;
  ke_numa_args numa;
  ke_deviceshare_args deviceshare;
  int32_t node_capacity;  /* max nodes this context will hold (device SoA is sized once), <= 2^22 - 1 */
  int32_t pod_batch;      /* B: pods evaluated per speculative batch in ke_schedule      */
  int32_t global_node_offset; /* first global node index held by this shard (multi-GPU)  */
  int32_t weight_reservation; /* profile Score weight of the Reservation plugin (scheduler-config.yaml:91-92:
                                 5000), 0 .. 2^20; scores only pods with matched reservations (ke_pod_reservations) */
  ke_ext_args ext;        /* NodeResourcesFitPlus / ScarceResourceAvoidance (all zero = disabled) */
  ke_fit_args fit;        /* NodeResourcesFit (all zero = not in the profile) */
} ke_config;

/* A Node object (+ the NodeInfo aggregates the framework keeps for it). */
typedef struct ke_node {
  int64_t allocatable[KE_NRES];      /* node.Status.Allocatable == NodeInfo.Allocatable           */
  int64_t raw_allocatable[KE_NRES];  /* annotation node.koordinator.sh/raw-allocatable, KE_ABSENT per key */
  int64_t requested[KE_NRES];        /* NodeInfo.Requested (MilliCPU, Memory)                    */
  double cpu_amplification_ratio;    /* annotation resource-amplification-ratio["cpu"]; -1 = not set */
  int64_t cpuset_allocated_cpus;     /* CPUs held by cpuset pods (resourceManager allocated count)  */
  /* annotation scheduling.koordinator.sh/usage-thresholds (apis/extension/load_aware.go:30-72) */
  int64_t custom_usage_thresholds[KE_NRES];      /* KE_ABSENT per key */
  int64_t custom_prod_usage_thresholds[KE_NRES]; /* KE_ABSENT per key */
  int64_t custom_agg_thresholds[KE_NRES];        /* KE_ABSENT per key */
  int64_t custom_agg_duration_ns;                /* 0 = nil / zero    */
  /* TopologyOptions.AmplificationRatios["cpu"] as reported on the NodeResourceTopology
   * (topology_options.go:150-162); Score prefers it over the node annotation (util.go:78-87).
   * -2 = the NRT carries no ratio map (Score then reads the node annotation). */
  double nrt_cpu_amplification_ratio;
  int32_t custom_agg_type;                       /* KE_AGG_*           */
  int32_t numa_topology_policy;    /* KE_NUMA_POLICY_*: getNUMATopologyPolicy (label, else NRT policy) */
  int32_t cpu_bind_policy;         /* KE_NODE_CPU_BIND_*: GetNodeCPUBindPolicy (label, else kubelet policy) */
  uint8_t has_custom_thresholds;   /* annotation present and valid JSON  */
  uint8_t custom_thresholds_error; /* annotation present but failed to unmarshal (helper.go:110) */
  uint8_t has_custom_agg;          /* AggregatedUsage != nil in the annotation */
  uint8_t amplification_error;     /* ratio annotation failed to unmarshal (plugin.go:421) */
  uint8_t cpu_topology_invalid;    /* TopologyOptions.CPUTopology set but !IsValid() (resource_manager.go:502-504) */
  uint8_t numa_allocate_strategy;  /* KE_NUMA_ALLOCATE_* (label overriding the args' NUMA allocate strategy) */
  uint8_t pad[6];
  int32_t allowed_pods;            /* NodeInfo.Allocatable.AllowedPodNumber (status.allocatable pods) */
  int32_t pod_count;               /* len(NodeInfo.Pods), reserve pods included; ke_schedule adds each placed pod */
} ke_node;

/* One AggregatedUsage entry of NodeMetric.Status.NodeMetric.AggregatedNodeUsages. */
typedef struct ke_aggregated_usage {
  int64_t duration_ns;
  ke_resource_map usage[KE_AGG_TYPES]; /* indexed by KE_AGG_*; n_keys == 0 means absent */
} ke_aggregated_usage;

/* One PodMetricInfo of NodeMetric.Status.PodsMetric. */
typedef struct ke_pod_metric {
  int64_t pod_key; /* interned namespace/name */
  int32_t priority_class; /* PodMetricInfo.Priority as KE_PRIORITY_* */
  int32_t pad;
  ke_resource_map usage;
} ke_pod_metric;

/* NodeMetric header (slo/v1alpha1 nodemetric_types.go:38-136).  Pod metrics and aggregated usages
 * are passed as separate arrays to ke_nodemetric_upsert. */
typedef struct ke_node_metric {
  int64_t update_time_ns;           /* valid if has_update_time */
  int64_t report_interval_seconds;  /* Spec.CollectPolicy.ReportIntervalSeconds, KE_ABSENT = nil */
  ke_resource_map node_usage;       /* Status.NodeMetric.NodeUsage */
  uint8_t has_update_time;
  uint8_t has_node_metric;          /* Status.NodeMetric != nil */
  uint8_t pad[6];
} ke_node_metric;

/* A pod as the plugins see it.  Classes are resolved by the caller with the reference helpers
 * GetPodPriorityClassWithDefault / GetPodQoSClassRaw (apis/extension/priority_utils.go:37-44,
 * qos_utils.go:57-62); requests/limits are resourceapi.PodRequests/PodLimits. */
typedef struct ke_pod {
  int64_t pod_key; /* interned namespace/name (matches ke_pod_metric.pod_key) */
  int64_t uid;
  int64_t requests[KE_RES_COUNT];
  int64_t limits[KE_RES_COUNT];
  int64_t custom_scaling_factors[KE_NRES];      /* annotation load-estimated-scaling-factors, KE_ABSENT per key */
  int64_t custom_seconds_after_scheduled;       /* KE_ABSENT = not set / unparsable */
  int64_t custom_seconds_after_initialized;     /* KE_ABSENT */
  int64_t scheduled_transition_ns;              /* PodScheduled=True LastTransitionTime, valid if has_scheduled */
  int64_t initialized_transition_ns;            /* Initialized=True LastTransitionTime, valid if has_initialized */
  int32_t priority_class; /* KE_PRIORITY_* (with default)  */
  int32_t qos_class;      /* KE_QOS_* (raw label)          */
  uint8_t is_daemonset;   /* an OwnerReference of Kind DaemonSet */
  uint8_t has_custom_scaling_factors; /* annotation parsed into a non-empty map */
  uint8_t has_scheduled;
  uint8_t has_initialized;
  uint8_t is_terminated;
  uint8_t has_resource_spec;          /* ResourceSpec annotation that failed to unmarshal (PreFilter Error) */
  uint8_t has_other_requests;         /* PodRequests has a non-zero resource outside KE_RES_*: 1 = each such name
                                         has a resource id (its request is a ke_pod.xres entry), 2 = some has none */
  uint8_t has_unsupported_device_requests; /* Huawei NPU device resources: unsupported */
  int64_t device_requests[KE_PDR_COUNT]; /* PodRequests of the device resources (Value()), 0 = absent */
  int32_t numa_topology_policy; /* NUMATopologySpec annotation: KE_NUMA_POLICY_* (NONE = unset) */
  int32_t numa_exclusive;       /* NUMATopologySpec.SingleNUMANodeExclusive: KE_NUMA_EXCLUSIVE_* */
  /* ResourceSpec annotation (apis/extension/resource.go): KE_CPU_BIND_* / KE_CPU_EXCL_* */
  int32_t cpu_bind_required;
  int32_t cpu_bind_preferred;
  int32_t cpu_exclusive;
  /* ElasticQuota (elasticquota/plugin_helper.go:64-82 getPodAssociateQuotaNameAndTreeID): 0 = no quota
   * (PreFilter Skip), else 1 + the index of the pod's quota in the last ke_quotas_load table. */
  int16_t quota;
  uint8_t quota_non_preemptible; /* extension.IsPodNonPreemptible (label preemptible=false) */
  uint8_t reservation_matched;   /* KE_RSV_*: how BeforePreFilter's matchedOrIgnored sets of this pod come about
                                    (transformer.go:93-145); KE_RSV_MATCHED pods list theirs with ke_pod_reservations */
  /* DeviceShare allocation annotations (apis/extension/device_share.go; parsed by utils.go:355-513) */
  int64_t gpu_ring_bus_bandwidth;      /* GPUPartitionSpec.RingBusBandwidth.Value(), KE_ABSENT = nil       */
  int32_t gpu_required_topology_scope; /* DeviceAllocateHints[gpu].RequiredTopologyScope: KE_SCOPE_*       */
  uint8_t gpu_partition_spec;          /* annotation GPUPartitionSpec present (honorGPUPartition)         */
  uint8_t gpu_partition_restricted;    /* GPUPartitionSpec.AllocatePolicy == Restricted                   */
  uint8_t device_joint_allocate;       /* DeviceJointAllocate annotation present (informational; the modelled
                                          joint allocation is ke_pod_device_hints.joint_*) */
  uint8_t device_hints;                /* KE_DHINT_* bits of DeviceAllocateHints this evaluator does not model */
  /* NodeResourcesFitPlus / ScarceResourceAvoidance PreScore (computePodResourceRequest): the resource ids
   * whose PodRequests value is > 0 (fitsPodRequestName / fitsRequest, scarce_resource_avoidance.go:109-150),
   * and per id calculatePodResourceRequest (node_resource_fit_plus_utils.go:138-203: containers' requests
   * with the 100m cpu / 200Mi memory defaults for a container without one, init containers' max); ids
   * not listed count 0.  Only the ids of NodeResourcesFitPlusArgs.Resources are read. */
  uint64_t xres_request_mask;
  int32_t n_xres;
  int32_t xres_id[KE_MAX_POD_XRES];
  int32_t device_hint; /* 1 + index into the ke_set_pod_device_hints table, 0 = no hints / joint allocation */
  int64_t xres_value[KE_MAX_POD_XRES];
} ke_pod;

/* DeviceAllocateHints[type] (apis/extension/device_share.go:151-195) + DeviceJointAllocate (:135-147) of one pod,
 * as parsePodDeviceShareExtensions reads them (deviceshare/utils.go:414-482).  Passed apart from ke_pod (most
 * pods have none): ke_set_pod_device_hints stores a table, ke_pod.device_hint = 1 + an index into it. */
#define KE_DSTRATEGY_NONE 0
#define KE_DSTRATEGY_APPLY_FOR_ALL 1     /* desired count = the node's devices of the type (matching the Selector) */
#define KE_DSTRATEGY_REQUESTS_AS_COUNT 2 /* desired count = the request, 1 (100 with DeviceLevel) per instance */
#define KE_DEXCL_NONE 0
#define KE_DEXCL_DEVICE_LEVEL 1          /* RequestsAsCount asks 100 per instance (devicehandler_default.go:84-86) */
#define KE_DEXCL_PCIE_LEVEL 2            /* nodeDevice.filter's PCIe intersection, whose result the reference
                                            discards (device_cache.go:382-385): no effect */
typedef struct ke_device_hint {
  ke_label_selector selector;    /* Selector: filterNodeDevice keeps the matching devices (device_allocator.go:140-169) */
  ke_label_selector vf_selector; /* VFSelector: mustAllocateVF, allocateVF over matching VF groups (:396-455)   */
  int32_t strategy;  /* KE_DSTRATEGY_* (DefaultDeviceHandler; the GPU handler ignores it) */
  int32_t exclusive; /* KE_DEXCL_* */
} ke_device_hint; /* 248 bytes */
typedef struct ke_pod_device_hints {
  ke_device_hint hint[KE_DEV_TYPES];
  int32_t invalid;        /* a Selector / VFSelector LabelSelectorAsSelector rejects: PreFilter UnschedulableAndUnresolvable */
  int32_t has_selectors;  /* state.hasSelectors: some hint of any device type has a Selector (utils.go:446-452) */
  /* DeviceJointAllocate.DeviceTypes after parsePodDeviceShareExtensions: the requested, non-ApplyForAll types in
   * annotation order (joint_n = 0: no joint allocation); RequiredScope SamePCIe */
  int32_t joint_n;
  int32_t joint_types[KE_DEV_TYPES];
  int32_t joint_same_pcie;
  int32_t pad;
} ke_pod_device_hints; /* 768 bytes */
/* The hint table ke_pod.device_hint indexes for the following ke_eval / ke_schedule / ke_pod_release calls
 * (copied; replaces the previous table). */
int ke_set_pod_device_hints(ke_ctx* ctx, int32_t n, const ke_pod_device_hints* hints);

/* GPU shared resource templates (GPUSharedResourceTemplates ConfigMap, gpu_shared_resource_templates_cache.go):
 * per node GPU model key (node labels gpu vendor / model -> "<vendor>-<model>", an id of ke_label_id) the named
 * per-GPU resource lists.  A shared-GPU pod whose per-GPU request names a key of
 * ke_deviceshare_args.template_matched_keys is allocated by template (allocateByTemplate, allocator_gpu.go:135-159). */
typedef struct ke_gpu_template {
  int32_t model_key; /* ke_label_id("<vendor>-<model>") */
  int32_t name;      /* ke_label_id(template name) */
  uint8_t has[KE_DKEYS];
  uint8_t pad[5];
  int64_t value[KE_DKEYS]; /* gpu-core, gpu-memory, gpu-memory-ratio (KE_DKEY_*) */
} ke_gpu_template; /* 40 bytes */
int ke_gpu_templates_load(ke_ctx* ctx, int32_t n, const ke_gpu_template* templates);
/* The node's device-level labels the allocator reads: secondaryDeviceWellPlanned (Device label,
 * apis/extension IsSecondaryDeviceWellPlanned) and the GPU template key of the node (0 = none). */
int ke_node_device_flags(ke_ctx* ctx, int32_t node, int32_t secondary_well_planned, int32_t gpu_model_key);

/* ke_pod.gpu_required_topology_scope: apiext.DeviceTopologyScope and its DeviceTopologyScopeLevel */
#define KE_SCOPE_NONE 0     /* ""                                                  */
#define KE_SCOPE_NODE 1     /* "Node"      level 1                                 */
#define KE_SCOPE_NUMA 2     /* "NUMANode"  level 2                                 */
#define KE_SCOPE_PCIE 3     /* "PCIe"      level 3                                 */
#define KE_SCOPE_DEVICE 4   /* "Device"    level 4                                 */
#define KE_SCOPE_UNKNOWN 5  /* any other non-empty string: required, level 0       */
/* ke_pod.device_hints: parts of the DeviceAllocateHints annotation outside the modelled path -> KE_ERR_UNSUPPORTED */
#define KE_DHINT_GPU_VF 2u          /* DeviceHint.VFSelector on the gpu type (defaultAllocateDevices' VF path for GPUs) */

/* One candidate of a pod's speculative top-k list (device order: best first). */
typedef struct ke_candidate {
  int32_t node;  /* node index, -1 = none */
  int32_t score; /* framework total score */
} ke_candidate;


/* ---- lifecycle ------------------------------------------------------------------------------- */
int ke_create(const ke_config* cfg, ke_ctx** out);
void ke_destroy(ke_ctx* ctx);
const char* ke_last_error(void);
int ke_abi_version(void);
/* sizeof() of ke_config, ke_node, ke_node_metric, ke_pod_metric, ke_aggregated_usage, ke_pod,
 * ke_resource_map, ke_loadaware_args, ke_numa_args, ke_deviceshare_args, ke_device, ke_numa_zone, ke_cpu,
 * ke_quota_args, ke_quota, ke_gpu_partition, ke_ext_args, ke_node_resource, ke_pod_allocation, ke_pod_device_hints,
 * ke_gpu_template, ke_reservation, ke_reservation_alloc, ke_reservation_resource (in that order) for binding-layout checks. */
int ke_abi_struct_sizes(int32_t* sizes, int32_t n);
/* 1 if this build has a usable HIP device and its gfx950 kernels loaded, else 0. */
int ke_device_available(void);

/* ---- state ingestion (informer events) ------------------------------------------------------- */
/* Insert or replace node `node` (0 <= node < node_capacity).  Keeps its NodeMetric / assigned pods. */
int ke_node_upsert(ke_ctx* ctx, int32_t node, const ke_node* n);
/* Node informer delete (the scheduler cache's RemoveNode, k8s v1.28.7): the node leaves the snapshot, so no
 * pod is evaluated against it (ke_eval reports KE_CODE_ERROR for it, ke_schedule never chooses it).  The state of
 * the other informers stays until their own events remove it — as the scheduler's caches keep it: the NodeMetric
 * (ke_nodemetric_delete), the podAssignCache (ke_pod_unassign / ke_pod_release), NodeInfo.Requested of pods still
 * bound there, the NRT topology (ke_node_topology_delete), the device cache (ke_node_devices_delete), the
 * node's reservations (ke_reservations_load).  ke_node_upsert brings the node back with that state. */
int ke_node_delete(ke_ctx* ctx, int32_t node);
/* NodeResourceTopology informer delete (topology_eventhandler.go:82-99 -> TopologyOptionsManager.Delete): the
 * node's TopologyOptions go away — no NUMA zones, no CPU topology (GetAvailableCPUs then sees no allocated CPUs),
 * no NRT amplification ratios (nrt_cpu_amplification_ratio -2).  Node fields the caller derived from the NRT
 * (kubelet topology / CPU manager policies without node labels) are the caller's to re-upsert. */
int ke_node_topology_delete(ke_ctx* ctx, int32_t node);
/* Bulk load nodes [0, n): equivalent to n ke_node_upsert calls (initial informer list). */
int ke_nodes_load(ke_ctx* ctx, int32_t n, const ke_node* nodes);
int ke_node_set_requested(ke_ctx* ctx, int32_t node, int64_t milli_cpu, int64_t memory);
int ke_node_set_cpuset_allocated(ke_ctx* ctx, int32_t node, int64_t cpus);
/* Replace the NodeMetric of `node` (lister Get succeeds afterwards). */
int ke_nodemetric_upsert(ke_ctx* ctx, int32_t node, const ke_node_metric* nm,
                         int32_t n_pod_metrics, const ke_pod_metric* pod_metrics,
                         int32_t n_aggregated, const ke_aggregated_usage* aggregated);
/* Bulk NodeMetric load for nodes [0,n): pod metrics / aggregated usages are flattened, node i owns
 * pod_metrics[pm_offsets[i] .. pm_offsets[i+1]) (offsets have n+1 entries). */
int ke_nodemetrics_load(ke_ctx* ctx, int32_t n, const ke_node_metric* nms,
                        const int64_t* pm_offsets, const ke_pod_metric* pod_metrics,
                        const int64_t* agg_offsets, const ke_aggregated_usage* aggregated);
int ke_nodemetric_delete(ke_ctx* ctx, int32_t node); /* lister Get -> NotFound */
/* podAssignCache.assign(nodeName, pod): `timestamp_ns` is used when the pod has no PodScheduled
 * condition (pod_assign_cache.go:99-122, timeNowFn fallback). */
int ke_pod_assign(ke_ctx* ctx, int32_t node, const ke_pod* pod, int64_t timestamp_ns);
int ke_pod_unassign(ke_ctx* ctx, int32_t node, int64_t uid);
/* Bulk podAssignCache.assign for the initial informer list: pod i goes to nodes[i]. */
int ke_pods_assign(ke_ctx* ctx, int32_t n, const int32_t* nodes, const ke_pod* pods, const int64_t* timestamps_ns);

/* DefaultEstimator.EstimatePod (loadaware/estimator/default_estimator.go:59-122) under this
 * context's args: est[KE_NRES] (cpu milli, memory bytes), KE_ABSENT for a resource without weight. */
int ke_estimate_pod(ke_ctx* ctx, const ke_pod* pod, int64_t* est);

/* DeviceShare node device cache (Device CRD informer, device_cache.go:518-568): replace the devices of
 * `node` (n may be 0: a cache entry without devices).  At most KE_MAX_MINORS devices per type. */
int ke_node_devices_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_device* devices);
/* NodeInfo.Allocatable / Requested of the node by resource id for NodeResourcesFitPlus and
 * ScarceResourceAvoidance (replaces the node's table; n = 0: none).  `requested` is what
 * calculateResourceAllocatableRequest reads (node_resource_fit_plus_utils.go:110-133): NonZeroRequested
 * for cpu / memory, Requested for every other resource.  Every resource the node advertises (allocatable
 * > 0, "pods" excluded: framework.Resource keeps it apart) must be listed for ScarceResourceAvoidance.
 * ke_schedule adds each placed pod's xres_value to its node's requested. */
typedef struct ke_node_resource {
  int32_t id;
  int32_t pad;
  int64_t allocatable;
  int64_t requested;
} ke_node_resource; /* 24 bytes */
int ke_node_resources_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_node_resource* res);
/* The node's current table (after the Reserves of past ke_schedule calls): up to cap entries, *n = count. */
int ke_node_resources_get(ke_ctx* ctx, int32_t node, int32_t cap, ke_node_resource* res, int32_t* n);
/* Drop the node's cache entry (getNodeDevice == nil: DeviceShare Filter passes, Score is 0). */
int ke_node_devices_delete(ke_ctx* ctx, int32_t node);

/* ---- Reservations (pkg/scheduler/plugins/reservation) -----------------------
 * The reservation cache as the scheduler's BeforePreFilter reads it (reservation/cache.go,
 * transformer.go:147-300).  Every pod sees each node's NodeInfo restored: a reservation that is available
 * (IsAvailable, no ParseError), not (AllocateOnce with allocated pods), has allocated pods and is not
 * matched by the pod gives back the part its owner pods already hold twice (restoreUnmatchedReservations,
 * transformer.go:447-473): Requested -= allocatable, += SubtractWithNonNegativeResult(allocatable, allocated),
 * NonZeroRequested likewise with the 100m / 200Mi defaults of a zero request.  `NodeInfo.Requested` passed
 * with ke_node_upsert / ke_node_set_requested (and the cpu / memory rows of ke_node_resources_set) must
 * include the reserve pods' requests, as the scheduler's NodeInfo does.  The restored values feed every
 * plugin that reads NodeInfo: NodeNUMAResource's amplified-cpu Filter and Score, NodeResourcesFitPlus.
 * Pods that match reservations take the nominated-reservation path below (ke_pod_reservations).
 * What a reservation's reserve pod holds beyond NodeInfo — a NUMA allocation or a cpuset in the resource manager
 * (nodenumaresource/reservation.go:185-259), device instances in the device cache (deviceshare/reservation.go:
 * 136-195) — comes with ke_reservations_load_ex (ke_reservation_alloc); `holds` states which (the records decide).
 * Allocatable names other than cpu / memory (pods, ephemeral storage, device resources, scalars) come with
 * ke_reservations_load_full as resource entries (ke_reservation_resource) by resource id (the context's
 * ke_ext_args id space, KE_MAX_XRES); the pod's request of such a name is its ke_pod.xres entry of that id. */
#define KE_RSV_POLICY_DEFAULT 0    /* spec.allocatePolicy "" */
#define KE_RSV_POLICY_ALIGNED 1    /* Aligned */
#define KE_RSV_POLICY_RESTRICTED 2 /* Restricted (ResourceNames = the allocatable's names) */
/* ke_reservation.holds bits */
#define KE_RSV_HOLDS_NUMA 1u     /* the reserve pod has NUMANodeResources in the resource manager            */
#define KE_RSV_HOLDS_CPUSET 2u   /* the reserve pod has a CPUSet in the resource manager                     */
#define KE_RSV_HOLDS_DEVICES 4u  /* the reserve pod has device instances in the DeviceShare device cache     */
#define KE_RSV_OTHER_ALLOCATABLE 8u /* status.allocatable names a resource other than cpu / memory (pods, GPU,
                                       scalars): scoreReservation / fitsReservation read them (scoring.go:191-210,
                                       plugin.go:499-569); must agree with the reservation's resource entries
                                       (ke_reservations_load_full; without them: KE_ERR_UNSUPPORTED) */
typedef struct ke_reservation {
  int32_t node;           /* status.nodeName as a node index                                     */
  uint8_t available;      /* IsAvailable() and no ParseError                                     */
  uint8_t allocate_once;  /* spec.allocateOnce                                                   */
  uint8_t allocate_policy; /* KE_RSV_POLICY_*                                                     */
  uint8_t holds;          /* KE_RSV_HOLDS_*: must agree with the ke_reservation_alloc record (without one:
                             KE_ERR_UNSUPPORTED); KE_RSV_OTHER_ALLOCATABLE: with the resource entries      */
  int32_t allocated_pods; /* GetAllocatedPods(): owner pods assigned to it                         */
  int32_t pad2;
  int64_t allocatable[KE_NRES]; /* status.allocatable = the reserve pod's requests: MilliCPU, Memory; a zero
                                   quantity is an absent resource name */
  int64_t allocated[KE_NRES];   /* status.allocated: the owner pods' requests                     */
  int64_t order;          /* label scheduling.koordinator.sh/reservation-order parsed (ParseInt), 0 = none */
  int64_t uid;            /* the Reservation's UID interned by the caller (release records find it by this; 0 = none) */
  int64_t reserved[KE_NRES]; /* rInfo.Reserved (GetNodeReservationFromAnnotation, reservation_info.go:88): the part
                                of cpu / memory fitsReservation's capacity and GetAvailable exclude (0 = none)     */
  uint8_t names_excluded;    /* bit r: cpu (0) / memory (1) left out of rInfo.ResourceNames by the Restricted
                                options annotation (GetReservationRestrictedResources, reservation.go:637-654)      */
  uint8_t pad3[7];
} ke_reservation; /* 88 bytes */
/* One status.allocatable entry of a reservation beyond cpu / memory (ke_reservations_load_full). */
#define KE_RSV_RES_PODS (-1) /* the "pods" entry: fitsReservation's allocated-pods cap (plugin.go:511-527) */
typedef struct ke_reservation_resource {
  int32_t id;          /* resource id (ke_ext_args id space, not KE_XRES_CPU / KE_XRES_MEMORY) or KE_RSV_RES_PODS */
  uint8_t excluded;    /* left out of rInfo.ResourceNames by the Restricted options annotation                  */
  uint8_t pad[3];
  int64_t allocatable; /* status.allocatable[name] (Value(); > 0)                                               */
  int64_t allocated;   /* status.allocated[name] (Mask(owners' requests, ResourceNames))                        */
  int64_t reserved;    /* rInfo.Reserved[name] (0 = none)                                                        */
} ke_reservation_resource; /* 32 bytes */
/* What a reservation's reserve pod holds beyond NodeInfo, and what its owner pods (rInfo.AssignedPods) hold:
 * the resource manager's NUMANodeResources / CPUSet of the reserve pod and of its owners
 * (resourceManager.GetAllocatedNUMAResource / GetAllocatedCPUSet, nodenumaresource/reservation.go:185-227), and
 * the device cache's allocations of both (nodeDevice.getUsed, deviceshare/reservation.go:148-180).  These
 * allocations must also be part of the node state given with ke_node_numa_set / ke_node_cpus_set /
 * ke_node_devices_set (the reserve pod and its owners are pods on the node, as the resource manager and the device
 * cache count them).  From them the evaluator derives, per pod and node, the plugins' reservation restore states:
 *  - every pod: the unmatched reservations with allocated pods give back what their owners hold twice --
 *    mergedUnmatchedUsed as reusableResources of the NUMA zones (getAvailableNUMANodeResources,
 *    node_allocation.go:221-243) and as DeviceShare's preemptible (calcFreeWithPreemptible,
 *    device_cache.go:322-365);
 *  - a KE_RSV_MATCHED pod: its matched reservations' NUMA / cpuset / device holdings are allocated from first
 *    (tryAllocateFromReservation, nodenumaresource/reservation.go:270-424, deviceshare/reservation.go:207-287)
 *    with the Aligned / Restricted policy of each, in the Filter, the nomination's FilterNominateReservation,
 *    Score and Reserve.
 * A placement into a reservation adds the pod's cpuset / NUMA allocation / device minors to the owners' part
 * (ke_reservation_allocs_get reads them back); its release removes them. */
typedef struct ke_reservation_alloc {
  int64_t numa[KE_MAX_NUMA * KE_NRES];       /* the reserve pod's NUMANodeResources: [2*id + r], 0 = none    */
  int64_t owner_numa[KE_MAX_NUMA * KE_NRES]; /* Σ the owner pods' NUMANodeResources                            */
  uint64_t cpuset[4];                        /* the reserve pod's CPUSet (bit c = CPU id c)                    */
  uint64_t owner_cpuset[4];                  /* ∪ the owner pods' CPUSets, taken as disjoint: each CPU counts
                                                one owner (owners sharing a CPU under MaxRefCount > 1 are
                                                parity-unpinned: releasing one would free the CPU for both) */
  uint64_t device_minors;                    /* bit 16*type + minor: instances the reserve pod holds           */
  uint64_t owner_device_minors;              /* bit 16*type + minor: instances an owner pod holds              */
  int64_t device[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS];       /* the reserve pod's used per instance, 0 = none */
  int64_t owner_device[KE_DEV_TYPES][KE_MAX_MINORS][KE_DKEYS]; /* Σ the owner pods' used per instance          */
} ke_reservation_alloc; /* 2,640 bytes */
/* ke_reservations_load with the holdings of each reservation (allocs[i] belongs to reservations[i]; NULL = none
 * holds anything).  The holds bits NUMA / CPUSET / DEVICES must agree with the records (else KE_ERR_INVALID);
 * the evaluator takes the holdings from the records. */
int ke_reservations_load_ex(ke_ctx* ctx, int32_t n, const ke_reservation* reservations,
                            const ke_reservation_alloc* allocs);
/* ke_reservations_load_ex with each reservation's allocatable names beyond cpu / memory: reservation i owns
 * res[res_offsets[i] .. res_offsets[i+1]) (res_offsets: n + 1 entries; NULL = no entries), distinct ids, each
 * with a positive allocatable.  KE_RSV_OTHER_ALLOCATABLE must be set exactly when a reservation has entries.  The
 * entries enter every path that reads the reservation's allocatable / allocated: the NodeInfo restore of the
 * scalars (NodeInfo.Requested.ScalarResources, NodeResourcesFit / FitPlus), the name check, fitsNode,
 * fitsReservation and scoreReservation of the nominated-reservation path, and the Reserve's allocated. */
int ke_reservations_load_full(ke_ctx* ctx, int32_t n, const ke_reservation* reservations,
                              const ke_reservation_alloc* allocs, const int32_t* res_offsets,
                              const ke_reservation_resource* res);
/* Reservation r's resource entries as Reserve / release left them: up to cap entries, *n = count. */
int ke_reservation_resources_get(ke_ctx* ctx, int32_t r, int32_t cap, ke_reservation_resource* out, int32_t* n);
/* The holdings as they stand (owner parts after the Reserves / releases of this context). */
int ke_reservation_allocs_get(ke_ctx* ctx, int32_t n, ke_reservation_alloc* out);
/* Generation of the loaded reservation set: bumped by every ke_reservations_load. */
int32_t ke_reservations_generation(ke_ctx* ctx);
/* Replace the reservation set (n = 0: none).  A pod placed into a reservation (below) updates its
 * allocated / allocated_pods here (ke_reservations_get reads them back). */
int ke_reservations_load(ke_ctx* ctx, int32_t n, const ke_reservation* reservations);
int ke_reservations_get(ke_ctx* ctx, int32_t n, ke_reservation* out);

/* Pods that match reservations (the nominated-reservation path).  ke_pod.reservation_matched: */
#define KE_RSV_NONE 0     /* matches no reservation: the restore above only                             */
#define KE_RSV_MATCHED 1  /* owner-matched reservations (MatchOwners, not unschedulable, taints tolerated,
                             ReservationAffinity / exact-match spec satisfied: the integrator's label logic,
                             transformer.go:97-146) listed with ke_pod_reservations                          */
#define KE_RSV_AFFINITY 2 /* a required reservation affinity: as KE_RSV_MATCHED, and the Reservation Filter
                             passes only nodes where a listed reservation fits (an empty list: unschedulable) */
#define KE_RSV_IGNORED 3  /* reservation-ignored pod (apis/extension/reservation.go:97-99): every available
                             reservation of every node is matchedOrIgnored (its reserve pod leaves NodeInfo, no
                             unmatched restore), no Reservation Filter / Score / Reserve; lists none.
                             KE_ERR_UNSUPPORTED outside ke_schedule and where it would read resources a
                             reservation holds (ke_reservation_alloc): a DeviceShare pod beside held devices, a
                             pod with a NUMA policy beside held NUMA resources or CPUs, any pod while those sit
                             on a NUMA-policy node.  A CPU-binding pod allocates with the held CPUs preferred
                             (tryAllocateIgnoreReservation)                                                     */
/* For each pod of the next ke_schedule call, the reservations (indices into the loaded set) it matches,
 * ids[offsets[p] .. offsets[p+1]) (with a reservation name in the affinity: only that one).  Only KE_RSV_MATCHED /
 * KE_RSV_AFFINITY pods may list any; the call consumes the lists.
 * For a KE_RSV_MATCHED pod the evaluator runs, as the Reservation plugin and the transformer do:
 *  - BeforePreFilter: of its listed reservations the available ones that are not AllocateOnce with
 *    allocated pods are "matched" on their nodes; restoreMatchedReservation (transformer.go:422-445)
 *    removes each one's reserve pod from NodeInfo (Requested and NonZeroRequested -= allocatable), the
 *    other reservations restore as for any pod;
 *  - Filter passes without a reservation affinity (plugin.go:351-354); with one (KE_RSV_AFFINITY) only nodes
 *    holding a matched reservation that fits (fitsNode, and fitsReservation for Restricted) pass
 *    (plugin.go:316-318, 368-441), and NominateReservation takes a node's only matched one unfiltered (:223-225);
 *  - PreScore / NominateReservation (scoring.go:42-109, nominator.go:207-278): per node the matched
 *    reservations passing FilterNominateReservation (plugin.go:707-738: resource names shared with the pod,
 *    fitsNode over the restored NodeInfo, fitsReservation for Restricted) are nominated by the smallest
 *    order, else by ScoreReservation (ties -> the lowest reservation index); the feasible node holding the
 *    smallest order (ties -> lowest node index) is preferredNode;
 *  - Score (scoring.go:111-139): 1000 for preferredNode, else ScoreReservation of the nominated one
 *    (MostAllocated over the reservation's allocatable, scoring.go:191-210), 0 without; DefaultNormalizeScore
 *    over the feasible nodes; weighted by ke_config.weight_reservation into the total;
 *  - Reserve (plugin.go:740-793, reservation_info.go:458-468): the nominated reservation of the chosen node
 *    takes Mask(pod requests, names) into allocated and one allocated pod (ke_pod_allocation.reservation); ke_pod_release gives it back (forgetPod,
 *    reservation_info.go:470-482).
 * fitsNode's pod-count check (plugin.go:450-453) is part of the nomination and the affinity Filter: len(Pods) of
 * the restored NodeInfo (ke_node.pod_count with the matched reserve pods removed) minus the node's matched
 * reservations, plus one, within ke_node.allowed_pods.
 * Refused (KE_ERR_UNSUPPORTED, by ke_schedule's argument checks before any pod of the call is scheduled): such a
 * pod with DeviceShare requests or resources outside KE_RES_* / xres (has_other_requests), one with a NUMA topology policy whose usable matched reservation holds
 * NUMA resources or a cpuset, a usable matched reservation holding NUMA resources or a cpuset on a node with a NUMA
 * topology policy; ke_eval of such a pod.  (Node-sharded contexts pick over every rank's pairs.)  The lists
 * are consumed by the next ke_schedule call, a refused one included. */
int ke_pod_reservations(ke_ctx* ctx, int32_t n_pods, const int32_t* offsets, const int32_t* ids);
/* NodeInfo.Requested / NonZeroRequested (MilliCPU, Memory) of `node` as the plugins see it for a pod that
 * matches no reservation (after the restore above and the Reserves of past ke_schedule calls). */
int ke_node_info_requested(ke_ctx* ctx, int32_t node, int64_t* requested /*[2]*/, int64_t* non_zero /*[2]*/);
/* The node's GPU partition indexer and policy as GPUAllocator.Allocate resolves them (allocator_gpu.go:77-82,
 * device_cache.go:532-545): has_table = the indexer is not nil (the Device's gpu-partitions annotation, else
 * the designated table of the node's GPU model), honor = the matching GPUPartitionPolicy label is Honor.
 * Partitions with the same (number_of_gpus, allocation_score) keep their table order; such a group may hold
 * at most 12 partitions (selectPartitionByBinPack's sort.Slice is stable only up to 12 elements), else
 * KE_ERR_UNSUPPORTED.  Kept across ke_node_devices_set; dropped with ke_node_devices_delete. */
int ke_node_gpu_partitions(ke_ctx* ctx, int32_t node, int32_t has_table, int32_t honor, int32_t n,
                           const ke_gpu_partition* partitions);
/* NodeResourceTopology informer + resource manager state of `node`: its NUMA zones (n <= KE_MAX_NUMA,
 * n = 0: no NUMA resources).  Read when the node's NUMA topology policy is not None. */
int ke_node_numa_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_numa_zone* zones);
/* The node's CPU topology and cpuset allocation state (TopologyOptions.CPUTopology + ReservedCPUs +
 * MaxRefCount, NodeAllocation.allocatedCPUs).  n = 0 clears it (no CPU topology).  With a CPU table the
 * allocated-CPU count of the amplified-CPU filter / score and the zones' cpuset counts are derived from
 * it (ke_node.cpuset_allocated_cpus and ke_numa_zone.cpuset_cpus are then ignored). */
int ke_node_cpus_set(ke_ctx* ctx, int32_t node, int32_t n, const ke_cpu* cpus, int32_t max_ref_count);
/* The cpuset each pod of the last ke_schedule received (NodeNUMAResource Reserve -> PreBind
 * resource-status annotation): out[pod][4] = a 256-bit CPU-id set, all zero without one. */
int ke_last_cpusets(ke_ctx* ctx, int32_t n, uint64_t* out);
/* The NUMA allocation each pod of the last ke_schedule received on its node (NodeNUMAResource Reserve
 * -> resourceManager.Update, resource_manager.go:194-258 / node_allocation.go:111-156): out[pod][2*id
 * + r] for NUMA id and resource r (cpu milli, memory), all zero for a pod without one.  The context
 * already applied them to its zones; a host keeping its own resource manager reads them here. */
int ke_last_numa_allocations(ke_ctx* ctx, int32_t n, int64_t* out);

/* ---- evaluation ------------------------------------------------------------------------------ */
/* Parity mode: Filter + Score of `n_pods` pods against every node, no state change.
 * Each output is optional (NULL) and laid out [pod][node]:
 *   status   uint8  KE_CODE_* of the first failing filter (profile order LoadAware, NodeNUMAResource)
 *   reason   uint8  KE_REASON_*
 *   la_score int16  LoadAwareScheduling.Score (0 for filtered-out nodes)
 *   numa_score int16 NodeNUMAResource.Score
 *   ds_score int16  DeviceShare.Score before NormalizeScore (the total uses the normalized score,
 *                   DefaultNormalizeScore over the pod's feasible nodes, scoring.go:109-111)
 *   total    int16  Σ weight·score over the plugins, -1 if the node is filtered out
 * and `best[pod]` is selectHost's choice (-1 if no feasible node; ties -> lowest node index). */
int ke_eval(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns,
            uint8_t* status, uint8_t* reason, int16_t* la_score, int16_t* numa_score,
            int16_t* ds_score, int16_t* total, int32_t* best);

/* Schedule `n_pods` pods in queue order, each one seeing the Reserve of all pods before it
 * (LoadAware podAssignCache.assign with timestamp now_ns, NodeInfo.Requested += pod requests).
 * chosen[p] = node index or -1 (unschedulable), score[p] = its framework total (or -1).
 * Bit-exact with one-pod-at-a-time scheduling (exact speculative batching). */
int ke_schedule(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns,
                int32_t* chosen, int32_t* score);

/* ke_schedule in two halves, so a scheduler loop can hand over its next queue slice while the device still
 * resolves the previous one (the same sequential semantics: a submitted call sees the Reserves of every call
 * submitted before it).  ke_schedule_submit checks the arguments (a refused call returns its code and submits
 * nothing), enqueues the call and returns a ticket; ke_schedule_wait(ticket) writes its chosen / score (as
 * ke_schedule) and makes it "the last ke_schedule" of ke_last_allocations / ke_unreserve.  `pods` must stay valid
 * until the wait.  Only a plain queue is enqueued behind a call in flight (no reservation-matched, NUMA-policy,
 * quota, DeviceShare or cpuset pod, no NUMA state, unsharded, pipelined, no node row to re-derive); any other
 * call first completes the calls in flight and runs at once (its outputs are kept for the wait).  Every other
 * entry point except the ke_last_* statistics completes the calls in flight first; the statistics describe the
 * last completed call.  Replaces nothing in the reference: scheduleOne's per-pod loop
 * (frameworkext/framework_extender_factory.go:159-192) is sequential, and so are the submitted calls. */
int ke_schedule_submit(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns, int64_t* ticket);
int ke_schedule_wait(ke_ctx* ctx, int64_t ticket, int32_t* chosen, int32_t* score);

/* Timing of the last ke_schedule call: device milliseconds of the whole queue, and per-batch
 * device service time (the batch's eval start -> its Reserve end) in milliseconds, n_batches entries. */
int ke_last_schedule_stats(ke_ctx* ctx, double* total_ms, int32_t* n_batches,
                           double* batch_ms, int32_t batch_ms_cap);
/* Per-pod scheduling latency of the last ke_schedule (pod dequeue -> node selected), in
 * milliseconds: from the ke_schedule call's entry (every pod of the call is dequeued then) to the end of its
 * batch's Reserve on the device, mapped onto the host clock through the call's device-side stamps aligned at
 * the host's return from the final stream synchronisation (an upper bound).  Includes the argument checks, row
 * refresh, pod upload, launch setup and the wait behind earlier batches of the same call. */
int ke_last_pod_latencies(ke_ctx* ctx, int32_t n, double* ms);
/* DeviceShare Reserve of the last ke_schedule (AutopilotAllocator.Allocate -> updateCacheUsed,
 * plugin.go:426-492): per pod, bit 16*type + minor set for every device instance allocated. */
int ke_last_device_allocations(ke_ctx* ctx, int32_t n, uint64_t* minors);

/* ---- Unreserve and pod release (ReservePlugin.Unreserve, pod informer deletes) -------------------
 * What one placement reserved, as the plugins keep it in CycleState / their caches:
 *   cpuset, numa     NodeNUMAResource PodAllocation.CPUSet / NUMANodeResources (state.allocation,
 *                    nodenumaresource/plugin.go:564-565; node_allocation.go:42-49)
 *   device_minors    DeviceShare state.allocationResult (deviceshare/plugin.go:491): the instances; the
 *                    amounts are the pod's per-instance request (what Reserve added, fillGPUTotalMem)
 *   quota_assigned   ElasticQuota: the pod's request is counted in its quota's used (ReservePod ran)
 * node = the node index ke_schedule returned (global index when sharded), -1 = not placed. */
typedef struct ke_pod_allocation {
  int32_t node;
  uint8_t quota_assigned;
  uint8_t pad[3];
  uint64_t cpuset[4];                   /* bit c = CPU id c (ke_last_cpusets)                 */
  int64_t numa[KE_MAX_NUMA * KE_NRES];  /* [2*id + r] per NUMA id (ke_last_numa_allocations) */
  uint64_t device_minors;               /* bit 16*type + minor (ke_last_device_allocations)   */
  /* allocateVF: the VF rank taken on each allocated RDMA / FPGA minor, -1 = none ([type - 1][minor]) */
  int8_t vf_rank[2][KE_MAX_MINORS];
  int32_t reservation;                  /* 1 + the index of the reservation the pod was assumed into (Reserve),
                                           0 = none */
  int32_t reservation_generation;       /* ke_reservations_generation() when the record was taken */
  int64_t reservation_uid;              /* that reservation's uid: a release finds it by uid when non-zero (a
                                           reservation no longer loaded forgets nothing), else by index, which
                                           must belong to the current generation (KE_ERR_INVALID otherwise) */
} ke_pod_allocation; /* 224 bytes */
/* ke_pod_release modes */
#define KE_RELEASE_UNRESERVE 0 /* the framework's Unreserve of every Reserve plugin + ForgetPod:
                                  loadaware podAssignCache.unAssign (load_aware.go:197-199),
                                  nodenumaresource resourceManager.Release (plugin.go:569-577,
                                  node_allocation.go:158-190), deviceshare updateCacheUsed(..., false)
                                  (plugin.go:498-516, device_cache.go:132-209), elasticquota UnreservePod
                                  (plugin.go:361, group_quota_manager.go:965-981), NodeInfo.RemovePod */
#define KE_RELEASE_DELETE 1    /* informer delete of an assigned pod: the same, and the quota also drops the
                                  pod's request (OnPodDelete, group_quota_manager.go:922-941;
                                  nodenumaresource pod_eventhandler.go:99-144, deviceshare
                                  eventhandler_pod.go:89-131) */
/* Each placement of the last ke_schedule as a release record (node -1 for an unplaced pod). */
int ke_last_allocations(ke_ctx* ctx, int32_t n, ke_pod_allocation* out);
/* Release `pod` from alloc->node: every plugin's state and the node's NodeInfo.Requested (and the
 * NodeResourcesFitPlus requested of its resources) lose exactly what its Reserve added, with the
 * reference's non-negative subtraction (quotav1.SubtractWithNonNegativeResult for NUMA zones and device
 * used, a device whose used becomes zero drops its used keys; RefCount-- per CPU, the CPU leaving the
 * allocation at 0; the zones' single / shared pod sets; quota used / non-preemptible used of the quota
 * and every ancestor clamped at 0, a system / default quota growing the tree total back).  Release each
 * placement at most once.  alloc->node == -1 with KE_RELEASE_DELETE removes only the quota request. */
int ke_pod_release(ke_ctx* ctx, const ke_pod* pod, const ke_pod_allocation* alloc, int32_t mode);
/* Unreserve of the pod at `queue_pos` of the last ke_schedule call (pod->uid must match): ke_pod_release
 * with the record ke_last_allocations reports, KE_RELEASE_UNRESERVE.  A second call for the same
 * position, or for an unplaced pod, is a no-op. */
int ke_unreserve(ke_ctx* ctx, const ke_pod* pod, int32_t queue_pos);

/* ---- ElasticQuota admission (pkg/scheduler/plugins/elasticquota) ----------
 * One quota tree.  Replaces GroupQuotaManager's runtime calculation and the plugin's PreFilter /
 * Reserve for the pods of a ke_schedule call:
 *  - runtime: RuntimeQuotaCalculator (core/runtime_quota_calculator.go:117-189) over the tree, fed by
 *    the limited requests of recursiveUpdateGroupTreeWithDeltaRequest (core/group_quota_manager.go:196-239)
 *    and refreshed top-down as refreshRuntimeNoLock (:286-353); requests are fixed for the call;
 *  - PreFilter (plugin.go:223-275): used + Mask(PodRequests, Max names) <= usedLimit (runtime on the
 *    tree's resource keys, or Max with EnableRuntimeQuota false / for system and default quotas), non-preemptible
 *    pods also against Min, EnableCheckParentQuota walks the ancestors (plugin_helper.go:281-301);
 *    a refused pod is unschedulable (chosen -1) and reserves nothing;
 *  - Reserve (core/group_quota_manager.go:700-760, ReservePod :943-963): the masked request is added
 *    to used (and non-preemptible used) of the quota and every ancestor.
 *  - system / default quotas (limit_is_max): used limit = Max; a Reserve into one with runtime quota on
 *    shrinks totalResourceExceptSystemAndDefaultUsed (updateClusterTotalResourceNoLock,
 *    group_quota_manager.go:127-151,268-271) and every later pod of the call sees runtime limits
 *    refreshed from the smaller total.
 * Not modelled: guaranteed usage (feature gate ElasticQuotaGuaranteeUsage, default off), hook plugins, quota-overuse revocation, preemption
 * (PostFilter); a zero-valued pod request counts as an absent key (checkQuotaRecursive masks on
 * ResourceNames(PodRequests), which keeps explicit zeros — ke_pod carries values, not key sets).
 * Resources: cpu (milli, getQuantityValue) and memory (bytes).  Values >= 0. */
#define KE_MAX_QUOTAS 255 /* ke_pod.quota - 1 fits a byte on the device */
typedef struct ke_quota_args {
  int64_t total[KE_NRES];            /* totalResourceExceptSystemAndDefaultUsed of the tree */
  uint8_t enable_runtime_quota;      /* ElasticQuotaArgs.EnableRuntimeQuota (v1beta3 default true) */
  uint8_t enable_check_parent_quota; /* ElasticQuotaArgs.EnableCheckParentQuota (default false) */
  /* 0 (the scheduler's NewGroupQuotaManager: scaleMinQuotaEnabled = true): when the Min of a parent's
   * children sums above the parent's runtime (the tree total for the root's children) on a resource,
   * the calculator shares with every child's Min scaled to int64(float64(total) * float64(Min) /
   * float64(ΣMin)) (ScaleMinQuotaManager.getScaledMinQuota, scale_minquota_when_over_root_res.go:129-184;
   * refreshRuntimeNoLock :320-328) — the state once every quota has been refreshed at the current
   * total.  System / default quotas (limit_is_max) stay out of the sums as they stay out of the
   * sharing.  1: the core package's test manager (Min unscaled). */
  uint8_t disable_scale_min_quota;
  /* Not on this path -> ke_quotas_load returns KE_ERR_UNSUPPORTED when set: the number of
   * ElasticQuotaArgs.HookPlugins (QuotaHookPlugin callbacks, core/hook_plugin.go), and the
   * ElasticQuotaGuaranteeUsage feature gate (Guaranteed raising the calculator's Min,
   * group_quota_manager.go:257,1074-1106). */
  uint8_t n_hook_plugins;
  uint8_t enable_guarantee_usage;
  uint8_t pad[3];
} ke_quota_args;
typedef struct ke_quota {
  int32_t parent;                 /* index of the parent quota; -1 = koordinator-root-quota */
  uint8_t has_max[KE_NRES];       /* keys of Spec.Max */
  uint8_t has_min[KE_NRES];       /* keys of Spec.Min */
  uint8_t allow_lent_resource;    /* AllowLentResource (label allow-lent-resource, default true) */
  uint8_t limit_is_max;           /* system / default quota: used limit = Max (group_quota_manager.go:297) */
  uint8_t pad[2];
  int64_t max[KE_NRES];
  int64_t min[KE_NRES];
  int64_t shared_weight[KE_NRES]; /* extension.GetSharedWeight: annotation, else Max */
  int64_t self_request[KE_NRES];  /* Σ Mask(PodRequests, Max) of the quota's own pods, pending and assigned */
  int64_t used[KE_NRES];          /* Used: assigned pods of the quota and of its descendants */
  int64_t non_preemptible_used[KE_NRES];
} ke_quota;
/* Load (replace) the tree, quotas in any order with parents by index; n <= KE_MAX_QUOTAS. */
int ke_quotas_load(ke_ctx* ctx, const ke_quota_args* args, const ke_quota* quotas, int32_t n);
/* The used limit PreFilter compares against (runtime, or Max) with its keys, and the quota's
 * current used / non-preemptible used (after the Reserves of the last ke_schedule). */
int ke_quota_state(ke_ctx* ctx, int32_t q, int64_t* limit, uint8_t* limit_has, int64_t* used, int64_t* np_used);

/* ---- wire-format decoders ------------------------------------------------
 * The informer objects as the apiserver serves them (JSON) -> the structs above, the way the reference's
 * listers and apis/extension helpers read them per call.  Context-free, host-only, thread-safe.  Malformed
 * objects -> KE_ERR_INVALID; values the structs cannot carry (a policy string outside the known ones,
 * thresholds on other resources, quantities beyond int64, ...) -> KE_ERR_UNSUPPORTED.
 *   ke_quantity_parse     resource.ParseQuantity + Value() / MilliValue() (both round up)
 *   ke_pod_key            the interned key ke_pod.pod_key / ke_pod_metric.pod_key use: FNV-1a 64 of
 *                         "namespace/name" (top bit cleared); ke_decode_pod / ke_decode_node_metric use it
 *   ke_decode_node        Node: status.allocatable; annotations node.koordinator.sh/raw-allocatable,
 *                         node.koordinator.sh/resource-amplification-ratio, scheduling.koordinator.sh/usage-thresholds
 *                         (node_resource_amplification.go:45-124, load_aware.go:42-72, default_estimator.go:124-143);
 *                         labels node.koordinator.sh/numa-topology-policy, cpu-bind-policy, numa-allocate-strategy
 *                         (numa_aware.go:54-59,354-369, nodenumaresource/util.go:41-47).  NodeInfo.Requested, the
 *                         cpuset count and the NodeResourceTopology-side fields (kubelet policies, NRT ratios,
 *                         CPU topology validity) are not in a Node object: left 0 / "no NRT".
 *   ke_decode_node_metric NodeMetric (slo/v1alpha1/nodemetric_types.go:38-136): header, up to pm_cap pod metrics
 *                         (nil entries skipped) and agg_cap aggregated usages.
 *   ke_decode_pod         Pod: PodRequests / PodLimits (k8s v1.28; restartable init containers -> UNSUPPORTED),
 *                         classes (priority_utils.go:37-58, qos_utils.go:32-68), DaemonSet owner, phase, the
 *                         PodScheduled / Initialized conditions, the LoadAware estimation annotations
 *                         (load_aware.go:75-100), ResourceSpec / NUMATopologySpec, the preemptible label, the
 *                         DeviceShare annotations; xres_names[id] = the resource name of id (NodeResourcesFitPlus /
 *                         ScarceResourceAvoidance, n_names <= KE_MAX_XRES).  ke_pod.quota is left 0: the caller
 *                         maps the quota label to its ke_quotas_load index.
 *   ke_decode_device      Device (scheduling/v1alpha1/device_types.go:32-67) as nodeDeviceCache builds it
 *                         (device_cache.go:518-568; `used` is the pods' business: 0), the gpu-partitions annotation
 *                         (table in ascending key order) and the gpu-partition-policy label.
 *   ke_decode_nrt         NodeResourceTopology (below). */
int ke_quantity_parse(const char* s, int64_t* value, int64_t* milli_value);
int64_t ke_pod_key(const char* ns, const char* name);
int ke_decode_node(const char* json, int64_t len, ke_node* out);
int ke_decode_node_metric(const char* json, int64_t len, ke_node_metric* nm, int32_t pm_cap, ke_pod_metric* pm,
                          int32_t* n_pm, int32_t agg_cap, ke_aggregated_usage* agg, int32_t* n_agg);
int ke_decode_pod(const char* json, int64_t len, int32_t n_names, const char* const* xres_names, ke_pod* out);
int ke_decode_device(const char* json, int64_t len, int32_t cap, ke_device* out, int32_t* n, int32_t part_cap,
                     ke_gpu_partition* parts, int32_t* n_parts, int32_t* has_table, int32_t* honor);
/* A pod's DeviceAllocateHints + DeviceJointAllocate annotations (parsePodDeviceShareExtensions,
 * deviceshare/utils.go:414-482; selectors through GetFastLabelSelector); *present = 0 when neither annotation
 * is set (the pod needs no hint entry).  Label strings are interned with ke_label_id. */
int ke_decode_pod_device_hints(const char* json, int64_t len, ke_pod_device_hints* out, int32_t* present);
/* The node-level device flags ke_node_device_flags takes: the Device's secondary-device-well-planned label and the
 * GPU template key of the Node ("<gpu vendor label>-<gpu model label>" interned; 0 without both labels). */
int ke_decode_device_flags(const char* device_json, int64_t device_len, const char* node_json, int64_t node_len,
                           int32_t* secondary_well_planned, int32_t* gpu_model_key);
/* NodeResourceTopology (NewTopologyOptions, nodenumaresource/topology_options.go:90-236): the zones of type
 * "Node" named node-<id> with their Allocatable cpu / memory (cpu less 1000 per reserved CPU of the zone), the CPU
 * table of the cpu-topology annotation (core id = socket << 16 | core) with the reserved CPUs (kubelet-managed
 * pod-cpu-allocs, kubelet reservedCPUs, the node-reservation reservedCPUs, an exclusive system-QoS cpuset) flagged,
 * and the node-level fields an NRT supplies, patched into *node (decode the Node first): the topology-manager
 * policy when the Node has no policy label, FullPCPUsOnly from a static kubelet with full-pcpus-only=true, the
 * NRT's cpu amplification ratio (-2 without a ratio map), and cpu_topology_invalid when no CPU is reported.  The
 * resource manager's allocation state (zone allocations, RefCounts, NUMA status) is the scheduler's own: 0. */
int ke_decode_nrt(const char* json, int64_t len, ke_node* node, int32_t zone_cap, ke_numa_zone* zones, int32_t* n_zones,
                  int32_t cpu_cap, ke_cpu* cpus, int32_t* n_cpus);
/* Reservation (apis/scheduling/v1alpha1/reservation_types.go) as the reservation cache builds its ReservationInfo
 * (frameworkext/reservation_info.go:87-130): available = scheduled (status.nodeName) and phase Available
 * (util/reservation/reservation.go:238-240; a malformed restricted-options annotation, a ParseError, clears it);
 * allocatable = ReservationRequests (status.allocatable when available, else the template's PodRequests,
 * reservation.go:393-404) -- cpu / memory into *out, every other non-zero name into res[] by its index in
 * xres_names ("pods" = KE_RSV_RES_PODS; a name without an id -> KE_ERR_UNSUPPORTED), *n_res entries;
 * allocated = status.allocated masked by rInfo.ResourceNames (the Restricted options annotation narrows them:
 * names_excluded / excluded); reserved = the node-reservation annotation (util/node.go:85-120); allocateOnce
 * (default true), allocatePolicy, the reservation-order label, allocated_pods = len(status.currentOwners), uid =
 * FNV-1a of metadata.uid.  *alloc (optional): the reserve pod's holdings from its device-allocated and
 * resource-status annotations (the owner parts are the owner pods': 0 here); holds is derived from them and from
 * the entries (KE_RSV_OTHER_ALLOCATABLE).  out->node is -1: the caller maps status.nodeName, copied NUL-terminated
 * into node_name[name_cap], to its node index. */
int ke_decode_reservation(const char* json, int64_t len, int32_t n_names, const char* const* xres_names,
                          ke_reservation* out, ke_reservation_alloc* alloc, int32_t res_cap, ke_reservation_resource* res,
                          int32_t* n_res, char* node_name, int32_t name_cap);

/* ---- node sharding across GPUs (one process per GPU) ------------------------------------------
 * Replaces the upstream Parallelizer's fan-out of per-node Filter/Score over goroutines
 * (cmd/koord-scheduler/app/server.go:417, Parallelism) with a fan-out of node ranges over GPUs.
 * Every rank holds the full node state (same ingestion calls on every rank) and evaluates only its
 * contiguous node range; per speculative batch the ranks exchange their per-pod top-k candidate
 * lists with one RCCL all-gather and every rank resolves the batch identically, so the replicas
 * stay bit-identical without exchanging rows.  Placements equal the unsharded ke_schedule. */
#define KE_COMM_ID_BYTES 128
/* RCCL unique id (ncclGetUniqueId), created once by rank 0 and broadcast to the others. */
int ke_comm_unique_id(uint8_t* id, int32_t id_bytes);
/* Collective: every rank calls it with the same id.  world in [1,8].  id == NULL with world > 1 is
 * loopback mode: this context evaluates every shard itself and merges locally (single-GPU tests of
 * the sharded path); world == 1 with an id runs the sharded path over a 1-rank communicator. */
int ke_shard_init(ke_ctx* ctx, int32_t rank, int32_t world, const uint8_t* id);
/* ke_shard_init with the collectives carried by the caller on the host (e.g. a gloo process group) instead of
 * RCCL: the same per-batch exchange -- the candidate lists' all-gather (op KE_COLL_ALL_GATHER: `count` words of this
 * rank into recv[world * count], rank-major), DeviceShare's NormalizeScore max and the staged Reservation pick's
 * reductions (KE_COLL_MAX / KE_COLL_MIN over `count` elements of dtype KE_COLL_*) -- each after the eval stream's
 * work so far completes.  fn returns 0 on success.  Readiness / test path of the multi-process protocol. */
#define KE_COLL_ALL_GATHER 0
#define KE_COLL_MAX 1
#define KE_COLL_MIN 2
#define KE_COLL_U32 0
#define KE_COLL_I32 1
#define KE_COLL_I64 2
#define KE_COLL_U64 3
typedef int32_t (*ke_host_collective)(void* user, int32_t op, int32_t dtype, const void* send, void* recv,
                                      int64_t count);
int ke_shard_init_host(ke_ctx* ctx, int32_t rank, int32_t world, ke_host_collective fn, void* user);
/* This rank's node range [lo, hi) for the current node count. */
int ke_shard_range(ke_ctx* ctx, int32_t* lo, int32_t* hi);

/* ---- measurement ----------------------------------------------------------------------------- */
/* Sample every `sample_every`-th batch of ke_schedule with HIP event pairs around each of its
 * kernels (0 = off).  ke_last_kernel_stats returns the average device milliseconds per launch of
 * the eval / select / resolve kernels over the sampled batches of the last ke_schedule. */
int ke_set_profiling(ke_ctx* ctx, int32_t sample_every);
int ke_last_kernel_stats(ke_ctx* ctx, double* eval_ms, double* select_ms, double* resolve_ms, int32_t* samples);
/* Per-batch statistics of the last ke_schedule: v8 = {eval ms, select ms (HIP-event samples on the eval
 * stream), fixup ms (k_fixup after its wait, pipelined batches), Reserve ms (in-kernel stamps: prologue +
 * replay, every batch), host enqueue ms of the whole call, hand-off ms (end of a pipelined batch's replay
 * -> start of the next one's), replay records fetched per batch (best unchanged candidates), rows changed
 * per batch}, the number of event samples, and how many batches ran pipelined. */
int ke_last_kernel_stats_ex(ke_ctx* ctx, double* v8, int32_t* samples, int32_t* pipelined_batches);
/* Pipelined schedule (default 1): batch b's eval + select overlap batch b-1's Reserve replay on a
 * second stream; the replay takes the stale candidate lists with batch b-1's changed nodes as
 * slots.  2 = pipelined with the lists made exact by a fixup kernel first (the round-3 schedule; ElasticQuota
 * runs always take it).  0 = one stream, every batch waits for the previous Reserve.  The placements are
 * identical in every mode. */
int ke_set_pipeline(ke_ctx* ctx, int32_t on);
/* Host wall milliseconds of the last ke_schedule by phase: argument checks, row refresh, pod upload,
 * launch setup, enqueue, wait for the device, statistics readback, host mirror of the Reserves. */
int ke_last_host_stats(ke_ctx* ctx, double* ms8);
/* Resolve kernel split of the last ke_schedule (in-kernel s_memrealtime stamps, every batch):
 * average ms per batch of candidate/row staging (prologue) and of the sequential replay. */
int ke_last_resolve_split(ke_ctx* ctx, double* prologue_ms, double* replay_ms);
/* Finer split (6 entries, ms per batch): prologue, the speculative replay's first round — predict (P),
 * reserve + evaluate the slots (R + S), verify (V) —, its later rounds, and the write-back (all of a one-wave
 * replay). */
int ke_debug_resolve_phases(ke_ctx* ctx, double* phases6);
/* The speculative replay's first round in detail (5 entries; the first four ms per batch): T's set-up, the
 * prediction loop (wave 0), the T maxima on wave 1 (its own rows or the T-row helpers' hand-off, concurrent with
 * the loop), wave 0's R; then the fraction of T batches whose maxima came from the helpers. */
int ke_debug_resolve_subphases(ke_ctx* ctx, double* sub5);
/* The progressive S of wave 1 in the first round of a batch with helper T maxima (4 entries, ms per batch): its
 * polls for the chunks' predictions, its record loads + Reserves of the chunks' slots, its rows, and its end after
 * T's set-up. */
int ke_debug_resolve_wave1(ke_ctx* ctx, double* w4);
/* BestEffort (pod, node) pairs the last ke_eval / ke_schedule evaluated in the compacted full-merge
 * pass (no preferred merged hint). */
int ke_debug_numa_deferred(ke_ctx* ctx, int64_t* n);
/* DeviceShare batches of the last ke_schedule that stopped early because a pod's NormalizeScore max may have
 * moved (their remaining pods were re-run as a new batch). */
int ke_debug_ds_cuts(ke_ctx* ctx, int32_t* cuts);
/* Reservation-matched pods of the last ke_schedule that ran fused behind their preceding plain segment (placed by
 * that call: out2[0]) and those whose speculation a plain pod of the segment broke (run again alone: out2[1]);
 * DESIGN.md §4k.  KOORDEVAL_RSV_FUSE=0 turns the fusion off. */
int ke_debug_rsv_fused(ke_ctx* ctx, int64_t* out2);
/* Diagnostic build only (-DKE_PROF_REPLAY): shader cycles per pod of the replay loop's phases since the
 * last call — best unchanged candidate, row fetch issue, re-evaluation, its wave max, decision / adoption,
 * Reserve, next pod's changed flags — and the pod count (cyc8[7]); zeros in the product build. */
int ke_debug_replay_phases(ke_ctx* ctx, double* cyc8);
/* The same per phase of another kernel of the diagnostic build: kernel 0 k_resolve (per pod), 1 k_numa_fallback
 * (per deferred pair), 2 k_cpuset_reserve (per pod), 3 k_select (per wave); each read clears that kernel's counters. */
int ke_debug_kernel_phases(ke_ctx* ctx, int32_t kernel, double* cyc8);
/* Speculative replay of plain batches: rounds per batch of the last ke_schedule that ended at a
 * failed prediction (0 = every pod of the batch took its best candidate not taken before). */
int ke_debug_spec_failed(ke_ctx* ctx, double* per_batch);
/* Number of nodes whose replay record (the Reserve replay's row-major copy of the node-only terms)
 * differs from one derived from the node's current device row (0 = consistent). */
int ke_debug_check_records(ke_ctx* ctx, int64_t now_ns, int64_t* mismatched_nodes);
/* Launch the batch eval kernel `iters` times back to back over the current node SoA for `n_pods`
 * (<= 64) pods and return the HIP-event average milliseconds per launch (roofline measurement). */
int ke_bench_eval_kernel(ke_ctx* ctx, int32_t n_pods, const ke_pod* pods, int64_t now_ns, int32_t iters,
                         double* avg_ms);

/* ---- introspection (tests, tools) ------------------------------------------------------------ */
/* sizeof() of one node row of the device SoA in bytes (algorithmic bytes per node per pass). */
int ke_row_bytes(void);
/* sizeof() of the per-pod record the kernels read (the device form of a ke_pod). */
int ke_pod_record_bytes(void);
/* Copy the device SoA rows of nodes [0,n) back to the host (n*ke_row_bytes() bytes) and, into
 * `host_rows`, the rows the host derives from its object state; lets tests check the GPU-side
 * patches against a from-scratch host derivation. */
int ke_debug_rows(ke_ctx* ctx, int32_t n, int64_t now_ns, void* device_rows, void* host_rows);
/* The folded LoadAware threshold U*(total, thr): the largest `used` with
 * int64(math.Round(float64(used)/float64(total)*100)) <= thr (load_aware.go:299), |used| <= 2^53. */
int64_t ke_debug_usage_bound(int64_t total, int64_t thr);
int32_t ke_num_nodes(ke_ctx* ctx);
/* The host object state of `node` after every Reserve / release so far: the Node (NodeInfo.Requested), its
 * CPU table (RefCount / ExclusivePolicy), NUMA zones (allocations, single / shared pod counts) and device
 * cache entry (used).  Up to *_cap entries each, counts in *n_*.  Tests compare it with the oracle's. */
int ke_debug_node_state(ke_ctx* ctx, int32_t node, ke_node* out, int32_t cpu_cap, ke_cpu* cpus, int32_t* n_cpus,
                        int32_t zone_cap, ke_numa_zone* zones, int32_t* n_zones, int32_t dev_cap, ke_device* devs,
                        int32_t* n_devs);

#ifdef __cplusplus
}
#endif
#endif /* KOORD_EVAL_H */
