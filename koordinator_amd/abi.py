"""ctypes mirror of include/koord_eval.h (the C-ABI boundary) and the loader for libkoordeval.so.

Only plain structs cross the boundary; this module is the Python-side equivalent of the cgo binding a
Go koord-scheduler would use.  Struct layouts are checked against the library's own
sizeof() values at load time (ke_abi_struct_sizes).
"""
import ctypes as C
import os

import numpy as np

ABI_VERSION = 13
ABSENT = -1

OK = 0
ERR_INVALID, ERR_UNSUPPORTED, ERR_DEVICE, ERR_NOT_FOUND, ERR_NO_DEVICE = -1, -2, -3, -4, -5

CODE_SUCCESS, CODE_ERROR, CODE_UNSCHEDULABLE, CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, CODE_SKIP = 0, 1, 2, 3, 5

REASON_NONE = 0
REASON_LA_NODEMETRIC_EXPIRED = 1
REASON_LA_USAGE_CPU = 2
REASON_LA_USAGE_MEMORY = 3
REASON_LA_AGG_USAGE_CPU = 4
REASON_LA_AGG_USAGE_MEMORY = 5
REASON_NUMA_INSUFFICIENT_AMPLIFIED_CPU = 16
REASON_NUMA_INVALID_AMPLIFICATION_RATIO = 17
REASON_NUMA_INVALID_CPU_TOPOLOGY = 18
REASON_NUMA_POLICY_CONFLICT = 19
REASON_NUMA_MISSING_RESOURCES = 20
REASON_NUMA_HINT_UNALIGNED = 21
REASON_NUMA_INSUFFICIENT_RESOURCES = 22
NUMA_POLICY_NONE, NUMA_POLICY_BEST_EFFORT, NUMA_POLICY_RESTRICTED, NUMA_POLICY_SINGLE_NUMA_NODE = 0, 1, 2, 3
NUMA_ALLOC_ENTRY, NUMA_ALLOC_CPU, NUMA_ALLOC_MEMORY = 1, 2, 4  # ke_numa_zone.has_allocated bits
NUMA_EXCLUSIVE_NONE, NUMA_EXCLUSIVE_PREFERRED, NUMA_EXCLUSIVE_REQUIRED = 0, 1, 2
CPU_BIND_UNSET, CPU_BIND_DEFAULT, CPU_BIND_FULL_PCPUS, CPU_BIND_SPREAD_BY_PCPUS, CPU_BIND_CONSTRAINED_BURST = 0, 1, 2, 3, 4
CPU_EXCL_NONE, CPU_EXCL_PCPU_LEVEL, CPU_EXCL_NUMA_NODE_LEVEL = 0, 1, 2
NODE_CPU_BIND_NONE, NODE_CPU_BIND_FULL_PCPUS_ONLY, NODE_CPU_BIND_SPREAD_BY_PCPUS = 0, 1, 2
NUMA_ALLOCATE_DEFAULT, NUMA_ALLOCATE_MOST, NUMA_ALLOCATE_LEAST = 0, 1, 2
REASON_NUMA_INVALID_REQUESTED_CPUS, REASON_NUMA_CPU_BIND_POLICY_CONFLICT = 23, 24
REASON_NUMA_SMT_ALIGNMENT, REASON_NUMA_INSUFFICIENT_CPUS = 25, 26
NUMA_STATUS_IDLE, NUMA_STATUS_SINGLE, NUMA_STATUS_SHARED = 0, 1, 2
MAX_NUMA = 8
MAX_CPUS = 256
REASON_DS_INVALID_REQUEST = 32
REASON_DS_INSUFFICIENT_GPU = 33
REASON_DS_INSUFFICIENT_RDMA = 34
REASON_DS_INSUFFICIENT_FPGA = 35
REASON_DS_MISSING_PARTITION_TABLE = 36
REASON_DS_UNSUPPORTED_GPU_REQUESTS = 37
REASON_DS_INSUFFICIENT_PARTITIONED = 38
REASON_DS_MISSING_TOPOLOGY_TREE = 39
REASON_DS_MULTI_SHARED_GPU = 40
REASON_DS_INSUFFICIENT_TOPOLOGY_SCOPED = 41
REASON_DS_INSUFFICIENT_GPU_TOPOLOGY = 42
REASON_DS_INSUFFICIENT_NUMA_SCOPED = 43
REASON_DS_INVALID_HINT = 44
REASON_DS_INSUFFICIENT_RDMA_VF = 45
REASON_DS_INSUFFICIENT_FPGA_VF = 46
REASON_DS_INSUFFICIENT_PRIMARY = 47
REASON_DS_JOINT_VIOLATION = 48
REASON_DS_NO_MATCHED_TEMPLATE = 49
REASON_RSV_INSUFFICIENT_CPUS = 50  # a required reservation affinity whose holding reservations satisfy none
REASON_RSV_INSUFFICIENT_DEVICES = 51
COLL_ALL_GATHER, COLL_MAX, COLL_MIN = 0, 1, 2  # ke_host_collective ops
COLL_U32, COLL_I32, COLL_I64, COLL_U64 = 0, 1, 2, 3  # ... and element types
HOST_COLLECTIVE = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_int64)
REASON_RSV_AFFINITY = 52  # the Reservation Filter of a reservation-affinity pod (reservation/plugin.go:316-318)
REASON_RSV_INSUFFICIENT_NUMA = 53  # an affinity pod's reservations cannot allocate on the NUMA affinity
REASON_FIT_TOO_MANY_PODS, REASON_FIT_INSUFFICIENT_CPU, REASON_FIT_INSUFFICIENT_MEMORY = 64, 65, 66
REASON_FIT_INSUFFICIENT_SCALAR = 67
# ke_pod.gpu_required_topology_scope (apiext.DeviceTopologyScope -> level)
SCOPE_NONE, SCOPE_NODE, SCOPE_NUMA, SCOPE_PCIE, SCOPE_DEVICE, SCOPE_UNKNOWN = range(6)
SCOPES = {"": SCOPE_NONE, "Node": SCOPE_NODE, "NUMANode": SCOPE_NUMA, "PCIe": SCOPE_PCIE, "Device": SCOPE_DEVICE}
# ke_pod.device_hints bits (DeviceAllocateHints fields the evaluator does not model)
DHINT_GPU_VF = 2
DSTRATEGY_NONE, DSTRATEGY_APPLY_FOR_ALL, DSTRATEGY_REQUESTS_AS_COUNT = 0, 1, 2
DEXCL_NONE, DEXCL_DEVICE_LEVEL, DEXCL_PCIE_LEVEL = 0, 1, 2
SEL_IN, SEL_NOT_IN, SEL_EXISTS, SEL_DOES_NOT_EXIST = 0, 1, 2, 3
MAX_LABELS, MAX_SEL_REQS, MAX_SEL_VALUES, MAX_VF_GROUPS = 8, 4, 4, 4
TEMPLATE_KEY_CORE, TEMPLATE_KEY_MEMORY, TEMPLATE_KEY_MEMORY_RATIO = 1, 2, 4
MAX_GPU_PARTITIONS = 64

DEV_GPU, DEV_RDMA, DEV_FPGA = 0, 1, 2
DEV_TYPES = 3
MAX_MINORS = 16
DKEY_GPU_CORE, DKEY_GPU_MEMORY, DKEY_GPU_MEMORY_RATIO = 0, 1, 2
DKEY_RDMA = DKEY_FPGA = 0
DKEYS = 3
PDR = {"nvidia.com/gpu": 0, "amd.com/gpu": 1, "koordinator.sh/gpu": 2, "koordinator.sh/gpu.shared": 3,
       "koordinator.sh/gpu-core": 4, "koordinator.sh/gpu-memory": 5, "koordinator.sh/gpu-memory-ratio": 6,
       "koordinator.sh/rdma": 7, "koordinator.sh/fpga": 8, "dcu.com/gpu": 9}
PDR_COUNT = 10
PDR_GPU = (0, 1, 2, 3, 4, 5, 6, 9)  # the GPU device type's names (DeviceResourceNames[GPU], utils.go:54-69)
# device resources the DeviceShare ABI does not model (utils.go:38-52): Huawei NPU
UNSUPPORTED_DEVICE_RESOURCES = {"huawei.com/npu-core", "huawei.com/npu-cpu", "huawei.com/npu-dvpp"}
DSW_GPU_MEMORY_RATIO, DSW_GPU_MEMORY, DSW_RDMA, DSW_FPGA = 0, 1, 2, 3

RES_CPU, RES_MEMORY, RES_BATCH_CPU, RES_BATCH_MEMORY, RES_MID_CPU, RES_MID_MEMORY = range(6)
RES_COUNT = 6
NRES = 2

PRIORITY_NONE, PRIORITY_PROD, PRIORITY_MID, PRIORITY_BATCH, PRIORITY_FREE = range(5)
QOS_NONE, QOS_LSE, QOS_LSR, QOS_LS, QOS_BE, QOS_SYSTEM = range(6)
AGG_NONE, AGG_AVG, AGG_P50, AGG_P90, AGG_P95, AGG_P99 = range(6)
AGG_TYPES = 6
STRATEGY_LEAST_ALLOCATED, STRATEGY_MOST_ALLOCATED = 0, 1

i64, i32, u8, f64 = C.c_int64, C.c_int32, C.c_uint8, C.c_double


class ResourceMap(C.Structure):
    _fields_ = [("value", i64 * NRES), ("present", u8 * NRES), ("pad", u8 * 2), ("n_keys", i32)]


class LoadAwareArgs(C.Structure):
    _fields_ = [
        ("node_metric_expiration_seconds", i64),
        ("resource_weights", i64 * NRES),
        ("usage_thresholds", i64 * NRES),
        ("prod_usage_thresholds", i64 * NRES),
        ("estimated_scaling_factors", i64 * NRES),
        ("estimated_seconds_after_pod_scheduled", i64),
        ("estimated_seconds_after_initialized", i64),
        ("agg_usage_thresholds", i64 * NRES),
        ("agg_usage_duration_ns", i64),
        ("agg_score_duration_ns", i64),
        ("agg_usage_type", i32),
        ("agg_score_type", i32),
        ("filter_expired_node_metrics", u8),
        ("enable_schedule_when_node_metrics_expired", u8),
        ("score_according_prod_usage", u8),
        ("allow_customize_estimation", u8),
        ("has_aggregated", u8),
        ("has_other_keys", u8),
        ("pad", u8 * 2),
    ]


class NumaArgs(C.Structure):
    _fields_ = [("weights", i64 * NRES), ("strategy", i32), ("numa_strategy", i32), ("default_cpu_bind_policy", i32),
                ("has_other_keys", u8), ("pad", u8 * 3)]


class Cpu(C.Structure):
    _fields_ = [("cpu_id", i32), ("core_id", i32), ("numa_id", i32), ("socket_id", i32), ("ref_count", i32),
                ("exclusive", u8), ("reserved", u8), ("pad", u8 * 2)]


class NumaZone(C.Structure):
    _fields_ = [
        ("id", i32),
        ("has", u8 * NRES),
        ("has_allocated", u8),
        ("numa_status", u8),
        ("capacity", i64 * NRES),
        ("allocated", i64 * NRES),
        ("cpuset_cpus", i32),
        ("single_pods", C.c_int16),
        ("shared_pods", C.c_int16),
    ]


class DeviceShareArgs(C.Structure):
    _fields_ = [("weights", i64 * 4), ("strategy", i32), ("template_matched_keys", u8), ("has_other_keys", u8),
                ("disable_numa_alignment", u8), ("pad", u8)]


class Labels(C.Structure):
    _fields_ = [("n", i32), ("key", i32 * MAX_LABELS), ("value", i32 * MAX_LABELS)]


class LabelRequirement(C.Structure):
    _fields_ = [("key", i32), ("op", i32), ("n_values", i32), ("values", i32 * MAX_SEL_VALUES)]


class LabelSelector(C.Structure):
    _fields_ = [("present", i32), ("n", i32), ("req", LabelRequirement * MAX_SEL_REQS)]


class VfGroup(C.Structure):
    _fields_ = [("labels", Labels), ("pad", i32), ("vfs", C.c_uint64)]


class Device(C.Structure):
    _fields_ = [
        ("type", i32),
        ("minor", i32),
        ("health", u8),
        ("has_total", u8 * DKEYS),
        ("has_used", u8 * DKEYS),
        ("has_topology", u8),
        ("total", i64 * DKEYS),
        ("used", i64 * DKEYS),
        ("numa_node", i32),
        ("pcie_rank", i32),
        ("labels", Labels),
        ("n_vf_groups", i32),
        ("vf_groups", VfGroup * MAX_VF_GROUPS),
        ("vf_allocated", C.c_uint64),
    ]


class DeviceHint(C.Structure):
    _fields_ = [("selector", LabelSelector), ("vf_selector", LabelSelector), ("strategy", i32), ("exclusive", i32)]


class PodDeviceHints(C.Structure):
    _fields_ = [("hint", DeviceHint * DEV_TYPES), ("invalid", i32), ("has_selectors", i32), ("joint_n", i32),
                ("joint_types", i32 * DEV_TYPES), ("joint_same_pcie", i32), ("pad", i32)]


class GpuTemplate(C.Structure):
    _fields_ = [("model_key", i32), ("name", i32), ("has", u8 * DKEYS), ("pad", u8 * 5), ("value", i64 * DKEYS)]


class GpuPartition(C.Structure):
    _fields_ = [("minors", C.c_uint32), ("number_of_gpus", i32), ("allocation_score", i32), ("pad", i32),
                ("ring_bus_bandwidth", i64)]


MAX_XRES = 64
XRES_CPU = 0
XRES_MEMORY = 1
MAX_FITPLUS = 4
MAX_POD_XRES = 8


class FitPlusResource(C.Structure):
    _fields_ = [("id", i32), ("type", i32), ("weight", i64)]


class ExtArgs(C.Structure):
    """NodeResourcesFitPlus / ScarceResourceAvoidance args + profile weights (koord_eval.h ke_ext_args)."""
    _fields_ = [("weight_fitplus", i64), ("weight_sra", i64), ("sra_resources", C.c_uint64), ("n_fitplus", i32),
                ("pad", i32), ("fitplus", FitPlusResource * MAX_FITPLUS)]


class FitArgs(C.Structure):
    """NodeResourcesFit args + profile weight (koord_eval.h ke_fit_args; upstream k8s, parity unpinned)."""
    _fields_ = [("weight", i64), ("strategy", i32), ("n_resources", i32), ("resources", FitPlusResource * MAX_FITPLUS),
                ("n_scalars", i32), ("scalars", i32 * 8), ("filter", u8), ("has_ignored", u8), ("pad", u8 * 2)]


class NodeResource(C.Structure):
    _fields_ = [("id", i32), ("pad", i32), ("allocatable", i64), ("requested", i64)]


class Config(C.Structure):
    _fields_ = [
        ("abi_version", i32),
        ("device_ordinal", i32),
        ("weight_loadaware", i64),
        ("weight_numa", i64),
        ("weight_deviceshare", i64),
        ("loadaware", LoadAwareArgs),
        ("numa", NumaArgs),
        ("deviceshare", DeviceShareArgs),
        ("node_capacity", i32),
        ("pod_batch", i32),
        ("global_node_offset", i32),
        ("weight_reservation", i32),
        ("ext", ExtArgs),
        ("fit", FitArgs),
    ]


class Node(C.Structure):
    _fields_ = [
        ("allocatable", i64 * NRES),
        ("raw_allocatable", i64 * NRES),
        ("requested", i64 * NRES),
        ("cpu_amplification_ratio", f64),
        ("cpuset_allocated_cpus", i64),
        ("custom_usage_thresholds", i64 * NRES),
        ("custom_prod_usage_thresholds", i64 * NRES),
        ("custom_agg_thresholds", i64 * NRES),
        ("custom_agg_duration_ns", i64),
        ("nrt_cpu_amplification_ratio", f64),
        ("custom_agg_type", i32),
        ("numa_topology_policy", i32),
        ("cpu_bind_policy", i32),
        ("has_custom_thresholds", u8),
        ("custom_thresholds_error", u8),
        ("has_custom_agg", u8),
        ("amplification_error", u8),
        ("cpu_topology_invalid", u8),
        ("numa_allocate_strategy", u8),
        ("pad", u8 * 6),
        ("allowed_pods", i32),
        ("pod_count", i32),
    ]


class AggregatedUsage(C.Structure):
    _fields_ = [("duration_ns", i64), ("usage", ResourceMap * AGG_TYPES)]


class PodMetric(C.Structure):
    _fields_ = [("pod_key", i64), ("priority_class", i32), ("pad", i32), ("usage", ResourceMap)]


class NodeMetric(C.Structure):
    _fields_ = [
        ("update_time_ns", i64),
        ("report_interval_seconds", i64),
        ("node_usage", ResourceMap),
        ("has_update_time", u8),
        ("has_node_metric", u8),
        ("pad", u8 * 6),
    ]


class Pod(C.Structure):
    _fields_ = [
        ("pod_key", i64),
        ("uid", i64),
        ("requests", i64 * RES_COUNT),
        ("limits", i64 * RES_COUNT),
        ("custom_scaling_factors", i64 * NRES),
        ("custom_seconds_after_scheduled", i64),
        ("custom_seconds_after_initialized", i64),
        ("scheduled_transition_ns", i64),
        ("initialized_transition_ns", i64),
        ("priority_class", i32),
        ("qos_class", i32),
        ("is_daemonset", u8),
        ("has_custom_scaling_factors", u8),
        ("has_scheduled", u8),
        ("has_initialized", u8),
        ("is_terminated", u8),
        ("has_resource_spec", u8),
        ("has_other_requests", u8),
        ("has_unsupported_device_requests", u8),
        ("device_requests", i64 * PDR_COUNT),
        ("numa_topology_policy", i32),
        ("numa_exclusive", i32),
        ("cpu_bind_required", i32),
        ("cpu_bind_preferred", i32),
        ("cpu_exclusive", i32),
        ("quota", C.c_int16),
        ("quota_non_preemptible", u8),
        ("reservation_matched", u8),
        ("gpu_ring_bus_bandwidth", i64),
        ("gpu_required_topology_scope", i32),
        ("gpu_partition_spec", u8),
        ("gpu_partition_restricted", u8),
        ("device_joint_allocate", u8),
        ("device_hints", u8),
        ("xres_request_mask", C.c_uint64),
        ("n_xres", i32),
        ("xres_id", i32 * MAX_POD_XRES),
        ("device_hint", i32),
        ("xres_value", i64 * MAX_POD_XRES),
    ]


MAX_QUOTAS = 255


class QuotaArgs(C.Structure):
    _fields_ = [("total", i64 * NRES), ("enable_runtime_quota", u8), ("enable_check_parent_quota", u8),
                ("disable_scale_min_quota", u8), ("n_hook_plugins", u8),
                ("enable_guarantee_usage", u8), ("pad", u8 * 3)]


class Quota(C.Structure):
    _fields_ = [
        ("parent", i32),
        ("has_max", u8 * NRES),
        ("has_min", u8 * NRES),
        ("allow_lent_resource", u8),
        ("limit_is_max", u8),
        ("pad", u8 * 2),
        ("max", i64 * NRES),
        ("min", i64 * NRES),
        ("shared_weight", i64 * NRES),
        ("self_request", i64 * NRES),
        ("used", i64 * NRES),
        ("non_preemptible_used", i64 * NRES),
    ]


RELEASE_UNRESERVE, RELEASE_DELETE = 0, 1  # ke_pod_release modes


class PodAllocation(C.Structure):
    """ke_pod_allocation: what one placement reserved (Unreserve / informer-delete record)."""
    _fields_ = [("node", i32), ("quota_assigned", u8), ("pad", u8 * 3), ("cpuset", C.c_uint64 * 4),
                ("numa", i64 * (MAX_NUMA * NRES)), ("device_minors", C.c_uint64),
                ("vf_rank", C.c_int8 * (2 * MAX_MINORS)), ("reservation", i32), ("reservation_generation", i32),
                ("reservation_uid", i64)]


RSV_NONE, RSV_MATCHED, RSV_AFFINITY, RSV_IGNORED = 0, 1, 2, 3  # ke_pod.reservation_matched
RSV_POLICY_DEFAULT, RSV_POLICY_ALIGNED, RSV_POLICY_RESTRICTED = 0, 1, 2
RSV_HOLDS_NUMA, RSV_HOLDS_CPUSET, RSV_HOLDS_DEVICES, RSV_OTHER_ALLOCATABLE = 1, 2, 4, 8  # ke_reservation.holds


class Reservation(C.Structure):  # ke_reservation
    _fields_ = [("node", i32), ("available", u8), ("allocate_once", u8), ("allocate_policy", u8), ("holds", u8),
                ("allocated_pods", i32), ("pad2", i32), ("allocatable", i64 * NRES), ("allocated", i64 * NRES),
                ("order", i64), ("uid", i64), ("reserved", i64 * NRES), ("names_excluded", u8), ("pad3", u8 * 7)]


RSV_RES_PODS = -1  # ke_reservation_resource.id of the "pods" entry


class ReservationResource(C.Structure):  # ke_reservation_resource
    _fields_ = [("id", i32), ("excluded", u8), ("pad", u8 * 3), ("allocatable", i64), ("allocated", i64),
                ("reserved", i64)]


class ReservationAlloc(C.Structure):  # ke_reservation_alloc
    _fields_ = [("numa", i64 * (MAX_NUMA * NRES)), ("owner_numa", i64 * (MAX_NUMA * NRES)),
                ("cpuset", C.c_uint64 * 4), ("owner_cpuset", C.c_uint64 * 4),
                ("device_minors", C.c_uint64), ("owner_device_minors", C.c_uint64),
                ("device", ((i64 * 3) * MAX_MINORS) * 3), ("owner_device", ((i64 * 3) * MAX_MINORS) * 3)]


STRUCTS = [Config, Node, NodeMetric, PodMetric, AggregatedUsage, Pod, ResourceMap, LoadAwareArgs, NumaArgs,
           DeviceShareArgs, Device, NumaZone, Cpu, QuotaArgs, Quota, GpuPartition, ExtArgs, NodeResource,
           PodAllocation, PodDeviceHints, GpuTemplate, Reservation, ReservationAlloc, ReservationResource]
RESERVATION_DTYPE = np.dtype(Reservation)
RESERVATION_RESOURCE_DTYPE = np.dtype(ReservationResource)
RESERVATION_ALLOC_DTYPE = np.dtype(ReservationAlloc)
POD_DEVICE_HINTS_DTYPE = np.dtype(PodDeviceHints)
GPU_TEMPLATE_DTYPE = np.dtype(GpuTemplate)
QUOTA_DTYPE = np.dtype(Quota)

# numpy views of the same layouts (bulk loads)
NODE_DTYPE = np.dtype(Node)
NODE_METRIC_DTYPE = np.dtype(NodeMetric)
POD_METRIC_DTYPE = np.dtype(PodMetric)
AGG_DTYPE = np.dtype(AggregatedUsage)
POD_DTYPE = np.dtype(Pod)
DEVICE_DTYPE = np.dtype(Device)
GPU_PARTITION_DTYPE = np.dtype(GpuPartition)
NUMA_ZONE_DTYPE = np.dtype(NumaZone)
CPU_DTYPE = np.dtype(Cpu)
NODE_RESOURCE_DTYPE = np.dtype(NodeResource)
POD_ALLOCATION_DTYPE = np.dtype(PodAllocation)

ROW_DTYPE = np.dtype([("f", np.int64, (18,)), ("flags", np.uint32), ("pad", np.uint32)])


def resource_csr(resources, n):
    """per reservation a list / array of ke_reservation_resource entries -> (int32 offsets [n + 1], entries)"""
    assert len(resources) == n
    parts = [np.ascontiguousarray(np.asarray(x, RESERVATION_RESOURCE_DTYPE).reshape(-1)) for x in resources]
    off = np.zeros(n + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in parts])
    res = np.concatenate(parts) if off[-1] else np.zeros(1, RESERVATION_RESOURCE_DTYPE)
    return off, np.ascontiguousarray(res)


def struct_array(items, ctype):
    """list of ctypes `ctype` structures | numpy array of np.dtype(ctype) -> contiguous numpy array"""
    dt = np.dtype(ctype)
    if isinstance(items, np.ndarray):
        return np.ascontiguousarray(items, dt)
    arr = np.zeros(len(items), dt)
    if len(items):
        buf = (ctype * len(items))(*items)
        arr[:] = np.frombuffer(buf, dtype=dt, count=len(items))
    return arr


def default_config(node_capacity, pod_batch=64, device_ordinal=0, global_node_offset=0):
    """ke_config with v1beta3 defaults (pkg/scheduler/apis/config/v1beta3/defaults.go:89-153) and the
    default profile's plugin weights 1/1 (config/manager/scheduler-config.yaml:85-94)."""
    cfg = Config()
    cfg.abi_version = ABI_VERSION
    cfg.device_ordinal = device_ordinal
    cfg.weight_loadaware = 1
    cfg.weight_numa = 1
    cfg.weight_deviceshare = 1
    cfg.weight_reservation = 5000  # config/manager/scheduler-config.yaml:91-92
    a = cfg.loadaware
    a.node_metric_expiration_seconds = 180
    a.resource_weights[:] = [1, 1]
    a.usage_thresholds[:] = [65, 95]
    a.prod_usage_thresholds[:] = [ABSENT, ABSENT]
    a.estimated_scaling_factors[:] = [85, 70]
    a.estimated_seconds_after_pod_scheduled = ABSENT
    a.estimated_seconds_after_initialized = ABSENT
    a.agg_usage_thresholds[:] = [ABSENT, ABSENT]
    a.agg_usage_type = AGG_NONE
    a.agg_score_type = AGG_NONE
    a.filter_expired_node_metrics = 1
    a.enable_schedule_when_node_metrics_expired = 0
    cfg.numa.weights[:] = [1, 1]
    cfg.numa.strategy = STRATEGY_LEAST_ALLOCATED
    cfg.numa.default_cpu_bind_policy = CPU_BIND_FULL_PCPUS  # v1beta3/defaults.go:50
    cfg.deviceshare.weights[:] = [1, 1, 1, 1]  # gpu-memory-ratio, gpu-memory, rdma, fpga (defaults.go:218-242)
    cfg.deviceshare.strategy = STRATEGY_LEAST_ALLOCATED
    cfg.node_capacity = node_capacity
    cfg.pod_batch = pod_batch
    cfg.global_node_offset = global_node_offset
    return cfg


_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KOORDEVAL_LIB") or os.path.join(_HERE, "libkoordeval.so")  # override: A/B builds

EXPORTS = {
    # name: (restype, argtypes)
    "ke_create": (C.c_int, [C.POINTER(Config), C.POINTER(C.c_void_p)]),
    "ke_destroy": (None, [C.c_void_p]),
    "ke_last_error": (C.c_char_p, []),
    "ke_abi_version": (C.c_int, []),
    "ke_abi_struct_sizes": (C.c_int, [C.POINTER(i32), i32]),
    "ke_device_available": (C.c_int, []),
    "ke_node_upsert": (C.c_int, [C.c_void_p, i32, C.POINTER(Node)]),
    "ke_nodes_load": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_node_delete": (C.c_int, [C.c_void_p, i32]),
    "ke_node_topology_delete": (C.c_int, [C.c_void_p, i32]),
    "ke_reservations_generation": (i32, [C.c_void_p]),
    "ke_last_pod_latencies": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_node_set_requested": (C.c_int, [C.c_void_p, i32, i64, i64]),
    "ke_node_set_cpuset_allocated": (C.c_int, [C.c_void_p, i32, i64]),
    "ke_nodemetric_upsert": (C.c_int, [C.c_void_p, i32, C.POINTER(NodeMetric), i32, C.c_void_p, i32, C.c_void_p]),
    "ke_nodemetrics_load": (C.c_int, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ke_nodemetric_delete": (C.c_int, [C.c_void_p, i32]),
    "ke_pod_assign": (C.c_int, [C.c_void_p, i32, C.POINTER(Pod), i64]),
    "ke_pod_unassign": (C.c_int, [C.c_void_p, i32, i64]),
    "ke_pods_assign": (C.c_int, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ke_estimate_pod": (C.c_int, [C.c_void_p, C.POINTER(Pod), C.c_void_p]),
    "ke_eval": (C.c_int, [C.c_void_p, i32, C.c_void_p, i64] + [C.c_void_p] * 7),
    "ke_node_devices_set": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p]),
    "ke_node_gpu_partitions": (C.c_int, [C.c_void_p, i32, i32, i32, i32, C.c_void_p]),
    "ke_node_devices_delete": (C.c_int, [C.c_void_p, i32]),
    "ke_node_numa_set": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p]),
    "ke_node_resources_set": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p]),
    "ke_quantity_parse": (C.c_int, [C.c_char_p, C.POINTER(i64), C.POINTER(i64)]),
    "ke_pod_key": (i64, [C.c_char_p, C.c_char_p]),
    "ke_decode_node": (C.c_int, [C.c_char_p, i64, C.POINTER(Node)]),
    "ke_decode_node_metric": (C.c_int, [C.c_char_p, i64, C.POINTER(NodeMetric), i32, C.c_void_p, C.POINTER(i32), i32,
                                        C.c_void_p, C.POINTER(i32)]),
    "ke_decode_pod": (C.c_int, [C.c_char_p, i64, i32, C.c_void_p, C.POINTER(Pod)]),
    "ke_decode_nrt": (C.c_int, [C.c_char_p, i64, C.POINTER(Node), i32, C.c_void_p, C.POINTER(i32), i32, C.c_void_p,
                                C.POINTER(i32)]),
    "ke_decode_device": (C.c_int, [C.c_char_p, i64, i32, C.c_void_p, C.POINTER(i32), i32, C.c_void_p, C.POINTER(i32),
                                   C.POINTER(i32), C.POINTER(i32)]),
    "ke_decode_reservation": (C.c_int, [C.c_char_p, i64, i32, C.c_void_p, C.POINTER(Reservation), C.c_void_p, i32,
                                        C.c_void_p, C.POINTER(i32), C.c_char_p, i32]),
    "ke_node_resources_get": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p, C.POINTER(i32)]),
    "ke_label_id": (i32, [C.c_char_p]),
    "ke_set_pod_device_hints": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_gpu_templates_load": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_node_device_flags": (C.c_int, [C.c_void_p, i32, i32, i32]),
    "ke_reservations_load": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_reservations_load_ex": (C.c_int, [C.c_void_p, i32, C.c_void_p, C.c_void_p]),
    "ke_reservations_load_full": (C.c_int, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ke_reservation_resources_get": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p, C.POINTER(i32)]),
    "ke_reservation_allocs_get": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_reservations_get": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_pod_reservations": (C.c_int, [C.c_void_p, i32, C.c_void_p, C.c_void_p]),
    "ke_node_info_requested": (C.c_int, [C.c_void_p, i32, C.POINTER(i64), C.POINTER(i64)]),
    "ke_decode_pod_device_hints": (C.c_int, [C.c_char_p, i64, C.POINTER(PodDeviceHints), C.POINTER(i32)]),
    "ke_decode_device_flags": (C.c_int, [C.c_char_p, i64, C.c_char_p, i64, C.POINTER(i32), C.POINTER(i32)]),
    "ke_last_device_allocations": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_last_numa_allocations": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_node_cpus_set": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p, i32]),
    "ke_last_cpusets": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_last_allocations": (C.c_int, [C.c_void_p, i32, C.c_void_p]),
    "ke_pod_release": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, i32]),
    "ke_unreserve": (C.c_int, [C.c_void_p, C.c_void_p, i32]),
    "ke_quotas_load": (C.c_int, [C.c_void_p, C.POINTER(QuotaArgs), C.c_void_p, i32]),
    "ke_quota_state": (C.c_int, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ke_schedule": (C.c_int, [C.c_void_p, i32, C.c_void_p, i64, C.c_void_p, C.c_void_p]),
    "ke_schedule_submit": (C.c_int, [C.c_void_p, i32, C.c_void_p, i64, C.c_void_p]),
    "ke_schedule_wait": (C.c_int, [C.c_void_p, i64, C.c_void_p, C.c_void_p]),
    "ke_last_schedule_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(i32), C.c_void_p, i32]),
    "ke_set_profiling": (C.c_int, [C.c_void_p, i32]),
    "ke_last_kernel_stats": (C.c_int, [C.c_void_p] + [C.POINTER(C.c_double)] * 3 + [C.POINTER(i32)]),
    "ke_last_kernel_stats_ex": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(i32), C.POINTER(i32)]),
    "ke_set_pipeline": (C.c_int, [C.c_void_p, i32]),
    "ke_debug_replay_phases": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ke_debug_kernel_phases": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p]),
    "ke_debug_check_records": (C.c_int, [C.c_void_p, i64, C.POINTER(i64)]),
    "ke_last_host_stats": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ke_last_resolve_split": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "ke_debug_resolve_phases": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ke_debug_resolve_subphases": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ke_debug_resolve_wave1": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ke_debug_numa_deferred": (C.c_int, [C.c_void_p, C.POINTER(i64)]),
    "ke_debug_ds_cuts": (C.c_int, [C.c_void_p, C.POINTER(i32)]),
    "ke_debug_rsv_fused": (C.c_int, [C.c_void_p, C.POINTER(i64)]),
    "ke_debug_spec_failed": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "ke_bench_eval_kernel": (C.c_int, [C.c_void_p, i32, C.c_void_p, i64, i32, C.POINTER(C.c_double)]),
    "ke_row_bytes": (C.c_int, []),
    "ke_pod_record_bytes": (C.c_int, []),
    "ke_debug_rows": (C.c_int, [C.c_void_p, i32, i64, C.c_void_p, C.c_void_p]),
    "ke_debug_usage_bound": (i64, [i64, i64]),
    "ke_num_nodes": (i32, [C.c_void_p]),
    "ke_debug_node_state": (C.c_int, [C.c_void_p, i32, C.c_void_p, i32, C.c_void_p, C.c_void_p, i32, C.c_void_p,
                                      C.c_void_p, i32, C.c_void_p, C.c_void_p]),
    "ke_comm_unique_id": (C.c_int, [C.c_void_p, i32]),
    "ke_shard_init": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p]),
    "ke_shard_init_host": (C.c_int, [C.c_void_p, i32, i32, C.c_void_p, C.c_void_p]),
    "ke_shard_range": (C.c_int, [C.c_void_p, C.POINTER(i32), C.POINTER(i32)]),
}
COMM_ID_BYTES = 128

_lib = None


def load_library(path=LIB_PATH):
    """Load libkoordeval.so (built by __graft_entry__.build()).  Raises if missing: there is no
    Python or CPU fallback for the evaluator."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    lib = C.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ke_abi_version() != ABI_VERSION:
        raise RuntimeError("libkoordeval.so ABI version mismatch")
    sizes = (i32 * len(STRUCTS))()
    lib.ke_abi_struct_sizes(sizes, len(STRUCTS))
    for s, n in zip(STRUCTS, sizes):
        if C.sizeof(s) != n:
            raise RuntimeError(f"ABI layout mismatch for {s.__name__}: python {C.sizeof(s)} != C {n}")
    if path == LIB_PATH:
        _lib = lib
    return lib


def ptr(arr):
    """void* of a numpy array (or None)."""
    if arr is None:
        return None
    return C.c_void_p(arr.ctypes.data)


def node_state(fn, h, i):
    """(Node, cpus, zones, devices) of node i from a ke_debug_node_state-shaped call (product or oracle)."""
    node = Node()
    cpus = np.zeros(MAX_CPUS, CPU_DTYPE)
    zones = np.zeros(MAX_NUMA, NUMA_ZONE_DTYPE)
    devs = np.zeros(DEV_TYPES * MAX_MINORS, DEVICE_DTYPE)
    nc, nz, nd = i32(), i32(), i32()
    rc = fn(h, int(i), C.byref(node), MAX_CPUS, ptr(cpus), C.byref(nc), MAX_NUMA, ptr(zones), C.byref(nz),
            len(devs), ptr(devs), C.byref(nd))
    if rc != OK:
        raise RuntimeError(f"node state rc={rc}")
    return node, cpus[:nc.value], zones[:nz.value], devs[:nd.value]
