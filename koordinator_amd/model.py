"""Kubernetes-object helpers: build the boundary structs (abi.py) from pod/node/NodeMetric descriptions.

This is what a Go caller gets from client-go and the reference's `apis/extension` helpers before it
crosses the C ABI: quantity parsing (k8s.io/apimachinery resource.Quantity, rounding up), pod request
aggregation (resourceapi.PodRequests/PodLimits), kube QoS and koordinator priority/QoS resolution
(apis/extension/priority_utils.go:37-58, qos_utils.go:32-68).  Tests and the bench use it to state
their inputs the way the reference's own tests do.
"""
import math
from fractions import Fraction

import numpy as np

from . import abi

NS = 1_000_000_000

_SUFFIX = {
    "n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000), "": Fraction(1),
    "k": Fraction(10**3), "M": Fraction(10**6), "G": Fraction(10**9), "T": Fraction(10**12),
    "P": Fraction(10**15), "E": Fraction(10**18),
    "Ki": Fraction(2**10), "Mi": Fraction(2**20), "Gi": Fraction(2**30), "Ti": Fraction(2**40),
    "Pi": Fraction(2**50), "Ei": Fraction(2**60),
}

RESOURCE_INDEX = {
    "cpu": abi.RES_CPU,
    "memory": abi.RES_MEMORY,
    "kubernetes.io/batch-cpu": abi.RES_BATCH_CPU,
    "kubernetes.io/batch-memory": abi.RES_BATCH_MEMORY,
    "kubernetes.io/mid-cpu": abi.RES_MID_CPU,
    "kubernetes.io/mid-memory": abi.RES_MID_MEMORY,
}

PRIORITY_BY_NAME = {"koord-prod": abi.PRIORITY_PROD, "koord-mid": abi.PRIORITY_MID,
                    "koord-batch": abi.PRIORITY_BATCH, "koord-free": abi.PRIORITY_FREE}
QOS_BY_NAME = {"LSE": abi.QOS_LSE, "LSR": abi.QOS_LSR, "LS": abi.QOS_LS, "BE": abi.QOS_BE,
               "SYSTEM": abi.QOS_SYSTEM}
AGG_BY_NAME = {"": abi.AGG_NONE, "avg": abi.AGG_AVG, "p50": abi.AGG_P50, "p90": abi.AGG_P90,
               "p95": abi.AGG_P95, "p99": abi.AGG_P99}

PRIORITY_PROD_VALUE_MAX = 9999
PRIORITY_MID_VALUE_MAX = 7999
PRIORITY_BATCH_VALUE_MIN = 5000


def parse_quantity(q):
    """resource.MustParse -> exact rational (decimal/binary SI suffixes, decimal exponents)."""
    if isinstance(q, (int, Fraction)):
        return Fraction(q)
    s = str(q).strip()
    for suf in ("Ki", "Mi", "Gi", "Ti", "Pi", "Ei"):
        if s.endswith(suf):
            return Fraction(s[:-2]) * _SUFFIX[suf]
    if "e" in s[1:] or "E" in s[1:]:
        mant, exp = s.replace("E", "e").split("e")
        return Fraction(mant) * Fraction(10) ** int(exp)
    if s and s[-1] in "numkMGTPE":
        return Fraction(s[:-1]) * _SUFFIX[s[-1]]
    return Fraction(s)


def value(q):  # Quantity.Value(): rounds up
    return math.ceil(parse_quantity(q))


def milli_value(q):  # Quantity.MilliValue(): rounds up
    return math.ceil(parse_quantity(q) * 1000)


def resource_value(name, q):
    """getResourceValue (loadaware/helper.go:147-152): cpu -> MilliValue, else Value."""
    return milli_value(q) if name == "cpu" else value(q)


_keys = {}


def pod_key(namespace, name):
    """Interned NamespacedName -> int64 key (what a Go shim would keep in a map)."""
    k = f"{namespace}/{name}"
    if k not in _keys:
        _keys[k] = len(_keys) + 1
    return _keys[k]


def _sum_lists(lists):
    out = {}
    for rl in lists:
        for k, v in (rl or {}).items():
            out[k] = out.get(k, Fraction(0)) + parse_quantity(v)
    return out


def pod_requests(containers, init_containers=(), overhead=None):
    """resourceapi.PodRequests (k8s v1.28): max(Σ containers, max init container) + overhead."""
    reqs = _sum_lists([c.get("requests") for c in containers])
    for ic in init_containers:
        for k, v in (ic.get("requests") or {}).items():
            reqs[k] = max(reqs.get(k, Fraction(0)), parse_quantity(v))
    for k, v in (overhead or {}).items():
        reqs[k] = reqs.get(k, Fraction(0)) + parse_quantity(v)
    return reqs


def pod_limits(containers, init_containers=(), overhead=None):
    lims = _sum_lists([c.get("limits") for c in containers])
    for ic in init_containers:
        for k, v in (ic.get("limits") or {}).items():
            lims[k] = max(lims.get(k, Fraction(0)), parse_quantity(v))
    for k, v in (overhead or {}).items():
        if k in lims:
            lims[k] = lims[k] + parse_quantity(v)
    return lims


def kube_qos(containers, init_containers=()):
    """k8s GetPodQOS (pkg/apis/core/v1/helper/qos, v1.28) over cpu/memory."""
    requests, limits = {}, {}
    guaranteed = True
    for c in list(containers) + list(init_containers):
        for k, v in (c.get("requests") or {}).items():
            if k in ("cpu", "memory") and parse_quantity(v) != 0:
                requests[k] = requests.get(k, 0) + parse_quantity(v)
        found = set()
        for k, v in (c.get("limits") or {}).items():
            if k in ("cpu", "memory") and parse_quantity(v) != 0:
                found.add(k)
                limits[k] = limits.get(k, 0) + parse_quantity(v)
        if not {"cpu", "memory"} <= found:
            guaranteed = False
    if not requests and not limits:
        return "BestEffort"
    if guaranteed:
        for k, v in requests.items():
            if limits.get(k) != v:
                guaranteed = False
                break
    if guaranteed and len(requests) == len(limits):
        return "Guaranteed"
    return "Burstable"


def priority_class_raw(labels, spec_priority):
    """GetPodPriorityClassRaw (apis/extension/priority.go:73-101)."""
    if "koordinator.sh/priority-class" in labels:
        return PRIORITY_BY_NAME.get(labels["koordinator.sh/priority-class"], abi.PRIORITY_NONE)
    if spec_priority is None:
        return abi.PRIORITY_NONE
    p = spec_priority
    if 9000 <= p <= 9999:
        return abi.PRIORITY_PROD
    if 7000 <= p <= 7999:
        return abi.PRIORITY_MID
    if 5000 <= p <= 5999:
        return abi.PRIORITY_BATCH
    if 3000 <= p <= 3999:
        return abi.PRIORITY_FREE
    return abi.PRIORITY_NONE


def qos_raw(labels):
    return QOS_BY_NAME.get(labels.get("koordinator.sh/qosClass"), abi.QOS_NONE)


def priority_class_with_default(labels, spec_priority, containers, init_containers=(), status_qos=None):
    """GetPodPriorityClassWithDefault (priority_utils.go:37-58); the kube QoS class is Status.QOSClass when set
    (GetKubeQosClass, qos_utils.go:72-78)."""
    p = priority_class_raw(labels, spec_priority)
    if p != abi.PRIORITY_NONE:
        return p
    q = qos_raw(labels)
    if q == abi.QOS_NONE:  # GetPodQoSClassWithKubeQoS
        q = {"Guaranteed": abi.QOS_LSR, "Burstable": abi.QOS_LS, "BestEffort": abi.QOS_BE}[
            status_qos or kube_qos(containers, init_containers)]
    if q in (abi.QOS_SYSTEM, abi.QOS_LSE, abi.QOS_LSR, abi.QOS_LS):
        return abi.PRIORITY_PROD
    if q == abi.QOS_BE:
        return abi.PRIORITY_BATCH
    return abi.PRIORITY_NONE


def _fill_resources(arr, rl):
    other = False
    for i in range(abi.RES_COUNT):
        arr[i] = 0
    for k, v in rl.items():
        if k in RESOURCE_INDEX:
            arr[RESOURCE_INDEX[k]] = milli_value(v) if k == "cpu" else value(v)
        elif v != 0:
            other = True
    return other


# Resource-name ids of NodeResourcesFitPlus / ScarceResourceAvoidance (koord_eval.h KE_XRES_*): cpu and memory
# fixed, every other name interned on first use (a Go shim keeps the same table per context).
XRES_IDS = {"cpu": abi.XRES_CPU, "memory": abi.XRES_MEMORY}
DEFAULT_MILLI_CPU_REQUEST = 100                 # schedutil.DefaultMilliCPURequest
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024      # schedutil.DefaultMemoryRequest


def xres_id(name):
    if name not in XRES_IDS:
        if len(XRES_IDS) >= abi.MAX_XRES:
            raise ValueError("more than 64 resource names")
        XRES_IDS[name] = len(XRES_IDS)
    return XRES_IDS[name]


def is_scalar_resource_name(name):
    """schedutil.IsScalarResourceName (k8s v1.28): extended (qualified, domain outside kubernetes.io, not
    "requests."-prefixed), hugepages-*, kubernetes.io/-prefixed native or attachable-volumes-* resources."""
    if name.startswith(("hugepages-", "attachable-volumes-")) or "kubernetes.io/" in name:
        return True
    i = name.find("/")
    return 0 < i < len(name) - 1 and not name.startswith("requests.")


def _nonzero_request(name, requests):
    """GetNonzeroRequestForResource (node_resource_fit_plus_utils.go:167-203): one container's request, rounded
    as Quantity.MilliValue() / Value()."""
    requests = requests or {}
    if name == "cpu":
        return milli_value(requests["cpu"]) if "cpu" in requests else DEFAULT_MILLI_CPU_REQUEST
    if name == "memory":
        return value(requests["memory"]) if "memory" in requests else DEFAULT_MEMORY_REQUEST
    if name != "ephemeral-storage" and not is_scalar_resource_name(name):
        return 0
    return value(requests[name]) if name in requests else 0


def fitplus_pod_request(name, containers, init_containers=()):
    """calculatePodResourceRequest (node_resource_fit_plus_utils.go:138-165), without pod Overhead."""
    r = sum(_nonzero_request(name, c.get("requests")) for c in containers)
    for ic in init_containers:
        r = max(r, _nonzero_request(name, ic.get("requests")))
    return r


def _fill_xres(p, reqs, containers, init_containers):
    """ke_pod.xres_*: the ids of the names PodRequests holds > 0 and their calculatePodResourceRequest."""
    names = [k for k, v in reqs.items() if v > 0]
    mask = 0
    for k in names:
        mask |= 1 << xres_id(k)
    p.xres_request_mask = mask
    if len(names) > abi.MAX_POD_XRES:
        raise ValueError("more than 8 requested resource names")
    p.n_xres = len(names)
    for e, k in enumerate(names):
        p.xres_id[e] = xres_id(k)
        p.xres_value[e] = fitplus_pod_request(k, containers, init_containers)


def make_node_resources(allocatable, requested=None):
    """NodeInfo Allocatable / (NonZero)Requested by resource id (ke_node_resource table).  `requested` is what
    calculateResourceAllocatableRequest reads: NonZeroRequested for cpu/memory, Requested otherwise."""
    requested = requested or {}
    names = list(dict.fromkeys(list(allocatable) + list(requested)))
    arr = np.zeros(len(names), abi.NODE_RESOURCE_DTYPE)
    for e, k in enumerate(names):
        arr[e]["id"] = xres_id(k)
        arr[e]["allocatable"] = resource_value(k, allocatable.get(k, 0))
        arr[e]["requested"] = resource_value(k, requested.get(k, 0))
    return arr


_uid = [0]


def make_pod(name="pod", namespace="default", requests=None, limits=None, containers=None,
             init_containers=(), overhead=None, priority=None, labels=None, owner_kind=None, uid=None,
             scheduled_at=None, initialized_at=None, custom_factors=None,
             custom_seconds_after_scheduled=None, custom_seconds_after_initialized=None,
             terminated=False, numa_policy=None, numa_exclusive=None, cpu_bind_required=None,
             cpu_bind_preferred=None, cpu_exclusive=None, gpu_partition_spec=None, device_hints=None,
             device_joint_allocate=None, status_qos=None):
    """A pod as the plugins see it.  `requests`/`limits` describe one container (MakePod().Req());
    `containers` gives the full list.  Times are ns.  numa_policy / numa_exclusive: the
    scheduling.koordinator.sh/numa-topology-spec annotation ('BestEffort' | 'Restricted' |
    'SingleNUMANode'; 'Required' | 'Preferred')."""
    labels = dict(labels or {})
    if containers is None:
        containers = [] if requests is None and limits is None else [{"requests": requests or {}, "limits": limits or {}}]
    p = abi.Pod()
    p.pod_key = pod_key(namespace, name)
    if uid is None:
        _uid[0] += 1
        uid = _uid[0]
    p.uid = uid
    reqs = pod_requests(containers, init_containers, overhead)
    lims = pod_limits(containers, init_containers, overhead)
    other = _fill_resources(p.requests, reqs)
    _fill_resources(p.limits, lims)
    p.has_other_requests = 1 if other else 0
    _fill_xres(p, reqs, containers, init_containers)
    for k, v in reqs.items():  # DeviceShare reads PodRequests (utils.go:392-412), Value() of each
        if k in abi.PDR and v != 0:
            p.device_requests[abi.PDR[k]] = value(v)
        elif k in abi.UNSUPPORTED_DEVICE_RESOURCES and v != 0:
            p.has_unsupported_device_requests = 1
    p.custom_scaling_factors[:] = [abi.ABSENT, abi.ABSENT]
    if custom_factors:
        p.has_custom_scaling_factors = 1
        for k, v in custom_factors.items():
            if k in ("cpu", "memory"):
                p.custom_scaling_factors[RESOURCE_INDEX[k]] = int(v)
    p.custom_seconds_after_scheduled = abi.ABSENT if custom_seconds_after_scheduled is None else custom_seconds_after_scheduled
    p.custom_seconds_after_initialized = abi.ABSENT if custom_seconds_after_initialized is None else custom_seconds_after_initialized
    if scheduled_at is not None:
        p.has_scheduled = 1
        p.scheduled_transition_ns = int(scheduled_at)
    if initialized_at is not None:
        p.has_initialized = 1
        p.initialized_transition_ns = int(initialized_at)
    p.priority_class = priority_class_with_default(labels, priority, containers, init_containers, status_qos)
    p.qos_class = qos_raw(labels)
    p.is_daemonset = 1 if owner_kind == "DaemonSet" else 0
    p.is_terminated = 1 if terminated else 0
    p.numa_topology_policy = {None: 0, "": 0, "BestEffort": 1, "Restricted": 2, "SingleNUMANode": 3}[numa_policy]
    p.numa_exclusive = {None: 0, "": 0, "Preferred": 1, "Required": 2}[numa_exclusive]
    # scheduling.koordinator.sh/resource-spec: requiredCPUBindPolicy / preferredCPUBindPolicy /
    # preferredCPUExclusivePolicy
    p.cpu_bind_required = CPU_BIND_BY_NAME[cpu_bind_required]
    p.cpu_bind_preferred = CPU_BIND_BY_NAME[cpu_bind_preferred]
    p.cpu_exclusive = CPU_EXCL_BY_NAME[cpu_exclusive]
    _device_annotations(p, gpu_partition_spec, device_hints, device_joint_allocate)
    return p


def _device_annotations(p, spec, hints, joint):
    """DeviceShare annotations (apis/extension/device_share.go) as utils.go:355-513 parses them:
    spec = GPUPartitionSpec {'allocatePolicy': 'BestEffort'|'Restricted', 'ringBusBandwidth': quantity};
    hints = DeviceAllocateHints {type: {'selector', 'vfSelector', 'allocateStrategy', 'requiredTopologyScope',
    'exclusivePolicy'}}; joint = DeviceJointAllocate {'deviceTypes': [...], 'requiredScope': ...}."""
    p.gpu_ring_bus_bandwidth = abi.ABSENT
    if spec is not None:
        p.gpu_partition_spec = 1
        p.gpu_partition_restricted = 1 if spec.get("allocatePolicy") == "Restricted" else 0
        if spec.get("ringBusBandwidth") is not None:
            p.gpu_ring_bus_bandwidth = value(spec["ringBusBandwidth"])
    bits = 0
    for t, h in (hints or {}).items():
        if h is None:
            continue
        if t == "gpu" and h.get("vfSelector") is not None:  # a GPU VFSelector is not modelled
            bits |= abi.DHINT_GPU_VF
        if t == "gpu" and h.get("requiredTopologyScope"):
            p.gpu_required_topology_scope = abi.SCOPES.get(h["requiredTopologyScope"], abi.SCOPE_UNKNOWN)
    p.device_hints = bits
    if joint:  # parsePodDeviceShareExtensions: keep the requested types without an ApplyForAll hint
        req = {"gpu": any(p.device_requests[i] for i in abi.PDR_GPU), "rdma": p.device_requests[abi.PDR["koordinator.sh/rdma"]] > 0,
               "fpga": p.device_requests[abi.PDR["koordinator.sh/fpga"]] > 0}
        kept = [t for t in joint.get("deviceTypes", [])
                if req.get(t) and ((hints or {}).get(t) or {}).get("allocateStrategy") != "ApplyForAll"]
        p.device_joint_allocate = 1 if kept else 0


DEV_TYPE_IDS = {"gpu": abi.DEV_GPU, "rdma": abi.DEV_RDMA, "fpga": abi.DEV_FPGA}
SEL_OPS = {"In": abi.SEL_IN, "NotIn": abi.SEL_NOT_IN, "Exists": abi.SEL_EXISTS, "DoesNotExist": abi.SEL_DOES_NOT_EXIST}


def label_id(text):
    from . import decode  # the process-wide string table lives in the library (ke_label_id)
    return decode.label_id(text) if text else 0


def make_labels(labels):
    """abi.Labels from a {key: value} dict"""
    out = abi.Labels()
    for k, v in (labels or {}).items():
        out.key[out.n] = label_id(k)
        out.value[out.n] = label_id(v)
        out.n += 1
    return out


def _selector(sel, out):
    """metav1.LabelSelector dict -> abi.LabelSelector (GetFastLabelSelector / LabelSelectorAsSelector);
    returns False when the conversion fails (an invalid operator / value count)"""
    if sel is None:
        return True
    out.present = 1
    ok = True
    for k, v in (sel.get("matchLabels") or {}).items():
        r = out.req[out.n]
        r.key, r.op, r.n_values = label_id(k), abi.SEL_IN, 1
        r.values[0] = label_id(v)
        out.n += 1
    for e in sel.get("matchExpressions") or []:
        r = out.req[out.n]
        r.key = label_id(e["key"])
        vals = e.get("values") or []
        r.n_values = len(vals)
        for i, v in enumerate(vals):
            r.values[i] = label_id(v)
        op = e.get("operator")
        r.op = SEL_OPS.get(op, abi.SEL_DOES_NOT_EXIST)
        if op not in SEL_OPS or (op in ("In", "NotIn")) != bool(vals):
            ok = False
        out.n += 1
    return ok


def make_device_hints(hints=None, joint=None):
    """ke_pod_device_hints from DeviceAllocateHints {type: {'selector', 'vfSelector', 'allocateStrategy',
    'exclusivePolicy'}} and DeviceJointAllocate {'deviceTypes', 'requiredScope'} dicts (utils.go:414-482)."""
    h = abi.PodDeviceHints()
    for t, d in (hints or {}).items():
        d = d or {}
        ok = _selector(d.get("selector"), abi.LabelSelector()) and _selector(d.get("vfSelector"), abi.LabelSelector())
        h.invalid |= 0 if ok else 1
        if d.get("selector") is not None:
            h.has_selectors = 1
        if t not in DEV_TYPE_IDS:
            continue
        x = h.hint[DEV_TYPE_IDS[t]]
        _selector(d.get("selector"), x.selector)
        _selector(d.get("vfSelector"), x.vf_selector)
        x.strategy = {"ApplyForAll": abi.DSTRATEGY_APPLY_FOR_ALL,
                      "RequestsAsCount": abi.DSTRATEGY_REQUESTS_AS_COUNT}.get(d.get("allocateStrategy"), 0)
        x.exclusive = {"DeviceLevel": abi.DEXCL_DEVICE_LEVEL, "PCIeLevel": abi.DEXCL_PCIE_LEVEL}.get(d.get("exclusivePolicy"), 0)
    if joint is not None:
        for t in joint.get("deviceTypes") or []:
            tid = DEV_TYPE_IDS.get(t)
            if tid is None or h.hint[tid].strategy == abi.DSTRATEGY_APPLY_FOR_ALL:
                continue
            if tid not in list(h.joint_types[:h.joint_n]):
                h.joint_types[h.joint_n] = tid
                h.joint_n += 1
        h.joint_same_pcie = 1 if joint.get("requiredScope") == "SamePCIe" else 0
    return h


def make_gpu_template(model_key, name, resources):
    t = abi.GpuTemplate()
    t.model_key, t.name = label_id(model_key), label_id(name)
    for k, v in resources.items():
        slot = {"koordinator.sh/gpu-core": 0, "koordinator.sh/gpu-memory": 1, "koordinator.sh/gpu-memory-ratio": 2}[k]
        t.has[slot] = 1
        t.value[slot] = value(v)
    return t


# GPUPartitionIndexOfNVIDIAHopper (allocator_gpu_helper.go:28-144): {number of GPUs: [minors, ...]}, score 1
HOPPER_PARTITIONS = {1: [[m] for m in range(8)], 2: [[0, 1], [2, 3], [4, 5], [6, 7]],
                     4: [[0, 1, 2, 3], [4, 5, 6, 7]], 8: [list(range(8))]}


def make_gpu_partitions(table):
    """GPUPartitionTable {number_of_gpus: [{'minors': [...], 'allocationScore': s, 'ringBusBandwidth': q}
    or [minors...]]} -> np.ndarray(GPU_PARTITION_DTYPE) in table order (allocationScore defaults to 0, as
    an omitted JSON field; the designated Hopper table gives 1)."""
    rows = []
    for n, parts in table.items():
        for q in parts:
            if not isinstance(q, dict):
                q = {"minors": q}
            rows.append((sum(1 << m for m in q["minors"]), int(n), int(q.get("allocationScore", 0)), 0,
                         abi.ABSENT if q.get("ringBusBandwidth") is None else value(q["ringBusBandwidth"])))
    return np.array(rows, dtype=abi.GPU_PARTITION_DTYPE)


def gpu_partition_state(device_table=None, device_labels=None, node_labels=None):
    """(has_table, honor, partitions) as GPUAllocator.Allocate resolves them (allocator_gpu.go:77-82):
    the Device's table (annotation scheduling.koordinator.sh/gpu-partitions) with the Device's
    partition-policy label, else the designated table of the node's GPU vendor/model labels with the
    node's label (GetDesignatedGPUPartitionIndexer, allocator_gpu_helper.go:146-162)."""
    policy_key, vendor_key, model_key = ("node.koordinator.sh/gpu-partition-policy", "node.koordinator.sh/gpu-vendor",
                                         "node.koordinator.sh/gpu-model")
    if device_table is not None:
        return True, (device_labels or {}).get(policy_key) == "Honor", make_gpu_partitions(device_table)
    labels = node_labels or {}
    honor = labels.get(policy_key) == "Honor"
    if labels.get(vendor_key, "") in ("", "nvidia") and labels.get(model_key) in ("H100", "H800", "H20"):
        table = {n: [{"minors": m, "allocationScore": 1} for m in ms] for n, ms in HOPPER_PARTITIONS.items()}
        return True, honor, make_gpu_partitions(table)
    return False, honor, None


CPU_BIND_BY_NAME = {None: 0, "": 0, "Default": 1, "FullPCPUs": 2, "SpreadByPCPUs": 3, "ConstrainedBurst": 4}
CPU_EXCL_BY_NAME = {None: 0, "": 0, "None": 0, "PCPULevel": 1, "NUMANodeLevel": 2}
NODE_CPU_BIND_BY_NAME = {None: 0, "": 0, "None": 0, "FullPCPUsOnly": 1, "SpreadByPCPUs": 2}


def make_cpus(rows, allocated=None, reserved=()):
    """A node's CPU table: rows [cpu, core, numa, socket]; allocated {cpu: (ref_count, exclusive name)}."""
    arr = np.zeros(len(rows), dtype=abi.CPU_DTYPE)
    for i, (cpu, core, numa, sock) in enumerate(rows):
        arr[i]["cpu_id"], arr[i]["core_id"], arr[i]["numa_id"], arr[i]["socket_id"] = cpu, core, numa, sock
        ref, excl = (allocated or {}).get(cpu, (0, None))
        arr[i]["ref_count"] = ref
        arr[i]["exclusive"] = CPU_EXCL_BY_NAME[excl]
        arr[i]["reserved"] = 1 if cpu in reserved else 0
    return arr


def _thr(arr, m):
    arr[:] = [abi.ABSENT, abi.ABSENT]
    for k, v in (m or {}).items():
        arr[RESOURCE_INDEX[k]] = int(v)


def make_node(allocatable=None, requested=None, raw_allocatable=None, amplification_ratio=None,
              nrt_amplification_ratio=None, cpuset_allocated_cpus=0, custom_usage_thresholds=None,
              custom_prod_usage_thresholds=None, custom_aggregated=None, custom_thresholds_error=False,
              amplification_error=False, cpu_topology_invalid=False):
    """A Node (+ NodeInfo.Requested).  custom_* model the usage-thresholds annotation
    (apis/extension/load_aware.go:30-72); custom_aggregated = dict(thresholds=, type=, duration_ns=)."""
    n = abi.Node()
    allocatable = allocatable or {}
    n.allocatable[:] = [milli_value(allocatable.get("cpu", 0)), value(allocatable.get("memory", 0))]
    if "pods" in allocatable:  # NodeInfo.Allocatable.AllowedPodNumber
        n.allowed_pods = min(value(allocatable["pods"]), 2**31 - 1)
    n.raw_allocatable[:] = [abi.ABSENT, abi.ABSENT]
    for k, v in (raw_allocatable or {}).items():
        n.raw_allocatable[RESOURCE_INDEX[k]] = resource_value(k, v)
    requested = requested or {}
    n.requested[:] = [milli_value(requested.get("cpu", 0)), value(requested.get("memory", 0))]
    n.cpu_amplification_ratio = -1.0 if amplification_ratio is None else float(amplification_ratio)
    n.nrt_cpu_amplification_ratio = -2.0 if nrt_amplification_ratio is None else float(nrt_amplification_ratio)
    n.cpuset_allocated_cpus = cpuset_allocated_cpus
    has_custom = custom_usage_thresholds is not None or custom_prod_usage_thresholds is not None or custom_aggregated is not None
    n.has_custom_thresholds = 1 if has_custom else 0
    _thr(n.custom_usage_thresholds, custom_usage_thresholds)
    _thr(n.custom_prod_usage_thresholds, custom_prod_usage_thresholds)
    _thr(n.custom_agg_thresholds, (custom_aggregated or {}).get("thresholds"))
    if custom_aggregated is not None:
        n.has_custom_agg = 1
        n.custom_agg_type = AGG_BY_NAME[custom_aggregated.get("type", "")]
        n.custom_agg_duration_ns = int(custom_aggregated.get("duration_ns", 0))
    n.custom_thresholds_error = 1 if custom_thresholds_error else 0
    n.amplification_error = 1 if amplification_error else 0
    n.cpu_topology_invalid = 1 if cpu_topology_invalid else 0
    return n


def resource_map(rl):
    m = abi.ResourceMap()
    rl = rl or {}
    for k, v in rl.items():
        if k in ("cpu", "memory"):
            i = RESOURCE_INDEX[k]
            m.value[i] = resource_value(k, v)
            m.present[i] = 1
    m.n_keys = len(rl)
    return m


def make_node_metric(update_time=None, report_interval_seconds=None, node_usage=None, has_node_metric=True,
                     pods=(), aggregated=()):
    """NodeMetric (slo/v1alpha1).  pods: [dict(namespace, name, priority('koord-prod'...), usage)];
    aggregated: [dict(duration_ns, usage={'p95': {...}})].  Returns (header, pod_metrics, aggregated)."""
    nm = abi.NodeMetric()
    if update_time is not None:
        nm.has_update_time = 1
        nm.update_time_ns = int(update_time)
    nm.report_interval_seconds = abi.ABSENT if report_interval_seconds is None else report_interval_seconds
    nm.has_node_metric = 1 if has_node_metric else 0
    nm.node_usage = resource_map(node_usage)
    pms = (abi.PodMetric * max(len(pods), 1))()
    for i, pm in enumerate(pods):
        pms[i].pod_key = pod_key(pm.get("namespace", "default"), pm["name"])
        pms[i].priority_class = PRIORITY_BY_NAME.get(pm.get("priority", ""), abi.PRIORITY_NONE)
        pms[i].usage = resource_map(pm.get("usage"))
    aggs = (abi.AggregatedUsage * max(len(aggregated), 1))()
    for i, ag in enumerate(aggregated):
        aggs[i].duration_ns = int(ag["duration_ns"])
        for t, rl in ag.get("usage", {}).items():
            aggs[i].usage[AGG_BY_NAME[t]] = resource_map(rl)
    return nm, pms, len(pods), aggs, len(aggregated)


DEVICE_TYPE_BY_NAME = {"gpu": abi.DEV_GPU, "rdma": abi.DEV_RDMA, "fpga": abi.DEV_FPGA}
DEVICE_KEYS = {
    abi.DEV_GPU: {"koordinator.sh/gpu-core": abi.DKEY_GPU_CORE, "koordinator.sh/gpu-memory": abi.DKEY_GPU_MEMORY,
                  "koordinator.sh/gpu-memory-ratio": abi.DKEY_GPU_MEMORY_RATIO},
    abi.DEV_RDMA: {"koordinator.sh/rdma": abi.DKEY_RDMA},
    abi.DEV_FPGA: {"koordinator.sh/fpga": abi.DKEY_FPGA},
}


def make_devices(devices):
    """DeviceShare node device cache entries: [dict(type='gpu'|'rdma'|'fpga', minor, health=True,
    total={resource: quantity}, used={resource: quantity}, topology={'nodeID': n, 'pcieID': str} | None)]
    -> np.ndarray(DEVICE_DTYPE)."""
    arr = np.zeros(len(devices), dtype=abi.DEVICE_DTYPE)
    pcie_ids = sorted({str(d["topology"].get("pcieID", "")) for d in devices if d.get("topology") is not None},
                      key=lambda x: x.encode())
    for i, d in enumerate(devices):
        t = DEVICE_TYPE_BY_NAME[d["type"]]
        dev = abi.Device()
        dev.type = t
        dev.minor = int(d["minor"])
        dev.health = 1 if d.get("health", True) else 0
        topo = d.get("topology")
        if topo is not None:  # DeviceInfo.Topology: NodeID + the PCIEID's rank in Go string order
            dev.has_topology = 1
            dev.numa_node = int(topo.get("nodeID", 0))
            dev.pcie_rank = pcie_ids.index(str(topo.get("pcieID", "")))
        for field, hfield, rl in (("total", "has_total", d.get("total")), ("used", "has_used", d.get("used"))):
            for k, q in (rl or {}).items():
                key = DEVICE_KEYS[t][k]
                getattr(dev, hfield)[key] = 1
                getattr(dev, field)[key] = value(q)
        dev.labels = make_labels(d.get("labels"))
        # VFGroups: VF rank = position of its BusID among the device's VFs in string order
        groups = d.get("vf_groups") or []
        bus = sorted((vf, g) for g, grp in enumerate(groups) for vf in grp.get("vfs", []))
        if t != abi.DEV_GPU:
            dev.n_vf_groups = len(groups)
            for g, grp in enumerate(groups):
                dev.vf_groups[g].labels = make_labels(grp.get("labels"))
            for r, (vf, g) in enumerate(bus):
                dev.vf_groups[g].vfs |= 1 << r
                if vf in (d.get("vf_allocated") or ()):
                    dev.vf_allocated |= 1 << r
        arr[i] = np.frombuffer(bytes(dev), dtype=abi.DEVICE_DTYPE)[0]
    return arr


def make_zones(zones):
    """NodeResourceTopology zones + the resource manager's allocation: [dict(id, cpu=quantity | None,
    memory=quantity | None, allocated={'cpu':..., 'memory':...} | None, cpuset_cpus=0)] ->
    np.ndarray(NUMA_ZONE_DTYPE).  A resource left out is absent from the zone's ResourceList; the
    allocation entry holds exactly the keys given in `allocated` ({} = an entry without keys)."""
    arr = np.zeros(len(zones), dtype=abi.NUMA_ZONE_DTYPE)
    for i, z in enumerate(zones):
        arr[i]["id"] = int(z["id"])
        for r, name in ((0, "cpu"), (1, "memory")):
            if z.get(name) is not None:
                arr[i]["has"][r] = 1
                arr[i]["capacity"][r] = resource_value(name, z[name])
        al = z.get("allocated")
        if al is not None:
            arr[i]["has_allocated"] = (abi.NUMA_ALLOC_ENTRY | (abi.NUMA_ALLOC_CPU if "cpu" in al else 0)
                                       | (abi.NUMA_ALLOC_MEMORY if "memory" in al else 0))
            arr[i]["allocated"][:] = [milli_value(al.get("cpu", 0)), value(al.get("memory", 0))]
        arr[i]["cpuset_cpus"] = int(z.get("cpuset_cpus", 0))
        arr[i]["numa_status"] = {"idle": 0, "single": 1, "shared": 2}[z.get("status", "idle")]
    return arr
