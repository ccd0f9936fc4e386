"""TEST INFRASTRUCTURE ONLY — ctypes handle over oracle/liboracle.so, the CPU restatement of the
reference plugins (oracle.c).  Importable only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; same method names as koordinator_amd.evaluator.Evaluator so parity tests can drive
both with identical calls.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from koordinator_amd import abi
from koordinator_amd.evaluator import as_pod_array

# or_rsv_state (oracle.h): RestoreReservation's matched state of one reservation
RSV_STATE_DTYPE = np.dtype([
    ("allocatable_cpus", np.uint64, (4,)), ("allocated_cpus", np.uint64, (4,)), ("remained_cpus", np.uint64, (4,)),
    ("numa_in", np.int32), ("pad", np.int32),
    ("numa_allocatable", np.int64, (16,)), ("numa_allocated", np.int64, (16,)), ("numa_remained", np.int64, (16,)),
    ("numa_remained_has", np.uint8, (16,)),
    ("dev_allocatable_minors", np.uint64), ("dev_allocated_minors", np.uint64), ("dev_remained_minors", np.uint64),
    ("dev_allocatable", np.int64, (3, 16, 3)), ("dev_allocated", np.int64, (3, 16, 3)),
    ("dev_remained", np.int64, (3, 16, 3))], align=True)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    V, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "or_create": (V, [C.POINTER(abi.Config), i32]),
        "or_destroy": (None, [V]),
        "or_node_upsert": (C.c_int, [V, i32, C.POINTER(abi.Node)]),
        "or_node_set_requested": (C.c_int, [V, i32, i64, i64]),
        "or_node_set_cpuset_allocated": (C.c_int, [V, i32, i64]),
        "or_nodemetric_upsert": (C.c_int, [V, i32, C.POINTER(abi.NodeMetric), i32, V, i32, V]),
        "or_nodemetric_delete": (C.c_int, [V, i32]),
        "or_pod_assign": (C.c_int, [V, i32, C.POINTER(abi.Pod), i64]),
        "or_pod_unassign": (C.c_int, [V, i32, i64]),
        "or_pods_assign": (C.c_int, [V, i32, V, V, V]),
        "or_la_filter": (C.c_int, [V, C.POINTER(abi.Pod), i32, i64, C.POINTER(C.c_int)]),
        "or_la_score": (i64, [V, C.POINTER(abi.Pod), i32, i64]),
        "or_numa_filter": (C.c_int, [V, C.POINTER(abi.Pod), i32, C.POINTER(C.c_int)]),
        "or_numa_score": (i64, [V, C.POINTER(abi.Pod), i32]),
        "or_estimate_pod": (None, [V, C.POINTER(abi.Pod), V]),
        "or_eval": (C.c_int, [V, i32, V, i64, V, V, V, V, V, V, V, C.c_int]),
        "or_schedule": (C.c_int, [V, i32, V, i64, V, V, V, V, V, C.c_int]),
        "or_node_devices_set": (C.c_int, [V, i32, i32, V]),
        "or_node_devices_delete": (C.c_int, [V, i32]),
        "or_node_delete": (C.c_int, [V, i32]),
        "or_node_topology_delete": (C.c_int, [V, i32]),
        "or_node_gpu_partitions": (C.c_int, [V, i32, i32, i32, i32, V]),
        "or_ds_prefilter": (C.c_int, [V, C.POINTER(abi.Pod), C.POINTER(C.c_int), V, V, V]),
        "or_set_pod_device_hints": (C.c_int, [V, i32, V]),
        "or_gpu_templates_load": (C.c_int, [V, i32, V]),
        "or_reservations_load": (C.c_int, [V, i32, V]),
        "or_reservations_get": (C.c_int, [V, i32, V]),
        "or_reservations_load_ex": (C.c_int, [V, i32, V, V]),
        "or_reservations_load_full": (C.c_int, [V, i32, V, V, V, V]),
        "or_reservation_resources_get": (C.c_int, [V, i32, i32, V, V]),
        "or_restore_state": (C.c_int, [V, i32, V]),
        "or_numa_reserve_from_rsv": (C.c_int, [V, V, i32, V, i32, i32, i32, V]),
        "or_numa_reserve_policy": (C.c_int, [V, V, i32, V, i32, i32, i32, C.c_uint32, V, V]),
        "or_numa_reserve_ignored": (C.c_int, [V, V, i32, V]),
        "or_reservation_allocs_get": (C.c_int, [V, i32, V]),
        "or_pod_reservations": (C.c_int, [V, i32, V, V]),
        "or_last_reservations": (C.c_int, [V, i32, V]),
        "or_reservation_score": (C.c_int64, [V, V]),
        "or_reservation_prescore": (i32, [V, V, V, i32, V, V]),
        "or_reservation_filter": (i32, [V, V, V, i32, i32]),
        "or_rsv_filter_with": (i32, [V, i32, V, i32, V, V, i32, i32]),
        "or_node_info_requested": (C.c_int, [V, i32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "or_node_device_flags": (C.c_int, [V, i32, i32, i32]),
        "or_last_vf_ranks": (C.c_int, [V, i32, V]),
        "or_ds_allocate": (C.c_int, [V, C.POINTER(abi.Pod), i32, i32, i32, V, V, V]),
        "or_ds_score_device": (i64, [V, i32, V, V, V, V, V, V]),
        "or_ds_rsv_direct": (i32, [V, C.POINTER(abi.Pod), i32, i32, V, V, V, V, V, i32, i32, i32, i32, V, V, V]),
        "or_normalize_scores": (None, [V, i32]),
        "or_topology_merge": (C.c_int, [i32, C.c_uint32, i32, V, V, V, V, V, V, V, V, V]),
        "or_node_numa_set": (C.c_int, [V, i32, i32, V]),
        "or_node_cpus_set": (C.c_int, [V, i32, i32, V, i32]),
        "or_node_resources_set": (C.c_int, [V, i32, i32, V]),
        "or_fitplus_score": (i64, [V, C.POINTER(abi.Pod), i32]),
        "or_sra_score": (i64, [V, C.POINTER(abi.Pod), i32]),
        "or_numa_distribute": (C.c_int, [V, i32, V, C.c_uint32, V]),
        "or_numa_allocate": (C.c_int, [V, i32, V, C.c_uint32, V, V]),
        "or_set_exact_cpusets": (None, [C.c_int]),
        "or_numa_exclusive_ok": (C.c_int, [C.c_uint32, i32, V, i32]),
        "or_take_cpus": (C.c_int, [V, i32, i32, V, V, V, i32, i32, i32, i32, V, V]),
        "or_spread_order": (C.c_int, [V, i32, V, i32, V]),
        "or_numa_hints": (C.c_int, [V, i32, V, i32, V, V, V, V, V]),
        "or_ds_filter": (C.c_int, [V, C.POINTER(abi.Pod), i32, C.POINTER(C.c_int)]),
        "or_ds_score": (i64, [V, C.POINTER(abi.Pod), i32]),
        "or_ds_reserve": (C.c_uint64, [V, C.POINTER(abi.Pod), i32]),
        "or_ds_numa_hints": (C.c_int, [V, i32, C.POINTER(abi.Pod), V, V, V, V, V, V, V]),
        "or_ds_numa_allocate": (C.c_int, [V, i32, C.POINTER(abi.Pod), C.c_uint32, V]),
        "or_usage_percent": (i64, [i64, i64]),
        "or_quotas_load": (C.c_int, [V, C.POINTER(abi.QuotaArgs), V, i32]),
        "or_quota_state": (C.c_int, [V, i32, V, V, V, V]),
        "or_pod_release": (C.c_int, [V, V, V, i32]),
        "or_debug_node_state": (C.c_int, [V, i32, V, i32, V, V, i32, V, V, i32, V, V]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


class Oracle:
    def __init__(self, cfg, n_nodes):
        self.lib = load()
        self.cfg = cfg
        self.n = n_nodes
        self.h = self.lib.or_create(C.byref(cfg), n_nodes)

    def close(self):
        if self.h:
            self.lib.or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_nodes(self):
        return self.n

    def upsert_node(self, i, node):
        assert self.lib.or_node_upsert(self.h, i, C.byref(node)) == 0

    def nodes_load(self, nodes):
        for i in range(len(nodes)):
            node = abi.Node.from_buffer_copy(np.ascontiguousarray(nodes[i : i + 1]).tobytes())
            self.upsert_node(i, node)

    def set_requested(self, i, milli_cpu, memory):
        assert self.lib.or_node_set_requested(self.h, i, milli_cpu, memory) == 0

    def set_cpuset_allocated(self, i, cpus):
        assert self.lib.or_node_set_cpuset_allocated(self.h, i, cpus) == 0

    def set_nodemetric(self, i, nm):
        hdr, pms, n_pm, aggs, n_agg = nm
        assert self.lib.or_nodemetric_upsert(self.h, i, C.byref(hdr), n_pm, C.cast(pms, C.c_void_p), n_agg,
                                             C.cast(aggs, C.c_void_p)) == 0

    def nodemetrics_load(self, headers, pm_offsets, pod_metrics, agg_offsets, aggregated):
        headers = np.ascontiguousarray(headers, dtype=abi.NODE_METRIC_DTYPE)
        pod_metrics = np.ascontiguousarray(pod_metrics, dtype=abi.POD_METRIC_DTYPE)
        aggregated = np.ascontiguousarray(aggregated, dtype=abi.AGG_DTYPE)
        for i in range(len(headers)):
            p0, p1 = int(pm_offsets[i]), int(pm_offsets[i + 1])
            a0, a1 = int(agg_offsets[i]), int(agg_offsets[i + 1])
            hdr = abi.NodeMetric.from_buffer_copy(headers[i : i + 1].tobytes())
            pm_ptr = C.c_void_p(pod_metrics.ctypes.data + p0 * abi.POD_METRIC_DTYPE.itemsize) if p1 > p0 else None
            ag_ptr = C.c_void_p(aggregated.ctypes.data + a0 * abi.AGG_DTYPE.itemsize) if a1 > a0 else None
            assert self.lib.or_nodemetric_upsert(self.h, i, C.byref(hdr), p1 - p0, pm_ptr, a1 - a0, ag_ptr) == 0

    def delete_nodemetric(self, i):
        assert self.lib.or_nodemetric_delete(self.h, i) == 0

    def assign(self, i, pod, timestamp_ns):
        assert self.lib.or_pod_assign(self.h, i, C.byref(pod), int(timestamp_ns)) == 0

    def assign_bulk(self, nodes, pods, timestamps_ns):
        nodes = np.ascontiguousarray(nodes, dtype=np.int32)
        pods = as_pod_array(pods)
        ts = np.ascontiguousarray(timestamps_ns, dtype=np.int64)
        assert self.lib.or_pods_assign(self.h, len(nodes), abi.ptr(nodes), abi.ptr(pods), abi.ptr(ts)) == 0

    def unassign(self, i, uid):
        assert self.lib.or_pod_unassign(self.h, i, uid) == 0

    def set_devices(self, i, devices):
        devices = np.ascontiguousarray(devices, dtype=abi.DEVICE_DTYPE)
        assert self.lib.or_node_devices_set(self.h, i, len(devices), abi.ptr(devices)) == 0

    def set_gpu_partitions(self, i, has_table, honor, partitions=None):
        parts = np.ascontiguousarray(partitions if partitions is not None else np.zeros(0, abi.GPU_PARTITION_DTYPE),
                                     dtype=abi.GPU_PARTITION_DTYPE)
        assert self.lib.or_node_gpu_partitions(self.h, i, int(bool(has_table)), int(bool(honor)), len(parts),
                                               abi.ptr(parts)) == 0

    def set_numa(self, i, zones):
        zones = np.ascontiguousarray(zones, dtype=abi.NUMA_ZONE_DTYPE)
        assert self.lib.or_node_numa_set(self.h, i, len(zones), abi.ptr(zones)) == 0

    def delete_devices(self, i):
        assert self.lib.or_node_devices_delete(self.h, i) == 0

    def delete_node(self, i):
        assert self.lib.or_node_delete(self.h, i) == 0

    def delete_topology(self, i):
        assert self.lib.or_node_topology_delete(self.h, i) == 0

    def set_resources(self, i, resources):
        res = np.ascontiguousarray(resources, dtype=abi.NODE_RESOURCE_DTYPE)
        assert self.lib.or_node_resources_set(self.h, i, len(res), abi.ptr(res)) == 0

    def fitplus_score(self, pod, i):
        return self.lib.or_fitplus_score(self.h, C.byref(pod), i)

    def sra_score(self, pod, i):
        return self.lib.or_sra_score(self.h, C.byref(pod), i)

    def set_cpus(self, i, cpus, max_ref_count=1):
        cpus = np.ascontiguousarray(cpus, dtype=abi.CPU_DTYPE)
        assert self.lib.or_node_cpus_set(self.h, i, len(cpus), abi.ptr(cpus), max_ref_count) == 0

    def numa_allocate(self, i, pod, mask):
        """resourceManager.Allocate with hint `mask` (0 = nil): None on error, else (out[16], cpuset words)."""
        out = np.zeros(16, np.int64)
        cpus = np.zeros(4, np.uint64)
        rc = self.lib.or_numa_allocate(self.h, i, C.byref(pod), mask, abi.ptr(out), abi.ptr(cpus))
        return None if rc < 0 else (out, cpus)

    def set_exact_cpusets(self, on):
        """Hints / admit run the CPU accumulator itself (the reference's shape) instead of its counts."""
        self.lib.or_set_exact_cpusets(1 if on else 0)

    def numa_distribute(self, i, pod, mask):
        """(ok, out[16]) of tryBestToDistributeEvenly on NUMA ids `mask` (None if options fail)."""
        out = np.zeros(16, np.int64)
        rc = self.lib.or_numa_distribute(self.h, i, C.byref(pod), mask, abi.ptr(out))
        return None if rc < 0 else (bool(rc), out)

    def numa_hints(self, i, pod, policy):
        """{resource index: [(mask, preferred, score)]} for the resources that have a hint list."""
        masks = np.zeros(2 * 255, np.uint32)
        pref = np.zeros(2 * 255, np.uint8)
        scores = np.zeros(2 * 255, np.int64)
        counts = np.zeros(2, np.int32)
        present = np.zeros(2, np.int32)
        rc = self.lib.or_numa_hints(self.h, i, C.byref(pod), policy, abi.ptr(masks), abi.ptr(pref), abi.ptr(scores),
                                    abi.ptr(counts), abi.ptr(present))
        if rc < 0:
            return None
        return {r: [(int(masks[r * 255 + k]), bool(pref[r * 255 + k]), int(scores[r * 255 + k]))
                    for k in range(counts[r])] for r in range(2) if present[r]}

    # per-plugin entry points (golden vectors)
    def la_filter(self, pod, node, now_ns):
        r = C.c_int()
        code = self.lib.or_la_filter(self.h, C.byref(pod), node, int(now_ns), C.byref(r))
        return code, r.value

    def la_score(self, pod, node, now_ns):
        return self.lib.or_la_score(self.h, C.byref(pod), node, int(now_ns))

    def numa_filter(self, pod, node):
        r = C.c_int()
        code = self.lib.or_numa_filter(self.h, C.byref(pod), node, C.byref(r))
        return code, r.value

    def numa_score(self, pod, node):
        return self.lib.or_numa_score(self.h, C.byref(pod), node)

    def ds_prefilter(self, pod):
        """(code, skip, count[3], req[3][3], req_has[3][3])"""
        skip = C.c_int()
        cnt = np.zeros(3, np.int32)
        req = np.zeros((3, 3), np.int64)
        has = np.zeros((3, 3), np.uint8)
        code = self.lib.or_ds_prefilter(self.h, C.byref(pod), C.byref(skip), abi.ptr(cnt), abi.ptr(req), abi.ptr(has))
        return code, bool(skip.value), cnt, req, has

    def set_pod_device_hints(self, hints):
        """the ke_set_pod_device_hints table (POD_DEVICE_HINTS_DTYPE array); ke_pod.device_hint = 1 + index"""
        h = abi.struct_array(hints, abi.PodDeviceHints)
        assert self.lib.or_set_pod_device_hints(self.h, len(h), abi.ptr(h)) == 0

    def gpu_templates_load(self, templates):
        t = abi.struct_array(templates, abi.GpuTemplate)
        assert self.lib.or_gpu_templates_load(self.h, len(t), abi.ptr(t)) == 0

    def reservations_load(self, reservations, allocs=None, resources=None):
        r = abi.struct_array(reservations, abi.Reservation)
        a = None
        if allocs is not None:
            a = abi.struct_array(allocs, abi.ReservationAlloc)
            assert len(a) == len(r)
        if resources is not None:
            off, res = abi.resource_csr(resources, len(r))
            rc = self.lib.or_reservations_load_full(self.h, len(r), abi.ptr(r), abi.ptr(a) if a is not None else None,
                                                    abi.ptr(off), abi.ptr(res))
        elif a is None:
            rc = self.lib.or_reservations_load(self.h, len(r), abi.ptr(r))
        else:
            rc = self.lib.or_reservations_load_ex(self.h, len(r), abi.ptr(r), abi.ptr(a))
        if rc != 0:
            raise RuntimeError(f"oracle reservations_load rc={rc}")
        self._n_resv = len(r)

    def reservation_resources_get(self, i):
        out = np.zeros(abi.MAX_XRES + 1, abi.RESERVATION_RESOURCE_DTYPE)
        n = C.c_int32()
        assert self.lib.or_reservation_resources_get(self.h, int(i), len(out), abi.ptr(out), C.byref(n)) == 0
        return out[:n.value]

    def numa_reserve_from_rsv(self, pod, node, ids, nom, required):
        """NodeNUMAResource Reserve's allocate-from-reservation (or_numa_reserve_from_rsv): (code, cpuset words)."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        ids = np.ascontiguousarray(ids, np.int32)
        out = np.zeros(4, np.uint64)
        rc = self.lib.or_numa_reserve_from_rsv(self.h, abi.ptr(p), int(node), abi.ptr(ids), len(ids), int(nom),
                                               int(required), abi.ptr(out))
        return rc, out

    def numa_reserve_policy(self, pod, node, ids, nom, required, aff):
        """NodeNUMAResource Reserve under a NUMA policy with a stored affinity (or_numa_reserve_policy):
        (code, NUMA allocation [2*id + r], cpuset words)."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        ids = np.ascontiguousarray(ids, np.int32)
        dist = np.zeros(16, np.int64)
        out = np.zeros(4, np.uint64)
        rc = self.lib.or_numa_reserve_policy(self.h, abi.ptr(p), int(node), abi.ptr(ids), len(ids), int(nom),
                                             int(required), int(aff), abi.ptr(dist), abi.ptr(out))
        return rc, dist, out

    def numa_reserve_ignored(self, pod, node):
        """tryAllocateIgnoreReservation's Reserve on a node without a NUMA policy: (code, cpuset words)."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        out = np.zeros(4, np.uint64)
        rc = self.lib.or_numa_reserve_ignored(self.h, abi.ptr(p), int(node), abi.ptr(out))
        return rc, out

    def restore_state(self, r):
        """RestoreReservation's matched state of reservation r (or_restore_state): a RSV_STATE_DTYPE record."""
        out = np.zeros(1, RSV_STATE_DTYPE)
        assert self.lib.or_restore_state(self.h, int(r), abi.ptr(out)) == 0
        return out[0]

    def reservation_allocs_get(self):
        out = np.zeros(getattr(self, "_n_resv", 0), abi.RESERVATION_ALLOC_DTYPE)
        assert self.lib.or_reservation_allocs_get(self.h, len(out), abi.ptr(out)) == 0
        return out

    def reservations_get(self):
        out = np.zeros(getattr(self, "_n_resv", 0), abi.RESERVATION_DTYPE)
        assert self.lib.or_reservations_get(self.h, len(out), abi.ptr(out)) == 0
        return out

    def pod_reservations(self, matches):
        off = np.zeros(len(matches) + 1, np.int32)
        off[1:] = np.cumsum([len(m) for m in matches])
        ids = np.ascontiguousarray(np.concatenate([np.asarray(m, np.int32) for m in matches]) if len(matches)
                                   else np.zeros(0, np.int32), np.int32)
        assert self.lib.or_pod_reservations(self.h, len(matches), abi.ptr(off), abi.ptr(ids)) == 0

    def reservation_prescore(self, pod, ids):
        """Reservation plugin PreScore + Score of `pod` matching reservations `ids` on every node:
        (preferredNode or -1, raw Score per node, nominated reservation per node)."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        ids = np.ascontiguousarray(ids, np.int32)
        raw = np.zeros(self.n, np.int64)
        nom = np.zeros(self.n, np.int32)
        pref = self.lib.or_reservation_prescore(self.h, abi.ptr(p), abi.ptr(ids), len(ids), abi.ptr(raw), abi.ptr(nom))
        return int(pref), raw, nom

    def reservation_filter(self, pod, ids, node):
        """The Reservation Filter of `pod` with a required reservation affinity over reservations `ids` on `node`."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        ids = np.ascontiguousarray(ids, np.int32)
        return bool(self.lib.or_reservation_filter(self.h, abi.ptr(p), abi.ptr(ids), len(ids), int(node)))

    def rsv_filter_with(self, r, pod, node, pod_requested, r_allocated, required, affinity):
        """filterWithReservations over reservation r alone with the given podRequested / rAllocated (cpu, memory,
        then per resource id): 0 ok, 1 by node, 2 by reservation, 3 none meets."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        pr = np.zeros(abi.NRES + abi.MAX_XRES, np.int64)
        ra = np.zeros(abi.NRES + abi.MAX_XRES, np.int64)
        for dst, src in ((pr, pod_requested), (ra, r_allocated)):
            for k, v in src.items():
                dst[k] = v
        return int(self.lib.or_rsv_filter_with(self.h, int(r), abi.ptr(p), int(node), abi.ptr(pr), abi.ptr(ra),
                                               int(required), int(affinity)))

    def reservation_score(self, reservation, pod):
        """scoreReservation of one reservation record for one pod (golden-vector entry point)."""
        r = abi.struct_array([reservation] if isinstance(reservation, abi.Reservation) else reservation, abi.Reservation)
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        return int(self.lib.or_reservation_score(abi.ptr(r), abi.ptr(p)))

    def node_info_requested(self, i):
        req, nz = (C.c_int64 * 2)(), (C.c_int64 * 2)()
        assert self.lib.or_node_info_requested(self.h, i, req, nz) == 0
        return list(req), list(nz)

    def set_device_flags(self, i, secondary_well_planned, gpu_model_key):
        assert self.lib.or_node_device_flags(self.h, i, int(secondary_well_planned), int(gpu_model_key)) == 0

    def ds_allocate(self, pod, node, reserve=False, scored=False):
        """AutopilotAllocator.Allocate: (status, reason, minors[3], vf_ranks[2][16])"""
        out = np.zeros(3, np.uint32)
        vf = np.zeros((2, abi.MAX_MINORS), np.int8)
        reason = np.zeros(1, np.int32)
        st = self.lib.or_ds_allocate(self.h, C.byref(pod), node, int(reserve), int(scored), abi.ptr(out), abi.ptr(vf),
                                     abi.ptr(reason))
        return st, int(reason[0]), out, vf

    def ds_rsv_direct(self, pod, node, matched, basic, m_alloc, m_allocd, mode=0, required=False, ignored=False,
                      scored=False):
        """DeviceShare's reservation restore state given directly (golden vectors of
        deviceshare/reservation_test.go:225 and scoring_test.go:670): matched = [(policy, allocatable, allocated,
        remained)], each deviceResources map {type: {minor: {key: value}}}.  mode 0 -> (code, reason, minors per type);
        mode 1 -> scoreWithReservation of entry 0."""
        n = len(matched)
        pol = np.array([m[0] for m in matched] or [0], dtype=np.int32)
        mm = np.concatenate([pack_dres(x) for m in matched for x in m[1:]]) if n else np.zeros(192, np.int64)
        out = np.zeros(3, np.uint32)
        score = np.zeros(1, np.int64)
        reason = np.zeros(1, np.int32)
        b, ma, md = pack_dres(basic), pack_dres(m_alloc), pack_dres(m_allocd)  # alive across the call
        code = self.lib.or_ds_rsv_direct(self.h, C.byref(pod), int(node), n, abi.ptr(pol), abi.ptr(mm),
                                         abi.ptr(b), abi.ptr(ma), abi.ptr(md), int(mode), int(required), int(ignored),
                                         int(scored), abi.ptr(out), abi.ptr(score), abi.ptr(reason))
        if mode == 1:
            return int(score[0])
        return int(code), int(reason[0]), [int(x) for x in out]

    def ds_score_device(self, dev_type, req, total, free):
        """each argument: (values[3], has[3])"""
        arrs = [np.ascontiguousarray(x, dtype) for pair in (req, total, free) for x, dtype in
                zip(pair, (np.int64, np.uint8))]
        return self.lib.or_ds_score_device(self.h, dev_type, *[abi.ptr(a) for a in arrs])

    def ds_filter(self, pod, node):
        r = C.c_int()
        code = self.lib.or_ds_filter(self.h, C.byref(pod), node, C.byref(r))
        return code, r.value

    def ds_score(self, pod, node):
        return self.lib.or_ds_score(self.h, C.byref(pod), node)

    def ds_reserve(self, pod, node):
        return self.lib.or_ds_reserve(self.h, C.byref(pod), node)

    def ds_numa_hints(self, pod, node):
        """DeviceShare's NUMA hints: (status, reason, none, copies, [(mask, preferred, score)])"""
        masks, pref, sc = np.zeros(255, np.uint32), np.zeros(255, np.uint8), np.zeros(255, np.int64)
        n, copies, none, reason = (np.zeros(1, np.int32) for _ in range(4))
        st = self.lib.or_ds_numa_hints(self.h, node, C.byref(pod), abi.ptr(masks), abi.ptr(pref), abi.ptr(sc),
                                       abi.ptr(n), abi.ptr(copies), abi.ptr(none), abi.ptr(reason))
        hints = [(int(masks[i]), bool(pref[i]), int(sc[i])) for i in range(int(n[0]))]
        return st, int(reason[0]), bool(none[0]), int(copies[0]), hints

    def ds_numa_allocate(self, pod, node, affinity):
        reason = np.zeros(1, np.int32)
        st = self.lib.or_ds_numa_allocate(self.h, node, C.byref(pod), affinity, abi.ptr(reason))
        return st, int(reason[0])

    def estimate_pod(self, pod):
        est = np.zeros(2, np.int64)
        self.lib.or_estimate_pod(self.h, C.byref(pod), abi.ptr(est))
        return est

    def eval(self, pods, now_ns, n_threads=0):
        pods = as_pod_array(pods)
        P, N = len(pods), self.n
        out = {
            "status": np.zeros((P, N), np.uint8),
            "reason": np.zeros((P, N), np.uint8),
            "la": np.zeros((P, N), np.int16),
            "numa": np.zeros((P, N), np.int16),
            "ds": np.zeros((P, N), np.int16),
            "total": np.zeros((P, N), np.int16),
            "best": np.zeros(P, np.int32),
        }
        rc = self.lib.or_eval(self.h, P, abi.ptr(pods), int(now_ns), abi.ptr(out["status"]), abi.ptr(out["reason"]),
                              abi.ptr(out["la"]), abi.ptr(out["numa"]), abi.ptr(out["ds"]), abi.ptr(out["total"]),
                              abi.ptr(out["best"]), n_threads)
        if rc != 0:
            raise RuntimeError(f"oracle eval rc={rc}")
        return out

    def schedule(self, pods, now_ns, n_threads=0, matches=None):
        pods = as_pod_array(pods)
        if matches is not None:
            self.pod_reservations(matches)
        chosen = np.zeros(len(pods), np.int32)
        score = np.zeros(len(pods), np.int32)
        self.last_device_allocations = np.zeros(len(pods), np.uint64)
        self.last_numa_allocations = np.zeros((len(pods), 16), np.int64)
        self.last_cpusets = np.zeros((len(pods), 4), np.uint64)
        rc = self.lib.or_schedule(self.h, len(pods), abi.ptr(pods), int(now_ns), abi.ptr(chosen), abi.ptr(score),
                                  abi.ptr(self.last_device_allocations), abi.ptr(self.last_numa_allocations),
                                  abi.ptr(self.last_cpusets), n_threads)
        if rc != 0:
            raise RuntimeError(f"oracle schedule rc={rc}")
        self._last = (pods, chosen)
        return chosen, score

    def last_allocations(self, n=None):
        """Release records of the last schedule() (same layout as Evaluator.last_allocations)."""
        pods, chosen = self._last
        n = len(chosen) if n is None else n
        out = np.zeros(n, abi.POD_ALLOCATION_DTYPE)
        out["node"] = chosen[:n]
        placed = chosen[:n] >= 0
        out["quota_assigned"] = placed & (pods["quota"][:n] > 0) & getattr(self, "_has_quotas", False)
        out["cpuset"] = np.where(placed[:, None], self.last_cpusets[:n], 0)
        out["numa"] = np.where(placed[:, None], self.last_numa_allocations[:n], 0)
        out["device_minors"] = np.where(placed, self.last_device_allocations[:n], 0)
        vf = np.full((len(chosen), 2 * abi.MAX_MINORS), -1, np.int8)
        self.lib.or_last_vf_ranks(self.h, len(chosen), abi.ptr(vf))
        out["vf_rank"] = np.where(placed[:, None], vf[:n], -1)
        rv = np.zeros(len(chosen), np.int32)
        self.lib.or_last_reservations(self.h, len(chosen), abi.ptr(rv))
        out["reservation"] = np.where(placed, rv[:n], 0)
        uids = self.reservations_get()["uid"]
        out["reservation_uid"] = [uids[r - 1] if r > 0 else 0 for r in out["reservation"]]
        return out

    def node_state(self, i):
        return abi.node_state(self.lib.or_debug_node_state, self.h, i)

    def release(self, pod, alloc, mode=abi.RELEASE_UNRESERVE):
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        a = np.ascontiguousarray(np.asarray(alloc, abi.POD_ALLOCATION_DTYPE).reshape(1))
        rc = self.lib.or_pod_release(self.h, abi.ptr(p), abi.ptr(a), int(mode))
        if rc != 0:
            raise RuntimeError(f"oracle release rc={rc}")

    def quotas_load(self, args, quotas):
        quotas = np.ascontiguousarray(quotas, abi.QUOTA_DTYPE)
        rc = self.lib.or_quotas_load(self.h, C.byref(args), abi.ptr(quotas), len(quotas))
        if rc != 0:
            raise RuntimeError(f"oracle quotas_load rc={rc}")
        self._has_quotas = True

    def quota_state(self, q):
        return _quota_state(self.lib.or_quota_state, self.h, q)


def _quota_state(fn, h, q):
    limit, used, npu = np.zeros(2, np.int64), np.zeros(2, np.int64), np.zeros(2, np.int64)
    has = np.zeros(2, np.uint8)
    rc = fn(h, int(q), abi.ptr(limit), abi.ptr(has), abi.ptr(used), abi.ptr(npu))
    if rc != 0:
        raise RuntimeError(f"quota state rc={rc}")
    return {"limit": limit, "limit_has": has.astype(bool), "used": used, "np_used": npu}


def pack_dres(d):
    """deviceResources per type -> the 192 int64 or_ds_rsv_direct reads: [type][minor][key 0..2, flags] (flags bit k:
    key k present, bit 3: the minor is in the map)"""
    w = np.zeros((abi.DEV_TYPES, 16, 4), np.int64)
    for t, minors in (d or {}).items():
        for m, keys in minors.items():
            w[t, m, 3] |= 8
            for k, v in keys.items():
                w[t, m, k] = v
                w[t, m, 3] |= 1 << k
    return w.reshape(-1)


def normalize_scores(scores):
    a = np.ascontiguousarray(scores, np.int64).copy()
    load().or_normalize_scores(abi.ptr(a), len(a))
    return a


def usage_percent(used, total):
    return load().or_usage_percent(used, total)


def topology_merge(policy, all_mask, lists):
    """Policy.Merge over raw lists: lists = [(kind, [(mask, preferred, score), ...])]; kind 0 list,
    1 nil list (no preference), 2 empty list.  Returns (admit, mask, preferred, unsatisfied, score)."""
    lib = load()
    kinds = np.array([k for k, _ in lists] or [0], np.int32)
    lens = np.array([len(h) for _, h in lists] or [0], np.int32)
    flat = [x for _, h in lists for x in h]
    masks = np.array([m for m, _, _ in flat] or [0], np.uint32)
    pref = np.array([int(p) for _, p, _ in flat] or [0], np.uint8)
    scores = np.array([s for _, _, s in flat] or [0], np.int64)
    om, op, ou, os_ = C.c_uint32(), C.c_uint8(), C.c_uint8(), C.c_int64()
    admit = lib.or_topology_merge(policy, all_mask, len(lists), abi.ptr(kinds), abi.ptr(lens), abi.ptr(masks),
                                  abi.ptr(pref), abi.ptr(scores), C.byref(om), C.byref(op), C.byref(ou),
                                  C.byref(os_))
    return bool(admit), om.value, bool(op.value), bool(ou.value), os_.value
