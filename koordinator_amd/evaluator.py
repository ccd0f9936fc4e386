"""Python handle over the C ABI (libkoordeval.so): the same calls a Go koord-scheduler makes via cgo.

`Evaluator` owns one ke_ctx (one GPU, one node shard).  State ingestion mirrors the informer events
the reference plugins consume; `eval` is the parity-mode Filter/Score matrix and `schedule` the
queue scheduler (findNodesThatFitPod + score + selectHost + Reserve per pod, exact speculative
batching on the device).  There is no CPU fallback: evaluation without the HIP device raises.
"""
import ctypes as C

import numpy as np

from . import abi


class KoordEvalError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"koord-eval error {code}: {msg}")
        self.code = code


def as_pod_array(pods):
    """list[abi.Pod] | np.ndarray(POD_DTYPE) -> contiguous np.ndarray(POD_DTYPE)."""
    if isinstance(pods, np.ndarray):
        assert pods.dtype == abi.POD_DTYPE
        return np.ascontiguousarray(pods)
    arr = np.zeros(len(pods), dtype=abi.POD_DTYPE)
    if len(pods):
        buf = (abi.Pod * len(pods))(*pods)
        arr[:] = np.frombuffer(buf, dtype=abi.POD_DTYPE, count=len(pods))
    return arr


class Evaluator:
    def __init__(self, cfg, lib=None):
        self.lib = lib or abi.load_library()
        self.cfg = cfg
        h = C.c_void_p()
        self._check(self.lib.ke_create(C.byref(cfg), C.byref(h)))
        self.h = h
        self._last_n, self._last_out = 0, {}
        self._inflight = {}  # ticket -> the submitted pod array (ke_schedule_submit reads it until the wait)

    # ---- plumbing --------------------------------------------------------------------------
    def _check(self, rc):
        if rc != abi.OK:
            raise KoordEvalError(rc, self.lib.ke_last_error().decode())
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.lib.ke_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def device(self):
        return bool(self.lib.ke_device_available())

    @property
    def num_nodes(self):
        return self.lib.ke_num_nodes(self.h)

    # ---- state ingestion --------------------------------------------------------------------
    def upsert_node(self, i, node):
        self._check(self.lib.ke_node_upsert(self.h, i, C.byref(node)))

    def nodes_load(self, nodes):
        nodes = np.ascontiguousarray(nodes, dtype=abi.NODE_DTYPE)
        self._check(self.lib.ke_nodes_load(self.h, len(nodes), abi.ptr(nodes)))

    def set_requested(self, i, milli_cpu, memory):
        self._check(self.lib.ke_node_set_requested(self.h, i, milli_cpu, memory))

    def set_cpuset_allocated(self, i, cpus):
        self._check(self.lib.ke_node_set_cpuset_allocated(self.h, i, cpus))

    def set_nodemetric(self, i, nm):
        """nm = model.make_node_metric(...) tuple."""
        hdr, pms, n_pm, aggs, n_agg = nm
        self._check(self.lib.ke_nodemetric_upsert(self.h, i, C.byref(hdr), n_pm, C.cast(pms, C.c_void_p), n_agg,
                                                   C.cast(aggs, C.c_void_p)))

    def nodemetrics_load(self, headers, pm_offsets, pod_metrics, agg_offsets, aggregated):
        headers = np.ascontiguousarray(headers, dtype=abi.NODE_METRIC_DTYPE)
        pm_offsets = np.ascontiguousarray(pm_offsets, dtype=np.int64)
        agg_offsets = np.ascontiguousarray(agg_offsets, dtype=np.int64)
        pod_metrics = np.ascontiguousarray(pod_metrics, dtype=abi.POD_METRIC_DTYPE)
        aggregated = np.ascontiguousarray(aggregated, dtype=abi.AGG_DTYPE)
        self._check(self.lib.ke_nodemetrics_load(self.h, len(headers), abi.ptr(headers), abi.ptr(pm_offsets),
                                                 abi.ptr(pod_metrics), abi.ptr(agg_offsets), abi.ptr(aggregated)))

    def delete_nodemetric(self, i):
        self._check(self.lib.ke_nodemetric_delete(self.h, i))

    def delete_node(self, i):
        """Node informer delete (ke_node_delete): out of the snapshot, other caches kept."""
        self._check(self.lib.ke_node_delete(self.h, i))

    def delete_topology(self, i):
        """NodeResourceTopology delete (ke_node_topology_delete)."""
        self._check(self.lib.ke_node_topology_delete(self.h, i))

    def assign(self, i, pod, timestamp_ns):
        self._check(self.lib.ke_pod_assign(self.h, i, C.byref(pod), int(timestamp_ns)))

    def assign_bulk(self, nodes, pods, timestamps_ns):
        nodes = np.ascontiguousarray(nodes, dtype=np.int32)
        pods = as_pod_array(pods)
        ts = np.ascontiguousarray(timestamps_ns, dtype=np.int64)
        self._check(self.lib.ke_pods_assign(self.h, len(nodes), abi.ptr(nodes), abi.ptr(pods), abi.ptr(ts)))

    def unassign(self, i, uid):
        self._check(self.lib.ke_pod_unassign(self.h, i, uid))

    def set_devices(self, i, devices):
        """DeviceShare node device cache entry (model.make_devices(...))."""
        devices = np.ascontiguousarray(devices, dtype=abi.DEVICE_DTYPE)
        self._check(self.lib.ke_node_devices_set(self.h, i, len(devices), abi.ptr(devices)))

    def delete_devices(self, i):
        self._check(self.lib.ke_node_devices_delete(self.h, i))

    def set_pod_device_hints(self, hints):
        """ke_set_pod_device_hints: the DeviceAllocateHints / DeviceJointAllocate table (POD_DEVICE_HINTS_DTYPE)
        ke_pod.device_hint indexes (1 + index)."""
        h = abi.struct_array(hints, abi.PodDeviceHints)
        self._check(self.lib.ke_set_pod_device_hints(self.h, len(h), abi.ptr(h)))

    def gpu_templates_load(self, templates):
        """ke_gpu_templates_load: GPU shared resource templates (GPU_TEMPLATE_DTYPE)."""
        t = abi.struct_array(templates, abi.GpuTemplate)
        self._check(self.lib.ke_gpu_templates_load(self.h, len(t), abi.ptr(t)))

    def reservations_load(self, reservations, allocs=None, resources=None):
        """ke_reservations_load(_ex / _full): the reservation cache (RESERVATION_DTYPE array), optionally each one's
        NUMA / cpuset / device holdings (RESERVATION_ALLOC_DTYPE array, one per reservation) and its allocatable
        names beyond cpu / memory (`resources`: per reservation a RESERVATION_RESOURCE_DTYPE array or list)."""
        r = abi.struct_array(reservations, abi.Reservation)
        a = None
        if allocs is not None:
            a = abi.struct_array(allocs, abi.ReservationAlloc)
            assert len(a) == len(r)
        if resources is not None:
            off, res = abi.resource_csr(resources, len(r))
            self._check(self.lib.ke_reservations_load_full(self.h, len(r), abi.ptr(r), abi.ptr(a) if a is not None else None,
                                                           abi.ptr(off), abi.ptr(res)))
        elif a is None:
            self._check(self.lib.ke_reservations_load(self.h, len(r), abi.ptr(r)))
        else:
            self._check(self.lib.ke_reservations_load_ex(self.h, len(r), abi.ptr(r), abi.ptr(a)))
        self._n_resv = len(r)

    def reservation_resources_get(self, i):
        """ke_reservation_resources_get: reservation i's entries beyond cpu / memory as Reserve / release left them."""
        out = np.zeros(abi.MAX_XRES + 1, abi.RESERVATION_RESOURCE_DTYPE)
        n = C.c_int32()
        self._check(self.lib.ke_reservation_resources_get(self.h, int(i), len(out), abi.ptr(out), C.byref(n)))
        return out[:n.value]

    def reservation_allocs_get(self):
        """ke_reservation_allocs_get: the holdings with the owner parts as Reserve / release left them."""
        out = np.zeros(getattr(self, "_n_resv", 0), abi.RESERVATION_ALLOC_DTYPE)
        self._check(self.lib.ke_reservation_allocs_get(self.h, len(out), abi.ptr(out)))
        return out

    def reservations_get(self):
        """ke_reservations_get: the reservation cache as Reserve / Unreserve left it."""
        out = np.zeros(getattr(self, "_n_resv", 0), abi.RESERVATION_DTYPE)
        self._check(self.lib.ke_reservations_get(self.h, len(out), abi.ptr(out)))
        return out

    def pod_reservations(self, matches):
        """ke_pod_reservations: per pod of the next schedule() the reservation indices it matches."""
        off = np.zeros(len(matches) + 1, np.int32)
        off[1:] = np.cumsum([len(m) for m in matches])
        ids = np.ascontiguousarray(np.concatenate([np.asarray(m, np.int32) for m in matches]) if len(matches)
                                   else np.zeros(0, np.int32), np.int32)
        self._check(self.lib.ke_pod_reservations(self.h, len(matches), abi.ptr(off), abi.ptr(ids)))

    def node_info_requested(self, i):
        """ke_node_info_requested: NodeInfo Requested / NonZeroRequested (MilliCPU, Memory) after the restore."""
        req, nz = (C.c_int64 * 2)(), (C.c_int64 * 2)()
        self._check(self.lib.ke_node_info_requested(self.h, i, req, nz))
        return list(req), list(nz)

    def set_device_flags(self, i, secondary_well_planned, gpu_model_key):
        """ke_node_device_flags: the Device's secondary-well-planned label and the node's GPU template key."""
        self._check(self.lib.ke_node_device_flags(self.h, i, int(secondary_well_planned), int(gpu_model_key)))

    def set_gpu_partitions(self, i, has_table, honor, partitions=None):
        """The node's GPU partition indexer + policy (model.gpu_partition_state(...))."""
        parts = np.ascontiguousarray(partitions if partitions is not None else np.zeros(0, abi.GPU_PARTITION_DTYPE),
                                     dtype=abi.GPU_PARTITION_DTYPE)
        self._check(self.lib.ke_node_gpu_partitions(self.h, i, int(bool(has_table)), int(bool(honor)), len(parts),
                                                    abi.ptr(parts)))

    def set_numa(self, i, zones):
        """NodeResourceTopology NUMA zones + their allocation (model.make_zones(...))."""
        zones = np.ascontiguousarray(zones, dtype=abi.NUMA_ZONE_DTYPE)
        self._check(self.lib.ke_node_numa_set(self.h, i, len(zones), abi.ptr(zones)))

    def set_resources(self, i, resources):
        """NodeResourcesFitPlus / ScarceResourceAvoidance table of node i (np.ndarray NODE_RESOURCE_DTYPE)."""
        res = np.ascontiguousarray(resources, dtype=abi.NODE_RESOURCE_DTYPE)
        self._check(self.lib.ke_node_resources_set(self.h, i, len(res), abi.ptr(res)))

    def get_resources(self, i):
        out = np.zeros(abi.MAX_XRES, abi.NODE_RESOURCE_DTYPE)
        n = abi.i32()
        self._check(self.lib.ke_node_resources_get(self.h, i, abi.MAX_XRES, abi.ptr(out), C.byref(n)))
        return out[:n.value]

    def set_cpus(self, i, cpus, max_ref_count=1):
        """CPU topology + cpuset allocation state (model.make_cpus(...)); an empty table clears it."""
        cpus = np.ascontiguousarray(cpus, dtype=abi.CPU_DTYPE)
        self._check(self.lib.ke_node_cpus_set(self.h, i, len(cpus), abi.ptr(cpus), max_ref_count))

    def estimate_pod(self, pod):
        est = np.zeros(2, np.int64)
        self._check(self.lib.ke_estimate_pod(self.h, C.byref(pod), abi.ptr(est)))
        return est

    # ---- node sharding (one process per GPU) ------------------------------------------------
    def shard_init(self, rank, world, unique_id=None):
        """Collective over `world` ranks with the same RCCL `unique_id` (bytes from comm_unique_id on
        rank 0); unique_id=None with world > 1 runs every shard in this context (loopback)."""
        buf = None
        if unique_id is not None:
            assert len(unique_id) == abi.COMM_ID_BYTES
            buf = C.create_string_buffer(bytes(unique_id), abi.COMM_ID_BYTES)
        self._check(self.lib.ke_shard_init(self.h, rank, world, buf))

    def shard_init_host(self, rank, world, collective):
        """ke_shard_init_host: the sharded path with its collectives carried on the host by
        collective(op, dtype, send: np.ndarray, world) -> np.ndarray (all-gather: world * len(send) elements
        rank-major; max / min: len(send) elements), e.g. koordinator_amd.shard.gloo_collective()."""
        dts = {abi.COLL_U32: np.uint32, abi.COLL_I32: np.int32, abi.COLL_I64: np.int64, abi.COLL_U64: np.uint64}

        def cb(user, op, dtype, send, recv, count):
            try:
                dt = np.dtype(dts[dtype])
                n = int(count)
                src = np.frombuffer((C.c_uint8 * (n * dt.itemsize)).from_address(send), dtype=dt).copy()
                out = np.ascontiguousarray(collective(int(op), dt, src, world), dtype=dt)
                m = n * (world if op == abi.COLL_ALL_GATHER else 1)
                assert out.size == m
                C.memmove(recv, out.ctypes.data, m * dt.itemsize)
                return 0
            except Exception:  # the library fails the call (KE_ERR_DEVICE)
                import traceback
                traceback.print_exc()
                return 1

        self._collective = abi.HOST_COLLECTIVE(cb)  # kept alive with the context
        self._check(self.lib.ke_shard_init_host(self.h, rank, world, self._collective, None))

    def shard_range(self):
        lo, hi = abi.i32(), abi.i32()
        self._check(self.lib.ke_shard_range(self.h, C.byref(lo), C.byref(hi)))
        return lo.value, hi.value

    # ---- evaluation -------------------------------------------------------------------------
    def eval(self, pods, now_ns):
        pods = as_pod_array(pods)
        P, N = len(pods), self.num_nodes
        out = {
            "status": np.zeros((P, N), np.uint8),
            "reason": np.zeros((P, N), np.uint8),
            "la": np.zeros((P, N), np.int16),
            "numa": np.zeros((P, N), np.int16),
            "ds": np.zeros((P, N), np.int16),
            "total": np.zeros((P, N), np.int16),
            "best": np.zeros(P, np.int32),
        }
        self._check(self.lib.ke_eval(self.h, P, abi.ptr(pods), int(now_ns), abi.ptr(out["status"]),
                                     abi.ptr(out["reason"]), abi.ptr(out["la"]), abi.ptr(out["numa"]),
                                     abi.ptr(out["ds"]), abi.ptr(out["total"]), abi.ptr(out["best"])))
        return out

    def schedule(self, pods, now_ns, matches=None):
        """ke_schedule; `matches` (optional): per pod the reservation indices it matches (KE_RSV_MATCHED pods)."""
        pods = as_pod_array(pods)
        if matches is not None:
            self.pod_reservations(matches)
        chosen = np.zeros(len(pods), np.int32)
        score = np.zeros(len(pods), np.int32)
        self._check(self.lib.ke_schedule(self.h, len(pods), abi.ptr(pods), int(now_ns), abi.ptr(chosen), abi.ptr(score)))
        self._last_n, self._last_out = len(pods), {}  # the per-pod allocations are read on first access
        return chosen, score

    def submit(self, pods, now_ns):
        """ke_schedule_submit: enqueue a queue slice behind the calls in flight; returns its ticket (wait() collects
        it).  The pod array is kept alive here until then."""
        pods = as_pod_array(pods)
        t = C.c_int64()
        self._check(self.lib.ke_schedule_submit(self.h, len(pods), abi.ptr(pods), int(now_ns), C.byref(t)))
        self._inflight[t.value] = pods
        return t.value

    def wait(self, ticket):
        """ke_schedule_wait: (chosen, score) of a submitted slice, as schedule() returns them."""
        pods = self._inflight[ticket]
        chosen = np.zeros(len(pods), np.int32)
        score = np.zeros(len(pods), np.int32)
        try:
            self._check(self.lib.ke_schedule_wait(self.h, int(ticket), abi.ptr(chosen), abi.ptr(score)))
        finally:
            del self._inflight[ticket]
        self._last_n, self._last_out = len(pods), {}
        return chosen, score

    def _last(self, name, shape, dtype, fn):
        if name not in self._last_out:
            a = np.zeros(shape, dtype)
            self._check(getattr(self.lib, fn)(self.h, self._last_n, abi.ptr(a)))
            self._last_out[name] = a
        return self._last_out[name]

    @property
    def last_device_allocations(self):
        """ke_last_device_allocations of the last schedule(): allocated minors per pod."""
        return self._last("dev", self._last_n, np.uint64, "ke_last_device_allocations")

    @property
    def last_numa_allocations(self):
        """ke_last_numa_allocations of the last schedule(): [pod][NUMA id * 2 + resource]."""
        return self._last("numa", (self._last_n, 16), np.int64, "ke_last_numa_allocations")

    @property
    def last_cpusets(self):
        """ke_last_cpusets of the last schedule(): 256-bit CPU-id set per pod."""
        return self._last("cpus", (self._last_n, 4), np.uint64, "ke_last_cpusets")

    def last_allocations(self, n=None):
        """Release records (np.ndarray POD_ALLOCATION_DTYPE) of the pods of the last schedule()."""
        n = self._last_n if n is None else n
        out = np.zeros(n, abi.POD_ALLOCATION_DTYPE)
        self._check(self.lib.ke_last_allocations(self.h, n, abi.ptr(out)))
        return out

    def release(self, pod, alloc, mode=abi.RELEASE_UNRESERVE):
        """ke_pod_release: Unreserve (or informer delete) of one placement; `pod` abi.Pod or a POD_DTYPE
        record, `alloc` a POD_ALLOCATION_DTYPE record."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        a = np.ascontiguousarray(np.asarray(alloc, abi.POD_ALLOCATION_DTYPE).reshape(1))
        self._check(self.lib.ke_pod_release(self.h, abi.ptr(p), abi.ptr(a), int(mode)))

    def unreserve(self, pod, queue_pos):
        """ke_unreserve: Unreserve of the pod at `queue_pos` of the last schedule()."""
        p = as_pod_array([pod] if isinstance(pod, abi.Pod) else np.asarray(pod).reshape(1))
        self._check(self.lib.ke_unreserve(self.h, abi.ptr(p), int(queue_pos)))

    def quotas_load(self, args, quotas):
        """ElasticQuota tree (include/koord_eval.h ke_quotas_load): runtime computed on the host,
        admission and Reserve applied inside schedule()."""
        quotas = np.ascontiguousarray(quotas, abi.QUOTA_DTYPE)
        self._check(self.lib.ke_quotas_load(self.h, C.byref(args), abi.ptr(quotas), len(quotas)))

    def quota_state(self, q):
        limit, used, npu = np.zeros(2, np.int64), np.zeros(2, np.int64), np.zeros(2, np.int64)
        has = np.zeros(2, np.uint8)
        self._check(self.lib.ke_quota_state(self.h, int(q), abi.ptr(limit), abi.ptr(has), abi.ptr(used), abi.ptr(npu)))
        return {"limit": limit, "limit_has": has.astype(bool), "used": used, "np_used": npu}

    def stats(self):
        total = C.c_double()
        nb = abi.i32()
        self._check(self.lib.ke_last_schedule_stats(self.h, C.byref(total), C.byref(nb), None, 0))
        per = np.zeros(max(nb.value, 1), np.float64)
        self._check(self.lib.ke_last_schedule_stats(self.h, None, None, abi.ptr(per), len(per)))
        return total.value, per[: nb.value]

    def pod_latencies(self, n):
        """per-pod latency (ms, ke_last_pod_latencies) of the n pods of the last schedule()"""
        out = np.zeros(n, np.float64)
        self._check(self.lib.ke_last_pod_latencies(self.h, n, abi.ptr(out)))
        return out

    def set_profiling(self, sample_every):
        self._check(self.lib.ke_set_profiling(self.h, sample_every))

    def rsv_fused(self):
        """(fused, gated): matched pods of the last schedule placed behind their plain segment in its call, and those
        a plain pod of the segment broke (run again alone) -- ke_debug_rsv_fused."""
        out = (abi.i64 * 2)()
        self._check(self.lib.ke_debug_rsv_fused(self.h, out))
        return int(out[0]), int(out[1])

    def ds_cuts(self):
        """DeviceShare batches of the last schedule that stopped early (NormalizeScore max may have moved)."""
        n = abi.i32()
        self._check(self.lib.ke_debug_ds_cuts(self.h, C.byref(n)))
        return n.value

    def numa_deferred(self):
        """BestEffort pairs of the last eval / schedule that needed the compacted full NUMA merge."""
        n = abi.i64()
        self._check(self.lib.ke_debug_numa_deferred(self.h, C.byref(n)))
        return n.value

    def check_records(self, now_ns):
        """Nodes whose replay record differs from one derived from their device row (0 = consistent)."""
        n = abi.i64()
        self._check(self.lib.ke_debug_check_records(self.h, int(now_ns), C.byref(n)))
        return n.value

    def set_pipeline(self, on):
        """Pipelined schedule (default): batch b's eval + select overlap batch b-1's Reserve replay.
        on: False / True, or "fixup" (pipelined with exact lists from the fixup kernel, ke_set_pipeline 2)."""
        self._check(self.lib.ke_set_pipeline(self.h, 2 if on == "fixup" else (1 if on else 0)))

    HOST_PHASES = ("checks", "refresh", "upload", "setup", "enqueue", "wait", "stats", "mirror")

    def host_stats(self):
        """Host wall ms of the last schedule() by phase (ke_last_host_stats)."""
        ms = np.zeros(8, np.float64)
        self._check(self.lib.ke_last_host_stats(self.h, abi.ptr(ms)))
        return dict(zip(self.HOST_PHASES, ms.tolist()))

    def kernel_stats(self):
        ms4 = np.zeros(8, np.float64)
        n, npipe = abi.i32(), abi.i32()
        self._check(self.lib.ke_last_kernel_stats_ex(self.h, abi.ptr(ms4), C.byref(n), C.byref(npipe)))
        p, r = C.c_double(), C.c_double()
        self._check(self.lib.ke_last_resolve_split(self.h, C.byref(p), C.byref(r)))
        sf = C.c_double()
        self._check(self.lib.ke_debug_spec_failed(self.h, C.byref(sf)))
        ph = np.zeros(6, np.float64)
        self._check(self.lib.ke_debug_resolve_phases(self.h, abi.ptr(ph)))
        sub = np.zeros(5, np.float64)
        self._check(self.lib.ke_debug_resolve_subphases(self.h, abi.ptr(sub)))
        w1 = np.zeros(4, np.float64)
        self._check(self.lib.ke_debug_resolve_wave1(self.h, abi.ptr(w1)))
        return {"eval_ms": ms4[0], "select_ms": ms4[1], "fixup_ms": ms4[2], "resolve_ms": ms4[3], "samples": n.value,
                "pipelined_batches": npipe.value, "enqueue_ms": ms4[4], "handoff_ms": ms4[5],
                "rows_fetched": ms4[6], "rows_changed": ms4[7], "spec_failed_rounds": sf.value,
                "resolve_prologue_ms": p.value, "resolve_replay_ms": r.value,
                "resolve_phases_ms": dict(zip(["prologue", "spec_predict", "spec_reserve_eval", "spec_verify", "spec_later_rounds", "writeback",
                                               "sub_t_setup", "sub_predict_loop", "sub_t_rows_wave1", "sub_reserve_R",
                                               "t_helper_hit"],
                                              ph.tolist() + sub.tolist())),
                "resolve_wave1_ms": dict(zip(["wait", "reserve", "rows", "end"], w1.tolist()))}

    def bench_eval_kernel(self, pods, now_ns, iters):
        pods = as_pod_array(pods)
        ms = C.c_double()
        self._check(self.lib.ke_bench_eval_kernel(self.h, len(pods), abi.ptr(pods), int(now_ns), iters, C.byref(ms)))
        return ms.value

    def node_state(self, i):
        """Host object state of node i: (Node, cpus, zones, devices) (ke_debug_node_state)."""
        return abi.node_state(self.lib.ke_debug_node_state, self.h, i)

    def debug_rows(self, now_ns, device=True):
        n = self.num_nodes
        host = np.zeros(n, abi.ROW_DTYPE)
        dev = np.zeros(n, abi.ROW_DTYPE) if device else None
        self._check(self.lib.ke_debug_rows(self.h, n, int(now_ns), abi.ptr(dev), abi.ptr(host)))
        return dev, host


def comm_unique_id(lib=None):
    """RCCL unique id for ke_shard_init, created on rank 0 (needs the HIP device)."""
    lib = lib or abi.load_library()
    buf = C.create_string_buffer(abi.COMM_ID_BYTES)
    rc = lib.ke_comm_unique_id(buf, abi.COMM_ID_BYTES)
    if rc != abi.OK:
        raise KoordEvalError(rc, lib.ke_last_error().decode())
    return buf.raw
