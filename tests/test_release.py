"""Unreserve / pod release at the boundary (ke_pod_release, ke_unreserve) on the host state, CPU only.

The reference undoes a Reserve per plugin: loadaware podAssignCache.unAssign (load_aware.go:197-199),
nodenumaresource resourceManager.Release (plugin.go:569-577 -> node_allocation.go:158-190), deviceshare
updateCacheUsed(..., false) (plugin.go:498-516, device_cache.go:184-209), elasticquota UnreservePod /
OnPodDelete (plugin.go:361, group_quota_manager.go:922-981).  These tests pin the oracle's release with the
reference's own Unreserve / release vectors and check the product's host release against the oracle on
random states (the GPU path is tests/test_gpu_release.py)."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, model, synth
from oracle.binding import Oracle


def alloc(node, cpuset=(), numa=None, minors=(), quota=False):
    a = np.zeros(1, abi.POD_ALLOCATION_DTYPE)[0]
    a["node"] = node
    for c in cpuset:
        a["cpuset"][c >> 6] |= np.uint64(1) << np.uint64(c & 63)
    for (z, r), v in (numa or {}).items():
        a["numa"][2 * z + r] = v
    m = 0
    for t, mi in minors:
        m |= 1 << (16 * t + mi)
    a["device_minors"] = m
    a["quota_assigned"] = 1 if quota else 0
    return a


def both(n_nodes, cfg=None):
    cfg = cfg or abi.default_config(n_nodes)
    return Evaluator(cfg), Oracle(cfg, n_nodes)


def states_equal(ev, o, i):
    n1, c1, z1, d1 = ev.node_state(i)
    n0, c0, z0, d0 = o.node_state(i)
    assert list(n1.requested) == list(n0.requested), i
    c1, c0 = np.sort(c1, order="cpu_id"), np.sort(c0, order="cpu_id")
    assert np.array_equal(c1["cpu_id"], c0["cpu_id"]) and np.array_equal(c1["ref_count"], c0["ref_count"]), i
    live = c1["ref_count"] > 0
    assert np.array_equal(c1["exclusive"][live], c0["exclusive"][live]), i
    for k in ("id", "has_allocated", "allocated", "numa_status", "single_pods", "shared_pods"):
        assert np.array_equal(z1[k], z0[k]), (i, k)
    for k in ("type", "minor", "has_used", "used"):
        assert np.array_equal(d1[k], d0[k]), (i, k)
    return c1, z1, d1


# buildCPUTopologyForTest(2, 1, 4, 2) (cpu_accumulator_test.go:30-57) with CoreID = SocketID<<16 | CoreID:
# 2 sockets x 1 NUMA node x 4 cores x 2 threads, CPU ids in (socket, core, thread) order
TOPO_2142 = [(c, ((c // 8) << 16) | (c // 2), c // 8, c // 8) for c in range(16)]
ZONES_2 = [{"id": 0, "cpu": "8", "memory": "16Gi"}, {"id": 1, "cpu": "8", "memory": "16Gi"}]


@pytest.mark.parametrize("h", ["product", "oracle"])
def test_golden_release_cpus(h):
    """TestNodeAllocationStateReleaseCPUs (node_allocation_test.go:99-121): addCPUs(1-4, PCPULevel) then
    release -> no CPU allocated, every RefCount 0."""
    ev, o = both(1)
    x = ev if h == "product" else o
    x.upsert_node(0, model.make_node(allocatable={"cpu": "16", "memory": "32Gi"}))
    zones = model.make_zones([dict(z, allocated={}) for z in ZONES_2])
    zones[0]["numa_status"] = abi.NUMA_STATUS_SINGLE  # the pod's CPUs all lie in NUMA node 0
    x.set_numa(0, zones)
    x.set_cpus(0, model.make_cpus(TOPO_2142, {c: (1, "PCPULevel") for c in (1, 2, 3, 4)}))
    pod = model.make_pod(name="p", requests={"cpu": "4"})
    x.release(pod, alloc(0, cpuset=(1, 2, 3, 4)))
    _, cpus, z, _ = x.node_state(0)
    assert (cpus["ref_count"] == 0).all() and (cpus["exclusive"] == 0).all()
    assert list(z["numa_status"]) == [abi.NUMA_STATUS_IDLE] * 2 and list(z["single_pods"]) == [0, 0]


@pytest.mark.parametrize("h", ["product", "oracle"])
def test_golden_release_shared_cpus(h):
    """Test_cpuAllocation_getAvailableCPUs (node_allocation_test.go:123-152): pod A on 1-4 and pod B on 2-5
    (PCPULevel), release A -> CPUs 2-5 keep RefCount 1 (available with MaxRefCount 1: 0-1,6-15)."""
    ev, o = both(1)
    x = ev if h == "product" else o
    x.upsert_node(0, model.make_node(allocatable={"cpu": "16", "memory": "32Gi"}))
    zones = model.make_zones([dict(z, allocated={}) for z in ZONES_2])
    zones[0]["numa_status"] = abi.NUMA_STATUS_SINGLE
    zones[0]["single_pods"] = 2  # A and B
    x.set_numa(0, zones)
    ref = {1: 1, 2: 2, 3: 2, 4: 2, 5: 1}
    x.set_cpus(0, model.make_cpus(TOPO_2142, {c: (k, "PCPULevel") for c, k in ref.items()}))
    x.release(model.make_pod(name="a", requests={"cpu": "4"}), alloc(0, cpuset=(1, 2, 3, 4)))
    _, cpus, z, _ = x.node_state(0)
    cpus = np.sort(cpus, order="cpu_id")
    held = [int(c) for c in cpus["cpu_id"][cpus["ref_count"] >= 1]]
    assert held == [2, 3, 4, 5] and (cpus["ref_count"][2:6] == 1).all()
    assert (cpus["exclusive"][2:6] == abi.CPU_EXCL_PCPU_LEVEL).all() and cpus["exclusive"][1] == 0
    assert z["single_pods"][0] == 1 and z["numa_status"][0] == abi.NUMA_STATUS_SINGLE


@pytest.mark.parametrize("h", ["product", "oracle"])
def test_golden_deviceshare_unreserve(h):
    """Test_Plugin_Unreserve "normal case" (deviceshare/plugin_test.go:4186-4480): GPU 0,1 (gpu-core 100,
    ratio 100, 16Gi), FPGA 0,1 and RDMA 0,1 (100 each) fully used by the pod; Unreserve -> every used entry
    deleted, free = total."""
    ev, o = both(1)
    x = ev if h == "product" else o
    x.upsert_node(0, model.make_node(allocatable={"cpu": "16", "memory": "32Gi"}))
    gpu = {"koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory-ratio": "100", "koordinator.sh/gpu-memory": "16Gi"}
    devs = [dict(type="gpu", minor=m, total=gpu, used=gpu) for m in (0, 1)]
    devs += [dict(type="fpga", minor=m, total={"koordinator.sh/fpga": "100"}, used={"koordinator.sh/fpga": "100"})
             for m in (0, 1)]
    devs += [dict(type="rdma", minor=m, total={"koordinator.sh/rdma": "100"}, used={"koordinator.sh/rdma": "100"})
             for m in (0, 1)]
    x.set_devices(0, model.make_devices(devs))
    pod = model.make_pod(name="test", requests={"nvidia.com/gpu": "2", "koordinator.sh/fpga": "200",
                                                "koordinator.sh/rdma": "200"})
    x.release(pod, alloc(0, minors=[(t, m) for t in range(3) for m in (0, 1)]))
    _, _, _, d = x.node_state(0)
    assert len(d) == 6 and (d["has_used"] == 0).all() and (d["used"] == 0).all()


def test_release_partial_device_keeps_keys():
    """SubtractWithNonNegativeResult keeps the keys of both lists and floors at 0; only an all-zero used
    list is deleted (device_cache.go:196-203)."""
    ev, o = both(1)
    gpu_t = {"koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory-ratio": "100", "koordinator.sh/gpu-memory": "16Gi"}
    for x in (ev, o):
        x.upsert_node(0, model.make_node(allocatable={"cpu": "16", "memory": "32Gi"}))
        x.set_devices(0, model.make_devices([
            dict(type="gpu", minor=0, total=gpu_t, used={"koordinator.sh/gpu-core": "70", "koordinator.sh/gpu-memory-ratio": "60",
                                                         "koordinator.sh/gpu-memory": "8Gi"}),
            dict(type="gpu", minor=1, total=gpu_t, used={"koordinator.sh/gpu-core": "10"}),
            dict(type="rdma", minor=0, total={"koordinator.sh/rdma": "100"}, used={"koordinator.sh/rdma": "30"})]))
        pod = model.make_pod(name="s", requests={"koordinator.sh/gpu-core": "50", "koordinator.sh/gpu-memory-ratio": "50",
                                                 "koordinator.sh/rdma": "50"})
        x.release(pod, alloc(0, minors=[(0, 0), (0, 1), (1, 0)]))
    _, _, d = states_equal(ev, o, 0)
    d = {(int(r["type"]), int(r["minor"])): r for r in d}
    assert list(d[(0, 0)]["used"]) == [20, 0, 10] and list(d[(0, 0)]["has_used"]) == [1, 1, 1]
    assert list(d[(0, 1)]["has_used"]) == [0, 0, 0]  # 10 - 50 floors at 0 everywhere: deleted
    assert list(d[(1, 0)]["has_used"]) == [0, 0, 0]


def test_release_numa_zone_allocation():
    """NodeAllocation.release: allocatedResources[id] = SubtractWithNonNegativeResult(entry, pod's)
    (node_allocation.go:184-189) on a node whose CPU topology is valid; a pod spanning zones 0 and 1 leaves
    both sharedNode sets."""
    ev, o = both(1)
    zones = model.make_zones([dict(ZONES_2[0], allocated={"cpu": "6", "memory": "4Gi"}),
                              dict(ZONES_2[1], allocated={"cpu": "2"})])
    zones["shared_pods"] = [1, 1]
    zones["numa_status"] = abi.NUMA_STATUS_SHARED
    for x in (ev, o):
        x.upsert_node(0, model.make_node(allocatable={"cpu": "16", "memory": "32Gi"}, requested={"cpu": "8"}))
        x.set_numa(0, zones)
        x.set_cpus(0, model.make_cpus(TOPO_2142, {c: (1, None) for c in (6, 7, 8, 9)}))
        pod = model.make_pod(name="p", requests={"cpu": "4", "memory": "6Gi"})
        x.release(pod, alloc(0, cpuset=(6, 7, 8, 9), numa={(0, 0): 2000, (0, 1): 6 << 30, (1, 0): 2000, (1, 1): 1 << 30}))
    cpus, z, _ = states_equal(ev, o, 0)
    assert (cpus["ref_count"] == 0).all()
    assert list(z["allocated"][0]) == [4000, 0] and list(z["allocated"][1]) == [0, 0]
    assert z["has_allocated"][1] == abi.NUMA_ALLOC_ENTRY | abi.NUMA_ALLOC_CPU | abi.NUMA_ALLOC_MEMORY
    assert list(z["numa_status"]) == [abi.NUMA_STATUS_IDLE] * 2
    n, _, _, _ = ev.node_state(0)
    assert list(n.requested) == [4000, -(6 << 30)]  # NodeInfo.RemovePod does not floor


def test_release_without_cpu_topology_keeps_zones():
    """Without a valid CPU topology resourceManager.Update recorded nothing (resource_manager.go:461-466),
    so the release leaves the zones alone."""
    ev, o = both(1)
    zones = model.make_zones([dict(ZONES_2[0], allocated={"cpu": "6"}), dict(ZONES_2[1], allocated={"cpu": "2"})])
    for x in (ev, o):
        x.upsert_node(0, model.make_node(allocatable={"cpu": "16", "memory": "32Gi"}))
        x.set_numa(0, zones)
        x.release(model.make_pod(name="p", requests={"cpu": "4"}), alloc(0, numa={(0, 0): 2000, (1, 0): 2000}))
    _, z, _ = states_equal(ev, o, 0)
    assert list(z["allocated"][:, 0]) == [6000, 2000]


def test_zone_counts_validation():
    ev, _ = both(1)
    ev.upsert_node(0, model.make_node(allocatable={"cpu": "16", "memory": "32Gi"}))
    z = model.make_zones(ZONES_2)
    z["single_pods"][0] = 2  # counts say Single, status says Idle
    with pytest.raises(Exception):
        ev.set_numa(0, z)
    z["numa_status"][0] = abi.NUMA_STATUS_SINGLE
    ev.set_numa(0, z)
    z = model.make_zones(ZONES_2)
    z["numa_status"][1] = abi.NUMA_STATUS_SHARED  # status alone: one pod in the shared set
    ev.set_numa(0, z)
    assert list(ev.node_state(0)[2]["shared_pods"]) == [0, 1]


def test_release_loadaware_and_requested_roundtrip():
    """podAssignCache.assign then release -> the node's folded LoadAware row is the one before the pod."""
    cl = synth.make_cluster(40, synth.BASE_SEED + 71)
    pods = synth.make_pods(40, synth.BASE_SEED + 171)
    ev = Evaluator(synth.config(40))
    synth.load_into(ev, cl)
    _, before = ev.debug_rows(synth.T0, device=False)
    for i in range(40):
        ev.assign(i, abi.Pod.from_buffer_copy(pods[i:i + 1].tobytes()), synth.T0)
        ev.set_requested(i, int(cl.nodes["requested"][i, 0] + pods["requests"][i, 0]),
                         int(cl.nodes["requested"][i, 1] + pods["requests"][i, 1]))
    _, mid = ev.debug_rows(synth.T0, device=False)
    assert not np.array_equal(before, mid)
    for i in range(40):
        ev.release(pods[i], alloc(i))
    _, after = ev.debug_rows(synth.T0, device=False)
    assert np.array_equal(before, after)


def _random_release_setup(seed, n=60):
    rng = np.random.default_rng(seed)
    cl, zones, tables = synth.make_c4_cluster(n, seed)
    devices = synth.make_devices(n, seed + 1)
    pods = synth.make_ds_pods(400, seed + 2, device_fraction=0.6)
    tc = int(pods["requests"][:, abi.RES_CPU].sum() * 0.6)
    tm = int(pods["requests"][:, abi.RES_MEMORY].sum() * 0.6)
    quotas = synth.make_quota_tree(seed + 3, 16, 4, tc, tm)
    quotas["limit_is_max"][0] = 1  # a system / default quota among the roots
    pods = synth.assign_quotas(pods, quotas, seed + 4)
    quotas["used"] = quotas["self_request"] // 2  # some of each quota's pods are assigned
    for q in range(len(quotas)):  # used of a parent covers its children's
        p = int(quotas["parent"][q])
        while p >= 0:
            quotas["used"][p] += quotas["used"][q]
            p = int(quotas["parent"][p])
    quotas["non_preemptible_used"] = quotas["used"] // 3
    return rng, cl, zones, tables, devices, pods, quotas, tc, tm


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_release_random_states_vs_oracle(seed):
    """Random placements' records released from C4 nodes (CPU tables + 8 zones with cpusets / allocations /
    single-shared sets), device caches and a quota tree with a system quota: the product's host state
    equals the oracle's after every release (Unreserve and informer delete)."""
    rng, cl, zones, tables, devices, pods, quotas, tc, tm = _random_release_setup(synth.BASE_SEED + 700 + seed)
    n = cl.n_nodes
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for x in (ev, o):
        synth.load_into(x, cl)
        synth.load_numa(x, zones)
        synth.load_cpus(x, tables)
        synth.load_devices(x, devices)
        x.quotas_load(synth.quota_args(tc, tm), quotas)
    for p in range(150):
        node = int(rng.integers(0, n))
        t, maxref = tables[node]
        held = [int(c) for c in t["cpu_id"][t["ref_count"] > 0]] if t is not None else []
        cs = list(rng.choice(held, min(len(held), int(rng.integers(0, 6))), replace=False)) if held else []
        numa = {(int(z), r): int(rng.integers(0, 3000)) * (1000 if r == 0 else 1 << 20)
                for z in range(8) for r in range(2) if rng.random() < 0.3}
        healthy = set()  # Reserve allocates healthy instances only (device_cache.go:558-560)
        if devices[node] is not None:
            healthy = {(int(d["type"]), int(d["minor"])) for d in devices[node] if d["health"]}
        minors = [tm for tm in sorted(healthy) if rng.random() < 0.3]
        a = alloc(node, cs, numa, minors, quota=rng.random() < 0.8)
        mode = abi.RELEASE_DELETE if rng.random() < 0.3 else abi.RELEASE_UNRESERVE
        for x in (ev, o):
            x.release(pods[p], a, mode)
        if p % 10 == 0:
            states_equal(ev, o, node)
    for i in range(n):
        states_equal(ev, o, i)
    for q in range(len(quotas)):
        a, b = ev.quota_state(q), o.quota_state(q)
        for k in ("limit", "limit_has", "used", "np_used"):
            assert np.array_equal(a[k], b[k]), (q, k)


def test_unreserve_requires_a_schedule():
    ev, _ = both(2)
    with pytest.raises(Exception):
        ev.unreserve(model.make_pod(name="x"), 0)
