"""Informer lifecycle at the boundary on the GPU: Node deletes and re-adds (ke_node_delete / ke_node_upsert), NRT
deletes (ke_node_topology_delete), release records that outlive a reservation reload (by uid), a refused call that
leaves no state behind, and the per-pod latency of SURVEY.md §8(d) (ke_last_pod_latencies) -- each bit-exact with
the oracle's twin of the same events."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, KoordEvalError, abi, synth
from oracle.binding import Oracle
from test_gpu_cpuset import assert_eval_equal, assert_schedule_equal
from test_gpu_ext import _cluster

pytestmark = pytest.mark.gpu


def _plain(n, seed):
    cl = synth.make_cluster(n, synth.BASE_SEED + seed)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
    return ev, o, cl


def _node_now(ev, o, i):
    """the node object as both hold it now (NodeInfo.Requested with the Reserves so far): what a re-add passes"""
    n1, n0 = ev.node_state(int(i))[0], o.node_state(int(i))[0]
    assert list(n1.requested) == list(n0.requested), i
    return n1


def _delete_readd(ev, o, cl, rng, frac=0.1):
    n = cl.n_nodes
    gone = rng.choice(n, int(n * frac), replace=False)
    for h in (ev, o):
        for i in gone:
            h.delete_node(int(i))
    return gone


def test_node_delete_and_readd_schedule_parity(gpu):
    """10 % of the nodes deleted between two queues, then half of them re-added with their other caches intact: the
    deleted nodes are evaluated nowhere (KE_CODE_ERROR in ke_eval, never chosen), the queues stay bit-exact with the
    oracle, and the replay records equal a from-scratch derivation."""
    ev, o, cl = _plain(3000, 1101)
    rng = np.random.default_rng(1102)
    q1 = synth.make_pods(1500, synth.BASE_SEED + 1103)
    c1, s1 = ev.schedule(q1, synth.T0)
    c0, s0 = o.schedule(q1, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    gone = _delete_readd(ev, o, cl, rng)
    pods = synth.make_pods(64, synth.BASE_SEED + 1104, key_base=8_000_000_000)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    assert_eval_equal(a, b)
    assert (a["status"][:, gone] == abi.CODE_ERROR).all() and (a["total"][:, gone] == -1).all()
    q2 = synth.make_pods(2000, synth.BASE_SEED + 1105, key_base=8_100_000_000)
    c1, s1 = ev.schedule(q2, synth.T0)
    c0, s0 = o.schedule(q2, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert not np.isin(c1, gone).any()
    assert ev.check_records(synth.T0) == 0
    back = gone[: len(gone) // 2]
    objs = [_node_now(ev, o, i) for i in back]
    for h in (ev, o):
        for i, nd in zip(back, objs):
            h.upsert_node(int(i), nd)
    q3 = synth.make_pods(2000, synth.BASE_SEED + 1106, key_base=8_200_000_000)
    c1, s1 = ev.schedule(q3, synth.T0)
    c0, s0 = o.schedule(q3, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.isin(c1, back).any()  # the re-added nodes take pods again
    assert not np.isin(c1, gone[len(gone) // 2:]).any()
    assert ev.check_records(synth.T0) == 0
    for i in list(back[:20]) + list(gone[-20:]):
        assert ev.node_info_requested(int(i))[0] == o.node_info_requested(int(i))[0], i


def test_node_delete_cpuset_numa_devices_parity(gpu):
    """Deletes on nodes with CPU tables / NUMA zones (amplified, FitPlus + SRA) and on DeviceShare nodes, with NRT
    deletes on a few: cpusets, NUMA allocations and device minors of the following queue equal the oracle's, and a
    pod placed before its node's delete is released from the deleted node's caches."""
    ev, o, tables = _cluster(600, 1111, cpus=True)
    rng = np.random.default_rng(1112)
    pods = synth.add_pod_xres(synth.make_pods(300, synth.BASE_SEED + 1113), synth.BASE_SEED + 1114)
    assert_schedule_equal(ev, o, pods, synth.T0)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    placed = np.flatnonzero(a1["node"] >= 0)
    gone = rng.choice(600, 60, replace=False)
    for h in (ev, o):
        for i in gone:
            h.delete_node(int(i))
        for i in gone[:10]:
            h.delete_topology(int(i))
    # pods bound to deleted nodes go away afterwards (pod GC): release from the ghost NodeInfo
    on_gone = [p for p in placed if a1["node"][p] in set(gone.tolist())][:10]
    for p in on_gone:
        ev.release(pods[p], a1[p], abi.RELEASE_DELETE)
        o.release(pods[p], a0[p], abi.RELEASE_DELETE)
    more = synth.add_pod_xres(synth.make_pods(300, synth.BASE_SEED + 1115, key_base=8_300_000_000),
                              synth.BASE_SEED + 1116)
    assert_eval_equal(ev.eval(more[:32], synth.T0), o.eval(more[:32], synth.T0))
    assert_schedule_equal(ev, o, more, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert ev.check_records(synth.T0) == 0
    for i in gone[:10]:
        n1, cpus1, z1, _ = ev.node_state(int(i))
        n0, cpus0, z0, _ = o.node_state(int(i))
        assert len(cpus1) == len(cpus0) == 0 and len(z1) == len(z0) == 0
    ev2, o2, _ = _cluster(400, 1117, devices=True)
    gone = rng.choice(400, 40, replace=False)
    for h in (ev2, o2):
        for i in gone:
            h.delete_node(int(i))
    dp = synth.make_ds_pods(200, synth.BASE_SEED + 1118)
    c1, s1 = ev2.schedule(dp, synth.T0)
    c0, s0 = o2.schedule(dp, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev2.last_device_allocations, o2.last_device_allocations)
    assert (ev2.last_device_allocations != 0).any()
    assert not np.isin(c1, gone).any()


def test_topology_delete_readd_keeps_allocation_parity(gpu):
    """NRT deletes between queues, cpuset pods released during the gap, then bare NRT re-adds
    (topology only, as the informer delivers them): the parked NodeAllocation comes back, so the next cpuset queue
    never hands out a CPU beyond MaxRefCount and stays bit-exact with the oracle (cpusets, NUMA allocations)."""
    from test_lifecycle import _bare
    n = 500
    cl = synth.make_cluster(n, synth.BASE_SEED + 1151, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + 1152)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
    pods = synth.make_numa_cpuset_pods(600, synth.BASE_SEED + 1153)
    assert_schedule_equal(ev, o, pods, synth.T0)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    cs_pods = np.flatnonzero((a1["node"] >= 0) & a1["cpuset"].any(axis=1))
    assert len(cs_pods) >= 10
    nodes = np.unique(a1["node"][cs_pods])[:30]
    for h in (ev, o):
        for i in nodes:
            h.delete_topology(int(i))
    for p in cs_pods[:8]:  # pod GC during the gap
        ev.release(pods[p], a1[p], abi.RELEASE_DELETE)
        o.release(pods[p], a0[p], abi.RELEASE_DELETE)
    for i in nodes:
        t, z = _bare(tabs[i][0], zones[i])
        for h in (ev, o):
            h.set_numa(int(i), z)
            h.set_cpus(int(i), t, tabs[i][1])
    more = synth.make_numa_cpuset_pods(600, synth.BASE_SEED + 1154, key_base=8_500_000_000)
    assert_schedule_equal(ev, o, more, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert ev.check_records(synth.T0) == 0
    for i in nodes:
        cpus1, cpus0 = ev.node_state(int(i))[1], o.node_state(int(i))[1]
        cpus1, cpus0 = np.sort(cpus1, order="cpu_id"), np.sort(cpus0, order="cpu_id")  # (table vs id order)
        assert np.array_equal(cpus1["ref_count"], cpus0["ref_count"]), i
        assert cpus1["ref_count"].max(initial=0) <= tabs[i][1], i
    assert sum(int(ev.node_state(int(i))[1]["ref_count"].sum()) for i in nodes) > 0


def test_refused_call_leaves_no_state(gpu):
    """a queue whose matched pod is refused (a pod binding CPUs whose reservation holds NUMA
    resources on a NUMA-policy node) fails in the argument checks, before any pod is scheduled -- the plain pods ahead
    of it are not Reserved and the matched restore is not left behind; the next queue equals an oracle that never
    saw the refused one."""
    ev, o, cl = _plain(400, 1121)
    node = abi.Node.from_buffer_copy(cl.nodes[7].tobytes())
    node.numa_topology_policy = abi.NUMA_POLICY_BEST_EFFORT
    rs = [abi.Reservation(node=7, available=1, holds=abi.RSV_HOLDS_NUMA), abi.Reservation(node=9, available=1)]
    rs[0].allocatable[0], rs[1].allocatable[0] = 4000, 4000
    al = np.zeros(2, abi.RESERVATION_ALLOC_DTYPE)
    al["numa"][0, 0] = 4000  # the reserve pod's NUMA resources: the matched path there is refused
    for h in (ev, o):
        h.upsert_node(7, node)
        h.reservations_load(rs, al)
    pods = synth.make_pods(200, synth.BASE_SEED + 1122)
    pods["reservation_matched"][150] = abi.RSV_MATCHED
    pods["qos_class"][150], pods["priority_class"][150] = abi.QOS_LSR, abi.PRIORITY_PROD  # binds CPUs
    pods["cpu_bind_required"][150] = abi.CPU_BIND_FULL_PCPUS  # under a required FullPCPUs policy: refused
    pods["requests"][150, abi.RES_CPU] = pods["limits"][150, abi.RES_CPU] = 2000
    pods["numa_topology_policy"][150] = 0
    pods["requests"][150, 2:] = 0
    pods["has_other_requests"][150] = 0
    pods["device_requests"][150] = 0
    matches = [[] for _ in range(200)]
    matches[150] = [0, 1]
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0, matches=matches)
    assert e.value.code == abi.ERR_UNSUPPORTED
    more = synth.make_pods(300, synth.BASE_SEED + 1123, key_base=8_400_000_000)
    c1, s1 = ev.schedule(more, synth.T0)
    c0, s0 = o.schedule(more, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert ev.check_records(synth.T0) == 0


def test_release_by_uid_after_reservation_reload(gpu):
    """A release record taken before a reservation reload finds its reservation by uid in the reordered set
    (an index of the old set would decrement another reservation)."""
    from test_gpu_reservations import _matched_setup, _resv_equal
    ev, o, pods, matches = _matched_setup(300, 1131, 200)
    rs = ev.reservations_get().copy()
    rs["uid"] = np.arange(1, len(rs) + 1) * 7919
    for h in (ev, o):
        h.reservations_load(rs)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    into = np.flatnonzero(a1["reservation"] > 0)
    assert len(into) >= 3
    assert np.array_equal(a1["reservation_uid"], a0["reservation_uid"])
    cur = _resv_equal(ev, o).copy()
    perm = np.random.default_rng(1132).permutation(len(cur))
    for h in (ev, o):
        h.reservations_load(cur[perm])  # the same reservations, another order
    for p in into:
        ev.release(pods[p], a1[p], abi.RELEASE_DELETE)
        o.release(pods[p], a0[p], abi.RELEASE_DELETE)
    after = _resv_equal(ev, o)
    back = np.argsort(perm)
    assert (after["allocated_pods"][back].sum() < cur["allocated_pods"].sum())
    stale = a1[into[0]].copy()
    stale["reservation_uid"] = 0  # an index of the old generation without a uid: refused
    with pytest.raises(KoordEvalError) as e:
        ev.release(pods[into[0]], stale, abi.RELEASE_DELETE)
    assert e.value.code == abi.ERR_INVALID


def test_pod_latency_definition(gpu):
    """ke_last_pod_latencies: per pod from the call's entry to its batch's Reserve end -- positive,
    non-decreasing in queue order for a plain queue, at least the batch's device service time, at most the call."""
    import time
    ev, o, cl = _plain(5000, 1141)
    pods = synth.make_pods(3000, synth.BASE_SEED + 1142)
    t = time.perf_counter()
    ev.schedule(pods, synth.T0)
    wall = (time.perf_counter() - t) * 1e3
    lat = ev.pod_latencies(len(pods))
    _, per_batch = ev.stats()
    assert (lat > 0).all() and (np.diff(lat) >= -1e-9).all()
    assert lat.max() <= wall + 1e-6
    assert lat[0] >= per_batch[0] - 1e-6
    assert lat[-1] > lat[0]
