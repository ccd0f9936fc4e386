"""Reservations on the GPU: with a reservation cache loaded, every pod that matches no
reservation is evaluated against the restored NodeInfo (restoreUnmatchedReservations, transformer.go:447-473) --
NodeNUMAResource's amplified-cpu Filter and Score and NodeResourcesFitPlus read it -- and pods that match
reservations take the nominated-reservation path (restoreMatchedReservation, the Reservation plugin's Score and
Reserve, k_rsv_pick), bit-exact with the oracle."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, synth
from oracle.binding import Oracle
from test_gpu_cpuset import assert_eval_equal
from test_gpu_ext import _cluster, _schedule_equal

pytestmark = pytest.mark.gpu


def _reservations(cl, seed, frac=0.4):
    rng = np.random.default_rng(seed)
    rs = []
    for i in range(cl.n_nodes):
        if rng.random() >= frac:
            continue
        for _ in range(int(rng.integers(1, 3))):
            r = abi.Reservation()
            r.node = i
            r.available = int(rng.random() < 0.95)
            r.allocate_once = int(rng.random() < 0.2)
            r.allocated_pods = int(rng.choice([0, 1, 1, 2]))
            for k in range(abi.NRES):
                a = int(cl.nodes["requested"][i, k]) // int(rng.integers(2, 6))
                a = a // 1000 * 1000 if k == 0 else a
                r.allocatable[k] = a
                r.allocated[k] = int(rng.choice([0, a // 2, a, a + (1000 if k == 0 else 2**30)]))
            rs.append(r)
    return rs


def test_reservation_restore_schedule_parity(gpu):
    ev, o, tables = _cluster(500, 941, cpus=True)
    cl = synth.make_cluster(500, synth.BASE_SEED + 941, amplified_fraction=0.2)  # _cluster's nodes
    rs = _reservations(cl, 942)
    for h in (ev, o):
        h.reservations_load(rs)
    pods = synth.add_pod_xres(synth.make_pods(400, synth.BASE_SEED + 943), synth.BASE_SEED + 944)
    assert_eval_equal(ev.eval(pods[:48], synth.T0), o.eval(pods[:48], synth.T0))
    _schedule_equal(ev, o, pods, tables)
    for i in range(0, 500, 37):
        assert ev.node_info_requested(i) == o.node_info_requested(i), i
    # a new reservation set: the restore moves, the rows follow
    rs2 = _reservations(cl, 945, frac=0.6)
    for h in (ev, o):
        h.reservations_load(rs2)
    more = synth.add_pod_xres(synth.make_pods(200, synth.BASE_SEED + 946, key_base=9_900_000_000),
                              synth.BASE_SEED + 947)
    assert_eval_equal(ev.eval(more[:48], synth.T0), o.eval(more[:48], synth.T0))
    c1, s1 = ev.schedule(more, synth.T0)
    c0, s0 = o.schedule(more, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert ev.check_records(synth.T0) == 0


def _matched_setup(n, seed, n_pods, affinity=0.0):
    """A FitPlus + amplified-cpu cluster whose NodeInfo holds the reserve pods of owner-grouped reservations
    (Default / Aligned / Restricted, AllocateOnce, orders, some already allocated), and a queue in which
    about 40 % of the eligible pods match one owner group's reservations (KE_RSV_MATCHED)."""
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    rs, grp = [], []
    for g in range(10):
        for _ in range(int(rng.integers(2, 7))):
            r = abi.Reservation(node=int(rng.integers(0, n)), available=int(rng.random() < 0.95),
                                allocate_once=int(rng.random() < 0.25), allocate_policy=int(rng.integers(0, 3)),
                                allocated_pods=int(rng.choice([0, 0, 1, 2])), order=int(rng.choice([0, 0, 0, 7, 3, 11])))
            r.allocatable[0] = int(rng.choice([0, 2000, 4000, 8000, 16000]))
            r.allocatable[1] = int(rng.choice([0, 4, 8, 16, 32])) * 2**30
            if r.allocated_pods:
                r.allocated[0], r.allocated[1] = r.allocatable[0] // 2, r.allocatable[1] // 4
            cl.nodes["requested"][r.node, 0] += r.allocatable[0]  # the reserve pod is in NodeInfo
            cl.nodes["requested"][r.node, 1] += r.allocatable[1]
            rs.append(r)
            grp.append(g)
    cfg = synth.ext_config(synth.config(n))
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    tables = synth.make_node_resources(cl, synth.BASE_SEED + seed + 1)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_node_resources(h, tables)
        h.reservations_load(rs)
    pods = synth.add_pod_xres(synth.make_pods(n_pods, synth.BASE_SEED + seed + 2), synth.BASE_SEED + seed + 3)
    cpuset = np.isin(pods["qos_class"], [abi.QOS_LSE, abi.QOS_LSR]) & (pods["priority_class"] == abi.PRIORITY_PROD)
    elig = ((pods["numa_topology_policy"] == 0) & (pods["requests"][:, 2:] == 0).all(1) & (pods["has_other_requests"] == 0)
            & (pods["device_requests"] == 0).all(1) & ~cpuset)
    grp = np.asarray(grp)
    matches = [[] for _ in range(n_pods)]
    for p in np.flatnonzero(elig & (rng.random(n_pods) < 0.4)):
        pods["reservation_matched"][p] = abi.RSV_AFFINITY if rng.random() < affinity else abi.RSV_MATCHED
        matches[p] = np.flatnonzero(grp == rng.integers(0, 10)).tolist()
        if pods["reservation_matched"][p] == abi.RSV_AFFINITY and rng.random() < 0.2:
            matches[p] = matches[p][:1] if rng.random() < 0.5 else []  # by name / no reservation left
    return ev, o, pods, matches


def _resv_equal(ev, o):
    a, b = ev.reservations_get(), o.reservations_get()
    assert np.array_equal(a["allocated"], b["allocated"]) and np.array_equal(a["allocated_pods"], b["allocated_pods"])
    return a


def test_matched_reservations_schedule_parity(gpu):
    """The nominated-reservation path: KE_RSV_MATCHED pods between plain ones in one queue --
    their matched restore, the Reservation plugin's preferredNode / nomination / normalized Score at weight 5000,
    Reserve into the nominated reservation -- bit-exact with the oracle on placements, totals, reservation
    state and release records; then Unreserve of a third of the matched placements and a second queue."""
    ev, o, pods, matches = _matched_setup(300, 961, 260)
    before = ev.reservations_get()
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    after = _resv_equal(ev, o)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(a1["reservation"], a0["reservation"])
    assert (a1["reservation"] > 0).sum() >= 5  # pods went into reservations
    assert (s1 >= 5000).sum() >= 5  # and carried the Reservation score
    assert (after["allocated_pods"] > before["allocated_pods"]).any()
    assert ev.check_records(synth.T0) == 0
    into = np.flatnonzero(a1["reservation"] > 0)
    for p in into[::3]:
        ev.unreserve(pods[p], int(p))
        o.release(pods[p], a0[p], abi.RELEASE_UNRESERVE)
    _resv_equal(ev, o)
    ev2, o2, more, m2 = _matched_setup(300, 961, 260)  # the same generator: a second queue of the same shape
    ev2.close()
    more["pod_key"] += 7_000_000_000
    more["uid"] += 7_000_000_000
    c1, s1 = ev.schedule(more, synth.T0, matches=m2)
    c0, s0 = o.schedule(more, synth.T0, matches=m2)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    _resv_equal(ev, o)
    assert ev.check_records(synth.T0) == 0


def test_ignored_pods_small_case(gpu):
    """KE_RSV_IGNORED on the device: the oracle test's three nodes (test_reservations.py ignored_case) -- two ignored
    pods take the reserved CPUs, the plain twins fit nowhere."""
    from test_reservations import ignored_case
    cl, cfg, tables, rs, pods = ignored_case()
    for v, want in ((abi.RSV_NONE, [-1, -1, -1]), (abi.RSV_IGNORED, [1, 1, -1])):
        ev = Evaluator(cfg)
        synth.load_into(ev, cl)
        synth.load_node_resources(ev, tables)
        ev.reservations_load(rs)
        pods["reservation_matched"][:] = v
        c, _ = ev.schedule(pods, synth.T0)
        assert c.tolist() == want
        assert ev.reservations_get()["allocated_pods"][0] == 0
        assert ev.check_records(synth.T0) == 0
        ev.close()


def test_ignored_pods_between_matched_and_plain(gpu):
    """Reservation-ignored pods (runs of them and single ones) between KE_RSV_MATCHED and plain pods of one queue:
    every available reservation's matched restore for them, the unmatched restore for the plain pods, the
    nominated-reservation path for the matched ones -- placements, totals, reservation state and release records
    bit-exact with the oracle; the ignored pods go into no reservation."""
    ev, o, pods, matches = _matched_setup(300, 981, 300)
    rng = np.random.default_rng(982)
    free = np.flatnonzero(pods["reservation_matched"] == abi.RSV_NONE)
    ign = free[rng.random(len(free)) < 0.35]
    ign = np.union1d(ign, free[(free >= 100) & (free < 140)])  # a long run
    pods["reservation_matched"][ign] = abi.RSV_IGNORED
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    _resv_equal(ev, o)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(a1["reservation"], a0["reservation"])
    assert (a1["reservation"][ign] == 0).all() and (c1[ign] >= 0).sum() >= 20
    assert ev.check_records(synth.T0) == 0
    for i in range(0, 300, 29):
        assert ev.node_info_requested(i) == o.node_info_requested(i), i
    more = synth.make_pods(120, synth.BASE_SEED + 983, key_base=8_800_000_000)
    more["reservation_matched"][::2] = abi.RSV_IGNORED
    c1, s1 = ev.schedule(more, synth.T0)
    c0, s0 = o.schedule(more, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    ev.close()


def test_matched_pods_with_numa_policies(gpu):
    """KE_RSV_MATCHED pods with their own NUMA topology policy (and cpuset / plain pods) on a cluster of NUMA-policy
    nodes beside cpu / memory reservations (no holdings): the matched restore moves NodeInfo.Requested only, which
    the hints do not read; the Reservation score and Reserve as for any matched pod -- placements, totals, NUMA
    allocations and reservation state bit-exact with the oracle."""
    n = 300
    rng = np.random.default_rng(991)
    cl = synth.make_cluster(n, synth.BASE_SEED + 991, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + 992)
    rs, grp = [], []
    for g in range(10):
        for _ in range(int(rng.integers(2, 7))):
            r = abi.Reservation(node=int(rng.integers(0, n)), available=1, allocate_once=int(rng.random() < 0.2),
                                allocate_policy=int(rng.integers(0, 3)), allocated_pods=int(rng.choice([0, 1])),
                                order=int(rng.choice([0, 0, 5])))
            r.allocatable[0] = int(rng.choice([2000, 4000, 8000]))
            r.allocatable[1] = int(rng.choice([4, 8, 16])) * 2**30
            if r.allocated_pods:
                r.allocated[0], r.allocated[1] = r.allocatable[0] // 2, r.allocatable[1] // 4
            cl.nodes["requested"][r.node, 0] += r.allocatable[0]
            cl.nodes["requested"][r.node, 1] += r.allocatable[1]
            rs.append(r)
            grp.append(g)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.reservations_load(rs)
    pods = synth.make_numa_cpuset_pods(300, synth.BASE_SEED + 993, policy_fraction=0.4)
    grp = np.asarray(grp)
    elig = ((pods["requests"][:, 2:] == 0).all(1) & (pods["has_other_requests"] == 0)
            & (pods["device_requests"] == 0).all(1))
    matches = [[] for _ in range(len(pods))]
    for p in np.flatnonzero(elig & (rng.random(len(pods)) < 0.5)):
        pods["reservation_matched"][p] = abi.RSV_MATCHED
        matches[p] = np.flatnonzero(grp == rng.integers(0, 10)).tolist()
    assert ((pods["reservation_matched"] == abi.RSV_MATCHED) & (pods["numa_topology_policy"] != 0)).sum() >= 10
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    _resv_equal(ev, o)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(a1["reservation"], a0["reservation"])
    pol = (pods["numa_topology_policy"] != 0) & (a1["reservation"] > 0)
    assert pol.sum() >= 2  # pods with their own NUMA policy went into reservations
    assert ev.check_records(synth.T0) == 0
    ev.close()


def test_matched_reservations_weight_one(gpu):
    """weight_reservation 1: the Reservation score mixes with the other plugins' totals instead of dominating;
    every matched pod matches all 40 reservations (several per node compete in NominateReservation)."""
    ev, o, pods, matches = _matched_setup(200, 971, 150)
    ev.close()
    n = 200
    rng = np.random.default_rng(972)
    cl = synth.make_cluster(n, synth.BASE_SEED + 971, amplified_fraction=0.2)
    cfg = synth.ext_config(synth.config(n))
    cfg.weight_reservation = 1
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    tables = synth.make_node_resources(cl, synth.BASE_SEED + 972)
    rs = []
    for i in rng.choice(n, 40, replace=False):
        r = abi.Reservation(node=int(i), available=1, order=int(rng.choice([0, 0, 4])))
        r.allocatable[0], r.allocatable[1] = 8000, 16 * 2**30
        cl.nodes["requested"][i, 0] += 8000
        cl.nodes["requested"][i, 1] += 16 * 2**30
        rs.append(r)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_node_resources(h, tables)
        h.reservations_load(rs)
    ids = list(range(len(rs)))
    matches = [ids if pods["reservation_matched"][p] else [] for p in range(len(pods))]
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    _resv_equal(ev, o)
    assert ev.check_records(synth.T0) == 0


def test_reservation_affinity_schedule_parity(gpu):
    """Required reservation affinity (KE_RSV_AFFINITY): the Reservation Filter keeps only nodes where a listed
    reservation fits, a one-reservation node nominates it unfiltered, an empty list leaves the pod unschedulable;
    mixed with KE_RSV_MATCHED and plain pods, bit-exact with the oracle."""
    ev, o, pods, matches = _matched_setup(300, 981, 260, affinity=0.5)
    aff = pods["reservation_matched"] == abi.RSV_AFFINITY
    assert aff.sum() >= 10
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    _resv_equal(ev, o)
    a1 = ev.last_allocations()
    assert np.array_equal(a1["reservation"], o.last_allocations()["reservation"])
    placed_aff = aff & (c1 >= 0)
    assert (a1["reservation"][placed_aff] > 0).all()  # an affinity pod is placed only into a reservation
    assert (c1[aff & np.array([len(m) == 0 for m in matches])] == -1).all()
    assert ev.check_records(synth.T0) == 0


def test_fits_node_other_resources_on_the_device(gpu):
    """The CPU test's single node (test_reservations.py::test_fits_node_checks_the_pods_other_resources) on the
    device: a matched pod whose scalar does not fit is not nominated, with it free it is -- as the oracle."""
    cl = synth.make_cluster(1, synth.BASE_SEED + 1412)
    cfg = synth.config(1)
    tab = np.zeros(3, abi.NODE_RESOURCE_DTYPE)
    tab["id"] = [abi.XRES_CPU, abi.XRES_MEMORY, 5]
    tab["allocatable"] = [cl.nodes["allocatable"][0, 0], cl.nodes["allocatable"][0, 1], 4]
    tab["requested"] = [cl.nodes["requested"][0, 0], cl.nodes["requested"][0, 1], 4]
    r = abi.Reservation(node=0, available=1)
    r.allocatable[0] = 2000
    pods = synth.make_pods(1, synth.BASE_SEED + 1412)
    pods["requests"][0, 0], pods["requests"][0, 1], pods["requests"][0, 2:] = 1000, 2**28, 0
    pods["has_other_requests"], pods["device_requests"], pods["numa_topology_policy"] = 0, 0, 0
    pods["n_xres"] = 1
    pods["xres_id"][0, 0], pods["xres_value"][0, 0] = 5, 1
    pods["reservation_matched"] = abi.RSV_MATCHED
    for used, into in ((4, 0), (3, 1)):
        tab["requested"][2] = used
        ev = Evaluator(cfg)
        synth.load_into(ev, cl)
        ev.set_resources(0, tab)
        ev.reservations_load([r])
        c, s = ev.schedule(pods, synth.T0, matches=[[0]])
        assert c.tolist() == [0] and ev.last_allocations()["reservation"].tolist() == [into]
        assert (s[0] >= 5000) == bool(into)
        ev.close()


def test_matched_batch_pods_parity(gpu):
    """KE_RSV_MATCHED pods requesting batch / mid resources (KE_RES_BATCH_* / MID_*, LoadAware's translated names):
    a reservation holds only cpu / memory, so they reach the Reservation plugin as fitsNode's other resources and
    nothing else -- placements, totals and reservation state bit-exact with the oracle."""
    ev, o, pods, matches = _matched_setup(300, 1001, 300)
    rng = np.random.default_rng(1002)
    lists = [m for m in matches if m]
    batch = np.flatnonzero((pods["requests"][:, 2:] != 0).any(1) & (pods["numa_topology_policy"] == 0)
                           & (pods["has_other_requests"] == 0) & (pods["device_requests"] == 0).all(1)
                           & (pods["reservation_matched"] == abi.RSV_NONE))
    assert len(batch) >= 10
    for p in batch[::2]:
        pods["reservation_matched"][p] = abi.RSV_MATCHED
        matches[p] = lists[int(rng.integers(len(lists)))]
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    _resv_equal(ev, o)
    assert np.array_equal(ev.last_allocations()["reservation"], o.last_allocations()["reservation"])
    assert ev.check_records(synth.T0) == 0
    ev.close()


@pytest.mark.parametrize("world,affinity", [(2, 0.0), (3, 0.4), (8, 0.0)])
def test_matched_reservations_sharded_loopback(gpu, world, affinity):
    """Node-sharded contexts (loopback: every shard in this context) with matched and affinity pods: the
    Reservation plugin runs in stages over each shard's pairs (k_rsv_stage; on real ranks an all-reduce between the
    stages) against the merged lists' top -- placements, totals, reservation state bit-exact with the oracle."""
    ev, o, pods, matches = _matched_setup(300, 1011 + world, 260, affinity=affinity)
    ev.shard_init(0, world, None)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    _resv_equal(ev, o)
    a1 = ev.last_allocations()
    assert np.array_equal(a1["reservation"], o.last_allocations()["reservation"])
    assert (a1["reservation"] > 0).sum() >= 5
    ev.close()


def _general_setup(n, seed, n_pods):
    """Reservations whose allocatable names batch-cpu / batch-memory / ephemeral storage / nvidia.com/gpu and
    "pods" besides cpu / memory (ke_reservations_load_full; resource ids of synth.XRES), some with a reserved part
    (the node-reservation annotation) or names left out of a Restricted one's ResourceNames, their reserve pods in
    NodeInfo (cpu / memory and the scalar rows); NodeResourcesFit (Filter + Score over the scalars) and FitPlus in
    the profile; about half of the eligible pods (batch and scalar requests included) match a group."""
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    tables = synth.make_node_resources(cl, synth.BASE_SEED + seed + 1)
    rs, ents, grp = [], [], []
    for g in range(8):
        for _ in range(int(rng.integers(2, 6))):
            node = int(rng.integers(0, n))
            r = abi.Reservation(node=node, available=int(rng.random() < 0.95), allocate_once=int(rng.random() < 0.2),
                                allocate_policy=int(rng.integers(0, 3)), allocated_pods=int(rng.choice([0, 0, 1, 2])),
                                order=int(rng.choice([0, 0, 0, 5, 9])))
            r.allocatable[0] = int(rng.choice([0, 2000, 4000, 8000]))
            r.allocatable[1] = int(rng.choice([0, 4, 8, 16])) * 2**30
            if r.allocated_pods:
                r.allocated[0], r.allocated[1] = r.allocatable[0] // 2, r.allocatable[1] // 4
            if rng.random() < 0.15:
                r.reserved[0] = r.allocatable[0] // 4
            if r.allocate_policy == abi.RSV_POLICY_RESTRICTED and rng.random() < 0.2:
                r.names_excluded = 1 << int(rng.integers(0, 2))
            e = []
            for rid, lo, hi, unit in ((2, 1, 8, 1000), (3, 1, 16, 2**30), (4, 1, 20, 2**30), (5, 1, 4, 1)):
                if rng.random() < 0.45:
                    a = int(rng.integers(lo, hi + 1)) * unit
                    al = int(rng.choice([0, a // 2, a])) if r.allocated_pods else 0
                    e.append((rid, a, al, int(rng.random() < 0.1) * (a // 4), int(rng.random() < 0.1)))
            if rng.random() < 0.2:
                e.append((abi.RSV_RES_PODS, int(rng.integers(1, 4)), 0, 0, 0))
            x = np.zeros(len(e), abi.RESERVATION_RESOURCE_DTYPE)
            for q, (rid, a, al, rsv, exc) in enumerate(e):
                x[q]["id"], x[q]["allocatable"], x[q]["allocated"], x[q]["reserved"], x[q]["excluded"] = rid, a, al, rsv, exc
            if len(e):
                r.holds |= abi.RSV_OTHER_ALLOCATABLE
            # the reserve pod is in NodeInfo: cpu / memory, and its scalars in the node's rows
            cl.nodes["requested"][node, 0] += r.allocatable[0]
            cl.nodes["requested"][node, 1] += r.allocatable[1]
            t = tables[node]
            for rid, a, _, _, _ in e:
                if rid == abi.RSV_RES_PODS:
                    continue
                hit = np.flatnonzero(t["id"] == rid)
                if len(hit):
                    t["requested"][hit[0]] += a
                else:
                    row = np.zeros(1, abi.NODE_RESOURCE_DTYPE)
                    row["id"], row["allocatable"], row["requested"] = rid, 2 * a, a
                    t = np.concatenate([t, row])
            tables[node] = t
            rs.append(r)
            ents.append(x)
            grp.append(g)
    cfg = synth.fit_config(synth.ext_config(synth.config(n)))
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_node_resources(h, tables)
        h.reservations_load(rs, resources=ents)
    pods = synth.add_pod_xres(synth.make_pods(n_pods, synth.BASE_SEED + seed + 2), synth.BASE_SEED + seed + 3)
    cpuset = np.isin(pods["qos_class"], [abi.QOS_LSE, abi.QOS_LSR]) & (pods["priority_class"] == abi.PRIORITY_PROD)
    elig = ((pods["numa_topology_policy"] == 0) & (pods["has_other_requests"] <= 1)
            & (pods["device_requests"] == 0).all(1) & ~cpuset)
    grp = np.asarray(grp)
    matches = [[] for _ in range(n_pods)]
    for p in np.flatnonzero(elig & (rng.random(n_pods) < 0.5)):
        pods["reservation_matched"][p] = abi.RSV_AFFINITY if rng.random() < 0.15 else abi.RSV_MATCHED
        matches[p] = np.flatnonzero(grp == rng.integers(0, 8)).tolist()
    return ev, o, pods, matches, rs


def test_general_reservation_resources_parity(gpu):
    """Reservations naming resources beyond cpu / memory (VERDICT r5 missing 2): the scalar NodeInfo restore every pod
    sees (NodeResourcesFit's Filter / Score and FitPlus rows), and for matched pods the name check, fitsNode's scalars,
    fitsReservation's pods cap / reserved / ResourceNames, scoreReservation over every name, Reserve's allocated per
    name -- bit-exact with the oracle on placements, totals and reservation state; then Unreserve and a second queue."""
    ev, o, pods, matches, rs = _general_setup(300, 1361, 240)
    assert sum(1 for m in matches if m) > 40
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    _resv_equal(ev, o)
    for i in range(len(rs)):
        a, b = ev.reservation_resources_get(i), o.reservation_resources_get(i)
        assert np.array_equal(a["allocated"], b["allocated"]), i
    assert any((ev.reservation_resources_get(i)["allocated"] > 0).any() for i in range(len(rs)))
    rec, rec0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(rec["reservation"], rec0["reservation"]) and (rec["reservation"] > 0).sum() > 5
    for p in np.flatnonzero(rec["reservation"] > 0)[::3]:
        ev.release(pods[p], rec[p])
        o.release(pods[p], rec0[p])
    _resv_equal(ev, o)
    for i in range(len(rs)):
        assert np.array_equal(ev.reservation_resources_get(i)["allocated"], o.reservation_resources_get(i)["allocated"])
    more = synth.add_pod_xres(synth.make_pods(120, synth.BASE_SEED + 1365, key_base=9_950_000_000),
                              synth.BASE_SEED + 1366)
    c1, s1 = ev.schedule(more, synth.T0)
    c0, s0 = o.schedule(more, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert ev.check_records(synth.T0) == 0
    ev.close()


@pytest.mark.parametrize("n_nodes", [300, 24], ids=["spread", "crowded"])
def test_fused_matched_pods_parity(gpu, n_nodes):
    """Matched pods fused behind their plain segment: nomination and rows taken before the segment ran,
    k_rsv_check gating the pod when a plain pod of the segment took a node of its reservations (then it runs again
    alone).  On 300 nodes most matched pods run fused; on 24 nodes, most carrying reservations, plain pods keep taking
    their nodes and the gate fires -- bit-exact with the oracle on placements, scores, reservation state and release
    records either way."""
    ev, o, pods, matches = _matched_setup(n_nodes, 977, 400)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    fused, gated = ev.rsv_fused()
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    _resv_equal(ev, o)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    for k in ("node", "reservation"):
        assert np.array_equal(a1[k], a0[k]), k
    assert fused >= 10
    if n_nodes == 24:
        assert gated >= 1
    assert ev.check_records(synth.T0) == 0
