"""Reservations whose reserve pods hold NUMA resources, cpusets and device instances (ke_reservations_load_ex,
SURVEY.md §8f rank 3) on the GPU: every pod that does not match them sees the plugins' restore states -- the
unmatched reservations' owners' part given back as NodeNUMAResource's reusableResources
(nodenumaresource/reservation.go:111-120, node_allocation.go:221-243) and as DeviceShare's preemptible
(deviceshare/reservation.go:99-108, device_cache.go:322-365) -- bit-exact with the oracle's restatement on eval
matrices, schedules, cpusets, NUMA allocations, device minors and the reservation state."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, KoordEvalError, abi, synth
from oracle.binding import Oracle
from test_gpu_cpuset import assert_eval_equal, assert_schedule_equal

pytestmark = pytest.mark.gpu


def holding_cluster(n, seed, devices=False, frac=0.3):
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1)
    devs = synth.make_devices(n, synth.BASE_SEED + seed + 2) if devices else None
    rs, al, res = synth.make_reservation_holdings(cl, synth.BASE_SEED + seed + 3, zones, tabs, devs, frac=frac)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        if devs is not None:
            synth.load_devices(h, devs)
        h.reservations_load(rs, al, res)
    return ev, o, cl, rs, al, res


def test_holdings_generator_covers_every_kind():
    _, _, _, rs, al, _ = holding_cluster(300, 1301, devices=True)
    h = rs["holds"]
    for bit in (abi.RSV_HOLDS_NUMA, abi.RSV_HOLDS_CPUSET, abi.RSV_HOLDS_DEVICES):
        assert ((h & bit) != 0).sum() >= 5, bit
    assert ((rs["allocated_pods"] > 0) & (h != 0)).sum() >= 10
    assert (al["owner_numa"] > 0).any() and al["owner_cpuset"].any() and (al["owner_device"] > 0).any()


@pytest.mark.parametrize("seed", [1311, 1312])
def test_holdings_unmatched_numa_cpuset_parity(gpu, seed):
    """NUMA-policy nodes (every policy) and cpuset pods: the zones' availability with the unmatched reservations'
    owners given back equals the oracle's restatement -- eval matrices, then a queue with Reserves."""
    ev, o, *_ = holding_cluster(400, seed)
    pods = synth.make_numa_cpuset_pods(500, synth.BASE_SEED + seed + 10)
    assert_eval_equal(ev.eval(pods[:64], synth.T0), o.eval(pods[:64], synth.T0))
    assert_schedule_equal(ev, o, pods, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert ev.check_records(synth.T0) == 0


def test_holdings_unmatched_deviceshare_parity(gpu):
    """DeviceShare pods: the instances the unmatched reservations' owners share with their reserve pods count once
    (calcFreeWithPreemptible) -- raw scores, totals, placements and device minors equal the oracle's."""
    ev, o, *_ = holding_cluster(400, 1321, devices=True, frac=0.5)
    pods = synth.make_ds_pods(400, synth.BASE_SEED + 1322)
    a, b = ev.eval(pods[:64], synth.T0), o.eval(pods[:64], synth.T0)
    assert_eval_equal(a, b)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)
    assert ev.check_records(synth.T0) == 0


def test_holdings_reload_and_release_parity(gpu):
    """A queue, then releases, then a reloaded set with other holdings: the restore states follow every change."""
    ev, o, cl, rs, al, res = holding_cluster(300, 1331, devices=True)
    pods = synth.make_numa_cpuset_pods(300, synth.BASE_SEED + 1332)
    assert_schedule_equal(ev, o, pods, synth.T0)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    for p in np.flatnonzero(a1["node"] >= 0)[::3]:
        ev.release(pods[p], a1[p], abi.RELEASE_DELETE)
        o.release(pods[p], a0[p], abi.RELEASE_DELETE)
    keep = np.arange(len(rs)) % 2 == 0
    for h in (ev, o):
        h.reservations_load(rs[keep], al[keep], [res[i] for i in np.flatnonzero(keep)])
    more = synth.make_numa_cpuset_pods(300, synth.BASE_SEED + 1333, key_base=6_500_000_000)
    assert_eval_equal(ev.eval(more[:48], synth.T0), o.eval(more[:48], synth.T0))
    assert_schedule_equal(ev, o, more, synth.T0)
    assert ev.check_records(synth.T0) == 0
    assert np.array_equal(ev.reservation_allocs_get(), o.reservation_allocs_get())


def cpuset_matched_setup(n, seed, n_pods, affinity=0.3, tight_pods=0.0, node_bind=True):
    """Nodes without NUMA policies carrying CPU tables, reservations whose reserve pods hold cpusets (owner pods
    holding part of them, every allocate policy), and a queue of cpuset pods of which ~40 % match the reservations
    of a few owner groups (KE_RSV_MATCHED, or KE_RSV_AFFINITY for `affinity` of them).  `tight_pods`: that fraction
    of the reservation nodes has its pod limit just at its pod count (fitsNode's pod check binds)."""
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.0)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1, policy_weights=(1, 0, 0, 0))
    if not node_bind:
        cl.nodes["cpu_bind_policy"] = 0
    rs, al, res = synth.make_reservation_holdings(cl, synth.BASE_SEED + seed + 2, zones, tabs, None, frac=0.5)
    for i in np.unique(rs["node"]):
        if rng.random() < tight_pods:
            cl.nodes["allowed_pods"][i] = cl.nodes["pod_count"][i] + int(rng.integers(-1, 2))
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.reservations_load(rs, al, res)
    pods = synth.make_cpuset_pods(n_pods, synth.BASE_SEED + seed + 3, cpuset_fraction=0.7)
    grp = rng.integers(0, 8, len(rs))
    matches = [[] for _ in range(n_pods)]
    ok = (pods["numa_topology_policy"] == 0) & (pods["requests"][:, 2:] == 0).all(1) & (pods["has_other_requests"] == 0) \
        & (pods["device_requests"] == 0).all(1)
    for p in np.flatnonzero(ok & (rng.random(n_pods) < 0.4)):
        pods["reservation_matched"][p] = abi.RSV_AFFINITY if rng.random() < affinity else abi.RSV_MATCHED
        matches[p] = np.flatnonzero(grp == rng.integers(0, 8)).tolist()
    return ev, o, pods, matches, rs


def _holdings_equal(ev, o):
    a, b = ev.reservations_get(), o.reservations_get()
    assert np.array_equal(a["allocated"], b["allocated"]) and np.array_equal(a["allocated_pods"], b["allocated_pods"])
    assert np.array_equal(ev.reservation_allocs_get(), o.reservation_allocs_get())


@pytest.mark.parametrize("seed,affinity,tight", [(1361, 0.0, 0.0), (1362, 0.5, 0.0), (1363, 0.3, 0.4)],
                         ids=["matched", "affinity", "pod-limits"])
def test_matched_cpuset_from_reservations_parity(gpu, seed, affinity, tight):
    """Cpuset pods matching reservations that hold cpusets (nodes without NUMA policies): NodeNUMAResource's Filter
    tries the matched reservations first (k_rsv_views: takePreferredCPUs on the reservations' CPUs, the Restricted
    policy's second allocation), the nomination filters them under an affinity, Reserve allocates from the
    nominated one -- placements, scores, cpusets, reservation state and owner cpusets bit-exact with the oracle;
    then Unreserve of part of them and a second queue."""
    ev, o, pods, matches, rs = cpuset_matched_setup(300, seed, 300, affinity, tight)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    diff = np.argwhere(np.any(ev.last_cpusets != o.last_cpusets, axis=1))
    assert len(diff) == 0, diff[:5].ravel().tolist()
    _holdings_equal(ev, o)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(a1["reservation"], a0["reservation"])
    into = np.flatnonzero(a1["reservation"] > 0)
    assert len(into) >= 5
    held = [p for p in into if rs["holds"][a1["reservation"][p] - 1] & abi.RSV_HOLDS_CPUSET and a1["cpuset"][p].any()]
    assert len(held) >= 2  # cpusets taken out of holding reservations
    for p in into[::3]:
        ev.unreserve(pods[p], int(p))
        o.release(pods[p], a0[p], abi.RELEASE_UNRESERVE)
    _holdings_equal(ev, o)
    more = synth.make_cpuset_pods(200, synth.BASE_SEED + seed + 7, key_base=7_700_000_000)
    m2 = [matches[p % len(matches)] if pods["reservation_matched"][p % len(matches)] else [] for p in range(len(more))]
    more["reservation_matched"] = [pods["reservation_matched"][p % len(matches)] for p in range(len(more))]
    more["numa_topology_policy"] = 0
    more["device_requests"] = 0
    more["has_other_requests"] = np.where(np.array([len(m) > 0 for m in m2]), 0, more["has_other_requests"])
    more["requests"][:, 2:] = np.where(np.array([len(m) > 0 for m in m2])[:, None], 0, more["requests"][:, 2:])
    c1, s1 = ev.schedule(more, synth.T0, matches=m2)
    c0, s0 = o.schedule(more, synth.T0, matches=m2)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    _holdings_equal(ev, o)
    assert ev.check_records(synth.T0) == 0


def test_ignored_pods_beside_held_cpusets(gpu):
    """Reservation-ignored pods in a cluster whose reservations hold NUMA resources and cpusets (nodes without NUMA
    policies), between cpuset pods and matched cpuset pods: every reservation's matched restore for them; an ignored
    cpuset pod allocates on a node with held CPUs through tryAllocateIgnoreReservation (one trial with every held
    CPU preferred, k_rsv_views; a failed trial fails Filter and Reserve), elsewhere from the node -- placements,
    scores, cpusets and reservation state bit-exact with the oracle.  An ignored pod with a NUMA policy under a required
    FullPCPUs binding is refused by both (preferredCPUs taken first may split cores)."""
    ev, o, pods, matches, rs = cpuset_matched_setup(300, 1371, 300, affinity=0.0, node_bind=False)
    cs = np.isin(pods["qos_class"], [abi.QOS_LSE, abi.QOS_LSR]) & (pods["priority_class"] == abi.PRIORITY_PROD)
    free = np.flatnonzero(pods["reservation_matched"] == abi.RSV_NONE)
    ign = free[::2]
    assert (~cs[ign]).sum() >= 20 and cs[ign].sum() >= 20
    pods["reservation_matched"][ign] = abi.RSV_IGNORED
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    diff = np.argwhere(np.any(ev.last_cpusets != o.last_cpusets, axis=1))
    assert len(diff) == 0, diff[:5].ravel().tolist()
    _holdings_equal(ev, o)
    a1 = ev.last_allocations()
    assert (a1["reservation"][ign] == 0).all()
    held = np.zeros(300, bool)
    held[rs["node"][(rs["holds"] & abi.RSV_HOLDS_CPUSET) != 0]] = True
    on_held = [p for p in ign if cs[p] and c1[p] >= 0 and held[c1[p]] and a1["cpuset"][p].any()]
    assert len(on_held) >= 3  # ignored cpuset pods placed on nodes with held CPUs
    assert ev.check_records(synth.T0) == 0
    bad = synth.make_cpuset_pods(4, synth.BASE_SEED + 1375, cpuset_fraction=1.0, key_base=7_900_000_000)
    bad["reservation_matched"][1] = abi.RSV_IGNORED
    bad["numa_topology_policy"][1] = abi.NUMA_POLICY_BEST_EFFORT
    bad["cpu_bind_required"][1] = abi.CPU_BIND_FULL_PCPUS
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(bad, synth.T0)
    assert e.value.code == abi.ERR_UNSUPPORTED
    with pytest.raises(RuntimeError, match=f"rc={abi.ERR_UNSUPPORTED}"):
        o.schedule(bad, synth.T0)


def test_matched_cpuset_sharded_loopback(gpu):
    """Matched cpuset pods from CPU-holding reservations in a node-sharded context (loopback, 3 shards): the views,
    the Filter / Reserve decisions and the staged Reservation pick -- bit-exact with the oracle."""
    ev, o, pods, matches, rs = cpuset_matched_setup(300, 1381, 200, affinity=0.3)
    ev.shard_init(0, 3, None)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    _holdings_equal(ev, o)


@pytest.mark.parametrize("seed", [1391, 1392])
def test_ignored_numa_pods_beside_held_numa(gpu, seed):
    """Reservation-ignored pods binding no CPUs (nodes without a bind policy) in a cluster whose reservations hold
    NUMA allocations and cpusets on nodes of every NUMA policy: their rows carry every reservation's matched restore,
    NodeNUMAResource's reusable resources being the reserve pods' whole NUMA allocations (mergedMatchedAllocatable,
    nodenumaresource/resource_manager.go:130-138; tryAllocateIgnoreReservation's mergedMatchedAllocated + Σ remained,
    reservation.go:437-490) -- in the hints, the zones' distribution and Reserve.  Pods with their own NUMA policy among
    them; cpuset pods between them.  Placements, scores, NUMA allocations, cpusets and reservation state bit-exact
    with the oracle (the CPU twin: test_reservations.py::test_ignored_numa_pod_reuses_the_held_zone)."""
    n = 400
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1)
    cl.nodes["cpu_bind_policy"] = 0
    rs, al, res = synth.make_reservation_holdings(cl, synth.BASE_SEED + seed + 3, zones, tabs, None, frac=0.5)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.reservations_load(rs, al, res)
    pods = synth.make_numa_cpuset_pods(400, synth.BASE_SEED + seed + 10, cpuset_fraction=0.3, policy_fraction=0.3)
    cs = np.isin(pods["qos_class"], [abi.QOS_LSE, abi.QOS_LSR]) & (pods["priority_class"] == abi.PRIORITY_PROD)
    pods["numa_topology_policy"][cs] = 0
    ign = np.flatnonzero(~cs)[::2]
    pods["reservation_matched"][ign] = abi.RSV_IGNORED
    assert len(ign) >= 100 and (pods["numa_topology_policy"][ign] != 0).sum() >= 20
    assert_schedule_equal(ev, o, pods, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    _holdings_equal(ev, o)
    c = ev.last_allocations()["node"]
    pol = cl.nodes["numa_topology_policy"] != 0
    held = np.zeros(n, bool)
    held[rs["node"][(rs["holds"] & abi.RSV_HOLDS_NUMA) != 0]] = True
    on_held = [p for p in ign if c[p] >= 0 and held[c[p]] and pol[c[p]] and ev.last_numa_allocations[p].any()]
    assert len(on_held) >= 3  # ignored pods given NUMA allocations on policy nodes with held zones
    assert ev.check_records(synth.T0) == 0


def numa_matched_setup(n, seed, n_pods, affinity):
    """Nodes of every NUMA policy without a CPU bind policy, reservations whose reserve pods hold NUMA amounts and
    cpusets (owners holding part of them, every allocate policy), a queue where half of the pods binding no CPUs --
    40 % of the queue carrying a NUMA policy of its own -- match the reservations of one of 8 owner groups
    (KE_RSV_MATCHED, or KE_RSV_AFFINITY for `affinity` of them), between cpuset pods."""
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1)
    cl.nodes["cpu_bind_policy"] = 0
    rs, al, res = synth.make_reservation_holdings(cl, synth.BASE_SEED + seed + 2, zones, tabs, None, frac=0.5)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.reservations_load(rs, al, res)
    pods = synth.make_numa_cpuset_pods(n_pods, synth.BASE_SEED + seed + 3, cpuset_fraction=0.3, policy_fraction=0.4)
    cs = np.isin(pods["qos_class"], [abi.QOS_LSE, abi.QOS_LSR]) & (pods["priority_class"] == abi.PRIORITY_PROD)
    grp = rng.integers(0, 8, len(rs))
    matches = [[] for _ in range(n_pods)]
    ok = ~cs & (pods["requests"][:, 2:] == 0).all(1) & (pods["has_other_requests"] == 0) \
        & (pods["device_requests"] == 0).all(1)
    for p in np.flatnonzero(ok & (rng.random(n_pods) < 0.5)):
        pods["reservation_matched"][p] = abi.RSV_AFFINITY if rng.random() < affinity else abi.RSV_MATCHED
        matches[p] = np.flatnonzero(grp == rng.integers(0, 8)).tolist()
    return cl, ev, o, pods, matches, rs


@pytest.mark.parametrize("seed,affinity", [(1401, 0.0), (1402, 0.5)], ids=["matched", "affinity"])
def test_matched_numa_policy_from_reservations_parity(gpu, seed, affinity):
    """Reservation-matched pods binding no CPUs under NUMA policies (the node's, or their own) on nodes of their
    reservations holding NUMA amounts / cpusets: NodeNUMAResource's hints over the allocate-from-reservation trials
    (k_numa_views: tryAllocateFromReservation per mask, then tryAllocateFromNode; nodenumaresource/resource_manager.go
    :586-594, reservation.go:270-424), FilterNominateReservation under an affinity, the Score and Reserve from the
    nominated reservation's allocation on the affinity (Restricted: over its remained) -- placements, scores, NUMA
    allocations, cpusets and the reservation state bit-exact with the oracle; then Unreserve of part of them and a
    second queue."""
    cl, ev, o, pods, matches, rs = numa_matched_setup(400, seed, 300, affinity)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    diff = np.argwhere(np.any(ev.last_numa_allocations != o.last_numa_allocations, axis=1))
    assert len(diff) == 0, diff[:5].ravel().tolist()
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    _holdings_equal(ev, o)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(a1["reservation"], a0["reservation"])
    pol = cl.nodes["numa_topology_policy"] != 0
    m = np.flatnonzero(pods["reservation_matched"] != 0)
    numa_into = [p for p in m if a1["reservation"][p] > 0 and c1[p] >= 0 and pol[c1[p]] and
                 ev.last_numa_allocations[p].any()]
    assert len(numa_into) >= 10  # NUMA allocations taken out of holding reservations on policy nodes
    assert sum(pods["numa_topology_policy"][p] != 0 for p in numa_into) >= 3  # pods with their own policy
    assert ev.check_records(synth.T0) == 0
    for p in np.flatnonzero(a1["reservation"] > 0)[::3]:
        ev.unreserve(pods[p], int(p))
        o.release(pods[p], a0[p], abi.RELEASE_UNRESERVE)
    _holdings_equal(ev, o)
    more = synth.make_numa_cpuset_pods(200, synth.BASE_SEED + seed + 7, cpuset_fraction=0.0, policy_fraction=0.4,
                                       key_base=7_800_000_000)
    m2 = [matches[p % len(matches)] for p in range(len(more))]
    more["reservation_matched"] = [pods["reservation_matched"][p % len(matches)] for p in range(len(more))]
    keep = np.array([len(x) > 0 for x in m2])
    more["requests"][:, 2:] = np.where(keep[:, None], 0, more["requests"][:, 2:])
    more["has_other_requests"] = np.where(keep, 0, more["has_other_requests"])
    more["device_requests"] = np.where(keep[:, None], 0, more["device_requests"])
    c1, s1 = ev.schedule(more, synth.T0, matches=m2)
    c0, s0 = o.schedule(more, synth.T0, matches=m2)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    _holdings_equal(ev, o)
    assert ev.check_records(synth.T0) == 0


def test_matched_numa_policy_sharded_loopback(gpu):
    """The same pods in a node-sharded context (loopback, 3 shards): the NUMA views, the staged Reservation pick
    (a Score error on any rank's feasible node fails the pod) -- bit-exact with the oracle."""
    cl, ev, o, pods, matches, rs = numa_matched_setup(300, 1403, 200, 0.3)
    ev.shard_init(0, 3, None)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    _holdings_equal(ev, o)


@pytest.mark.parametrize("order2,placed", [(1, False), (0, True)], ids=["r2-nominated", "r1-nominated"])
def test_numa_score_error_parity(gpu, order2, placed):
    """NodeNUMAResource's Score error on a feasible node (the nominated reservation's allocation and the node's own
    both fail on the stored affinity) fails the pod's cycle although another node is feasible (RSV_PAIR_SCORE_ERROR
    in k_rsv_pick); with the other reservation nominated the pod is placed -- as the oracle (the CPU twin:
    test_reservations.py::test_numa_score_error_fails_the_pod)."""
    from test_reservations import score_error_case
    cl, full, empty, r, a, pods = score_error_case()
    r["order"][1] = order2
    cfg = synth.config(2)
    ev, o = Evaluator(cfg), Oracle(cfg, 2)
    for h in (ev, o):
        synth.load_into(h, cl)
        for i in range(2):
            h.delete_nodemetric(i)
        h.set_numa(0, full)
        h.set_numa(1, empty)
        h.reservations_load(r, a)
    c1, s1 = ev.schedule(pods, synth.T0, matches=[[0, 1]])
    c0, s0 = o.schedule(pods, synth.T0, matches=[[0, 1]])
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0), (c1, c0)
    assert (c1[0] >= 0) == placed
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    _holdings_equal(ev, o)


def numa_bind_matched_setup(n, seed, n_pods, affinity):
    """numa_matched_setup with CPU bind policies on the nodes (none / SpreadByPCPUs) and matched pods binding CPUs:
    whole-CPU requests, the pods' required bind policies outside FullPCPUs (the refusal: preferredCPUs taken first may
    split cores there), half of the queue matching the reservations of one of 8 owner groups."""
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1, bind_weights=(0.6, 0.0, 0.4))
    rs, al, res = synth.make_reservation_holdings(cl, synth.BASE_SEED + seed + 2, zones, tabs, None, frac=0.5)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.reservations_load(rs, al, res)
    pods = synth.make_numa_cpuset_pods(n_pods, synth.BASE_SEED + seed + 3, cpuset_fraction=0.5, policy_fraction=0.4)
    pods["requests"][:, abi.RES_CPU] = np.maximum(1000, pods["requests"][:, abi.RES_CPU] // 1000 * 1000)
    pods["limits"][:, abi.RES_CPU] = np.maximum(pods["limits"][:, abi.RES_CPU], pods["requests"][:, abi.RES_CPU])
    pods["cpu_bind_required"][np.isin(pods["cpu_bind_required"], [abi.CPU_BIND_DEFAULT, abi.CPU_BIND_FULL_PCPUS])] = \
        abi.CPU_BIND_SPREAD_BY_PCPUS
    grp = rng.integers(0, 8, len(rs))
    matches = [[] for _ in range(n_pods)]
    ok = (pods["requests"][:, 2:] == 0).all(1) & (pods["has_other_requests"] == 0) & (pods["device_requests"] == 0).all(1)
    for p in np.flatnonzero(ok & (rng.random(n_pods) < 0.5)):
        pods["reservation_matched"][p] = abi.RSV_AFFINITY if rng.random() < affinity else abi.RSV_MATCHED
        matches[p] = np.flatnonzero(grp == rng.integers(0, 8)).tolist()
    return cl, ev, o, pods, matches, rs


@pytest.mark.parametrize("seed,affinity", [(1421, 0.0), (1422, 0.5)], ids=["matched", "affinity"])
def test_matched_binding_pods_numa_policy_parity(gpu, seed, affinity):
    """Reservation-matched pods binding CPUs under NUMA policies on nodes of their reservations holding NUMA amounts /
    cpusets: k_numa_views' views carry preferredCPUs (the hint view's mergedMatchedRemainCPUs, a trial's
    mergedMatchedAllocatedCPUs + its remainedCPUs, a Restricted trial's remainedCPUs) -- per-view CPU availability,
    trimNUMANodeResources, allocateCPUSet's take by counts -- and after the nomination the cpuset pass (k_rsv_views over
    the allocation's zones) gives Reserve's cpuset and the Score's requested cpu (scoring.go:179-185).  Placements,
    scores, NUMA allocations, cpusets and the reservation state bit-exact with the oracle (allocateCPUSet itself)."""
    cl, ev, o, pods, matches, rs = numa_bind_matched_setup(300, seed, 250, affinity)
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0), np.argwhere(s1 != s0)[:5].ravel().tolist()
    diff = np.argwhere(np.any(ev.last_numa_allocations != o.last_numa_allocations, axis=1))
    assert len(diff) == 0, diff[:5].ravel().tolist()
    diff = np.argwhere(np.any(ev.last_cpusets != o.last_cpusets, axis=1))
    assert len(diff) == 0, diff[:5].ravel().tolist()
    _holdings_equal(ev, o)
    a1 = ev.last_allocations()
    pol = cl.nodes["numa_topology_policy"] != 0
    m = np.flatnonzero(pods["reservation_matched"] != 0)
    into = [p for p in m if a1["reservation"][p] > 0 and c1[p] >= 0 and (pol[c1[p]] or pods["numa_topology_policy"][p])
            and a1["cpuset"][p].any() and ev.last_numa_allocations[p].any()]
    assert len(into) >= 10  # binding pods given cpusets and NUMA allocations out of holding reservations
    assert ev.check_records(synth.T0) == 0


def test_matched_binding_pod_full_pcpus_refused(gpu):
    """A matched pod under a required FullPCPUs policy (its own, or the node's FullPCPUsOnly) beside a reservation
    holding NUMA amounts / CPUs under a NUMA policy: KE_ERR_UNSUPPORTED from both (preferredCPUs taken first may
    split cores there, which the per-view counts do not see)."""
    cl, ev, o, pods, matches, rs = numa_bind_matched_setup(300, 1423, 60, 0.0)
    pol = cl.nodes["numa_topology_policy"] != 0
    holding = [r for r in range(len(rs)) if pol[rs["node"][r]] and rs["holds"][r] & (abi.RSV_HOLDS_NUMA | abi.RSV_HOLDS_CPUSET)
               and rs["available"][r]]
    assert holding
    bad = pods[:1].copy()
    bad["priority_class"], bad["qos_class"] = abi.PRIORITY_PROD, abi.QOS_LSR
    bad["requests"][0, :] = 0
    bad["requests"][0, abi.RES_CPU], bad["requests"][0, abi.RES_MEMORY] = 2000, 2**30
    bad["cpu_bind_required"], bad["cpu_bind_preferred"] = abi.CPU_BIND_FULL_PCPUS, abi.CPU_BIND_FULL_PCPUS
    bad["has_other_requests"], bad["device_requests"] = 0, 0
    bad["reservation_matched"] = abi.RSV_MATCHED
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(bad, synth.T0, matches=[[holding[0]]])
    assert e.value.code == abi.ERR_UNSUPPORTED
    with pytest.raises(RuntimeError, match=f"rc={abi.ERR_UNSUPPORTED}"):
        o.schedule(bad, synth.T0, matches=[[holding[0]]])


def test_numa_policy_golden_cases_through_schedule(gpu):
    """TestPlugin_Reserve's NUMA-policy cases (plugin_test.go:1268-1398, tests/golden/reservation_restore.json) as
    whole scheduling cycles of the matched pod on the test's node -- the binding pod's (preferring FullPCPUs)
    included: GPU and oracle agree on placement, score, cpuset, NUMA allocation and reservation state; the binding
    Restricted case takes the test's cpus 4-7 and 4 cpu on NUMA node 0 (:1268-1297)."""
    from test_reservations import POLICY, _reserve_node, policy_reservation, policy_pod, _cpus
    for case in POLICY:
        hs = [_reserve_node(case, 1391, Evaluator(synth.config(1))), _reserve_node(case, 1391)]
        r, a = policy_reservation(case)
        pods = np.array([policy_pod(case)])
        pods["reservation_matched"] = abi.RSV_AFFINITY if case["required"] else abi.RSV_MATCHED
        out = []
        for h in hs:
            h.reservations_load(r, a)
            c, s = h.schedule(pods, synth.T0, matches=[[0]])
            out.append((c, s, h.last_cpusets.copy(), h.last_numa_allocations.copy(), h.last_allocations()["reservation"]))
        for x, y in zip(*out):
            assert np.array_equal(x, y), case["name"]
        if case["name"] == "numa_cpuset_restricted":
            c, s, cpus, numa, into = out[0]
            assert c[0] == 0 and into[0] == 1
            assert np.array_equal(cpus[0], _cpus(case["want_cpus"]))
            assert numa[0][0] == 4000 and not numa[0][1:].any()


@pytest.mark.parametrize("seed", [1431, 1432])
def test_ignored_binding_pods_numa_policy_parity(gpu, seed):
    """Reservation-ignored pods binding CPUs under NUMA policies (the node's or their own) beside reservations holding
    NUMA amounts / cpusets: every mask's Allocate in their hints is tryAllocateIgnoreReservation (reservation.go:437-490:
    reservedCPUsFromIgnored preferred, the held amounts reusable), the hint view prefers mergedMatchedRemainCPUs
    (resource_manager.go:130-138); Score and Reserve from the same allocation (k_numa_views with one trial, then the
    cpuset pass).  Placements, scores, NUMA allocations, cpusets and reservation state bit-exact with the oracle."""
    n = 300
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1, bind_weights=(0.6, 0.0, 0.4))
    rs, al, res = synth.make_reservation_holdings(cl, synth.BASE_SEED + seed + 2, zones, tabs, None, frac=0.5)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.reservations_load(rs, al, res)
    pods = synth.make_numa_cpuset_pods(250, synth.BASE_SEED + seed + 3, cpuset_fraction=0.5, policy_fraction=0.4)
    pods["requests"][:, abi.RES_CPU] = np.maximum(1000, pods["requests"][:, abi.RES_CPU] // 1000 * 1000)
    pods["limits"][:, abi.RES_CPU] = np.maximum(pods["limits"][:, abi.RES_CPU], pods["requests"][:, abi.RES_CPU])
    pods["cpu_bind_required"][np.isin(pods["cpu_bind_required"], [abi.CPU_BIND_DEFAULT, abi.CPU_BIND_FULL_PCPUS])] = \
        abi.CPU_BIND_SPREAD_BY_PCPUS
    ign = np.flatnonzero((pods["device_requests"] == 0).all(1) & (rng.random(250) < 0.5))
    pods["reservation_matched"][ign] = abi.RSV_IGNORED
    assert_schedule_equal(ev, o, pods, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    _holdings_equal(ev, o)
    c, a = ev.last_allocations()["node"], ev.last_allocations()
    pol = cl.nodes["numa_topology_policy"] != 0
    held = np.zeros(n, bool)
    held[rs["node"][(rs["holds"] & (abi.RSV_HOLDS_NUMA | abi.RSV_HOLDS_CPUSET)) != 0]] = True
    on_held = [p for p in ign if c[p] >= 0 and held[c[p]] and (pol[c[p]] or pods["numa_topology_policy"][p])
               and a["cpuset"][p].any()]
    assert len(on_held) >= 10  # ignored binding pods given cpusets on policy nodes with held CPUs
    assert ev.check_records(synth.T0) == 0


def many_per_node_setup(n, seed, n_pods, layers=12):
    """`layers` rounds of reservation holdings on every node (each round's reserve pods hold NUMA amounts / cpusets out
    of what the earlier rounds left), so a node carries up to `layers` NUMA/CPU-holding reservations; matched pods list
    every reservation of three random nodes (more than 8 holding ones on a node: beyond the earlier NV_MAX of 8)."""
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1)
    cl.nodes["cpu_bind_policy"] = 0
    rs, al, res = [], [], []
    for layer in range(layers):
        r, a, x = synth.make_reservation_holdings(cl, synth.BASE_SEED + seed + 10 + layer, zones, tabs, None, frac=1.0)
        rs.append(r), al.append(a), res.extend(x)
    rs, al = np.concatenate(rs), np.concatenate(al)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.reservations_load(rs, al, res)
    pods = synth.make_numa_cpuset_pods(n_pods, synth.BASE_SEED + seed + 3, cpuset_fraction=0.3, policy_fraction=0.4)
    cs = np.isin(pods["qos_class"], [abi.QOS_LSE, abi.QOS_LSR]) & (pods["priority_class"] == abi.PRIORITY_PROD)
    ok = ~cs & (pods["requests"][:, 2:] == 0).all(1) & (pods["has_other_requests"] == 0) \
        & (pods["device_requests"] == 0).all(1)
    matches = [[] for _ in range(n_pods)]
    for p in np.flatnonzero(ok & (rng.random(n_pods) < 0.9)):
        pods["reservation_matched"][p] = abi.RSV_MATCHED
        nodes = rng.choice(n, 3, replace=False)
        matches[p] = np.flatnonzero(np.isin(rs["node"], nodes)).tolist()
    holds = (al["numa"] != 0).any(1) | (al["cpuset"] != 0).any(1)
    per_node = np.bincount(rs["node"][holds & (rs["available"] != 0)], minlength=n)
    return cl, ev, o, pods, matches, per_node, rs


def test_matched_numa_policy_many_reservations_per_node(gpu):
    """More than 8 (up to NV_MAX = 31) NUMA/CPU-holding matched reservations on one node under NUMA policies:
    k_numa_views runs one lane per trial and per requiredResources view (2 + 2 x 31 lanes = the wave) -- placements,
    scores, NUMA allocations, cpusets and reservation state bit-exact with the oracle."""
    cl, ev, o, pods, matches, per_node, _ = many_per_node_setup(48, 1501, 160)
    assert per_node.max() > 8
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    _holdings_equal(ev, o)
    a1, a0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(a1["reservation"], a0["reservation"])
    into = np.flatnonzero(a1["reservation"] > 0)
    assert len(into) >= 8 and (per_node[c1[into]] > 8).sum() >= 3  # placed into reservations of crowded nodes
    assert ev.check_records(synth.T0) == 0
