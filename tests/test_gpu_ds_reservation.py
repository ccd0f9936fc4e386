"""DeviceShare allocate-from-reservation on the GPU: reservation-matched and
-ignored DeviceShare pods over reservations whose reserve pods hold GPU / RDMA instances.  k_ds_views runs each
pod's allocator views (per matched reservation: mergedMatchedAllocated + its remained preemptible, its minors
preferred, a Restricted one's minors required with requiredDeviceResources; the node's own with the matched
allocatable; an ignored pod's tryAllocateIgnoreReservation), the host takes DeviceShare's Filter / nomination
(FilterNominateReservation + the normalized ScoreReservation) / Score / Reserve decisions from them, the eval and
Reserve kernels apply them -- placements, totals, device minors, reservation state and owner parts bit-exact with
the oracle, whose restatement is pinned by tests/test_ds_reservation.py."""
import numpy as np
import pytest

import ds_rsv_cases as dc
from koordinator_amd import Evaluator, abi, model, synth
from oracle.binding import Oracle

pytestmark = pytest.mark.gpu


def _both(cfg, n):
    return [Evaluator(cfg), Oracle(cfg, n)]


def _state_equal(ev, o, n):
    a, b = ev.reservations_get(), o.reservations_get()
    assert np.array_equal(a["allocated"], b["allocated"]) and np.array_equal(a["allocated_pods"], b["allocated_pods"])
    assert np.array_equal(ev.reservation_allocs_get(), o.reservation_allocs_get())
    for r in range(len(a)):
        assert np.array_equal(ev.reservation_resources_get(r), o.reservation_resources_get(r)), r
    for i in range(n):
        d1, d0 = ev.node_state(i)[3], o.node_state(i)[3]
        assert np.array_equal(d1, d0), i


def _schedule_equal(ev, o, pods, matches):
    c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
    c0, s0 = o.schedule(pods, synth.T0, matches=matches)
    bad = np.flatnonzero((c1 != c0) | (s1 != s0))
    assert len(bad) == 0, [(int(p), int(c1[p]), int(c0[p]), int(s1[p]), int(s0[p])) for p in bad[:5]]
    a1, a0 = ev.last_allocations(), o.last_allocations()
    assert np.array_equal(a1["reservation"], a0["reservation"])
    assert np.array_equal(a1["device_minors"], a0["device_minors"])
    return c1, a1


@pytest.mark.parametrize("seed,affinity,strategy", [(7101, 0.0, None), (7102, 0.4, None),
                                                    (7103, 0.2, abi.STRATEGY_MOST_ALLOCATED)],
                         ids=["matched", "affinity", "most-allocated"])
def test_ds_matched_from_reservations_parity(gpu, seed, affinity, strategy):
    """A queue of DeviceShare and plain pods, half of them matching one owner group's device-holding reservations
    (every allocate policy), a tenth reservation-ignored: bit-exact placements / scores / minors / state; then
    Unreserve of a third of the pods placed into reservations and a second queue."""
    (ev, o), pods, matches, rs = dc.setup(_both, 240, seed, 320, affinity=affinity, strategy=strategy)
    c1, a1 = _schedule_equal(ev, o, pods, matches)
    _state_equal(ev, o, 240)
    ds = pods["device_requests"].any(1)
    into = np.flatnonzero((a1["reservation"] > 0) & ds & (a1["device_minors"] != 0))
    assert len(into) >= 5  # DeviceShare pods placed into device-holding reservations
    from_rsv = 0  # ... taking devices the reservation holds
    allocs = ev.reservation_allocs_get()
    for p in into:
        from_rsv += int((int(a1["device_minors"][p]) & int(allocs["device_minors"][a1["reservation"][p] - 1])) != 0)
    assert from_rsv >= 3
    ign = np.flatnonzero((pods["reservation_matched"] == abi.RSV_IGNORED) & ds & (c1 >= 0))
    assert len(ign) >= 3 and (a1["reservation"][ign] == 0).all()
    assert ev.check_records(synth.T0) == 0
    for p in np.flatnonzero(a1["reservation"] > 0)[::3]:
        ev.unreserve(pods[p], int(p))
        o.release(pods[p], o.last_allocations()[p], abi.RELEASE_UNRESERVE)
    _state_equal(ev, o, 240)
    (e2,), more, m2, _ = dc.setup(lambda cfg, n: [Oracle(cfg, n)], 240, seed, 200, affinity=affinity)
    more["pod_key"] += 7_000_000_000
    more["uid"] += 7_000_000_000
    _schedule_equal(ev, o, more, m2)
    _state_equal(ev, o, 240)
    assert ev.check_records(synth.T0) == 0


def test_ds_matched_sharded_loopback(gpu):
    """The same path in a node-sharded context (loopback, 3 shards): views, decisions and the staged pick."""
    (ev, o), pods, matches, rs = dc.setup(_both, 240, 7111, 200, affinity=0.3)
    ev.shard_init(0, 3, None)
    _schedule_equal(ev, o, pods, matches)
    _state_equal(ev, o, 240)


def _filter_nominate_case(h, owned):
    """deviceshare/plugin_test.go:2681-2823 through the whole cycle: GPUs 1 and 2 (100 / 8Gi / 100), reservation-1's
    reserve pod holding GPU 1 whole; `owned`: allocated-pod-1 (assigned to it) holds GPUs 1 and 2."""
    gi8 = 8 * GI
    h.upsert_node(0, model.make_node(allocatable={"cpu": "96", "memory": "512Gi"}))
    used = {1: [200, 2 * gi8, 200], 2: [100, gi8, 100]} if owned else {1: [100, gi8, 100]}
    devs = np.zeros(2, abi.DEVICE_DTYPE)
    for q, m in enumerate((1, 2)):
        devs[q]["type"], devs[q]["minor"], devs[q]["health"] = abi.DEV_GPU, m, 1
        devs[q]["has_total"][:] = 1
        devs[q]["total"][:] = [100, gi8, 100]
        if m in used:
            devs[q]["has_used"][:] = 1
            devs[q]["used"][:] = used[m]
    h.set_devices(0, devs)
    t = np.zeros(3, abi.NODE_RESOURCE_DTYPE)
    for e, (rid, av) in enumerate(((abi.XRES_CPU, 96000), (abi.XRES_MEMORY, 512 * GI), (KOORD_GPU, 200))):
        t[e]["id"], t[e]["allocatable"] = rid, av
    h.set_resources(0, t)
    r = np.zeros(1, abi.RESERVATION_DTYPE)
    a = np.zeros(1, abi.RESERVATION_ALLOC_DTYPE)
    r[0]["node"], r[0]["available"], r[0]["holds"] = 0, 1, abi.RSV_HOLDS_DEVICES
    a[0]["device_minors"] = 1 << 1
    a[0]["device"][abi.DEV_GPU, 1] = [100, gi8, 100]
    if owned:
        r[0]["allocated_pods"] = 1
        a[0]["owner_device_minors"] = 1 << 1
        a[0]["owner_device"][abi.DEV_GPU, 1] = [100, gi8, 100]
    h.reservations_load(r, a)


GI = synth.GI
KOORD_GPU = 14


@pytest.mark.parametrize("owned", [False, True], ids=["fits", "owned-out"])
def test_filter_nominate_reservation_case(gpu, owned):
    """The reference's FilterNominateReservation case as a schedule: a koordinator.sh/gpu 100 pod with a reservation
    affinity to reservation-1 takes GPU 1 from it; once allocated-pod-1 holds the GPU the pod fits nowhere."""
    ev, o = _both(synth.config(1), 1)
    for h in (ev, o):
        _filter_nominate_case(h, owned)
    pod = model.make_pod(requests={"koordinator.sh/gpu": "100"})
    pod.reservation_matched = abi.RSV_AFFINITY
    pod.n_xres, pod.xres_id[0], pod.xres_value[0], pod.xres_request_mask = 1, KOORD_GPU, 100, 1 << KOORD_GPU
    pods = np.frombuffer(bytes(pod), dtype=abi.POD_DTYPE).copy()
    c1, a1 = _schedule_equal(ev, o, pods, [[0]])
    if owned:
        assert c1[0] == -1
    else:
        assert c1[0] == 0 and a1["reservation"][0] == 1 and int(a1["device_minors"][0]) == 1 << 1
    _state_equal(ev, o, 1)
