"""Reservations (first part): the reservation cache's NodeInfo restore every pod that
matches no reservation sees (restoreUnmatchedReservations, transformer.go:447-473), in the product's host state
and in the oracle, pinned by TestRestoreReservation (tests/golden/reservations.json); pods that match a
reservation are refused at the boundary."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, synth
from koordinator_amd.evaluator import KoordEvalError
from oracle.binding import Oracle

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "reservations.json")))["cases"]


def reservation(node, d):
    r = abi.Reservation()
    r.node = node
    r.available = int(d["available"])
    r.allocate_once = int(d["allocate_once"])
    r.allocated_pods = d["allocated_pods"]
    for k in range(abi.NRES):
        r.allocatable[k] = d["allocatable"][k]
        r.allocated[k] = d["allocated"][k]
    return r


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_restore_golden(case):
    cfg = synth.config(4)
    ev, o = Evaluator(cfg), Oracle(cfg, 4)
    node = abi.Node()
    for k in range(abi.NRES):
        node.allocatable[k] = case["node"]["allocatable"][k]
        node.raw_allocatable[k] = abi.ABSENT
        node.requested[k] = case["node"]["requested"][k]
        node.custom_usage_thresholds[k] = node.custom_prod_usage_thresholds[k] = abi.ABSENT
        node.custom_agg_thresholds[k] = abi.ABSENT
    node.cpu_amplification_ratio = -1.0
    node.nrt_cpu_amplification_ratio = -2.0
    res = np.zeros(2, abi.NODE_RESOURCE_DTYPE)
    res["id"] = [abi.RES_CPU, abi.RES_MEMORY]
    res["allocatable"] = case["node"]["allocatable"]
    res["requested"] = case["node"]["requested"]  # NonZeroRequested: every pod requests both
    rs = [reservation(2, d) for d in case["reservations"]]
    for h in (ev, o):
        h.upsert_node(2, node)
        h.set_resources(2, res)
        h.reservations_load(rs)
        req, nz = h.node_info_requested(2)
        assert req == case["want_requested"]
        assert nz == case["want_requested"]
    ev.close()


def test_restore_rules_product_equals_oracle():
    """AllocateOnce, unavailable, zero-allocated and over-allocated reservations, zero-request keys (the 100m /
    200Mi NonZero defaults), several reservations per node: product host state = oracle."""
    rng = np.random.default_rng(5)
    n = 16
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    cl = synth.make_cluster(n, synth.BASE_SEED + 901)
    res = np.zeros((n, 2), abi.NODE_RESOURCE_DTYPE)
    for h in (ev, o):
        synth.load_into(h, cl)
    for i in range(n):
        res[i]["id"] = [abi.RES_CPU, abi.RES_MEMORY]
        res[i]["allocatable"] = cl.nodes["allocatable"][i, :2]
        res[i]["requested"] = cl.nodes["requested"][i, :2]
        for h in (ev, o):
            h.set_resources(i, res[i])
    rs = []
    for _ in range(40):
        r = abi.Reservation()
        r.node = int(rng.integers(0, n))
        r.available = int(rng.random() < 0.9)
        r.allocate_once = int(rng.random() < 0.3)
        r.allocated_pods = int(rng.choice([0, 0, 1, 2, 3]))
        for k in range(abi.NRES):
            a = int(rng.choice([0, 1000, 4000, 8000])) * (1 if k == 0 else 2**20)
            r.allocatable[k] = a
            r.allocated[k] = int(rng.choice([0, a // 2, a, a + 1000]))
        rs.append(r)
    for h in (ev, o):
        h.reservations_load(rs)
    for i in range(n):
        assert ev.node_info_requested(i) == o.node_info_requested(i), i
    ev.close()


def test_matched_pod_checks():
    """KE_RSV_MATCHED needs ke_pod_reservations lists; affinity / ignored pods and ke_eval of a matched pod are
    refused; lists for other pods or of another length are invalid (host checks, no device call)."""
    cfg = synth.config(4)
    ev = Evaluator(cfg)
    synth.load_into(ev, synth.make_cluster(4, synth.BASE_SEED + 903))
    ev.reservations_load([abi.Reservation(node=0, available=1)])
    pods = synth.make_pods(2, synth.BASE_SEED + 902)
    pods["reservation_matched"][1] = abi.RSV_MATCHED
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0)
    assert e.value.code == abi.ERR_INVALID
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0, matches=[[0], []])  # listed for a pod that is not KE_RSV_MATCHED
    assert e.value.code == abi.ERR_INVALID
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0, matches=[[]])  # another queue length
    assert e.value.code == abi.ERR_INVALID
    with pytest.raises(KoordEvalError) as e:
        ev.pod_reservations([[], [1]])  # no such reservation
    assert e.value.code == abi.ERR_NOT_FOUND
    pods["reservation_matched"][1] = abi.RSV_IGNORED
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0)
    assert e.value.code == abi.ERR_UNSUPPORTED
    pods["reservation_matched"][1] = abi.RSV_AFFINITY
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0)  # an affinity pod needs its (possibly empty) list staged
    assert e.value.code == abi.ERR_INVALID
    pods["reservation_matched"][1] = abi.RSV_MATCHED
    pods["requests"][1][abi.RES_BATCH_CPU] = 1000  # a scalar request
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0, matches=[[], [0]])
    assert e.value.code == abi.ERR_UNSUPPORTED
    with pytest.raises(KoordEvalError) as e:
        ev.eval(pods, synth.T0)
    assert e.value.code == abi.ERR_UNSUPPORTED
    ev.close()


SCORE_CASES = json.load(open(os.path.join(HERE, "golden", "reservation_scores.json")))["cases"]


@pytest.mark.parametrize("case", SCORE_CASES, ids=[c["name"] for c in SCORE_CASES])
def test_reservation_score_golden(case):
    """The oracle's Reservation PreScore / NominateReservation / Score against TestScore, TestScoreWithOrder and
    TestNominateReservation."""
    n = len(case["nodes"])
    cfg = synth.config(n)
    o = Oracle(cfg, n)
    for i, nd in enumerate(case["nodes"]):
        node = abi.Node()
        for k in range(abi.NRES):
            node.allocatable[k] = nd["allocatable"][k]
            node.raw_allocatable[k] = abi.ABSENT
            node.requested[k] = nd["requested"][k]
            node.custom_usage_thresholds[k] = node.custom_prod_usage_thresholds[k] = abi.ABSENT
            node.custom_agg_thresholds[k] = abi.ABSENT
        node.cpu_amplification_ratio = -1.0
        node.nrt_cpu_amplification_ratio = -2.0
        o.upsert_node(i, node)
    rs = []
    for d in case["reservations"]:
        r = abi.Reservation(node=d["node"], available=1, order=d["order"])
        for k in range(abi.NRES):
            r.allocatable[k], r.allocated[k] = d["allocatable"][k], d["allocated"][k]
        rs.append(r)
    o.reservations_load(rs)
    pod = synth.make_pods(1, synth.BASE_SEED + 904)
    pod["requests"][0][:] = 0
    pod["requests"][0][:2] = case["pod"]
    pod["reservation_matched"][0] = abi.RSV_MATCHED
    pref, raw, nom = o.reservation_prescore(pod[0], list(range(len(rs))))
    if case["want_score"] is not None:
        assert list(raw) == case["want_score"]
    if case["want_nominated"] is not None:
        assert list(nom) == case["want_nominated"]


FILTER_CASES = json.load(open(os.path.join(HERE, "golden", "reservation_filters.json")))["cases"]


@pytest.mark.parametrize("case", FILTER_CASES, ids=[c["name"] for c in FILTER_CASES])
def test_reservation_filter_golden(case):
    """The oracle's Reservation Filter with a reservation affinity (fitsNode / fitsReservation) against
    Test_filterWithReservations."""
    cfg = synth.config(1)
    o = Oracle(cfg, 1)
    node = abi.Node()
    for k in range(abi.NRES):
        node.allocatable[k] = case["node"]["allocatable"][k]
        node.raw_allocatable[k] = abi.ABSENT
        node.requested[k] = case["node"]["requested"][k]
        node.custom_usage_thresholds[k] = node.custom_prod_usage_thresholds[k] = abi.ABSENT
        node.custom_agg_thresholds[k] = abi.ABSENT
    node.cpu_amplification_ratio = -1.0
    node.nrt_cpu_amplification_ratio = -2.0
    o.upsert_node(0, node)
    d = case["reservation"]
    r = abi.Reservation(node=0, available=1, allocate_policy=d["allocate_policy"])
    for k in range(abi.NRES):
        r.allocatable[k], r.allocated[k] = d["allocatable"][k], d["allocated"][k]
    o.reservations_load([r])
    pod = synth.make_pods(1, synth.BASE_SEED + 905)
    pod["requests"][0][:] = 0
    pod["requests"][0][:2] = case["pod"]
    pod["reservation_matched"][0] = abi.RSV_AFFINITY
    assert o.reservation_filter(pod[0], [0], 0) == case["want"]
