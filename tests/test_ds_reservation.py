"""DeviceShare allocate-from-reservation on the oracle, pinned by the reference's own tests
(tests/golden/ds_reservation.json, tests/golden/make_ds_rsv_fixtures.py): Test_tryAllocateFromReservation
(deviceshare/reservation_test.go:225-888), TestScoreReservation (scoring_test.go:670-1240) and
Test_Plugin_FilterNominateReservation (plugin_test.go:2681-2823), each with its restore state given directly.  The
GPU path is compared with the oracle on clusters of device-holding reservations in tests/test_gpu_ds_reservation.py."""
import pytest

import cases
from koordinator_amd import abi, model
from oracle.binding import Oracle, normalize_scores

DS_RSV = cases.load("ds_reservation.json")
TYPES = {"gpu": abi.DEV_GPU, "rdma": abi.DEV_RDMA}
NAMES = {abi.DEV_GPU: ["koordinator.sh/gpu-core", "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio"],
         abi.DEV_RDMA: ["koordinator.sh/rdma"]}
POD_KEYS = {"gpu_core": "koordinator.sh/gpu-core", "gpu_memory": "koordinator.sh/gpu-memory",
            "gpu_memory_ratio": "koordinator.sh/gpu-memory-ratio", "rdma": "koordinator.sh/rdma",
            "koord_gpu": "koordinator.sh/gpu"}


def dres(d):
    """fixture deviceResources -> {type: {minor: {key: value}}}"""
    out = {}
    for tn, minors in (d or {}).items():
        t = TYPES[tn]
        out[t] = {}
        for m, v in minors.items():
            vals = v if isinstance(v, list) else [v]
            out[t][int(m)] = {k: x for k, x in enumerate(vals) if x is not None}
    return out


def devices(case):
    used = dres(case["used"])
    devs = []
    for tn, minors in case["devices"].items():
        t = TYPES[tn]
        for m, v in minors.items():
            vals = v if isinstance(v, list) else [v]
            u = used.get(t, {}).get(int(m), {})
            devs.append({"type": tn, "minor": int(m), "total": {NAMES[t][k]: x for k, x in enumerate(vals)},
                         "used": {NAMES[t][k]: x for k, x in u.items()}})
    return model.make_devices(devs)


def setup(case):
    cfg = abi.default_config(1)
    if case.get("strategy") == "most":
        cfg.deviceshare.strategy = abi.STRATEGY_MOST_ALLOCATED
    o = Oracle(cfg, 1)
    o.upsert_node(0, model.make_node(allocatable={"cpu": "96", "memory": "512Gi"}))
    o.set_devices(0, devices(case))
    pod = model.make_pod(requests={POD_KEYS[k]: str(v) for k, v in case["pod"].items()})
    matched = [(m["policy"], dres(m["allocatable"]), dres(m["allocated"]), dres(m["remained"]))
               for m in case["matched"]]
    return o, pod, matched


def test_fixture_counts():
    assert len(DS_RSV["try"]) == 14 and len(DS_RSV["score"]) == 11


@pytest.mark.parametrize("case", DS_RSV["try"], ids=lambda c: c["name"])
def test_try_allocate_from_reservation(lib, case):
    o, pod, matched = setup(case)
    code, reason, out = o.ds_rsv_direct(pod, 0, matched, dres(case["basic"]), dres(case["matched_allocatable"]),
                                        dres(case["matched_allocated"]), required=case["required"],
                                        ignored=case["ignored"])
    assert code == case["want_code"] if case["want_code"] < 2 else code == abi.CODE_UNSCHEDULABLE, \
        (case["source"], code, reason)
    if case["want_code"] == 0:
        got = {tn: [m for m in range(16) if (out[t] >> m) & 1] for tn, t in TYPES.items() if out[t]}
        assert got == case["want_minors"], case["source"]
    elif case["want_code"] == 2:
        want = abi.REASON_RSV_INSUFFICIENT_DEVICES if case["want_reason"] == "rsv" else abi.REASON_DS_INSUFFICIENT_GPU
        assert reason == want, case["source"]
    else:
        assert out == [0, 0, 0]


@pytest.mark.parametrize("case", DS_RSV["score"], ids=lambda c: c["name"])
def test_score_reservation(lib, case):
    o, pod, matched = setup(case)
    s = o.ds_rsv_direct(pod, 0, matched, dres(case["basic"]), dres(case["matched_allocatable"]),
                        dres(case["matched_allocated"]), mode=1)
    assert s == case["want_score"], case["source"]
    if case["want_normalize"] is not None:  # DefaultReservationNormalizeScore over the one-entry list
        assert normalize_scores([s]) == [case["want_normalize"]], case["source"]


def test_filter_nominate_reservation_full_cycle(lib):
    """Test_Plugin_FilterNominateReservation (plugin_test.go:2681-2823) through the oracle's whole cycle (the GPU
    twin: tests/test_gpu_ds_reservation.py): the affinity pod takes GPU 1 out of reservation-1, and fits nowhere
    once allocated-pod-1 holds GPUs 1 and 2."""
    import test_gpu_ds_reservation as g
    for owned in (False, True):
        o = Oracle(abi.default_config(1), 1)
        g._filter_nominate_case(o, owned)
        pod = model.make_pod(requests={"koordinator.sh/gpu": "100"})
        pod.reservation_matched = abi.RSV_AFFINITY
        pod.n_xres, pod.xres_id[0], pod.xres_value[0], pod.xres_request_mask = 1, g.KOORD_GPU, 100, 1 << g.KOORD_GPU
        c, s = o.schedule([pod], cases.NOW, matches=[[0]])
        a = o.last_allocations()
        if owned:
            assert c[0] == -1
        else:
            assert c[0] == 0 and a["reservation"][0] == 1 and int(a["device_minors"][0]) == 1 << 1
            assert int(o.reservation_allocs_get()["owner_device"][0, abi.DEV_GPU, 1, 0]) == 100


def test_ds_matched_checks_agree(lib):
    """The refusals of the DeviceShare allocate-from-reservation path agree between the product's argument checks
    and the oracle: a hinted DeviceShare pod (or one with a NUMA policy) matching a device-holding reservation is
    refused; a plain DeviceShare pod passes the checks (the product then needs its device)."""
    import ds_rsv_cases as dc
    from koordinator_amd import Evaluator, KoordEvalError
    (ev, o), pods, matches, rs = dc.setup(lambda cfg, n: [Evaluator(cfg), Oracle(cfg, n)], 60, 7201, 40, match=1.0,
                                          affinity=0.0, ignored=0.0)
    dsp = [p for p in range(len(pods)) if pods["device_requests"][p].any() and matches[p]
           and any(rs["available"][r] for r in matches[p])]
    p = dsp[0]
    one = pods[p:p + 1].copy()
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(one, cases.NOW, matches=[matches[p]])
    assert e.value.code == abi.ERR_NO_DEVICE
    one["numa_topology_policy"] = abi.NUMA_POLICY_BEST_EFFORT
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(one, cases.NOW, matches=[matches[p]])
    assert e.value.code == abi.ERR_UNSUPPORTED
    with pytest.raises(RuntimeError, match=f"rc={abi.ERR_UNSUPPORTED}"):
        o.schedule(one, cases.NOW, matches=[matches[p]])
    one["numa_topology_policy"] = 0
    one["reservation_matched"] = abi.RSV_IGNORED
    one["numa_topology_policy"] = abi.NUMA_POLICY_RESTRICTED
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(one, cases.NOW)
    assert e.value.code == abi.ERR_UNSUPPORTED
    with pytest.raises(RuntimeError, match=f"rc={abi.ERR_UNSUPPORTED}"):
        o.schedule(one, cases.NOW, matches=[[]])
    ev.close()
