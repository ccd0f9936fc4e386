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
