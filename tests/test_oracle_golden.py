"""Pin the oracle: every known-answer vector transcribed from the reference's Go tests
(tests/golden/) must come out of the CPU restatement unchanged."""
import pytest

import cases
from oracle.binding import Oracle

LA_FILTER = cases.load("loadaware_filter.json")
LA_SCORE = cases.load("loadaware_score.json")
EST = cases.load("estimator.json")
NUMA = cases.load("numa.json")


@pytest.mark.parametrize("case", LA_FILTER, ids=[c["name"] for c in LA_FILTER])
def test_loadaware_filter(case):
    o = Oracle(cases.make_cfg(case), 1)
    pod = cases.setup_loadaware(o, case)
    code, reason = o.la_filter(pod, 0, cases.NOW)
    assert (code, reason) == (case["want"]["code"], case["want"]["reason"]), case["source"]


@pytest.mark.parametrize("case", LA_SCORE, ids=[c["name"] for c in LA_SCORE])
def test_loadaware_score(case):
    o = Oracle(cases.make_cfg(case), 1)
    pod = cases.setup_loadaware(o, case)
    assert o.la_score(pod, 0, cases.NOW) == case["want"]["score"], case["source"]


@pytest.mark.parametrize("case", EST, ids=[c["name"] for c in EST])
def test_estimator(case):
    o = Oracle(cases.make_cfg(case), 1)
    est = o.estimate_pod(cases.make_pod(case["pod"]))
    assert list(est) == [case["want"]["cpu"], case["want"]["memory"]], case["source"]


@pytest.mark.parametrize("case", NUMA, ids=[c["name"] for c in NUMA])
def test_numa(case):
    nodes = cases.make_numa_nodes(case)
    o = Oracle(cases.make_cfg(case, len(nodes)), len(nodes))
    for i, n in enumerate(nodes):
        o.upsert_node(i, n)
    pod = cases.make_pod(case["pod"])
    if case["op"] == "score":
        got = [o.numa_score(pod, i) for i in range(len(nodes))]
        assert got == case["want"]["scores"], case["source"]
    else:
        code, reason = o.numa_filter(pod, 0)
        assert (code, reason) == (case["want"]["code"], case["want"]["reason"]), case["source"]
