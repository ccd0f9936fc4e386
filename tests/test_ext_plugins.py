"""NodeResourcesFitPlus / ScarceResourceAvoidance: the oracle pinned by the reference's
Score tests (tests/golden/ext_plugins.json), the pod-side PreScore helper, and the boundary's validation.
CPU only; the GPU parity of the fused path is in test_gpu_ext.py."""
import ctypes as C

import numpy as np
import pytest

import cases
from koordinator_amd import Evaluator, abi, model, synth
from oracle.binding import Oracle

EXT = cases.load("ext_plugins.json")


def ext_cfg(case, n_nodes):
    cfg = synth.config(n_nodes)
    cfg.weight_loadaware = cfg.weight_numa = cfg.weight_deviceshare = 0
    x = cfg.ext
    if case["plugin"] == "fitplus":
        x.weight_fitplus = 1
        x.n_fitplus = len(case["args"])
        for q, (name, typ, w) in enumerate(case["args"]):
            x.fitplus[q].id, x.fitplus[q].type, x.fitplus[q].weight = model.xres_id(name), typ, w
    else:
        x.weight_sra = 1
        x.sra_resources = sum(1 << model.xres_id(n) for n in case["args"])
    return cfg


def ext_setup(handle, case):
    for i, nd in enumerate(case["nodes"]):
        handle.upsert_node(i, model.make_node(allocatable={k: v for k, v in nd["allocatable"].items()
                                                            if k in ("cpu", "memory")}))
        handle.set_resources(i, model.make_node_resources(nd["allocatable"], nd["requested"]))
    return model.make_pod(containers=case["pod"]["containers"])


@pytest.mark.parametrize("case", EXT, ids=[c["name"] for c in EXT])
def test_oracle_ext_golden(case):
    o = Oracle(ext_cfg(case, len(case["nodes"])), len(case["nodes"]))
    pod = ext_setup(o, case)
    score = o.fitplus_score if case["plugin"] == "fitplus" else o.sra_score
    got = [score(pod, i) for i in range(len(case["nodes"]))]
    assert got == case["want"], case["source"]
    if case.get("order") == "gt":
        assert got[0] > got[1]
    if case.get("order") == "lt":
        assert got[0] < got[1]


@pytest.mark.parametrize("case", EXT, ids=[c["name"] for c in EXT])
def test_oracle_ext_total(case):
    """The framework total of the oracle's eval is the plugin score times its weight."""
    o = Oracle(ext_cfg(case, len(case["nodes"])), len(case["nodes"]))
    pod = ext_setup(o, case)
    r = o.eval([pod], cases.NOW)
    assert [int(t) for t in r["total"][0]] == case["want"]


def test_fitplus_pod_request_defaults():
    """calculatePodResourceRequest: nonzero defaults per container, init containers' max."""
    cs = [{"requests": {"cpu": "500m"}}, {"requests": {"memory": "1Gi"}}]
    assert model.fitplus_pod_request("cpu", cs) == 500 + 100
    assert model.fitplus_pod_request("memory", cs) == 200 * 2**20 + 2**30
    assert model.fitplus_pod_request("cpu", cs, [{"requests": {"cpu": "2"}}]) == 2000
    assert model.fitplus_pod_request("nvidia.com/gpu", cs) == 0
    p = model.make_pod(containers=cs)
    assert p.xres_request_mask == (1 << abi.XRES_CPU) | (1 << abi.XRES_MEMORY)
    assert sorted(p.xres_value[:p.n_xres]) == sorted([600, 200 * 2**20 + 2**30])


def test_ext_config_validation(lib):
    cfg = synth.ext_config(synth.config(4))
    ev = Evaluator(cfg)
    ev.close()
    bad = synth.ext_config(synth.config(4), w_fitplus=8)  # (1 + 1 + 1 + 8 + 1) * 100 > 1022 (10-bit key score)
    with pytest.raises(Exception, match="weights"):
        Evaluator(bad)
    # the shipped profile's six Score plugins at weight 1 (600) fit the widened key
    Evaluator(synth.fit_config(synth.ext_config(synth.config(4)))).close()
    bad = synth.ext_config(synth.config(4))
    bad.ext.fitplus[1].id = bad.ext.fitplus[0].id
    with pytest.raises(Exception, match="twice"):
        Evaluator(bad)
    bad = synth.ext_config(synth.config(4))
    bad.ext.n_fitplus = 5
    with pytest.raises(Exception, match="at most 4"):
        Evaluator(bad)


def test_node_resources_roundtrip_and_validation(lib):
    ev = Evaluator(synth.ext_config(synth.config(4)))
    t = model.make_node_resources({"cpu": "8", "nvidia.com/gpu": "4"}, {"cpu": "1"})
    ev.set_resources(2, t)
    got = ev.get_resources(2)
    assert got.tolist() == t.tolist()
    dup = np.concatenate([t, t[:1]])
    with pytest.raises(Exception, match="twice"):
        ev.set_resources(2, dup)
    neg = t.copy()
    neg[0]["requested"] = -1
    with pytest.raises(Exception, match="negative"):
        ev.set_resources(2, neg)
    with pytest.raises(Exception):
        ev.set_resources(9, t)  # beyond node_capacity


def test_pod_xres_validation(lib):
    ev = Evaluator(synth.ext_config(synth.config(4)))
    p = model.make_pod(requests={"cpu": "1"})
    p.n_xres = 9
    with pytest.raises(Exception, match="n_xres"):
        ev.schedule(np.frombuffer(bytes(p), dtype=abi.POD_DTYPE).copy(), cases.NOW)
