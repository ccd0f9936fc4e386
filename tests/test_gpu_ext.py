"""NodeResourcesFitPlus + ScarceResourceAvoidance fused into the gfx950 pass: the
product through the C ABI against the oracle — the transcribed Score tests, eval matrices and sequential
schedules (placements, framework totals, the nodes' (NonZero)Requested after the Reserves), alone and next to
NUMA policies, cpuset pods, DeviceShare pods and node sharding."""
import numpy as np
import pytest

import cases
from koordinator_amd import Evaluator, abi, synth
from oracle.binding import Oracle
from test_ext_plugins import EXT, ext_cfg, ext_setup
from test_gpu_cpuset import assert_eval_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", EXT, ids=[c["name"] for c in EXT])
def test_golden_ext_through_product(gpu, case):
    ev = Evaluator(ext_cfg(case, len(case["nodes"])))
    pod = ext_setup(ev, case)
    r = ev.eval([pod], cases.NOW)
    assert [int(t) for t in r["total"][0]] == case["want"], case["source"]


def _cluster(n, seed, numa=False, cpus=False, devices=False, batch=64, **ext):
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2 if cpus else 0.0)
    cfg = synth.ext_config(synth.config(n, pod_batch=batch), **ext)
    if devices:
        cfg.weight_numa = 0  # keep Σ weights * 100 <= 510 with five Score plugins
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    tables = synth.make_node_resources(cl, synth.BASE_SEED + seed + 1)
    zones = tabs = devs = None
    if cpus:
        zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 2)
    elif numa:
        zones = synth.make_numa(cl, synth.BASE_SEED + seed + 2, zone_counts=(2, 4))
    if devices:
        devs = synth.make_devices(n, synth.BASE_SEED + seed + 3)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_node_resources(h, tables)
        if zones is not None:
            synth.load_numa(h, zones)
        if tabs is not None:
            synth.load_cpus(h, tabs)
        if devs is not None:
            synth.load_devices(h, devs)
    return ev, o, tables


def _expected_tables(tables, pods, chosen):
    """The nodes' tables after the Reserves: NodeInfo (NonZero)Requested += each placed pod's requests."""
    want = [{int(r["id"]): [int(r["allocatable"]), int(r["requested"])] for r in t} for t in tables]
    for p, node in enumerate(chosen):
        if node < 0:
            continue
        for e in range(int(pods["n_xres"][p])):
            rid, v = int(pods["xres_id"][p, e]), int(pods["xres_value"][p, e])
            want[node].setdefault(rid, [0, 0])[1] += v
    return want


def _schedule_equal(ev, o, pods, tables=None):
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    if tables is not None:
        want = _expected_tables(tables, pods, c1)
        for i in range(len(tables)):
            got = {int(r["id"]): [int(r["allocatable"]), int(r["requested"])] for r in ev.get_resources(i)}
            assert {k: v for k, v in got.items() if v != [0, 0]} == {k: v for k, v in want[i].items() if v != [0, 0]}, i
    return c1


def test_ext_eval_matrix_parity(gpu):
    ev, o, _ = _cluster(700, 301)
    pods = synth.add_pod_xres(synth.make_pods(80, synth.BASE_SEED + 302), synth.BASE_SEED + 303)
    assert_eval_equal(ev.eval(pods, synth.T0), o.eval(pods, synth.T0))


@pytest.mark.parametrize("ext", [dict(), dict(w_sra=0), dict(w_fitplus=0), dict(w_fitplus=2, w_sra=0)],
                         ids=["both", "fitplus", "sra", "fitplus-w2"])
def test_ext_schedule_parity(gpu, ext):
    ev, o, tables = _cluster(600, 311, **ext)
    pods = synth.add_pod_xres(synth.make_pods(700, synth.BASE_SEED + 312), synth.BASE_SEED + 313)
    _schedule_equal(ev, o, pods, tables)
    more = synth.add_pod_xres(synth.make_pods(40, synth.BASE_SEED + 314), synth.BASE_SEED + 315)
    assert_eval_equal(ev.eval(more, synth.T0), o.eval(more, synth.T0))


def test_ext_schedule_batch_invariance(gpu):
    pods = synth.add_pod_xres(synth.make_pods(300, synth.BASE_SEED + 322), synth.BASE_SEED + 323)
    out = []
    for b in (1, 7, 64):
        ev, _, _ = _cluster(400, 321, batch=b)
        out.append(ev.schedule(pods, synth.T0))
    for c, s in out[1:]:
        assert np.array_equal(c, out[0][0]) and np.array_equal(s, out[0][1])


def test_ext_with_numa_policies(gpu):
    ev, o, tables = _cluster(400, 331, numa=True)
    pods = synth.add_pod_xres(synth.make_numa_pods(300, synth.BASE_SEED + 332), synth.BASE_SEED + 333)
    assert_eval_equal(ev.eval(pods[:40], synth.T0), o.eval(pods[:40], synth.T0))
    _schedule_equal(ev, o, pods, tables)


def test_ext_with_cpuset_pods(gpu):
    ev, o, tables = _cluster(240, 341, cpus=True)
    pods = synth.add_pod_xres(synth.make_numa_cpuset_pods(160, synth.BASE_SEED + 342), synth.BASE_SEED + 343)
    _schedule_equal(ev, o, pods, tables)


def test_ext_with_deviceshare_pods(gpu):
    ev, o, tables = _cluster(300, 351, devices=True)
    pods = synth.add_pod_xres(synth.make_ds_pods(200, synth.BASE_SEED + 352), synth.BASE_SEED + 353)
    _schedule_equal(ev, o, pods, tables)


def test_ext_sharded_loopback(gpu):
    ev, o, tables = _cluster(500, 361)
    ev.shard_init(0, 3, None)
    pods = synth.add_pod_xres(synth.make_pods(300, synth.BASE_SEED + 362), synth.BASE_SEED + 363)
    _schedule_equal(ev, o, pods, tables)
