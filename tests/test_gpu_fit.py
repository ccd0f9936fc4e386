"""NodeResourcesFit on the GPU: its Filter ahead of the koordinator Filters and its LeastAllocated /
MostAllocated Score beside LoadAware, NodeNUMAResource, DeviceShare, NodeResourcesFitPlus and ScarceResourceAvoidance
(six Score plugins at weight 1 -- the widened 10-bit score key), bit-exact with the oracle on eval matrices (status,
reason, totals) and schedules (placements, totals, NodeInfo tables, pod rooms) on every evaluation path: the record-
based plain batches and the speculative replay (pipelined and serial), the row path of NUMA / cpuset / DeviceShare
batches, batch sizes 1 / 7 / 64.  The oracle's NodeResourcesFit is parity unpinned (upstream k8s, not in tree)."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, synth
from oracle.binding import Oracle
from test_gpu_cpuset import assert_eval_equal
from test_gpu_ext import _expected_tables

pytestmark = pytest.mark.gpu


def _fit_cluster(n, seed, batch=64, cpus=False, devices=False, strategy=abi.STRATEGY_LEAST_ALLOCATED, tight=True):
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2 if cpus else 0.0)
    if tight:  # some nodes one pod short of AllowedPodNumber: "Too many pods" after one placement
        cl.nodes["allowed_pods"][::9] = cl.nodes["pod_count"][::9] + 1
        cl.nodes["allowed_pods"][::23] = cl.nodes["pod_count"][::23]
    cfg = synth.fit_config(synth.ext_config(synth.config(n, pod_batch=batch)), strategy=strategy)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    tables = synth.make_node_resources(cl, synth.BASE_SEED + seed + 1)
    zones = tabs = devs = None
    if cpus:
        zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 2)
    if devices:
        devs = synth.make_devices(n, synth.BASE_SEED + seed + 3)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_node_resources(h, tables)
        if zones is not None:
            synth.load_numa(h, zones)
            synth.load_cpus(h, tabs)
        if devs is not None:
            synth.load_devices(h, devs)
    return ev, o, tables, cl


def _pods(n, seed, key_base=1_000_000_000):
    return synth.add_fit_defaults(synth.add_pod_xres(synth.make_pods(n, synth.BASE_SEED + seed, key_base=key_base),
                                                     synth.BASE_SEED + seed + 1))


def _schedule_equal(ev, o, pods, tables, n):
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    want = _expected_tables(tables, pods, c1)
    for i in range(0, n, 7):
        got = {int(r["id"]): [int(r["allocatable"]), int(r["requested"])] for r in ev.get_resources(i)}
        assert {k: v for k, v in got.items() if v != [0, 0]} == {k: v for k, v in want[i].items() if v != [0, 0]}, i
        n1, n0 = ev.node_state(i)[0], o.node_state(i)[0]
        assert n1.pod_count == n0.pod_count and list(n1.requested) == list(n0.requested), i
    return c1


def test_fit_eval_matrix_parity(gpu):
    ev, o, _, _ = _fit_cluster(900, 1401)
    pods = _pods(96, 1402)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    assert_eval_equal(a, b)
    for r in (abi.REASON_FIT_TOO_MANY_PODS, abi.REASON_FIT_INSUFFICIENT_SCALAR):
        assert (a["reason"] == r).any(), r  # the Filter's reasons occur


@pytest.mark.parametrize("batch,pipeline", [(64, True), (64, False), (7, True), (1, False)],
                         ids=["b64-pipelined", "b64-serial", "b7", "b1"])
def test_fit_schedule_parity(gpu, batch, pipeline):
    """Plain batches: k_eval_plain / the speculative replay / k_fixup with the Fit Filter and Score in fast_total."""
    ev, o, tables, cl = _fit_cluster(1200, 1411, batch=batch)
    ev.set_pipeline(pipeline)
    pods = _pods(1500, 1412)
    c1 = _schedule_equal(ev, o, pods, tables, 1200)
    full = np.flatnonzero(cl.nodes["allowed_pods"] <= cl.nodes["pod_count"] + 1)
    assert (np.bincount(c1[c1 >= 0], minlength=1200)[full] <= 1).all()  # AllowedPodNumber holds
    assert ev.check_records(synth.T0) == 0
    # release a fifth of the placements (pod room and requests back), then a second queue
    a1, a0 = ev.last_allocations(), o.last_allocations()
    for p in np.flatnonzero(c1 >= 0)[::5]:
        ev.release(pods[p], a1[p], abi.RELEASE_DELETE)
        o.release(pods[p], a0[p], abi.RELEASE_DELETE)
    more = _pods(600, 1414, key_base=7_000_000_000)
    c2, s2 = ev.schedule(more, synth.T0)
    c0, s0 = o.schedule(more, synth.T0)
    assert np.array_equal(c2, c0) and np.array_equal(s2, s0)
    assert ev.check_records(synth.T0) == 0


def test_fit_most_allocated_and_cpusets(gpu):
    """MostAllocated, on a cluster with CPU tables and NUMA zones (cpuset singletons: eval_pair and
    k_cpuset_reserve carry the Fit Filter / Score / Reserve)."""
    ev, o, tables, _ = _fit_cluster(500, 1421, cpus=True, strategy=abi.STRATEGY_MOST_ALLOCATED)
    pods = _pods(400, 1422)
    assert_eval_equal(ev.eval(pods[:40], synth.T0), o.eval(pods[:40], synth.T0))
    _schedule_equal(ev, o, pods, tables, 500)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    assert ev.check_records(synth.T0) == 0


def test_fit_with_deviceshare(gpu):
    """DeviceShare batches (speculative DeviceShare replay on the rows) with the Fit Filter over the device scalar."""
    ev, o, tables, _ = _fit_cluster(400, 1431, devices=True)
    pods = synth.add_fit_defaults(synth.add_pod_xres(synth.make_ds_pods(300, synth.BASE_SEED + 1432),
                                                     synth.BASE_SEED + 1433))
    assert_eval_equal(ev.eval(pods[:32], synth.T0), o.eval(pods[:32], synth.T0))
    _schedule_equal(ev, o, pods, tables, 400)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)
    assert ev.check_records(synth.T0) == 0
