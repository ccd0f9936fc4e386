"""DeviceShare as a NUMA hint provider on the GPU: device pods on NUMA-policy nodes (or
with a pod NUMA policy) run the topology manager's Admit over NodeNUMAResource's lists plus DeviceShare's
(GetPodTopologyHints, topology_hint.go:38-120), DeviceShare Allocate on the merged affinity
(topology_hint.go:122-212), Filter skipped / Score and Reserve on the stored affinity — bit-exact with the
oracle, whose restatement the transcribed Go vectors pin (tests/golden/ds_numa.json,
test_oracle_golden.py::test_ds_numa_hints)."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, synth
from oracle.binding import Oracle
from test_gpu_cpuset import assert_eval_equal

pytestmark = pytest.mark.gpu


def _both(n, seed, disable=False, zone_counts=(2, 4, 8), cpus=False):
    cl = synth.make_cluster(n, synth.BASE_SEED + seed, amplified_fraction=0.2 if cpus else 0.0)
    if cpus:
        zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1, zone_counts=zone_counts)
    else:
        zones, tabs = synth.make_numa(cl, synth.BASE_SEED + seed + 1, zone_counts=zone_counts), None
    devs = synth.make_devices(n, synth.BASE_SEED + seed + 2)
    synth.add_device_numa(devs, zones, synth.BASE_SEED + seed + 3)
    cfg = synth.config(n)
    cfg.deviceshare.disable_numa_alignment = int(disable)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        if tabs:
            synth.load_cpus(h, tabs)
        synth.load_devices(h, devs)
    return ev, o


def _cpuset_ds_pods(n, seed):
    """Binding pods (LSE/LSR koord-prod, NUMA specs on a fifth) of which half request devices."""
    pods = synth.make_numa_cpuset_pods(n, synth.BASE_SEED + seed)
    dsp = synth.make_ds_pods(n, synth.BASE_SEED + seed + 1)
    pods["device_requests"] = dsp["device_requests"]
    pods["has_other_requests"] = dsp["has_other_requests"]
    return pods


def _schedule_equal(ev, o, pods):
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations), \
        np.argwhere(ev.last_device_allocations != o.last_device_allocations)[:5].ravel().tolist()
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations), \
        np.argwhere(np.any(ev.last_numa_allocations != o.last_numa_allocations, axis=1))[:5].ravel().tolist()
    return c1


VARIANTS = {
    "zones-2-4-8": {},
    "zones-2": {"zone_counts": (2,)},
    "alignment-disabled": {"disable": True},
}


@pytest.mark.parametrize("name", list(VARIANTS))
def test_ds_numa_eval_parity(gpu, name):
    ev, o = _both(200, 701, **VARIANTS[name])
    pods = synth.make_ds_numa_pods(160, synth.BASE_SEED + 702)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    assert_eval_equal(a, b)
    reasons = set(np.unique(a["reason"][a["status"] != 0]).tolist())
    if not VARIANTS[name].get("disable"):
        assert abi.REASON_DS_INSUFFICIENT_NUMA_SCOPED in reasons


@pytest.mark.parametrize("name", list(VARIANTS))
def test_ds_numa_schedule_parity(gpu, name):
    ev, o = _both(96, 711, **VARIANTS[name])
    pods = synth.make_ds_numa_pods(240, synth.BASE_SEED + 712)
    c = _schedule_equal(ev, o, pods)
    dev = pods["device_requests"].any(axis=1)
    assert ((c >= 0) & dev).sum() > 20 and np.any(ev.last_numa_allocations != 0)
    more = synth.make_ds_numa_pods(40, synth.BASE_SEED + 713, key_base=9_700_000_000)
    assert_eval_equal(ev.eval(more, synth.T0), o.eval(more, synth.T0))
    assert ev.check_records(synth.T0) == 0


def test_ds_numa_cpuset_pods(gpu):
    """Binding pods with devices: the cpuset take joins every NUMA allocation check and Reserve runs on
    k_cpuset_reserve, DeviceShare's Reserve on the stored affinity."""
    ev, o = _both(120, 721, cpus=True, zone_counts=(2, 4))
    pods = _cpuset_ds_pods(200, 722)
    assert_eval_equal(ev.eval(pods[:80], synth.T0), o.eval(pods[:80], synth.T0))
    c = _schedule_equal(ev, o, pods)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    assert (c >= 0).sum() > 60
