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


def test_ds_numa_merge_beyond_walk(gpu):
    """A BestEffort merge over more than MERGE_BUDGET (2^20) hint permutations runs merge_exact (ke_merge.h)
    instead of the permutation walk: 6-zone BestEffort nodes with one GPU and one RDMA NIC per zone, pods
    asking 4 whole GPUs + an RDMA NIC.  NodeNUMAResource's cpu / memory lists hold up to 63 masks each and
    DeviceShare's two copies the 22 masks of >= 4 zones (no preferred merged hint: DeviceShare's minimal size
    is 4, the resources' 1), so a pair folds up to 63 x 63 x 22 x 22 = 1.9M permutations; the oracle walks
    every one of them (policy.go:198-299)."""
    n = 6
    cl = synth.make_cluster(n, synth.BASE_SEED + 731)
    zones = synth.make_numa(cl, synth.BASE_SEED + 732, zone_counts=(6,), policy_weights=(0, 1, 0, 0),
                            no_zone_fraction=0.0, missing_memory_fraction=0.0, allocated_fraction=0.2)
    devs = []
    for i in range(n):
        d = np.zeros(12, abi.DEVICE_DTYPE)
        for z in range(6):
            g, r = d[z], d[6 + z]
            g["type"], g["minor"], g["health"] = abi.DEV_GPU, z, 1
            g["has_total"][:] = 1
            g["total"][:] = [100, synth.GPU_MEM, 100]
            r["type"], r["minor"], r["health"] = abi.DEV_RDMA, z, 1
            r["has_total"][0] = 1
            r["total"][0] = 100
            for x in (g, r):
                x["has_topology"], x["numa_node"], x["pcie_rank"] = 1, z, z
        if i % 3 == 1:  # a used GPU: fewer feasible masks on this node
            d[2]["has_used"][:] = 1
            d[2]["used"][:] = [100, synth.GPU_MEM, 100]
        devs.append(d)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_devices(h, devs)
    pods = synth.make_pods(6, synth.BASE_SEED + 733, key_base=9_800_000_000)
    for j in range(len(pods)):
        r = pods["device_requests"][j]
        r[abi.PDR["koordinator.sh/gpu-core"]] = 400
        r[abi.PDR["koordinator.sh/gpu-memory-ratio"]] = 400
        r[abi.PDR["koordinator.sh/rdma"]] = 100 if j % 2 == 0 else 50
        pods["has_other_requests"][j] = 1
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    assert_eval_equal(a, b)
    assert (a["status"] == 0).sum() >= 6
    _schedule_equal(ev, o, pods)
