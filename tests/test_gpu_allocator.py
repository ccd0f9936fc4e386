"""GPUAllocator.Allocate on the GPU: partitions (allocateByPartition +
selectPartitionByBinPack, allocator_gpu.go:177-296) and topology scopes (allocateByDeviceTopology /
allocateFromScope, :312-451), bit-exact with the oracle, whose restatement the transcribed Go vectors pin
(tests/golden/gpu_allocator.json, test_oracle_golden.py::test_gpu_allocator)."""
import numpy as np
import pytest

import cases
from koordinator_amd import Evaluator, abi, model, synth
from oracle.binding import Oracle
from test_oracle_golden import GPU_ALLOC, gpu_alloc_cfg, gpu_alloc_setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", GPU_ALLOC, ids=[c["name"] for c in GPU_ALLOC])
def test_gpu_allocator_golden_on_device(gpu, case):
    """The Go vectors through the product: Filter status/reason from ke_eval, minors from ke_schedule."""
    ev = Evaluator(gpu_alloc_cfg(case))
    pod = gpu_alloc_setup(ev, case)
    r = ev.eval([pod], cases.NOW)
    want = case["want"]
    assert (int(r["status"][0, 0]), int(r["reason"][0, 0])) == (want["code"], want["reason"]), case["source"]
    chosen, _ = ev.schedule([pod], cases.NOW)
    if want["code"]:
        assert chosen[0] == -1
    else:
        mask = int(ev.last_device_allocations[0])
        assert [m for m in range(16) if mask >> m & 1] == want["minors"], case["source"]


def _cluster(n, seed, topology=True, partitions=True):
    cl = synth.make_cluster(n, seed)
    devs = synth.make_devices(n, seed + 1)
    if topology:
        synth.add_gpu_topology(devs, seed + 2)
    states = synth.make_partition_states(n, seed + 3) if partitions else None
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_devices(h, devs)
        if states:
            synth.load_partition_states(h, states)
    return ev, o


@pytest.mark.parametrize("topology,partitions", [(True, True), (True, False), (False, True)])
def test_gpu_allocator_eval_parity(gpu, topology, partitions):
    ev, o = _cluster(400, 601, topology, partitions)
    pods = synth.make_gpu_alloc_pods(160, 602)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    for k in ("status", "reason", "la", "numa", "total", "best"):
        assert np.array_equal(a[k], b[k]), (k, np.argwhere(a[k] != b[k])[:5].tolist())
    reasons = set(np.unique(a["reason"][a["status"] != 0]).tolist())
    if partitions:
        assert {abi.REASON_DS_MISSING_PARTITION_TABLE, abi.REASON_DS_UNSUPPORTED_GPU_REQUESTS,
                abi.REASON_DS_INSUFFICIENT_PARTITIONED} <= reasons
    if topology:
        assert {abi.REASON_DS_INSUFFICIENT_TOPOLOGY_SCOPED, abi.REASON_DS_MISSING_TOPOLOGY_TREE} <= reasons


@pytest.mark.parametrize("topology,partitions", [(True, True), (True, False)])
def test_gpu_allocator_schedule_parity(gpu, topology, partitions):
    """Reserve picks the minors: every later pod sees them in the device state."""
    ev, o = _cluster(96, 611, topology, partitions)
    pods = synth.make_gpu_alloc_pods(320, 612)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations), \
        np.argwhere(ev.last_device_allocations != o.last_device_allocations)[:5].ravel().tolist()
    placed = int((c1 >= 0).sum())
    assert 0 < placed < len(pods)
    more = synth.make_gpu_alloc_pods(40, 613, key_base=9_500_000_000)
    a, b = ev.eval(more, synth.T0), o.eval(more, synth.T0)
    for k in ("status", "reason", "total", "best"):
        assert np.array_equal(a[k], b[k]), k
