"""BASELINE configs through the product at (or near) their own shapes, bit-exact with the oracle
(VERDICT r01 "parity holes"):
  - C4: the config's own generator (synth.make_c4_cluster / make_c4_pods: 128-CPU 2x4x8x2 hosts, NUMA
    policy mix 40/30/30, FullPCPUs LSR/LSE pods) through ke_schedule — placements, scores, cpusets and
    the per-zone NUMA allocations (nodenumaresource/plugin.go:318-406, cpu_accumulator.go:29-232);
  - C5: the full 20k-node cluster (8 GPUs + 2 RDMA per node) with the 64-leaf ElasticQuota tree —
    placements, scores, device minors and every quota's used;
  - an ElasticQuota tree of > 128 quotas, so the replay's quota register banks 2-3 (quotas 128-254) are
    exercised.
The C3 prefix (50k nodes, 2048 pods) is tests/test_gpu_parity.py::test_schedule_large_cluster_prefix."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, synth
from oracle.binding import Oracle

pytestmark = pytest.mark.gpu


def test_c4_generator_schedule_parity(gpu):
    n, p = 400, 200
    cl, zones, tables = synth.make_c4_cluster(n, synth.BASE_SEED + 4)
    pods = synth.make_c4_pods(p, synth.BASE_SEED + 104)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tables)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    diff = np.argwhere(np.any(ev.last_cpusets != o.last_cpusets, axis=1))
    assert len(diff) == 0, f"cpusets differ for pods {diff[:5].ravel().tolist()}"
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    placed = int((c1 >= 0).sum())
    assert placed > p // 2 and np.any(ev.last_cpusets != 0) and np.any(ev.last_numa_allocations != 0)
    # the state after the queue evaluates identically, and the replay records follow every Reserve
    more = synth.make_c4_pods(24, synth.BASE_SEED + 105, key_base=9_000_000_000)
    a, b = ev.eval(more, synth.T0), o.eval(more, synth.T0)
    for k in ("status", "reason", "la", "numa", "total", "best"):
        assert np.array_equal(a[k], b[k]), k
    assert ev.check_records(synth.T0) == 0


def test_c4_full_cluster_prefix(gpu):
    """C4 at its own 50k-node size: the first 12 pods of the bench queue (tools/cpuset_bench.py
    --survey) bit-exact with the oracle -- placements, scores, cpusets, NUMA allocations.  The oracle takes
    about 2.3 s per pod here at 16 threads, so the prefix is short."""
    n, p = 50_000, 12
    cl, zones, tables = synth.make_c4_cluster(n, synth.BASE_SEED + 4)
    pods = synth.make_c4_pods(p, synth.BASE_SEED + 104)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tables)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_cpusets, o.last_cpusets)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert (c1 >= 0).all() and np.any(ev.last_cpusets != 0)


def test_c5_full_cluster_quota_prefix(gpu):
    n, p = 20_000, 640
    cl = synth.make_cluster(n, synth.BASE_SEED + 5)
    devices = synth.make_devices(n, synth.BASE_SEED + 55)
    pods = synth.make_ds_pods(p, synth.BASE_SEED + 105, device_fraction=0.5)
    tc = int(pods["requests"][:, abi.RES_CPU].sum() * 0.6)
    tm = int(pods["requests"][:, abi.RES_MEMORY].sum() * 0.6)
    quotas = synth.make_quota_tree(synth.BASE_SEED + 305, 64, 8, tc, tm)
    pods = synth.assign_quotas(pods, quotas, synth.BASE_SEED + 306)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_devices(h, devices)
        h.quotas_load(synth.quota_args(tc, tm), quotas)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)
    for i in range(len(quotas)):
        a, b = ev.quota_state(i), o.quota_state(i)
        for k in ("limit", "used", "np_used"):
            assert np.array_equal(a[k], b[k]), (i, k)
    refused = int(((c1 < 0) & (pods["quota"] > 0)).sum())
    assert 0 < refused < p and int((ev.last_device_allocations != 0).sum()) > 50
    assert ev.check_records(synth.T0) == 0


@pytest.mark.parametrize("runtime", [True, False])
def test_quota_tree_beyond_128(gpu, runtime):
    """24 parents + 192 leaves: leaves and ancestors live in every register bank of the replay."""
    n = 1200
    cl = synth.make_cluster(n, synth.BASE_SEED + 97)
    pods = synth.make_pods(2600, synth.BASE_SEED + 197)
    tc = int(pods["requests"][:, abi.RES_CPU].sum() * 0.5)
    tm = int(pods["requests"][:, abi.RES_MEMORY].sum() * 0.5)
    q = synth.make_quota_tree(synth.BASE_SEED + 397, 192, 8, tc, tm)
    assert len(q) == 216
    pods = synth.assign_quotas(pods, q, synth.BASE_SEED + 398, no_quota_fraction=0.05)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        h.quotas_load(synth.quota_args(tc, tm, runtime, True), q)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    hi = 0
    for i in range(len(q)):
        a, b = ev.quota_state(i), o.quota_state(i)
        for k in ("limit", "used", "np_used"):
            assert np.array_equal(a[k], b[k]), (i, k)
        hi += i >= 128 and int(a["used"].sum()) > 0
    assert hi > 20  # quotas in banks 2-3 were reserved into
    assert 0 < int(((c1 < 0) & (pods["quota"] > 0)).sum()) < len(pods)
