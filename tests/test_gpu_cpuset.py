"""GPU parity for cpuset pods (NodeNUMAResource with NUMA policy None): the cpuset PreFilter state,
requestCPUBind, the amplified-cpu Filter / Score of binding pods, the bind-policy / SMT checks, the
required policies' trial allocation, and Reserve through the device CPU accumulator
(k_cpuset_reserve) — against the reference's plugin_test.go vectors and the oracle, bit-exact
(status, reason, scores, chosen node, cpuset)."""
import numpy as np
import pytest

import cases
from koordinator_amd import Evaluator, abi, model, synth
from oracle.binding import Oracle

pytestmark = pytest.mark.gpu

CPUSET = cases.load("cpuset.json")


@pytest.mark.parametrize("case", CPUSET, ids=[f'{c["op"]}: {c["name"]}' for c in CPUSET])
def test_golden_cpuset_plugin(gpu, case):
    ev = Evaluator(abi.default_config(1))
    pod = cases.setup_cpuset_case(ev, case)
    if case["op"] == "filter":
        r = ev.eval([pod], cases.NOW)
        assert (int(r["status"][0, 0]), int(r["reason"][0, 0])) == (case["want"]["code"], case["want"]["reason"]), \
            case["source"]
        return
    chosen, _ = ev.schedule([pod], cases.NOW)
    if case["want"]["fails"]:
        assert chosen[0] == -1, case["source"]
        return
    assert chosen[0] == 0, case["source"]
    assert cases.bits_cpus(ev.last_cpusets[0]) == cases.parse_cpuset(case["want"]["cpuset"]), case["source"]


def cpuset_both(n_nodes, seed, batch=64, numa_most=False, most=False, **kw):
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + seed, amplified_fraction=0.3)
    tabs = synth.make_cpus(cl, synth.BASE_SEED + seed + 1, **kw)
    cfg = synth.config(n_nodes, pod_batch=batch)
    if numa_most:
        cfg.numa.numa_strategy = abi.STRATEGY_MOST_ALLOCATED
    if most:
        cfg.numa.strategy = abi.STRATEGY_MOST_ALLOCATED
    ev, o = Evaluator(cfg), Oracle(cfg, n_nodes)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_cpus(h, tabs)
    return ev, o


def assert_eval_equal(a, b):
    for k in ("status", "reason", "la", "numa", "total", "best"):
        mism = np.argwhere(a[k] != b[k])
        assert len(mism) == 0, f"{k}: {len(mism)} mismatches, first {mism[:5].tolist()}"


def assert_schedule_equal(ev, o, pods, now):
    c1, s1 = ev.schedule(pods, now)
    c0, s0 = o.schedule(pods, now)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].tolist()
    assert np.array_equal(s1, s0)
    diff = np.argwhere(np.any(ev.last_cpusets != o.last_cpusets, axis=1))
    assert len(diff) == 0, f"cpusets differ for pods {diff[:5].ravel().tolist()}"
    return c1


@pytest.mark.parametrize("variant", ["least", "numa-most", "most"])
def test_cpuset_eval_matrix_parity(gpu, variant):
    """Every (pod, node): PreFilter invalid requests, node-forced binding, amplified binding cpu,
    topology / bind-policy / SMT / trial-allocation outcomes and the scores equal the oracle's."""
    ev, o = cpuset_both(300, 201, numa_most=variant == "numa-most", most=variant == "most")
    pods = synth.make_cpuset_pods(120, synth.BASE_SEED + 203)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    assert_eval_equal(a, b)
    reasons = set(np.unique(a["reason"]).tolist())
    for r in (abi.REASON_NUMA_INVALID_REQUESTED_CPUS, abi.REASON_NUMA_CPU_BIND_POLICY_CONFLICT,
              abi.REASON_NUMA_SMT_ALIGNMENT, abi.REASON_NUMA_INSUFFICIENT_CPUS, abi.REASON_NUMA_INVALID_CPU_TOPOLOGY):
        assert r in reasons, r


@pytest.mark.parametrize("variant", ["least", "numa-most"])
def test_cpuset_schedule_parity(gpu, variant):
    """Sequential placements: each binding pod's cpuset from the device accumulator equals the
    oracle's (takeCPUs), failed Reserves leave the pod unplaced, later pods see the patched CPU
    tables, allocated counts and NodeInfo; a second queue and an eval see the host mirror."""
    ev, o = cpuset_both(300, 211, numa_most=variant == "numa-most")
    pods = synth.make_cpuset_pods(160, synth.BASE_SEED + 213)
    c = assert_schedule_equal(ev, o, pods, synth.T0)
    assert (c >= 0).sum() > 100
    assert np.any(ev.last_cpusets != 0)
    more = synth.make_cpuset_pods(40, synth.BASE_SEED + 214, key_base=5_000_000_000)
    assert_eval_equal(ev.eval(more, synth.T0), o.eval(more, synth.T0))
    assert_schedule_equal(ev, o, more, synth.T0)
    assert ev.check_records(synth.T0) == 0  # cpuset Reserves keep the replay records current


def test_cpuset_schedule_shared_cpus(gpu):
    """MaxRefCount 2-3 everywhere (CPU sharing: RefCount in the sorts), dense allocations."""
    ev, o = cpuset_both(200, 221, max_ref_choices=(2, 3), allocated_choices=(0.3, 0.6, 0.9))
    pods = synth.make_cpuset_pods(160, synth.BASE_SEED + 223, cpuset_fraction=0.8)
    assert_schedule_equal(ev, o, pods, synth.T0)


def test_cpuset_schedule_node_bind_everywhere(gpu):
    """Every node forces binding: every cpu-requesting pod binds (singleton batches throughout)."""
    ev, o = cpuset_both(160, 231, bind_weights=(0.0, 0.5, 0.5))
    pods = synth.make_cpuset_pods(100, synth.BASE_SEED + 233, cpuset_fraction=0.3)
    assert_schedule_equal(ev, o, pods, synth.T0)


def test_cpuset_sharded_loopback(gpu):
    ev, o = cpuset_both(1100, 241)
    pods = synth.make_cpuset_pods(96, synth.BASE_SEED + 243)
    ev.shard_init(0, 3, None)
    assert_schedule_equal(ev, o, pods, synth.T0)


def test_cpuset_edge_cases(gpu):
    """No CPU tables at all, a request larger than the node, an exhausted node (Reserve fails after a
    preferred-policy Filter passes), and a cleared table."""
    cfg = abi.default_config(3)
    ev, o = Evaluator(cfg), Oracle(cfg, 3)
    rows = cases.test_topology(1, 1, 4, 2)  # 8 CPUs, 2 per core
    for h in (ev, o):
        for i in range(3):
            h.upsert_node(i, model.make_node(allocatable={"cpu": "8", "memory": "64Gi"}))
        h.set_cpus(1, model.make_cpus(rows))
        h.set_cpus(2, model.make_cpus(rows, {c: (1, None) for c in range(6)}))
    big = cases.cpuset_pod({"kind": "cpuset", "cpu": "16"})
    pref = cases.cpuset_pod({"kind": "cpuset", "cpu": "4", "preferred": "SpreadByPCPUs"})
    req = cases.cpuset_pod({"kind": "cpuset", "cpu": "4", "required": "FullPCPUs"})
    plain = model.make_pod(requests={"cpu": "1"})
    pods = [big, pref, req, plain, pref, pref, req]
    assert_eval_equal(ev.eval(pods, cases.NOW), o.eval(pods, cases.NOW))
    assert_schedule_equal(ev, o, pods, cases.NOW)
    for h in (ev, o):
        h.set_cpus(1, model.make_cpus([]))
    assert_eval_equal(ev.eval(pods, cases.NOW), o.eval(pods, cases.NOW))


# ---- cpusets under NUMA topology policies (config 4) ----------------------------------------------
NUMA_CPUSET = [c for c in cases.load("numa_cpuset.json") if c["op"] == "node_score"]


@pytest.mark.parametrize("case", NUMA_CPUSET, ids=[c["name"] for c in NUMA_CPUSET])
def test_golden_numa_node_score(gpu, case):
    """TestNUMANodeScore through the product: Filter + Score under SingleNUMANode / Restricted, incl. an
    LSR pod whose requested cpu is the node's cpuset count (scoring.go:179-185)."""
    cfg = abi.default_config(len(case["nodes"]))
    cfg.numa.strategy = abi.STRATEGY_MOST_ALLOCATED
    ev = Evaluator(cfg)
    pod = cases.setup_numa_score_case(ev, case)
    r = ev.eval([pod], cases.NOW)
    assert list(r["status"][0]) == [abi.CODE_SUCCESS] * len(case["nodes"]), case["source"]
    assert [int(x) for x in r["numa"][0]] == case["want"]["scores"], case["source"]


def numa_cpuset_both(n_nodes, seed, no_la=True, batch=64, numa_most=False, **kw):
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + seed, amplified_fraction=0.3)
    zs, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1, **kw)
    cfg = synth.config(n_nodes, pod_batch=batch)
    if no_la:
        cfg.loadaware.usage_thresholds[:] = [abi.ABSENT, abi.ABSENT]
    if numa_most:
        cfg.numa.numa_strategy = abi.STRATEGY_MOST_ALLOCATED
    ev, o = Evaluator(cfg), Oracle(cfg, n_nodes)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zs)
        synth.load_cpus(h, tabs)
    return ev, o


NUMA_VARIANTS = {
    "mixed": dict(),
    "eight-zones-shared": dict(zone_counts=(8,), max_ref_choices=(2, 3)),
    "forced-binding": dict(bind_weights=(0.2, 0.4, 0.4), policy_weights=(0, 1, 1, 1)),
    "hint-most": dict(numa_most=True, zone_counts=(2, 4)),
}


@pytest.mark.parametrize("name", list(NUMA_VARIANTS))
def test_numa_cpuset_eval_matrix_parity(gpu, name):
    """Binding pods under every policy: trimmed availability, whole-CPU splits, per-zone CPU counts,
    nil affinities, the cpuset NUMA-scope score — every (pod, node) equal to the oracle."""
    ev, o = numa_cpuset_both(240, 401, **NUMA_VARIANTS[name])
    pods = synth.make_numa_cpuset_pods(72, synth.BASE_SEED + 403)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    assert_eval_equal(a, b)
    assert np.any(a["status"] == abi.CODE_SUCCESS)


@pytest.mark.parametrize("name", ["mixed", "eight-zones-shared", "forced-binding"])
def test_numa_cpuset_schedule_parity(gpu, name):
    """Sequential placements: per-zone accumulator takes, NUMA allocations and cpusets, the zones'
    entries / statuses patched for later pods of the queue, then a second queue and an eval."""
    ev, o = numa_cpuset_both(240, 411, **NUMA_VARIANTS[name])
    pods = synth.make_numa_cpuset_pods(160, synth.BASE_SEED + 413)
    c = assert_schedule_equal(ev, o, pods, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert (c >= 0).sum() > 80
    more = synth.make_numa_cpuset_pods(40, synth.BASE_SEED + 414, key_base=7_000_000_000)
    assert_eval_equal(ev.eval(more, synth.T0), o.eval(more, synth.T0))
    assert_schedule_equal(ev, o, more, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)


def test_numa_cpuset_pod_policies_on_policy_none_nodes(gpu):
    """Nodes without a policy: binding pods take CPUs node-wide (zones without an allocation entry
    gain cpusets), later pods with their own policy create entries there — under a cpu ratio > 1 an
    entry's cpu carries its zone's cpuset adjustment (node_allocation.go:221-243)."""
    ev, o = numa_cpuset_both(240, 441, policy_weights=(1, 0, 0, 0), cpuset_fraction=(0.0, 0.1))
    pods = synth.make_numa_cpuset_pods(200, synth.BASE_SEED + 443, policy_fraction=0.5)
    assert_schedule_equal(ev, o, pods, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    more = synth.make_numa_cpuset_pods(40, synth.BASE_SEED + 444, policy_fraction=0.5, key_base=7_500_000_000)
    assert_eval_equal(ev.eval(more, synth.T0), o.eval(more, synth.T0))


def test_numa_cpuset_with_load_aware(gpu):
    ev, o = numa_cpuset_both(240, 421, no_la=False)
    pods = synth.make_numa_cpuset_pods(96, synth.BASE_SEED + 423)
    assert_eval_equal(ev.eval(pods, synth.T0), o.eval(pods, synth.T0))
    assert_schedule_equal(ev, o, pods, synth.T0)


def test_numa_cpuset_sharded_loopback(gpu):
    ev, o = numa_cpuset_both(1100, 431)
    pods = synth.make_numa_cpuset_pods(96, synth.BASE_SEED + 433)
    ev.shard_init(0, 3, None)
    assert_schedule_equal(ev, o, pods, synth.T0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
