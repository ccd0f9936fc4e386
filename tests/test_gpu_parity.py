"""GPU parity: the gfx950 path (libkoordeval.so through the C ABI) against the oracle and the golden
vectors.  Bit-exact on every status, reason, per-plugin score, framework total and selected node."""
import numpy as np
import pytest

import cases
from koordinator_amd import Evaluator, abi, model, synth
from oracle.binding import Oracle

pytestmark = pytest.mark.gpu

LA_FILTER = cases.load("loadaware_filter.json")
LA_SCORE = cases.load("loadaware_score.json")
NUMA = cases.load("numa.json")


# ---- golden vectors through the product ----------------------------------------------------------
@pytest.mark.parametrize("case", LA_FILTER, ids=[c["name"] for c in LA_FILTER])
def test_golden_loadaware_filter(gpu, case):
    ev = Evaluator(cases.make_cfg(case))
    pod = cases.setup_loadaware(ev, case)
    r = ev.eval([pod], cases.NOW)
    assert (int(r["status"][0, 0]), int(r["reason"][0, 0])) == (case["want"]["code"], case["want"]["reason"])


@pytest.mark.parametrize("case", LA_SCORE, ids=[c["name"] for c in LA_SCORE])
def test_golden_loadaware_score(gpu, case):
    # Go's TestScore calls Score without Filter: disable the thresholds so every node reaches Score
    cfg = cases.make_cfg(case)
    cfg.loadaware.usage_thresholds[:] = [abi.ABSENT, abi.ABSENT]
    cfg.loadaware.filter_expired_node_metrics = 0
    ev = Evaluator(cfg)
    pod = cases.setup_loadaware(ev, case)
    r = ev.eval([pod], cases.NOW)
    assert r["status"][0, 0] == abi.CODE_SUCCESS
    assert int(r["la"][0, 0]) == case["want"]["score"], case["source"]


@pytest.mark.parametrize("case", NUMA, ids=[c["name"] for c in NUMA])
def test_golden_numa(gpu, case):
    nodes = cases.make_numa_nodes(case)
    ev = Evaluator(cases.make_cfg(case, len(nodes)))
    for i, n in enumerate(nodes):
        ev.upsert_node(i, n)
    r = ev.eval([cases.make_pod(case["pod"])], cases.NOW)
    if case["op"] == "score":
        assert [int(x) for x in r["numa"][0]] == case["want"]["scores"], case["source"]
    else:
        assert (int(r["status"][0, 0]), int(r["reason"][0, 0])) == (case["want"]["code"], case["want"]["reason"])


# ---- synthetic clusters: full matrices vs the oracle --------------------------------------------
def both(cfg, cl):
    ev, o = Evaluator(cfg), Oracle(cfg, cl.n_nodes)
    synth.load_into(ev, cl)
    synth.load_into(o, cl)
    return ev, o


def assert_eval_equal(a, b):
    for k in ("status", "reason", "la", "numa", "total", "best"):
        mism = np.argwhere(a[k] != b[k])
        assert len(mism) == 0, f"{k}: {len(mism)} mismatches, first {mism[:5].tolist()}"


VARIANTS = {
    "default": dict(),
    "amplified": dict(amplified=0.3),
    "aggregated": dict(agg=True),
    "prod-thresholds": dict(prod=True),
    "most-allocated": dict(most=True),
    "customize": dict(windows=True),
}


def variant_cfg(n, v, batch=64):
    cfg = synth.config(n, pod_batch=batch)
    a = cfg.loadaware
    if v.get("agg"):
        a.has_aggregated = 1
        a.agg_usage_thresholds[:] = [60, 90]
        a.agg_usage_type = abi.AGG_P95
        a.agg_usage_duration_ns = 300 * synth.NS
        a.agg_score_type = abi.AGG_P95
        a.agg_score_duration_ns = 0
    if v.get("prod"):
        a.prod_usage_thresholds[:] = [55, 85]
        a.score_according_prod_usage = 1
    if v.get("most"):
        cfg.numa.strategy = abi.STRATEGY_MOST_ALLOCATED
    if v.get("windows"):
        a.estimated_seconds_after_pod_scheduled = 7200  # pre-existing pods (t0-3600s) are re-estimated
        a.allow_customize_estimation = 1
    return cfg


@pytest.mark.parametrize("name", list(VARIANTS))
def test_eval_matrix_parity(gpu, name):
    v = VARIANTS[name]
    cl = synth.make_cluster(777, synth.BASE_SEED + 11, amplified_fraction=v.get("amplified", 0.0))
    pods = synth.make_pods(96, synth.BASE_SEED + 12)
    ev, o = both(variant_cfg(cl.n_nodes, v), cl)
    assert_eval_equal(ev.eval(pods, synth.T0), o.eval(pods, synth.T0))


def test_eval_zero_pods_and_single_node(gpu):
    cl = synth.make_cluster(1, synth.BASE_SEED + 13)
    ev, o = both(synth.config(1), cl)
    assert ev.eval(synth.make_pods(0, 1), synth.T0)["best"].shape == (0,)
    pods = synth.make_pods(5, synth.BASE_SEED + 14)
    assert_eval_equal(ev.eval(pods, synth.T0), o.eval(pods, synth.T0))


def test_eval_time_advances(gpu):
    """now past NodeMetric expiry: the device recomputes expiry from `now` (no stale rows)."""
    cl = synth.make_cluster(300, synth.BASE_SEED + 15)
    ev, o = both(synth.config(300), cl)
    pods = synth.make_pods(8, synth.BASE_SEED + 16)
    for now in (synth.T0, synth.T0 + 3600 * synth.NS, synth.T0 + 10**7 * synth.NS):
        assert_eval_equal(ev.eval(pods, now), o.eval(pods, now))


# ---- schedule: sequential placements vs the oracle ------------------------------------------------
def test_schedule_parity_config1(gpu):
    """BASELINE config 1: 1k nodes x 1k pods, every placement identical to one-at-a-time scheduling."""
    cl = synth.make_cluster(1000, synth.BASE_SEED + 1)
    pods = synth.make_pods(1000, synth.BASE_SEED + 101)
    ev, o = both(synth.config(1000), cl)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5]
    assert np.array_equal(s1, s0)
    # the device's Reserve patches equal a from-scratch host derivation of the object state
    dev, host = ev.debug_rows(synth.T0)
    assert np.array_equal(dev["f"], host["f"]) and np.array_equal(dev["flags"], host["flags"])
    # and the state after the queue evaluates identically
    more = synth.make_pods(64, synth.BASE_SEED + 102)
    assert_eval_equal(ev.eval(more, synth.T0), o.eval(more, synth.T0))


@pytest.mark.parametrize("name", ["amplified", "prod-thresholds", "most-allocated", "aggregated", "customize"])
def test_schedule_parity_variants(gpu, name):
    v = VARIANTS[name]
    cl = synth.make_cluster(640, synth.BASE_SEED + 21, amplified_fraction=v.get("amplified", 0.0))
    pods = synth.make_pods(700, synth.BASE_SEED + 22)
    ev, o = both(variant_cfg(cl.n_nodes, v), cl)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5]
    assert np.array_equal(s1, s0)


def test_schedule_parity_config2_prefix(gpu):
    """BASELINE config 2 cluster (5k nodes), first 1500 pods of its 10k queue."""
    cl = synth.make_cluster(5000, synth.BASE_SEED + 2)
    pods = synth.make_pods(1500, synth.BASE_SEED + 102)
    ev, o = both(synth.config(5000), cl)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)


@pytest.mark.parametrize("batch", [1, 7, 64])
def test_schedule_batch_size_invariance(gpu, batch):
    """Exact speculative batching: any batch size gives the one-pod-at-a-time result (batch 1)."""
    cl = synth.make_cluster(400, synth.BASE_SEED + 31)
    pods = synth.make_pods(300, synth.BASE_SEED + 32)
    ev1 = Evaluator(synth.config(400, pod_batch=1))
    evb = Evaluator(synth.config(400, pod_batch=batch))
    synth.load_into(ev1, cl)
    synth.load_into(evb, cl)
    a = ev1.schedule(pods, synth.T0)
    b = evb.schedule(pods, synth.T0)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_schedule_split_queue_is_idempotent(gpu):
    """Scheduling a queue in one call or in two consecutive calls gives the same placements."""
    cl = synth.make_cluster(2000, synth.BASE_SEED + 41)
    pods = synth.make_pods(900, synth.BASE_SEED + 42)
    ev1 = Evaluator(synth.config(2000))
    ev2 = Evaluator(synth.config(2000))
    synth.load_into(ev1, cl)
    synth.load_into(ev2, cl)
    a, _ = ev1.schedule(pods, synth.T0)
    b1, _ = ev2.schedule(pods[:333], synth.T0)
    b2, _ = ev2.schedule(pods[333:], synth.T0)
    assert np.array_equal(a, np.concatenate([b1, b2]))


def test_schedule_unschedulable_pods(gpu):
    """Pods that fit nowhere come back -1 and do not change any node."""
    cl = synth.make_cluster(64, synth.BASE_SEED + 51)
    ev, o = both(synth.config(64), cl)
    huge = model.make_pod(requests={"cpu": "100000", "memory": "1Ti"}, limits={"cpu": "100000", "memory": "1Ti"})
    pods = synth.make_pods(40, synth.BASE_SEED + 52)
    seq = [huge] + [pods[i] for i in range(20)] + [huge] + [pods[i] for i in range(20, 40)]
    seq_arr = np.concatenate([np.frombuffer(bytes(p), dtype=abi.POD_DTYPE) if isinstance(p, abi.Pod) else p[None]
                              for p in seq])
    c1, s1 = ev.schedule(seq_arr, synth.T0)
    c0, s0 = o.schedule(seq_arr, synth.T0)
    assert c1[0] == -1 and c1[21] == -1
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)


def test_schedule_large_cluster_prefix(gpu):
    """BASELINE config 3 cluster (50k nodes) and queue: first 2048 pods (32 pipelined 64-pod batches)
    vs the oracle, bit-exact, then the rows the device patched vs a from-scratch host derivation."""
    cl = synth.make_cluster(50_000, synth.BASE_SEED + 3)
    pods = synth.make_pods(2048, synth.BASE_SEED + 103)
    ev, o = both(synth.config(50_000), cl)
    c1, s1 = ev.schedule(pods, synth.T0)
    assert ev.kernel_stats()["pipelined_batches"] == 32
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    dev, host = ev.debug_rows(synth.T0)
    assert np.array_equal(dev, host)
    assert ev.check_records(synth.T0) == 0


@pytest.mark.parametrize("per_call", [5000, 100_000], ids=["driver-calls", "one-call"])
def test_c3_full_queue_fixture(gpu, per_call):
    """the headline run end to end -- all 100,000 pods of the config-3 queue on the 50k-node
    cluster (1,563 pipelined batches: stale lists, helpers, k_patch), in the driver's 5,000-pod calls and in one
    call -- against the oracle's full-queue fixture (tests/golden/make_c3_fixture.py), every placement and
    score bit-exact, the rows and records exact afterwards."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_c3_fixture import build_inputs, inputs_digest
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_placements.npz"))
    cl, pods = build_inputs()
    assert str(g["digest"]) == inputs_digest(cl, pods), "generator changed: regenerate the fixture"
    ev = Evaluator(synth.config(cl.n_nodes))
    synth.load_into(ev, cl)
    chosen, score = [], []
    for s in range(0, len(pods), per_call):
        c, sc = ev.schedule(pods[s:s + per_call], synth.T0)
        chosen.append(c)
        score.append(sc)
    chosen, score = np.concatenate(chosen), np.concatenate(score)
    bad = np.flatnonzero((chosen != g["chosen"]) | (score != g["score"].astype(np.int32)))
    assert len(bad) == 0, (len(bad), bad[:5].tolist())
    assert (chosen >= 0).sum() > 90_000
    dev, host = ev.debug_rows(synth.T0)
    assert np.array_equal(dev, host)
    assert ev.check_records(synth.T0) == 0


# ---- the stale-list run's options: T-row helpers, progressive R+S, patched early eval -----------------
@pytest.mark.parametrize("helpers,patch,ignore,ahead,parts,fixm",
                         [("0", "1", "0", "1", "8", "1"), ("4", "0", "0", "1", "8", "1"), ("4", "1", "1", "1", "8", "1"),
                          ("8", "1", "0", "1", "8", "1"), ("4", "1", "0", "0", "8", "1"), ("0", "1", "0", "0", "8", "1"),
                          ("4", "1", "0", "1", "1", "1"), ("4", "1", "0", "1", "8", "0")],
                         ids=["no-helpers", "no-patch", "helpers-ignored", "8-helpers", "patch-then-select",
                              "patch-then-select-no-helpers", "one-part-select", "merge-in-select"])
@pytest.mark.parametrize("n_nodes,n_pods,seed", [(20_000, 3000, 71), (150, 2500, 72)])
def test_stale_run_options_match_oracle(gpu, monkeypatch, n_nodes, n_pods, seed, helpers, patch, ignore, ahead, parts,
                                       fixm):
    """The stale-list run with its helper workgroups off / on (progressive R+S) / on but ignored (the replay's
    own T rows after the barrier), with the eval waiting for batch b-2 instead of batch b-3, and with batch b-2's
    changed nodes patched into the scores before the select (k_patch) instead of into the select-ahead lists
    (k_fixlist), with the split select's parts merged by k_fixlist or by the select's last part: every variant places
    exactly as the oracle and leaves exact rows and records (KOORDEVAL_* are read per device context)."""
    monkeypatch.setenv("KOORDEVAL_T_HELPERS", helpers)
    monkeypatch.setenv("KOORDEVAL_EVAL_PATCH", patch)
    monkeypatch.setenv("KOORDEVAL_T_HELPERS_IGNORE", ignore)
    monkeypatch.setenv("KOORDEVAL_SELECT_AHEAD", ahead)
    monkeypatch.setenv("KOORDEVAL_SELECT_PARTS", parts)  # 8: split selects at 20k nodes (parts of >= 4096 nodes)
    monkeypatch.setenv("KOORDEVAL_FIX_MERGE", fixm)  # 0: the split select merges its parts, not k_fixlist
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + seed)
    pods = synth.make_pods(n_pods, synth.BASE_SEED + 100 + seed)
    ev, o = both(synth.config(n_nodes), cl)
    c1, s1 = ev.schedule(pods, synth.T0)
    ks = ev.kernel_stats()
    assert ks["pipelined_batches"] > 0
    hit = ks["resolve_phases_ms"]["t_helper_hit"]
    assert hit == 0 if helpers == "0" or ignore == "1" else hit > 0
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    dev, host = ev.debug_rows(synth.T0)
    assert np.array_equal(dev, host)
    assert ev.check_records(synth.T0) == 0


# ---- pipelined schedule (two streams, stale lists -> the replay's T slots, or k_fixup) ---------------
@pytest.mark.parametrize("mode", [True, "fixup"], ids=["stale-slots", "fixup"])
@pytest.mark.parametrize("n_nodes,n_pods,seed", [(20_000, 3000, 71), (150, 2500, 72), (40, 1200, 73)])
def test_pipeline_matches_serial_and_oracle(gpu, n_nodes, n_pods, seed, mode):
    """Batch b's eval/select against the stale snapshot (batch b-1 still resolving) give the same placements
    as the serial one-stream schedule and the oracle, whether the replay takes the stale lists with batch
    b-1's changed nodes as slots or k_fixup makes them exact first.  The small clusters make every batch
    touch most candidate lists (most pods take a node the previous batch changed)."""
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + seed)
    pods = synth.make_pods(n_pods, synth.BASE_SEED + 100 + seed)
    ev, o = both(synth.config(n_nodes), cl)
    ev.set_pipeline(mode)
    es = Evaluator(synth.config(n_nodes))
    synth.load_into(es, cl)
    es.set_pipeline(False)
    c1, s1 = ev.schedule(pods, synth.T0)
    assert ev.kernel_stats()["pipelined_batches"] > 0
    c2, s2 = es.schedule(pods, synth.T0)
    assert es.kernel_stats()["pipelined_batches"] == 0
    assert np.array_equal(c1, c2) and np.array_equal(s1, s2)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert ev.check_records(synth.T0) == 0 and es.check_records(synth.T0) == 0
    es.close()


@pytest.mark.parametrize("name", ["prod-thresholds", "most-allocated", "amplified"])
def test_pipeline_with_unschedulable_and_variants(gpu, name):
    """Pipelined batches whose predecessor placed nothing (chosen -1); MostAllocated scores rise on the
    touched nodes (nothing in the exactness argument assumes they fall)."""
    v = VARIANTS[name]
    cl = synth.make_cluster(64, synth.BASE_SEED + 51, amplified_fraction=v.get("amplified", 0.0))
    cfg = variant_cfg(64, v)
    ev, o = both(cfg, cl)
    huge = model.make_pod(requests={"cpu": "100000", "memory": "1Ti"}, limits={"cpu": "100000", "memory": "1Ti"})
    pods = synth.make_pods(600, synth.BASE_SEED + 75)
    hp = np.frombuffer(bytes(huge), dtype=abi.POD_DTYPE)
    seq = np.concatenate([np.repeat(hp, 64), pods[:200], np.repeat(hp, 70), pods[200:]])
    c1, s1 = ev.schedule(seq, synth.T0)
    c0, s0 = o.schedule(seq, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert (c1 == -1).sum() >= 64 and ev.kernel_stats()["pipelined_batches"] > 0


# ---- node sharding (loopback: every shard's eval/select + k_merge in one context) -----------------
@pytest.mark.parametrize("world", [2, 3, 8])
def test_schedule_sharded_loopback_parity(gpu, world):
    """Per-shard top-k_j lists merged by k_merge give the unsharded placements (config-1 cluster)."""
    cl = synth.make_cluster(3000, synth.BASE_SEED + 61)
    pods = synth.make_pods(700, synth.BASE_SEED + 62)
    ev, o = both(synth.config(3000), cl)
    ev.shard_init(0, world, None)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5]
    assert np.array_equal(s1, s0)


def test_shard_ranges_match_host_plan(gpu):
    from koordinator_amd import shard
    cl = synth.make_cluster(5000, synth.BASE_SEED + 63)
    ev = Evaluator(synth.config(5000))
    synth.load_into(ev, cl)
    for world in (1, 2, 4, 8):
        got = []
        for r in range(world):
            ev.shard_init(r, world, None)
            got.append(ev.shard_range())
        assert got == [shard.node_range(5000, r, world) for r in range(world)]


def test_rccl_single_rank_communicator(gpu):
    """The real RCCL path (unique id, ncclCommInitRank, in-place ncclAllGather, k_merge) with a
    1-rank communicator: placements equal the oracle's."""
    from koordinator_amd.evaluator import comm_unique_id
    uid = comm_unique_id()
    assert len(uid) == abi.COMM_ID_BYTES
    cl = synth.make_cluster(2000, synth.BASE_SEED + 64)
    pods = synth.make_pods(300, synth.BASE_SEED + 65)
    ev, o = both(synth.config(2000), cl)
    ev.shard_init(0, 1, uid)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)


# ---- DeviceShare ---------------------------------------------------------------------------------
DS = [c for c in cases.load("deviceshare.json") if c["op"] in ("filter", "score")]


@pytest.mark.parametrize("case", DS, ids=[c["name"] for c in DS])
def test_golden_deviceshare(gpu, case):
    ev = Evaluator(cases.ds_cfg(case))
    pod = cases.setup_ds(ev, case)
    r = ev.eval([pod], cases.NOW)
    want = case["want"]
    assert (int(r["status"][0, 0]), int(r["reason"][0, 0])) == (want["code"], want["reason"]), case["source"]
    if case["op"] == "score":
        assert int(r["ds"][0, 0]) == want["score"], case["source"]


def ds_both(n_nodes, seed, strategy=abi.STRATEGY_LEAST_ALLOCATED, batch=64):
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + seed)
    dv = synth.make_devices(n_nodes, synth.BASE_SEED + seed + 50)
    cfg = synth.config(n_nodes, pod_batch=batch)
    cfg.deviceshare.strategy = strategy
    ev, o = Evaluator(cfg), Oracle(cfg, n_nodes)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_devices(h, dv)
    return ev, o


@pytest.mark.parametrize("strategy", [abi.STRATEGY_LEAST_ALLOCATED, abi.STRATEGY_MOST_ALLOCATED])
def test_deviceshare_eval_matrix_parity(gpu, strategy):
    ev, o = ds_both(700, 81, strategy)
    pods = synth.make_ds_pods(48, synth.BASE_SEED + 82)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    for k in ("status", "reason", "la", "numa", "ds", "total", "best"):
        mism = np.argwhere(a[k] != b[k])
        assert len(mism) == 0, f"{k}: {len(mism)} mismatches, first {mism[:5].tolist()}"


@pytest.mark.parametrize("strategy", [abi.STRATEGY_LEAST_ALLOCATED, abi.STRATEGY_MOST_ALLOCATED])
def test_deviceshare_schedule_parity(gpu, strategy):
    """Mixed queue: DeviceShare pods (batched with the plain pods, NormalizeScore over all feasible nodes);
    placements, scores and the allocated device minors equal the oracle's."""
    ev, o = ds_both(1500, 83, strategy)
    pods = synth.make_ds_pods(600, synth.BASE_SEED + 84)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5]
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)
    # the device state after the queue evaluates identically (device cache patched by Reserve)
    more = synth.make_ds_pods(32, synth.BASE_SEED + 85)
    a, b = ev.eval(more, synth.T0), o.eval(more, synth.T0)
    for k in ("status", "ds", "total", "best"):
        assert np.array_equal(a[k], b[k]), k
    assert ev.check_records(synth.T0) == 0


@pytest.mark.parametrize("strategy", [abi.STRATEGY_LEAST_ALLOCATED, abi.STRATEGY_MOST_ALLOCATED])
def test_deviceshare_batches_exact(gpu, strategy):
    """DeviceShare pods share speculative batches: each pod's NormalizeScore max is checked in the replay and
    the batch stops where it may have moved (MostAllocated moves it often).  Every batch size gives the
    oracle's placements, scores and device minors."""
    pods = synth.make_ds_pods(400, synth.BASE_SEED + 94, device_fraction=0.7)
    ref = None
    for b in (1, 7, 64):
        ev, o = ds_both(900, 93, strategy, batch=b)
        c1, s1 = ev.schedule(pods, synth.T0)
        if ref is None:
            c0, s0 = o.schedule(pods, synth.T0)
            ref = (c0, s0, o.last_device_allocations.copy())
        assert np.array_equal(c1, ref[0]), (b, np.argwhere(c1 != ref[0])[:5].ravel().tolist())
        assert np.array_equal(s1, ref[1]), b
        assert np.array_equal(ev.last_device_allocations, ref[2]), b
        assert ev.check_records(synth.T0) == 0
        if b == 64 and strategy == abi.STRATEGY_MOST_ALLOCATED:
            assert ev.ds_cuts() > 0  # the max moves under MostAllocated: the cut path ran


def test_deviceshare_sharded_loopback(gpu):
    ev, o = ds_both(2000, 86)
    pods = synth.make_ds_pods(300, synth.BASE_SEED + 87)
    ev.shard_init(0, 3, None)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)


def test_deviceshare_rccl_single_rank(gpu):
    from koordinator_amd.evaluator import comm_unique_id
    ev, o = ds_both(1200, 88)
    pods = synth.make_ds_pods(200, synth.BASE_SEED + 89)
    ev.shard_init(0, 1, comm_unique_id())
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)


def test_deviceshare_cache_delete_and_unhealthy(gpu):
    """Dropping a node's device cache makes DeviceShare pass with score 0 there; unhealthy GPUs have
    an empty total (device_cache.go:558-560)."""
    ev, o = ds_both(300, 90)
    for h in (ev, o):
        for i in range(0, 300, 7):
            h.delete_devices(i)
    pods = synth.make_ds_pods(40, synth.BASE_SEED + 91)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    for k in ("status", "reason", "ds", "total", "best"):
        assert np.array_equal(a[k], b[k]), k


# ---- NUMA topology policies (non-cpuset pods) ------------------------------------------------------
def numa_both(n_nodes, seed, zone_counts=(1, 2, 4, 8), batch=64, hint_most=False, most=False, status_fraction=0.0,
              policy_weights=(0.1, 0.3, 0.3, 0.3)):
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + seed, amplified_fraction=0.3)
    zs = synth.make_numa(cl, synth.BASE_SEED + seed + 50, zone_counts=zone_counts, status_fraction=status_fraction,
                         policy_weights=policy_weights)
    cfg = synth.config(n_nodes, pod_batch=batch)
    if hint_most:
        cfg.numa.numa_strategy = abi.STRATEGY_MOST_ALLOCATED
    if most:
        cfg.numa.strategy = abi.STRATEGY_MOST_ALLOCATED
    ev, o = Evaluator(cfg), Oracle(cfg, n_nodes)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zs)
    return ev, o


@pytest.mark.parametrize("variant", ["least", "hint-most", "most"])
def test_numa_policy_eval_matrix_parity(gpu, variant):
    """Every policy, 1/2/4/8 zones: FilterByNUMANode, hint generation, merge + admit, allocation by the
    hint and the NUMA-scope score equal the oracle's on every (pod, node)."""
    ev, o = numa_both(400, 91, hint_most=variant == "hint-most", most=variant == "most")
    pods = synth.make_pods(48, synth.BASE_SEED + 92)
    assert_eval_equal(ev.eval(pods, synth.T0), o.eval(pods, synth.T0))


def test_numa_policy_schedule_parity(gpu):
    """Sequential placements with NUMA Reserve: batches re-evaluate nodes whose zones earlier pods of
    the batch allocated; per-pod zone allocations equal the oracle's."""
    ev, o = numa_both(400, 93, zone_counts=(1, 2, 4))
    pods = synth.make_pods(320, synth.BASE_SEED + 94)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5]
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert np.any(ev.last_numa_allocations != 0)
    more = synth.make_pods(32, synth.BASE_SEED + 95)
    assert_eval_equal(ev.eval(more, synth.T0), o.eval(more, synth.T0))
    assert ev.check_records(synth.T0) == 0


def test_numa_policy_sharded_loopback(gpu):
    ev, o = numa_both(1100, 96, zone_counts=(2, 4))
    pods = synth.make_pods(160, synth.BASE_SEED + 97)
    ev.shard_init(0, 3, None)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)


def test_numa_policy_edge_cases(gpu):
    """Hand-built zones: no zones, a single zone (SingleNUMANode -> nil affinity), zones without a
    memory key, exhausted zones, amplified cpu with NRT ratios, amplification errors; pods asking for
    cpu only, memory only, both, or nothing NUMA-relevant."""
    Z = model.make_zones
    layouts = [
        None,
        Z([{"id": 0, "cpu": "16", "memory": "64Gi"}]),
        Z([{"id": 0, "cpu": "8", "memory": "32Gi"}, {"id": 1, "cpu": "8", "memory": "32Gi"}]),
        Z([{"id": 0, "cpu": "8", "memory": "32Gi", "allocated": {"cpu": "8", "memory": "1Gi"}},
           {"id": 1, "cpu": "8", "memory": "32Gi", "allocated": {"cpu": "1", "memory": "32Gi"}}]),
        Z([{"id": 0, "cpu": "4"}, {"id": 1, "cpu": "4", "memory": "16Gi"}, {"id": 3, "cpu": "4", "memory": "16Gi"}]),
        Z([{"id": k, "cpu": "2", "memory": "8Gi", "allocated": {"cpu": str(k % 3), "memory": f"{k}Gi"}}
           for k in range(8)]),
        Z([{"id": 2, "cpu": "6", "memory": "6Gi", "allocated": {"cpu": "2"}, "cpuset_cpus": 1},
           {"id": 5, "cpu": "6", "memory": "6Gi"}]),
    ]
    nodes, zones = [], []
    for pol in range(4):
        for li, lay in enumerate(layouts):
            for amp in ("none", "annot", "nrt", "error"):
                n = model.make_node(allocatable={"cpu": "16", "memory": "64Gi"}, requested={"cpu": "2"},
                                    amplification_ratio=1.5 if amp == "annot" else None,
                                    nrt_amplification_ratio=1.5 if amp == "nrt" else None,
                                    amplification_error=amp == "error",
                                    cpuset_allocated_cpus=1 if li == 6 and amp != "none" else 0)
                n.numa_topology_policy = pol
                nodes.append(n)
                zones.append(lay)
    cfg = abi.default_config(len(nodes))
    cfg.numa.weights[:] = [1, 1]
    ev, o = Evaluator(cfg), Oracle(cfg, len(nodes))
    for h in (ev, o):
        for i, (n, z) in enumerate(zip(nodes, zones)):
            h.upsert_node(i, n)
            if z is not None:
                h.set_numa(i, z)
    reqs = [{"cpu": "1"}, {"cpu": "3"}, {"cpu": "9"}, {"cpu": "17"}, {"memory": "8Gi"}, {"memory": "40Gi"},
            {"cpu": "2", "memory": "20Gi"}, {"cpu": "7", "memory": "2Gi"}, {"cpu": "12", "memory": "48Gi"},
            {}, {"kubernetes.io/batch-cpu": "1000"}]
    pods = [model.make_pod(name=f"p{i}", requests=r) for i, r in enumerate(reqs)]
    a, b = ev.eval(pods, cases.NOW), o.eval(pods, cases.NOW)
    assert_eval_equal(a, b)
    for code in (abi.CODE_UNSCHEDULABLE, abi.CODE_UNSCHEDULABLE_AND_UNRESOLVABLE):
        assert np.any(a["status"] == code)
    for reason in (abi.REASON_NUMA_MISSING_RESOURCES, abi.REASON_NUMA_HINT_UNALIGNED,
                   abi.REASON_NUMA_INSUFFICIENT_RESOURCES):
        assert np.any(a["reason"] == reason), reason
    # and sequentially: the zones fill up as the queue is placed
    queue = [model.make_pod(name=f"q{i}", requests=r) for i, r in enumerate(reqs * 4)]
    c1, s1 = ev.schedule(queue, cases.NOW)
    c0, s0 = o.schedule(queue, cases.NOW)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    assert_eval_equal(ev.eval(pods, cases.NOW), o.eval(pods, cases.NOW))


NUMA_VEC = [c for c in cases.load("numa_policy.json") if c["op"] in ("affinity", "hints")
            or c["name"] == "allocate with CPU Share and allocated and amplified ratios"]


@pytest.mark.parametrize("case", NUMA_VEC, ids=[f'{c["op"]}: {c["name"]}' for c in NUMA_VEC])
def test_golden_numa_policy_path(gpu, case):
    """The reference's NUMA vectors observable through ke_schedule: the zones the pod's allocation
    lands on (= the stored affinity) and the amounts, against the expectation and the oracle."""
    ev, o = Evaluator(cases.numa_case_cfg(case)), Oracle(cases.numa_case_cfg(case), 1)
    pod = cases.setup_numa_case(ev, case)
    cases.setup_numa_case(o, case)
    c1, s1 = ev.schedule([pod], cases.NOW)
    c0, s0 = o.schedule([pod], cases.NOW)
    assert c1[0] == 0 and (c1[0], s1[0]) == (c0[0], s0[0])
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
    alloc = ev.last_numa_allocations[0].reshape(8, 2)
    zones = [z for z in range(8) if alloc[z].any()]
    if case["op"] == "affinity":
        assert zones == case["want"]["bits"], case["source"]
    elif case["op"] == "hints":  # BestEffort admits the single preferred hint
        assert zones == case["want"]["hints"]["cpu"][0][0], case["source"]
    else:  # the single-zone hints do not fit: the merged hint is {0,1}, split 1.75 / 1.75
        got = {str(z): alloc[z].tolist() for z in zones}
        assert got == {z: cases.quantity_vec(rl) for z, rl in case["want"]["alloc"].items()}, case["source"]


@pytest.mark.parametrize("nodes", ["node-policies", "no-node-policies"])
def test_numa_pod_policy_eval_parity(gpu, nodes):
    """Pods with their own numa-topology-spec: conflicts with the node's policy, the merged policy,
    SingleNUMANodeExclusive against zones already single / shared."""
    w = (0.1, 0.3, 0.3, 0.3) if nodes == "node-policies" else (1, 0, 0, 0)
    ev, o = numa_both(400, 98, status_fraction=0.4, policy_weights=w)
    pods = synth.make_numa_pods(48, synth.BASE_SEED + 99, policy_fraction=0.6)
    a, b = ev.eval(pods, synth.T0), o.eval(pods, synth.T0)
    assert_eval_equal(a, b)
    if nodes == "node-policies":
        assert np.any(a["reason"] == abi.REASON_NUMA_POLICY_CONFLICT)


def test_numa_pod_policy_schedule_parity(gpu):
    ev, o = numa_both(300, 100, zone_counts=(1, 2, 4), status_fraction=0.4)
    pods = synth.make_numa_pods(256, synth.BASE_SEED + 101, policy_fraction=0.5)
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5]
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
