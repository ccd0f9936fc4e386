"""ElasticQuota admission on the GPU path: schedules with a quota tree are
bit-exact with the oracle — placements, scores, and every quota's used / non-preemptible used after
the queue — through the batched replay (k_resolve<.., QUOTA>) and the singleton Reserve
(k_cpuset_reserve: DeviceShare pods, config 5)."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, synth
from oracle.binding import Oracle

pytestmark = pytest.mark.gpu


def tight_tree(pods, seed, frac):
    """A 64-leaf tree whose total is `frac` of the queue's requests: runtime, Max and Min all bind."""
    tot_cpu = int(pods["requests"][:, abi.RES_CPU].sum() * frac)
    tot_mem = int(pods["requests"][:, abi.RES_MEMORY].sum() * frac)
    q = synth.make_quota_tree(seed, 64, 8, tot_cpu, tot_mem)
    pods = synth.assign_quotas(pods, q, seed + 1)
    return q, pods, tot_cpu, tot_mem


def check_same(ev, o, n_quotas, pods):
    c1, s1 = ev.schedule(pods, synth.T0)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5]
    assert np.array_equal(s1, s0)
    for i in range(n_quotas):
        a, b = ev.quota_state(i), o.quota_state(i)
        for k in ("limit", "used", "np_used"):
            assert np.array_equal(a[k], b[k]), (i, k, a[k], b[k])
    return c1


@pytest.mark.parametrize("runtime,check_parent", [(True, False), (True, True), (False, True)])
def test_quota_schedule_parity_batched(gpu, runtime, check_parent):
    n = 2000
    cl = synth.make_cluster(n, synth.BASE_SEED + 91)
    pods = synth.make_pods(2500, synth.BASE_SEED + 191)
    q, pods, tc, tm = tight_tree(pods, 301, 0.5)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    args = synth.quota_args(tc, tm, runtime, check_parent)
    for h in (ev, o):
        synth.load_into(h, cl)
        h.quotas_load(args, q)
    c = check_same(ev, o, len(q), pods)
    refused = int(((c < 0) & (pods["quota"] > 0)).sum())
    assert 0 < refused < len(pods)  # the tree binds for some pods and not for all


def test_quota_schedule_parity_deviceshare(gpu):
    """Config 5 shape: DeviceShare pods (singleton batches) and plain pods under one quota tree."""
    n = 1500
    cl = synth.make_cluster(n, synth.BASE_SEED + 93)
    dv = synth.make_devices(n, synth.BASE_SEED + 143)
    pods = synth.make_ds_pods(500, synth.BASE_SEED + 193)
    q, pods, tc, tm = tight_tree(pods, 303, 0.6)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_devices(h, dv)
        h.quotas_load(synth.quota_args(tc, tm), q)
    check_same(ev, o, len(q), pods)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)


def test_quota_used_carries_across_calls(gpu):
    """A second schedule call sees the used of the first (device table kept, not re-uploaded)."""
    n = 600
    cl = synth.make_cluster(n, synth.BASE_SEED + 95)
    pods = synth.make_pods(900, synth.BASE_SEED + 195)
    q, pods, tc, tm = tight_tree(pods, 305, 0.4)
    cfg = synth.config(n, pod_batch=16)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        h.quotas_load(synth.quota_args(tc, tm), q)
    check_same(ev, o, len(q), pods[:450])
    check_same(ev, o, len(q), pods[450:])


@pytest.mark.parametrize("runtime", [True, False])
def test_quota_default_quota_pods(gpu, runtime):
    """Pods of the default quota (limit_is_max) between batched and singleton pods: with runtime quota
    each placed one shrinks the tree total and refreshes every runtime limit (the call is cut after it,
    group_quota_manager.go:268-271); placements and every quota's limit / used equal the oracle's."""
    from test_quota import with_default_quota
    n = 1500
    cl = synth.make_cluster(n, synth.BASE_SEED + 96)
    dv = synth.make_devices(n, synth.BASE_SEED + 146)
    pods = synth.make_ds_pods(900, synth.BASE_SEED + 196, device_fraction=0.2)
    q, pods, tc, tm = tight_tree(pods, 306, 0.5)
    q = with_default_quota(q, tc // 2, tm // 2)
    pods["quota"][3::37] = len(q)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_devices(h, dv)
        h.quotas_load(synth.quota_args(tc, tm, runtime, True), q)
    c = check_same(ev, o, len(q), pods)
    assert ((c >= 0) & (pods["quota"] == len(q))).sum() > 5
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)
    assert len(ev.stats()[1]) > 0
    # a call whose only (or last) pod is a default-quota pod refreshes the runtime total too; the
    # calls after it admit against the refreshed limits
    extra = synth.make_pods(12, synth.BASE_SEED + 197, key_base=9_950_000_000)
    extra["quota"] = pods["quota"][:12]
    extra["quota"][[0, 3, 7, 11]] = len(q)
    placed = 0
    for lo, hi in ((0, 1), (1, 4), (4, 8), (8, 12)):  # alone, then three calls ending in a default-quota pod
        placed += int((check_same(ev, o, len(q), extra[lo:hi]) >= 0).sum())
    assert placed > 0
