"""ke_schedule_submit / ke_schedule_wait on the GPU: slices submitted one or two ahead of their collection place
exactly as one ke_schedule over the whole queue and as the oracle; an informer event between a submission and its
wait, a slice that cannot run behind another (DeviceShare pods) and out-of-order waits complete the calls in flight
in submission order; the release records follow the collected call."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, KoordEvalError, abi, synth
from oracle.binding import Oracle

pytestmark = pytest.mark.gpu


def _pair(n, seed):
    cl = synth.make_cluster(n, synth.BASE_SEED + seed)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
    return ev, o, cl


@pytest.mark.parametrize("ahead", [1, 2])
def test_submit_ahead_matches_oracle(gpu, ahead):
    ev, o, _ = _pair(6000, 1301)
    pods = synth.make_pods(8 * 700, synth.BASE_SEED + 1302)
    sl = [pods[i * 700:(i + 1) * 700] for i in range(8)]
    tickets, got_c, got_s = [], [], []
    for i in range(8):
        tickets.append(ev.submit(sl[i], synth.T0))
        if len(tickets) > ahead:
            c, s = ev.wait(tickets.pop(0))
            got_c.append(c)
            got_s.append(s)
    while tickets:
        c, s = ev.wait(tickets.pop(0))
        got_c.append(c)
        got_s.append(s)
    c0, s0 = o.schedule(pods, synth.T0)
    assert np.array_equal(np.concatenate(got_c), c0) and np.array_equal(np.concatenate(got_s), s0)
    assert ev.kernel_stats()["pipelined_batches"] > 0
    dev, host = ev.debug_rows(synth.T0)  # (completes nothing: no call in flight)
    assert np.array_equal(dev, host)
    assert ev.check_records(synth.T0) == 0
    ev.close()


def test_events_and_serial_slices_between_submissions(gpu):
    """A pod assignment (informer event) while slices are in flight, a slice with unschedulable pods, and waits
    collected out of order: every call sees the earlier ones (oracle twin)."""
    ev, o, _ = _pair(3000, 1303)
    rng = np.random.default_rng(1304)
    q = [synth.make_pods(600, synth.BASE_SEED + 1305 + i, key_base=5_000_000_000 + i * 10_000) for i in range(4)]
    q[2]["requests"][::7, abi.RES_CPU] = 10 ** 9  # unschedulable pods in the third slice
    c_exp = []
    t0 = ev.submit(q[0], synth.T0)
    t1 = ev.submit(q[1], synth.T0)
    c_exp.append(o.schedule(q[0], synth.T0))
    c_exp.append(o.schedule(q[1], synth.T0))
    # an informer event while two slices are in flight (a pod bound elsewhere): both complete first, then it applies
    node = int(rng.integers(3000))
    other = abi.Pod.from_buffer_copy(synth.make_pods(1, synth.BASE_SEED + 1309, key_base=7_000_000_000)[0].tobytes())
    for h in (ev, o):
        h.assign(node, other, synth.T0)
    t2 = ev.submit(q[2], synth.T0)
    c_exp.append(o.schedule(q[2], synth.T0))
    t3 = ev.submit(q[3], synth.T0)
    c_exp.append(o.schedule(q[3], synth.T0))
    got = {t: ev.wait(t) for t in (t3, t1, t0, t2)}  # out of order
    for t, (c0, s0) in zip((t0, t1, t2, t3), c_exp):
        assert np.array_equal(got[t][0], c0) and np.array_equal(got[t][1], s0)
    # the release records follow the last collected call (t2)
    rec = ev.last_allocations(600)
    assert np.array_equal(rec["node"], got[t2][0])
    with pytest.raises(KoordEvalError) as e:  # collected already
        ev._check(ev.lib.ke_schedule_wait(ev.h, t2, None, None))
    assert e.value.code == abi.ERR_NOT_FOUND
    dev, host = ev.debug_rows(synth.T0)
    assert np.array_equal(dev, host)
    ev.close()


def test_deviceshare_slice_runs_behind_the_calls_in_flight(gpu):
    """A slice with DeviceShare pods is not enqueued behind a call in flight: submit completes the earlier slices,
    runs it at once, and its wait returns the same placements as the oracle."""
    from test_gpu_parity import ds_both
    ev, o = ds_both(1500, 1306, abi.STRATEGY_LEAST_ALLOCATED)
    plain = synth.make_pods(800, synth.BASE_SEED + 1307)
    dsp = synth.make_ds_pods(60, synth.BASE_SEED + 1308, key_base=6_000_000_000)
    tail = synth.make_pods(500, synth.BASE_SEED + 1310, key_base=6_100_000_000)
    t0 = ev.submit(plain, synth.T0)
    t1 = ev.submit(dsp, synth.T0)
    t2 = ev.submit(tail, synth.T0)
    exp = [o.schedule(q, synth.T0) for q in (plain, dsp, tail)]
    for t, (c0, s0) in zip((t0, t1, t2), exp):
        c, s = ev.wait(t)
        assert np.array_equal(c, c0) and np.array_equal(s, s0)
    ev.close()


def _records_equal(a, b):
    for k in ("node", "cpuset", "numa", "device_minors", "vf_rank", "reservation", "quota_assigned"):
        assert np.array_equal(a[k], b[k]), k


def test_wait_switches_every_release_record(gpu):
    """a plain slice A in flight, a DeviceShare slice B that runs at once (its device minors written),
    then wait(A): A's release records carry A's nodes and no device minors of B; an Unreserve of an A pod releases
    only what A reserved; wait(B) then switches to B's records, whose minors equal the oracle's (both twins keep the
    same state throughout: dev rows, records, next queue)."""
    from test_gpu_parity import ds_both
    ev, o = ds_both(1200, 1311, abi.STRATEGY_LEAST_ALLOCATED)
    qa = synth.make_pods(400, synth.BASE_SEED + 1312)
    qb = synth.make_ds_pods(40, synth.BASE_SEED + 1313, key_base=6_200_000_000)
    ta = ev.submit(qa, synth.T0)
    tb = ev.submit(qb, synth.T0)  # completes A's device work, runs B at once
    ca, _ = o.schedule(qa, synth.T0)
    rec_a = o.last_allocations()
    cb, _ = o.schedule(qb, synth.T0)  # (the device ran B at its submission)
    rec_b = o.last_allocations()
    ga, _ = ev.wait(ta)
    assert np.array_equal(ga, ca)
    got_a = ev.last_allocations(len(qa))
    _records_equal(got_a, rec_a)
    assert not got_a["device_minors"].any()
    p = int(np.flatnonzero(ca >= 0)[3])
    ev.unreserve(qa[p], p)  # A's record: the LoadAware / NodeInfo part only, no device minors of B's pod p
    o.release(qa[p], rec_a[p])
    gb, _ = ev.wait(tb)
    assert np.array_equal(gb, cb)
    _records_equal(ev.last_allocations(len(qb)), rec_b)
    assert rec_b["device_minors"].any()
    tail = synth.make_ds_pods(60, synth.BASE_SEED + 1314, key_base=6_300_000_000)
    c1, s1 = ev.schedule(tail, synth.T0)
    c0, s0 = o.schedule(tail, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)
    assert ev.check_records(synth.T0) == 0
    ev.close()
