"""CPU side of the wire-format ingestion test (tests/wire.py): every generated object decodes through the
C ABI, and the oracle schedules the decoded cluster (the GPU comparison is tests/test_gpu_wire.py)."""
import numpy as np

import wire
from koordinator_amd import synth
from oracle.binding import Oracle

NOW = wire.T0 * 10**9


def test_decoded_cluster_schedules_in_the_oracle(lib):
    n = 60
    objs = wire.make_objects(n, 200, 120, 5)
    o = Oracle(synth.config(n), n)
    pods = wire.ingest([o], objs, NOW)
    assert len(pods) == 120
    c, s = o.schedule(pods, NOW)
    assert int((c >= 0).sum()) > 40
    assert (s[c >= 0] > 0).all()
    # the decoded pods: every class of the generator is present
    assert len(set(pods["priority_class"].tolist())) >= 2 and pods["device_requests"].any()
