"""CPU-side sanity of the DeviceShare generator through the oracle (development tool)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from koordinator_amd import synth  # noqa: E402
from oracle.binding import Oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
cl = synth.make_cluster(N, synth.BASE_SEED + 83)
dv = synth.make_devices(N, synth.BASE_SEED + 133)
pods = synth.make_ds_pods(600, synth.BASE_SEED + 84)
o = Oracle(synth.config(N), N)
synth.load_into(o, cl)
synth.load_devices(o, dv)
t = time.time()
c, s = o.schedule(pods, synth.T0)
print(f"{time.time() - t:.1f}s placed {(c >= 0).sum()} / {len(c)}, device allocations {(o.last_device_allocations != 0).sum()}")
