"""Summarise the rocprofv3 PMC passes of tools/gpu_check.sh (FETCH_SIZE / WRITE_SIZE of k_eval_batch per
launch, one pass per counter and shape) into profiles/<round>/pmc_eval_traffic.json, which bench.py
reports as roofline.traffic for the matching workload.

Correction (MI355X_MICROARCH.md, HBM): gfx950 FETCH_SIZE tallies half the bytes of wide coalesced reads;
calibrated here on the 4M-node B=1 pass, whose SoA is read exactly once (raw FETCH = 1/2 x 592 MB)."""
import csv
import glob
import json
import os
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_s1"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01/pmc_eval_traffic.json"
out = {}
for f in sorted(glob.glob(os.path.join(src, "*", "run_counter_collection.csv"))):
    tag = os.path.basename(os.path.dirname(f))
    m = re.match(r"(FETCH_SIZE|WRITE_SIZE)nodes(\d+)pods(\d+)", tag)
    if not m:
        continue
    ctr, nodes, pods = m.group(1), int(m.group(2)), int(m.group(3))
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_eval_batch" in r["Kernel_Name"]]
    if not vals:
        continue
    e = out.setdefault(f"nodes{nodes}pods{pods}", {"nodes": nodes, "pods": pods})
    kb = sum(vals) / len(vals)
    e[ctr.lower() + "_kb_raw"] = kb
    e["launches"] = len(vals)
    if ctr == "FETCH_SIZE":
        e["fetch_bytes"] = kb * 1024 * 2  # gfx950: x2
    else:
        e["write_bytes"] = kb * 1024
for e in out.values():
    if "fetch_bytes" in e and "write_bytes" in e:
        e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
os.makedirs(os.path.dirname(dst), exist_ok=True)
json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({src}), tools/eval_probe.py",
           "shapes": out}, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
