"""Summarise the rocprofv3 PMC passes of tools/pmc_bench.sh into profiles/<round>/pmc_bench.json.

Per kernel (name up to its template/argument list) and counter: the mean over dispatches of the value each
dispatch reports (rows of one dispatch and counter summed).  Derived per kernel:
  traffic_bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024   (FETCH_SIZE / WRITE_SIZE are KB; gfx950 tallies
                  a wide coalesced read at half its bytes, MI355X_MICROARCH.md "HBM")
  valu_busy     = SQ_ACTIVE_INST_VALU x 4 / SIMDs / (GRBM_GUI_ACTIVE / XCDs)   (share of SIMD cycles issuing
                  VALU; SQ_ACTIVE_INST_VALU counts quad-cycles, GRBM_GUI_ACTIVE sums the 8 XCDs)
  valu_per_wave, salu_per_wave, vmem_per_wave, ...: instructions per wave
  wave_wait_share / wave_issue_stall_share / wave_active_share: SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
                  SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
Usage: python tools/pmc_summary.py gpurun_out/TAG --tag config3_nodes50000_batch64_world1_serial \
           --out profiles/r02/pmc_bench.json [--source "..."]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

SIMDS, XCDS = 256 * 4, 8


def base_name(k):
    k = re.sub(r"^void ", "", k)
    return re.split(r"[<(]", k, maxsplit=1)[0].strip().split("::")[-1]


def read_pass(d):
    """{kernel: {counter: mean per dispatch}}, {kernel: dispatches}"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = base_name(row.get("Kernel_Name", ""))
                key = (k, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    means = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
    counts = {k: max(len(v) for v in cs.values()) for k, cs in agg.items()}
    return means, counts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    kernels = collections.defaultdict(dict)
    dispatches = {}
    for p in sorted(glob.glob(os.path.join(a.root, "*/"))):
        means, counts = read_pass(p)
        for k, cs in means.items():
            kernels[k].update(cs)
            dispatches[k] = max(dispatches.get(k, 0), counts[k])
    out = {}
    for k, c in sorted(kernels.items()):
        e = {"dispatches": dispatches[k], "counters": c}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["fetch_bytes"] = 2 * c["FETCH_SIZE"] * 1024
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
            e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        waves = c.get("SQ_WAVES")
        if waves:
            for name, ctr in (("valu", "SQ_INSTS_VALU"), ("salu", "SQ_INSTS_SALU"), ("branch", "SQ_INSTS_BRANCH"),
                              ("lds", "SQ_INSTS_LDS"), ("smem", "SQ_INSTS_SMEM"), ("vmem_rd", "SQ_INSTS_VMEM_RD"),
                              ("vmem_wr", "SQ_INSTS_VMEM_WR")):
                if ctr in c:
                    e[f"{name}_per_wave"] = c[ctr] / waves
        if "SQ_ACTIVE_INST_VALU" in c and c.get("GRBM_GUI_ACTIVE"):
            e["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / (c["GRBM_GUI_ACTIVE"] / XCDS)
        if c.get("SQ_WAVE_CYCLES"):
            for name, ctr in (("wave_wait_share", "SQ_WAIT_ANY"), ("wave_issue_stall_share", "SQ_WAIT_INST_ANY"),
                              ("wave_active_share", "SQ_ACTIVE_INST_ANY")):
                if ctr in c:
                    e[name] = c[ctr] / c["SQ_WAVE_CYCLES"]
        out[k] = e
    doc = json.load(open(a.out)) if os.path.exists(a.out) else {}
    doc["source"] = a.source or doc.get("source", "")
    doc["formulas"] = __doc__.split("Usage:")[0].strip()
    doc.setdefault("workloads", {})[a.tag] = out
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({k: {x: v for x, v in e.items() if x != "counters"} for k, e in out.items()}, indent=1))


if __name__ == "__main__":
    main()
