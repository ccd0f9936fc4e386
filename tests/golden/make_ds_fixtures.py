"""Transcription of DeviceShare known-answer tests into tests/golden/deviceshare.json.

Same rules as make_fixtures.py: the reference is Go and cannot run here, so every case
is restated by hand from the Go test table it cites (paths relative to haoyann/koordinator).  Only data
is written: the node device cache (per device instance: total = deviceTotal, used = deviceUsed; the
tables' deviceFree always equals total - used, checked below), the pod's device requests and the
expected status / score / per-instance requests.

Cases that depend on features outside the modelled path (reservations, preemptible devices, Huawei NPU
shared-resource templates, GPU topology trees) are not transcribed; DESIGN.md lists them.

Run:  python tests/golden/make_ds_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SCORING = "pkg/scheduler/plugins/deviceshare/scoring_test.go"
PLUGIN = "pkg/scheduler/plugins/deviceshare/plugin_test.go"

CORE, MEM, RATIO = "koordinator.sh/gpu-core", "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio"
RDMA, FPGA = "koordinator.sh/rdma", "koordinator.sh/fpga"
KGPU, SHARED = "koordinator.sh/gpu", "koordinator.sh/gpu.shared"

UNSCHED, UNRESOLVABLE = 2, 3
R_INVALID, R_GPU, R_RDMA, R_FPGA = 32, 33, 34, 35


def gpu(minor, total, used=None):
    return {"type": "gpu", "minor": minor, "total": total, "used": used or {}}


def dev(t, minor, total, used=None):
    return {"type": t, "minor": minor, "total": total, "used": used or {}}


G16 = {CORE: "100", RATIO: "100", MEM: "16Gi"}  # gpuResources, scoring_test.go:47-51
U25 = {CORE: "25", RATIO: "25", MEM: "4Gi"}
U75 = {CORE: "75", RATIO: "75", MEM: "12Gi"}

cases = []


def score(name, src, devices, requests, want, strategy="LeastAllocated", code=0, reason=0, cache=True):
    cases.append({"name": name, "source": src, "op": "score", "strategy": strategy, "cache": cache,
                  "devices": devices, "pod": {"requests": requests},
                  "want": {"score": want, "code": code, "reason": reason}})


def filt(name, src, devices, requests, code=0, reason=0, cache=True):
    cases.append({"name": name, "source": src, "op": "filter", "cache": cache, "devices": devices,
                  "pod": {"requests": requests}, "want": {"code": code, "reason": reason}})


# ---- DeviceShare.Score: TestScore (scoring_test.go:40-590) -------------------------------------------
score("empty node info", f"{SCORING}:77-83", [], {CORE: "100", RATIO: "100"}, 0, cache=False)
score("no device resources", f"{SCORING}:84-101", [], {CORE: "100", RATIO: "100"}, 0,
      code=UNRESOLVABLE, reason=R_GPU)
score("completely idle node", f"{SCORING}:102-128", [gpu(0, G16)], {CORE: "100", RATIO: "100"}, 50)
score("multiple GPU devices and completely idle", f"{SCORING}:129-166", [gpu(0, G16), gpu(1, G16)],
      {CORE: "50", RATIO: "50"}, 87)
score("remaining device resources 1", f"{SCORING}:167-208", [gpu(0, G16, U25)], {CORE: "50", RATIO: "50"}, 50)
score("remaining device resources 2", f"{SCORING}:209-250", [gpu(0, G16, U25)], {CORE: "50", MEM: "8Gi"}, 50)
score("remaining device resources with MostAllocated strategy 1", f"{SCORING}:251-293", [gpu(0, G16, U25)],
      {CORE: "50", RATIO: "50"}, 50, strategy="MostAllocated")
score("remaining device resources with MostAllocated strategy 2", f"{SCORING}:294-336", [gpu(0, G16, U25)],
      {CORE: "50", MEM: "8Gi"}, 50, strategy="MostAllocated")
score("requested multiple resources on the remaining resources of the node", f"{SCORING}:337-441",
      [gpu(0, {CORE: "1000", RATIO: "1000", MEM: "160Gi"}, U25), dev("rdma", 0, {RDMA: "1000"}, {RDMA: "50"})],
      {CORE: "50", RATIO: "50", RDMA: "25"}, 186)

# ---- resourceAllocationScorer.scoreDevice (scoring_test.go:1252-1327): one instance, total/free ------
for name, src, req, tot, free, strategy, want in [
    ("completely idle", f"{SCORING}:1261-1273", "50", "100", "100", "LeastAllocated", 50),
    ("completely used", f"{SCORING}:1274-1286", "50", "100", "0", "LeastAllocated", 0),
    ("remaining resources", f"{SCORING}:1287-1299", "30", "100", "50", "LeastAllocated", 20),
    ("remaining resources with MostAllocated", f"{SCORING}:1300-1313", "30", "100", "50", "MostAllocated", 80),
]:
    cases.append({"name": name, "source": src, "op": "score_device", "strategy": strategy,
                  "request": {RATIO: req}, "total": {RATIO: tot}, "free": {RATIO: free}, "want": {"score": want}})

# ---- NormalizeScore: TestScoreExtension (scoring_test.go:599-668) --------------------------------------
for name, src, raw, want in [
    ("node score 0", f"{SCORING}:606-620", [0], [0]),
    ("only one node has score", f"{SCORING}:621-635", [10], [100]),
    ("node score exceeded maxScore", f"{SCORING}:636-658", [200, 10], [100, 5]),
]:
    cases.append({"name": name, "source": src, "op": "normalize", "raw": raw, "want": {"scores": want}})

# ---- DeviceShare.Filter: Test_Plugin_Filter (plugin_test.go:1117-2680) ---------------------------------
filt("error missing nodecache", f"{PLUGIN}:1156-1162", [], {CORE: "100", RATIO: "100"}, cache=False)
filt("insufficient device resource 1", f"{PLUGIN}:1163-1181", [], {CORE: "100", RATIO: "100"},
     UNRESOLVABLE, R_GPU)
filt("insufficient device resource 2", f"{PLUGIN}:1182-1245", [gpu(0, G16, U25)], {CORE: "100", RATIO: "100"},
     UNSCHED, R_GPU)
filt("insufficient device resource 3", f"{PLUGIN}:1246-1333", [gpu(0, G16, U25), dev("fpga", 0, {FPGA: "100"})],
     {CORE: "100", RATIO: "100", FPGA: "100"}, UNSCHED, R_GPU)
filt("insufficient device resource 4", f"{PLUGIN}:1334-1426",
     [gpu(0, G16, U25), dev("fpga", 0, {FPGA: "100"}, {FPGA: "50"})],
     {CORE: "100", RATIO: "100", FPGA: "100"}, UNSCHED, R_GPU)
filt("sufficient device resource 1", f"{PLUGIN}:1574-1622", [dev("fpga", 0, {FPGA: "100"})], {FPGA: "100"})
filt("sufficient device resource 2", f"{PLUGIN}:1623-1692",
     [dev("fpga", 0, {FPGA: "100"}, {FPGA: "25"}), dev("fpga", 1, {FPGA: "100"})], {FPGA: "100"})
filt("sufficient device resource 3", f"{PLUGIN}:1693-1769", [dev("fpga", 0, {FPGA: "100"}), gpu(0, G16)],
     {CORE: "100", RATIO: "100"})
filt("sufficient device resource 4", f"{PLUGIN}:1770-1854", [gpu(0, G16, U75), gpu(1, G16)],
     {CORE: "100", RATIO: "100"})
filt("sufficient device resource 5", f"{PLUGIN}:1855-1938", [gpu(0, G16, U75), gpu(1, G16)], {RATIO: "100"})
filt("sufficient device resource 6", f"{PLUGIN}:1939-2002", [gpu(0, G16, U75), gpu(1, G16)], {MEM: "16Gi"})
G80 = {CORE: "100", RATIO: "100", MEM: "80Gi"}
filt("pod stuck when use multi gpu", f"{PLUGIN}:2398-2610", [gpu(m, G80) for m in range(9)],
     {SHARED: "4", MEM: "160G"})

# ---- PreFilter: Test_Plugin_PreFilter (plugin_test.go:497-1110) ---------------------------------------
def pre(name, src, requests, code=0, skip=False, per=None):
    """per: {type: (count, per-instance requests)} — preFilterState.podRequests/gpuRequirements"""
    cases.append({"name": name, "source": src, "op": "prefilter", "pod": {"requests": requests},
                  "want": {"code": code, "skip": skip, "per": per or {}}})


pre("skip non device pod", f"{PLUGIN}:505-514", {}, skip=True)
pre("pod has invalid fpga request", f"{PLUGIN}:515-538", {FPGA: "101"}, code=UNRESOLVABLE)
pre("pod has invalid gpu request 1", f"{PLUGIN}:539-562", {KGPU: "101"}, code=UNRESOLVABLE)
pre("pod has invalid gpu request 2", f"{PLUGIN}:563-586", {CORE: "100"}, code=UNRESOLVABLE)
pre("pod has invalid gpu request 3", f"{PLUGIN}:587-610", {RATIO: "101"}, code=UNRESOLVABLE)
pre("pod has valid gpu request 1", f"{PLUGIN}:663-704", {KGPU: "100"}, per={"gpu": (1, {CORE: "100", RATIO: "100"})})
pre("pod has valid gpu request 2", f"{PLUGIN}:705-744", {RATIO: "100"}, per={"gpu": (1, {RATIO: "100"})})
pre("pod has valid gpu request 3", f"{PLUGIN}:745-784", {MEM: "8Gi"}, per={"gpu": (1, {MEM: "8Gi"})})
pre("pod has valid gpu request 4", f"{PLUGIN}:785-827", {CORE: "100", MEM: "8Gi"},
    per={"gpu": (1, {CORE: "100", MEM: "8Gi"})})
pre("pod has valid gpu request 5", f"{PLUGIN}:828-870", {CORE: "100", RATIO: "100"},
    per={"gpu": (1, {CORE: "100", RATIO: "100"})})
pre("pod has valid fpga request", f"{PLUGIN}:976-1008", {FPGA: "100"}, per={"fpga": (1, {FPGA: "100"})})
pre("pod has valid gpu & rdma request", f"{PLUGIN}:1009-1054", {KGPU: "100", RDMA: "100"},
    per={"gpu": (1, {CORE: "100", RATIO: "100"}), "rdma": (1, {RDMA: "100"})})
pre("skip zero requests", f"{PLUGIN}:1055-1083", {KGPU: "0"}, skip=True)


def check():
    from fractions import Fraction

    def q(v):
        s = str(v)
        for suf, m in (("Gi", 2**30), ("G", 10**9)):
            if s.endswith(suf):
                return Fraction(s[: -len(suf)]) * m
        return Fraction(s)

    for c in cases:
        for d in c.get("devices", []):
            for k, v in d["used"].items():
                assert q(v) <= q(d["total"][k]), (c["name"], d)


def main():
    check()
    with open(os.path.join(HERE, "deviceshare.json"), "w") as f:
        json.dump({"source": "haoyann/koordinator DeviceShare tests, transcribed by make_ds_fixtures.py",
                   "cases": cases}, f, indent=1)
    print(f"deviceshare.json: {len(cases)} cases")


if __name__ == "__main__":
    main()
