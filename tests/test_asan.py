"""Sanitizer build of the host code (-fsanitize=address on host code).

`make -C koordinator_amd/csrc asan` builds ke_host / ke_capi / ke_decode / ke_json with AddressSanitizer + UBSan
(no recovery) into tests/asan/fuzz_main.cpp's driver, the device entry points answered "no device"
(tests/asan/no_device.cpp).  The driver mutates a corpus of apiserver documents (the decode fixtures of
tests/golden/decode.json and generated Node / Pod / NodeMetric / Device / NodeResourceTopology objects) and
feeds every mutation to every decoder and what decodes to the informer-facing ingestion, assign and release
entry points.  Bounded: a fixed iteration count and seed, a few seconds of CPU."""
import json
import os
import subprocess

import numpy as np
import pytest

import cases
import test_decode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "koordinator_amd", "csrc")
BIN = os.path.join(CSRC, "build_asan", "ke_asan_fuzz")


def corpus_docs():
    docs = []
    for c in cases.load("decode.json"):
        docs.append((c["kind"], c["object"]))
    rng = np.random.default_rng(5)
    for i in range(40):
        doc, _ = test_decode.random_pod(rng, i)
        docs.append(("pod", doc))
    docs.append(("node", test_decode.node_doc({"cpu": "32", "memory": "128Gi"}, {
        "node.koordinator.sh/raw-allocatable": '{"cpu":"48","memory":"256Gi"}',
        "node.koordinator.sh/resource-amplification-ratio": '{"cpu":1.5}',
        "scheduling.koordinator.sh/usage-thresholds": json.dumps({"usageThresholds": {"cpu": 60}, "aggregated": {
            "usageThresholds": {"cpu": 70}, "usageAggregationType": "p95", "usageAggregatedDuration": "5m"}})},
        {"node.koordinator.sh/numa-topology-policy": "BestEffort"})))
    docs.append(("nodemetric", {"metadata": {"name": "n"}, "spec": {"metricCollectPolicy": {"reportIntervalSeconds": 60}},
                                "status": {"updateTime": "2023-11-14T22:13:20Z", "nodeMetric": {
                                    "nodeUsage": {"resources": {"cpu": "4", "memory": "8Gi"}},
                                    "aggregatedNodeUsages": [{"duration": "5m", "usage": {
                                        "p95": {"resources": {"cpu": "6", "memory": "9Gi"}}}}]},
                                    "podsMetric": [{"namespace": "ns", "name": "p1", "priority": "koord-prod",
                                                    "podUsage": {"resources": {"cpu": "1", "memory": "1Gi"}}}]}}))
    gpu = {"koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory": "80Gi", "koordinator.sh/gpu-memory-ratio": "100"}
    docs.append(("device", {"metadata": {"name": "n", "labels": {"node.koordinator.sh/gpu-partition-policy": "Honor"},
                                         "annotations": {"scheduling.koordinator.sh/gpu-partitions": json.dumps(
                                             {"1": [{"minors": [0], "allocationScore": 1}], "2": [{"minors": [0, 1]}]})}},
                            "spec": {"devices": [{"type": "gpu", "minor": m, "health": True, "resources": gpu,
                                                  "topology": {"nodeID": m // 2, "pcieID": str(m)}} for m in range(4)]
                                     + [{"type": "rdma", "minor": 0, "health": True,
                                         "resources": {"koordinator.sh/rdma": "100"}}]}}))
    return docs


@pytest.fixture(scope="module")
def fuzz_bin():
    r = subprocess.run(["make", "-C", CSRC, "-s", "asan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return BIN


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_decoders_and_ingestion_under_asan(fuzz_bin, tmp_path, seed):
    corpus = tmp_path / "corpus.txt"
    with open(corpus, "w") as f:
        for kind, doc in corpus_docs():
            f.write(kind + "\t" + json.dumps(doc) + "\n")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([fuzz_bin, str(corpus), "20000", str(seed)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-4000:])
    assert "fuzz ok" in r.stdout
