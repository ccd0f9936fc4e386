"""Transcription of NUMA topology known-answer tests into tests/golden/numa_policy.json.

Same rules as make_fixtures.py (hand transcription, each case cites its Go test lines; paths relative to
haoyann/koordinator).  Cases:

* topologymanager Policy.Merge cases (frameworkext/topologymanager/policy_test.go): provider hint lists
  -> merged hint (NUMANodeAffinity, Preferred) and admit.  The Go tables leave `Unsatisfied` and `Score`
  unset in their expectations; only the affinity, Preferred and admit are compared.

Hint: [bits or None, preferred].  Provider: None (no hints) | {} (empty map) | {resource: None | [] | [hints]}.

Run:  python tests/golden/make_numa_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
POLICY = "pkg/scheduler/frameworkext/topologymanager/policy_test.go"

ALL = "all"  # NewTestBitMask(numaNodes...)


def H(bits, pref=True):
    return [bits, pref]


# commonPolicyMergeTestCases (policy_test.go:63-346): one expectation for every policy
COMMON = [
    ("Two providers, 1 hint each, same mask, both preferred 1/2", 66, [{"resource1": [H([0])]}, {"resource2": [H([0])]}], [0], True),
    ("Two providers, 1 hint each, same mask, both preferred 2/2", 95, [{"resource1": [H([1])]}, {"resource2": [H([1])]}], [1], True),
    ("Two providers, 1 no hints, 1 single hint preferred 1/2", 124, [None, {"resource": [H([0])]}], [0], True),
    ("Two providers, 1 no hints, 1 single hint preferred 2/2", 144, [None, {"resource": [H([1])]}], [1], True),
    ("Two providers, 1 with 2 hints, 1 with single hint matching 1/2", 164,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0])]}], [0], True),
    ("Two providers, 1 with 2 hints, 1 with single hint matching 2/2", 197,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([1])]}], [1], True),
    ("Two providers, both with 2 hints, matching narrower preferred hint from both", 230,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0]), H([0, 1], False)]}], [0], True),
    ("Ensure less narrow preferred hints are chosen over narrower non-preferred hints", 267,
     [{"resource1": [H([1]), H([0, 1], False)]}, {"resource2": [H([0]), H([1]), H([0, 1], False)]}], [1], True),
    ("Multiple resources, same provider", 308,
     [{"resource1": [H([1]), H([0, 1], False)], "resource2": [H([0]), H([1]), H([0, 1], False)]}], [1], True),
]

# per-policy mergeTestCases: (name, line, providers, expected bits (ALL / None = nil), preferred, admit)
BEST_EFFORT = [
    ("Two providers, 2 hints each, same mask (some with different bits), same preferred", 350,
     [{"resource1": [H([0, 1]), H([0, 2])]}, {"resource2": [H([0, 1]), H([0, 2])]}], [0, 1], True),
    ("NUMATopologyHint not set", 387, [], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map", 395, [{}], ALL, True),
    ("NUMATopologyHintProvider returns -nil map from provider", 407, [{"resource": None}], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map from provider", 421, [{"resource": []}], ALL, False),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil", 435,
     [{"resource": [H(None, True)]}], ALL, True),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil", 455,
     [{"resource": [H(None, False)]}], ALL, False),
    ("Two providers, 1 hint each, no common mask", 475, [{"resource1": [H([0])]}, {"resource2": [H([1])]}], ALL, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2", 505,
     [{"resource1": [H([0])]}, {"resource2": [H([0], False)]}], [0], False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2", 535,
     [{"resource1": [H([1])]}, {"resource2": [H([1], False)]}], [1], False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 1/2", 565,
     [{"resource1": [H([0])]}, {"resource2": [H([0, 1])]}], ALL, False),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching", 595,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0, 1], False)]}], ALL, False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 2/2", 629,
     [{"resource1": [H([1])]}, {"resource2": [H([0, 1])]}], ALL, False),
]
RESTRICTED = [
    ("Two providers, 2 hints each, same mask (some with different bits), same preferred", 664,
     [{"resource1": [H([0, 1]), H([0, 2])]}, {"resource2": [H([0, 1]), H([0, 2])]}], [0, 1], True),
    ("NUMATopologyHint not set", 701, [], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map", 709, [{}], ALL, True),
    ("NUMATopologyHintProvider returns -nil map from provider", 721, [{"resource": None}], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map from provider", 735, [{"resource": []}], ALL, False),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil", 749,
     [{"resource": [H(None, True)]}], ALL, True),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil", 768,
     [{"resource": [H(None, False)]}], ALL, False),
    ("Two providers, 1 hint each, no common mask", 788, [{"resource1": [H([0])]}, {"resource2": [H([1])]}], ALL, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2", 818,
     [{"resource1": [H([0])]}, {"resource2": [H([0], False)]}], [0], False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2", 848,
     [{"resource1": [H([1])]}, {"resource2": [H([1], False)]}], [1], False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 1/2", 878,
     [{"resource1": [H([0])]}, {"resource2": [H([0, 1])]}], [0], False),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching", 909,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0, 1], False)]}], [0], False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 2/2", 944,
     [{"resource1": [H([1])]}, {"resource2": [H([0, 1])]}], [1], False),
]
SINGLE = [
    ("NUMATopologyHint not set", 980, [], None, True),
    ("NUMATopologyHintProvider returns empty non-nil map", 988, [{}], None, True),
    ("NUMATopologyHintProvider returns -nil map from provider", 1000, [{"resource": None}], None, True),
    ("NUMATopologyHintProvider returns empty non-nil map from provider", 1014, [{"resource": []}], None, False),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil", 1028,
     [{"resource": [H(None, True)]}], None, True),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil", 1047,
     [{"resource": [H(None, False)]}], None, False),
    ("Two providers, 1 hint each, no common mask", 1067, [{"resource1": [H([0])]}, {"resource2": [H([1])]}], None, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2", 1097,
     [{"resource1": [H([0])]}, {"resource2": [H([0], False)]}], None, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2", 1127,
     [{"resource1": [H([1])]}, {"resource2": [H([1], False)]}], None, False),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching", 1157,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0, 1], False)]}], None, False),
    ("Single NUMA hint generation", 1191,
     [{"resource1": [H([0, 1])], "resource2": [H([0]), H([1]), H([0, 1], False)]}], None, False),
    ("One no-preference provider", 1225, [{"resource1": [H([0]), H([1]), H([0, 1], False)]}, None], [0], True),
]

cases = []
for policy, numa_nodes, table, src_end in (
        ("BestEffort", [0, 1, 2, 3], BEST_EFFORT, 660),
        ("Restricted", [0, 1, 2, 3], RESTRICTED, 976),
        ("SingleNUMANode", [0, 1], SINGLE, 1256)):
    for name, line, providers, bits, pref in COMMON:
        exp = bits
        if policy == "SingleNUMANode" and bits == numa_nodes:
            exp = None
        cases.append({"name": f"{policy}: {name}", "source": f"{POLICY}:{line}", "op": "merge", "policy": policy,
                      "numa_nodes": numa_nodes, "providers": providers,
                      "want": {"bits": exp, "preferred": pref, "admit": pref or policy == "BestEffort"}})
    for name, line, providers, bits, pref in table:
        exp = numa_nodes if bits == ALL else bits
        admit = True if policy == "BestEffort" else pref
        cases.append({"name": f"{policy}: {name}", "source": f"{POLICY}:{line}", "op": "merge", "policy": policy,
                      "numa_nodes": numa_nodes, "providers": providers,
                      "want": {"bits": exp, "preferred": pref, "admit": admit}})

def main():
    with open(os.path.join(HERE, "numa_policy.json"), "w") as f:
        json.dump({"source": "haoyann/koordinator topologymanager / nodenumaresource tests, transcribed by "
                             "make_numa_fixtures.py", "cases": cases}, f, indent=1)
    print(f"numa_policy.json: {len(cases)} cases")


if __name__ == "__main__":
    main()
