"""Transcription of the reference's known-answer tests into JSON fixtures (tests/golden/*.json).

The reference is Go and cannot be built or run here (no Go toolchain / module cache),
so its golden vectors are transcribed by hand from the test tables below, each case citing the
file:line of the Go test it restates (paths relative to haoyann/koordinator).  Only data is written:
inputs in Kubernetes-object terms and the expected status / score.

Time convention: every time is an offset in seconds from the instant the plugin method runs
("now" = 0).  time.Now() evaluated while building a Go test table maps to -0.002, an informer
assign during the test run (no PodScheduled condition) to -0.001, preserving the Go ordering.

Run:  python tests/golden/make_fixtures.py   (rewrites the JSON files next to this script)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LA = "pkg/scheduler/plugins/loadaware/load_aware_test.go"
EST = "pkg/scheduler/plugins/loadaware/estimator/default_estimator_test.go"
NUMA_SCORE = "pkg/scheduler/plugins/nodenumaresource/scoring_test.go"
NUMA_PLUGIN = "pkg/scheduler/plugins/nodenumaresource/plugin_test.go"

T_TABLE = -0.002   # time.Now() while building the test table
T_INFORMER = -0.001  # podAssignCache.assign at informer sync (timeNowFn fallback)

NODE_96 = {"allocatable": {"cpu": "96", "memory": "512Gi"}}
PROD_MAX = 9999
MID_MAX = 7999
BATCH_MIN = 5000

UNSCHED = 2
REASON = {
    "expired": 1, "usage_cpu": 2, "usage_memory": 3, "agg_cpu": 4, "agg_memory": 5,
    "numa_insufficient": 16,
}


def nm(usage=None, update=T_TABLE, pods=(), aggregated=(), has_node_metric=True, report=60):
    return {"update_time_s": update, "report_interval_seconds": report, "node_usage": usage,
            "has_node_metric": has_node_metric, "pods": list(pods), "aggregated": list(aggregated)}


def g16_32(name="test-pod-1", **kw):
    """the 16-core / 32Gi guaranteed pod used throughout TestScore"""
    d = {"name": name, "requests": {"cpu": "16", "memory": "32Gi"}, "limits": {"cpu": "16", "memory": "32Gi"}}
    d.update(kw)
    return d


def prod_pod(name, **kw):  # schedulertesting.MakePod().Namespace("default").Name(name).Priority(ProdValueMax)
    d = {"name": name, "priority": PROD_MAX}
    d.update(kw)
    return d


# --------------------------------------------------------------------------------------------------
# LoadAwareScheduling.Filter
# --------------------------------------------------------------------------------------------------
la_filter = []


def lf(name, src, want_code=0, want_reason=0, **kw):
    case = {"name": name, "source": src, "plugin": "loadaware", "op": "filter", "node": NODE_96,
            "args": {}, "node_metric": None, "assigned_pods": [], "pod": {},
            "want": {"code": want_code, "reason": want_reason}}
    case.update(kw)
    la_filter.append(case)


# TestFilterExpiredNodeMetric  load_aware_test.go:149-267 (defaults; node has no allocatable)
EMPTY_NODE = {"allocatable": {}}
lf("expired: healthy nodeMetrics", f"{LA}:156-173", node=EMPTY_NODE, node_metric=nm(update=T_TABLE, has_node_metric=False))
lf("expired: nil updateTime", f"{LA}:175-187", UNSCHED, REASON["expired"], node=EMPTY_NODE,
   node_metric=nm(update=None, has_node_metric=False))
lf("expired: expired updateTime", f"{LA}:189-206", UNSCHED, REASON["expired"], node=EMPTY_NODE,
   node_metric=nm(update=-180 + T_TABLE, has_node_metric=False))

# TestEnableScheduleWhenNodeMetricsExpired  load_aware_test.go:269-426
lf("enable-expired: healthy nodeMetrics", f"{LA}:277-294", node=EMPTY_NODE, node_metric=nm(has_node_metric=False))
lf("enable-expired: enabled, nil updateTime", f"{LA}:296-309", node=EMPTY_NODE,
   args={"enable_schedule_when_node_metrics_expired": True}, node_metric=nm(update=None, has_node_metric=False))
lf("enable-expired: enabled, expired updateTime", f"{LA}:311-329", node=EMPTY_NODE,
   args={"enable_schedule_when_node_metrics_expired": True},
   node_metric=nm(update=-180 + T_TABLE, has_node_metric=False))
lf("enable-expired: disabled, nil updateTime", f"{LA}:331-344", UNSCHED, REASON["expired"], node=EMPTY_NODE,
   args={"enable_schedule_when_node_metrics_expired": False}, node_metric=nm(update=None, has_node_metric=False))
lf("enable-expired: disabled, expired updateTime", f"{LA}:346-364", UNSCHED, REASON["expired"], node=EMPTY_NODE,
   args={"enable_schedule_when_node_metrics_expired": False},
   node_metric=nm(update=-180 + T_TABLE, has_node_metric=False))

# TestFilterUsage  load_aware_test.go:554-1583: FilterExpiredNodeMetrics=false (:1475); `pods` are
# informer pods with PodScheduled at now-10s (:1500-1506); the default test pod is &corev1.Pod{}.
FU = {"filter_expired_node_metrics": False}
SCHED_10S = -10.0


def fu_args(**kw):
    d = dict(FU)
    d.update(kw)
    return d


def fu_pods(*pods):
    return [{"pod": p, "scheduled_at_s": SCHED_10S} for p in pods]


PM_PROD_30_200 = {"name": "prod-pod-1", "priority": "koord-prod", "usage": {"cpu": "30", "memory": "200Gi"}}
PM_PROD_33_300 = {"name": "prod-pod-2", "priority": "koord-prod", "usage": {"cpu": "33", "memory": "300Gi"}}
PM_PROD_30_100 = {"name": "prod-pod-1", "priority": "koord-prod", "usage": {"cpu": "30", "memory": "100Gi"}}
PM_PROD_23_200 = {"name": "prod-pod-2", "priority": "koord-prod", "usage": {"cpu": "23", "memory": "200Gi"}}
PM_NONE_23_200 = {"name": "prod-pod-2", "usage": {"cpu": "23", "memory": "200Gi"}}
P95_5M = {"duration_s": 300, "usage": {"p95": {"cpu": "70", "memory": "256Gi"}}}

lf("usage: normal usage", f"{LA}:571-597", args=fu_args(), node_metric=nm({"cpu": "60", "memory": "256Gi"}))
lf("usage: node missing NodeMetrics", f"{LA}:599-602", args=fu_args())
lf("usage: exceed cpu usage", f"{LA}:604-630", UNSCHED, REASON["usage_cpu"], args=fu_args(),
   node_metric=nm({"cpu": "70", "memory": "256Gi"}))
lf("usage: exceed p95 cpu usage", f"{LA}:632-678", UNSCHED, REASON["agg_cpu"],
   args=fu_args(aggregated={"usage_thresholds": {"cpu": 60}, "usage_aggregation_type": "p95",
                            "usage_aggregated_duration_s": 300}),
   node_metric=nm({"cpu": "30", "memory": "100Gi"}, aggregated=[P95_5M]))
lf("usage: exceed memory usage", f"{LA}:680-706", UNSCHED, REASON["usage_memory"], args=fu_args(),
   node_metric=nm({"cpu": "30", "memory": "500Gi"}))
lf("usage: exceed memory usage by custom usage thresholds", f"{LA}:708-737", UNSCHED, REASON["usage_memory"],
   args=fu_args(), node=dict(NODE_96, custom_usage_thresholds={"memory": 60}),
   node_metric=nm({"cpu": "30", "memory": "316Gi"}))
lf("usage: exceed p95 cpu usage by custom usage", f"{LA}:739-785", UNSCHED, REASON["agg_cpu"], args=fu_args(),
   node=dict(NODE_96, custom_aggregated={"thresholds": {"cpu": 60}, "type": "p95", "duration_s": 300}),
   node_metric=nm({"cpu": "30", "memory": "100Gi"}, aggregated=[P95_5M]))
lf("usage: disable filter exceed memory usage", f"{LA}:787-816", args=fu_args(usage_thresholds={"memory": 0}),
   node_metric=nm({"cpu": "30", "memory": "500Gi"}))
lf("usage: prod usage filter is not enabled by default", f"{LA}:818-876",
   args=fu_args(usage_thresholds={"cpu": 100, "memory": 100}),
   node_metric=nm({"cpu": "63", "memory": "500Gi"}, pods=[PM_PROD_30_200, PM_PROD_33_300]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")))
lf("usage: filter prod cpu usage", f"{LA}:878-941", UNSCHED, REASON["usage_cpu"],
   args=fu_args(usage_thresholds={"cpu": 100, "memory": 100}, prod_usage_thresholds={"cpu": 50, "memory": 100}),
   node_metric=nm({"cpu": "63", "memory": "500Gi"}, pods=[PM_PROD_30_200, PM_PROD_33_300]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")), pod=prod_pod("prod-pod-3"))
lf("usage: filter prod memory usage", f"{LA}:943-1006", UNSCHED, REASON["usage_memory"],
   args=fu_args(usage_thresholds={"cpu": 100, "memory": 100}, prod_usage_thresholds={"cpu": 100, "memory": 50}),
   node_metric=nm({"cpu": "63", "memory": "500Gi"}, pods=[PM_PROD_30_200, PM_PROD_33_300]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")), pod=prod_pod("prod-pod-3"))
lf("usage: filter prod memory usage with custom usage configuration", f"{LA}:1008-1075", UNSCHED,
   REASON["usage_memory"],
   args=fu_args(usage_thresholds={"cpu": 100, "memory": 100}, prod_usage_thresholds={"cpu": 100, "memory": 100}),
   node=dict(NODE_96, custom_prod_usage_thresholds={"cpu": 100, "memory": 50}),
   node_metric=nm({"cpu": "63", "memory": "500Gi"}, pods=[PM_PROD_30_200, PM_PROD_33_300]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")), pod=prod_pod("prod-pod-3"))
lf("usage: filter daemonset pod exceed cpu usage", f"{LA}:1077-1104", args=fu_args(),
   node_metric=nm({"cpu": "70", "memory": "256Gi"}), pod=prod_pod("test-pod", owner_kind="DaemonSet"))
lf("usage: filter prod cpu usage with new pod request configuration", f"{LA}:1106-1169", UNSCHED,
   REASON["usage_cpu"],
   args=fu_args(usage_thresholds={"cpu": 65, "memory": 100}, prod_usage_thresholds={"cpu": 60, "memory": 100}),
   node_metric=nm({"cpu": "53", "memory": "500Gi"}, pods=[PM_PROD_30_100, PM_PROD_23_200]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")),
   pod=prod_pod("prod-pod-3", requests={"cpu": "20", "memory": "100Gi"}))
lf("usage: filter mid cpu usage with new pod request configuration", f"{LA}:1171-1233", UNSCHED,
   REASON["usage_cpu"],
   args=fu_args(usage_thresholds={"cpu": 65, "memory": 100}, prod_usage_thresholds={"cpu": 60, "memory": 100}),
   node_metric=nm({"cpu": "53", "memory": "300Gi"}, pods=[PM_PROD_30_100, PM_NONE_23_200]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")),
   pod={"name": "prod-pod-3", "priority": MID_MAX,
        "requests": {"kubernetes.io/mid-cpu": "12k", "kubernetes.io/mid-memory": "100Gi"}})
lf("usage: filter memory usage with new pod request configuration", f"{LA}:1235-1298", UNSCHED,
   REASON["usage_memory"],
   args=fu_args(usage_thresholds={"cpu": 65, "memory": 85}, prod_usage_thresholds={"cpu": 60, "memory": 80}),
   node_metric=nm({"cpu": "53", "memory": "300Gi"}, pods=[PM_PROD_30_100, PM_PROD_23_200]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")),
   pod=prod_pod("prod-pod-3", requests={"cpu": "1", "memory": "165Gi"}))
lf("usage: filter mid memory usage with new pod request configuration", f"{LA}:1300-1362", UNSCHED,
   REASON["usage_memory"],
   args=fu_args(usage_thresholds={"cpu": 65, "memory": 85}, prod_usage_thresholds={"cpu": 60, "memory": 80}),
   node_metric=nm({"cpu": "53", "memory": "300Gi"}, pods=[PM_PROD_30_100, PM_NONE_23_200]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"), prod_pod("prod-pod-2")),
   pod={"name": "prod-pod-3", "priority": MID_MAX,
        "requests": {"kubernetes.io/mid-cpu": "1k", "kubernetes.io/mid-memory": "200Gi"}})
lf("usage: filter prod memory usage with assignedCache pod", f"{LA}:1364-1416", UNSCHED, REASON["usage_memory"],
   args=fu_args(usage_thresholds={"cpu": 65, "memory": 85}, prod_usage_thresholds={"cpu": 60, "memory": 70}),
   node_metric=nm({"cpu": "53", "memory": "300Gi"}, pods=[PM_PROD_30_100]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"),
                         prod_pod("prod-pod-2", requests={"cpu": "1", "memory": "200Gi"})),
   pod=prod_pod("prod-pod-3", requests={"cpu": "1", "memory": "200Gi"}))
lf("usage: filter mid cpu usage with assignedCache pod", f"{LA}:1418-1470", UNSCHED, REASON["usage_cpu"],
   args=fu_args(usage_thresholds={"cpu": 65, "memory": 85}, prod_usage_thresholds={"cpu": 60, "memory": 70}),
   node_metric=nm({"cpu": "33", "memory": "110Gi"}, pods=[PM_PROD_30_100]),
   assigned_pods=fu_pods(prod_pod("prod-pod-1"),
                         {"name": "mid-pod-2", "priority": MID_MAX,
                          "requests": {"kubernetes.io/mid-cpu": "20k", "kubernetes.io/mid-memory": "200Gi"}}),
   pod={"name": "mid-pod-3", "priority": MID_MAX,
        "requests": {"kubernetes.io/mid-cpu": "20k", "kubernetes.io/mid-memory": "200Gi"}})

# --------------------------------------------------------------------------------------------------
# LoadAwareScheduling.Score  TestScore  load_aware_test.go:1585-2547 (node 96 / 512Gi, :2484-2491)
# --------------------------------------------------------------------------------------------------
la_score = []


def ls(name, src, want, **kw):
    case = {"name": name, "source": src, "plugin": "loadaware", "op": "score", "node": NODE_96,
            "args": {}, "node_metric": None, "assigned_pods": [], "pod": g16_32(), "want": {"score": want}}
    case.update(kw)
    la_score.append(case)


def informer_assigned(*pods):  # created through the clientset, no PodScheduled condition
    return [{"pod": p, "timestamp_s": T_INFORMER} for p in pods]


P95_SCORE = {"score_aggregation_type": "p95", "score_aggregated_duration_s": 300}
ls("score node with expired nodeMetric", f"{LA}:1598-1622", 0, pod={},
   node_metric=nm({}, update=-180 + T_TABLE))
ls("score empty node", f"{LA}:1624-1671", 90, node_metric=nm({}))
ls("score node missing NodeMetrics", f"{LA}:1673-1700", 0)
ls("score load node", f"{LA}:1702-1752", 72, node_metric=nm({"cpu": "32", "memory": "10Gi"}))
ls("score load node with p95", f"{LA}:1754-1827", 72, args={"aggregated": P95_SCORE},
   node_metric=nm({"cpu": "0", "memory": "0Gi"}, aggregated=[
       {"duration_s": 300, "usage": {"p95": {"cpu": "32", "memory": "10Gi"}, "p99": {"cpu": "50", "memory": "70Gi"}}}]))
ls("score load node with p95 but have not reported usage", f"{LA}:1829-1883", 90, args={"aggregated": P95_SCORE},
   node_metric=nm({"cpu": "0", "memory": "0Gi"}))
ls("score load node with p95 but have not reported usage and have assigned pods", f"{LA}:1885-1980", 81,
   args={"aggregated": P95_SCORE},
   assigned_pods=informer_assigned(g16_32("assigned-pod-1")),
   node_metric=nm({"cpu": "0", "memory": "0Gi"},
                  pods=[{"name": "assigned-pod-1", "usage": {"cpu": "1", "memory": "1Gi"}}]))
ls("score load node with just assigned pod", f"{LA}:1982-2061", 63,
   assigned_pods=informer_assigned(g16_32("assigned-pod-1")),
   node_metric=nm({"cpu": "32", "memory": "10Gi"}))
ls("score load node with just assigned pod where after updateTime", f"{LA}:2063-2142", 63,
   assigned_pods=informer_assigned(g16_32("assigned-pod-1")),
   node_metric=nm({"cpu": "32", "memory": "10Gi"}, update=-10 + T_TABLE))
ls("score load node with just assigned pod where before updateTime", f"{LA}:2144-2223", 63,
   assigned_pods=informer_assigned(g16_32("assigned-pod-1")),
   node_metric=nm({"cpu": "32", "memory": "10Gi"}))
ls("score batch Pod", f"{LA}:2225-2273", 90,
   pod={"name": "test-pod-1", "priority": BATCH_MIN,
        "requests": {"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"},
        "limits": {"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"}},
   node_metric=nm({}))
ls("score prod Pod", f"{LA}:2275-2367", 38, args={"score_according_prod_usage": True},
   pod={"name": "prod-pod-1", "priority": PROD_MAX,
        "requests": {"cpu": "16000", "memory": "32Gi"}, "limits": {"cpu": "16000", "memory": "32Gi"}},
   assigned_pods=informer_assigned(g16_32("assign-prod-pod-1", priority=PROD_MAX)),
   node_metric=nm({}, pods=[{"name": "assign-prod-pod-1", "priority": "koord-prod",
                             "usage": {"cpu": "30", "memory": "100Gi"}}]))
ls("score request less than limit", f"{LA}:2369-2416", 90,
   pod={"name": "test-pod-1", "requests": {"cpu": "8", "memory": "16Gi"}, "limits": {"cpu": "16", "memory": "32Gi"}},
   node_metric=nm({}))
ls("score empty pod", f"{LA}:2418-2455", 99, pod={"name": "test-pod-1"}, node_metric=nm({}))

# --------------------------------------------------------------------------------------------------
# DefaultEstimator.EstimatePod  TestDefaultEstimatorEstimatePod  default_estimator_test.go:33-290
# --------------------------------------------------------------------------------------------------
estimator = []


def es(name, src, pod, want, **kw):
    case = {"name": name, "source": src, "plugin": "loadaware", "op": "estimate", "args": {}, "pod": pod,
            "want": {"cpu": want[0], "memory": want[1]}}
    case.update(kw)
    estimator.append(case)


G4_8 = {"requests": {"cpu": "4", "memory": "8Gi"}, "limits": {"cpu": "4", "memory": "8Gi"}}
es("estimate empty pod", f"{EST}:43-58", {"containers": [{"name": "main"}]}, (250, 200 * 1024 * 1024))
es("estimate guaranteed pod", f"{EST}:60-83", G4_8, (3400, 6012954214))
es("estimate burstable pod", f"{EST}:85-108",
   {"requests": {"cpu": "4", "memory": "8Gi"}, "limits": {"cpu": "8", "memory": "8Gi"}}, (6800, 6012954214))
es("estimate guaranteed pod and zoomed cpu factors", f"{EST}:110-136", G4_8, (4000, 6012954214),
   args={"estimated_scaling_factors": {"cpu": 110}})
es("estimate guaranteed pod and zoomed memory factors", f"{EST}:138-164", G4_8, (3400, 8589934592),
   args={"estimated_scaling_factors": {"memory": 110}})
es("estimate Batch pod", f"{EST}:166-196",
   {"labels": {"koordinator.sh/qosClass": "BE"}, "priority": BATCH_MIN,
    "requests": {"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"},
    "limits": {"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"}}, (3400, 6012954214))
es("estimate pod only has request", f"{EST}:198-225",
   {"labels": {"koordinator.sh/qosClass": "LS"}, "priority": PROD_MAX,
    "requests": {"cpu": "4", "memory": "8Gi"}}, (3200, 6871947674),
   args={"estimated_scaling_factors": {"cpu": 80, "memory": 80}})
es("estimate pod with customized factors", f"{EST}:227-258",
   {"labels": {"koordinator.sh/qosClass": "LS"}, "priority": PROD_MAX, "custom_factors": {"cpu": 100},
    "requests": {"cpu": "4", "memory": "8Gi"}}, (4000, 6871947674),
   args={"estimated_scaling_factors": {"cpu": 80, "memory": 80}, "allow_customize_estimation": True})

# --------------------------------------------------------------------------------------------------
# NodeNUMAResource (non-cpuset pods, NUMA policy None)
# --------------------------------------------------------------------------------------------------
numa = []
DEFAULT_RES = {"cpu": 1, "memory": 1}


def make_node_amp(cpu, mem, ratio):
    """plugin_test.go:123-129 makeNode: raw-allocatable = capacity, cpu allocatable amplified"""
    return {"capacity_cpu": cpu, "memory": mem, "amplification_ratio": ratio}


# TestScoreWithAmplifiedCPUs  scoring_test.go:556-833 (non-cpuset requested pods)
numa.append({"name": "ScoringStrategy MostAllocated, non-cpuset pod", "source": f"{NUMA_SCORE}:568-583",
             "plugin": "numa", "op": "score", "numa_args": {"strategy": "MostAllocated", "weights": DEFAULT_RES},
             "pod": {"requests": {"cpu": "8", "memory": "16Gi"}, "priority": PROD_MAX},
             "nodes": [make_node_amp("32", "40Gi", 1.0), make_node_amp("64", "60Gi", 2.0),
                       make_node_amp("32", "40Gi", 2.0)],
             "existing": [], "want": {"scores": [32, 16, 26]}})
numa.append({"name": "ScoringStrategy MostAllocated, non-cpuset pods, and existing cpuset pod on node",
             "source": f"{NUMA_SCORE}:605-627", "plugin": "numa", "op": "score",
             "numa_args": {"strategy": "MostAllocated", "weights": DEFAULT_RES},
             "pod": {"requests": {"cpu": "8", "memory": "16Gi"}, "priority": PROD_MAX},
             "nodes": [make_node_amp("32", "40Gi", 1.0), make_node_amp("64", "60Gi", 2.0)],
             "nrt": [True, True],
             "existing": [{"node": 0, "cpu": "20", "memory": "4Gi", "cpuset": True},
                          {"node": 1, "cpu": "20", "memory": "4Gi", "cpuset": True}],
             "want": {"scores": [68, 35]}})
numa.append({"name": "ScoringStrategy LeastAllocated, no cpuset pod", "source": f"{NUMA_SCORE}:679-697",
             "plugin": "numa", "op": "score", "numa_args": {"strategy": "LeastAllocated", "weights": DEFAULT_RES},
             "pod": {"requests": {"cpu": "8", "memory": "16Gi"}, "priority": PROD_MAX},
             "nodes": [make_node_amp("32", "40Gi", 1.0), make_node_amp("64", "60Gi", 2.0)],
             "existing": [{"node": 0, "cpu": "20", "memory": "4Gi", "cpuset": False},
                          {"node": 1, "cpu": "20", "memory": "4Gi", "cpuset": False}],
             "want": {"scores": [31, 72]}})
numa.append({"name": "ScoringStrategy LeastAllocated, non-cpuset pod with existing cpuset pods",
             "source": f"{NUMA_SCORE}:699-721", "plugin": "numa", "op": "score",
             "numa_args": {"strategy": "LeastAllocated", "weights": DEFAULT_RES},
             "pod": {"requests": {"cpu": "8", "memory": "16Gi"}, "priority": PROD_MAX},
             "nodes": [make_node_amp("32", "40Gi", 1.0), make_node_amp("64", "60Gi", 2.0)],
             "nrt": [True, True],
             "existing": [{"node": 0, "cpu": "20", "memory": "4Gi", "cpuset": True},
                          {"node": 1, "cpu": "20", "memory": "4Gi", "cpuset": True}],
             "want": {"scores": [31, 64]}})

# TestFilterWithAmplifiedCPUs  plugin_test.go:913-1024 (non-cpuset requested pods; node = 32 CPUs, 40Gi)
for name, src, pod_cpu, exist_cpu, exist_cpuset, nrt, ratio, want in [
    ("no resources requested always fits", f"{NUMA_PLUGIN}:924-930", None, "4", False, False, 2.0, 0),
    ("no filtering without node cpu amplification", f"{NUMA_PLUGIN}:931-937", "32", "32", False, False, 1.0, 0),
    ("cpu fits on no NRT node", f"{NUMA_PLUGIN}:938-944", "32", "32", False, False, 2.0, 0),
    ("insufficient cpu", f"{NUMA_PLUGIN}:945-952", "32", "64", False, False, 2.0, UNSCHED),
    ("insufficient cpu with cpuset pod on node", f"{NUMA_PLUGIN}:953-961", "32", "32", True, True, 2.0, UNSCHED),
]:
    numa.append({"name": name, "source": src, "plugin": "numa", "op": "filter",
                 "numa_args": {"strategy": "LeastAllocated", "weights": DEFAULT_RES},
                 "pod": ({"requests": {"cpu": pod_cpu}, "priority": PROD_MAX} if pod_cpu else {}),
                 "nodes": [make_node_amp("32", "40Gi", ratio)], "nrt": [nrt],
                 "existing": [{"node": 0, "cpu": exist_cpu, "cpuset": exist_cpuset}],
                 "want": {"code": want, "reason": REASON["numa_insufficient"] if want else 0}})


def main():
    out = {
        "loadaware_filter.json": la_filter,
        "loadaware_score.json": la_score,
        "estimator.json": estimator,
        "numa.json": numa,
    }
    for fn, cases in out.items():
        with open(os.path.join(HERE, fn), "w") as f:
            json.dump({"generated_by": "tests/golden/make_fixtures.py", "reference": "haoyann/koordinator",
                       "cases": cases}, f, indent=1, sort_keys=True)
        print(f"{fn}: {len(cases)} cases")


if __name__ == "__main__":
    main()
