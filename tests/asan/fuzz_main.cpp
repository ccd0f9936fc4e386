// TEST INFRASTRUCTURE ONLY — bounded fuzzing of the host code under AddressSanitizer + UBSan
// (`make -C koordinator_amd/csrc asan`, driven by tests/test_asan.py).
//
// The wire-format decoders parse apiserver JSON (untrusted input): every seed document of the corpus is mutated
// (byte flips, cuts, duplicated ranges, JSON fragments, numbers at the int64 / float64 edges, splices of two
// seeds) and fed to every decoder, whatever its kind.  What decodes is then pushed through the informer-facing
// entry points of a context (node / NodeMetric / device / NUMA / CPU ingestion, assign, release, the host row
// derivation).  Any memory error, overflow or other undefined behaviour aborts the run (-fno-sanitize-recover).
//
// usage: ke_asan_fuzz <corpus: one "kind<TAB>json" per line> <iterations> <seed>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "../../include/koord_eval.h"

namespace {

const char* const FRAGMENTS[] = {"{", "}", "[", "]", "\"", ":", ",", "null", "true", "false", "-0", "1e309", "-1e309",
                                 "9223372036854775807", "9223372036854775808", "-9223372036854775809", "0.000000001",
                                 "1.5Gi", "1Ei", "8Ei", "100m", "1n", "1e-9", "\"\\u0000\"", "\"\\ud800\"", "\"\\",
                                 "\"cpu\"", "\"memory\"", "\"nvidia.com/gpu\"", "\"koordinator.sh/gpu-core\"",
                                 "\"annotations\"", "\"labels\"", "\"resources\"", "\"requests\"", "{\"cpu\":\"1\"}",
                                 "[[[[[[[[", "]]]]]]]]", "\"2023-11-14T22:13:20Z\"", "\"2023-13-45T99:99:99Z\"",
                                 "\"5m\"", "\"-5m\"", "\"9999999h\"", "0x10", "+1", ".5", "1.", "00", "\xff", "\x00"};

std::string mutate(std::mt19937_64& rng, const std::string& base, const std::vector<std::string>& corpus) {
  std::string s = base;
  const int n = 1 + (int)(rng() % 6);
  for (int k = 0; k < n; k++) {
    const size_t len = s.size();
    switch (rng() % 7) {
      case 0:  // flip a byte
        if (len) s[rng() % len] ^= (char)(1u << (rng() % 8));
        break;
      case 1: {  // cut a range
        if (!len) break;
        const size_t a = rng() % len, b = a + rng() % (len - a + 1);
        s.erase(a, b - a);
        break;
      }
      case 2: {  // duplicate a range
        if (!len) break;
        const size_t a = rng() % len, b = a + rng() % std::min<size_t>(len - a + 1, 256);
        s.insert(rng() % (len + 1), s.substr(a, b - a));
        break;
      }
      case 3: {  // insert a JSON fragment
        const char* f = FRAGMENTS[rng() % (sizeof(FRAGMENTS) / sizeof(FRAGMENTS[0]))];
        s.insert(rng() % (len + 1), f, std::strlen(f) ? std::strlen(f) : 1);
        break;
      }
      case 4: {  // replace a number-ish run with an edge value
        if (!len) break;
        const size_t a = rng() % len;
        size_t b = a;
        while (b < len && ((s[b] >= '0' && s[b] <= '9') || s[b] == '.' || s[b] == '-')) b++;
        const char* f = FRAGMENTS[11 + rng() % 9];
        s.replace(a, b - a, f);
        break;
      }
      case 5: {  // splice with another seed
        const std::string& o = corpus[rng() % corpus.size()];
        if (o.empty() || !len) break;
        const size_t a = rng() % len, b = rng() % o.size();
        s = s.substr(0, a) + o.substr(b);
        break;
      }
      default:  // truncate
        if (len) s.resize(rng() % len);
    }
  }
  return s;
}

ke_pod_allocation random_alloc(std::mt19937_64& rng, int32_t node) {
  ke_pod_allocation a{};
  a.node = node;
  a.quota_assigned = (uint8_t)(rng() & 1);
  for (int w = 0; w < 4; w++) a.cpuset[w] = rng() & rng();
  for (int w = 0; w < KE_MAX_NUMA * KE_NRES; w++) a.numa[w] = (int64_t)(rng() % 4) * (int64_t)(rng() % (1ull << 40));
  a.device_minors = rng() & rng() & 0xFFFFFFFFFFFFull;
  return a;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s corpus iterations seed\n", argv[0]);
    return 2;
  }
  std::vector<std::string> kinds, docs;
  std::ifstream in(argv[1]);
  for (std::string line; std::getline(in, line);) {
    const size_t t = line.find('\t');
    if (t == std::string::npos) continue;
    kinds.push_back(line.substr(0, t));
    docs.push_back(line.substr(t + 1));
  }
  if (docs.empty()) {
    std::fprintf(stderr, "empty corpus\n");
    return 2;
  }
  const long iters = std::atol(argv[2]);
  std::mt19937_64 rng((uint64_t)std::atoll(argv[3]));
  // a context without a device: ingestion, release and the host derivation only
  ke_config cfg{};
  cfg.abi_version = KE_ABI_VERSION;
  cfg.weight_loadaware = cfg.weight_numa = cfg.weight_deviceshare = 1;
  cfg.loadaware.node_metric_expiration_seconds = 180;
  for (int r = 0; r < KE_NRES; r++) {
    cfg.loadaware.resource_weights[r] = 1;
    cfg.loadaware.usage_thresholds[r] = r ? 95 : 65;
    cfg.loadaware.prod_usage_thresholds[r] = KE_ABSENT;
    cfg.loadaware.estimated_scaling_factors[r] = r ? 70 : 85;
    cfg.loadaware.agg_usage_thresholds[r] = KE_ABSENT;
    cfg.numa.weights[r] = 1;
  }
  cfg.loadaware.estimated_seconds_after_pod_scheduled = KE_ABSENT;
  cfg.loadaware.estimated_seconds_after_initialized = KE_ABSENT;
  cfg.loadaware.filter_expired_node_metrics = 1;
  for (int i = 0; i < 4; i++) cfg.deviceshare.weights[i] = 1;
  cfg.node_capacity = 64;
  cfg.pod_batch = 64;
  ke_ctx* ctx = nullptr;
  if (ke_create(&cfg, &ctx) != KE_OK) {
    std::fprintf(stderr, "ke_create: %s\n", ke_last_error());
    return 1;
  }
  const char* names[] = {"cpu", "memory", "kubernetes.io/batch-cpu", "nvidia.com/gpu", "ephemeral-storage"};
  long decoded = 0, rejected = 0;
  std::vector<ke_pod> pods;
  for (long it = 0; it < iters; it++) {
    const size_t pick = rng() % docs.size();
    const std::string s = it % 8 == 0 ? docs[pick] : mutate(rng, docs[pick], docs);
    const int32_t node = (int32_t)(rng() % 64);
    ke_node n{};
    int rc = ke_decode_node(s.data(), (int64_t)s.size(), &n);
    if (rc == KE_OK && ke_node_upsert(ctx, node, &n) == KE_OK) decoded++;
    else rejected++;
    ke_node_metric nm{};
    ke_pod_metric pm[8];
    ke_aggregated_usage ag[4];
    int32_t npm = 0, nag = 0;
    if (ke_decode_node_metric(s.data(), (int64_t)s.size(), &nm, 8, pm, &npm, 4, ag, &nag) == KE_OK) {
      decoded++;
      ke_nodemetric_upsert(ctx, node, &nm, npm < 8 ? npm : 8, pm, nag < 4 ? nag : 4, ag);
    }
    ke_pod p{};
    if (ke_decode_pod(s.data(), (int64_t)s.size(), 5, names, &p) == KE_OK) {
      decoded++;
      if (ke_pod_assign(ctx, node, &p, 1700000000000000000LL) == KE_OK) pods.push_back(p);
      int64_t est[KE_NRES];
      ke_estimate_pod(ctx, &p, est);
    }
    ke_device dev[48];
    ke_gpu_partition parts[KE_MAX_GPU_PARTITIONS];
    int32_t nd = 0, np = 0, ht = 0, hon = 0;
    if (ke_decode_device(s.data(), (int64_t)s.size(), 48, dev, &nd, KE_MAX_GPU_PARTITIONS, parts, &np, &ht, &hon) == KE_OK) {
      decoded++;
      ke_node_devices_set(ctx, node, nd < 48 ? nd : 48, dev);
      ke_node_gpu_partitions(ctx, node, ht, hon, np < KE_MAX_GPU_PARTITIONS ? np : KE_MAX_GPU_PARTITIONS, parts);
    }
    ke_numa_zone zones[KE_MAX_NUMA];
    ke_cpu cpus[KE_MAX_CPUS];
    int32_t nz = 0, nc = 0;
    ke_node nn = n;
    if (ke_decode_nrt(s.data(), (int64_t)s.size(), &nn, KE_MAX_NUMA, zones, &nz, KE_MAX_CPUS, cpus, &nc) == KE_OK) {
      decoded++;
      ke_node_numa_set(ctx, node, nz < KE_MAX_NUMA ? nz : KE_MAX_NUMA, zones);
      ke_node_cpus_set(ctx, node, nc < KE_MAX_CPUS ? nc : KE_MAX_CPUS, cpus, 1 + (int32_t)(rng() % 3));
    }
    int64_t v, mv;
    ke_quantity_parse(s.c_str(), &v, &mv);
    if (!pods.empty() && rng() % 4 == 0) {  // release a recorded pod with a random record
      const ke_pod& q = pods[rng() % pods.size()];
      const ke_pod_allocation a = random_alloc(rng, rng() % 8 ? node : -1);
      ke_pod_release(ctx, &q, &a, (int32_t)(rng() % 2));
    }
    if (it % 64 == 63) {  // the host folding of every node (no device rows)
      std::vector<unsigned char> rows((size_t)ke_num_nodes(ctx) * 152 + 1);
      ke_debug_rows(ctx, ke_num_nodes(ctx), 1700000000000000000LL + it, nullptr, rows.data());
      ke_node st{};
      ke_debug_node_state(ctx, node, &st, 0, nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr);
      if (pods.size() > 4096) pods.clear();
    }
  }
  ke_destroy(ctx);
  std::printf("fuzz ok: %ld iterations, %ld decoded objects, %ld rejected node documents\n", iters, decoded, rejected);
  return 0;
}
