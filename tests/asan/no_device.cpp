// TEST INFRASTRUCTURE ONLY — the sanitizer build of the host code (tests/asan/, `make -C koordinator_amd/csrc asan`).
// The gfx950 kernels are not part of it: this translation unit stands in for ke_kernels.hip's host entry points
// with "no device" answers, so the ASan/UBSan executable exercises the informer-facing host code (ingestion,
// folding, release, the JSON decoders) on the CPU.  The product library never links this file.
#include "../../koordinator_amd/csrc/ke_host.h"

namespace ke {
static int none() { return fail(KE_ERR_NO_DEVICE, "sanitizer build: no device"); }
int device_available() { return 0; }
int device_create(Context*) { return none(); }
void device_destroy(Context*) {}
int device_eval(Context*, int32_t, const ke_pod*, int64_t, uint8_t*, uint8_t*, int16_t*, int16_t*, int16_t*, int16_t*,
                int32_t*) { return none(); }
int device_schedule(Context*, int32_t, const ke_pod*, int64_t, int32_t*, int32_t*) { return none(); }
int device_rsv_result(Context*, int32_t*) { return none(); }
int device_rsv_gate(const Context*) { return 0; }
int device_refresh(Context*, int64_t, bool) { return none(); }
int device_schedule_enqueue(Context*, int32_t, const ke_pod*, int64_t, bool, DevFinish*) { return none(); }
void device_swap_call_buffers(Context*) {}
void device_quiesce(Context*) {}
bool device_refresh_pending(const Context*, int64_t) { return false; }
bool device_async_ok(const Context*, int32_t) { return false; }
int device_rsv_views(Context*, const ke_pod&, int64_t, const std::vector<RsvView>&, std::vector<RsvViewOut>&) {
  return none();
}
int device_ds_views(Context*, const ke_pod&, int64_t, const std::vector<DsView>&, std::vector<DsViewOut>&) {
  return none();
}
int device_numa_views(Context*, const ke_pod&, int64_t, const std::vector<NumaRsvView>&, std::vector<NumaRsvOut>&) {
  return none();
}
int device_quota_sync(Context*) { return KE_OK; }
int device_debug_rows(Context*, int32_t, Row*) { return none(); }
int device_set_profiling(Context*, int32_t) { return none(); }
int device_set_pipeline(Context*, int32_t) { return none(); }
int device_replay_phases(Context*, int, double*) { return none(); }
int device_check_records(Context*, int64_t, int64_t*) { return none(); }
int device_bench_eval(Context*, int32_t, const ke_pod*, int64_t, int32_t, double*) { return none(); }
int device_comm_unique_id(uint8_t*) { return none(); }
int device_shard_init(Context*, int, int, const uint8_t*) { return none(); }
int device_shard_init_host(Context*, int, int, ke_host_collective, void*) { return none(); }
int device_shard_range(Context*, int*, int*) { return none(); }
bool device_sharded(const Context*) { return false; }
}  // namespace ke
