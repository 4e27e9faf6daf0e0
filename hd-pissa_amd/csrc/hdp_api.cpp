// Status / error plumbing of the C-ABI (include/hdpissa.h).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "hdp_common.h"

namespace hdp {
static thread_local char g_err[1024] = "";

bool sync_debug() {
  static const bool on = [] {
    const char* e = getenv("HDP_SYNC_DEBUG");
    return e && e[0] == '1';
  }();
  return on;
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
// ---- live kernel timing -----------------------------------------------------------------
static const char* const kKernelNames[K_COUNT] = {
    "merge", "adam", "delta_gemm", "delta_gemm_multiseg", "probe_p1", "probe_p2", "probe_finish", "probe_reduce",
    "probe_sweep_a", "probe_sweep_b", "probe_sweep_c", "svd_gemm", "delta_pack", "fold_bf16"};
struct TimingRec {
  int kid;
  hipEvent_t a, b;
  double bytes, flops;
};
struct TimingAgg {
  int64_t launches = 0;
  double ms = 0.0, bytes = 0.0, flops = 0.0;
};
static std::mutex g_tmu;
static bool g_timing = false;
static std::vector<TimingRec> g_pending;
static std::vector<hipEvent_t> g_pool;
static TimingAgg g_agg[K_COUNT];

bool timing_on() { return g_timing; }

hipEvent_t timing_event() {
  std::lock_guard<std::mutex> lk(g_tmu);
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void timing_record(int kid, hipEvent_t a, hipEvent_t b, double bytes, double flops) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_pending.push_back({kid, a, b, bytes, flops});
}

// fold every pending record into the aggregates (waits for its stop event)
static int timing_drain() {
  std::lock_guard<std::mutex> lk(g_tmu);
  int rc = HDP_OK;
  for (const TimingRec& r : g_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
      set_error("hdp_timing: event query failed");
      rc = HDP_EHIP;
    } else {
      TimingAgg& g = g_agg[r.kid];
      g.launches += 1;
      g.ms += ms;
      g.bytes += r.bytes;
      g.flops += r.flops;
    }
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_pending.clear();
  return rc;
}
}  // namespace hdp

extern "C" int hdp_timing_enable(int on) {
  const int prev = hdp::g_timing ? 1 : 0;
  hdp::g_timing = on != 0;
  return prev;
}

extern "C" int hdp_timing_reset(void) {
  const int rc = hdp::timing_drain();
  std::lock_guard<std::mutex> lk(hdp::g_tmu);
  for (auto& g : hdp::g_agg) g = hdp::TimingAgg{};
  return rc;
}

extern "C" int hdp_timing_kernels(void) { return hdp::K_COUNT; }

extern "C" int hdp_timing_query(int kid, const char** name, int64_t* launches, double* total_ms, double* bytes,
                                double* flops) {
  HDP_CHECK_ARG(kid >= 0 && kid < hdp::K_COUNT, "hdp_timing_query: kernel id %d out of range", kid);
  const int rc = hdp::timing_drain();
  if (rc != HDP_OK) return rc;
  std::lock_guard<std::mutex> lk(hdp::g_tmu);
  const hdp::TimingAgg& g = hdp::g_agg[kid];
  if (name) *name = hdp::kKernelNames[kid];
  if (launches) *launches = g.launches;
  if (total_ms) *total_ms = g.ms;
  if (bytes) *bytes = g.bytes;
  if (flops) *flops = g.flops;
  return HDP_OK;
}

extern "C" int hdp_abi_version(void) { return HDP_ABI_VERSION; }
extern "C" const char* hdp_last_error(void) { return hdp::g_err; }
