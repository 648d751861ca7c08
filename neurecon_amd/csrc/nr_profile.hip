// neurecon_amd — opt-in per-kernel timing with HIP events (bench.py roofline numbers).
// Disabled by default; when enabled each library kernel launch is bracketed by two events on its
// own stream, so the measured duration is that kernel's, not the surrounding step's.
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "nr_common.h"

namespace nr {

struct ProfRec {
  const char* name;
  double units;
  hipEvent_t a, b;
  int slot;  // >= 0: device count copied into g_counts[slot] (units = min(units, count * mult))
  int mult;
};
static std::mutex g_mu;
static std::vector<ProfRec> g_recs;
static std::atomic<bool> g_on{false};
static std::string g_prefix;  // record only kernels whose name starts with this (empty: all)
constexpr int kCountSlots = 1 << 16;
static int* g_counts = nullptr;  // device slots for the device-side unit counts of compacted launches
static int g_nslots = 0;

bool prof_on() { return g_on.load(); }

ProfScope::ProfScope(const char* name, double units, hipStream_t st, const int* dev_units, int mult)
    : st_(st), on_(g_on.load()) {
  if (!on_) return;
  {  // the prefix is written by nr_profile_filter under g_mu (possibly from another thread)
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_prefix.empty() && std::string(name).compare(0, g_prefix.size(), g_prefix) != 0) {
      on_ = false;
      return;
    }
  }
  ProfRec r{name, units, nullptr, nullptr, -1, mult};
  // timing-only events: no system-scope fence (its cache writeback / invalidate put ~10 us of idle GPU
  // after every recorded launch); nr_profile_read synchronises the device before reading them
  if (hipEventCreateWithFlags(&r.a, hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(&r.b, hipEventDisableSystemFence) != hipSuccess) {
    on_ = false;
    return;
  }
  (void)hipEventRecord(r.a, st);
  std::lock_guard<std::mutex> lk(g_mu);
  if (dev_units) {
    if (!g_counts) (void)hipMalloc(&g_counts, sizeof(int) * kCountSlots);
    if (g_counts && g_nslots < kCountSlots) {
      r.slot = g_nslots++;
      (void)hipMemcpyAsync(g_counts + r.slot, dev_units, sizeof(int), hipMemcpyDeviceToDevice, st);
    }
  }
  g_recs.push_back(r);
  idx_ = g_recs.size() - 1;
}

ProfScope::~ProfScope() {
  if (!on_) return;
  std::lock_guard<std::mutex> lk(g_mu);
  (void)hipEventRecord(g_recs[idx_].b, st_);
}

}  // namespace nr

using namespace nr;

extern "C" int nr_profile_enable(int on) {
  g_on = on != 0;
  return NR_OK;
}
extern "C" int nr_profile_filter(const char* prefix) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_prefix = prefix ? prefix : "";
  return NR_OK;
}

extern "C" int nr_profile_read(NrKernelStat* out, int max, int* n_out) {
  NR_REQUIRE(n_out, NR_ERR_ARG, "nr_profile_read: null n_out");
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<NrKernelStat> acc;
  std::vector<int> counts(g_nslots > 0 ? g_nslots : 1, 0);
  (void)hipDeviceSynchronize();
  if (g_nslots > 0) {
    (void)hipMemcpy(counts.data(), g_counts, sizeof(int) * g_nslots, hipMemcpyDeviceToHost);
  }
  for (auto& r : g_recs) {
    if (r.slot >= 0) {
      const double dev = (double)counts[r.slot] * r.mult;
      if (dev < r.units) r.units = dev;
    }
    float ms = 0.f;
    if (hipEventSynchronize(r.b) == hipSuccess) (void)hipEventElapsedTime(&ms, r.a, r.b);
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
    NrKernelStat* s = nullptr;
    for (auto& x : acc)
      if (std::string(x.name) == r.name) s = &x;
    if (!s) {
      NrKernelStat z{};
      snprintf(z.name, sizeof(z.name), "%s", r.name);
      acc.push_back(z);
      s = &acc.back();
    }
    s->launches += 1;
    s->ms += ms;
    s->units += r.units;
  }
  g_recs.clear();
  g_nslots = 0;
  int n = 0;
  for (auto& x : acc)
    if (n < max && out) out[n++] = x;
  *n_out = n;
  return NR_OK;
}
