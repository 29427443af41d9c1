// Native launch profiler (see prof.h).
//
// Weighted sampling: launches whose algorithmic work is at or above always_threshold(kind) are
// always timed (weight 1); smaller ones are timed one in g_every (hashed, weight g_every). The
// read-out is a Horvitz-Thompson estimate: launches = sum w, work = sum w*work, ms = sum w*t.
// The large launches carry most of the time, so the estimate's variance comes only from the
// small-launch tail.
#include <atomic>
#include <mutex>
#include <vector>

#include "common.h"
#include "prof.h"
#include "../../include/rdeic_hip.h"

std::atomic<long long> g_launch_counts[RDEIC_COUNT_KINDS];

void rdeic_count_launch(int kind) {
  if (kind >= 0 && kind < RDEIC_COUNT_KINDS) g_launch_counts[kind].fetch_add(1, std::memory_order_relaxed);
}

extern "C" int64_t rdeic_launch_count(int32_t kind) {
  if (kind < 0 || kind >= RDEIC_COUNT_KINDS) return RDEIC_EINVAL;
  return g_launch_counts[kind].load(std::memory_order_relaxed);
}

extern "C" int rdeic_launch_count_reset(void) {
  for (auto& c : g_launch_counts) c.store(0, std::memory_order_relaxed);
  return RDEIC_OK;
}

namespace {
struct Slot { hipEvent_t a = nullptr, b = nullptr; int kind = -1; double work = 0.0; double weight = 1.0; long long key = 0; };
std::vector<Slot> g_slots;
int g_used = 0;
bool g_on = false;
int g_every = 1;     // time one small launch in g_every (per kind)
long g_seen[8] = {};
double g_bytes_n = 0.0, g_bytes = 0.0;  // RDEIC_PROF_CONV_BYTES (every launch while profiling)
std::mutex g_mu;

double always_threshold(int kind) {
  // FLOP for the conv / attention kinds, bytes for the GroupNorm kinds
  return (kind <= RDEIC_PROF_ATTN_SMALL || kind == RDEIC_PROF_GEMM || kind == RDEIC_PROF_ATTN_D512) ? 50e9 : 64e6;
}
}  // namespace

int rdeic_prof_begin(hipStream_t s, int kind, double work) {
  if (!g_on) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on || g_used >= (int)g_slots.size()) return -1;
  double weight = 1.0;
  if (kind >= 0 && kind < 8 && g_every > 1 && work < always_threshold(kind)) {
    // hashed sample (splitmix64 finaliser of the per-kind launch counter): unbiased even when the
    // per-step launch count is a multiple of g_every
    unsigned long long z = (unsigned long long)(g_seen[kind]++) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (z % (unsigned long long)g_every != 0) return -1;
    weight = (double)g_every;
  }
  const int i = g_used++;
  g_slots[i].kind = -1;
  g_slots[i].weight = weight;
  if (hipEventRecord(g_slots[i].a, s) != hipSuccess) return -1;
  return i;
}

void rdeic_prof_add_bytes(double bytes) {
  if (!g_on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on) return;
  g_bytes_n += 1.0;
  g_bytes += bytes;
}

void rdeic_prof_end(int slot, hipStream_t s, int kind, double work, long long key) {
  if (slot < 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (hipEventRecord(g_slots[slot].b, s) != hipSuccess) return;
  g_slots[slot].kind = kind;
  g_slots[slot].work = work;
  g_slots[slot].key = key;
}

extern "C" int rdeic_prof_start(int32_t capacity, int32_t every) {
  if (capacity <= 0 || every <= 0) return RDEIC_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  while ((int)g_slots.size() < capacity) {
    Slot sl;
    // timing-only events: no system-scope fence (no L2 writeback / invalidate per marker, which
    // otherwise costs the profiled run several % of its step time); callers synchronise the
    // device before rdeic_prof_read
    if (hipEventCreateWithFlags(&sl.a, hipEventDisableSystemFence) != hipSuccess ||
        hipEventCreateWithFlags(&sl.b, hipEventDisableSystemFence) != hipSuccess)
      return RDEIC_ELAUNCH;
    g_slots.push_back(sl);
  }
  g_used = 0;
  g_bytes_n = g_bytes = 0.0;
  g_every = every;
  for (long& c : g_seen) c = 0;
  g_on = true;
  return RDEIC_OK;
}

extern "C" int rdeic_prof_stop(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = false;
  return g_used;
}

extern "C" int rdeic_prof_read(int32_t kind, int64_t* launches, double* work, double* ms) {
  if (!launches || !work || !ms) return RDEIC_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  if (kind == RDEIC_PROF_CONV_BYTES) {
    *launches = (int64_t)(g_bytes_n + 0.5); *work = g_bytes; *ms = 0.0;
    return RDEIC_OK;
  }
  double n = 0.0, w = 0.0, t_ms = 0.0;
  for (int i = 0; i < g_used; ++i) {
    const Slot& sl = g_slots[i];
    if (sl.kind != kind) continue;
    if (hipEventSynchronize(sl.b) != hipSuccess) return RDEIC_ELAUNCH;
    float t = 0.f;
    if (hipEventElapsedTime(&t, sl.a, sl.b) != hipSuccess) return RDEIC_ELAUNCH;
    n += sl.weight; w += sl.weight * sl.work; t_ms += sl.weight * t;
  }
  *launches = (int64_t)(n + 0.5); *work = w; *ms = t_ms;
  return RDEIC_OK;
}

extern "C" int rdeic_prof_read_keys(int32_t kind, int64_t* keys, int64_t* launches, double* work, double* ms,
                                    int32_t cap) {
  if (!keys || !launches || !work || !ms || cap <= 0) return RDEIC_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<long long> ks;
  std::vector<double> n, w, t;
  for (int i = 0; i < g_used; ++i) {
    const Slot& sl = g_slots[i];
    if (sl.kind != kind) continue;
    if (hipEventSynchronize(sl.b) != hipSuccess) return RDEIC_ELAUNCH;
    float e = 0.f;
    if (hipEventElapsedTime(&e, sl.a, sl.b) != hipSuccess) return RDEIC_ELAUNCH;
    size_t j = 0;
    while (j < ks.size() && ks[j] != sl.key) ++j;
    if (j == ks.size()) { ks.push_back(sl.key); n.push_back(0.0); w.push_back(0.0); t.push_back(0.0); }
    n[j] += sl.weight; w[j] += sl.weight * sl.work; t[j] += sl.weight * e;
  }
  const int m = (int)ks.size() < cap ? (int)ks.size() : cap;
  for (int j = 0; j < m; ++j) {
    keys[j] = ks[j]; launches[j] = (int64_t)(n[j] + 0.5); work[j] = w[j]; ms[j] = t[j];
  }
  return m;
}
