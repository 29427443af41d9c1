// Native launch profiler: HIP events recorded by the launchers themselves, on the stream each
// kernel runs on, into a preallocated ring of event pairs (no allocation, no Python per launch).
// Enabled by rdeic_prof_start(); bench.py reads per-kind totals with rdeic_prof_read() after
// its timed region. Kinds: see include/rdeic_hip.h (RDEIC_PROF_*).
#pragma once
#include <hip/hip_runtime.h>

void rdeic_count_launch(int kind);  // RDEIC_COUNT_* (include/rdeic_hip.h): which kernel family a launcher chose

void rdeic_prof_add_bytes(double bytes);  // RDEIC_PROF_CONV_BYTES accumulator (no-op when profiling is off)
int rdeic_prof_begin(hipStream_t s, int kind, double work);           // slot, or -1 (off / full / not sampled)
void rdeic_prof_end(int slot, hipStream_t s, int kind, double work, long long key = 0);  // no-op for slot < 0

// key: an optional launch-shape tag (rdeic_prof_read_keys aggregates per (kind, key))
struct ProfScope {
  int slot; hipStream_t s; int kind; double work; long long key;
  ProfScope(hipStream_t s_, int kind_, double work_, long long key_ = 0)
      : slot(rdeic_prof_begin(s_, kind_, work_)), s(s_), kind(kind_), work(work_), key(key_) {}
  ~ProfScope() { rdeic_prof_end(slot, s, kind, work, key); }
};
