// Event-based per-kernel timing on the stream the kernels are launched on (bench roofline numbers).
// Each scope records a HIP event pair; `work` carries the scope's algorithmic FLOPs or bytes so that
// achieved rate = sum(work) / sum(time).  An optional filter restricts recording to one scope name so
// a timed region pays only for the events of the kernel being measured.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

namespace qlx {

struct Profiler {
  struct Acc { double us = 0.0, work = 0.0; unsigned long long launches = 0; };
  struct Rec { const char* name; hipEvent_t a, b; double work; };
  bool enabled = false;
  std::string filter;   // empty = record every scope
  unsigned stride = 1;  // with a filter: record every stride-th launch of that scope (sampling keeps the event cost
                        // of a timed region small)
  unsigned long long seen = 0;
  std::vector<Rec> pending;
  std::vector<hipEvent_t> pool;
  std::map<std::string, Acc> acc;
  std::vector<Rec> open;   // nested scopes (a == nullptr: filtered out)

  hipEvent_t take() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  void begin(const char* name, hipStream_t s, double work) {
    if (!enabled) return;
    if (!filter.empty() && (filter != name || (seen++ % stride) != 0)) { open.push_back({name, nullptr, nullptr, 0.0}); return; }
    hipEvent_t a = take();
    (void)hipEventRecord(a, s);
    open.push_back({name, a, nullptr, work});
  }
  void end(hipStream_t s) {
    if (!enabled || open.empty()) return;
    Rec r = open.back();
    open.pop_back();
    if (!r.a) return;
    r.b = take();
    (void)hipEventRecord(r.b, s);
    pending.push_back(r);
  }
  // Event pair bound to one kernel dispatch (hipExtLaunchKernelGGL start/stop events): no marker packets
  // around the kernel, so the elapsed time is the kernel's own, as a kernel trace reports it.  Both null when
  // the scope is not recorded.
  void ext(const char* name, double work, hipEvent_t* a, hipEvent_t* b) {
    *a = *b = nullptr;
    if (!enabled || (!filter.empty() && filter != name)) return;
    if (!filter.empty() && (seen++ % stride) != 0) return;
    *a = take();
    *b = take();
    pending.push_back({name, *a, *b, work});
  }
  void collect() {   // after the stream is synchronised
    for (auto& r : pending) {
      float ms = 0.0f;
      (void)hipEventSynchronize(r.b);
      (void)hipEventElapsedTime(&ms, r.a, r.b);
      Acc& slot = acc[r.name];
      slot.us += ms * 1000.0;
      slot.work += r.work;
      slot.launches += 1;
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    pending.clear();
  }
  void reset() { collect(); acc.clear(); }
  ~Profiler() {
    for (auto& r : pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto& r : open) if (r.a) (void)hipEventDestroy(r.a);
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

struct ProfScope {
  Profiler* p;
  hipStream_t s;
  ProfScope(Profiler* p_, const char* name, hipStream_t s_, double work = 0.0) : p(p_), s(s_) {
    if (p) p->begin(name, s, work);
  }
  ~ProfScope() { if (p) p->end(s); }
};

}  // namespace qlx
