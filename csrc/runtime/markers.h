// roctx ranges around the native step's phases: a rocprofv3 --marker-trace of
// a training step shows forward / per-bucket backward / communicator join / SGD. The marker
// library (rocprofiler-sdk-roctx, ROCm's) is loaded at first use with dlopen, so the extension
// links no profiler library; without it (or with CS_ROCTX=0) every call is a no-op. The ranges
// bracket the HOST enqueue of each phase (the step never blocks the host); the kernel trace of
// the same run gives the device side. Replaces the reference's only instrument, the
// datetime-based "average time" print (master/part1/part1.py:39-44).
#pragma once
#include <dlfcn.h>
#include <stdlib.h>

namespace cs {

struct Roctx {
  using push_t = int (*)(const char*);
  using pop_t = int (*)();
  push_t push = nullptr;
  pop_t pop = nullptr;
  static const Roctx& get() {
    static const Roctx r = [] {
      Roctx x;
      const char* e = getenv("CS_ROCTX");
      if (e != nullptr && atoi(e) == 0) return x;
      void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
      if (h == nullptr) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
      if (h == nullptr) return x;
      x.push = reinterpret_cast<push_t>(dlsym(h, "roctxRangePushA"));
      x.pop = reinterpret_cast<pop_t>(dlsym(h, "roctxRangePop"));
      if (x.push == nullptr || x.pop == nullptr) x.push = nullptr, x.pop = nullptr;
      return x;
    }();
    return r;
  }
};

// RAII range: Range r("cs.forward");
class Range {
 public:
  explicit Range(const char* name) {
    const Roctx& r = Roctx::get();
    if (r.push != nullptr) {
      r.push(name);
      on_ = true;
    }
  }
  ~Range() { end(); }
  void end() {
    if (on_) Roctx::get().pop();
    on_ = false;
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_ = false;
};

inline bool roctx_available() { return Roctx::get().push != nullptr; }

}  // namespace cs
