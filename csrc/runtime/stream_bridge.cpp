#include <stdlib.h>

#include <stdexcept>

#include "kernels/launchers.h"
#include "runtime/device_comm.h"

namespace cs {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("StreamBridge: ") + what + ": " + hipGetErrorString(e));
}
constexpr size_t kForkEvents = 64;
}  // namespace

StreamBridge::StreamBridge(unsigned event_flags) {
  mode_ = 2;
  if (const char* e = getenv("CS_COMM_FORK")) mode_ = atoi(e);
  if (mode_ != 0 && mode_ != 2) throw std::runtime_error("CS_COMM_FORK: 0 (HIP events) or 2 (kernel stream links)");
  if (const char* e = getenv("CS_COMM_LINK_TIMEOUT_S")) timeout_s_ = atof(e);
  if (mode_ == 0) {
    fork_events_.resize(kForkEvents);
    for (auto& ev : fork_events_) hip_ok(hipEventCreateWithFlags(&ev, event_flags), "event");
    hip_ok(hipEventCreateWithFlags(&join_event_, event_flags), "event");
  } else {
    void* p = nullptr;
    hip_ok(hipMalloc(&p, 4 * sizeof(unsigned long long)), "hipMalloc(link counters)");
    hip_ok(hipMemset(p, 0, 4 * sizeof(unsigned long long)), "hipMemset(link counters)");
    dev_ = static_cast<unsigned long long*>(p);
    void* h = nullptr;
    hip_ok(hipHostMalloc(&h, sizeof(int), hipHostMallocMapped), "hipHostMalloc(link error word)");
    err_ = static_cast<int*>(h);
    *err_ = 0;
    hip_ok(hipDeviceSynchronize(), "sync");
  }
}

StreamBridge::~StreamBridge() {
  for (auto& ev : fork_events_) hipEventDestroy(ev);
  if (join_event_) hipEventDestroy(join_event_);
  if (dev_) hipFree(dev_);
  if (err_) hipHostFree(err_);
}

void StreamBridge::fork(hipStream_t compute, hipStream_t comm) {
  if (mode_ == 2) {
    hip_ok(cs_link_signal(dev_ + 0, compute), "link signal (fork)");
    hip_ok(cs_link_wait(dev_ + 0, dev_ + 1, err_, timeout_s_, comm), "link wait (fork)");
    return;
  }
  hipEvent_t e = fork_events_[next_fork_++ % fork_events_.size()];
  hip_ok(hipEventRecord(e, compute), "hipEventRecord(fork)");
  hip_ok(hipStreamWaitEvent(comm, e, 0), "hipStreamWaitEvent(fork)");
}

void StreamBridge::join(hipStream_t comm, hipStream_t compute) {
  if (mode_ == 2) {
    hip_ok(cs_link_signal(dev_ + 2, comm), "link signal (join)");
    hip_ok(cs_link_wait(dev_ + 2, dev_ + 3, err_, timeout_s_, compute), "link wait (join)");
    return;
  }
  hip_ok(hipEventRecord(join_event_, comm), "hipEventRecord(join)");
  hip_ok(hipStreamWaitEvent(compute, join_event_, 0), "hipStreamWaitEvent(join)");
}

std::string StreamBridge::error() const {
  if (err_ != nullptr && __atomic_load_n(err_, __ATOMIC_ACQUIRE) != 0)
    return "stream link wait timed out (a fork/join signal never arrived)";
  return std::string();
}

}  // namespace cs
