#include <stdlib.h>

#include <stdexcept>
#include <vector>

#include "kernels/launchers.h"
#include "runtime/device_comm.h"

namespace cs {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("StreamBridge: ") + what + ": " + hipGetErrorString(e));
}
constexpr size_t kForkEvents = 64;

double g_link_timeout = [] {
  const char* e = getenv("CS_COMM_LINK_TIMEOUT_S");
  return e ? atof(e) : 1800.0;
}();

int* abort_word() {
  static int* w = [] {
    void* h = nullptr;
    hip_ok(hipHostMalloc(&h, sizeof(int), hipHostMallocMapped), "hipHostMalloc(link abort word)");
    *static_cast<int*>(h) = 0;
    return static_cast<int*>(h);
  }();
  return w;
}
}  // namespace

void set_link_timeout(double seconds) {
  if (getenv("CS_COMM_LINK_TIMEOUT_S") != nullptr) return;  // the environment wins
  g_link_timeout = seconds > 0.0 ? seconds : 1800.0;
}
double link_timeout() { return g_link_timeout; }
void abort_links() { __atomic_store_n(abort_word(), 1, __ATOMIC_RELEASE); }
void reset_link_abort() { __atomic_store_n(abort_word(), 0, __ATOMIC_RELEASE); }

StreamLink::StreamLink() {
  (void)abort_word();
  void* p = nullptr;
  hip_ok(hipMalloc(&p, 2 * sizeof(unsigned long long)), "hipMalloc(link counters)");
  hip_ok(hipMemset(p, 0, 2 * sizeof(unsigned long long)), "hipMemset(link counters)");
  dev_ = static_cast<unsigned long long*>(p);
  void* h = nullptr;
  hip_ok(hipHostMalloc(&h, sizeof(int), hipHostMallocMapped), "hipHostMalloc(link error word)");
  err_ = static_cast<int*>(h);
  *err_ = 0;
  hip_ok(hipDeviceSynchronize(), "sync");
}

StreamLink::~StreamLink() {
  if (dev_) hipFree(dev_);
  if (err_) hipHostFree(err_);
}

void StreamLink::signal(hipStream_t producer) {
  hip_ok(cs_link_signal(dev_, producer), "link signal");
  ++pending_;
}

unsigned long long* StreamLink::defer() {
  ++pending_;
  return dev_;
}

void StreamLink::wait(hipStream_t consumer) {
  if (pending_ == 0) return;  // nothing signalled since the last wait
  hip_ok(cs_link_wait(dev_, dev_ + 1, err_, abort_word(), g_link_timeout, consumer, pending_), "link wait");
  pending_ = 0;
}

std::string StreamLink::error() const {
  const int e = err_ != nullptr ? __atomic_load_n(err_, __ATOMIC_ACQUIRE) : 0;
  if (e == 1)
    return "stream link wait timed out after " + std::to_string(g_link_timeout) +
           " s (its signal never arrived; the consumer ran unordered)";
  if (e == 2) return "stream link wait aborted (abort_links)";
  return std::string();
}

namespace {
// a non-blocking stream at the lowest (or highest) priority, bound to a hardware queue by one
// tiny fill (queues are taken when a stream first runs work)
hipStream_t bound_stream(bool high) {
  int least = 0, greatest = 0;
  hip_ok(hipDeviceGetStreamPriorityRange(&least, &greatest), "stream priorities");
  hipStream_t s = nullptr;
  hip_ok(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, high ? greatest : least), "reserved stream");
  void* scratch = nullptr;
  hip_ok(hipMalloc(&scratch, 256), "reserved stream scratch");
  hip_ok(hipMemsetAsync(scratch, 0, 256, s), "bind reserved stream");
  hip_ok(hipStreamSynchronize(s), "bind reserved stream");
  hip_ok(hipFree(scratch), "reserved stream scratch");
  return s;
}
}  // namespace

hipStream_t reserved_comm_stream() {
  static hipStream_t comm = bound_stream(true);
  return comm;
}

hipStream_t reserved_side_stream() {
  static hipStream_t side = bound_stream(false);
  return side;
}

hipStream_t reserved_lag_stream() {
  static hipStream_t lag = bound_stream(false);
  return lag;
}

void reserve_streams() {
  (void)reserved_side_stream();
  (void)reserved_comm_stream();
}

bool streams_share_queue(hipStream_t a, hipStream_t b, double timeout_s) {
  if (a == b) return true;
  void* p = nullptr;
  hip_ok(hipMalloc(&p, 2 * sizeof(unsigned long long)), "hipMalloc(queue probe)");
  void* h = nullptr;
  hip_ok(hipHostMalloc(&h, sizeof(int), hipHostMallocMapped), "hipHostMalloc(queue probe error word)");
  int* err = static_cast<int*>(h);
  *err = 0;
  auto* cnt = static_cast<unsigned long long*>(p);
  hip_ok(hipMemset(cnt, 0, 2 * sizeof(unsigned long long)), "hipMemset(queue probe)");
  hip_ok(hipDeviceSynchronize(), "sync");
  hip_ok(cs_link_wait(cnt, cnt + 1, err, abort_word(), timeout_s, b, 1), "queue probe wait");
  hip_ok(cs_link_signal(cnt, a), "queue probe signal");
  hip_ok(hipStreamSynchronize(b), "queue probe sync");
  hip_ok(hipStreamSynchronize(a), "queue probe sync");
  const bool shared = __atomic_load_n(err, __ATOMIC_ACQUIRE) != 0;
  hipFree(p);
  hipHostFree(h);
  return shared;
}

bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

StreamBridge::StreamBridge(unsigned event_flags) {
  mode_ = 2;
  if (const char* e = getenv("CS_COMM_FORK")) mode_ = atoi(e);
  if (mode_ != 0 && mode_ != 2) throw std::runtime_error("CS_COMM_FORK: 0 (HIP events) or 2 (kernel stream links)");
  // events always exist: a fork/join inside a graph capture must be an event edge (a stream
  // joins a capture only through an event; a link's kernels on a non-capturing stream would run
  // at once instead of being recorded)
  fork_events_.resize(kForkEvents);
  for (auto& ev : fork_events_) hip_ok(hipEventCreateWithFlags(&ev, event_flags), "event");
  hip_ok(hipEventCreateWithFlags(&join_event_, event_flags), "event");
  if (mode_ == 2) {
    fork_link_ = std::make_unique<StreamLink>();
    join_link_ = std::make_unique<StreamLink>();
  }
}

StreamBridge::~StreamBridge() {
  for (auto& ev : fork_events_) hipEventDestroy(ev);
  if (join_event_) hipEventDestroy(join_event_);
}

void StreamBridge::fork(hipStream_t compute, hipStream_t comm) {
  if (mode_ == 2 && !stream_capturing(compute)) {
    fork_link_->signal(compute);
    fork_link_->wait(comm);
    return;
  }
  hipEvent_t e = fork_events_[next_fork_++ % fork_events_.size()];
  hip_ok(hipEventRecord(e, compute), "hipEventRecord(fork)");
  hip_ok(hipStreamWaitEvent(comm, e, 0), "hipStreamWaitEvent(fork)");
}

void StreamBridge::join(hipStream_t comm, hipStream_t compute) {
  if (mode_ == 2 && !stream_capturing(compute)) {
    join_link_->signal(comm);
    join_link_->wait(compute);
    return;
  }
  hip_ok(hipEventRecord(join_event_, comm), "hipEventRecord(join)");
  hip_ok(hipStreamWaitEvent(compute, join_event_, 0), "hipStreamWaitEvent(join)");
}

std::string StreamBridge::error() const {
  if (fork_link_) {
    std::string e = fork_link_->error();
    if (e.empty()) e = join_link_->error();
    return e;
  }
  return std::string();
}

}  // namespace cs
