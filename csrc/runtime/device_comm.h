// Stream-ordered communicator interface the C++ engines drive.
//
// The engine's data-parallel step (VggEngine::step) only needs four things from a
// transport: an all-reduce and a broadcast that run behind a fork from a compute
// stream, a join back into a compute stream, and the rank/world. Three
// implementations share that contract:
//  * RcclComm   — the production data plane: RCCL over xGMI on a dedicated comm stream
//                 (one GPU per rank, rccl_comm.h);
//  * StagedComm — the same collectives through a c10d ProcessGroup (gloo) with host
//                 staging, so the exact C++ step runs with N ranks that share ONE GPU
//                 (RCCL refuses two ranks on one device) and on the 1-GPU test box;
//  * ProbeComm  — world 1, every collective replaced by a delay kernel plus an exact
//                 scramble / unscramble of the buffer on the comm stream: a missing fork
//                 or join in the engine shows up as a bitwise mismatch (ordering test).
// Contract of every collective: with fork = true the comm stream first waits for everything
// already enqueued on `compute` (fork = false: no fork, ordered only behind what the comm
// stream already holds — `compute` may be the null stream, so "no fork" is a flag, never a
// null stream); the collective runs on the comm stream; join(compute) makes `compute` wait
// for everything enqueued on the comm stream so far. Nothing blocks the
// host except where an implementation says so (StagedComm).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <memory>
#include <string>
#include <vector>

namespace cs {

class DeviceComm {
 public:
  virtual ~DeviceComm() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual hipStream_t stream() const = 0;
  virtual const char* kind() const = 0;
  virtual void all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t compute,
                          bool fork) = 0;
  virtual void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t compute, bool fork) = 0;
  virtual void join(hipStream_t compute) = 0;
  // async error polling: "" when healthy
  virtual std::string async_error() { return std::string(); }
  virtual void abort() {}
  // collectives issued so far (tests / fault injection)
  virtual int64_t calls() const { return 0; }
  // the host waits inside a collective for the GPU to reach it (StagedComm's host staging):
  // every stream-link signal must be launched before one is issued
  virtual bool host_blocking() const { return false; }
};

// whether `s` is being captured into a graph (links fall back to events there)
bool stream_capturing(hipStream_t s);

// RcclComm's (high-priority) comm stream, created once per process and bound to a hardware
// queue on creation (one tiny fill runs on it). Measured on MI355X (round 2): a stream created
// after other streams have taken the process's hardware queues (GPU_MAX_HW_QUEUES) shares a
// queue, and every fork/join link handoff with it stalls (a 0.72 ms VGG-11 step went to 2.8 ms
// with 8-40 busy streams created first). reserve_streams() creates it now: call it before
// anything else creates streams (NativeTrainer and bench.py do).
hipStream_t reserved_comm_stream();
// the engine's side stream (weight gradients + their SGD, VggEngine overlap), lowest priority,
// reserved the same way
hipStream_t reserved_side_stream();
// the engine's lag stream (world 1: the top blocks' weight gradients deferred into the next
// step's forward), lowest priority, bound on first use — NOT by reserve_streams(), so a run that
// never defers (every world > 1 run) does not spend a hardware queue on it
hipStream_t reserved_lag_stream();
void reserve_streams();
// Start-up self-check of the queue assumption the stream links rely on: true when `a` and `b`
// run on ONE hardware queue. A link wait with a short timeout is enqueued on `b` ahead of its
// signal on `a`: on separate queues the signal releases the wait at once; on a shared (in-order)
// queue the signal sits behind the wait, which then ends by its timeout (bounded: never a hang).
bool streams_share_queue(hipStream_t a, hipStream_t b, double timeout_s = 0.25);

// One-direction kernel stream link (stream_link.hip): signal(producer) enqueues a one-lane
// counter bump; wait(consumer) makes the consumer wait for EVERY signal issued so far (the
// host counts them; the device keeps the expected count, so captured graphs replay
// correctly). A wait releases its consumer early only on abort_links() or after the
// process-wide link timeout; either sets error().
// Link timeout: set_link_timeout(s) (the trainer passes its communicator timeout,
// cfg.timeout_s; CS_COMM_LINK_TIMEOUT_S overrides; default 1800 s), read at each wait's enqueue.
void set_link_timeout(double seconds);
double link_timeout();
// host abort word polled by every link wait: set by the step watchdog / communicator abort so
// waiting kernels end (error 2) instead of spinning to the timeout; reset_link_abort() re-arms
void abort_links();
void reset_link_abort();
class StreamLink {
 public:
  StreamLink();
  ~StreamLink();
  StreamLink(const StreamLink&) = delete;
  StreamLink& operator=(const StreamLink&) = delete;
  void signal(hipStream_t producer);
  // signal folded into the NEXT kernel launched on the producer stream: returns the counter that
  // kernel must bump (once, at its start: it starts only after everything before it on that
  // stream completed — the same edge as a signal launch, without a launch of its own)
  unsigned long long* defer();
  void wait(hipStream_t consumer);
  std::string error() const;

 private:
  unsigned long long* dev_ = nullptr;  // [count, expect]
  int* err_ = nullptr;                 // host-mapped error word: 1 timeout, 2 aborted
  unsigned long long pending_ = 0;     // signals issued since the last wait
};

// The fork / join machinery every communicator shares (CS_COMM_FORK selects it):
//  2 = kernel stream links (default; stream_link.hip: a one-lane signal kernel on the
//      producer, a bounded one-lane wait kernel on the consumer — no HIP event at all);
//  0 = HIP events (record on the producer stream, wait on the consumer stream).
// Measured on MI355X, VGG-11 B=64 C++ step at world 1, fork/join only (no collective
// kernels), profiles/r2_dp_plumbing.md: no comm 0.755 ms; events 0.855 ms with ONE bucket
// and 0.872 ms with six (any event pair on the compute stream costs ~100 us per step);
// links 0.757 / 0.765 ms; one-rank RCCL with six bucket all-reduces 0.867 (events) vs
// 0.786 ms (links).
// Inside a graph capture the bridge always uses events (how a second stream joins a capture).
// A link's timeout shows up in error().
class StreamBridge {
 public:
  explicit StreamBridge(unsigned event_flags = hipEventDisableTiming);
  ~StreamBridge();
  StreamBridge(const StreamBridge&) = delete;
  StreamBridge& operator=(const StreamBridge&) = delete;
  void fork(hipStream_t compute, hipStream_t comm);  // comm waits for compute
  void join(hipStream_t comm, hipStream_t compute);  // compute waits for comm
  std::string error() const;
  int mode() const { return mode_; }

 private:
  int mode_ = 0;
  std::vector<hipEvent_t> fork_events_;
  size_t next_fork_ = 0;
  hipEvent_t join_event_ = nullptr;
  std::unique_ptr<StreamLink> fork_link_, join_link_;
};

inline size_t comm_dtype_bytes(ncclDataType_t dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}

}  // namespace cs
