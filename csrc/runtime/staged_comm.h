// Host-staged communicator over a c10d ProcessGroup (gloo): the engine's DeviceComm
// contract with a transport that works where RCCL cannot run — N ranks sharing ONE
// MI355X (RCCL refuses duplicate devices: "Duplicate GPU detected", measured on the
// gpurun box) and CPU-side rehearsals of the multi-rank C++ step.
//
// Each collective: fork (the comm stream waits for `compute`), D2H copy of the buffer
// into a pinned staging area, host sync, the ProcessGroup collective on the host copy,
// then an async H2D copy back on the comm stream; join() orders `compute` behind it.
// So everything the engine does around the collective (which stream it forks from,
// what it enqueues before join) is exercised exactly as with RcclComm, while the wire
// is gloo. AVG = SUM then x(1/world) on the host — the same bytes the torch.distributed
// facade produces for gloo (distributed.py all_reduce), so runs through either path
// agree bitwise for power-of-two worlds.
// The host blocks inside each collective: this is a test/rehearsal transport, never
// the data plane of a multi-GPU job (that is RcclComm).
#pragma once
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <string>
#include <vector>

#include "runtime/device_comm.h"

namespace cs {

class StagedComm final : public DeviceComm {
 public:
  bool host_blocking() const override { return true; }
  // group_name: a registered c10d group (torch.distributed group.group_name)
  StagedComm(const std::string& group_name, int device);
  ~StagedComm() override;
  StagedComm(const StagedComm&) = delete;
  StagedComm& operator=(const StagedComm&) = delete;

  int rank() const override { return rank_; }
  int world() const override { return world_; }
  hipStream_t stream() const override { return stream_; }
  const char* kind() const override { return "staged"; }
  int64_t calls() const override { return calls_; }
  void all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t compute,
                  bool fork = true) override;
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t compute, bool fork = true) override;
  void join(hipStream_t compute) override;
  std::string async_error() override { return error_.empty() ? bridge_.error() : error_; }
  void abort() override;

 private:
  at::Tensor stage_in(const void* buf, size_t count, ncclDataType_t dt);
  void stage_out(void* buf, size_t count, ncclDataType_t dt);
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  hipStream_t stream_ = nullptr;
  StreamBridge bridge_;
  void* pinned_ = nullptr;
  size_t pinned_bytes_ = 0;
  int rank_ = 0, world_ = 1, device_ = 0;
  int64_t calls_ = 0;
  std::string error_;
  bool aborted_ = false;
};

// World-1 ordering probe: every collective becomes, on the comm stream, an exact scramble
// of the buffer (x2 for floats, +1 for integers), a spin of `spin_us` microseconds, and
// the exact inverse (spin_us < 0: no kernels at all — the fork/join plumbing alone, for
// measurement). A correct caller (fork before, join
// after) sees the buffer unchanged, so a probe run is bitwise equal to a no-comm run;
// a missing fork lets the scramble race the producer, a missing join lets the consumer
// read a scrambled or stale buffer — either shows up as a mismatch.
class ProbeComm final : public DeviceComm {
 public:
  // gbps > 0: the xGMI model — no scramble; every all-reduce is a spin of spin_us + the ring time
  // 2 (W-1)/W * bytes / gbps of a W-GPU ring, every broadcast spin_us + bytes / gbps, so the step
  // runs its fork / collective / comm-stream SGD / join schedule with modelled collective durations
  // ctas > 0: each modelled collective also occupies that many CUs with busy workgroups
  ProbeComm(int device, double spin_us, double gbps = 0.0, int world = 8, int ctas = 0);
  ~ProbeComm() override;
  ProbeComm(const ProbeComm&) = delete;
  ProbeComm& operator=(const ProbeComm&) = delete;
  int rank() const override { return 0; }
  int world() const override { return 1; }
  hipStream_t stream() const override { return stream_; }
  const char* kind() const override { return "probe"; }
  int64_t calls() const override { return calls_; }
  void all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t compute,
                  bool fork = true) override;
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t compute, bool fork = true) override;
  void join(hipStream_t compute) override;
  std::string async_error() override { return bridge_.error(); }

 private:
  void scramble(void* buf, size_t count, ncclDataType_t dt);
  hipStream_t stream_ = nullptr;
  StreamBridge bridge_;
  double spin_us_ = 0.0, gbps_ = 0.0;
  int model_world_ = 8;
  int ctas_ = 0;
  float* sink_ = nullptr;
  int64_t calls_ = 0;
};

}  // namespace cs
