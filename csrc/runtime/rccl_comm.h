// Native RCCL communicator (one process per MI355X, collectives over xGMI).
//
// Replaces the reference's gloo/TCP process group as the gradient data plane
// (SURVEY.md §2.2 N17-N21, §5.8): one ncclComm_t built from a unique id that the
// Python side shares through the c10d TCPStore, a dedicated high-priority comm
// stream, and fork/join between the caller's compute stream and the comm stream
// (StreamBridge: HIP events or kernel stream links, device_comm.h) — so every
// collective is stream-ordered, never blocks the host,
// overlaps with whatever the compute stream does next, and can be captured into
// a hipGraph. Averaging uses ncclAvg (the reference divides by 4 in a separate
// pass, master/part2b/part2b.py:44).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "runtime/device_comm.h"

namespace cs {

class RcclComm final : public DeviceComm {
 public:
  static std::string unique_id();  // 128 raw bytes (NCCL_UNIQUE_ID_BYTES)
  // ncclGetVersion() of the RCCL library actually loaded (torch's, not necessarily the header's)
  static int runtime_version();
  static int header_version() { return NCCL_VERSION_CODE; }

  // max_ctas > 0: RCCL compute budget (ncclConfig_t maxCTAs, minCTAs <= it) so the bucketed
  // all-reduces overlapping the backward take at most that many CUs from the conv GEMMs
  // (SURVEY.md §5.8); 0 = RCCL's own choice
  RcclComm(const std::string& uid, int rank, int world, int device, bool high_priority = true, int max_ctas = 0);
  int max_ctas() const { return max_ctas_; }
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const override { return rank_; }
  int world() const override { return world_; }
  hipStream_t stream() const override { return stream_; }
  const char* kind() const override { return "rccl"; }
  int64_t calls() const override { return calls_; }

  // All calls: the comm stream first waits for everything already enqueued on
  // `compute`; the collective then runs on the comm stream. join() makes `compute`
  // wait for everything enqueued on the comm stream so far.
  void all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t compute,
                  bool fork = true) override;
  void broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t compute, bool fork = true) override;
  void all_gather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t compute);
  void reduce_scatter(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                      hipStream_t compute);
  void reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op, int root,
              hipStream_t compute);
  void gather(const void* send, void* recv, size_t count, ncclDataType_t dt, int root, hipStream_t compute);
  void scatter(const void* send, void* recv, size_t count, ncclDataType_t dt, int root, hipStream_t compute);
  void all_to_all(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t compute);
  void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t compute);
  void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t compute);
  void group_start(hipStream_t compute);  // forks once for the whole group
  void group_end();
  void join(hipStream_t compute) override;
  // async error polling: returns "" when healthy
  std::string async_error() override;
  void abort() override;

 private:
  void fork(hipStream_t compute);
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  bool own_stream_ = true;  // false: the process-wide reserved comm stream (never destroyed)
  // (CS_COMM_FORK=1, stream memory operations hipStreamWriteValue64 / hipStreamWaitValue64 on
  // signal memory, was measured and dropped: 59.7k img/s vs 70.3-73.3k with events on the
  // one-rank probe, profiles/r1_dp_plumbing_probe.md)
  StreamBridge bridge_;
  int rank_ = 0, world_ = 1, device_ = 0, max_ctas_ = 0;
  int group_depth_ = 0;
  bool aborted_ = false;
  int64_t calls_ = 0;
};

}  // namespace cs
