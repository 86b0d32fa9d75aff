#include "runtime/rccl_comm.h"

#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "runtime/fault.h"

namespace cs {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}
void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error in ") + what + ": " + ncclGetErrorString(r));
}
constexpr size_t kForkEvents = 64;
}  // namespace

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device, bool high_priority)
    : rank_(rank), world_(world), device_(device) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclComm: unique id must be 128 bytes");
  if (rank < 0 || rank >= world) throw std::runtime_error("RcclComm: bad rank");
  hip_ok(hipSetDevice(device), "hipSetDevice");
  int lo = 0, hi = 0;
  hip_ok(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
  hip_ok(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, high_priority ? hi : lo), "stream");
  // fork/join events only order two streams of this device: no system-scope fence needed
  // (CS_COMM_EVENT_FLAGS: 0 timing-free default events, 1 + hipEventDisableSystemFence,
  // 2 + hipEventReleaseToDevice)
  unsigned flags = hipEventDisableTiming;
  int mode = 1;
  if (const char* e = getenv("CS_COMM_EVENT_FLAGS")) mode = atoi(e);
  if (mode == 1) flags |= hipEventDisableSystemFence;
  if (mode == 2) flags |= hipEventReleaseToDevice;
  fork_events_.resize(kForkEvents);
  for (auto& e : fork_events_) hip_ok(hipEventCreateWithFlags(&e, flags), "event");
  hip_ok(hipEventCreateWithFlags(&join_event_, flags), "event");
  if (const char* e = getenv("CS_COMM_FORK")) value_sync_ = atoi(e) == 1;
  if (value_sync_) {
    void *p = nullptr, *q = nullptr;  // signal memory comes in 8-byte allocations
    hip_ok(hipExtMallocWithFlags(&p, sizeof(uint64_t), hipMallocSignalMemory), "signal memory");
    hip_ok(hipExtMallocWithFlags(&q, sizeof(uint64_t), hipMallocSignalMemory), "signal memory");
    fork_ctr_ = static_cast<uint64_t*>(p);
    join_ctr_ = static_cast<uint64_t*>(q);
    hip_ok(hipMemset(p, 0, sizeof(uint64_t)), "memset signal");
    hip_ok(hipMemset(q, 0, sizeof(uint64_t)), "memset signal");
    hip_ok(hipDeviceSynchronize(), "sync");
  }
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  nccl_ok(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
}

RcclComm::~RcclComm() {
  if (comm_ != nullptr) {
    if (!aborted_) {
      hipStreamSynchronize(stream_);
      ncclCommDestroy(comm_);
    }
  }
  for (auto& e : fork_events_) hipEventDestroy(e);
  if (join_event_) hipEventDestroy(join_event_);
  if (fork_ctr_ != nullptr) hipFree(fork_ctr_);
  if (join_ctr_ != nullptr) hipFree(join_ctr_);
  if (stream_) hipStreamDestroy(stream_);
}

void RcclComm::fork(hipStream_t compute) {
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  // inside ncclGroupStart/End the first op's fork covers the whole group
  if (value_sync_) {
    ++fork_seq_;
    hip_ok(hipStreamWriteValue64(compute, fork_ctr_, fork_seq_, 0), "hipStreamWriteValue64(fork)");
    hip_ok(hipStreamWaitValue64(stream_, fork_ctr_, fork_seq_, hipStreamWaitValueGte, ~0ull),
           "hipStreamWaitValue64(fork)");
    return;
  }
  hipEvent_t e = fork_events_[next_fork_++ % kForkEvents];
  hip_ok(hipEventRecord(e, compute), "hipEventRecord(fork)");
  hip_ok(hipStreamWaitEvent(stream_, e, 0), "hipStreamWaitEvent(fork)");
}

void RcclComm::join(hipStream_t compute) {
  if (value_sync_) {
    ++join_seq_;
    hip_ok(hipStreamWriteValue64(stream_, join_ctr_, join_seq_, 0), "hipStreamWriteValue64(join)");
    hip_ok(hipStreamWaitValue64(compute, join_ctr_, join_seq_, hipStreamWaitValueGte, ~0ull),
           "hipStreamWaitValue64(join)");
    return;
  }
  hip_ok(hipEventRecord(join_event_, stream_), "hipEventRecord(join)");
  hip_ok(hipStreamWaitEvent(compute, join_event_, 0), "hipStreamWaitEvent(join)");
}

void RcclComm::all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t compute,
                          bool do_fork) {
  ++calls_;
  fault_point("all_reduce", rank_);
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  if (do_fork) fork(compute);
  nccl_ok(ncclAllReduce(buf, buf, count, dt, op, comm_, stream_), "ncclAllReduce");
}

void RcclComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t compute,
                         bool do_fork) {
  ++calls_;
  fault_point("broadcast", rank_);
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  if (do_fork) fork(compute);  // no fork: ordered only behind what the comm stream already has
  nccl_ok(ncclBroadcast(buf, buf, count, dt, root, comm_, stream_), "ncclBroadcast");
}

void RcclComm::all_gather(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t compute) {
  ++calls_;
  fork(compute);
  nccl_ok(ncclAllGather(send, recv, count, dt, comm_, stream_), "ncclAllGather");
}

void RcclComm::reduce_scatter(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                              hipStream_t compute) {
  ++calls_;
  fork(compute);
  nccl_ok(ncclReduceScatter(send, recv, count, dt, op, comm_, stream_), "ncclReduceScatter");
}

void RcclComm::reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op, int root,
                      hipStream_t compute) {
  ++calls_;
  fork(compute);
  nccl_ok(ncclReduce(send, recv, count, dt, op, root, comm_, stream_), "ncclReduce");
}

void RcclComm::gather(const void* send, void* recv, size_t count, ncclDataType_t dt, int root, hipStream_t compute) {
  ++calls_;
  fork(compute);
  nccl_ok(ncclGather(send, recv, count, dt, root, comm_, stream_), "ncclGather");
}

void RcclComm::scatter(const void* send, void* recv, size_t count, ncclDataType_t dt, int root,
                       hipStream_t compute) {
  ++calls_;
  fork(compute);
  nccl_ok(ncclScatter(send, recv, count, dt, root, comm_, stream_), "ncclScatter");
}

void RcclComm::all_to_all(const void* send, void* recv, size_t count, ncclDataType_t dt, hipStream_t compute) {
  ++calls_;
  fork(compute);
  nccl_ok(ncclAllToAll(send, recv, count, dt, comm_, stream_), "ncclAllToAll");
}

void RcclComm::send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t compute) {
  ++calls_;
  if (group_depth_ == 0) fork(compute);
  nccl_ok(ncclSend(buf, count, dt, peer, comm_, stream_), "ncclSend");
}

void RcclComm::recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t compute) {
  ++calls_;
  if (group_depth_ == 0) fork(compute);
  nccl_ok(ncclRecv(buf, count, dt, peer, comm_, stream_), "ncclRecv");
}

void RcclComm::group_start(hipStream_t compute) {
  if (group_depth_ == 0) fork(compute);
  ++group_depth_;
  nccl_ok(ncclGroupStart(), "ncclGroupStart");
}

void RcclComm::group_end() {
  --group_depth_;
  nccl_ok(ncclGroupEnd(), "ncclGroupEnd");
}

std::string RcclComm::async_error() {
  if (aborted_) return "aborted";
  ncclResult_t r = ncclSuccess;
  if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
  return r == ncclSuccess ? std::string() : std::string(ncclGetErrorString(r));
}

void RcclComm::abort() {
  if (comm_ != nullptr && !aborted_) {
    ncclCommAbort(comm_);
    aborted_ = true;
  }
}

}  // namespace cs
