#include "runtime/staged_comm.h"

#include <torch/csrc/distributed/c10d/GroupRegistry.hpp>

#include <stdexcept>

#include "kernels/launchers.h"
#include "runtime/fault.h"

namespace cs {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("StagedComm/ProbeComm: ") + what + ": " + hipGetErrorString(e));
}

at::ScalarType torch_dtype(ncclDataType_t dt) {
  switch (dt) {
    case ncclFloat32: return at::kFloat;
    case ncclFloat64: return at::kDouble;
    case ncclFloat16: return at::kHalf;
    case ncclBfloat16: return at::kBFloat16;
    case ncclInt64: return at::kLong;
    case ncclInt32: return at::kInt;
    case ncclUint8: return at::kByte;
    case ncclInt8: return at::kChar;
    default: throw std::runtime_error("StagedComm: unsupported dtype");
  }
}

void make_stream(int device, hipStream_t* s) {
  hip_ok(hipSetDevice(device), "hipSetDevice");
  hip_ok(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "stream");
}
}  // namespace

// ------------------------------------------------------------------------------ StagedComm

StagedComm::StagedComm(const std::string& group_name, int device) : device_(device) {
  pg_ = c10d::resolve_process_group(group_name);
  TORCH_CHECK(pg_, "StagedComm: no process group named ", group_name);
  rank_ = pg_->getRank();
  world_ = pg_->getSize();
  make_stream(device, &stream_);
}

StagedComm::~StagedComm() {
  if (stream_) hipStreamSynchronize(stream_);
  if (pinned_) hipHostFree(pinned_);
  if (stream_) hipStreamDestroy(stream_);
}

at::Tensor StagedComm::stage_in(const void* buf, size_t count, ncclDataType_t dt) {
  const size_t bytes = count * comm_dtype_bytes(dt);
  if (bytes > pinned_bytes_) {
    hip_ok(hipStreamSynchronize(stream_), "sync before regrow");
    if (pinned_) hip_ok(hipHostFree(pinned_), "hipHostFree");
    pinned_ = nullptr;
    hip_ok(hipHostMalloc(&pinned_, bytes, hipHostMallocDefault), "hipHostMalloc");
    pinned_bytes_ = bytes;
  }
  // stream order: the previous collective's H2D copy out of pinned_ completes before this copy in
  hip_ok(hipMemcpyAsync(pinned_, buf, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
  hip_ok(hipStreamSynchronize(stream_), "sync D2H");
  return at::from_blob(pinned_, {(int64_t)count}, at::TensorOptions().dtype(torch_dtype(dt)).device(at::kCPU));
}

void StagedComm::stage_out(void* buf, size_t count, ncclDataType_t dt) {
  hip_ok(hipMemcpyAsync(buf, pinned_, count * comm_dtype_bytes(dt), hipMemcpyHostToDevice, stream_), "H2D");
}

void StagedComm::all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t compute,
                            bool do_fork) {
  TORCH_CHECK(!aborted_, "StagedComm: communicator aborted");
  ++calls_;
  fault_point("all_reduce", rank_);
  if (do_fork) bridge_.fork(compute, stream_);
  at::Tensor t = stage_in(buf, count, dt);
  c10d::AllreduceOptions o;
  switch (op) {
    case ncclSum: case ncclAvg: o.reduceOp = c10d::ReduceOp::SUM; break;
    case ncclMax: o.reduceOp = c10d::ReduceOp::MAX; break;
    case ncclMin: o.reduceOp = c10d::ReduceOp::MIN; break;
    case ncclProd: o.reduceOp = c10d::ReduceOp::PRODUCT; break;
    default: TORCH_CHECK(false, "StagedComm: unsupported reduce op");
  }
  std::vector<at::Tensor> v{t};
  try {
    pg_->allreduce(v, o)->wait();
  } catch (const std::exception& e) {
    error_ = e.what();
    throw;
  }
  if (op == ncclAvg) {
    TORCH_CHECK(at::isFloatingType(t.scalar_type()), "StagedComm: avg needs a floating dtype");
    t.mul_(1.0 / world_);
  }
  stage_out(buf, count, dt);
}

void StagedComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int root, hipStream_t compute,
                           bool do_fork) {
  TORCH_CHECK(!aborted_, "StagedComm: communicator aborted");
  ++calls_;
  fault_point("broadcast", rank_);
  if (do_fork) bridge_.fork(compute, stream_);
  at::Tensor t = stage_in(buf, count, dt);
  c10d::BroadcastOptions o;
  o.rootRank = root;
  std::vector<at::Tensor> v{t};
  try {
    pg_->broadcast(v, o)->wait();
  } catch (const std::exception& e) {
    error_ = e.what();
    throw;
  }
  if (rank_ != root) stage_out(buf, count, dt);
}

void StagedComm::join(hipStream_t compute) { bridge_.join(stream_, compute); }

void StagedComm::abort() {
  if (aborted_) return;
  aborted_ = true;
  error_ = error_.empty() ? "aborted" : error_;
  pg_->abort();
}

// ------------------------------------------------------------------------------ ProbeComm

ProbeComm::ProbeComm(int device, double spin_us, double gbps, int world, int ctas)
    : spin_us_(spin_us), gbps_(gbps), model_world_(world < 2 ? 2 : world), ctas_(ctas) {
  if (ctas_ < 0 || ctas_ > 256) throw std::runtime_error("ProbeComm: ctas must be in [0, 256]");
  make_stream(device, &stream_);
  if (ctas_ > 0) {
    void* p = nullptr;
    hip_ok(hipMalloc(&p, 256 * sizeof(float)), "probe sink");
    sink_ = static_cast<float*>(p);
  }
}

ProbeComm::~ProbeComm() {
  if (stream_) hipStreamSynchronize(stream_);
  if (stream_) hipStreamDestroy(stream_);
  if (sink_) hipFree(sink_);
}

void ProbeComm::scramble(void* buf, size_t count, ncclDataType_t dt) {
  if (spin_us_ < 0.0) return;  // fork/join only: prices the stream plumbing alone
  int kind;
  switch (dt) {
    case ncclFloat32: kind = CS_SCRAMBLE_F32; break;
    case ncclInt64: kind = CS_SCRAMBLE_I64; break;
    case ncclInt32: kind = CS_SCRAMBLE_I32; break;
    default: throw std::runtime_error("ProbeComm: unsupported dtype");
  }
  // scramble at once (a consumer that does not wait for the join reads x2 values), hold it
  // for spin_us, then restore; a producer that the fork did not wait for overwrites the
  // scrambled values and the restore halves its output
  hip_ok(cs_comm_scramble(buf, (int64_t)count, kind, 0, stream_), "scramble");
  hip_ok(cs_comm_spin(spin_us_, stream_), "spin");
  hip_ok(cs_comm_scramble(buf, (int64_t)count, kind, 1, stream_), "unscramble");
}

void ProbeComm::all_reduce(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t, hipStream_t compute,
                           bool do_fork) {
  ++calls_;
  fault_point("all_reduce", 0);
  if (do_fork) bridge_.fork(compute, stream_);
  if (gbps_ > 0.0) {  // xGMI ring model: 1e3 B/us per GB/s
    const double bytes = (double)count * (dt == ncclInt64 || dt == ncclFloat64 ? 8 : 4);
    const double w = (double)model_world_;
    hip_ok(cs_comm_spin(spin_us_ + 2.0 * (w - 1.0) / w * bytes / (gbps_ * 1e3), stream_, ctas_, sink_), "model spin");
    return;
  }
  scramble(buf, count, dt);
}

void ProbeComm::broadcast(void* buf, size_t count, ncclDataType_t dt, int, hipStream_t compute, bool do_fork) {
  ++calls_;
  fault_point("broadcast", 0);
  if (do_fork) bridge_.fork(compute, stream_);
  if (gbps_ > 0.0) {
    const double bytes = (double)count * (dt == ncclInt64 || dt == ncclFloat64 ? 8 : 4);
    hip_ok(cs_comm_spin(spin_us_ + bytes / (gbps_ * 1e3), stream_, ctas_, sink_), "model spin");
    return;
  }
  scramble(buf, count, dt);
}

void ProbeComm::join(hipStream_t compute) { bridge_.join(stream_, compute); }

}  // namespace cs
