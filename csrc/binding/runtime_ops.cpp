// pybind11 bindings of the native runtime: the RCCL communicator and the VGG engine.
// Collectives take torch tensors and run stream-ordered w.r.t. torch's current stream.
#include "binding/torch_util.h"
#include "runtime/markers.h"
#include "runtime/rccl_comm.h"
#include "runtime/staged_comm.h"
#include "runtime/vgg_engine.h"

namespace {

using csb::cur_stream;

ncclDataType_t nccl_dtype(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "RcclComm: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "RcclComm: unknown reduce op ", op);
  return ncclSum;
}

void check_gpu(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
}

}  // namespace

void register_runtime(pybind11::module& m) {
  m.def("reserve_streams", &cs::reserve_streams,
        "create (once per process) the native engine's side stream and the communicator's stream and bind "
        "each to a hardware queue; call it before other code creates streams");
  namespace py = pybind11;
  m.def(
      "queue_probe",
      [](intptr_t comm_stream, double timeout_s, bool with_comm) {
        // pairs of {main = the current stream, side = the engine's side stream, comm} that share one
        // hardware queue (device_comm.h streams_share_queue); comm_stream 0 = the reserved comm stream.
        // with_comm = false (no communicator: world 1): only main/side — the comm stream is never
        // used then, and a shared queue there must not turn the overlap off
        hipStream_t main_s = cur_stream(), side = cs::reserved_side_stream();
        hipStream_t comm = comm_stream ? reinterpret_cast<hipStream_t>(comm_stream) : cs::reserved_comm_stream();
        std::vector<std::string> out;
        const std::pair<const char*, std::pair<hipStream_t, hipStream_t>> pairs[] = {
            {"main/side", {main_s, side}}, {"main/comm", {main_s, comm}}, {"side/comm", {side, comm}}};
        for (const auto& pr : pairs) {
          if (!with_comm && pr.second.second == comm) continue;
          if (cs::streams_share_queue(pr.second.first, pr.second.second, timeout_s)) out.emplace_back(pr.first);
        }
        return out;
      },
      py::arg("comm_stream") = 0, py::arg("timeout_s") = 0.25, py::arg("with_comm") = true,
      "start-up check: which of the main / side / comm streams share a hardware queue");
  m.def("rccl_unique_id", []() { return py::bytes(cs::RcclComm::unique_id()); });
  m.def("rccl_version", []() { return py::make_tuple(cs::RcclComm::runtime_version(), cs::RcclComm::header_version()); },
        "(ncclGetVersion() of the loaded RCCL, NCCL_VERSION_CODE of the header built against)");
  // the engine's communicator interface (device_comm.h): RcclComm, StagedComm, ProbeComm
  py::class_<cs::DeviceComm>(m, "DeviceComm")
      .def_property_readonly("rank", &cs::DeviceComm::rank)
      .def_property_readonly("world_size", &cs::DeviceComm::world)
      .def_property_readonly("kind", [](cs::DeviceComm& c) { return std::string(c.kind()); })
      .def("calls", &cs::DeviceComm::calls)
      .def("stream_ptr", [](cs::DeviceComm& c) { return reinterpret_cast<intptr_t>(c.stream()); })
      .def("all_reduce",
           [](cs::DeviceComm& c, torch::Tensor t, const std::string& op) {
             check_gpu(t, "tensor");
             c.all_reduce(t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), cur_stream(), true);
           },
           py::arg("tensor"), py::arg("op") = "sum")
      .def("broadcast",
           [](cs::DeviceComm& c, torch::Tensor t, int root) {
             check_gpu(t, "tensor");
             c.broadcast(t.data_ptr(), t.numel(), nccl_dtype(t), root, cur_stream(), true);
           })
      .def("join", [](cs::DeviceComm& c) { c.join(cur_stream()); })
      .def("async_error", &cs::DeviceComm::async_error)
      .def("abort", &cs::DeviceComm::abort);
  m.def("roctx_available", &cs::roctx_available, "whether the native step emits roctx phase ranges");
  m.def("roctx_push", [](const std::string& n) {
    const auto& r = cs::Roctx::get();
    if (r.push) r.push(n.c_str());
  });
  m.def("roctx_pop", []() {
    const auto& r = cs::Roctx::get();
    if (r.pop) r.pop();
  });
  m.def("set_link_timeout", &cs::set_link_timeout,
        "stream-link wait timeout in seconds (the communicator timeout; CS_COMM_LINK_TIMEOUT_S overrides)");
  m.def("link_timeout", &cs::link_timeout);
  m.def("abort_links", &cs::abort_links, "release every waiting stream-link kernel with an error (watchdog path)");
  m.def("reset_link_abort", &cs::reset_link_abort);
  // diagnostic shader-clock sampler (clock_probe.hip, scripts/ramp_clock.py)
  m.def(
      "clock_sampler",
      [](torch::Tensor out, torch::Tensor stop, intptr_t stream) {
        check_gpu(out, "out");
        check_gpu(stop, "stop");
        TORCH_CHECK(out.scalar_type() == at::kLong && stop.scalar_type() == at::kInt && stop.numel() >= 1,
                    "clock_sampler: int64 out, int32 stop");
        const int64_t n = out.numel() / 2 - 1;
        TORCH_CHECK(n >= 1 && n < (1 << 30), "clock_sampler: out must hold >= 2 pairs");
        TORCH_CHECK(stream != 0, "clock_sampler: give it a stream of its own");
        CS_LAUNCH(cs_clock_sampler(reinterpret_cast<unsigned long long*>(out.data_ptr()), static_cast<int>(n),
                                       stop.data_ptr<int>(), reinterpret_cast<hipStream_t>(stream)));
      },
      "start the sampler on `stream`: (s_memrealtime, s_memtime) pairs into out until stop is set");
  m.def("clock_stamp", [](torch::Tensor slots, int i) {
    check_gpu(slots, "slots");
    TORCH_CHECK(slots.scalar_type() == at::kLong && i >= 0 && i < slots.numel(), "clock_stamp: index out of range");
    CS_LAUNCH(cs_clock_stamp(reinterpret_cast<unsigned long long*>(slots.data_ptr()), i, cur_stream()));
  });
  m.def("clock_stop", [](torch::Tensor stop) {
    check_gpu(stop, "stop");
    TORCH_CHECK(stop.scalar_type() == at::kInt, "clock_stop: int32 stop");
    CS_LAUNCH(cs_clock_stop(stop.data_ptr<int>(), cur_stream()));
  });
  py::class_<cs::StagedComm, cs::DeviceComm>(m, "StagedComm")
      .def(py::init<const std::string&, int>(), py::arg("group_name"), py::arg("device"));
  py::class_<cs::ProbeComm, cs::DeviceComm>(m, "ProbeComm")
      .def(py::init<int, double, double, int, int>(), py::arg("device"), py::arg("spin_us") = 20.0,
           py::arg("gbps") = 0.0, py::arg("world") = 8, py::arg("ctas") = 0);
  py::class_<cs::RcclComm, cs::DeviceComm>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int rank, int world, int device, bool high_priority, int max_ctas) {
             return new cs::RcclComm(std::string(uid), rank, world, device, high_priority, max_ctas);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("high_priority") = true,
           py::arg("max_ctas") = 0)
      .def_property_readonly("max_ctas", &cs::RcclComm::max_ctas)
      .def("all_gather",
           [](cs::RcclComm& c, torch::Tensor in, torch::Tensor out) {
             check_gpu(in, "in"); check_gpu(out, "out");
             TORCH_CHECK(out.numel() == in.numel() * c.world() && out.scalar_type() == in.scalar_type(),
                         "all_gather: out must hold world * in.numel() elements");
             c.all_gather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dtype(in), cur_stream());
           })
      .def("reduce_scatter",
           [](cs::RcclComm& c, torch::Tensor in, torch::Tensor out, const std::string& op) {
             check_gpu(in, "in"); check_gpu(out, "out");
             TORCH_CHECK(in.numel() == out.numel() * c.world() && out.scalar_type() == in.scalar_type(),
                         "reduce_scatter: in must hold world * out.numel() elements");
             c.reduce_scatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dtype(in), nccl_op(op), cur_stream());
           },
           py::arg("input"), py::arg("output"), py::arg("op") = "sum")
      .def("reduce",
           [](cs::RcclComm& c, torch::Tensor t, int root, const std::string& op) {
             check_gpu(t, "tensor");
             c.reduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), root, cur_stream());
           },
           py::arg("tensor"), py::arg("root"), py::arg("op") = "sum")
      .def("gather",
           [](cs::RcclComm& c, torch::Tensor in, c10::optional<torch::Tensor> out, int root) {
             check_gpu(in, "in");
             void* o = nullptr;
             if (c.rank() == root) {
               TORCH_CHECK(out.has_value() && out->numel() == in.numel() * c.world(), "gather: root needs out");
               check_gpu(*out, "out");
               o = out->data_ptr();
             }
             c.gather(in.data_ptr(), o, in.numel(), nccl_dtype(in), root, cur_stream());
           })
      .def("scatter",
           [](cs::RcclComm& c, c10::optional<torch::Tensor> in, torch::Tensor out, int root) {
             check_gpu(out, "out");
             const void* i = nullptr;
             if (c.rank() == root) {
               TORCH_CHECK(in.has_value() && in->numel() == out.numel() * c.world(), "scatter: root needs in");
               check_gpu(*in, "in");
               i = in->data_ptr();
             }
             c.scatter(i, out.data_ptr(), out.numel(), nccl_dtype(out), root, cur_stream());
           })
      .def("all_to_all",
           [](cs::RcclComm& c, torch::Tensor in, torch::Tensor out) {
             check_gpu(in, "in"); check_gpu(out, "out");
             TORCH_CHECK(in.numel() == out.numel() && in.numel() % c.world() == 0, "all_to_all: sizes");
             c.all_to_all(in.data_ptr(), out.data_ptr(), in.numel() / c.world(), nccl_dtype(in), cur_stream());
           })
      .def("send",
           [](cs::RcclComm& c, torch::Tensor t, int peer) {
             check_gpu(t, "tensor");
             c.send(t.data_ptr(), t.numel(), nccl_dtype(t), peer, cur_stream());
           })
      .def("recv",
           [](cs::RcclComm& c, torch::Tensor t, int peer) {
             check_gpu(t, "tensor");
             c.recv(t.data_ptr(), t.numel(), nccl_dtype(t), peer, cur_stream());
           })
      .def("group_start", [](cs::RcclComm& c) { c.group_start(cur_stream()); })
      .def("group_end", &cs::RcclComm::group_end);

  py::class_<cs::VggEngine>(m, "VggEngine")
      .def(py::init<int64_t, std::vector<int64_t>, std::vector<int64_t>, std::vector<int64_t>, int64_t, int64_t,
                    torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>())
      .def("set_data", &cs::VggEngine::set_data)
      .def("idx", &cs::VggEngine::idx)
      .def("set_perm", &cs::VggEngine::set_perm)
      .def("cursor", &cs::VggEngine::cursor)
      .def("loss", &cs::VggEngine::loss)
      .def("correct", &cs::VggEngine::correct)
      .def("logits", &cs::VggEngine::logits)
      .def("num_blocks", &cs::VggEngine::num_blocks)
      .def("tensor", &cs::VggEngine::tensor)
      .def("forward_train", &cs::VggEngine::forward_train)
      .def("backward", &cs::VggEngine::backward, py::arg("hi"), py::arg("lo"), py::arg("B"), py::arg("join") = true)
      .def("set_overlap", &cs::VggEngine::set_overlap)
      .def("sgd", &cs::VggEngine::sgd)
      .def("forward_eval", &cs::VggEngine::forward_eval)
      .def("step", &cs::VggEngine::step, py::arg("B"), py::arg("comm").none(true), py::arg("bucket_blocks"),
           py::arg("bucket_ranges"), py::arg("broadcast_buffers"), py::arg("lr"), py::arg("momentum"),
           py::arg("wd"), py::arg("dampening"))
      .def("set_sgd_first", &cs::VggEngine::set_sgd_first)
      .def("set_sgd_tail", &cs::VggEngine::set_sgd_tail)
      .def("set_debug_skip", &cs::VggEngine::set_debug_skip)
      .def("set_timing", &cs::VggEngine::set_timing)
      .def("set_math", &cs::VggEngine::set_math)
      .def("phase_times", &cs::VggEngine::phase_times)
      .def("link_error", &cs::VggEngine::link_error)
      .def("set_conv0_direct", &cs::VggEngine::set_conv0_direct)
      .def("set_conv0_bn_fold", &cs::VggEngine::set_conv0_bn_fold)
      .def("set_conv0_sgd_fold", &cs::VggEngine::set_conv0_sgd_fold)
      .def("set_conv0_batch_fold", &cs::VggEngine::set_conv0_batch_fold)
      .def("set_head_bn_fold", &cs::VggEngine::set_head_bn_fold)
      .def("set_side_sgd_tail", &cs::VggEngine::set_side_sgd_tail)
      .def("conv0_direct", &cs::VggEngine::conv0_direct)
      .def("join_lag", &cs::VggEngine::join_lag)
      .def("set_comm_defer", &cs::VggEngine::set_comm_defer)
      .def("set_f3_probe", &cs::VggEngine::set_f3_probe)
      .def("params_changed", &cs::VggEngine::params_changed)
      .def("amax", &cs::VggEngine::amax)
      .def("comm_defer", &cs::VggEngine::comm_defer)
      .def("defer_pending", &cs::VggEngine::defer_pending)
      .def("set_bn_fused_rows", &cs::VggEngine::set_bn_fused_rows)
      .def("set_tile", &cs::VggEngine::set_tile, py::arg("block"), py::arg("mode"), py::arg("bm"), py::arg("bn"),
           py::arg("splits"), py::arg("bk") = 16, py::arg("stage") = 0)
      .def("get_tile", &cs::VggEngine::get_tile)
      .def("autotune", &cs::VggEngine::autotune)
      .def("run_conv", &cs::VggEngine::run_conv);
}
