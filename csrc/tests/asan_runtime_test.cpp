// Host-side AddressSanitizer run of the native C++ runtime: the same
// runtime sources that go into _C.so (runtime/*.cpp + the kernels' host launchers), built
// with `-Xarch_host -fsanitize=address` (host code only — device code is never
// sanitized) into a standalone program, so ASan's runtime is linked first without any
// preload. Build: python -m cs744_pytorch_distributed_tutorial_amd._build --asan
//
// Without a GPU it checks the host-only pieces (the CS744_FAULT parser). On an MI355X it
// also drives the runtime the way the trainers do: a VGG-11 VggEngine on flat buffers
// (layout as runtime/engine.py FlatLayout), forward/backward/SGD, the C++ DDP step through
// the ordering-probe communicator with kernel stream links AND with HIP events, a
// one-rank RcclComm step, abort, and teardown — any heap misuse in that code aborts the
// run with an ASan report.
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <torch/torch.h>

#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "runtime/fault.h"
#include "runtime/rccl_comm.h"
#include "runtime/staged_comm.h"
#include "runtime/vgg_engine.h"

namespace {

int failures = 0;
void check(bool ok, const char* what) {
  printf("[asan-test] %-58s %s\n", what, ok ? "ok" : "FAILED");
  if (!ok) ++failures;
}

void fault_parser() {
  setenv("CS744_FAULT", "all_reduce@2:0:raise,broadcast:*:delay:0.001", 1);
  cs::fault_point("all_reduce", 0);  // first matching call: no fault
  bool raised = false;
  try {
    cs::fault_point("all_reduce", 0);
  } catch (const std::runtime_error&) {
    raised = true;
  }
  check(raised, "fault spec: all_reduce@2 raises on the 2nd call");
  cs::fault_point("all_reduce", 1);  // other rank
  cs::fault_point("broadcast", 7);   // delay
  setenv("CS744_FAULT", "bogus", 1);
  raised = false;
  try {
    cs::fault_point("x", 0);
  } catch (const std::runtime_error&) {
    raised = true;
  }
  check(raised, "fault spec: malformed spec is rejected");
  unsetenv("CS744_FAULT");
}

// VGG-11 flat layout (runtime/engine.py FlatLayout): fc1 first, then blocks last -> first,
// each tensor 64-float aligned; BN buffers in block order
struct Layout {
  std::vector<int64_t> desc, offs, buf_offs;
  int64_t total = 0, buf_total = 0;
};

int64_t align64(int64_t n) { return (n + 63) / 64 * 64; }

Layout vgg11_layout() {
  struct Blk { int cin, cout, hw, pool; };
  const int cfg[] = {64, -1, 128, -1, 256, 256, -1, 512, 512, -1, 512, 512, -1};
  std::vector<Blk> b;
  int cin = 3, hw = 32;
  for (int e : cfg) {
    if (e < 0) {
      b.back().pool = 1;
      hw /= 2;
    } else {
      b.push_back({cin, e, hw, 0});
      cin = e;
    }
  }
  Layout L;
  const int nb = (int)b.size();
  std::vector<int64_t> w(nb), bi(nb), g(nb), be(nb);
  int64_t off = 0;
  const int64_t fc_w = off;
  off = align64(off + 10 * 512);
  const int64_t fc_b = off;
  off = align64(off + 10);
  for (int l = nb - 1; l >= 0; --l) {
    w[l] = off;
    off = align64(off + (int64_t)b[l].cout * b[l].cin * 9);
    bi[l] = off;
    off = align64(off + b[l].cout);
    g[l] = off;
    off = align64(off + b[l].cout);
    be[l] = off;
    off = align64(off + b[l].cout);
  }
  L.total = off;
  int64_t boff = 0;
  for (int l = 0; l < nb; ++l) {
    L.desc.insert(L.desc.end(), {l == 0 ? 4 : b[l].cin, b[l].cout, b[l].hw, b[l].pool});
    L.offs.insert(L.offs.end(), {w[l], bi[l], g[l], be[l]});
    L.buf_offs.push_back(boff);
    boff = align64(boff + b[l].cout);
    L.buf_offs.push_back(boff);
    boff = align64(boff + b[l].cout);
  }
  L.offs.push_back(fc_w);
  L.offs.push_back(fc_b);
  L.buf_total = boff;
  return L;
}

struct Model {
  torch::Tensor params, grads, mom, bufs, nbt;
  std::unique_ptr<cs::VggEngine> engine;
  torch::Tensor data, labels, aug;
};

Model make_model(const Layout& L, int B) {
  const auto f32 = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA);
  Model m;
  torch::manual_seed(5000);
  m.params = torch::randn({L.total}, f32) * 0.05;
  m.grads = torch::zeros({L.total}, f32);
  m.mom = torch::zeros({L.total}, f32);
  m.bufs = torch::zeros({L.buf_total}, f32);
  for (size_t l = 0; l + 1 < L.buf_offs.size(); l += 2)  // running_var = 1
    m.bufs.narrow(0, L.buf_offs[l + 1], L.desc[2 * l + 1]).fill_(1.0);
  m.nbt = torch::zeros({(int64_t)L.desc.size() / 4}, f32.dtype(torch::kInt64));
  m.engine = std::make_unique<cs::VggEngine>(B, L.desc, L.offs, L.buf_offs, 512, 10, m.params, m.grads, m.mom,
                                             m.bufs, m.nbt);
  const int N = 256;
  m.data = torch::randint(0, 256, {N, 32, 32, 3}, f32.dtype(torch::kUInt8));
  m.labels = torch::randint(0, 10, {N}, f32.dtype(torch::kInt64));
  auto aug = torch::zeros({N, 3}, torch::TensorOptions().dtype(torch::kInt32));
  aug.select(1, 0).fill_(4);
  aug.select(1, 1).fill_(4);
  m.aug = aug.to(torch::kCUDA);
  m.engine->set_data(0, m.data, m.labels, m.aug);
  m.engine->set_data(1, m.data, m.labels, m.aug);
  m.engine->set_perm(torch::arange(N, torch::TensorOptions().dtype(torch::kInt64)));
  return m;
}

void engine_runs(const Layout& L) {
  const int B = 16;
  Model m = make_model(L, B);
  // three block-aligned buckets: fc1 + blocks 7..5, blocks 4..2, blocks 1..0
  const std::vector<int64_t> blocks = {5, 2, 0};
  // bucket k ends where block bucket_blocks[k] ends: the start of block (lo - 1)'s weights
  auto end_of = [&](int lo) { return lo == 0 ? L.total : L.offs[4 * (lo - 1)]; };
  std::vector<int64_t> br;
  int64_t at = 0;
  for (int64_t lo : blocks) {
    const int64_t e = end_of((int)lo);
    br.push_back(at);
    br.push_back(e - at);
    at = e;
  }
  check(at == L.total, "bucket ranges tile the flat buffer");
  m.engine->forward_train(B);
  m.engine->backward(7, 0, B);
  m.engine->sgd(0.1, 0.9, 1e-4, 0.0, 0, L.total);
  hipDeviceSynchronize();
  const float l0 = m.engine->loss().item<float>();
  check(std::isfinite(l0), "eager forward / backward / SGD");
  for (int mode : {2, 0}) {  // kernel stream links, then HIP events
    setenv("CS_COMM_FORK", mode == 2 ? "2" : "0", 1);
    cs::ProbeComm probe(0, 20.0);
    for (int s = 0; s < 3; ++s) m.engine->step(B, &probe, blocks, br, true, 0.1, 0.9, 1e-4, 0.0);
    hipDeviceSynchronize();
    check(probe.calls() == 3 * (3 + 2) && probe.async_error().empty(),
          mode == 2 ? "C++ DDP step through ProbeComm (stream links)" : "C++ DDP step through ProbeComm (events)");
  }
  unsetenv("CS_COMM_FORK");
  {
    cs::RcclComm rc(cs::RcclComm::unique_id(), 0, 1, 0);
    for (int s = 0; s < 2; ++s) m.engine->step(B, &rc, blocks, br, true, 0.1, 0.9, 1e-4, 0.0);
    hipDeviceSynchronize();
    check(rc.async_error().empty() && std::isfinite(m.engine->loss().item<float>()), "C++ DDP step, one-rank RCCL");
    rc.abort();
    bool raised = false;
    try {
      m.engine->step(B, &rc, blocks, br, true, 0.1, 0.9, 1e-4, 0.0);
    } catch (const std::runtime_error&) {
      raised = true;
    }
    check(raised && rc.async_error() == "aborted", "collective after abort raises");
    hipDeviceSynchronize();
  }
  m.engine->forward_eval(B);
  hipDeviceSynchronize();
  check(m.engine->correct().item<int>() >= 0, "eval forward");
  std::vector<double> us = m.engine->autotune(B, 1);
  check(us.size() == 24, "autotune sweep");
}

}  // namespace

int main() {
  fault_parser();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    printf("[asan-test] no GPU: host-only checks done, %d failure(s)\n", failures);
    return failures ? 1 : 0;
  }
  hipSetDevice(0);
  const Layout L = vgg11_layout();
  check(L.total >= 9231114, "VGG-11 flat layout (>= 9,231,114 params)");
  engine_runs(L);  // every engine / communicator object is destroyed inside (checked by ASan)
  printf("[asan-test] done, %d failure(s)\n", failures);
  fflush(stdout);
  // Leave without the shared libraries' exit-time finalizers: under ASan's allocator the ROCm
  // runtime's own teardown (libamdhip64 -> libhsa-runtime64 from __cxa_finalize) reads
  // uninitialised heap and faults, with no frame of this program on the stack. Nothing of ours
  // runs after this point; everything this program created was destroyed above.
  std::_Exit(failures ? 1 : 0);
}
