// Kernel-based cross-stream dependency ("stream link") — the engine's alternative to HIP
// events for forking collectives off the compute stream and joining them back.
//
// Measured on MI355X (profiles/r2_dp_plumbing.md): one HIP event record + cross-stream wait
// per gradient bucket costs the compute stream ~15 us each (6 buckets + join: 0.757 ->
// 0.873 ms per VGG-11 step with NO collective kernels at all). A link is two tiny kernels:
//   signal (producer stream): one lane bumps a device counter (agent-scope atomic add);
//   wait   (consumer stream): one lane advances its own expected count and polls the counter
//          (relaxed agent-scope loads + s_sleep) until it is reached, then exits.
// The producers' writes are already released by the AQL kernel-boundary fence before the
// signal kernel starts (in-order queue), and the consumer's next kernel starts with its own
// acquire. Counters are monotonic and the expected count lives on the device, so a link is
// graph-capturable. Every wait is bounded (timeout -> error word in host-mapped memory, the
// host's async_error() sees it): a lost signal can never hang the GPU.
#include "common.h"
#include "launchers.h"

namespace {

__global__ __launch_bounds__(64) void link_signal_kernel(unsigned long long* count) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(count, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) void link_wait_kernel(const unsigned long long* count, unsigned long long* expect,
                                                       int* err, unsigned long long timeout_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long e = __hip_atomic_load(expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1ull;
  __hip_atomic_store(expect, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e) {
    if (wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
}

}  // namespace

hipError_t cs_link_signal(unsigned long long* count, hipStream_t stream) {
  hipLaunchKernelGGL(link_signal_kernel, dim3(1), dim3(64), 0, stream, count);
  return hipGetLastError();
}

hipError_t cs_link_wait(const unsigned long long* count, unsigned long long* expect, int* err, double timeout_s,
                        hipStream_t stream) {
  const double t = timeout_s < 1e-3 ? 1e-3 : (timeout_s > 60.0 ? 60.0 : timeout_s);
  hipLaunchKernelGGL(link_wait_kernel, dim3(1), dim3(64), 0, stream, count, expect, err,
                     (unsigned long long)(t * 1e8));  // wall_clock64: 100 MHz
  return hipGetLastError();
}
