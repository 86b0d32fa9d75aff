// Kernel-based cross-stream dependency ("stream link") — the engine's alternative to HIP
// events for forking collectives off the compute stream and joining them back.
//
// Measured on MI355X (profiles/r2_dp_plumbing.md): one HIP event record + cross-stream wait
// per gradient bucket costs the compute stream ~15 us each (6 buckets + join: 0.757 ->
// 0.873 ms per VGG-11 step with NO collective kernels at all). A link is two tiny kernels:
//   signal (producer stream): one lane bumps a device counter (agent-scope atomic add);
//   wait   (consumer stream): one lane advances its own expected count by the number of
//          signals issued since the previous wait (host-tracked) and polls the counter
//          (relaxed agent-scope loads + s_sleep) until it is reached, then exits.
// The producers' writes are already released by the AQL kernel-boundary fence before the
// signal kernel starts (in-order queue), and the consumer's next kernel starts with its own
// acquire. Counters are monotonic and the expected count lives on the device, so a link is
// graph-capturable. A wait never releases its consumer before the signal except
//  * on the host's abort word (host-mapped, set by the step watchdog / communicator abort:
//    the run is failing anyway) -> error word 2, or
//  * after timeout_s -> error word 1. The engine ties timeout_s to the communicator timeout
//    (cfg.timeout_s, >= the step watchdog), so a late peer is waited for, not raced: an early
//    release would let SGD read a bucket that an all-reduce is still writing.
// Either error makes the host's next check raise; a lost signal can never hang the GPU for
// longer than the timeout.
#include "common.h"
#include "launchers.h"

namespace {

// relaxed: the producers' data is released by the kernel boundary (AQL release fence of the
// previous kernel on this in-order queue) before this kernel starts; a release here would add
// an L2 write-back of everything dirty (measured ~5.5 us per signal behind GEMMs vs ~1 us)
__global__ __launch_bounds__(64) void link_signal_kernel(unsigned long long* count) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(count, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) void link_wait_kernel(unsigned long long* count, unsigned long long* expect,
                                                       int* err, const int* abort, unsigned long long timeout_ticks,
                                                       unsigned long long delta, unsigned long long zero) {
  if (threadIdx.x != 0) return;
  // Both words are read with atomic read-modify-writes, never plain or sc1 loads: consecutive
  // waits of one link run on different XCDs, and a device-scope load is served by the reading
  // XCD's own L2, which can hold a stale copy of a line the other XCDs updated (measured: a wait
  // that read an old `expect` released its stream before the producer's signal — a data race
  // that showed up as rare wrong gradients; a poller that caches `count` can spin to its timeout).
  // Device-scope atomics are performed at the memory side, so they always see the latest value.
  const unsigned long long e =
      __hip_atomic_fetch_add(expect, delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + delta;
  const unsigned long long t0 = wall_clock64();
  // (`zero` is a kernel argument, 0 at run time: with a literal 0 the compiler turns the
  // read-modify-write back into a plain load)
  for (unsigned it = 0; __hip_atomic_fetch_add(count, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e; ++it) {
    if ((it & 255) == 255) {  // host-side checks every 256 polls (a PCIe read each)
      if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
        __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      if (wall_clock64() - t0 > timeout_ticks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
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

hipError_t cs_link_wait(const unsigned long long* count, unsigned long long* expect, int* err, const int* abort,
                        double timeout_s, hipStream_t stream, unsigned long long delta) {
  const double t = timeout_s < 1e-3 ? 1e-3 : (timeout_s > 86400.0 ? 86400.0 : timeout_s);
  hipLaunchKernelGGL(link_wait_kernel, dim3(1), dim3(64), 0, stream, const_cast<unsigned long long*>(count), expect, err,
                     abort, (unsigned long long)(t * 1e8), delta, 0ull);  // wall_clock64: 100 MHz
  return hipGetLastError();
}
