// Diagnostic: the shader clock over a training run (scripts/ramp_clock.py), for the start-up
// ramp question "same cycles at a lower clock, or more cycles?" under the real concurrent
// schedule. rocprofv3 --pmc cannot answer it there: counter collection serialises the dispatches,
// and the serialised kernels run the same time early and late (profiles/r6_ramp_pmc.txt).
//
//   sampler (its own stream, one wave, lane 0): every ~`sleep` x 64 cycles reads s_memtime
//     (shader-clock ticks) and s_memrealtime (100 MHz) and stores the pair; ends after
//     `max_samples` or once the stop word is set — every path of the loop reaches one of the two.
//   stamp (main stream, one lane): s_memrealtime into slots[i] — step boundaries on the same axis.
//   stop (main stream): sets the stop word after the last step.
// Counters are read with s_memtime / s_memrealtime; everything goes to memory through ordinary
// vector stores. Not used by the engine.
#include "common.h"
#include "launchers.h"

namespace {

__global__ __launch_bounds__(64) void clock_sampler_kernel(unsigned long long* out, int max_samples, int* stop,
                                                           int zero) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < max_samples; ++i) {
    const unsigned long long real = __builtin_amdgcn_s_memrealtime();
    const unsigned long long clk = __builtin_amdgcn_s_memtime();
    out[2 * i] = real;
    out[2 * i + 1] = clk;
    // read-modify-write of 0: served at the memory side, never a stale line in this XCD's L2
    if (__hip_atomic_fetch_add(stop, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      out[2 * i + 2] = 0ull;  // terminator (the buffer holds max_samples + 1 pairs)
      return;
    }
    __builtin_amdgcn_s_sleep(127);
    __builtin_amdgcn_s_sleep(127);
  }
}

__global__ __launch_bounds__(64) void clock_stamp_kernel(unsigned long long* slots, int i) {
  if (threadIdx.x == 0) slots[i] = __builtin_amdgcn_s_memrealtime();
}

__global__ __launch_bounds__(64) void clock_stop_kernel(int* stop) {
  if (threadIdx.x == 0) __hip_atomic_store(stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

hipError_t cs_clock_sampler(unsigned long long* out, int max_samples, int* stop, hipStream_t stream) {
  if (max_samples < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(clock_sampler_kernel, dim3(1), dim3(64), 0, stream, out, max_samples, stop, 0);
  return hipGetLastError();
}

hipError_t cs_clock_stamp(unsigned long long* slots, int i, hipStream_t stream) {
  hipLaunchKernelGGL(clock_stamp_kernel, dim3(1), dim3(64), 0, stream, slots, i);
  return hipGetLastError();
}

hipError_t cs_clock_stop(int* stop, hipStream_t stream) {
  hipLaunchKernelGGL(clock_stop_kernel, dim3(1), dim3(64), 0, stream, stop);
  return hipGetLastError();
}
