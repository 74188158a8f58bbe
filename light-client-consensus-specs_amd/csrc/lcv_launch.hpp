// lcv_launch.hpp — the one kernel shape of liblcv.so: one lane per item, 64-lane workgroups (one
// wave), a grid of ceil(n / 64) workgroups.  lcv_hip.hip only sees the declaration of
// lcv_hip_launch<F>; each lcv_k_*.hip unit defines the kernel and explicitly instantiates the
// launcher for its functors (LCV_KERNEL_UNIT), so the heavy stages compile as separate, parallel
// translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

template <class F> hipError_t lcv_hip_launch(const F& f, uint32_t n, hipStream_t s);

#ifdef LCV_KERNEL_UNIT
template <class F>
__global__ __launch_bounds__(64, 1) void k_items(F f, uint32_t n) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i < n) f(i);
}
template <class F> hipError_t lcv_hip_launch(const F& f, uint32_t n, hipStream_t s) {
  const uint32_t blocks = (n + 63u) / 64u;
  hipLaunchKernelGGL(k_items<F>, dim3(blocks), dim3(64), 0, s, f, n);
  return hipGetLastError();
}
#define LCV_INSTANTIATE(F) template hipError_t lcv_hip_launch<F>(const F&, uint32_t, hipStream_t);
#endif
