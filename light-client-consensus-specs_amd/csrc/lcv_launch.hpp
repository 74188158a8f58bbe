// lcv_launch.hpp — the one kernel shape of liblcv.so: one lane per item, 64-lane workgroups (one
// wave), a grid of ceil(n / 64) workgroups.  lcv_hip.hip only sees the declaration of
// lcv_hip_launch<F>; each lcv_k_*.hip unit defines the kernel and explicitly instantiates the
// launcher for its functors (LCV_KERNEL_UNIT), so the heavy stages compile as separate, parallel
// translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

template <class F> hipError_t lcv_hip_launch(const F& f, uint32_t n, hipStream_t s);
template <class F> hipError_t lcv_hip_launch_team(const F& f, uint32_t n, hipStream_t s);
template <class F> hipError_t lcv_hip_launch_sop(const F& f, uint32_t n, hipStream_t s, uint32_t g = 0);
template <class F> hipError_t lcv_hip_launch_sop_fan(const F& f, uint32_t n, hipStream_t s);
// the fan engine's lanes per product: 3 (its Karatsuba sub-products split, lcv_sop_fan.hpp) or 1
#ifndef LCV_FAN_SPLIT
#define LCV_FAN_SPLIT 1
#endif
#define LCV_FAN_PARTS (LCV_FAN_SPLIT ? 3u : 1u)

#ifdef LCV_KERNEL_UNIT
template <class F>
__global__ __launch_bounds__(64, 1) void k_items(F f, uint32_t n) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i < n) f(i);
}
// LCV_WAVE_ITEMS (lcv_k_lat.hip): one item per 64-lane wave, every lane running it (the wave-cooperative
// square-root chains, lcv_wave.hpp)
template <class F>
__global__ __launch_bounds__(64, 1) void k_wave(F f, uint32_t n) {
  (void)n;
  f(blockIdx.x);
}
template <class F> hipError_t lcv_hip_launch(const F& f, uint32_t n, hipStream_t s) {
#if defined(LCV_WAVE_ITEMS)
  hipLaunchKernelGGL(k_wave<F>, dim3(n), dim3(64), 0, s, f, n);
#else
  const uint32_t blocks = (n + 63u) / 64u;
  hipLaunchKernelGGL(k_items<F>, dim3(blocks), dim3(64), 0, s, f, n);
#endif
  return hipGetLastError();
}
// Team kernels: F::TEAM lanes cooperate on one item (64 / TEAM items per wave), exchanging values
// through F::LDS_WORDS words of LDS per item (plus F::SHARED_WORDS shared by the block's teams); the item's work is f.rounds() rounds separated by
// barriers (every lane of a team reads what the previous rounds wrote).
template <class F>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(168))) void k_team(F f, uint32_t n) {
  constexpr uint32_t T = F::TEAM, G = 64 / F::TEAM;
  __shared__ uint32_t lds[F::SHARED_WORDS + G * F::LDS_WORDS];
  const uint32_t team = threadIdx.x / T, lane = threadIdx.x % T;
  const uint32_t item = blockIdx.x * G + team;
  const bool active = team < G && item < n;
  uint32_t* my = lds + F::SHARED_WORDS + (team < G ? team : 0) * F::LDS_WORDS;
  const uint32_t R = f.rounds();
  for (uint32_t r = 0; r < R; ++r) {
    if (active) f(item, lane, r, my, lds);
    __syncthreads();
  }
}
template <class F> hipError_t lcv_hip_launch_team(const F& f, uint32_t n, hipStream_t s) {
  constexpr uint32_t G = 64 / F::TEAM;
  const uint32_t blocks = (n + G - 1) / G;
  hipLaunchKernelGGL(k_team<F>, dim3(blocks), dim3(64), 0, s, f, n);
  return hipGetLastError();
}
// the reductions' q p table after the constants (lcv_sop.hpp SOP_QP_WORDS, checked in k_sop)
#define LCV_SOP_QP_WORDS 128u
// SOP functors (lcv_functors_sop.hpp): the k_sop round loop, g items per one-wave block (g = 0: the
// most that fit, 64 / TEAM; fewer items per wave = more waves per SIMD for the same batch)
template <class F> __global__ void k_sop(F f, uint32_t n, uint32_t g);
template <class F> hipError_t lcv_hip_launch_sop(const F& f, uint32_t n, hipStream_t s, uint32_t g) {
  constexpr uint32_t G = 64 / F::TEAM;
  if (g == 0 || g > G) g = G;
  const uint32_t blocks = (n + g - 1) / g;
  const size_t lds_bytes = 4 * (size_t)(F::SHARED_WORDS + LCV_SOP_QP_WORDS + g * F::LDS_WORDS);
  hipLaunchKernelGGL(k_sop<F>, dim3(blocks), dim3(64), lds_bytes, s, f, n, g);
  return hipGetLastError();
}
// the fan engine (latency mode, lcv_sop_fan.hpp): one item per block of TEAM x MAXK x F::FAN_PARTS lanes
// (whole waves), and at least 16 lanes per op when the ops' reductions run on rows of 16 lanes (LCV_FAN_ROW,
// lcv_sop_row.hpp)
#ifndef LCV_FAN_ROW
#define LCV_FAN_ROW 1
#endif
#ifndef LCV_FAN_ROW_MAX_TEAM  // row tails for programs of at most this many ops a round (fexp 12, h2c 8; the
#define LCV_FAN_ROW_MAX_TEAM 16  // fused Miller program's 32 rows would fill 8 waves: slower, profiles/r06_ab)
#endif
template <class F> constexpr bool lcv_fan_rows() { return LCV_FAN_ROW && F::TEAM <= LCV_FAN_ROW_MAX_TEAM; }
template <class F> constexpr uint32_t lcv_fan_threads() {
  constexpr uint32_t a = ((F::TEAM * F::MAXK * F::FAN_PARTS + 63) / 64) * 64;
  constexpr uint32_t b = lcv_fan_rows<F>() ? ((16 * F::TEAM + 63) / 64) * 64 : 0;
  return a > b ? a : b;
}
template <class F> __global__ void k_sop_fan(F f, uint32_t n);
template <class F> hipError_t lcv_hip_launch_sop_fan(const F& f, uint32_t n, hipStream_t s) {
  constexpr uint32_t NT = lcv_fan_threads<F>();
  const size_t lds_bytes = 4 * (size_t)(F::SHARED_WORDS + LCV_SOP_QP_WORDS + ((F::LDS_WORDS + 1u) & ~1u)) +
                           8 * (size_t)F::TEAM * 28;
  hipLaunchKernelGGL(k_sop_fan<F>, dim3(n), dim3(NT), lds_bytes, s, f, n);
  return hipGetLastError();
}
#define LCV_INSTANTIATE_SOP(F) template hipError_t lcv_hip_launch_sop<F>(const F&, uint32_t, hipStream_t, uint32_t);
#define LCV_INSTANTIATE_SOP_FAN(F) template hipError_t lcv_hip_launch_sop_fan<F>(const F&, uint32_t, hipStream_t);
#define LCV_INSTANTIATE(F) template hipError_t lcv_hip_launch<F>(const F&, uint32_t, hipStream_t);
#define LCV_INSTANTIATE_TEAM(F) template hipError_t lcv_hip_launch_team<F>(const F&, uint32_t, hipStream_t);
#endif
