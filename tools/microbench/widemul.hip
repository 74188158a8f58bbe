// Lone-wave latency of a chain of Montgomery products: the narrow per-lane product (fp_mul, the batch
// engine) against wide ones (one product spread over a wave's lanes: the latency engine).  Every chain
// must end on the same value.  Variants of the wide product:
//   v1  lcv_field.hpp fp_mul_wide (one accumulator per phase, readlane broadcasts)
//   v2  two accumulators per phase (even / odd terms: half the dependent mad chain), readlane broadcasts
//   v3  v2 with the T / M words broadcast through LDS (one store per lane, 128-bit broadcast reads)
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../light-client-consensus-specs_amd/csrc widemul.hip -o widemul
#include <hip/hip_runtime.h>
#include <stdio.h>
#define LCV_FP_CALL 1
#include "lcv_field.hpp"
using namespace lcv;

// (hi:acc) += (hi1:acc1)
__device__ __forceinline__ void acc_merge(uint64_t& acc, uint32_t& hi, uint64_t acc1, uint32_t hi1) {
  uint32_t lo = (uint32_t)acc, mid = (uint32_t)(acc >> 32), c;
  lo = addc32(lo, (uint32_t)acc1, 0u, c);
  mid = addc32(mid, (uint32_t)(acc1 >> 32), c, c);
  hi = hi + hi1 + c;
  acc = ((uint64_t)mid << 32) | lo;
}

template <int V>
__device__ void mul_var(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  const uint32_t lane = wide_lane();
  uint32_t* bs = wide_scratch();
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    LCV_UNROLL for (int j = 0; j < 12; ++j) bs[WIDE_OFF + j] = b[j];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t* bl = bs + WIDE_OFF + lane;
  uint64_t acc = 0, acc1 = 0;
  uint32_t hi = 0, hi1 = 0;
  LCV_UNROLL for (int i = 0; i < 12; i += 2) { mac_vv(acc, hi, a[i], bl[-i]); mac_vv(acc1, hi1, a[i + 1], bl[-i - 1]); }
  acc_merge(acc, hi, acc1, hi1);
  const uint32_t T = wide_norm<24>(acc, hi);
  const uint32_t* np = wide_lds + WIDE_OFF + lane;
  const uint32_t* pp = wide_lds + WIDE_WIN + WIDE_OFF + lane;
  uint32_t tw[12], mw[12];
  if constexpr (V == 3) {
    __builtin_amdgcn_wave_barrier();
    bs[40 + lane] = T;  // words 40.. of the window: beyond the operand's zero pad reads? (pad reads stop at 16 + 63 - 0 = 79)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    LCV_UNROLL for (int i = 0; i < 12; ++i) tw[i] = bs[40 + i];
  } else {
    LCV_UNROLL for (int i = 0; i < 12; ++i) tw[i] = __builtin_amdgcn_readlane(T, i);
  }
  acc = 0; acc1 = 0; hi = 0; hi1 = 0;
  LCV_UNROLL for (int i = 0; i < 12; i += 2) { mac_vv(acc, hi, np[-i], tw[i]); mac_vv(acc1, hi1, np[-i - 1], tw[i + 1]); }
  acc_merge(acc, hi, acc1, hi1);
  const uint32_t M = wide_norm<12>(acc, hi);
  if constexpr (V == 3) {
    __builtin_amdgcn_wave_barrier();
    bs[40 + lane] = M;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    LCV_UNROLL for (int i = 0; i < 12; ++i) mw[i] = bs[40 + i];
  } else {
    LCV_UNROLL for (int i = 0; i < 12; ++i) mw[i] = __builtin_amdgcn_readlane(M, i);
  }
  acc = T; acc1 = 0; hi = 0; hi1 = 0;
  LCV_UNROLL for (int i = 0; i < 12; i += 2) { mac_vv(acc, hi, pp[-i], mw[i]); mac_vv(acc1, hi1, pp[-i - 1], mw[i + 1]); }
  acc_merge(acc, hi, acc1, hi1);
  const uint32_t U = wide_norm<25>(acc, hi);
  uint32_t u[12];
  if constexpr (V == 3) {
    __builtin_amdgcn_wave_barrier();
    bs[40 + lane] = U;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    LCV_UNROLL for (int j = 0; j < 12; ++j) u[j] = bs[52 + j];
    __builtin_amdgcn_wave_barrier();
    if (lane >= 40) bs[lane] = 0;   // restore the zero pad the operand reads rely on
    __builtin_amdgcn_wave_barrier();
  } else {
    LCV_UNROLL for (int j = 0; j < 12; ++j) u[j] = __builtin_amdgcn_readlane(U, 12 + j);
  }
  fp_reduce_once(r, u);
}

__device__ void init_xy(fp& x, fp& y, uint32_t t) {
  for (int j = 0; j < 12; ++j) { x.v[j] = 0x1234567u * (j + 1) + t; y.v[j] = 0x9abcdefu * (j + 3); }
  x.v[11] &= 0x0fffffffu; y.v[11] &= 0x0fffffffu;
}
__global__ void k_narrow(uint32_t* out, int n) {
  fp x, y;
  init_xy(x, y, threadIdx.x);
  for (int k = 0; k < n; ++k) fp_mul(x, x, y);
  if (threadIdx.x == 0) for (int j = 0; j < 12; ++j) out[j] = x.v[j];
}
template <int V>
__global__ void k_wide(uint32_t* out, int n) {
  wide_init();
  fp x, y;
  init_xy(x, y, 0);
  for (int k = 0; k < n; ++k) {
    fp r;
    if constexpr (V == 1) fp_mul_wide(r.v, x.v, y.v);
    else mul_var<V>(r.v, x.v, y.v);
    x = r;
  }
  if (threadIdx.x == 0) for (int j = 0; j < 12; ++j) out[12 * V + j] = x.v[j];
}
template <class K>
float timed(K kern, uint32_t* d, int n) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d, 16); hipDeviceSynchronize();
  hipEventRecord(a); hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d, n); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return 1000.0f * ms / n;
}
int main() {
  uint32_t* d; (void)hipMalloc(&d, 4096); (void)hipMemset(d, 0, 4096);
  const int N = 4000;
  printf("narrow: %.3f us per product (lone wave, %d chained)\n", timed(k_narrow, d, N), N);
  printf("wide v1: %.3f us\n", timed(k_wide<1>, d, N));
  printf("wide v2: %.3f us\n", timed(k_wide<2>, d, N));
  printf("wide v3: %.3f us\n", timed(k_wide<3>, d, N));
  uint32_t h[48]; (void)hipMemcpy(h, d, 192, hipMemcpyDeviceToHost);
  int same = 1;
  for (int v = 1; v <= 3; ++v) for (int j = 0; j < 12; ++j) same &= h[j] == h[12 * v + j];
  printf("results %s\n", same ? "IDENTICAL" : "DIFFER");
  return same ? 0 : 1;
}
