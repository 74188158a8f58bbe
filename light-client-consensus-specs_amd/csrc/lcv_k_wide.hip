// lcv_k_wide.hip — kernel unit of the latency engine (small batches, lcv_set_latency_mode): signature
// decoding and the SSWU maps — the per-update chains of Fp exponentiations (square roots, Legendre
// symbols) that sit on a single update's critical path — run ONE item per wave, its values replicated
// in every lane and every Montgomery product spread over the wave's lanes (lcv_field.hpp fp_mul_wide;
// LCV_WIDE makes it this unit's fp_mul).  Results are the batch engine's bit for bit (the unique
// Montgomery quotient, the same final reduction).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#define LCV_FP_CALL 0
#define LCV_WIDE 1
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

template <class F>
__global__ __launch_bounds__(64) void k_items_wide(F f, uint32_t n) {
  lcv::wide_init();
  if (blockIdx.x < n) f(blockIdx.x);  // every lane: the same item
}
template <class F> hipError_t lcv_hip_launch_wide(const F& f, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_items_wide<F>, dim3(n), dim3(64), 0, s, f, n);
  return hipGetLastError();
}

template hipError_t lcv_hip_launch_wide<F_sig>(const F_sig&, uint32_t, hipStream_t);
template hipError_t lcv_hip_launch_wide<F_h2c_map>(const F_h2c_map&, uint32_t, hipStream_t);
