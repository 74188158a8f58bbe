// lcv_k_wide.hip — kernel unit of the latency engine (small batches, lcv_set_latency_mode): ONE item per
// workgroup, its values replicated across each wave and every Montgomery product spread over the
// wave's lanes (lcv_field.hpp fp_mul_wide; LCV_WIDE makes it this unit's fp_mul).  Signature decoding and
// the SSWU maps run their per-item code on one wave per item (k_items_wide); the SOP pairing and
// hash_to_G2 programs run one wave per team lane (k_sop_wide, lcv_wide_sop.hpp).  Results are the batch
// engine's bit for bit (the same programs, the unique Montgomery quotient, the same final reductions).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#define LCV_FP_CALL 0
#define LCV_WIDE 1
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"
#include "lcv_functors_sop.hpp"
#include "lcv_wide_sop.hpp"

template <class F>
__global__ __launch_bounds__(64) void k_items_wide(F f, uint32_t n) {
  lcv::wide_init();
  if (blockIdx.x < n) f(blockIdx.x);  // every lane: the same item
}
template <class F> hipError_t lcv_hip_launch_wide(const F& f, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_items_wide<F>, dim3(n), dim3(64), 0, s, f, n);
  return hipGetLastError();
}

// wave t of the workgroup is team lane t of item blockIdx.x.  The round headers are copied into LDS at
// the start; each round prefetches the next round's record of its op into registers (the loads land
// while the round computes), so no global-memory latency sits on the round's critical path.
template <class F>
__global__ __launch_bounds__(64 * 12) void k_sop_wide(F f, uint32_t n) {
  static_assert(F::TEAM <= 12 && F::TEAM <= lcv::WIDE_MAX_WAVES, "one wave per team lane");
  constexpr uint32_t RW = 4 + 3 * F::MAXK;
  extern __shared__ uint32_t lds[];
  lcv::wide_init();
  const uint32_t item = blockIdx.x, t = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t R = f.P.rounds, ns = f.P.nslots;
  uint32_t* hl = lds + F::SHARED_WORDS + F::LDS_WORDS;  // 3 words per round: h0, record offset, words
  uint32_t* my = lds + F::SHARED_WORDS;
  for (uint32_t k = threadIdx.x; k < F::SHARED_WORDS; k += blockDim.x) lds[k] = f.P.consts[k];
  for (uint32_t k = threadIdx.x; k < 3 * R; k += blockDim.x) hl[k] = f.P.hdr[4 * (k / 3) + k % 3];
  if (item < n) f.prologue(item, t, my);
  __syncthreads();
  const uint32_t* io_in = f.io_in(item);
  uint32_t* io_out = f.io_out(item);
  uint32_t cur[RW], nxt[RW];
  {
    const uint32_t* w = f.P.rec + hl[1] + t * hl[2];
    LCV_UNROLL for (uint32_t j = 0; j < RW; ++j) cur[j] = w[j];
  }
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t h0 = __builtin_amdgcn_readfirstlane(hl[3 * r]);
    if (r + 1 < R) {  // the next round's record (records are followed by >= 3 MAXK words of the table)
      const uint32_t* w = f.P.rec + __builtin_amdgcn_readfirstlane(hl[3 * r + 4]) +
                          t * __builtin_amdgcn_readfirstlane(hl[3 * r + 5]);
      LCV_UNROLL for (uint32_t j = 0; j < RW; ++j) nxt[j] = w[j];
    }
    lcv::sop_exec_wide<F::MAXK>(h0, cur, my, lds, ns, io_in, io_out);
    __syncthreads();
    LCV_UNROLL for (uint32_t j = 0; j < RW; ++j) cur[j] = nxt[j];
  }
  if (item < n) f.epilogue(item, t, my);
}
template <class F> hipError_t lcv_hip_launch_sop_wide(const F& f, uint32_t n, hipStream_t s) {
  const size_t lds_bytes = 4 * ((size_t)F::SHARED_WORDS + F::LDS_WORDS + 3 * (size_t)f.P.rounds);
  hipLaunchKernelGGL(k_sop_wide<F>, dim3(n), dim3(64 * F::TEAM), lds_bytes, s, f, n);
  return hipGetLastError();
}

template hipError_t lcv_hip_launch_wide<F_sig>(const F_sig&, uint32_t, hipStream_t);
template hipError_t lcv_hip_launch_wide<F_h2c_map>(const F_h2c_map&, uint32_t, hipStream_t);
template hipError_t lcv_hip_launch_sop_wide<F_sop_lines>(const F_sop_lines&, uint32_t, hipStream_t);
template hipError_t lcv_hip_launch_sop_wide<F_sop_acc>(const F_sop_acc&, uint32_t, hipStream_t);
template hipError_t lcv_hip_launch_sop_wide<F_sop_fexp>(const F_sop_fexp&, uint32_t, hipStream_t);
template hipError_t lcv_hip_launch_sop_wide<F_sop_h2c>(const F_sop_h2c&, uint32_t, hipStream_t);
