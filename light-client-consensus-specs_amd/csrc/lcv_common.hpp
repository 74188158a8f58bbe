// lcv_common.hpp — compilation-target macros shared by the HIP build (liblcv.so, gfx950)
// and the host-simulation test build (liblcv_hostsim.so, g++: the same per-item code run on
// CPU so that the arithmetic can be checked against the oracle without a GPU).
#pragma once
// work-space slots of a context (up to eight batches in flight) and the events that order a slot's two streams
enum { LCV_SLOTS = 8 };
// lcv_set_latency_mode's default: batches of at most this many rows run the SOP programs on the fan engine
enum : unsigned long long { LCV_FAN_MAX_DEFAULT = 64 };
enum { EV_START = 0, EV_PRE, EV_H2C, EV_SIDE, EV_H2D, EV_COUNT };  // EV_H2D: the slot's staged batch has left host memory
#include <stddef.h>
#include <stdint.h>

#if defined(LCV_HOSTSIM)
#define LCV_FN static inline
#define LCV_NOINLINE static __attribute__((noinline))
#define LCV_OUTLINE static inline
#define LCV_CMEM static const
#define LCV_UNROLL _Pragma("GCC unroll 64")
#define LCV_NOUNROLL _Pragma("GCC unroll 1")
#define LCV_GLOBAL_PTR
#define LCV_HDFN static inline
#else
#include <hip/hip_runtime.h>
#define LCV_FN __device__ __forceinline__
#define LCV_NOINLINE __device__ __noinline__
#define LCV_OUTLINE static __device__ __noinline__
#define LCV_CMEM static __constant__ const
#define LCV_UNROLL _Pragma("unroll")
#define LCV_NOUNROLL _Pragma("unroll 1")
#define LCV_HDFN __host__ __device__ __forceinline__  // layout arithmetic shared with the host driver
#endif

// Field multiplication strategy on the device:
//   LCV_FP_CALL=1 : fp_mul/fp_sqr are real (non-inlined) functions taking the 24 limbs as scalar
//                   VGPR arguments and returning 12 limbs in VGPRs (keeps kernels I-cache sized);
//   LCV_FP_CALL=0 : fully inlined everywhere.
#ifndef LCV_FP_CALL
#if defined(LCV_HOSTSIM)
#define LCV_FP_CALL 0
#else
#define LCV_FP_CALL 1
#endif
#endif

// Op counting (test-only host-simulation build with -DLCV_OPCOUNT): Fp multiplications, Fp
// additions/subtractions/halvings, SHA-256 compressions and (3) SOP-engine 12x12-limb products or
// Montgomery reductions (each half of a reduced Fp multiplication), per stage -> the roofline numerator.
#if defined(LCV_HOSTSIM) && defined(LCV_OPCOUNT)
#include <atomic>
namespace lcv { extern std::atomic<unsigned long long> g_ops[4]; }
#define LCV_COUNT(k) ((void)lcv::g_ops[k].fetch_add(1, std::memory_order_relaxed))
#else
#define LCV_COUNT(k) ((void)0)
#endif

#define LCV_COPY12(dst, src) do { LCV_UNROLL for (int _i = 0; _i < 12; ++_i) (dst)[_i] = (src)[_i]; } while (0)

namespace lcv {

LCV_FN uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// add / subtract with carry.  On the device clang's __builtin_addc/__builtin_subc lower to one
// v_add_co/v_addc_co (v_sub_co/v_subb_co) per limb; 64-bit temporaries would cost ~4 instructions.
LCV_FN uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
#if defined(__clang__)
  unsigned co;
  const uint32_t r = __builtin_addc(a, b, cin, &co);
  cout = co;
  return r;
#else
  const uint64_t s = (uint64_t)a + b + cin;
  cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
LCV_FN uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
#if defined(__clang__)
  unsigned bo;
  const uint32_t r = __builtin_subc(a, b, bin, &bo);
  bout = bo;
  return r;
#else
  const uint64_t s = (uint64_t)a - b - bin;
  bout = (uint32_t)(s >> 63);
  return (uint32_t)s;
#endif
}

LCV_FN uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
LCV_FN uint32_t ld_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
LCV_FN void st_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
LCV_FN uint64_t ld_le64(const uint8_t* p) { return (uint64_t)ld_le32(p) | ((uint64_t)ld_le32(p + 4) << 32); }

}  // namespace lcv
