// lcv_field.hpp — BLS12-381 base field Fp and its quadratic extension Fp2 = Fp[u]/(u^2+1).
//
// Representation: 12 x 32-bit little-endian limbs, Montgomery form with R = 2^384, always fully
// reduced into [0, p).  Multiplication is CIOS Montgomery with the "no-carry" shortcut (valid
// because the top limb of p, 0x1a0111ea, is below 2^31 - 1): each 32x32+64 step maps to one
// v_mad_u64_u32 on gfx950.  This is the arithmetic under `bls.FastAggregateVerify`
// (reference call site sync-protocol.md:464; algorithm restated from the BLS12-381 standard,
// see oracle/bls12_381.py for the CPU restatement the tests compare against).
#pragma once
#include "lcv_common.hpp"
#include "lcv_consts.inc"
#include "lcv_col28.hpp"
#include "lcv_wave.hpp"

namespace lcv {

struct fp { uint32_t v[12]; };
struct fp2 { fp c0, c1; };

#define LCV_FP_SET(r, INIT) do { constexpr uint32_t _lcv_k[12] = INIT; LCV_UNROLL for (int _i = 0; _i < 12; ++_i) (r).v[_i] = _lcv_k[_i]; } while (0)
#define LCV_FP2_SET(r, NAME) do { LCV_FP_SET((r).c0, NAME##_C0); LCV_FP_SET((r).c1, NAME##_C1); } while (0)

LCV_FN void fp_zero(fp& r) { LCV_UNROLL for (int i = 0; i < 12; ++i) r.v[i] = 0; }
LCV_FN void fp_one(fp& r) { LCV_FP_SET(r, LCV_ONE_INIT); }
LCV_FN bool fp_is_zero(const fp& a) {
  uint32_t x = 0;
  LCV_UNROLL for (int i = 0; i < 12; ++i) x |= a.v[i];
  return x == 0;
}
LCV_FN bool fp_eq(const fp& a, const fp& b) {
  uint32_t x = 0;
  LCV_UNROLL for (int i = 0; i < 12; ++i) x |= a.v[i] ^ b.v[i];
  return x == 0;
}
LCV_FN void fp_sel(fp& r, bool c, const fp& a, const fp& b) {  // r = c ? a : b
  LCV_UNROLL for (int i = 0; i < 12; ++i) r.v[i] = c ? a.v[i] : b.v[i];
}

// t (< 2p) -> t mod p
LCV_FN void fp_reduce_once(uint32_t r[12], const uint32_t t[12]) {
  constexpr uint32_t PL[12] = LCV_P_INIT;
  uint32_t d[12];
  uint32_t br = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) d[j] = subc32(t[j], PL[j], br, br);
  LCV_UNROLL for (int j = 0; j < 12; ++j) r[j] = br ? t[j] : d[j];
}

LCV_FN void fp_add(fp& r, const fp& a, const fp& b) {
  LCV_COUNT(1);
  uint32_t s[12];
  uint32_t c = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) s[j] = addc32(a.v[j], b.v[j], c, c);
  fp_reduce_once(r.v, s);
}

LCV_FN void fp_sub(fp& r, const fp& a, const fp& b) {
  LCV_COUNT(1);
  constexpr uint32_t PL[12] = LCV_P_INIT;
  uint32_t d[12];
  uint32_t br = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) d[j] = subc32(a.v[j], b.v[j], br, br);
  const uint32_t m = 0u - br;
  uint32_t c = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) r.v[j] = addc32(d[j], PL[j] & m, c, c);
}

LCV_FN void fp_dbl(fp& r, const fp& a) { fp_add(r, a, a); }
LCV_FN void fp_neg(fp& r, const fp& a) {
  fp z;
  fp_zero(z);
  fp_sub(r, z, a);
}
LCV_FN void fp_half(fp& r, const fp& a) {
  LCV_COUNT(1);
  constexpr uint32_t PL[12] = LCV_P_INIT;
  const uint32_t m = 0u - (a.v[0] & 1u);
  uint32_t t[12];
  uint32_t c = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) t[j] = addc32(a.v[j], PL[j] & m, c, c);
  LCV_UNROLL for (int j = 0; j < 11; ++j) r.v[j] = (t[j] >> 1) | (t[j + 1] << 31);
  r.v[11] = (t[11] >> 1) | (c << 31);
}

// CIOS Montgomery multiplication, no-carry variant.  r may alias a or b.  Each inner step is
// v_mad_u64_u32 (a_j * b_i + t_j, exact in 64 bits) and an add-with-carry of the running carry
// (a_j b_i + t_j + A < 2^64, so the high word absorbs the carry without overflow).
LCV_FN void fp_mul_impl(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  constexpr uint32_t PL[12] = LCV_P_INIT;
  uint32_t t[12];
  LCV_UNROLL for (int j = 0; j < 12; ++j) t[j] = 0;
  LCV_UNROLL for (int i = 0; i < 12; ++i) {
    const uint32_t bi = b[i];
    uint64_t c = (uint64_t)a[0] * bi + t[0];
    uint32_t A = (uint32_t)(c >> 32);
    const uint32_t m = (uint32_t)c * LCV_NP0;
    uint64_t c2 = (uint64_t)m * PL[0] + (uint32_t)c;
    uint32_t C = (uint32_t)(c2 >> 32);
    LCV_UNROLL for (int j = 1; j < 12; ++j) {
      c = (uint64_t)a[j] * bi + t[j];
      uint32_t co, co2;
      const uint32_t lo = addc32((uint32_t)c, A, 0u, co);
      A = (uint32_t)(c >> 32) + co;
      c2 = (uint64_t)m * PL[j] + lo;
      t[j - 1] = addc32((uint32_t)c2, C, 0u, co2);
      C = (uint32_t)(c2 >> 32) + co2;
    }
    t[11] = A + C;
  }
  fp_reduce_once(r, t);
}

// Device: product-scanning (FIPS) Montgomery multiplication on a 96-bit column accumulator.  One
// multiply-accumulate = v_mad_u64_u32 (64-bit addend, carry-out to an SGPR pair) + v_addc_co_u32
// into the top word: 2 instructions per 32x32 product instead of CIOS's mad + carry fix-ups.
// Operands may be <= 2p (the engine's lazily reduced combinations): ab + mp < 2^384 * 3p.
#ifndef LCV_FP_PS
#define LCV_FP_PS 1
#endif
#if LCV_FP_PS && !defined(LCV_HOSTSIM)
LCV_FN void mac_vv(uint64_t& acc, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(hi)
      : "v"(x), "v"(y));
}
LCV_FN void mac_vs(uint64_t& acc, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(hi)
      : "v"(x), "s"(y));
}
LCV_FN void fp_mul_ps(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  constexpr uint32_t PL[12] = LCV_P_INIT;
  uint32_t m[12], t[12];
  uint64_t acc = 0;
  uint32_t hi = 0;
  LCV_UNROLL for (int k = 0; k < 12; ++k) {
    LCV_UNROLL for (int i = 0; i < k; ++i) mac_vs(acc, hi, m[i], PL[k - i]);
    LCV_UNROLL for (int i = 0; i <= k; ++i) mac_vv(acc, hi, a[i], b[k - i]);
    m[k] = (uint32_t)acc * LCV_NP0;
    mac_vs(acc, hi, m[k], PL[0]);  // low word becomes 0
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  LCV_UNROLL for (int k = 12; k < 23; ++k) {
    LCV_UNROLL for (int i = k - 11; i < 12; ++i) {
      mac_vv(acc, hi, a[i], b[k - i]);
      mac_vs(acc, hi, m[i], PL[k - i]);
    }
    t[k - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[11] = (uint32_t)acc;
  fp_reduce_once(r, t);
}
// Squaring, product scanning: the cross products a_i a_j (i < j) of a column are accumulated once and
// doubled (78 + 12 multiply-accumulates for the square instead of 144) — the windowed square-root
// exponentiations of signature decoding and SSWU are ~80% squarings.
LCV_FN void fp_sqr_ps(uint32_t r[12], const uint32_t a[12]) {
  constexpr uint32_t PL[12] = LCV_P_INIT;
  uint32_t m[12], t[12];
  uint64_t acc = 0;
  uint32_t hi = 0;
  LCV_UNROLL for (int k = 0; k < 23; ++k) {
    // cross terms of column k, doubled: 2 * sum_{i < j, i + j = k} a_i a_j
    uint64_t x = 0;
    uint32_t xh = 0;
    LCV_UNROLL for (int i = (k > 11 ? k - 11 : 0); 2 * i < k; ++i) mac_vv(x, xh, a[i], a[k - i]);
    {  // (xh:x) <<= 1, then acc += it
      const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32);
      const uint32_t d2 = (xh << 1) | (x1 >> 31), d1 = (x1 << 1) | (x0 >> 31), d0 = x0 << 1;
      uint32_t lo = (uint32_t)acc, mid = (uint32_t)(acc >> 32), c;
      lo = addc32(lo, d0, 0u, c);
      mid = addc32(mid, d1, c, c);
      hi = hi + d2 + c;
      acc = ((uint64_t)mid << 32) | lo;
    }
    if ((k & 1) == 0) mac_vv(acc, hi, a[k >> 1], a[k >> 1]);
    if (k < 12) {
      LCV_UNROLL for (int i = 0; i < k; ++i) mac_vs(acc, hi, m[i], PL[k - i]);
      m[k] = (uint32_t)acc * LCV_NP0;
      mac_vs(acc, hi, m[k], PL[0]);  // low word becomes 0
    } else {
      LCV_UNROLL for (int i = k - 11; i < 12; ++i) mac_vs(acc, hi, m[i], PL[k - i]);
      t[k - 12] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[11] = (uint32_t)acc;
  fp_reduce_once(r, t);
}
// Round 3: the same Montgomery product / square through the 28-bit column engine (lcv_col28.hpp): no
// carry chain, one subtractive Karatsuba level, independent columns for a lone wave's issue
#ifndef LCV_FP_C28
#define LCV_FP_C28 1
#endif
#if LCV_FP_C28
LCV_FN void fp_mul_c28r(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t t[13];
  fp_mul_c28(t, a, b);
  fp_reduce_once(r, t);
}
LCV_FN void fp_sqr_c28r(uint32_t r[12], const uint32_t a[12]) {
  uint32_t t[13];
  fp_sqr_c28(t, a);
  fp_reduce_once(r, t);
}
#define LCV_SQR_IMPL fp_sqr_c28r
#define LCV_MUL_IMPL fp_mul_c28r
#else
#define LCV_SQR_IMPL fp_sqr_ps
#define LCV_MUL_IMPL fp_mul_ps
#endif

#elif defined(LCV_CPU_FAST)
// CPU-baseline build only (liblcv_cpu.so, bench.py's cpu_baseline leg): the same Montgomery product
// (R = 2^384, identical representation and results) on 6 x 64-bit limbs with 128-bit products, the
// natural x86-64 shape; the device and the test host simulation keep the 12 x 32-bit code above.
static inline void fp_mul_cpu64(uint32_t r[12], const uint32_t a32[12], const uint32_t b32[12]) {
  constexpr uint32_t PL[12] = LCV_P_INIT;
  uint64_t a[6], b[6], p[6];
  for (int k = 0; k < 6; ++k) {
    a[k] = (uint64_t)a32[2 * k] | ((uint64_t)a32[2 * k + 1] << 32);
    b[k] = (uint64_t)b32[2 * k] | ((uint64_t)b32[2 * k + 1] << 32);
    p[k] = (uint64_t)PL[2 * k] | ((uint64_t)PL[2 * k + 1] << 32);
  }
  uint64_t inv = 1;
  for (int k = 0; k < 6; ++k) inv *= 2 - p[0] * inv;  // p^-1 mod 2^64 (Newton)
  const uint64_t n0 = 0 - inv;
  uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; ++i) {
    unsigned __int128 c = 0;
    for (int j = 0; j < 6; ++j) {
      c += (unsigned __int128)a[j] * b[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[6] = (uint64_t)c;
    t[7] = (uint64_t)(c >> 64);
    const uint64_t m = t[0] * n0;
    c = (unsigned __int128)m * p[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 6; ++j) {
      c += (unsigned __int128)m * p[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[5] = (uint64_t)c;
    t[6] = t[7] + (uint64_t)(c >> 64);
  }
  uint32_t t32[12];
  for (int k = 0; k < 6; ++k) { t32[2 * k] = (uint32_t)t[k]; t32[2 * k + 1] = (uint32_t)(t[k] >> 32); }
  fp_reduce_once(r, t32);
}
#define LCV_MUL_IMPL fp_mul_cpu64
#else
#define LCV_MUL_IMPL fp_mul_impl
#endif

#if LCV_FP_CALL && !defined(LCV_HOSTSIM)
struct fp_ret { uint32_t v[12]; };
// Limbs travel as 24 scalar VGPR arguments / 12 returned VGPRs (clang's AMDGPU ABI passes
// aggregates > 16 registers through the stack, scalars in v0..v31).
__device__ __noinline__ fp_ret fp_mul_call(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4,
                                           uint32_t a5, uint32_t a6, uint32_t a7, uint32_t a8, uint32_t a9,
                                           uint32_t a10, uint32_t a11, uint32_t b0, uint32_t b1, uint32_t b2,
                                           uint32_t b3, uint32_t b4, uint32_t b5, uint32_t b6, uint32_t b7,
                                           uint32_t b8, uint32_t b9, uint32_t b10, uint32_t b11) {
  const uint32_t a[12] = {a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11};
  const uint32_t b[12] = {b0, b1, b2, b3, b4, b5, b6, b7, b8, b9, b10, b11};
  fp_ret r;
  LCV_MUL_IMPL(r.v, a, b);
  return r;
}
LCV_FN void fp_mul(fp& r, const fp& a, const fp& b) {
  fp_ret x = fp_mul_call(a.v[0], a.v[1], a.v[2], a.v[3], a.v[4], a.v[5], a.v[6], a.v[7], a.v[8], a.v[9], a.v[10],
                         a.v[11], b.v[0], b.v[1], b.v[2], b.v[3], b.v[4], b.v[5], b.v[6], b.v[7], b.v[8], b.v[9],
                         b.v[10], b.v[11]);
  LCV_COPY12(r.v, x.v);
}
#else
LCV_FN void fp_mul(fp& r, const fp& a, const fp& b) {
  LCV_COUNT(0);
  LCV_MUL_IMPL(r.v, a.v, b.v);
}
#endif

#if LCV_FP_CALL && !defined(LCV_HOSTSIM) && defined(LCV_SQR_IMPL)
__device__ __noinline__ fp_ret fp_sqr_call(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4, uint32_t a5,
                                           uint32_t a6, uint32_t a7, uint32_t a8, uint32_t a9, uint32_t a10,
                                           uint32_t a11) {
  const uint32_t a[12] = {a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11};
  fp_ret r;
  LCV_SQR_IMPL(r.v, a);
  return r;
}
LCV_FN void fp_sqr(fp& r, const fp& a) {
  fp_ret x = fp_sqr_call(a.v[0], a.v[1], a.v[2], a.v[3], a.v[4], a.v[5], a.v[6], a.v[7], a.v[8], a.v[9], a.v[10],
                         a.v[11]);
  LCV_COPY12(r.v, x.v);
}
#else
LCV_FN void fp_sqr(fp& r, const fp& a) { fp_mul(r, a, a); }
#endif

// Exponentiation by a fixed public exponent held in constant memory (wave-uniform branch).
#define LCV_DEF_POW(fname, EXPARR, NBITS)                                  \
  LCV_FN void fname(fp& r, const fp& a) {                                  \
    fp acc = a;                                                            \
    LCV_NOUNROLL for (int i = (NBITS) - 2; i >= 0; --i) {                  \
      fp_sqr(acc, acc);                                                    \
      if ((EXPARR[i >> 5] >> (i & 31)) & 1u) fp_mul(acc, acc, a);          \
    }                                                                      \
    r = acc;                                                               \
  }
LCV_DEF_POW(fp_inv_fermat, LCV_EXP_P_MINUS_2, LCV_EXP_P_MINUS_2_BITS)    // a^(p-2) (inv0: 0 -> 0)
// Sliding-window (w = 4, odd powers a^1..a^15) exponentiation by a fixed public exponent: for the
// 379-bit sqrt exponents 378 squarings + ~86 multiplications instead of 378 + ~228.  The window walk
// depends only on the exponent, so every branch is wave-uniform; the table entry is a select chain.
#define LCV_DEF_POW_W4(fname, EXPARR, NBITS)                                              \
  LCV_FN void fname(fp& r, const fp& a) {                                                 \
    fp tab[8], a2;                                                                        \
    tab[0] = a;                                                                           \
    fp_sqr(a2, a);                                                                        \
    LCV_UNROLL for (int k = 1; k < 8; ++k) fp_mul(tab[k], tab[k - 1], a2);               \
    fp acc = a;                                                                           \
    bool started = false;                                                                 \
    int i = (NBITS) - 1;                                                                  \
    LCV_NOUNROLL while (i >= 0) {                                                         \
      if (!((EXPARR[i >> 5] >> (i & 31)) & 1u)) {                                         \
        fp_sqr(acc, acc);                                                                 \
        --i;                                                                              \
        continue;                                                                         \
      }                                                                                   \
      int j = i - 3 < 0 ? 0 : i - 3;                                                      \
      while (!((EXPARR[j >> 5] >> (j & 31)) & 1u)) ++j;                                   \
      uint32_t w = 0;                                                                     \
      for (int k = i; k >= j; --k) {                                                      \
        w = (w << 1) | ((EXPARR[k >> 5] >> (k & 31)) & 1u);                               \
        if (started) fp_sqr(acc, acc);                                                    \
      }                                                                                   \
      fp m = tab[0];                                                                      \
      LCV_UNROLL for (int k = 1; k < 8; ++k) if ((w >> 1) == (uint32_t)k) m = tab[k];     \
      if (started) fp_mul(acc, acc, m); else acc = m;                                     \
      started = true;                                                                     \
      i = j - 1;                                                                          \
    }                                                                                     \
    r = acc;                                                                              \
  }
// The same window walk on 28-bit limbs with R = 2^392 (lcv_col28.hpp fp_sqr_lf / fp_mul_lf): the operand
// conversions, the packing of each product into words and its conditional subtraction leave the chain (a
// limb value < 2p squares to < 2p), so a product is its multiply-adds and quotient chain only.  In: a R ->
// a 2^392 (one product with the raw constant 2^392 mod p); out: the chain's a^e 2^392 -> a^e R (one product
// with 2^376) after packing and one subtraction.  Results equal the word-form walk's (both are fully reduced).
// LCV_POW_LF 1 (the host simulation; the latency-mode twins until round 5 v6, now LCV_POW_LF 3 below): 4-bit
// window, table in LDS — a lone wave's SSWU maps 1.55 -> 1.13 ms; at full batches the 28 KB LDS table per block crowds the co-resident final exponentiation
// (LDS- and VGPR-bound at 12 waves per CU) and the serving loop measured 0.5-1 % slower.  LCV_POW_LF 2 (the
// batch kernels): 3-bit window, four table entries in registers (the 4-bit register table spilled 624 B per
// lane): serving loop +1.3 %, one batch at a time -3.7 % (profiles/r05_v5/pow_ab.txt).  0: the word form.
#ifndef LCV_POW_LF
#if defined(LCV_CPU_FAST)
#define LCV_POW_LF 0  // the CPU baseline: its 64-bit limb products beat 28-bit columns on a scalar core
#elif defined(LCV_HOSTSIM)
#define LCV_POW_LF 1  // the host simulation runs the limb form, so the CPU tests check it against the oracle
#else
#define LCV_POW_LF 2  // batch kernels: limb form, 3-bit window, table in registers
#endif
#endif
#if LCV_POW_LF
LCV_FN void fp_lf_in(uint32_t L[14], const fp& a) {
  fp c, t;
  LCV_FP_SET(c, LCV_2E392_RAW_INIT);
  fp_mul(t, a, c);
  sop_to28<12, 14>(L, t.v);
}
LCV_FN void fp_lf_out(fp& r, const uint32_t L[14]) {
  uint32_t w[12];
  LCV_UNROLL for (int k = 0; k < 12; ++k) {  // word k = bits 32k .. 32k + 31 of the limb string (< 2^382)
    const int b = 32 * k, j = b / 28, s = b % 28;
    uint32_t x = L[j] >> s;
    if (j + 1 < 14) x |= L[j + 1] << (28 - s);
    if (s > 24 && j + 2 < 14) x |= L[j + 2] << (56 - s);
    w[k] = x;
  }
  fp t, c;
  fp_reduce_once(t.v, w);
  LCV_FP_SET(c, LCV_2E376_RAW_INIT);
  fp_mul(r, t, c);
}
// the window table a^1, a^3, .., a^15 (8 x 14 limbs per lane): in LDS on the device — one 28 KB buffer per
// 64-lane block of a per-item kernel (k_items; every caller of these chains is one), lane-interleaved, read at a
// wave-uniform index (the exponent is public) — instead of 112 VGPRs and a select chain per window
#if defined(__HIP_DEVICE_COMPILE__) && LCV_POW_LF == 1
LCV_FN uint32_t* pow_lf_table() {
  __shared__ uint32_t t[8 * 14 * 64];
  return t + (threadIdx.x & 63u);
}
#define LCV_POW_WB 4
#define LCV_POW_TAB(k, q) tabp[((k) * 14 + (q)) * 64]
#define LCV_POW_TAB_DECL uint32_t* tabp = pow_lf_table();
#define LCV_POW_TAB_GET(m, idx) LCV_UNROLL for (int q = 0; q < 14; ++q) m[q] = LCV_POW_TAB(idx, q);
#else
// registers (LCV_POW_LF 2: a 3-bit window, four entries, for the batch kernels' register budget; the host
// simulation: 4 bits); the entry is picked by wave-uniform branches (the exponent is public)
#define LCV_POW_WB (LCV_POW_LF == 2 ? 3 : 4)
#define LCV_POW_TAB(k, q) tabh[k][q]
#define LCV_POW_TAB_DECL uint32_t tabh[1 << (LCV_POW_WB - 1)][14];
#define LCV_POW_TAB_GET(m, idx)                                                           \
  LCV_UNROLL for (int q = 0; q < 14; ++q) m[q] = tabh[0][q];                              \
  LCV_UNROLL for (int k = 1; k < (1 << (LCV_POW_WB - 1)); ++k)                             \
    if ((idx) == (uint32_t)k) LCV_UNROLL for (int q = 0; q < 14; ++q) m[q] = tabh[k][q];
#endif
#define LCV_DEF_POW_LF(fname, EXPARR, NBITS)                                              \
  LCV_FN void fname(fp& r, const fp& a_) {                                                \
    uint32_t a[14], t[14], a2[14], acc[14];                                               \
    LCV_POW_TAB_DECL                                                                      \
    fp_lf_in(a, a_);                                                                      \
    LCV_UNROLL for (int j = 0; j < 14; ++j) LCV_POW_TAB(0, j) = a[j];                     \
    fp_sqr_lf(a2, a);                                                                     \
    LCV_UNROLL for (int j = 0; j < 14; ++j) t[j] = a[j];                                  \
    LCV_UNROLL for (int k = 1; k < (1 << (LCV_POW_WB - 1)); ++k) {                         \
      fp_mul_lf(t, t, a2);                                                                \
      LCV_UNROLL for (int j = 0; j < 14; ++j) LCV_POW_TAB(k, j) = t[j];                   \
    }                                                                                     \
    LCV_UNROLL for (int j = 0; j < 14; ++j) acc[j] = a[j];                                \
    bool started = false;                                                                 \
    int i = (NBITS) - 1;                                                                  \
    LCV_NOUNROLL while (i >= 0) {                                                         \
      if (!((EXPARR[i >> 5] >> (i & 31)) & 1u)) {                                         \
        fp_sqr_lf(acc, acc);                                                              \
        --i;                                                                              \
        continue;                                                                         \
      }                                                                                   \
      int j = i - (LCV_POW_WB - 1) < 0 ? 0 : i - (LCV_POW_WB - 1);                         \
      while (!((EXPARR[j >> 5] >> (j & 31)) & 1u)) ++j;                                   \
      uint32_t w = 0;                                                                     \
      for (int k = i; k >= j; --k) {                                                      \
        w = (w << 1) | ((EXPARR[k >> 5] >> (k & 31)) & 1u);                               \
        if (started) fp_sqr_lf(acc, acc);                                                 \
      }                                                                                   \
      uint32_t m[14];                                                                     \
      LCV_POW_TAB_GET(m, w >> 1)                                                          \
      if (started) fp_mul_lf(acc, acc, m);                                                \
      else LCV_UNROLL for (int q = 0; q < 14; ++q) acc[q] = m[q];                         \
      started = true;                                                                     \
      i = j - 1;                                                                          \
    }                                                                                     \
    fp_lf_out(r, acc);                                                                    \
  }
#if defined(__HIP_DEVICE_COMPILE__) && LCV_POW_LF == 3
// LCV_POW_LF 3 (the latency-mode twins, one item per wave): the same window walk with each product spread
// over the wave (lcv_wave.hpp wv_mul; the 4-bit window table is one register per entry)
#define LCV_DEF_POW_WAVE(fname, SCHED, NSCHED)                                            \
  LCV_FN void fname(fp& r, const fp& a_) {                                                \
    WaveTabs T;                                                                           \
    wv_tabs(T);                                                                           \
    uint32_t L[14];                                                                       \
    fp_lf_in(L, a_);                                                                      \
    const uint32_t a = wv_scatter(L);                                                     \
    uint32_t tab[8];                                                                      \
    tab[0] = a;                                                                           \
    const uint32_t a2 = wv_mul(a, a, T);                                                  \
    LCV_UNROLL for (int k = 1; k < 8; ++k) tab[k] = wv_mul(tab[k - 1], a2, T);            \
    uint32_t e = SCHED[0], acc = tab[0];                                                  \
    LCV_UNROLL for (int k = 1; k < 8; ++k) acc = (e >> 16) == (uint32_t)k ? tab[k] : acc; \
    LCV_NOUNROLL for (int t = 1; t < (NSCHED); ++t) {                                     \
      e = SCHED[t];                                                                       \
      LCV_NOUNROLL for (uint32_t q = e & 0xFFFFu; q > 0; --q) acc = wv_mul(acc, acc, T);  \
      const uint32_t idx = e >> 16;                                                       \
      if (idx != 0xFFFFu) {                                                               \
        uint32_t m = tab[0];                                                              \
        LCV_UNROLL for (int k = 1; k < 8; ++k) m = idx == (uint32_t)k ? tab[k] : m;        \
        acc = wv_mul(acc, m, T);                                                          \
      }                                                                                   \
    }                                                                                     \
    wv_gather(L, acc);                                                                    \
    fp_lf_out(r, L);                                                                      \
  }
LCV_DEF_POW_WAVE(fp_pow_p1d4, LCV_SCHED_P_PLUS_1_DIV_4, LCV_SCHED_P_PLUS_1_DIV_4_N)  // sqrt candidate
LCV_DEF_POW_WAVE(fp_pow_p3d4, LCV_SCHED_P_MINUS_3_DIV_4, LCV_SCHED_P_MINUS_3_DIV_4_N)
#else
LCV_DEF_POW_LF(fp_pow_p1d4, LCV_EXP_P_PLUS_1_DIV_4, LCV_EXP_P_PLUS_1_DIV_4_BITS)  // sqrt candidate
LCV_DEF_POW_LF(fp_pow_p3d4, LCV_EXP_P_MINUS_3_DIV_4, LCV_EXP_P_MINUS_3_DIV_4_BITS)
#endif
#else
LCV_DEF_POW_W4(fp_pow_p1d4, LCV_EXP_P_PLUS_1_DIV_4, LCV_EXP_P_PLUS_1_DIV_4_BITS)  // sqrt candidate
LCV_DEF_POW_W4(fp_pow_p3d4, LCV_EXP_P_MINUS_3_DIV_4, LCV_EXP_P_MINUS_3_DIV_4_BITS)
#endif
LCV_DEF_POW(fp_pow_pm1d2, LCV_EXP_P_MINUS_1_DIV_2, LCV_EXP_P_MINUS_1_DIV_2_BITS)  // Legendre

// ---- conversions (raw = canonical integer limbs, not Montgomery)
LCV_FN void fp_to_mont(fp& r, const fp& raw) {
  fp r2;
  LCV_FP_SET(r2, LCV_R2_INIT);
  fp_mul(r, raw, r2);
}
LCV_FN void fp_from_mont(fp& raw, const fp& a) {
  fp one;
  fp_zero(one);
  one.v[0] = 1;
  fp_mul(raw, a, one);
}
LCV_FN void fp_raw_from_be48(fp& r, const uint8_t* p) {
  LCV_UNROLL for (int k = 0; k < 12; ++k) r.v[k] = ld_be32(p + 44 - 4 * k);
}
LCV_FN void fp_raw_to_be48(uint8_t* p, const fp& r) {
  LCV_UNROLL for (int k = 0; k < 12; ++k) st_be32(p + 44 - 4 * k, r.v[k]);
}
// a < b on raw limbs
LCV_FN bool fp_raw_lt(const fp& a, const fp& b) {
  uint32_t br = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) (void)subc32(a.v[j], b.v[j], br, br);
  return br != 0;
}
LCV_FN bool fp_raw_lt_p(const fp& a) {
  fp p;
  LCV_FP_SET(p, LCV_P_INIT);
  return fp_raw_lt(a, p);
}
// "lexicographically largest": canonical value > (p-1)/2
LCV_FN bool fp_is_large(const fp& a_mont) {
  fp raw, half;
  fp_from_mont(raw, a_mont);
  LCV_FP_SET(half, LCV_HALF_P_RAW_INIT);
  return fp_raw_lt(half, raw);
}
LCV_FN void fp_to_be48(uint8_t* p, const fp& a_mont) {
  fp raw;
  fp_from_mont(raw, a_mont);
  fp_raw_to_be48(p, raw);
}
LCV_FN void fp_from_be48_mont(fp& r, const uint8_t* p) {  // caller guarantees value < p
  fp raw;
  fp_raw_from_be48(raw, p);
  fp_to_mont(r, raw);
}

// ---- Bernstein-Yang "safegcd" inversion, variable time (Bernstein & Yang, "Fast constant-time gcd
// computation and modular inversion", TCHES 2019; batching of the var-time divsteps as described in
// libsecp256k1's doc/safegcd_implementation.md).  Values are 13 signed 30-bit limbs (limbs 0..11 in
// [0, 2^30), limb 12 signed).  Each batch runs 30 divsteps on the low words of f, g only, giving a
// 2x2 matrix (u v; q r) with |u| + |v| <= 2^30, then applies it to the full f, g (exact division by
// 2^30) and to the Bezout coefficients d, e modulo p.  Invariants: f = d a, g = e a (mod p); the loop
// ends at g = 0 with f = +-1, so a^-1 = +-d.  Every lane runs the same instruction stream except the
// short divstep loop: ~30 batches instead of round 1's ~760 branchy shift/subtract steps of a binary
// extended Euclid (tools/microbench/soptrace.hip: that SOP inversion round took 0.4 ms per 10^4 items).
struct s30 { int32_t v[13]; };
constexpr int32_t kM30 = 0x3FFFFFFF;

// 30 divsteps on (eta = -delta, f0, g0): returns eta, t = (u, v, q, r) with
// [f'; g'] 2^30 = t [f; g]  (f odd throughout; the steps that only halve g run at once via ctz,
// the additions of f to odd g cancel up to min(eta + 1, remaining, 12) low bits at once)
LCV_FN int32_t by_divsteps30(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  // f^-1 mod 2^12 by Newton (f odd: f * f = 1 mod 8); f only changes on a swap
  uint32_t x = f;
  x *= 2u - f * x;
  x *= 2u - f * x;
  int i = 30;
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xFFFFFFFFu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // delta > 0 and g odd: (f, g) <- (g, -f)
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
      x = f;
      x *= 2u - f * x;
      x *= 2u - f * x;
    }
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 0xFFFu;
    const uint32_t w = (0u - g * x) & m;  // g + w f = 0 mod 2^min(limit, 12)
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int32_t)u; t[1] = (int32_t)v; t[2] = (int32_t)q; t[3] = (int32_t)r;
  return eta;
}

// [d; e] <- (t [d; e] + p [md; me]) / 2^30, md / me chosen so the low 30 bits vanish; d, e stay in
// (-2p, p) (md / me also add p when the input is negative)
LCV_FN void by_update_de(s30& d, s30& e, const int32_t t[4]) {
  constexpr int32_t PS[13] = LCV_P_S30_INIT;
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[12] >> 31, se = e.v[12] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((LCV_PINV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)kM30);
  me -= (int32_t)((LCV_PINV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)kM30);
  cd += (int64_t)PS[0] * md;
  ce += (int64_t)PS[0] * me;
  cd >>= 30;
  ce >>= 30;
  LCV_UNROLL for (int k = 1; k < 13; ++k) {
    const int32_t dk = d.v[k], ek = e.v[k];
    cd += (int64_t)u * dk + (int64_t)v * ek + (int64_t)PS[k] * md;
    ce += (int64_t)q * dk + (int64_t)r * ek + (int64_t)PS[k] * me;
    d.v[k - 1] = (int32_t)cd & kM30;
    cd >>= 30;
    e.v[k - 1] = (int32_t)ce & kM30;
    ce >>= 30;
  }
  d.v[12] = (int32_t)cd;
  e.v[12] = (int32_t)ce;
}

// [f; g] <- t [f; g] / 2^30 (exact)
LCV_FN void by_update_fg(s30& f, s30& g, const int32_t t[4]) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
  LCV_UNROLL for (int k = 1; k < 13; ++k) {
    const int32_t fk = f.v[k], gk = g.v[k];
    cf += (int64_t)u * fk + (int64_t)v * gk;
    cg += (int64_t)q * fk + (int64_t)r * gk;
    f.v[k - 1] = (int32_t)cf & kM30;
    cf >>= 30;
    g.v[k - 1] = (int32_t)cg & kM30;
    cg >>= 30;
  }
  f.v[12] = (int32_t)cf;
  g.v[12] = (int32_t)cg;
}

LCV_FN void fp_inv_by(fp& r, const fp& a_mont) {
  constexpr int32_t PS[13] = LCV_P_S30_INIT;
  constexpr uint32_t PL[12] = LCV_P_INIT;
  s30 f, g, d, e;
  // g = the Montgomery representative a R (< p), 30 bits per limb
  LCV_UNROLL for (int k = 0; k < 13; ++k) {
    const int b = 30 * k, w = b >> 5, s = b & 31;
    uint32_t x = a_mont.v[w] >> s;
    if (s > 2 && w + 1 < 12) x |= a_mont.v[w + 1] << (32 - s);
    g.v[k] = (int32_t)(x & (uint32_t)kM30);
    f.v[k] = PS[k];
    d.v[k] = 0;
    e.v[k] = 0;
  }
  e.v[0] = 1;
  int32_t eta = -1;
  // <= 1101 divsteps for 381-bit inputs (BY Theorem 11.2: floor((49 d + 57) / 17)), i.e. <= 37 batches
  LCV_NOUNROLL for (int it = 0; it < 40; ++it) {
    LCV_COUNT(1); LCV_COUNT(1); LCV_COUNT(1); LCV_COUNT(1);  // op counter: four 13-limb linear combinations
    int32_t t[4];
    eta = by_divsteps30(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    by_update_de(d, e, t);
    by_update_fg(f, g, t);
    int32_t z = 0;
    LCV_UNROLL for (int k = 0; k < 13; ++k) z |= g.v[k];
    if (z == 0) break;
  }
  // d in (-2p, p) as a 13-word two's complement integer; limbs 0..11 fill bits 0..359 exactly
  uint32_t x[13];
  LCV_UNROLL for (int w = 0; w < 13; ++w) x[w] = 0;
  LCV_UNROLL for (int k = 0; k < 12; ++k) {
    const int b = 30 * k, w = b >> 5, s = b & 31;
    x[w] |= (uint32_t)d.v[k] << s;
    if (s > 2) x[w + 1] |= (uint32_t)d.v[k] >> (32 - s);
  }
  x[11] |= (uint32_t)d.v[12] << 8;
  x[12] = (uint32_t)(d.v[12] >> 24);
  LCV_UNROLL for (int pass = 0; pass < 2; ++pass) {  // + p while negative
    const uint32_t m = 0u - (x[12] >> 31);
    uint32_t c = 0;
    LCV_UNROLL for (int j = 0; j < 12; ++j) x[j] = addc32(x[j], PL[j] & m, c, c);
    x[12] = x[12] + c;
  }
  // a^-1 = f d with f = +-1 (limb 12 of f is 0 or -1): p - d for f = -1 (d != 0)
  uint32_t nz = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) nz |= x[j];
  const uint32_t neg = (f.v[12] < 0 && nz != 0) ? 0xFFFFFFFFu : 0u;
  fp y;
  uint32_t br = 0;
  LCV_UNROLL for (int j = 0; j < 12; ++j) {
    const uint32_t n = subc32(PL[j], x[j], br, br);
    y.v[j] = neg ? n : x[j];
  }
  // y = (a R)^-1  ->  a^-1 R = y R^3 R^-1
  fp r3;
  LCV_FP_SET(r3, LCV_R3_INIT);
  fp_mul(r, y, r3);
}

// Fp inversion (inv0: 0 -> 0) for every stage: Bernstein-Yang above
LCV_FN void fp_inv(fp& r, const fp& a) { fp_inv_by(r, a); }

// ============================================================================ Fp2
LCV_FN void fp2_zero(fp2& r) { fp_zero(r.c0); fp_zero(r.c1); }
LCV_FN void fp2_one(fp2& r) { fp_one(r.c0); fp_zero(r.c1); }
LCV_FN bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
LCV_FN bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
LCV_FN void fp2_sel(fp2& r, bool c, const fp2& a, const fp2& b) { fp_sel(r.c0, c, a.c0, b.c0); fp_sel(r.c1, c, a.c1, b.c1); }
LCV_FN void fp2_add(fp2& r, const fp2& a, const fp2& b) { fp_add(r.c0, a.c0, b.c0); fp_add(r.c1, a.c1, b.c1); }
LCV_FN void fp2_sub(fp2& r, const fp2& a, const fp2& b) { fp_sub(r.c0, a.c0, b.c0); fp_sub(r.c1, a.c1, b.c1); }
LCV_FN void fp2_dbl(fp2& r, const fp2& a) { fp_dbl(r.c0, a.c0); fp_dbl(r.c1, a.c1); }
LCV_FN void fp2_neg(fp2& r, const fp2& a) { fp_neg(r.c0, a.c0); fp_neg(r.c1, a.c1); }
LCV_FN void fp2_half(fp2& r, const fp2& a) { fp_half(r.c0, a.c0); fp_half(r.c1, a.c1); }
LCV_FN void fp2_conj(fp2& r, const fp2& a) { r.c0 = a.c0; fp_neg(r.c1, a.c1); }
LCV_FN void fp2_mul_fp(fp2& r, const fp2& a, const fp& s) { fp_mul(r.c0, a.c0, s); fp_mul(r.c1, a.c1, s); }

// Karatsuba: 3 Fp multiplications.  r may alias a or b.
LCV_FN void fp2_mul(fp2& r, const fp2& a, const fp2& b) {
  fp t0, t1, t2, t3;
  fp_mul(t0, a.c0, b.c0);
  fp_mul(t1, a.c1, b.c1);
  fp_add(t2, a.c0, a.c1);
  fp_add(t3, b.c0, b.c1);
  fp_mul(t2, t2, t3);
  fp_sub(r.c0, t0, t1);
  fp_sub(t2, t2, t0);
  fp_sub(r.c1, t2, t1);
}
// (a0 + a1 u)^2 = (a0+a1)(a0-a1) + 2 a0 a1 u
LCV_FN void fp2_sqr(fp2& r, const fp2& a) {
  fp t0, t1, t2;
  fp_add(t0, a.c0, a.c1);
  fp_sub(t1, a.c0, a.c1);
  fp_mul(t2, a.c0, a.c1);
  fp_mul(r.c0, t0, t1);
  fp_dbl(r.c1, t2);
}
// multiply by xi = 1 + u
LCV_FN void fp2_mul_xi(fp2& r, const fp2& a) {
  fp t;
  fp_sub(t, a.c0, a.c1);
  fp_add(r.c1, a.c0, a.c1);
  r.c0 = t;
}
LCV_FN void fp2_inv(fp2& r, const fp2& a) {
  fp t0, t1;
  fp_sqr(t0, a.c0);
  fp_sqr(t1, a.c1);
  fp_add(t0, t0, t1);
  fp_inv(t1, t0);
  fp_mul(r.c0, a.c0, t1);
  fp_mul(t0, a.c1, t1);
  fp_neg(r.c1, t0);
}
LCV_FN void fp2_norm(fp& n, const fp2& a) {
  fp t;
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
}

// Square root given alpha = norm(a)^((p+1)/4) (so alpha^2 == norm(a) iff a is a square).
// Two-exponentiation method: delta = (a0 + alpha)/2, t = delta^((p-3)/4), c = t*delta,
// s = t^2 delta = +-1; then sqrt(a) = (c, a1 t/2) if s == 1 else (-a1 t/2, c).
// a1 == 0 is handled by the same exponentiation on delta = a0.  Returns y^2 == a.
LCV_FN bool fp2_sqrt_alpha(fp2& y, const fp2& a, const fp& alpha) {
  const bool a1z = fp_is_zero(a.c1);
  fp delta;
  fp_add(delta, a.c0, alpha);
  fp_half(delta, delta);
  fp_sel(delta, a1z, a.c0, delta);
  fp t, c, s;
  fp_pow_p3d4(t, delta);
  fp_mul(c, t, delta);
  fp_mul(s, c, t);
  fp one;
  fp_one(one);
  const bool s_one = fp_eq(s, one);
  fp u, nu;
  fp_half(u, a.c1);
  fp_mul(u, u, t);
  fp_neg(nu, u);
  fp zero;
  fp_zero(zero);
  // a1 == 0: (c, 0) if s==1 or delta==0 else (0, c); general: (c, u) if s==1 else (-u, c)
  const bool first = a1z ? (s_one || fp_is_zero(delta)) : s_one;
  fp y0a, y1a;
  fp_sel(y0a, a1z, zero, nu);      // second-form real part
  fp_sel(y1a, a1z, zero, u);       // first-form imaginary part
  fp_sel(y.c0, first, c, y0a);
  fp_sel(y.c1, first, y1a, c);
  fp2 chk;
  fp2_sqr(chk, y);
  return fp2_eq(chk, a);
}
LCV_FN bool fp2_sqrt(fp2& y, const fp2& a) {
  fp n, alpha;
  fp2_norm(n, a);
  fp_pow_p1d4(alpha, n);
  return fp2_sqrt_alpha(y, a, alpha);
}
// is_square(a) via the norm; also returns alpha for reuse by fp2_sqrt_alpha
LCV_FN bool fp2_is_square_alpha(const fp2& a, fp& alpha) {
  fp n, chk;
  fp2_norm(n, a);
  fp_pow_p1d4(alpha, n);
  fp_sqr(chk, alpha);
  return fp_eq(chk, n);
}
// RFC 9380 sgn0 for m = 2 (on canonical values)
LCV_FN uint32_t fp2_sgn0(const fp2& a) {
  fp r0, r1;
  fp_from_mont(r0, a.c0);
  fp_from_mont(r1, a.c1);
  const uint32_t sign0 = r0.v[0] & 1u;
  const uint32_t zero0 = fp_is_zero(r0) ? 1u : 0u;
  const uint32_t sign1 = r1.v[0] & 1u;
  return sign0 | (zero0 & sign1);
}

}  // namespace lcv
