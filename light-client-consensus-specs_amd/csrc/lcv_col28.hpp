// lcv_col28.hpp — 28-bit-limb column arithmetic for Montgomery products on gfx950 (R = 2^384): operands
// converted from 12 x 32-bit words to 14 limbs of 28 bits, products accumulated into independent 64-bit
// column accumulators (a 28 x 28-bit product is below 2^56: no carry adds; one v_mad_u64_u32 per limb
// product), one subtractive Karatsuba level over 7-limb halves, and the Montgomery reduction as thirteen
// 28-bit quotient digits and one 20-bit digit.  Used by the SOP engine (lcv_sop.hpp: K products per
// reduction) and by fp_mul / fp_sqr of the per-item kernels (lcv_field.hpp).  The arithmetic of
// bls.FastAggregateVerify (reference call site sync-protocol.md:464).
#pragma once
#include "lcv_common.hpp"
#include "lcv_consts.inc"

// Instruction-class accounting (tools/sop_iclass.py): with -DLCV_SOP_MARKERS the device build places an
// assembler comment at the start of each region of an SOP round (operands, conversion, MACs, join,
// reduction, tail steps: lcv_sop.hpp), so the compiled kernel's instructions can be attributed to them.
// Never set in the product build (a comment-only inline asm still constrains the scheduler).
#if defined(__HIP_DEVICE_COMPILE__) && defined(LCV_SOP_MARKERS)
#define SOP_MARK(name) asm volatile("; sopmark " name)
#else
#define SOP_MARK(name) ((void)0)
#endif

namespace lcv {

enum : uint32_t { SOP_M28 = 0x0FFFFFFFu };

// ---------------------------------------------------------------------------- 28-bit limb constants
struct Limbs28 { uint32_t v[15]; };
// 12 x 32-bit words -> 28-bit limbs (constexpr: the modulus and its shifted copies)
constexpr Limbs28 limbs28_of(const uint32_t (&w)[12], int shift = 0) {
  Limbs28 r{};
  for (int l = 0; l < 15; ++l) {
    uint32_t x = 0;
    for (int b = 0; b < 28; ++b) {
      const int g = 28 * l + b - shift;
      if (g >= 0 && g < 384 && ((w[g / 32] >> (g % 32)) & 1u)) x |= 1u << b;
    }
    r.v[l] = x;
  }
  return r;
}
constexpr uint32_t np28_of(uint32_t p0) {  // -p^-1 mod 2^28
  uint32_t inv = 1;
  for (int i = 0; i < 5; ++i) inv *= 2u - p0 * inv;
  return (0u - inv) & SOP_M28;
}
constexpr uint32_t kPw[12] = LCV_P_INIT;
constexpr Limbs28 kP28 = limbs28_of(kPw);
constexpr uint32_t kNP28 = np28_of(kP28.v[0]);

// NW 32-bit words -> NL 28-bit limbs (NL * 28 >= the value's bits; a limb reads at most two words)
template <int NW, int NL>
LCV_FN void sop_to28(uint32_t o[], const uint32_t w[]) {
  LCV_UNROLL for (int l = 0; l < NL; ++l) {
    const int b = 28 * l, k = b / 32, s = b % 32;
    uint32_t x = w[k] >> s;
    if (s > 4 && k + 1 < NW) x |= w[k + 1] << (32 - s);
    o[l] = (l == NL - 1 && 28 * NL >= 32 * NW) ? x : x & SOP_M28;
  }
}

// column accumulators: col[i + j] += x_i y_j (one v_mad_u64_u32 per product, no carry).  FIRST: the
// op's first product writes the columns instead (the first pair of column c is i = 0 or j = 13), and
// the one column it does not reach is zeroed.
template <int NX, bool FIRST>
LCV_FN void sop_mac28(uint64_t col[28], const uint32_t x[15], const uint32_t y[14]) {
  LCV_UNROLL for (int i = 0; i < NX; ++i)
    LCV_UNROLL for (int j = 0; j < 14; ++j) {
      if (FIRST && (i == 0 || j == 13)) col[i + j] = (uint64_t)x[i] * y[j];
      else col[i + j] += (uint64_t)x[i] * y[j];
    }
  if (FIRST && NX == 14) col[27] = 0;
}

// One Karatsuba level over the 7-limb halves (B = 2^196), subtractive form:
//   X Y = P0 + (P0 + P2 + D) B + P2 B^2,  P0 = X0 Y0, P2 = X1 Y1, D = (X0 - X1)(Y1 - Y0)
// The limb differences are signed 29-bit values, so D accumulates with signed multiply-adds in signed
// 64-bit columns (|D column| <= 7 * 2^56 per product: any K <= 15 fits).  The three 7 x 7 products (147
// multiply-adds instead of 196) accumulate over ALL of an op's products (the combination is linear), so
// the join below runs once per op; every joined column is a true (non-negative) column sum.
template <bool FIRST, class A>
LCV_FN void sop_mac7(A c[13], const uint32_t* x, const uint32_t* y) {
  LCV_UNROLL for (int i = 0; i < 7; ++i)
    LCV_UNROLL for (int j = 0; j < 7; ++j) {
      if (FIRST && (i == 0 || j == 6)) c[i + j] = (uint64_t)x[i] * y[j];
      else c[i + j] += (uint64_t)x[i] * y[j];
    }
}
template <bool FIRST>
LCV_FN void sop_mac7s(int64_t c[13], const int32_t* x, const int32_t* y) {
  LCV_UNROLL for (int i = 0; i < 7; ++i)
    LCV_UNROLL for (int j = 0; j < 7; ++j) {
      if (FIRST && (i == 0 || j == 6)) c[i + j] = (int64_t)x[i] * y[j];
      else c[i + j] += (int64_t)x[i] * y[j];
    }
}
template <bool FIRST>
LCV_FN void sop_kara_mac(uint64_t p0[13], uint64_t p2[13], int64_t pd[13], const uint32_t x[15], const uint32_t y[14]) {
  SOP_MARK("kara");
  int32_t xd[7], yd[7];
  LCV_UNROLL for (int i = 0; i < 7; ++i) { xd[i] = (int32_t)(x[i] - x[i + 7]); yd[i] = (int32_t)(y[i + 7] - y[i]); }
  sop_mac7<FIRST>(p0, x, y);
  sop_mac7<FIRST>(p2, x + 7, y + 7);
  sop_mac7s<FIRST>(pd, xd, yd);
}
LCV_FN void sop_kara_join(uint64_t col[28], const uint64_t p0[13], const uint64_t p2[13], const int64_t pd[13]) {
  LCV_UNROLL for (int c = 0; c < 28; ++c) {
    uint64_t v = c < 13 ? p0[c] : 0;
    if (c >= 7 && c < 20) v += p0[c - 7] + p2[c - 7] + (uint64_t)pd[c - 7];
    if (c >= 14 && c < 27) v += p2[c - 14];
    col[c] = v;
  }
}

// r (13 words) = (T + M p) / 2^384, T = sum col[c] 2^(28 c), M < 2^384 the Montgomery quotient:
// thirteen 28-bit digits and a 20-bit one (384 = 13 * 28 + 20)
LCV_FN void sop_redc28(uint32_t r[13], uint64_t col[28]) {
  uint64_t carry = 0, v;
  LCV_UNROLL for (int i = 0; i < 13; ++i) {
    v = col[i] + carry;
    const uint32_t q = ((uint32_t)v * kNP28) & SOP_M28;
    carry = (v + (uint64_t)q * kP28.v[0]) >> 28;  // the low 28 bits vanish
    LCV_UNROLL for (int j = 1; j < 14; ++j) col[i + j] += (uint64_t)q * kP28.v[j];
  }
  v = col[13] + carry;
  const uint32_t q = ((uint32_t)v * kNP28) & 0xFFFFFu;
  v += (uint64_t)q * kP28.v[0];  // the low 20 bits vanish
  LCV_UNROLL for (int j = 1; j < 14; ++j) col[13 + j] += (uint64_t)q * kP28.v[j];
  // columns 13..27 -> 28-bit limbs L (L[0] = bits 0..27 of column 13, whose low 20 bits are 0), then
  // word k of the result is bits 20 + 32 k .. 51 + 32 k of the limb string
  SOP_MARK("normalise");
  uint32_t L[16];
  L[0] = (uint32_t)v & SOP_M28;
  carry = v >> 28;
  LCV_UNROLL for (int c = 14; c < 28; ++c) {
    const uint64_t t = col[c] + carry;
    L[c - 13] = (uint32_t)t & SOP_M28;
    carry = t >> 28;
  }
  L[15] = (uint32_t)carry;
  SOP_MARK("pack");
  LCV_UNROLL for (int k = 0; k < 13; ++k) {
    const int b = 20 + 32 * k, j = b / 28, s = b % 28;
    uint32_t x = L[j] >> s;
    x |= L[j + 1] << (28 - s);
    if (s > 24) x |= L[j + 2] << (56 - s);
    r[k] = x;
  }
}


// R = 2^392 (fourteen full 28-bit digits): L (14 limbs) = (T + M p) / 2^392, normalised 28-bit limbs, for the
// limb-form exponentiation chains (lcv_field.hpp fp_pow_lf), whose values never leave 28-bit limbs
LCV_FN void sop_redc28_392(uint32_t L[14], uint64_t col[28]) {
  uint64_t carry = 0;
  LCV_UNROLL for (int i = 0; i < 14; ++i) {
    const uint64_t v = col[i] + carry;
    const uint32_t q = ((uint32_t)v * kNP28) & SOP_M28;
    carry = (v + (uint64_t)q * kP28.v[0]) >> 28;  // the low 28 bits vanish
    LCV_UNROLL for (int j = 1; j < 14; ++j) col[i + j] += (uint64_t)q * kP28.v[j];
  }
  LCV_UNROLL for (int c = 14; c < 28; ++c) {
    const uint64_t t = col[c] + carry;
    L[c - 14] = (uint32_t)t & SOP_M28;
    carry = t >> 28;
  }
}

// squaring forms: c = x x over 7 limbs (cross products doubled: 28 multiply-adds) and its signed twin
template <class A, class L>
LCV_FN void col_sqr7(A c[13], const L* x) {
  LCV_UNROLL for (int k = 0; k < 13; ++k) c[k] = 0;
  LCV_UNROLL for (int i = 0; i < 7; ++i) {
    const L xi2 = x[i] + x[i];
    c[2 * i] += (A)x[i] * (A)x[i];
    LCV_UNROLL for (int j = i + 1; j < 7; ++j) c[i + j] += (A)xi2 * (A)x[j];
  }
}
// Montgomery square / product of fully reduced (or <= 2p) operands through the column engine:
// r = a b R^-1 mod p (one conditional subtraction: (T + M p) / R < 4p^2 / R + p < 2p)
LCV_FN void fp_mul_c28(uint32_t r[13], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t X[15], Y[14];
  sop_to28<12, 14>(X, a);
  sop_to28<12, 14>(Y, b);
  uint64_t p0[13], p2[13], col[28];
  int64_t pd[13];
  sop_kara_mac<true>(p0, p2, pd, X, Y);
  sop_kara_join(col, p0, p2, pd);
  sop_redc28(r, col);
}
LCV_FN void fp_sqr_c28(uint32_t r[13], const uint32_t a[12]) {
  uint32_t X[14];
  sop_to28<12, 14>(X, a);
  int32_t d[7];
  LCV_UNROLL for (int i = 0; i < 7; ++i) d[i] = (int32_t)(X[i] - X[i + 7]);
  uint64_t p0[13], p2[13], col[28];
  int64_t s[13];
  col_sqr7(p0, X);
  col_sqr7(p2, X + 7);
  col_sqr7(s, d);
  LCV_UNROLL for (int k = 0; k < 13; ++k) s[k] = -s[k];  // D = (X0 - X1)(X1 - X0) = -(X0 - X1)^2
  sop_kara_join(col, p0, p2, s);
  sop_redc28(r, col);
}

// limb-form Montgomery square / product with R = 2^392 (values < 2p stay < 2p: (T + M p) / R < 4p^2 / R + p)
LCV_FN void fp_sqr_lf(uint32_t r[14], const uint32_t a[14]) {
  LCV_COUNT(0);  // op counter (host simulation, -DLCV_OPCOUNT): one Fp multiplication
  int32_t d[7];
  LCV_UNROLL for (int i = 0; i < 7; ++i) d[i] = (int32_t)(a[i] - a[i + 7]);
  uint64_t p0[13], p2[13], col[28];
  int64_t s[13];
  col_sqr7(p0, a);
  col_sqr7(p2, a + 7);
  col_sqr7(s, d);
  LCV_UNROLL for (int k = 0; k < 13; ++k) s[k] = -s[k];
  sop_kara_join(col, p0, p2, s);
  sop_redc28_392(r, col);
}
LCV_FN void fp_mul_lf(uint32_t r[14], const uint32_t a[14], const uint32_t b[14]) {
  LCV_COUNT(0);
  uint32_t x[15];
  LCV_UNROLL for (int i = 0; i < 14; ++i) x[i] = a[i];
  x[14] = 0;
  uint64_t p0[13], p2[13], col[28];
  int64_t pd[13];
  sop_kara_mac<true>(p0, p2, pd, x, b);
  sop_kara_join(col, p0, p2, pd);
  sop_redc28_392(r, col);
}

}  // namespace lcv
