// lcv_sop_fan.hpp — the fan engine: the SOP programs (lcv_sop.hpp, tools/gen_sop.py) with the K products
// of every op fanned out over K lanes, for the latency path (lcv_set_latency_mode: batches of a few
// updates, the reference's one-update-per-call usage, sync-protocol.md:512 -> :464).  One item per block
// of TEAM x MAXK lanes (up to three waves); lane k * TEAM + o computes product k of op o.
//
// A lone item pays the latency of every instruction of a round: on the batch engine one lane runs an op's
// K products back to back (K x ~150 multiply-adds plus operand conversion) and then its reduction, so an
// op of K = 7 (the Miller accumulation's Fp12 squaring) costs ~7 products of latency.  Here a round is
//   products   lane (o, k) forms X_k, Y_k and their Karatsuba columns (lcv_col28.hpp), joined: 28 true
//              column sums of X_k Y_k, added into the op's 28-column LDS accumulator (64-bit LDS atomics);
//   reduce     after a block barrier, lane (o, 0) — the first wave holds every op's — reads the sums,
//              zeroes the accumulator, runs the batch engine's Montgomery reduction and its tail (add-ins,
//              conditional subtractions, store, shadow: lcv::sop_tail).
// The column sums are the batch engine's exactly (the join is linear and every joined column is a true,
// non-negative column sum below the op's bound), so every result is the batch engine's bit for bit
// (tests/test_latency_gpu.py).  Device-only; the host simulation runs the batch engine.
//
// Split products (LCV_FAN_SPLIT, the default): a lone wave issues a product's 147 multiply-adds back to
// back, ~1 us of a ~2.9 us final-exponentiation round (measured by removing them).  So each product's
// three Karatsuba sub-products go to three lanes (part 0: X0 Y0, 1: X1 Y1, 2: (X0 - X1)(Y1 - Y0), 7 x 7
// limbs, B = 2^196): 49 signed multiply-adds per lane (28-bit limbs are non-negative int32s, so one
// v_mad_i64_i32 stream serves all three parts without divergence), added into the op's columns at
// 0 and 7 (part 0), 14 and 7 (part 1) and 7 (part 2): X Y = P0 + (P0 + P2 + D) B + P2 B^2.  A signed
// partial sum may wrap in the 64-bit LDS column; the op's complete column is the true non-negative sum.
#pragma once
#include "lcv_sop.hpp"

#ifndef LCV_FAN_SPLIT
#define LCV_FAN_SPLIT 1
#endif
#ifndef LCV_FAN_X_CUT  // timing experiments only: 1 no operand reads, 2 no conversion, 3 no multiply-adds, 4 limb-form operands
#define LCV_FAN_X_CUT 0
#endif
#ifndef LCV_FAN_FLAT_TWO
#define LCV_FAN_FLAT_TWO 1
#endif
#ifndef LCV_FAN_PARTS
#define LCV_FAN_PARTS (LCV_FAN_SPLIT ? 3u : 1u)
#endif

namespace lcv {

enum : uint32_t { FAN_COLS = 28 };  // 64-bit columns of an op's LDS accumulator

// product k of an op (K > 0, k < K), given its record words (x terms, y terms, m): its 28 joined columns
LCV_FN void sop_fan_product(uint64_t col[28], uint32_t xw, uint32_t yw, uint32_t mk, uint32_t k, uint32_t masks,
                            bool mflag, const SopBase& base) {
  uint32_t Xw[13], Yw[12], X[15], Y[14];
  sop_operand(Xw, xw, (masks >> k) & 1u, base);
  sop_operand(Yw, yw, (masks >> (16 + k)) & 1u, base);
  Xw[12] = 0;
  if (mflag) {  // X *= m (m < 2^16): 13 words
    uint32_t carry = 0;
    LCV_UNROLL for (int j = 0; j < 12; ++j) {
      const uint64_t t = (uint64_t)Xw[j] * mk + carry;
      Xw[j] = (uint32_t)t;
      carry = (uint32_t)(t >> 32);
    }
    Xw[12] = carry;
  }
  sop_to28<12, 14>(Y, Yw);
  sop_to28<13, 14>(X, Xw);  // m X < 2^392 in every product round (LCV_SOP_SCHOOLBOOK 0)
  uint64_t p0[13], p2[13];
  int64_t pd[13];
  sop_kara_mac<true>(p0, p2, pd, X, Y);
  sop_kara_join(col, p0, p2, pd);
}

// part `part` (0, 1, 2) of product k: its 13 signed columns (placed by the caller, see above)
LCV_FN void sop_fan_part(int64_t c[13], uint32_t xw, uint32_t yw, uint32_t mk, uint32_t k, uint32_t masks,
                         bool mflag, uint32_t part, const SopBase& base) {
  uint32_t Xw[13], Yw[12], X[15], Y[14];
#if LCV_FAN_X_CUT == 4  // timing: operands as if stored as 28-bit limbs (16 words a slot; wrong results)
  {
    uint32_t La[16], Lb[16];
    const uint32_t* pa = sop_pterm(xw & 0xFFFFu, base);
    LCV_UNROLL for (int j = 0; j < 16; ++j) La[j] = pa[j];
    if ((masks >> k) & 1u) {
      const uint32_t* pb = sop_pterm(xw >> 16, base);
      LCV_UNROLL for (int j = 0; j < 16; ++j) La[j] += pb[j];
    }
    const uint32_t* qa = sop_pterm(yw & 0xFFFFu, base);
    LCV_UNROLL for (int j = 0; j < 16; ++j) Lb[j] = qa[j];
    if ((masks >> (16 + k)) & 1u) {
      const uint32_t* qb = sop_pterm(yw >> 16, base);
      LCV_UNROLL for (int j = 0; j < 16; ++j) Lb[j] += qb[j];
    }
    int32_t a[7], b[7];
    const bool p0 = part == 0, p1 = part == 1;
    LCV_UNROLL for (int i = 0; i < 7; ++i) {
      const int32_t xl = (int32_t)La[i], xh = (int32_t)La[i + 7], yl = (int32_t)Lb[i], yh = (int32_t)Lb[i + 7];
      a[i] = p0 ? xl : (p1 ? xh : xl - xh);
      b[i] = p0 ? yl : (p1 ? yh : yh - yl);
    }
    sop_mac7s<true>(c, a, b);
    (void)mflag; (void)mk; (void)Xw; (void)Yw; (void)X; (void)Y;
    return;
  }
#endif
#if LCV_FAN_X_CUT == 1  // timing experiments only (wrong results): no operand reads
  LCV_UNROLL for (int j = 0; j < 12; ++j) { Xw[j] = xw * (j + 1); Yw[j] = yw + j; }
#elif LCV_FAN_FLAT_TWO
  // a one-term operand's second handle is the zero slot (tools/gen_sop.py asserts it), so when any product of the
  // round has a two-term X (or Y) — a wave-uniform test — every lane adds its second term: no exec-mask region
  sop_operand(Xw, xw, (masks & 0xFFFFu) != 0u, base);
  sop_operand(Yw, yw, (masks >> 16) != 0u, base);
#else
  sop_operand(Xw, xw, (masks >> k) & 1u, base);
  sop_operand(Yw, yw, (masks >> (16 + k)) & 1u, base);
#endif
  Xw[12] = 0;
  if (mflag) {  // X *= m (m < 2^16): 13 words
    uint32_t carry = 0;
    LCV_UNROLL for (int j = 0; j < 12; ++j) {
      const uint64_t t = (uint64_t)Xw[j] * mk + carry;
      Xw[j] = (uint32_t)t;
      carry = (uint32_t)(t >> 32);
    }
    Xw[12] = carry;
  }
#if LCV_FAN_X_CUT == 2  // no conversion or part selection: words as limbs
  int32_t a[7], b[7];
  LCV_UNROLL for (int i = 0; i < 7; ++i) { a[i] = (int32_t)(Xw[i + part] & SOP_M28); b[i] = (int32_t)(Yw[i + part] & SOP_M28); }
  (void)X; (void)Y;
#else
  sop_to28<12, 14>(Y, Yw);
  sop_to28<13, 14>(X, Xw);
  int32_t a[7], b[7];
  const bool p0 = part == 0, p1 = part == 1;
  LCV_UNROLL for (int i = 0; i < 7; ++i) {
    const int32_t xl = (int32_t)X[i], xh = (int32_t)X[i + 7], yl = (int32_t)Y[i], yh = (int32_t)Y[i + 7];
    a[i] = p0 ? xl : (p1 ? xh : xl - xh);
    b[i] = p0 ? yl : (p1 ? yh : yh - yl);
  }
#endif
#if LCV_FAN_X_CUT == 3  // no multiply-adds: the inputs as columns
  LCV_UNROLL for (int i = 0; i < 13; ++i) c[i] = (int64_t)a[i % 7] + b[(i + 3) % 7];
#else
  sop_mac7s<true>(c, a, b);
#endif
}

}  // namespace lcv
